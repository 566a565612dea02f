"""Ranking metrics with the reference's exact (partly non-standard) definitions.

Drop-in for ``src/metrics/ranking.py`` (same function names, argument order
and error behaviour).  Semantics kept on purpose:

* ndcg: the ideal DCG is built from the predicted list's OWN hit labels
  sorted descending, clamped with max(ideal, 1)  (ranking.py:29-40);
* map divides by |truth|, not min(k, |truth|)   (ranking.py:43-54);
* hr / arhr return SUMS over users, not means    (ranking.py:75-91).

Pinned by tests/golden/ranking_cases.json (computed with the reference).
"""
import numpy as np

__all__ = ["precision_k_score", "recall_k_score", "ndcg_k_score", "map_k_score",
           "mrr_k_score", "hr_k_score", "arhr_k_score", "evaluateCV", "evaluateLOOV"]


def _check(a, b, k, what="yss_true"):
    if len(a) != len(b) or len(a) == 0 or k <= 0:
        raise ValueError("len(%s) != len(yss_pred) or len(%s)==0 or k<=0!" % (what, what))


def _hits(truth, pred, k):
    """0/1 hit label of each of the first k predictions."""
    return [1 if p in truth else 0 for p in list(pred)[:k]]


def _dcg(labels):
    return sum(((2.0 ** l) - 1.0) / np.log2(pos + 2.0) for pos, l in enumerate(labels))


def precision_k_score(yss_true, yss_pred, k=5):
    _check(yss_true, yss_pred, k)
    tot = 0.0
    for truth, pred in zip(yss_true, yss_pred):
        tot += len(set(list(pred)[:k]) & set(truth)) / float(k)
    return tot / len(yss_true)


def recall_k_score(yss_true, yss_pred, k=5):
    _check(yss_true, yss_pred, k)
    tot = 0.0
    for truth, pred in zip(yss_true, yss_pred):
        tot += len(set(list(pred)[:k]) & set(truth)) / max(float(len(truth)), 1.0)
    return tot / len(yss_true)


def ndcg_k_score(yss_true, yss_pred, k=5):
    _check(yss_true, yss_pred, k)
    tot = 0.0
    for truth, pred in zip(yss_true, yss_pred):
        labels = _hits(truth, pred, k)
        tot += _dcg(labels) / max(_dcg(sorted(labels, reverse=True)), 1.0)
    return tot / len(yss_true)


def map_k_score(yss_true, yss_pred, k=5):
    _check(yss_true, yss_pred, k)
    tot = 0
    for truth, pred in zip(yss_true, yss_pred):
        n_hit, ap = 0, 0
        for pos, p in enumerate(list(pred)[:k]):
            if p in truth:
                n_hit += 1
                ap += n_hit / (pos + 1.0)
        tot += ap / len(truth)
    return tot / len(yss_true)


def mrr_k_score(yss_true, yss_pred, k=5):
    _check(yss_true, yss_pred, k)
    tot = 0
    for truth, pred in zip(yss_true, yss_pred):
        for pos, p in enumerate(list(pred)[:k]):
            if p in truth:
                tot += 1 / (pos + 1.0)
                break
    return tot / len(yss_true)


def hr_k_score(ys_true, yss_pred, k=5):
    _check(ys_true, yss_pred, k, "ys_true")
    tot = 0.0
    for t, pred in zip(ys_true, yss_pred):
        tot += t in set(list(pred)[:k])
    return tot


def arhr_k_score(ys_true, yss_pred, k=5):
    _check(ys_true, yss_pred, k, "ys_true")
    tot = 0.0
    for t, pred in zip(ys_true, yss_pred):
        head = list(pred)[:k]
        if t in head:
            tot += 1.0 / (head.index(t) + 1)
    return tot


_CV = {"pre": precision_k_score, "recall": recall_k_score, "ndcg": ndcg_k_score,
       "map": map_k_score, "mrr": mrr_k_score}
_LOOV = {"hr": hr_k_score, "arhr": arhr_k_score}


def evaluateCV(yss_true, yss_pred, eval_metrics, k=5):
    """Unknown metric names give None, as in ranking.py:94-109."""
    return [_CV[m](yss_true, yss_pred, k) if m in _CV else None for m in eval_metrics]


def evaluateLOOV(ys_true, yss_pred, eval_metrics, k=5):
    return [_LOOV[m](ys_true, yss_pred, k) if m in _LOOV else None for m in eval_metrics]
