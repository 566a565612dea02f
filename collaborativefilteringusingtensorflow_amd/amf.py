"""AMF drop-in, reference mode (src/models/others/models/amf.py:12-248).

Constructor order of amf.py:13-19.  What the reference actually computes
(SURVEY 0.5): epochs 0 .. e_s-1 minimise softplus(-x) + reg*L2 with one
Adagrad; at the end of the first epoch ``iter > 3*max_iter/5`` (amf.py:243-244)
training switches to a second train op with its OWN fresh Adagrad whose loss
adds reg_adv * softplus(-clip(x + Δ, -80, 1e8)).  Δ stays 0 because
``__update_adv__`` builds tf.assign ops that are never run (amf.py:117-137),
so the adversarial term only rescales the BPR gradient where -80 <= x <= 1e8.
``adv_method="rand"`` crashes the reference graph build (amf.py:126-127:
tf.assign on a bound method); it is rejected here with ValueError.

``amf_mode="apr"`` (not in the reference's constructor; SURVEY A.4 "optional
apr mode") runs the ``adv_method="grad"`` assigns as written instead:
Δ = epsilon * l2_normalize(dL_embed/dX) per step (include/cf_engine.h
amf_mode).  The default "reference" is what amf.py computes.
"""
from . import _native as N
from ._model import PairwiseModel


class AMF(PairwiseModel):
    MODEL = N.CF_AMF

    def __init__(self, n_users, n_items, topN=5, split_method='cv',
                 eval_metrics=['pre', 'recall', 'mrr', 'ndcg'], epsilon=.5, reg_adv=1.,
                 adv_method="grad", reg=0.02, n_factors=20, batch_size=100, max_iter=80, lr=0.1,
                 init_mean=0.0, init_stddev=0.1, device='GPU', seed=None, verbose=True, amf_mode="reference"):
        if adv_method != "grad":
            raise ValueError("adv_method=%r: only 'grad' builds in the reference "
                             "(amf.py:126-127 fails for 'rand')" % (adv_method,))
        if amf_mode not in N.AMF_MODES:
            raise ValueError("amf_mode=%r: 'reference' or 'apr'" % (amf_mode,))
        super(AMF, self).__init__(n_users, n_items, topN, split_method, eval_metrics,
                                  n_factors, batch_size, max_iter, lr, init_mean, init_stddev,
                                  device, seed, verbose)
        self._epsilon, self._reg_adv, self._adv_method = float(epsilon), float(reg_adv), adv_method
        self._reg = float(reg)
        self._amf_mode = amf_mode
        self._isAdver = False

    def _engine_kwargs(self):
        return dict(reg=self._reg, reg_adv=self._reg_adv, epsilon=self._epsilon,
                    amf_mode=self._amf_mode)

    def _log_line(self, fold, it, aveloss, scores, timecost):
        prefix = 'amf' if self._isAdver else 'bpr'
        return (prefix + " %s_fold=%d iter=%2d: " % (self._split_method, fold, it + 1)
                + "TraLoss=%.2f lr=%.4f" % (aveloss, self._lr) + "\tTst@" + str(self._topN) + ":"
                + " ".join(m + "=%.4f" % s for m, s in zip(self._eval_metrics, scores)))

    def _after_epoch(self, it):
        if it > 3 * self._max_iter / 5. and not self._isAdver:
            self._isAdver = True
            self._engine.begin_phase(1)

    def train(self, fold, trasR, tstsR, sampler):
        self._isAdver = False
        return super(AMF, self).train(fold, trasR, tstsR, sampler)
