"""CPU ORACLE -- test infrastructure, NOT part of the product.

A-priori fp32 rounding bounds for the BPRMF / AMF step of ``cf_oracle``.

The float64 oracle is the exact step (up to 1e-16).  TF1's CPU path and the
engine compute the same step in float32, with their own summation orders:
TF1 sums a row's duplicate gradients with ``UnsortedSegmentSum`` before
``SparseApplyAdagrad`` (bprmf.py:83-88), the engine with LDS run sums,
partial rows, slot rows and hardware float atomics.  Which
order is "right" is not defined by the reference, so the parity band must
admit every order's rounding -- and nothing more.

``bpr_step_bounded`` advances the float64 oracle by one step exactly as
``cf_oracle.bpr_step`` / ``amf_step`` do and, beside it, an elementwise
bound E >= |fp32 result - float64 result| for ANY float32 implementation of
the step that

* forms each dot product, each gradient row and each dedup-sum in float32
  in any order (any summation tree, with or without fused multiply-add);
* evaluates the logistic derivative c = -1/(1+e^x) with expf and a
  reciprocal within a few ulps, and Adagrad's rsqrt within one ulp
  (``cf_device.h`` adagrad_delta / rcp_1p);
* starts from tables within the carried bound E of the float64 ones.

It is standard forward error analysis (Higham, "Accuracy and Stability of
Numerical Algorithms", 2nd ed., 3.1 and 4.2):
u = 2^-24, gamma(n) = n u / (1 - n u);
|fl(sum_k a_k) - sum_k a_k| <= gamma(n-1) sum_k |a_k| for every order;
|fl(a . b) - a . b| <= gamma(n) sum_k |a_k b_k|;
errors in the inputs are carried to first order with magnitudes inflated by
their own bounds (|a| + e_a), so second-order terms are covered too.

Nothing in here is fitted to a measurement: no constant was chosen after
seeing a GPU result.  The bound is tight enough to catch a one-occurrence
accumulation bug on a hot row: for a row summing n terms the summation part
is gamma(n-1) sum|g_k| ~ n^2 u |g|, i.e. 5 % of ONE term at n = 900.

The CPU tests (tests/test_fp32_bound.py) check that the float32 oracle, the
float32 oracle with every dedup-sum taken in a shuffled order and in
reverse, and a float32 Kahan-free pairwise sum all stay inside E, and that
dropping one occurrence of a hot row, or applying it twice, falls outside.
"""
import numpy as np

from .cf_oracle import _c_bpr, _neg_log_sigmoid, _softplus, ACC_INIT

U32 = 2.0 ** -24           # unit roundoff of IEEE binary32, round to nearest
FX = 2.0 ** -32            # the deterministic mode's fixed-point unit
# ulps budget of the transcendental pieces on gfx950 (cf_device.h):
# c = -rcp(1 + expf(x)): expf <= 1 ulp (2u), the add (u), rcp <= 1 ulp (2u),
# the sign-less product with the AMF scale (u)  -> 6u, plus u per unit |x|
# for an argument reduction of expf that is not exact
C_ULPS = 6.0
# g * lr * rsq(acc): rsq <= 1 ulp (2u), two products (2u), the subtract's
# operand (u), and one spare                                      -> 6u
ADA_ULPS = 6.0

TABLES = ("user", "item", "acc_user", "acc_item")


def gamma(n):
    n = np.asarray(n, dtype=np.float64)
    return n * U32 / (1.0 - n * U32)


# the accumulators start at float32(0.1) on the engine, 0.1 in the float64 oracle
ACC0_ERR = abs(float(np.float32(ACC_INIT)) - ACC_INIT)


def zero_bounds(U, V, acc_exact=False):
    """E for tables that were set from the same float32 values on both sides;
    the accumulators differ by float32(0.1) - 0.1 unless ``acc_exact`` (the
    oracle was started from the engine's own accumulators)."""
    a = 0.0 if acc_exact else ACC0_ERR
    return {"user": np.zeros(U.shape), "item": np.zeros(V.shape),
            "acc_user": np.full(U.shape, a), "acc_item": np.full(V.shape, a)}


def _sigmoid_prime_max(x, dx):
    """max of sigma'(t) = sigma(t)(1 - sigma(t)) over [x - dx, x + dx]: sigma'
    is unimodal with its peak 1/4 at 0, so take the point nearest to 0."""
    t = np.clip(0.0, x - dx, x + dx)
    s = 1.0 / (1.0 + np.exp(-t))
    return s * (1.0 - s)


def _dedup_adagrad_bounded(X, A, EX, EA, rows, grads, egrads, lr):
    """cf_oracle.dedup_adagrad in float64, plus the bound.

    grads / egrads: [n_occ, d] per-occurrence gradient rows and their bounds.
    Sum of a row's n occurrences in any order: sum_k e_k + gamma(2n) sum_k
    (|g_k| + e_k) -- gamma(2n), not gamma(n-1), so that a form that splits
    each occurrence into two addends (the engine's item records add
    alpha_k X_k and beta_k V_row separately) is covered -- plus
    n 2^-32 for the fixed-point terms of the deterministic mode and one
    rounding of the result.  Then acc' = acc + G^2 and
    X' = X - lr G rsqrt(acc')."""
    rows = np.asarray(rows).reshape(-1)
    uniq, inv, cnt = np.unique(rows, return_inverse=True, return_counts=True)
    d = X.shape[1]
    G = np.zeros((uniq.shape[0], d))
    eG = np.zeros_like(G)
    M = np.zeros_like(G)
    np.add.at(G, inv, grads)
    np.add.at(eG, inv, egrads)
    np.add.at(M, inv, np.abs(grads) + egrads)
    n = cnt[:, None].astype(np.float64)
    eG += gamma(2 * n) * M + n * FX
    eG += U32 * (np.abs(G) + eG)
    # acc' = acc + G*G
    A0, eA0 = A[uniq], EA[uniq]
    A1 = A0 + G * G
    mG = np.abs(G) + eG
    eA1 = eA0 + (2.0 * np.abs(G) + eG) * eG + 2.0 * U32 * (A0 + eA0 + mG * mG)
    # X' = X - lr G / sqrt(acc')
    # acc' >= amin > 0 on every fp32 path; where the carried bound no longer
    # keeps acc' off 0 the bound on X' is infinite (it only happens to the
    # carried multi-step bound of a hot row, never to a one-step one)
    amin = A1 - eA1
    ok = amin > 0
    amin = np.where(ok, amin, 1.0)
    T = lr * G / np.sqrt(A1)
    prop = np.where(ok, lr * (eG / np.sqrt(amin) + mG * eA1 / (2.0 * amin * np.sqrt(amin))), np.inf)
    X0, eX0 = X[uniq], EX[uniq]
    X1 = X0 - T
    eX1 = eX0 + prop + ADA_ULPS * U32 * (np.abs(T) + prop) + U32 * (np.abs(X1) + eX0 + prop)
    A[uniq] = A1
    X[uniq] = X1
    EA[uniq] = eA1
    EX[uniq] = eX1
    return uniq


def _no_nan(E):
    """A bound carried over many steps can reach inf (see
    _dedup_adagrad_bounded); a later product of it with an exact 0 (an
    untouched row's E = 0) is NaN in IEEE arithmetic.  NaN compares false with
    everything, so it would read as 'no bound' silently: make it inf, which is
    sound (an upper bound) and which the tests count and limit
    (tests/conftest.py assert_close(max_excluded=...), LocalStepCheck)."""
    for t in E:
        np.copyto(E[t], np.inf, where=np.isnan(E[t]))


def bpr_step_bounded(U, V, AU, AV, E, pairs, negs, reg, lr=0.1, adversarial=None, reg_adv=1.0):
    """One BPRMF step (bprmf.py:52-88; = cf_oracle.bpr_step) or, with
    ``adversarial`` not None, one AMF step (amf.py:139-162; = amf_step), on the
    float64 tables in place, and E (dict over TABLES) advanced to bound the
    float32 result.  Returns the pre-update loss."""
    with np.errstate(invalid="ignore", over="ignore"):
        loss = _bpr_step_bounded(U, V, AU, AV, E, pairs, negs, reg, lr, adversarial, reg_adv)
    _no_nan(E)
    return loss


def _bpr_step_bounded(U, V, AU, AV, E, pairs, negs, reg, lr, adversarial, reg_adv):
    pairs = np.asarray(pairs)
    Bn = pairs.shape[0]
    negs = np.asarray(negs).reshape(Bn, -1)
    W = negs.shape[1]
    d = U.shape[1]
    u_idx, i_idx = pairs[:, 0], pairs[:, 1]
    Uu, Vi, Vj = U[u_idx], V[i_idx], V[negs]                     # [B,d] [B,d] [B,W,d]
    eU, eVi, eVj = E["user"][u_idx], E["item"][i_idx], E["item"][negs]
    mU, mVi, mVj = np.abs(Uu) + eU, np.abs(Vi) + eVi, np.abs(Vj) + eVj
    x = np.sum(Uu * Vi, axis=1)[:, None] - np.sum(Uu[:, None, :] * Vj, axis=-1)   # [B,W]
    # x = <u, v_i> - <u, v_j> or <u, v_i - v_j>: d products and d+1 adds
    mag = np.sum(mU[:, None, :] * (mVi[:, None, :] + mVj), axis=-1)
    dx = (np.sum(eU[:, None, :] * (mVi[:, None, :] + mVj)
                 + np.abs(Uu)[:, None, :] * (eVi[:, None, :] + eVj), axis=-1)
          + gamma(d + 2) * mag)
    c = _c_bpr(x)
    dc = _sigmoid_prime_max(x, dx) * dx + np.abs(c) * (C_ULPS + np.abs(x)) * U32
    if adversarial:
        inside = ((x >= -80.0) & (x <= 1e8)).astype(np.float64)
        scale = 1.0 + reg_adv * inside
        c = c * scale
        dc = dc * scale + 2.0 * U32 * np.abs(c)     # the rounded scale and the product
    ac = np.abs(c)
    s = c.sum(axis=1)                                            # [B]
    # gradient rows (bpr_loss_grads) and their bounds
    gU = (c[:, :, None] * (Vi[:, None, :] - Vj)).sum(axis=1) + reg * Uu
    eGU = ((dc[:, :, None] * (mVi[:, None, :] + mVj) + ac[:, :, None] * (eVi[:, None, :] + eVj)).sum(axis=1)
           + reg * eU
           + gamma(2 * W + 3) * (((ac + dc)[:, :, None] * (mVi[:, None, :] + mVj)).sum(axis=1) + reg * mU))
    gVi = s[:, None] * Uu + reg * Vi
    S1, SD = ac.sum(axis=1)[:, None], dc.sum(axis=1)[:, None]
    eGVi = SD * mU + S1 * eU + reg * eVi + gamma(W + 2) * ((S1 + SD) * mU + reg * mVi)
    gVj = -c[:, :, None] * Uu[:, None, :] + reg * Vj
    eGVj = (dc[:, :, None] * mU[:, None, :] + ac[:, :, None] * eU[:, None, :] + reg * eVj
            + gamma(2) * ((ac + dc)[:, :, None] * mU[:, None, :] + reg * mVj))
    reg_loss = reg * 0.5 * (np.sum(Uu * Uu) + np.sum(Vi * Vi) + np.sum(Vj * Vj))
    if adversarial is None:
        loss = np.sum(_neg_log_sigmoid(x)) + reg_loss
    else:
        loss = np.sum(_softplus(-x)) + reg_loss
        if adversarial:
            loss += reg_adv * np.sum(_softplus(-np.clip(x, -80.0, 1e8)))
    _dedup_adagrad_bounded(U, AU, E["user"], E["acc_user"], u_idx, gU, eGU, lr)
    _dedup_adagrad_bounded(V, AV, E["item"], E["acc_item"],
                           np.concatenate([i_idx, negs.reshape(-1)]),
                           np.concatenate([gVi, gVj.reshape(-1, d)]),
                           np.concatenate([eGVi, eGVj.reshape(-1, d)]), lr)
    return float(loss)


def reset_acc(AU, AV, E):
    """AMF's phase switch: a fresh optimizer (amf.py:157-162)."""
    AU[...] = ACC_INIT
    AV[...] = ACC_INIT
    E["acc_user"][...] = ACC0_ERR
    E["acc_item"][...] = ACC0_ERR


# ----------------------------------------------------------------------------
# CML  (cml.py:55-129; = cf_oracle.cml_step)
# ----------------------------------------------------------------------------
def _clip_bounded(X, EX, clip_norm):
    """tf.clip_by_norm(X, c, axes=[1]) on every row (cml.py:119-129), exact
    math in float64 (a row with |x| <= c is left exactly as it is), and the
    bound of an fp32 clip of rows within EX of X: the clip is 1-Lipschitz in
    L2, so an element moves by at most the row's ||EX||_2; the norm's and the
    scaling's rounding (and a row the fp32 norm puts on the other side of c)
    by (gamma(d + 4) + 3u) (|x| + e).  A row whose norm is below c by more
    than its error bound is not clipped on either side: E unchanged (the
    engine leaves an untouched row bit-identical)."""
    d = X.shape[1]
    n = np.sqrt(np.sum(X * X, axis=1, keepdims=True))
    en = np.sqrt(np.sum(EX * EX, axis=1, keepdims=True))
    rel = gamma(d + 4) + 3.0 * U32
    maybe = (n + en) * (1.0 + rel) >= clip_norm
    scale = np.where(n > clip_norm, clip_norm / np.where(n > 0, n, 1.0), 1.0)
    X *= scale
    EX[...] = np.where(maybe, en + rel * (np.abs(X) / scale + EX), EX)


def cml_step_bounded(U, V, AU, AV, E, pairs, negs, margin, reg_cov, clip_norm,
                     use_rank_weight=True, lr=0.1, n_items=None):
    """cml_step_bounded_ (below) with inf for NaN in E (_no_nan)."""
    with np.errstate(invalid="ignore", over="ignore"):
        loss = cml_step_bounded_(U, V, AU, AV, E, pairs, negs, margin, reg_cov, clip_norm,
                                 use_rank_weight, lr, n_items)
    _no_nan(E)
    return loss


def cml_step_bounded_(U, V, AU, AV, E, pairs, negs, margin, reg_cov, clip_norm,
                      use_rank_weight=True, lr=0.1, n_items=None):
    """One CML step (cml.py:55-129; = cf_oracle.cml_step) on the float64 tables
    in place, and E advanced to bound the float32 result.

    CML has discontinuities: the hinge (z > 0), the rank weight's indicators
    (dp - dn_w + margin > 0) and the argmin's ties (TF's _MinOrMaxGrad splits
    the gradient among exact ties).  A pair whose z, indicators or minimum are
    within their own rounding bound of a threshold may legitimately take
    either branch in fp32: every row it touches gets E = inf (excluded from
    the check; the tests assert how few there are).  Otherwise the branches
    are those of the float64 step and the bound follows the BPR one.
    Magnitudes of the item gradients count |U_u| + |V| (not the difference
    U_u - V) so that the item-record form alpha U_u + beta V is
    covered.  Returns the pre-update loss."""
    pairs = np.asarray(pairs)
    Bn = pairs.shape[0]
    negs = np.asarray(negs).reshape(Bn, -1)
    W = negs.shape[1]
    d = U.shape[1]
    if n_items is None:
        n_items = V.shape[0]
    u_idx, i_idx = pairs[:, 0], pairs[:, 1]
    Uu, Vi, Vj = U[u_idx], V[i_idx], V[negs]
    eU, eVi, eVj = E["user"][u_idx], E["item"][i_idx], E["item"][negs]
    du = Uu - Vi
    e_du = eU + eVi + U32 * np.abs(du)
    dp = np.sum(du * du, axis=1)
    e_dp = np.sum((2.0 * np.abs(du) + e_du) * e_du, axis=1) + gamma(d) * np.sum((np.abs(du) + e_du) ** 2, axis=1)
    dnv = Uu[:, None, :] - Vj
    e_dnv = eU[:, None, :] + eVj + U32 * np.abs(dnv)
    dn = np.sum(dnv * dnv, axis=-1)
    e_dn = (np.sum((2.0 * np.abs(dnv) + e_dnv) * e_dnv, axis=-1)
            + gamma(d) * np.sum((np.abs(dnv) + e_dnv) ** 2, axis=-1))
    m = dn.min(axis=1)
    e_m = e_dn.max(axis=1)
    # branch ambiguity
    amb = np.zeros(Bn, dtype=bool)
    t = dp[:, None] - dn + margin
    e_t = e_dp[:, None] + e_dn + 2.0 * U32 * (dp[:, None] + dn + abs(margin))
    if use_rank_weight:
        amb |= np.any(np.abs(t) <= e_t, axis=1)
    z = dp - m + margin
    e_z = e_dp + e_m + 2.0 * U32 * (dp + m + abs(margin))
    amb |= np.abs(z) <= e_z
    ties = dn == m[:, None]
    near = (np.abs(dn - m[:, None]) <= e_dn + e_m[:, None]) & ~ties
    amb |= np.any(near, axis=1)
    if use_rank_weight:
        imp = (t > 0).astype(np.float64)
        r = imp.mean(axis=1) * n_items
        lw = np.log(r + 1.0)
        e_lw = 3.0 * U32 + 2.0 * U32 * np.abs(lw)
    else:
        lw = np.ones(Bn)
        e_lw = np.zeros(Bn)
    loss = np.sum(np.maximum(z, 0.0) * lw)
    pos = z > 0
    a = pos * lw
    e_a = pos * e_lw
    cnt = ties.sum(axis=1, keepdims=True).astype(np.float64)
    share = ties / cnt
    e_share = U32 * share
    coef = 2.0 * a[:, None] * share                                   # [B,W]
    e_coef = 2.0 * (e_a[:, None] * share + a[:, None] * e_share) + 2.0 * U32 * coef
    rc = reg_cov if reg_cov > 0 else 0.0
    A2, eA2 = 2.0 * a[:, None], 2.0 * e_a[:, None]
    mU, mVi, mVj = np.abs(Uu) + eU, np.abs(Vi) + eVi, np.abs(Vj) + eVj
    # gradients (cf_oracle.cml_step) and their bounds
    gU = A2 * du - (coef[:, :, None] * dnv).sum(axis=1) + rc * Uu
    eGU = (eA2 * np.abs(du) + A2 * e_du
           + (e_coef[:, :, None] * np.abs(dnv) + coef[:, :, None] * e_dnv).sum(axis=1) + rc * eU
           + gamma(W + 4) * ((A2 + eA2) * (mU + mVi)
                             + ((coef + e_coef)[:, :, None] * (mU[:, None, :] + mVj)).sum(axis=1) + rc * mU))
    gVi = -A2 * du + rc * Vi
    eGVi = (eA2 * np.abs(du) + A2 * e_du + rc * eVi
            + gamma(4) * ((A2 + eA2) * (mU + mVi) + rc * mVi))
    gVj = coef[:, :, None] * dnv + rc * Vj
    eGVj = (e_coef[:, :, None] * np.abs(dnv) + coef[:, :, None] * e_dnv + rc * eVj
            + gamma(4) * ((coef + e_coef)[:, :, None] * (mU[:, None, :] + mVj) + rc * mVj))
    if rc > 0:
        loss += rc * 0.5 * (np.sum(Uu * Uu) + np.sum(Vi * Vi) + np.sum(Vj * Vj))
    # an ambiguous pair's rows: no bound (nor where a carried inf met a 0)
    eGU, eGVi, eGVj = (np.nan_to_num(x, nan=np.inf) for x in (eGU, eGVi, eGVj))
    eGU[amb] = np.inf
    eGVi[amb] = np.inf
    eGVj[amb] = np.inf
    _dedup_adagrad_bounded(U, AU, E["user"], E["acc_user"], u_idx, gU, eGU, lr)
    _dedup_adagrad_bounded(V, AV, E["item"], E["acc_item"], np.concatenate([i_idx, negs.reshape(-1)]),
                           np.concatenate([gVi, gVj.reshape(-1, d)]),
                           np.concatenate([eGVi, eGVj.reshape(-1, d)]), lr)
    _clip_bounded(U, E["user"], clip_norm)
    _clip_bounded(V, E["item"], clip_norm)
    return float(loss)
