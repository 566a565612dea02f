"""Host preprocessing and samplers of the tuple models (PRIGP, CPLR).

The similarity / top-K / coefficient steps are checked against a literal
transcription of the reference methods (prigp.py:62-87, cplr_u.py:66-96 and
the row normalisation at cplr_u.py:194-197) on random binary matrices; the
samplers against the invariants of sampler_prigp.py:24-52 and
sampler_uitj_ranking.py:22-38.  CPU only."""
import numpy as np
import pytest
import scipy.sparse as sp

from collaborativefilteringusingtensorflow_amd import _tuple as T


def literal_calsim(trasR):
    simMat = (np.dot(trasR, trasR.T)).toarray()
    for ind in range(trasR.shape[0]):
        den = np.linalg.norm(trasR[ind, :].toarray())
        if den > 0:
            simMat[ind, :] = simMat[ind, :] / den
            simMat[:, ind] = simMat[:, ind] / den
        simMat[ind, ind] = 0
    return simMat


def literal_topk(array, topK, cplr):
    for ind in range(array.shape[0]):
        row_sim = np.zeros((array.shape[1]))
        if cplr:
            inds = np.argsort(array[ind, :])[-topK:] if topK < len(array[ind, :].nonzero()[0]) \
                else array[ind, :].nonzero()[0]
        else:
            inds = np.argsort(array[ind, :])[-topK:]
        for ind_ in inds:
            row_sim[ind_] = array[ind, ind_]
        array[ind, :] = row_sim
    return array


def literal_calcoef(trasR, simMat, n_items, cplr):
    coef = sp.lil_matrix(trasR.shape)
    for user in set(trasR.nonzero()[0]):
        user_predict = np.zeros(n_items)
        for nn_user in simMat[user, :].nonzero()[0]:
            if cplr:
                user_predict += simMat[user, nn_user] * trasR[nn_user].toarray()[0]
            else:
                user_predict += trasR[nn_user].toarray()[0] > 0
        coef[user, :] = sp.lil_matrix(user_predict)
    return coef


def random_R(seed, nu=60, ni=80, p=0.1):
    rng = np.random.RandomState(seed)
    M = (rng.random_sample((nu, ni)) < p).astype(np.float32)
    M[3, :] = 0          # a user without interactions
    return sp.lil_matrix(M)


@pytest.mark.parametrize("cplr,topK", [(False, 5), (False, 40), (True, 5), (True, 200)])
def test_tuple_preprocessing_matches_literal_reference(cplr, topK):
    R = random_R(1 + topK)
    S_ref = literal_topk(literal_calsim(R), topK, cplr)
    S = T.top_k_rows(T.user_similarity(R), topK, keep_short_rows=cplr)
    np.testing.assert_allclose(S, S_ref, rtol=1e-12, atol=1e-15)
    C_ref = literal_calcoef(R, S_ref, R.shape[1], cplr)
    C = T.coefficients(S, R, weighted=cplr)
    np.testing.assert_allclose(C.toarray(), C_ref.toarray(), rtol=1e-12, atol=1e-15)
    if cplr:
        Cn_ref = C_ref.copy()
        for i in range(Cn_ref.shape[0]):
            with np.errstate(invalid="ignore", divide="ignore"):
                ave = Cn_ref[i, :].sum() / Cn_ref[i, :].nnz
            if ave > 0:
                Cn_ref[i, :] /= ave
        np.testing.assert_allclose(T.normalise_rows(C).toarray(), Cn_ref.toarray(), rtol=1e-12)


@pytest.mark.parametrize("native", [True, False])
def test_prigp_sampler_invariants(native):
    R = random_R(5)
    S = T.top_k_rows(T.user_similarity(R), 5)
    C = T.coefficients(S, R, weighted=False)
    s = T.PRIGPSampler(R, C, batch_size=50, seed=3, native=native)
    Cd = C.toarray()
    for _ in range(30):
        b = s.next_batch()
        assert b.shape == (50, 5)
        for u, i, j, t, k in b:
            assert R[u, i] != 0 and R[u, j] == 0
            if C[u, :].nnz == 0:
                assert (t, k) == (i, j)
            else:
                assert Cd[u, t] != 0
                assert Cd[u, k] == 0 or Cd[u, t] > Cd[u, k]


@pytest.mark.parametrize("native", [True, False])
def test_uitj_sampler_invariants(native):
    R = random_R(6)
    C = T.normalise_rows(T.coefficients(T.top_k_rows(T.user_similarity(R), 200, True), R, True))
    s = T.UITJSampler(R, C, batch_size=40, seed=4, native=native)
    Cd = C.toarray()
    for _ in range(30):
        tup, coefs = s.next_batch()
        assert tup.shape == (40, 4) and coefs.shape == (40, 2)
        for (u, i, t, j), (ci, ct) in zip(tup, coefs):
            assert R[u, i] != 0 and R[u, t] == 0 and Cd[u, t] != 0
            assert R[u, j] == 0 and Cd[u, j] == 0
            assert np.float32(ci) == np.float32(Cd[u, i]) and np.float32(ct) == np.float32(Cd[u, t])


@pytest.mark.parametrize("seed", [0, 3, 12345])
def test_native_tuple_samplers_reproduce_the_python_stream(seed):
    """cf_tuple_sampler draws exactly what the Python restatements draw from
    RandomState(seed): same shuffles, randint rejections and randn calls,
    across epoch boundaries."""
    R = random_R(7)
    S = T.user_similarity(R)
    Cp = T.coefficients(T.top_k_rows(S.copy(), 5), R, weighted=False)
    py = T.PRIGPSampler(R, Cp, batch_size=64, seed=seed, native=False)
    nat = T.PRIGPSampler(R, Cp, batch_size=64, seed=seed)
    nb = 3 * (R.nnz // 64) + 2                     # three epochs and then some
    for _ in range(nb):
        np.testing.assert_array_equal(nat.next_batch(), py.next_batch())
    Cc = T.normalise_rows(T.coefficients(T.top_k_rows(S.copy(), 50, True), R, True))
    py = T.UITJSampler(R, Cc, batch_size=80, seed=seed, native=False)
    nat = T.UITJSampler(R, Cc, batch_size=80, seed=seed)
    for _ in range(40):
        (a, ca), (b, cb) = nat.next_batch(), py.next_batch()
        np.testing.assert_array_equal(a, b)
        np.testing.assert_array_equal(ca.astype(np.float32), cb.astype(np.float32))
