"""Caller buffers in HIP device memory (torch tensors) through the C ABI
(SURVEY 8(b)): device batches are unpacked and range-checked on the device,
tables and top-k results move device-to-device, and every result equals the
host-buffer path on the same inputs."""
import numpy as np
import pytest

from conftest import get_stream
from oracle import cf_oracle as O

pytestmark = pytest.mark.gpu


def engines(model, fold1, d=16, W=1, G=1, **kw):
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    rng = np.random.RandomState(4)
    U = O.init_table(rng, (943, d))
    V = O.init_table(rng, (1682, d))
    b = O.init_table(rng, (1682,))
    out = []
    for _ in range(2):
        e = Engine(model, 943, 1682, d, n_neg=W, gsize=G, **kw)
        e.set_interactions(fold1["train_indptr"], fold1["train_indices"])
        e.set_table("user", U)
        e.set_table("item", V)
        if model in ("gbpr", "prigp", "cplr"):
            e.set_table("bias", b)
        out.append(e)
    return out


def same(a, b):
    for t in ("user", "item", "acc_user", "acc_item"):
        x, y = a.get_table(t), b.get_table(t)
        assert np.max(np.abs(x - y)) <= 1e-6 * max(np.max(np.abs(x)), 1e-30), t


@pytest.mark.parametrize("model,stream", [("bpr", "rank_b100_w5"), ("gbpr", "gbpr_b100_g3_w2"),
                                          ("cml", "rank_b50_w5")])
def test_device_batches_match_host(streams, fold1, model, stream):
    import torch
    st = get_stream(streams, stream)
    W = st["negs"].shape[2]
    G = st["groups"].shape[2] if "groups" in st else 1
    h, dv = engines(model, fold1, W=W, G=G)
    for s in range(8):
        pr, ng = st["pairs"][s], st["negs"][s]
        gr = st["groups"][s] if "groups" in st else None
        lh = h.step(pr, ng, gr)
        ld = dv.step(torch.from_numpy(pr).cuda(), torch.from_numpy(ng).cuda(),
                     torch.from_numpy(gr).cuda() if gr is not None else None)
        assert abs(lh - ld) <= 1e-6 * abs(lh)
    same(h, dv)
    users = np.arange(0, 943, 3, dtype=np.int32)
    ih, vh = h.score_topk(users, 10, return_values=True)
    idd, vd = dv.score_topk(torch.from_numpy(users).cuda(), 10, return_values=True)
    assert idd.is_cuda and vd.is_cuda
    np.testing.assert_array_equal(ih, idd.cpu().numpy())
    np.testing.assert_allclose(vh, vd.cpu().numpy(), rtol=1e-6)
    h.close()
    dv.close()


def test_device_tuples_match_host(fold1):
    import torch
    h, dv = engines("cplr", fold1, reg=0.02, alpha=0.7, beta=1.3, gamma=0.5)
    rng = np.random.RandomState(9)
    for s in range(6):
        tup = np.stack([rng.randint(0, 943, 200)] + [rng.randint(0, 1682, 200) for _ in range(3)],
                       1).astype(np.int32)
        coefs = rng.gamma(1.0, 1.0, (200, 2)).astype(np.float32)
        lh = h.step_plr(tup, coefs)
        ld = dv.step_plr(torch.from_numpy(tup).cuda(), torch.from_numpy(coefs).cuda())
        assert abs(lh - ld) <= 1e-6 * abs(lh)
    same(h, dv)
    for t in ("bias", "acc_bias"):
        np.testing.assert_allclose(h.get_table(t), dv.get_table(t), rtol=1e-6)
    h.close()
    dv.close()


def test_device_tables_and_errors(fold1):
    import torch
    from collaborativefilteringusingtensorflow_amd import _native as N
    from collaborativefilteringusingtensorflow_amd.engine import _dev
    import ctypes
    e, _ = engines("bpr", fold1)
    V = torch.randn(1682, 16, device="cuda")
    vt, vp = _dev(V, torch.float32, ctypes.c_float)
    N.check(e._L.cf_set_table(e._h, N.TABLES["item"], vp, vt.numel()), "cf_set_table")
    np.testing.assert_array_equal(e.get_table("item"), V.cpu().numpy())
    out = torch.empty(1682, 16, device="cuda")
    N.check(e._L.cf_get_table(e._h, N.TABLES["item"],
                              ctypes.cast(out.data_ptr(), ctypes.POINTER(ctypes.c_float)), out.numel()),
            "cf_get_table")
    assert torch.equal(out, V)
    bad = torch.tensor([[0, 1], [5, 1682]], dtype=torch.int32, device="cuda")
    with pytest.raises(N.NativeError, match="row 1 has an id out of range"):
        e.step(bad, torch.tensor([[2], [3]], dtype=torch.int32, device="cuda"))
    dpairs = torch.tensor([[0, 1]], dtype=torch.int32, device="cuda")
    hnegs = np.array([[2]], np.int32)
    with pytest.raises(N.NativeError, match="all host or all device"):
        N.check(e._L.cf_step(e._h, ctypes.cast(dpairs.data_ptr(), ctypes.POINTER(ctypes.c_int32)),
                             hnegs.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), None, 1, None),
                "cf_step")
    e.step(np.array([[0, 1]], np.int32), np.array([[2]], np.int32))   # still usable
    e.close()
