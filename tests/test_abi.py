"""C-ABI boundary checks that need no GPU: the library loads, exports every
function include/cf_engine.h declares, the ctypes struct matches the header,
defaults match the reference constructors, and the engine refuses to run
without a HIP device (no CPU fallback)."""
import ctypes
import re

import numpy as np
import pytest

from collaborativefilteringusingtensorflow_amd import _native as N


def test_every_header_symbol_is_exported_and_bound():
    L = N.lib()
    syms = N.header_symbols()
    assert len(syms) >= 25
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing
    unbound = [s for s in syms if s not in N.SIGNATURES]
    assert not unbound, unbound
    extra = [s for s in N.SIGNATURES if s not in syms]
    assert not extra, extra


def test_config_struct_matches_header():
    with open(N.HEADER_PATH) as f:
        text = f.read()
    body = text[text.index("typedef struct cf_config {"):text.index("} cf_config;")]
    fields = re.findall(r"^\s*(int32_t|int64_t|uint64_t|float)\s+([a-z_0-9, ]+);", body, re.M)
    names = []
    for _t, ns in fields:
        names += [n.strip() for n in ns.split(",")]
    assert names == [f[0] for f in N.CfConfig._fields_]


def test_defaults_follow_reference_constructors():
    cfg = N.CfConfig()
    N.lib().cf_config_defaults(ctypes.byref(cfg))
    assert cfg.n_factors == 20 and abs(cfg.reg - 0.02) < 1e-6          # bprmf.py:15
    assert abs(cfg.lr - 0.1) < 1e-6 and abs(cfg.acc_init - 0.1) < 1e-6  # TF1 Adagrad
    assert abs(cfg.rho - 0.5) < 1e-6                                   # gbprmf.py:14
    assert abs(cfg.margin - 1.5) < 1e-6 and cfg.use_rank_weight == 1   # cml.py:16
    assert abs(cfg.reg_adv - 1.0) < 1e-6 and abs(cfg.epsilon - 0.5) < 1e-6  # amf.py:15
    assert cfg.amf_mode == N.CF_AMF_REFERENCE   # what amf.py computes (Δ = 0)


def test_amf_mode_names_and_rejections():
    """amf_mode: the header's enum values, the drop-in's names, and the
    class's ValueError before any device work (CPU)."""
    with open(N.HEADER_PATH) as f:
        text = f.read()
    assert re.search(r"CF_AMF_REFERENCE\s*=\s*0", text) and re.search(r"CF_AMF_APR\s*=\s*1", text)
    assert N.AMF_MODES == {"reference": 0, "apr": 1}
    from collaborativefilteringusingtensorflow_amd.amf import AMF
    with pytest.raises(ValueError):
        AMF(10, 10, amf_mode="rand")


def test_kernel_ids_match_header():
    with open(N.HEADER_PATH) as f:
        text = f.read()
    for name, kid in N.KERNELS.items():
        m = re.search(r"CF_K_%s\s*=\s*(\d+)" % name.upper(), text)
        assert m and int(m.group(1)) == kid, name


def test_no_cpu_fallback():
    if N.device_count() > 0:
        pytest.skip("a GPU is visible")
    from collaborativefilteringusingtensorflow_amd.engine import Engine
    with pytest.raises(N.NativeError, match="no HIP device"):
        Engine("bpr", 10, 10, 4)


def test_last_error_and_einval_paths():
    L = N.lib()
    cfg = N.CfConfig()
    L.cf_config_defaults(ctypes.byref(cfg))
    cfg.n_users, cfg.n_items, cfg.n_factors = 10, 10, 999
    h = ctypes.c_void_p()
    assert L.cf_create(ctypes.byref(cfg), ctypes.byref(h)) == -1
    assert b"n_factors" in L.cf_last_error()
    assert L.cf_create(None, ctypes.byref(h)) == -1


def test_synth_graph_deterministic_and_shardable():
    from collaborativefilteringusingtensorflow_amd.engine import synth_degrees, synth_graph
    ip, ix = synth_graph(2000, 500, 20.0, 0.8, 7, n_threads=3)
    ip2, ix2 = synth_graph(2000, 500, 20.0, 0.8, 7, n_threads=1)
    assert np.array_equal(ip, ip2) and np.array_equal(ix, ix2)
    assert np.array_equal(ip, synth_degrees(2000, 20.0, 7))
    deg = np.diff(ip)
    assert deg.min() >= 1 and abs(deg.mean() - 20.0) < 1.0
    for u in range(0, 2000, 97):
        row = ix[ip[u]:ip[u + 1]]
        assert np.all(np.diff(row) > 0) and row.min() >= 0 and row.max() < 500
    # any user range regenerates exactly the same rows
    sp, sx = synth_graph(2000, 500, 20.0, 0.8, 7, u_begin=700, u_end=1300)
    assert np.array_equal(sp, ip[700:1301] - ip[700])
    assert np.array_equal(sx, ix[ip[700]:ip[1300]])
    # Zipf popularity: the most popular items dominate
    cnt = np.bincount(ix, minlength=500)
    assert cnt.max() > 10 * np.median(cnt)


def test_ensemble_no_cpu_fallback_and_einval():
    L = N.lib()
    h = ctypes.c_void_p()
    assert L.cf_ens_create(10, 10, 9, 4, 0.1, 0.1, 0.1, 0, ctypes.byref(h)) == -1   # K > 8
    assert b"K 1..8" in L.cf_last_error()
    if N.device_count() > 0:
        return
    from collaborativefilteringusingtensorflow_amd.ensemble import EnsembleEngine
    with pytest.raises(N.NativeError, match="no HIP device"):
        EnsembleEngine(10, 10, 3, 4)
