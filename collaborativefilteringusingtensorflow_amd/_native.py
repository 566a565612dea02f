"""ctypes binding of the C ABI in include/cf_engine.h (libcf_engine.so).

The product has no CPU fallback: if the shared library is missing, or no HIP
device is visible when an engine is created, the calls raise.
"""
import ctypes
import os
import re

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CF_ENGINE_LIB", os.path.join(_PKG, "build", "libcf_engine.so"))
HEADER_PATH = os.path.join(os.path.dirname(_PKG), "include", "cf_engine.h")

CF_BPR, CF_GBPR, CF_CML, CF_AMF, CF_PLR = 0, 1, 2, 3, 4
CF_PLR_PRIGP, CF_PLR_CPLR = 0, 1
CF_AMF_REFERENCE, CF_AMF_APR = 0, 1
AMF_MODES = {"reference": CF_AMF_REFERENCE, "apr": CF_AMF_APR}
MODEL_IDS = {"bpr": CF_BPR, "bprmf": CF_BPR, "gbpr": CF_GBPR, "gbprmf": CF_GBPR,
             "cml": CF_CML, "amf": CF_AMF, "plr": CF_PLR, "prigp": CF_PLR, "cplr": CF_PLR}
TABLES = {"user": 0, "item": 1, "bias": 2, "acc_user": 3, "acc_item": 4, "acc_bias": 5}
KERNELS = {"sample": 0, "step": 1, "apply": 2, "apply_dense": 3, "clip": 4, "score": 5,
           "topk": 6, "slot": 7, "apply_prep": 8, "grad_prep": 9, "apply_slot": 10,
           "item_reduce": 11, "psort": 12, "step_remote": 13, "epoch_order": 14}
STATUS = {0: "CF_OK", -1: "CF_EINVAL", -2: "CF_EHIP", -3: "CF_ESTATE", -4: "CF_ENOMEM", -5: "CF_EAGAIN",
          -6: "CF_ENUMERIC"}
CF_EAGAIN = -5


class NativeError(RuntimeError):
    pass


class CfConfig(ctypes.Structure):
    _fields_ = [
        ("model", ctypes.c_int32),
        ("n_factors", ctypes.c_int32),
        ("n_users", ctypes.c_int64),
        ("n_items", ctypes.c_int64),
        ("n_neg", ctypes.c_int32),
        ("gsize", ctypes.c_int32),
        ("lr", ctypes.c_float),
        ("reg", ctypes.c_float),
        ("rho", ctypes.c_float),
        ("margin", ctypes.c_float),
        ("reg_cov", ctypes.c_float),
        ("clip_norm", ctypes.c_float),
        ("reg_adv", ctypes.c_float),
        ("epsilon", ctypes.c_float),
        ("acc_init", ctypes.c_float),
        ("use_rank_weight", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("dense_item_apply", ctypes.c_int32),
        ("plr_kind", ctypes.c_int32),
        ("seed", ctypes.c_uint64),
        ("alpha", ctypes.c_float),
        ("beta", ctypes.c_float),
        ("gamma", ctypes.c_float),
        ("amf_mode", ctypes.c_int32),
    ]


_P = ctypes.c_void_p
_I32 = ctypes.c_int32
_I64 = ctypes.c_int64
_U64 = ctypes.c_uint64
_F = ctypes.c_float
_PI32 = ctypes.POINTER(ctypes.c_int32)
_PI64 = ctypes.POINTER(ctypes.c_int64)
_PF = ctypes.POINTER(ctypes.c_float)
_PD = ctypes.POINTER(ctypes.c_double)

# name -> (restype, argtypes); must cover every function declared in the header
SIGNATURES = {
    "cf_version": (ctypes.c_char_p, []),
    "cf_last_error": (ctypes.c_char_p, []),
    "cf_device_count": (ctypes.c_int, [_PI32]),
    "cf_config_defaults": (None, [ctypes.POINTER(CfConfig)]),
    "cf_create": (ctypes.c_int, [ctypes.POINTER(CfConfig), ctypes.POINTER(_P)]),
    "cf_destroy": (ctypes.c_int, [_P]),
    "cf_set_stream": (ctypes.c_int, [_P, _P]),
    "cf_synchronize": (ctypes.c_int, [_P]),
    "cf_set_interactions": (ctypes.c_int, [_P, _PI64, _PI32, _I64]),
    "cf_init_params": (ctypes.c_int, [_P, _F, _F, _I32, _U64]),
    "cf_set_table": (ctypes.c_int, [_P, _I32, _PF, _I64]),
    "cf_get_table": (ctypes.c_int, [_P, _I32, _PF, _I64]),
    "cf_set_params": (ctypes.c_int, [_P, _PF, _PF, _PF, _PF, _PF, _PF]),
    "cf_get_params": (ctypes.c_int, [_P, _PF, _PF, _PF, _PF, _PF, _PF]),
    "cf_step": (ctypes.c_int, [_P, _PI32, _PI32, _PI32, _I32, _PD]),
    "cf_train_steps": (ctypes.c_int, [_P, _I32, _I32, _PD]),
    "cf_train_epoch": (ctypes.c_int, [_P, _I32, _PD]),
    "cf_sample": (ctypes.c_int, [_P, _I32, _PI32, _PI32, _PI32]),
    "cf_get_sampler_state": (ctypes.c_int, [_P, _PI64, _PI64]),
    "cf_set_sampler_state": (ctypes.c_int, [_P, _I64, _I64]),
    "cf_begin_phase": (ctypes.c_int, [_P, _I32]),
    "cf_bind_item_grad": (ctypes.c_int, [_P, _P, _I64]),
    "cf_step_local": (ctypes.c_int, [_P, _I32, _PI32, _PI32, _PI32]),
    "cf_step_items": (ctypes.c_int, [_P]),
    "cf_step_local_draw": (ctypes.c_int, [_P, _I32]),
    "cf_bind_item_grad_split": (ctypes.c_int, [_P, _P, _I64, _P, _I64]),
    "cf_clear_item_grad": (ctypes.c_int, [_P]),
    "cf_step_items_range": (ctypes.c_int, [_P, _I64, _I64, _P, _P]),
    "cf_bind_table": (ctypes.c_int, [_P, _I32, _P, _I64]),
    "cf_step_local_grad": (ctypes.c_int, [_P, _I32, _PI32, _PI32, _PI32]),
    "cf_bind_apr_item_grad": (ctypes.c_int, [_P, _P, _I64]),
    "cf_step_local_apr_embed": (ctypes.c_int, [_P, _I32, _PI32, _PI32]),
    "cf_step_local_apply": (ctypes.c_int, [_P, _I32]),
    "cf_step_item_reduce": (ctypes.c_int, [_P, _I32]),
    "cf_item_piece_rows": (ctypes.c_int, [_P, _I32, _I32, _PI64, _PI64]),
    "cf_take_loss": (ctypes.c_int, [_P, _PD]),
    "cf_step_plr": (ctypes.c_int, [_P, _PI32, _I32, _PF, _I32, _PD]),
    "cf_set_shard": (ctypes.c_int, [_P, _I32, _I32, _PI64]),
    "cf_set_group_source": (ctypes.c_int, [_P, _PI64, _PI32, _I64]),
    "cf_bind_exchange": (ctypes.c_int, [_P, _P, _P, _P, _I64, _P, _P, _P, _I64]),
    "cf_xchg_begin": (ctypes.c_int, [_P, _I32, _PI32, _PI32, _PI32, _PI32]),
    "cf_xchg_draw": (ctypes.c_int, [_P, _I32, _P, _PI32]),
    "cf_xchg_adopt": (ctypes.c_int, [_P, _I32]),
    "cf_step_path": (ctypes.c_int, [_P, _I32, _PI32]),
    "cf_xchg_serve": (ctypes.c_int, [_P, _I64]),
    "cf_xchg_grad": (ctypes.c_int, [_P]),
    "cf_xchg_grad_part": (ctypes.c_int, [_P, _I32]),
    "cf_xchg_finish_items": (ctypes.c_int, [_P]),
    "cf_xchg_finish": (ctypes.c_int, [_P, _I64]),
    "cf_score_topk": (ctypes.c_int, [_P, _PI32, _I32, _I32, _P, _PI32, _PF]),
    "cf_score_topk_ex": (ctypes.c_int, [_P, _PI32, _I32, _I32, _I32, _P, _PI32, _PF]),
    "cf_set_option": (ctypes.c_int, [_P, ctypes.c_char_p, _I64]),
    "cf_profile_enable": (ctypes.c_int, [_P, _I32]),
    "cf_profile_read": (ctypes.c_int, [_P, _I32, _PD, _PI64]),
    "cf_profile_reset": (ctypes.c_int, [_P]),
    "cf_ratings_load": (ctypes.c_int, [ctypes.c_char_p, _I64, _I64, _I32, ctypes.POINTER(_P), _PI64]),
    "cf_ratings_csr": (ctypes.c_int, [_P, _I32, ctypes.c_double, _PI64, _PI32, _PD, _PI64]),
    "cf_ratings_free": (ctypes.c_int, [_P]),
    "cf_mt_sampler_create": (ctypes.c_int, [_PI64, _PI32, _I64, _I64, _I32, _I32, _I32, _I32,
                                            ctypes.c_uint32, ctypes.POINTER(_P)]),
    "cf_mt_sampler_next": (ctypes.c_int, [_P, _PI32, _PI32, _PI32]),
    "cf_mt_sampler_state": (ctypes.c_int, [_P, _PI64, _PI64]),
    "cf_mt_sampler_free": (ctypes.c_int, [_P]),
    "cf_tuple_sampler_create": (ctypes.c_int, [_I32, _PI64, _PI32, _I64, _I64, _PI64, _PI32, _PD,
                                                _I32, ctypes.c_uint32, ctypes.POINTER(_P)]),
    "cf_tuple_sampler_next": (ctypes.c_int, [_P, _PI32, _PF]),
    "cf_tuple_sampler_free": (ctypes.c_int, [_P]),
    "cf_ens_create": (ctypes.c_int, [_I64, _I64, _I32, _I32, _F, _F, _F, _I32, ctypes.POINTER(_P)]),
    "cf_ens_destroy": (ctypes.c_int, [_P]),
    "cf_ens_init_params": (ctypes.c_int, [_P, _F, _F, _I32, _U64]),
    "cf_ens_set_lr": (ctypes.c_int, [_P, _F]),
    "cf_ens_set_table": (ctypes.c_int, [_P, _I32, _PF, _I64]),
    "cf_ens_get_table": (ctypes.c_int, [_P, _I32, _PF, _I64]),
    "cf_ens_set_interactions": (ctypes.c_int, [_P, _PI64, _PI32, _I64]),
    "cf_ens_step": (ctypes.c_int, [_P, _PI32, _I32, _PD]),
    "cf_ens_take_loss": (ctypes.c_int, [_P, _PD]),
    "cf_ens_step_w": (ctypes.c_int, [_P, _PI32, _PI32, _I32, _I32, _F, _I32, _PD]),
    "cf_ens_score_topk": (ctypes.c_int, [_P, _PI32, _I32, _I32, _I32, _PI32, _PF]),
    "cf_synth_degrees": (ctypes.c_int, [_I64, ctypes.c_double, _U64, _I64, _I64, _PI64]),
    "cf_synth_items": (ctypes.c_int, [_I64, ctypes.c_double, _U64, _I64, _I64, _PI64, _PI32, _I32]),
    "cf_synth_item_users": (ctypes.c_int, [_I64, _I64, ctypes.c_double, ctypes.c_double, _U64, _PI64,
                                           _PI32, _I32]),
}

_lib = None


def header_symbols(path=HEADER_PATH):
    """Function names declared in include/cf_engine.h."""
    with open(path) as f:
        text = f.read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(cf_[a-z_0-9]+)\s*\(", text)))


def _preload_torch_hip():
    """One HIP runtime per process.  PyTorch ships its own libamdhip64 /
    libhsa-runtime64 (same sonames as /opt/rocm's); if this library loaded
    /opt/rocm's first, a later ``torch.cuda`` init would start a second
    runtime and find no device.  Loading torch's copies first (RTLD_GLOBAL,
    without importing torch) makes the engine bind to them, so engine and
    torch share one runtime in either import order.  CF_HIP_RUNTIME=system
    keeps /opt/rocm's."""
    if os.environ.get("CF_HIP_RUNTIME", "") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    d = os.path.join(os.path.dirname(spec.origin), "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)


def lib():
    """Load libcf_engine.so once; raise NativeError if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    _preload_torch_hip()
    if not os.path.exists(LIB_PATH):
        raise NativeError(
            "libcf_engine.so not found at %s -- build it with "
            "`python -m collaborativefilteringusingtensorflow_amd.csrc.build` "
            "(there is no CPU fallback)" % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status, what=""):
    if status != 0:
        msg = lib().cf_last_error().decode("utf-8", "replace")
        raise NativeError("%s failed: %s (%s)" % (what, msg, STATUS.get(status, status)))


def device_count():
    n = ctypes.c_int32(0)
    lib().cf_device_count(ctypes.byref(n))
    return int(n.value)
