"""Build libcf_engine.so for gfx950 in-tree (hipcc cross-compiles without a GPU).

    python -m collaborativefilteringusingtensorflow_amd.csrc.build [--force]

Objects and the shared library go to collaborativefilteringusingtensorflow_amd/build/
(git-ignored, but shipped to the GPU box by gpurun).
"""
import concurrent.futures as cf
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
ROOT = os.path.dirname(PKG)
# CF_BUILD_VARIANT=<name> + CF_EXTRA_FLAGS="-D..." build an experimental
# variant into build/variants/<name>/ (load it with CF_ENGINE_LIB=<path>)
VARIANT = os.environ.get("CF_BUILD_VARIANT", "")
OUT = os.path.join(PKG, "build", "variants", VARIANT) if VARIANT else os.path.join(PKG, "build")
LIB = os.path.join(OUT, "libcf_engine.so")
# cf_kernels.hip and the per-model gradient units share cf_kernels_impl.h; the
# split lets the pool below compile the heavy instantiations in parallel
SOURCES = ["cf_grad_bpr.hip", "cf_grad_amf.hip", "cf_grad_cml.hip", "cf_grad_gbpr.hip", "cf_grad_plr.hip",
           "cf_kernels.hip", "cf_eval.hip", "cf_engine.cpp", "cf_synth.cpp", "cf_ingest.cpp",
           "cf_mt_sampler.cpp", "cf_ensemble.hip", "cf_det.hip", "cf_epoch.hip"]
HEADERS = ["cf_kernels.h", "cf_device.h", "cf_kernels_impl.h", os.path.join(ROOT, "include", "cf_engine.h")]
ARCH = os.environ.get("CF_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=" + ARCH, "-munsafe-fp-atomics",
         "-Wall", "-Wno-unused-function", "-Wno-pass-failed", "-I" + os.path.join(ROOT, "include")]
FLAGS += os.environ.get("CF_EXTRA_FLAGS", "").split()


def _newer(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(src):
    path = os.path.join(HERE, src)
    obj = os.path.join(OUT, src + ".o")
    deps = [path] + [h if os.path.isabs(h) else os.path.join(HERE, h) for h in HEADERS]
    if not _newer(obj, deps):
        return obj
    cmd = [HIPCC] + FLAGS + ["-c", path, "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC] + FLAGS + ["-x", "hip", "-c", path, "-o", obj]
    subprocess.run(cmd, check=True)
    return obj


def build(force=False, verbose=True):
    os.makedirs(OUT, exist_ok=True)
    if force:
        for f in os.listdir(OUT):
            if f.endswith(".o") or f.endswith(".so"):
                os.remove(os.path.join(OUT, f))
    with cf.ThreadPoolExecutor(max_workers=int(os.environ.get("CF_BUILD_JOBS", "8"))) as ex:
        objs = list(ex.map(_compile, SOURCES))
    if _newer(LIB, objs):
        subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH, "-o", LIB] + objs
                       + ["-lpthread"], check=True)
    if verbose:
        print("built", LIB)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv)
