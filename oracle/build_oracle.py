"""Build and load the C oracle (test infrastructure only).

    python -m oracle.build_oracle

Output: oracle/build/libcf_oracle.so (git-ignored; ships to the GPU box).
There is no oracle/_ref build: the reference is pure Python over TF1 and has
no C/C++ sources to compile.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "cf_oracle.c")
LIB = os.path.join(HERE, "build", "libcf_oracle.so")


def build(verbose=True):
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(SRC):
        subprocess.run(["gcc", "-O2", "-std=c11", "-fopenmp", "-fPIC", "-shared", "-o", LIB, SRC,
                        "-lm"], check=True)
    if verbose:
        print("built", LIB)
    return LIB


class OracleCfg(ctypes.Structure):
    _fields_ = [("model", ctypes.c_int), ("d", ctypes.c_int), ("W", ctypes.c_int),
                ("G", ctypes.c_int), ("n_users", ctypes.c_int64), ("n_items", ctypes.c_int64),
                ("lr", ctypes.c_float), ("reg", ctypes.c_float), ("rho", ctypes.c_float),
                ("margin", ctypes.c_float), ("reg_cov", ctypes.c_float),
                ("clip_norm", ctypes.c_float), ("reg_adv", ctypes.c_float),
                ("use_rank_weight", ctypes.c_int), ("adversarial", ctypes.c_int)]


class OracleState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in
                ("U", "V", "b", "AU", "AV", "Ab", "GU", "GV", "Gb", "tU", "tV", "listU", "listV")]


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


class COracle(object):
    """Holds fp32 tables and the scratch the C step needs."""

    MODELS = {"bpr": 0, "gbpr": 1, "cml": 2, "amf": 3}

    def __init__(self, model, U, V, b=None, W=1, G=1, lr=0.1, reg=0.02, rho=0.5, margin=1.0,
                 reg_cov=1.0, clip_norm=1.0, reg_adv=1.0, use_rank_weight=True, max_batch=1 << 17):
        self.L = ctypes.CDLL(build(verbose=False))
        self.L.oracle_step.restype = ctypes.c_double
        self.L.oracle_step.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_int]
        self.L.oracle_train_mt.restype = ctypes.c_double
        self.L.oracle_train_mt.argtypes = ([ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_int,
                                           ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                           ctypes.c_void_p, ctypes.c_int])
        self.L.oracle_train.restype = ctypes.c_double
        self.L.oracle_train.argtypes = ([ctypes.c_void_p] * 5 + [ctypes.c_int64, ctypes.c_int,
                                        ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p,
                                        ctypes.c_void_p])
        self.U = np.array(U, dtype=np.float32, order="C", copy=True)   # never alias the caller
        self.V = np.array(V, dtype=np.float32, order="C", copy=True)
        nu, d = self.U.shape
        ni = self.V.shape[0]
        self.b = (np.array(b, dtype=np.float32, copy=True) if b is not None
                  else np.zeros(1, np.float32))
        self.AU = np.full_like(self.U, 0.1)
        self.AV = np.full_like(self.V, 0.1)
        self.Ab = np.full_like(self.b, 0.1)
        self.GU = np.zeros_like(self.U)
        self.GV = np.zeros_like(self.V)
        self.Gb = np.zeros_like(self.b)
        self.tU = np.zeros(nu, np.uint8)
        self.tV = np.zeros(ni, np.uint8)
        occ = max_batch * (1 + max(W, G))
        self.listU = np.zeros(min(occ, nu) + 1, np.int32)
        self.listV = np.zeros(min(occ, ni) + 1, np.int32)
        self.cfg = OracleCfg(self.MODELS[model], d, W, G, nu, ni, lr, reg, rho, margin, reg_cov,
                             clip_norm, reg_adv, 1 if use_rank_weight else 0, 0)
        self.st = OracleState(*[_p(a) for a in (self.U, self.V, self.b, self.AU, self.AV, self.Ab,
                                                self.GU, self.GV, self.Gb, self.tU, self.tV,
                                                self.listU, self.listV)])
        self._keep = None

    def set_adversarial(self, on):
        self.cfg.adversarial = 1 if on else 0
        if on:
            self.AU[...] = 0.1
            self.AV[...] = 0.1

    def step(self, pairs, negs, groups=None):
        pairs = np.ascontiguousarray(pairs, np.int32)
        negs = np.ascontiguousarray(negs, np.int32)
        groups = np.ascontiguousarray(groups, np.int32) if groups is not None else None
        return self.L.oracle_step(ctypes.byref(self.cfg), ctypes.byref(self.st), _p(pairs),
                                  _p(negs), _p(groups), pairs.shape[0])

    def train(self, indptr, indices, pairs_coo, B, n_steps, seed):
        indptr = np.ascontiguousarray(indptr, np.int64)
        indices = np.ascontiguousarray(indices, np.int32)
        pairs_coo = np.ascontiguousarray(pairs_coo, np.int32)
        bp = np.zeros((B, 2), np.int32)
        bn = np.zeros((B, self.cfg.W), np.int32)
        return self.L.oracle_train(ctypes.byref(self.cfg), ctypes.byref(self.st), _p(indptr),
                                   _p(indices), _p(pairs_coo), indices.shape[0], B,
                                   n_steps, seed & 0xFFFFFFFFFFFFFFFF, _p(bp), _p(bn))

    def train_mt(self, indptr, indices, pairs_coo, B, n_steps, seed, n_threads):
        """oracle_train's work unit on n_threads cores (BPR / AMF only)."""
        indptr = np.ascontiguousarray(indptr, np.int64)
        indices = np.ascontiguousarray(indices, np.int32)
        pairs_coo = np.ascontiguousarray(pairs_coo, np.int32)
        bp = np.zeros((B, 2), np.int32)
        bn = np.zeros((B, self.cfg.W), np.int32)
        r = self.L.oracle_train_mt(ctypes.byref(self.cfg), ctypes.byref(self.st), _p(indptr),
                                   _p(indices), _p(pairs_coo), indices.shape[0], B, n_steps,
                                   seed & 0xFFFFFFFFFFFFFFFF, _p(bp), _p(bn), int(n_threads))
        if r < 0:
            raise ValueError("oracle_train_mt covers BPR / AMF only")
        return r


if __name__ == "__main__":
    build()
