"""ctypes loader of oracle/_build/liboracle.so (TEST INFRASTRUCTURE ONLY)."""

import ctypes
import os
import subprocess
from ctypes import POINTER, c_float, c_int32, c_int64, c_uint8, c_uint32, c_uint64, c_void_p

import numpy as np

_DIR = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_DIR, "_build", "liboracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", _DIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        h = ctypes.CDLL(LIB)
        h.oracle_philox.argtypes = [c_void_p, c_uint32, c_uint32, c_void_p, c_int64]
        h.oracle_log2.argtypes = [c_float]
        h.oracle_log2.restype = c_float
        h.oracle_gumbel.argtypes = [c_float]
        h.oracle_gumbel.restype = c_float
        h.oracle_sample.argtypes = [c_void_p, c_int64, c_void_p, c_int32, c_int64, c_uint32,
                                    c_uint32, c_uint64, c_uint32, c_int32, c_void_p]
        h.oracle_gumbel_table.argtypes = [c_uint32, c_uint32, c_uint64, c_uint32, c_int64,
                                          c_int32, c_void_p]
        h.oracle_env_reset.argtypes = [c_void_p, c_int64, c_int32, c_uint32, c_uint32, c_uint32,
                                       c_void_p]
        h.oracle_env_step.argtypes = [c_void_p, c_void_p, c_int32, c_int64, c_int32, c_uint32,
                                      c_uint32, c_uint32, c_void_p, c_void_p, c_void_p]
        _lib = h
    return _lib


def _p(a):
    return a.ctypes.data_as(c_void_p)


def philox(ctr, k0, k1):
    ctr = np.ascontiguousarray(ctr, dtype=np.uint32).reshape(-1, 4)
    out = np.empty_like(ctr)
    lib().oracle_philox(_p(ctr), k0 & 0xFFFFFFFF, k1 & 0xFFFFFFFF, _p(out), ctr.shape[0])
    return out


def sample(logits, buckets, k0, k1, step, env_offset=0, sample=True):
    lg = np.ascontiguousarray(logits, dtype=np.float32)
    off = np.concatenate([[0], np.cumsum(buckets)]).astype(np.int32)
    N = lg.shape[0]
    K = len(buckets)
    out = np.empty((N, K), dtype=np.int32)
    lib().oracle_sample(_p(lg), lg.shape[1], _p(off), K, N, k0, k1, step, env_offset,
                        1 if sample else 0, _p(out))
    return out


def gumbel_table(k0, k1, step, env_offset, N, A):
    out = np.empty((N, A), dtype=np.float32)
    lib().oracle_gumbel_table(k0, k1, step, env_offset, N, A, _p(out))
    return out


class Env:
    """C twin of the synthetic dummy env."""

    def __init__(self, N, D, k0, k1, env_offset=0):
        self.N, self.D, self.k0, self.k1, self.eoff = N, D, k0, k1, env_offset
        self.state = np.zeros((N, 4), dtype=np.int32)
        self.obs = np.zeros((N, D), dtype=np.float32)
        self.rew = np.zeros(N, dtype=np.float32)
        self.done = np.zeros(N, dtype=np.uint8)

    def reset(self):
        lib().oracle_env_reset(_p(self.state), self.N, self.D, self.k0, self.k1, self.eoff,
                               _p(self.obs))
        return self.obs.copy()

    def step(self, actions):
        a = np.ascontiguousarray(actions, dtype=np.int32)
        lib().oracle_env_step(_p(self.state), _p(a), a.shape[1], self.N, self.D, self.k0,
                              self.k1, self.eoff, _p(self.obs), _p(self.rew), _p(self.done))
        return self.obs.copy(), self.rew.copy(), self.done.copy()
