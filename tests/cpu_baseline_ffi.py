"""ctypes binding of the multi-threaded CPU baseline (oracle/libcpu_mf.so, oracle/cpu_mf.cpp).

Baseline / test infrastructure only: bench.py's cpu_baseline leg times it on the host cores (MUMPS itself
is not available offline, BASELINE.md section 4 "Fallback"), tests/test_oracle.py checks it against the
one-thread oracle.  Same analyze / factorize / inertia / solve contract as the C-ABI."""
import ctypes
import os
import subprocess

import numpy as np

_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_LIB_PATH = os.path.join(_ROOT, "oracle", "libcpu_mf.so")
_lib = None
_i64p = ctypes.POINTER(ctypes.c_int64)
_f64p = ctypes.POINTER(ctypes.c_double)


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            subprocess.run(["make", "-s", "-C", os.path.join(_ROOT, "oracle")], check=True)
        lib = ctypes.CDLL(_LIB_PATH)
        lib.cpu_mf_create.restype = ctypes.c_void_p
        lib.cpu_mf_destroy.argtypes = [ctypes.c_void_p]
        lib.cpu_mf_analyze.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, _i64p, _i64p]
        lib.cpu_mf_factorize.argtypes = [ctypes.c_void_p, _f64p]
        lib.cpu_mf_inertia.argtypes = [ctypes.c_void_p, _i64p, _i64p, _i64p]
        lib.cpu_mf_solve.argtypes = [ctypes.c_void_p, _f64p, _f64p]
        lib.cpu_mf_last_error.argtypes = [ctypes.c_void_p]
        lib.cpu_mf_last_error.restype = ctypes.c_char_p
        _lib = lib
    return _lib


def threads():
    return int(_load().cpu_mf_threads())


class CpuMF:
    def __init__(self):
        self.lib = _load()
        self.h = self.lib.cpu_mf_create()

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.cpu_mf_destroy(self.h)
            self.h = None

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(self.lib.cpu_mf_last_error(self.h).decode())

    def analyze(self, n, rows, cols):
        self.n = int(n)
        self._r = np.ascontiguousarray(rows, dtype=np.int64)
        self._c = np.ascontiguousarray(cols, dtype=np.int64)
        self._check(self.lib.cpu_mf_analyze(self.h, self.n, len(self._r), self._r.ctypes.data_as(_i64p),
                                            self._c.ctypes.data_as(_i64p)))

    def factorize(self, values):
        self._v = np.ascontiguousarray(values, dtype=np.float64)
        self._check(self.lib.cpu_mf_factorize(self.h, self._v.ctypes.data_as(_f64p)))

    def inertia(self):
        p, q, z = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.cpu_mf_inertia(self.h, ctypes.byref(p), ctypes.byref(q), ctypes.byref(z)))
        return (p.value, q.value, z.value)

    def solve(self, rhs):
        b = np.ascontiguousarray(rhs, dtype=np.float64)
        x = np.empty(self.n)
        self._check(self.lib.cpu_mf_solve(self.h, b.ctypes.data_as(_f64p), x.ctypes.data_as(_f64p)))
        return x
