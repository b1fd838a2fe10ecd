"""ctypes binding of the CPU parity oracle (oracle/liboracle_kkt.so).

Test infrastructure only: tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg are the
only callers.  The oracle restates the MUMPS 5.8.0 semantics that Uno configures in
uno/ingredients/subproblem_solvers/MUMPS/MUMPSSolver.cpp:16-36,82 (see oracle/kkt_oracle.h).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_ROOT = os.path.dirname(_HERE)
_LIB_PATH = os.path.join(_ROOT, "oracle", "liboracle_kkt.so")
_lib = None

_i64p = ctypes.POINTER(ctypes.c_int64)
_f64p = ctypes.POINTER(ctypes.c_double)


def _load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(_LIB_PATH):
        subprocess.run(["make", "-s", "-C", os.path.join(_ROOT, "oracle")], check=True)
    lib = ctypes.CDLL(_LIB_PATH)
    lib.oracle_kkt_create.restype = ctypes.c_void_p
    lib.oracle_kkt_destroy.argtypes = [ctypes.c_void_p]
    lib.oracle_kkt_set_option.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_double]
    lib.oracle_kkt_analyze.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, _i64p, _i64p]
    lib.oracle_kkt_factorize.argtypes = [ctypes.c_void_p, _f64p]
    lib.oracle_kkt_inertia.argtypes = [ctypes.c_void_p, _i64p, _i64p, _i64p]
    lib.oracle_kkt_solve.argtypes = [ctypes.c_void_p, _f64p, _f64p]
    lib.oracle_kkt_stats.argtypes = [ctypes.c_void_p, _f64p]
    lib.oracle_kkt_scaling.argtypes = [ctypes.c_void_p, _f64p, _f64p]
    lib.oracle_kkt_last_error.argtypes = [ctypes.c_void_p]
    lib.oracle_kkt_last_error.restype = ctypes.c_char_p
    _lib = lib
    return lib


def _i64(a):
    a = np.ascontiguousarray(a, dtype=np.int64)
    return a, a.ctypes.data_as(_i64p)


def _f64(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_f64p)


class OracleKKT:
    """CPU oracle with the same analyze / factorize / inertia / solve contract as the C-ABI."""

    def __init__(self, **options):
        self.lib = _load()
        self.h = self.lib.oracle_kkt_create()
        for k, v in options.items():
            self._check(self.lib.oracle_kkt_set_option(self.h, k.encode(), float(v)))
        self.n = 0

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.oracle_kkt_destroy(self.h)
            self.h = None

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(self.lib.oracle_kkt_last_error(self.h).decode())

    def analyze(self, n, rows, cols):
        r, rp = _i64(rows)
        c, cp = _i64(cols)
        self.n = int(n)
        self._check(self.lib.oracle_kkt_analyze(self.h, self.n, len(r), rp, cp))

    def factorize(self, values):
        v, vp = _f64(values)
        self._check(self.lib.oracle_kkt_factorize(self.h, vp))

    def inertia(self):
        p, q, z = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.oracle_kkt_inertia(self.h, ctypes.byref(p), ctypes.byref(q), ctypes.byref(z)))
        return (p.value, q.value, z.value)

    def solve(self, rhs):
        b, bp = _f64(rhs)
        x = np.zeros(self.n, dtype=np.float64)
        self._check(self.lib.oracle_kkt_solve(self.h, bp, x.ctypes.data_as(_f64p)))
        return x

    def stats(self):
        out = np.zeros(7, dtype=np.float64)
        self.lib.oracle_kkt_stats(self.h, out.ctypes.data_as(_f64p))
        keys = ["nnz_L", "supernodes", "pivots_2x2", "delayed", "null_pivots", "flops", "max_front"]
        return dict(zip(keys, out.tolist()))


def _scaling(self):
    """(scale by original index, null-pivot threshold) of the last factorization."""
    sc = np.empty(self.n)
    th = ctypes.c_double()
    self._check(self.lib.oracle_kkt_scaling(self.h, sc.ctypes.data_as(_f64p), ctypes.byref(th)))
    return sc, th.value


OracleKKT.scaling = _scaling
