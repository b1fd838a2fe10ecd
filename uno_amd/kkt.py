"""ctypes binding of the MI355X KKT backend (uno_amd/libuno_kkt.so, C ABI in include/uno_kkt.h).

This is the Python-side mirror of Uno's linear-solver plugin surface, used by the tests and by
bench.py; the production drop-in is the C++ adapter in integration/ (see INTEGRATION.md).  Method
names follow uno/ingredients/subproblem_solvers/DirectSymmetricIndefiniteLinearSolver.hpp:11-25 and
uno/ingredients/subproblem_solvers/SymmetricIndefiniteLinearSolver.hpp:20-33.

There is no CPU fallback: if the HIP library is missing or no GPU is visible, every call raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# UNO_KKT_LIB: an A/B build of the library elsewhere (experiments only; the tests and the bench use the in-tree one)
LIB_PATH = os.environ.get("UNO_KKT_LIB") or os.path.join(_HERE, "libuno_kkt.so")
GEN_PATH = os.path.join(_HERE, "libarrowband.so")

UNO_KKT_OK = 0
UNO_KKT_ERR_ARG = -1
_ERR_NAMES = {-1: "ERR_ARG", -2: "ERR_STATE", -3: "ERR_HIP", -4: "ERR_PIVOT", -5: "ERR_NOMEM", -6: "ERR_NODEVICE"}

_i64p = ctypes.POINTER(ctypes.c_int64)
_f64p = ctypes.POINTER(ctypes.c_double)


class KKTStats(ctypes.Structure):
    _fields_ = [
        ("n", ctypes.c_int64), ("nnz", ctypes.c_int64), ("nnz_unique", ctypes.c_int64), ("nnz_L", ctypes.c_int64),
        ("n_fronts", ctypes.c_int64), ("n_levels", ctypes.c_int64), ("max_front", ctypes.c_int64),
        ("n_dense", ctypes.c_int64), ("pivots_2x2", ctypes.c_int64), ("pivots_null", ctypes.c_int64),
        ("pivots_relaxed", ctypes.c_int64), ("factorizations", ctypes.c_int64), ("solves", ctypes.c_int64),
        ("flops", ctypes.c_double), ("analysis_seconds", ctypes.c_double), ("bytes_L", ctypes.c_double),
        ("bytes_cb", ctypes.c_double), ("fronts_merged", ctypes.c_int64), ("solve_grid", ctypes.c_int64),
        ("solve_aborts", ctypes.c_int64), ("factor_df_fronts", ctypes.c_int64), ("factor_df_aborts", ctypes.c_int64),
        ("refinements", ctypes.c_int64), ("refinements_skipped", ctypes.c_int64), ("last_backward_error", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


EXPORTED_SYMBOLS = [
    "uno_kkt_create", "uno_kkt_destroy", "uno_kkt_set_option", "uno_kkt_analyze", "uno_kkt_factorize",
    "uno_kkt_set_values", "uno_kkt_fill_values", "uno_kkt_factorize_update", "uno_kkt_inertia", "uno_kkt_solve", "uno_kkt_stats",
    "uno_kkt_kernel_times", "uno_kkt_reset_kernel_times", "uno_kkt_stream", "uno_kkt_last_error",
    "uno_kkt_version", "uno_kkt_comm_unique_id", "uno_kkt_attach_rccl", "uno_kkt_group_create",
    "uno_kkt_group_destroy", "uno_kkt_attach_local", "uno_kkt_dist_info", "uno_kkt_rhs_setup",
    "uno_kkt_assemble_rhs", "uno_kkt_assemble_direction", "uno_kkt_symv", "uno_kkt_quadratic_product",
    "uno_kkt_barrier_setup", "uno_kkt_barrier_count", "uno_kkt_assemble_barrier", "uno_kkt_attach_host",
    "uno_kkt_stage_values", "uno_kkt_augmented_setup", "uno_kkt_assemble_augmented",
]


class KKTDistInfo(ctypes.Structure):
    _fields_ = [
        ("rank", ctypes.c_int64), ("world", ctypes.c_int64), ("subtrees", ctypes.c_int64),
        ("top_fronts", ctypes.c_int64), ("my_fronts", ctypes.c_int64), ("own_rows", ctypes.c_int64),
        ("top_rows", ctypes.c_int64), ("my_flops", ctypes.c_double), ("top_flops", ctypes.c_double),
        ("est_imbalance", ctypes.c_double), ("partitioned", ctypes.c_int64), ("est_efficiency", ctypes.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}

_lib = None


def load_library():
    """Load libuno_kkt.so (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(LIB_PATH)
    vp = ctypes.c_void_p
    lib.uno_kkt_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    lib.uno_kkt_destroy.argtypes = [vp]
    lib.uno_kkt_destroy.restype = None
    lib.uno_kkt_set_option.argtypes = [vp, ctypes.c_char_p, ctypes.c_double]
    lib.uno_kkt_analyze.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, _i64p, _i64p]
    lib.uno_kkt_factorize.argtypes = [vp, ctypes.c_void_p, ctypes.c_int]
    lib.uno_kkt_factorize_update.argtypes = [vp, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
    lib.uno_kkt_stage_values.argtypes = [vp, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
    lib.uno_kkt_set_values.argtypes = [vp, _i64p, _f64p, ctypes.c_int64]
    lib.uno_kkt_fill_values.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_double]
    lib.uno_kkt_inertia.argtypes = [vp, _i64p, _i64p, _i64p]
    lib.uno_kkt_solve.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int]
    lib.uno_kkt_stats.argtypes = [vp, ctypes.POINTER(KKTStats)]
    lib.uno_kkt_kernel_times.argtypes = [vp, ctypes.c_char_p, ctypes.c_int, _f64p, _i64p, ctypes.c_int]
    lib.uno_kkt_reset_kernel_times.argtypes = [vp]
    lib.uno_kkt_stream.argtypes = [vp]
    lib.uno_kkt_stream.restype = ctypes.c_void_p
    lib.uno_kkt_last_error.argtypes = [vp]
    lib.uno_kkt_last_error.restype = ctypes.c_char_p
    lib.uno_kkt_version.restype = ctypes.c_char_p
    lib.uno_kkt_comm_unique_id.argtypes = [ctypes.c_char_p]
    lib.uno_kkt_attach_rccl.argtypes = [vp, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
    lib.uno_kkt_group_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    lib.uno_kkt_group_destroy.argtypes = [vp]
    lib.uno_kkt_group_destroy.restype = None
    lib.uno_kkt_attach_local.argtypes = [vp, vp, ctypes.c_int]
    lib.uno_kkt_dist_info.argtypes = [vp, ctypes.POINTER(KKTDistInfo)]
    lib.uno_kkt_attach_host.argtypes = [vp, ctypes.POINTER(HostCommStruct), ctypes.c_int, ctypes.c_int]
    lib.uno_kkt_debug_scaling.argtypes = [vp, _f64p, _f64p]
    lib.uno_kkt_debug_comm_trace.argtypes = [vp, _i64p, ctypes.c_int64, ctypes.c_int]
    lib.uno_kkt_debug_comm_trace.restype = ctypes.c_int64
    lib.uno_kkt_barrier_setup.argtypes = [vp, ctypes.c_int64, _f64p, _f64p]
    lib.uno_kkt_barrier_count.argtypes = [vp]
    lib.uno_kkt_barrier_count.restype = ctypes.c_int64
    lib.uno_kkt_assemble_barrier.argtypes = [vp, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.uno_kkt_augmented_setup.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64]
    lib.uno_kkt_assemble_augmented.argtypes = [vp, ctypes.c_double, vp, vp, vp, vp, vp, vp]
    lib.uno_kkt_debug_partition.argtypes = [ctypes.c_int64, ctypes.c_int64, _i64p, _i64p, ctypes.c_int,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, _i64p]
    lib.uno_kkt_debug_partition.restype = ctypes.c_int64
    lib.uno_kkt_debug_partition_gate.argtypes = [ctypes.c_int64, ctypes.c_int64, _i64p, _i64p, ctypes.c_int, ctypes.c_double,
                                                 _f64p, _i64p]
    lib.uno_kkt_rhs_setup.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _i64p, _i64p]
    lib.uno_kkt_assemble_rhs.argtypes = [vp, vp, vp, vp, vp, vp]
    lib.uno_kkt_assemble_direction.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp, vp, vp, vp,
                                               ctypes.c_double, ctypes.c_double, vp, vp, vp, vp, _f64p]
    lib.uno_kkt_symv.argtypes = [vp, vp, vp]
    lib.uno_kkt_quadratic_product.argtypes = [vp, vp, vp, _f64p]
    _lib = lib
    return lib


class KKTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"uno_kkt {_ERR_NAMES.get(code, code)}: {msg}")
        self.code = code


def _i64(a):
    a = np.ascontiguousarray(a, dtype=np.int64)
    return a, a.ctypes.data_as(_i64p)


def _f64(a):
    a = np.ascontiguousarray(a, dtype=np.float64)
    return a, a.ctypes.data_as(_f64p)


class HipKKT:
    """Thin object over one uno_kkt handle (analyze / factorize / inertia / solve)."""

    def __init__(self, device=0, **options):
        self.lib = load_library()
        h = ctypes.c_void_p()
        rc = self.lib.uno_kkt_create(ctypes.byref(h), int(device))
        if rc != UNO_KKT_OK:
            raise KKTError(rc, "uno_kkt_create failed (no HIP device?)")
        self.h = h
        self.n = 0
        for k, v in options.items():
            self.set_option(k, v)

    def close(self):
        if getattr(self, "h", None):
            self.lib.uno_kkt_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def _check(self, rc):
        if rc != UNO_KKT_OK:
            raise KKTError(rc, self.lib.uno_kkt_last_error(self.h).decode())

    def set_option(self, name, value):
        self._check(self.lib.uno_kkt_set_option(self.h, name.encode(), float(value)))

    def analyze(self, n, rows, cols):
        r, rp = _i64(rows)
        c, cp = _i64(cols)
        if len(r) != len(c):
            raise ValueError("rows and cols differ in length")
        self.n = int(n)
        self._check(self.lib.uno_kkt_analyze(self.h, self.n, len(r), rp, cp))

    def factorize(self, values=None, device_ptr=None):
        """values: host array (COO order), or device_ptr (int address), or neither (reuse)."""
        if device_ptr is not None:
            self._check(self.lib.uno_kkt_factorize(self.h, ctypes.c_void_p(int(device_ptr)), 1))
        elif values is not None:
            v, vp = _f64(values)
            # the previous array may still be page-locked by the library (option pin_host_values): it stays
            # referenced until the call has unregistered it, so it is never freed while registered
            prev, self._v_keep = getattr(self, "_v_keep", None), v
            self._check(self.lib.uno_kkt_factorize(self.h, v.ctypes.data_as(ctypes.c_void_p), 0))
            del prev
        else:
            self._check(self.lib.uno_kkt_factorize(self.h, None, 0))

    def factorize_update(self, values, first, count):
        """Refactorize after a host edit of positions [first, first+count) of `values` (the array of the
        previous host factorization): only that range is uploaded."""
        v, _ = _f64(values)
        # the library may page-lock this buffer (pin_host_values) and copies from it asynchronously: it stays
        # referenced until the factorization has been queried (inertia) -- _in_flight
        self._in_flight().append(v)
        self._check(self.lib.uno_kkt_factorize_update(self.h, v.ctypes.data_as(ctypes.c_void_p), int(first), int(count)))

    def stage_values(self, values, first, count):
        """Asynchronous upload of values[first, first+count) (host array, COO order); the next factorize()
        without arguments factors the staged values (uno_kkt_stage_values)."""
        v, _ = _f64(values)
        # every staged chunk's source (a converted temporary for a non-float64 / non-contiguous input) stays
        # referenced until the factorization that reads it has been queried: the copies are asynchronous
        self._in_flight().append(v)
        self._check(self.lib.uno_kkt_stage_values(self.h, v.ctypes.data_as(ctypes.c_void_p), int(first), int(count)))

    def _in_flight(self):
        if not hasattr(self, "_v_in_flight"):
            self._v_in_flight = []
        return self._v_in_flight

    def fill_values(self, first, count, value):
        self._check(self.lib.uno_kkt_fill_values(self.h, int(first), int(count), float(value)))

    def set_values(self, positions, values):
        p, pp = _i64(positions)
        v, vp = _f64(values)
        self._check(self.lib.uno_kkt_set_values(self.h, pp, vp, len(p)))

    def inertia(self):
        p, q, z = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.uno_kkt_inertia(self.h, ctypes.byref(p), ctypes.byref(q), ctypes.byref(z)))
        self._factor_consumed()
        return (p.value, q.value, z.value)

    def _factor_consumed(self):
        """The factorization is complete (inertia / solve waited for it): its staged / updated sources were
        consumed.  A buffer the library page-locked stays referenced by _v_keep / the list's last entry until
        another one replaces it."""
        if getattr(self, "_v_in_flight", None):
            self._v_in_flight = self._v_in_flight[-1:]

    def solve(self, rhs):
        b, _ = _f64(rhs)
        x = np.zeros(self.n, dtype=np.float64)
        self._check(self.lib.uno_kkt_solve(self.h, b.ctypes.data_as(ctypes.c_void_p),
                                           x.ctypes.data_as(ctypes.c_void_p), 0))
        self._factor_consumed()
        return x

    def solve_device(self, rhs_ptr, x_ptr):
        self._check(self.lib.uno_kkt_solve(self.h, ctypes.c_void_p(int(rhs_ptr)), ctypes.c_void_p(int(x_ptr)), 1))
        self._factor_consumed()  # uno_kkt_solve finishes the queued factorization before it enqueues the solve

    def debug_comm_trace(self, clear=False):
        """Transport calls recorded since the last clear (option comm_trace=1): list of (op, peer, bytes, redop),
        op in send / recv / allreduce / broadcast / group_begin / group_end; before every send / recv / collective an
        ("order", on_main_stream, unjoined_side_streams_mask, -1) record; None without a traced transport."""
        k = int(self.lib.uno_kkt_debug_comm_trace(self.h, None, 0, 0))
        if k < 0:
            return None
        buf = np.zeros(4 * max(k, 1), dtype=np.int64)
        self.lib.uno_kkt_debug_comm_trace(self.h, buf.ctypes.data_as(_i64p), len(buf), 1 if clear else 0)
        names = ("send", "recv", "allreduce", "broadcast", "group_begin", "group_end", "order")
        return [(names[int(buf[4 * i])], int(buf[4 * i + 1]), int(buf[4 * i + 2]), int(buf[4 * i + 3])) for i in range(k)]

    def debug_scaling(self):
        """(scale by original index, ||A_pre||_inf) of the last factorization (uno_kkt_debug.h)."""
        sc = np.empty(self.n)
        an = ctypes.c_double()
        self._check(self.lib.uno_kkt_debug_scaling(self.h, sc.ctypes.data_as(_f64p), ctypes.byref(an)))
        return sc, an.value

    def barrier_setup(self, lb, ub):
        """Bounds of the variables (host), PrimalDualInteriorPointProblem.cpp:56-78; returns the number of
        barrier diagonal entries."""
        lb, lbp = _f64(lb)
        ub, ubp = _f64(ub)
        self._check(self.lib.uno_kkt_barrier_setup(self.h, len(lb), lbp, ubp))
        return int(self.lib.uno_kkt_barrier_count(self.h))

    def assemble_barrier(self, x_ptr, zl_ptr, zu_ptr, values_ptr):
        """Sigma into the COO values at values_ptr (all DEVICE addresses)."""
        self._check(self.lib.uno_kkt_assemble_barrier(self.h, ctypes.c_void_p(int(x_ptr)), ctypes.c_void_p(int(zl_ptr)),
                                                      ctypes.c_void_p(int(zu_ptr)), ctypes.c_void_p(int(values_ptr))))

    def augmented_setup(self, reg_size, nnz_hess, nnz_jac):
        """Segment lengths of the augmented COO values (after barrier_setup), uno_kkt_augmented_setup."""
        self._check(self.lib.uno_kkt_augmented_setup(self.h, int(reg_size), int(nnz_hess), int(nnz_jac)))

    def assemble_augmented(self, hess_scale, hess_ptr, jac_ptr, x_ptr, zl_ptr, zu_ptr, values_ptr):
        """The whole COO value array in Uno's insertion order on the device (Subproblem::assemble_augmented_matrix):
        0 on the regularization diagonal, hess_scale * hess, Sigma, jac.  DEVICE addresses (0 for an empty segment)."""
        P = lambda a: ctypes.c_void_p(int(a)) if a else None
        self._check(self.lib.uno_kkt_assemble_augmented(self.h, float(hess_scale), P(hess_ptr), P(jac_ptr), P(x_ptr),
                                                        P(zl_ptr), P(zu_ptr), P(values_ptr)))

    def stats(self):
        s = KKTStats()
        self._check(self.lib.uno_kkt_stats(self.h, ctypes.byref(s)))
        return s.as_dict()

    def stream(self):
        return self.lib.uno_kkt_stream(self.h)

    def kernel_times(self):
        names = ctypes.create_string_buffer(512)
        ms = np.zeros(16, dtype=np.float64)
        cnt = np.zeros(16, dtype=np.int64)
        k = self.lib.uno_kkt_kernel_times(self.h, names, 512, ms.ctypes.data_as(_f64p), cnt.ctypes.data_as(_i64p), 16)
        keys = names.value.decode().split(",")
        return {keys[i]: (float(ms[i]), int(cnt[i])) for i in range(k)}

    def reset_kernel_times(self):
        self._check(self.lib.uno_kkt_reset_kernel_times(self.h))

    # ---- device-side vector work (A10, A11, A15); vector arguments are device addresses (int) ----
    def rhs_setup(self, n_vars, n_cons, jac_con, jac_var):
        c, cp = _i64(jac_con)
        v, vpp = _i64(jac_var)
        self._check(self.lib.uno_kkt_rhs_setup(self.h, int(n_vars), int(n_cons), len(c), cp, vpp))

    def assemble_rhs(self, grad, cons, y, jac_values, rhs):
        P = lambda a: ctypes.c_void_p(int(a))
        self._check(self.lib.uno_kkt_assemble_rhs(self.h, P(grad), P(cons), P(y), P(jac_values), P(rhs)))

    def assemble_direction(self, n_vars, n_cons, solution, x, lb, ub, zl, zu, mu, tau_min, dx, dy, dzl, dzu):
        P = lambda a: ctypes.c_void_p(int(a))
        steps = np.zeros(2)
        self._check(self.lib.uno_kkt_assemble_direction(self.h, int(n_vars), int(n_cons), P(solution), P(x), P(lb), P(ub),
                                                        P(zl), P(zu), float(mu), float(tau_min), P(dx), P(dy), P(dzl),
                                                        P(dzu), steps.ctypes.data_as(_f64p)))
        return float(steps[0]), float(steps[1])

    def symv(self, x_ptr, y_ptr):
        self._check(self.lib.uno_kkt_symv(self.h, ctypes.c_void_p(int(x_ptr)), ctypes.c_void_p(int(y_ptr))))

    def quadratic_product(self, x_ptr, y_ptr):
        r = ctypes.c_double()
        self._check(self.lib.uno_kkt_quadratic_product(self.h, ctypes.c_void_p(int(x_ptr)), ctypes.c_void_p(int(y_ptr)),
                                                       ctypes.byref(r)))
        return r.value

    # ---- multi-GPU (one factorization partitioned over ranks; attach before analyze) ----
    def attach_rccl(self, unique_id, rank, world):
        self._check(self.lib.uno_kkt_attach_rccl(self.h, bytes(unique_id), int(rank), int(world)))

    def attach_local(self, group, rank):
        self._check(self.lib.uno_kkt_attach_local(self.h, group.g, int(rank)))

    def attach_host(self, comm, rank, world):
        """Host-staged transport (uno_kkt_attach_host) driven by `comm` (e.g. GlooComm); one process per rank."""
        self._host_comm = comm  # the callbacks must outlive the handle
        self._check(self.lib.uno_kkt_attach_host(self.h, ctypes.byref(comm.struct), int(rank), int(world)))

    def dist_info(self):
        d = KKTDistInfo()
        self._check(self.lib.uno_kkt_dist_info(self.h, ctypes.byref(d)))
        return d.as_dict()


def rccl_unique_id():
    """ncclGetUniqueId (128 bytes) for uno_kkt_attach_rccl; call on rank 0 and share out of band."""
    lib = load_library()
    buf = ctypes.create_string_buffer(128)
    rc = lib.uno_kkt_comm_unique_id(buf)
    if rc != UNO_KKT_OK:
        raise KKTError(rc, "ncclGetUniqueId failed")
    return buf.raw


_CB_SEND = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)
_CB_GROUP_END = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p)


class HostCommStruct(ctypes.Structure):
    """uno_kkt_host_comm_t (include/uno_kkt.h)"""
    _fields_ = [("ctx", ctypes.c_void_p), ("send", _CB_SEND), ("recv", _CB_SEND), ("group_end", _CB_GROUP_END),
                ("allreduce", _CB_SEND), ("broadcast", _CB_SEND)]


class GlooComm:
    """Host-staged exchange of uno_kkt_attach_host over torch.distributed (gloo backend, an initialised
    default group): send / recv post isend / irecv on the staged host buffer, group_end waits for them,
    allreduce / broadcast are the blocking collectives (8-byte elements; u64 values are bit patterns of
    non-negative doubles or counters, below 2^63, so int64 arithmetic is exact)."""

    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group, self.pending = torch, dist, group, []

        def view(buf, nbytes, dtype):
            raw = (ctypes.c_uint8 * nbytes).from_address(buf)
            return torch.frombuffer(raw, dtype=dtype)

        def guard(fn):
            def run(*a):
                try:
                    fn(*a)
                    return 0
                except Exception as e:  # noqa: BLE001 -- reported to the library as a failed exchange
                    import sys
                    print(f"[GlooComm] {e!r}", file=sys.stderr)
                    return -1
            return run

        def send(ctx, buf, nbytes, peer):
            t = view(buf, nbytes, torch.uint8)
            self.pending.append((dist.isend(t, int(peer), group=self.group), t))

        def recv(ctx, buf, nbytes, peer):
            t = view(buf, nbytes, torch.uint8)
            self.pending.append((dist.irecv(t, int(peer), group=self.group), t))

        def group_end(ctx):
            for w, _ in self.pending:
                w.wait()
            self.pending.clear()

        def allreduce(ctx, buf, count, op):
            t = view(buf, 8 * count, torch.int64 if op in (0, 1) else torch.float64)
            ro = dist.ReduceOp.SUM if op in (0, 3) else dist.ReduceOp.MAX
            dist.all_reduce(t, op=ro, group=self.group)

        def broadcast(ctx, buf, nbytes, root):
            dist.broadcast(view(buf, nbytes, torch.uint8), int(root), group=self.group)

        self._cbs = (_CB_SEND(guard(send)), _CB_SEND(guard(recv)), _CB_GROUP_END(guard(group_end)),
                     _CB_SEND(guard(allreduce)), _CB_SEND(guard(broadcast)))
        self.struct = HostCommStruct(None, *self._cbs)


class LocalGroup:
    """In-process group of `world` ranks (one host thread per rank, e.g. several ranks on one GPU)."""

    def __init__(self, world):
        self.lib = load_library()
        self.g = ctypes.c_void_p()
        rc = self.lib.uno_kkt_group_create(ctypes.byref(self.g), int(world))
        if rc != UNO_KKT_OK:
            raise KKTError(rc, "group create failed")
        self.world = int(world)

    def close(self):
        if getattr(self, "g", None):
            self.lib.uno_kkt_group_destroy(self.g)
            self.g = None

    def __del__(self):
        self.close()


def debug_partition(n, rows, cols, world):
    """Host-only analysis + subtree partition: (owner per front (-1 = top), parent per front, subtrees)."""
    lib = load_library()
    r, rp = _i64(rows)
    c, cp = _i64(cols)
    cap = max(16, int(n))
    owner = np.zeros(cap, dtype=np.int32)
    parent = np.zeros(cap, dtype=np.int32)
    ns = ctypes.c_int64()
    nf = lib.uno_kkt_debug_partition(int(n), len(r), rp, cp, int(world), owner.ctypes.data_as(ctypes.c_void_p),
                                     parent.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(ns))
    if nf < 0:
        raise KKTError(UNO_KKT_ERR_ARG if nf == -1 else nf, "debug_partition failed")
    return owner[:nf].copy(), parent[:nf].copy(), ns.value


def debug_partition_gate(n, rows, cols, world, min_efficiency=0.5):
    """Host-only: (partition?, estimated efficiency, subtrees) of the multi-GPU gate of uno_kkt_analyze."""
    lib = load_library()
    r, rp = _i64(rows)
    c, cp = _i64(cols)
    eff, ns = ctypes.c_double(), ctypes.c_int64()
    rc = lib.uno_kkt_debug_partition_gate(int(n), len(r), rp, cp, int(world), float(min_efficiency), ctypes.byref(eff),
                                          ctypes.byref(ns))
    if rc < 0:
        raise KKTError(UNO_KKT_ERR_ARG, "debug_partition_gate failed")
    return bool(rc), eff.value, ns.value


# ---------------------------------------------------------------------------------------------
# Uno plugin-surface mirror (names as in the reference)
# ---------------------------------------------------------------------------------------------

class SparseSymmetricMatrix:
    """Mirror of SparseSymmetricMatrix<COOFormat<size_t,double>> (uno/linear_algebra/COOFormat.hpp:19-141):
    regularization diagonal inserted first by reset(), insert() appends, set_regularization()
    overwrites entries[index + offset], duplicates kept (summed by the solver)."""

    def __init__(self, dimension, capacity, regularization_size):
        self._dimension = int(dimension)
        self.regularization_size = int(regularization_size)
        self.capacity = int(capacity) + self.regularization_size
        self.reset()

    def reset(self):
        r = self.regularization_size
        self.rows = list(range(r))
        self.cols = list(range(r))
        self.entries = [0.0] * r

    def dimension(self):
        return self._dimension

    def number_nonzeros(self):
        return len(self.entries)

    def insert(self, row_index, column_index, term):
        self.rows.append(int(row_index))
        self.cols.append(int(column_index))
        self.entries.append(float(term))

    def finalize_column(self, column_index):
        pass

    def set_regularization(self, indices, offset, factor):
        for i in indices:
            self.entries[i + offset] = float(factor)

    def smallest_diagonal_entry(self, max_dimension):
        d = np.zeros(max_dimension)
        for r, c, v in zip(self.rows, self.cols, self.entries):
            if r == c and r < max_dimension:
                d[r] += v
        return float(d.min())

    def arrays(self):
        return (np.asarray(self.rows, dtype=np.int64), np.asarray(self.cols, dtype=np.int64),
                np.asarray(self.entries, dtype=np.float64))

    def product(self, x):
        """SymmetricMatrix::product (uno/linear_algebra/SymmetricMatrix.hpp:100-109)."""
        r, c, v = self.arrays()
        y = np.zeros(self._dimension)
        np.add.at(y, r, v * x[c])
        off = r != c
        np.add.at(y, c[off], v[off] * x[r[off]])
        return y


class HipLDLSolver:
    """Mirror of DirectSymmetricIndefiniteLinearSolver<size_t,double> backed by the GPU
    (the C++ adapter integration/HIPLDLSolver.cpp is the production form)."""

    def __init__(self, device=0, **options):
        self.kkt = HipKKT(device, **options)
        self.dimension = 0

    def initialize_memory(self, number_variables, number_constraints, number_hessian_nonzeros, regularization_size):
        self.dimension = number_variables + number_constraints

    def do_symbolic_analysis(self, matrix):
        r, c, _ = matrix.arrays()
        self.kkt.analyze(matrix.dimension(), r, c)

    def do_numerical_factorization(self, matrix):
        self.kkt.factorize(matrix.arrays()[2])

    def solve_indefinite_system(self, matrix, rhs, result=None):
        x = self.kkt.solve(np.asarray(rhs, dtype=np.float64))
        if result is not None:
            result[:] = x
        return x

    def get_inertia(self):
        return self.kkt.inertia()

    def number_negative_eigenvalues(self):
        return self.kkt.inertia()[1]

    def number_zero_eigenvalues(self):
        return self.kkt.inertia()[2]

    def matrix_is_singular(self):
        return self.number_zero_eigenvalues() > 0

    def rank(self):
        return self.kkt.n - self.number_zero_eigenvalues()


class UnstableRegularization(RuntimeError):
    """uno/ingredients/regularization_strategies/UnstableRegularization.hpp:10-15"""


def regularize_augmented_matrix(matrix, primal_indices, dual_indices, dual_regularization_parameter,
                                expected_inertia, linear_solver, state, options=None, trace=None):
    """Mirror of PrimalDualRegularization::regularize_augmented_matrix
    (uno/ingredients/regularization_strategies/PrimalDualRegularization.hpp:133-219) with the
    default option values (uno/options/DefaultOptions.cpp).  `state` carries
    previous_primal_regularization and symbolic_analysis_performed across calls."""
    o = dict(regularization_failure_threshold=1e40, primal_regularization_initial_factor=1e-4,
             dual_regularization_fraction=1e-8, primal_regularization_lb=1e-20,
             primal_regularization_decrease_factor=3.0, primal_regularization_fast_increase_factor=100.0,
             primal_regularization_slow_increase_factor=8.0, threshold_unsuccessful_attempts=8)
    if options:
        o.update(options)
    primal, dual = 0.0, 0.0
    attempts = 1
    if not state.get("symbolic_analysis_performed"):
        linear_solver.do_symbolic_analysis(matrix)
        state["symbolic_analysis_performed"] = True
    linear_solver.do_numerical_factorization(matrix)
    inertia = tuple(linear_solver.get_inertia())
    if trace is not None:
        trace.append((primal, dual, inertia))
    if inertia == tuple(expected_inertia):
        return primal, dual, attempts
    if linear_solver.matrix_is_singular():
        dual = o["dual_regularization_fraction"] * dual_regularization_parameter
    prev = state.get("previous_primal_regularization", 0.0)
    if prev == 0.0:
        primal = o["primal_regularization_initial_factor"]
    else:
        primal = max(o["primal_regularization_lb"], prev / o["primal_regularization_decrease_factor"])
    matrix.set_regularization(primal_indices, 0, primal)
    matrix.set_regularization(dual_indices, len(primal_indices), -dual)
    while True:
        linear_solver.do_numerical_factorization(matrix)
        attempts += 1
        inertia = tuple(linear_solver.get_inertia())
        if trace is not None:
            trace.append((primal, dual, inertia))
        if inertia == tuple(expected_inertia):
            state["previous_primal_regularization"] = primal
            return primal, dual, attempts
        if prev == 0.0 or o["threshold_unsuccessful_attempts"] < attempts:
            primal *= o["primal_regularization_fast_increase_factor"]
        else:
            primal *= o["primal_regularization_slow_increase_factor"]
        if primal <= o["regularization_failure_threshold"]:
            matrix.set_regularization(primal_indices, 0, primal)
            matrix.set_regularization(dual_indices, len(primal_indices), -dual)
        else:
            raise UnstableRegularization()


# ---------------------------------------------------------------------------------------------
# synthetic inputs
# ---------------------------------------------------------------------------------------------

_gen = None

SEEDS = {"C2": 0x5EED0002, "C3": 0x5EED0003, "C5": 0x5EED0005}


def _load_gen():
    global _gen
    if _gen is None:
        if not os.path.exists(GEN_PATH):
            raise RuntimeError(f"{GEN_PATH} not built")
        g = ctypes.CDLL(GEN_PATH)
        g.arrowband_size.argtypes = [ctypes.c_int64, _i64p, _i64p]
        g.arrowband_size.restype = ctypes.c_int64
        g.arrowband_generate.argtypes = [ctypes.c_int64, ctypes.c_uint64, _i64p, _i64p, _f64p]
        g.arrowband_generate.restype = ctypes.c_int64
        g.arrowband_rhs.argtypes = [ctypes.c_int64, ctypes.c_uint64, _f64p]
        g.coo_symv.argtypes = [ctypes.c_int64, ctypes.c_int64, _i64p, _i64p, _f64p, _f64p, _f64p]
        _gen = g
    return _gen


def arrowband(N, seed):
    """Return (n, nv, m, rows, cols, vals, rhs) of the arrowband KKT of dimension N."""
    g = _load_gen()
    nv, m = ctypes.c_int64(), ctypes.c_int64()
    nnz = g.arrowband_size(int(N), ctypes.byref(nv), ctypes.byref(m))
    rows = np.empty(nnz, dtype=np.int64)
    cols = np.empty(nnz, dtype=np.int64)
    vals = np.empty(nnz, dtype=np.float64)
    got = g.arrowband_generate(int(N), int(seed), rows.ctypes.data_as(_i64p), cols.ctypes.data_as(_i64p),
                               vals.ctypes.data_as(_f64p))
    if got != nnz:
        raise ValueError(f"arrowband generation failed for N={N}")
    rhs = np.empty(int(N), dtype=np.float64)
    g.arrowband_rhs(int(N), int(seed), rhs.ctypes.data_as(_f64p))
    return int(N), nv.value, m.value, rows, cols, vals, rhs


def coo_symv(n, rows, cols, vals, x):
    g = _load_gen()
    r, rp = _i64(rows)
    c, cp = _i64(cols)
    v, vp = _f64(vals)
    xx, xp = _f64(x)
    y = np.zeros(int(n), dtype=np.float64)
    g.coo_symv(int(n), len(r), rp, cp, vp, xp, y.ctypes.data_as(_f64p))
    return y
