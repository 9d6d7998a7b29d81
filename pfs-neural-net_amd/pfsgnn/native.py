"""ctypes binding of libpfsgnn.so (the C ABI in include/pfsgnn.h) as an op backend.

This is the only compute backend of the product.  There is no fallback: if
the shared library is missing, or the process has no MI355X visible, every
entry point raises ``NativeUnavailable`` -- the hot path never silently runs
in PyTorch or on the CPU.

Tensors are passed as raw device pointers on torch's current HIP stream, so
PyTorch is only the allocator / stream / collective plumbing here.
"""
import ctypes
import os

import torch

from .sparse import SparseEdgeOps, SparseGeo

_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpfsgnn.so")
# tuning builds (tools/variants.sh): PFSGNN_LIB_VARIANT=<name> loads
# pfsgnn/libpfsgnn_<name>.so, an in-tree build of the same sources with other
# compile-time knobs
if os.environ.get("PFSGNN_LIB_VARIANT"):
    _LIB_PATH = os.path.join(os.path.dirname(_LIB_PATH),
                             "libpfsgnn_" + os.environ["PFSGNN_LIB_VARIANT"] + ".so")
# (a test-only build elsewhere in the tree, by path: tests/native/libpfsgnn_lossexact.so)
if os.environ.get("PFSGNN_LIB_PATH"):
    _LIB_PATH = os.environ["PFSGNN_LIB_PATH"]


class NativeUnavailable(RuntimeError):
    pass


_lib = None

P = ctypes.c_void_p
I = ctypes.c_int
LL = ctypes.c_longlong
FL = ctypes.c_float
SZ = ctypes.c_size_t
ULL = ctypes.c_ulonglong


class Seg(ctypes.Structure):
    """pfsgnn_seg (include/pfsgnn.h): one row block of a concatenated node input."""
    _fields_ = [("x", ctypes.c_void_p), ("rows", ctypes.c_int), ("col", ctypes.c_int),
                ("per_graph", ctypes.c_int)]


SEGP = ctypes.POINTER(Seg)


class Red(ctypes.Structure):
    """pfsgnn_red (include/pfsgnn.h): one pending cross-block reduction."""
    _fields_ = [("part", ctypes.c_void_p), ("nb", ctypes.c_int), ("plen", ctypes.c_size_t),
                ("ldp", ctypes.c_int), ("rows", ctypes.c_int), ("cols", ctypes.c_int),
                ("out", ctypes.c_void_p), ("ldo", ctypes.c_int), ("add", ctypes.c_int),
                ("scale", ctypes.c_float)]


REDP = ctypes.POINTER(Red)


class Sliced(ctypes.Structure):
    """pfsgnn_sliced_t (include/pfsgnn.h): a general batch cut into slices of 16
    fibers for the fused edge kernels (pfsgnn_sliced.hip)."""
    _fields_ = [("fib", ctypes.c_void_p), ("base", ctypes.c_void_p), ("len", ctypes.c_void_p),
                ("cls", ctypes.c_void_p), ("pco", ctypes.c_void_p), ("EP", ctypes.c_longlong),
                ("E", ctypes.c_longlong), ("maxdeg", ctypes.c_int)]


SLP = ctypes.POINTER(Sliced)


class OSeg(ctypes.Structure):
    """pfsgnn_oseg (include/pfsgnn.h): one row block of an input-gradient output."""
    _fields_ = [("x", ctypes.c_void_p), ("rows", ctypes.c_int), ("add", ctypes.c_int)]


OSEGP = ctypes.POINTER(OSeg)


class WgJob(ctypes.Structure):
    """pfsgnn_wgrad_job (include/pfsgnn.h): one deferred weight gradient."""
    _fields_ = [("dY", ctypes.c_void_p), ("M", ctypes.c_int), ("segs", SEGP), ("nseg", ctypes.c_int),
                ("N", ctypes.c_int), ("act_in", ctypes.c_int), ("dW", ctypes.c_void_p),
                ("lddw", ctypes.c_int), ("db", ctypes.c_void_p), ("dbscale", ctypes.c_float)]


WGJP = ctypes.POINTER(WgJob)


class GemmJob(ctypes.Structure):
    """pfsgnn_gemm_job (include/pfsgnn.h): one product of a batched launch."""
    _fields_ = [("W", ctypes.c_void_p), ("ldw", ctypes.c_int), ("trans", ctypes.c_int),
                ("M", ctypes.c_int), ("K", ctypes.c_int), ("segs", SEGP), ("nseg", ctypes.c_int),
                ("N", ctypes.c_int), ("b", ctypes.c_void_p), ("bscale", ctypes.c_float),
                ("act_in", ctypes.c_int), ("Z", ctypes.c_void_p), ("Y", ctypes.c_void_p),
                ("add", ctypes.c_int)]


GMJP = ctypes.POINTER(GemmJob)


class LinMap(ctypes.Structure):
    """pfsgnn_linmap (include/pfsgnn.h): out = W[:, col0:col0+O] . Y + b."""
    _fields_ = [("W", ctypes.c_void_p), ("ldw", ctypes.c_int), ("col0", ctypes.c_int),
                ("nk", ctypes.c_int), ("b", ctypes.c_void_p), ("out", ctypes.c_void_p)]


LINMP = ctypes.POINTER(LinMap)


def _ptrs(*names):
    return [(n, ctypes.c_void_p) for n in names]


class ClassBwd(ctypes.Structure):
    """pfsgnn_class_bwd (include/pfsgnn.h): a block's class-side backward."""
    _fields_ = ([("G", I), ("NF", I), ("NC", I), ("F", I), ("pend", ctypes.c_void_p * 4),
                 ("pend_n", I * 4), ("npend", I)]
                + _ptrs("V", "w", "y1", "r1", "r2", "gZ", "gW1", "gW2") + [("gH", I)]
                + _ptrs("gu_up", "gV", "gdZ", "dwp", "gu", "g_xs", "g_xt",
                        "Yp", "mu", "var", "gamma", "Z", "W1", "W2", "Wt2")
                + [("eps", FL)]
                + _ptrs("dgamma", "dbeta", "dYp", "dZ", "gxt_in", "g_agg", "gu_t", "g_hsum"))


class BlockTail(ctypes.Structure):
    """pfsgnn_block_tail (include/pfsgnn.h): a block tail on a complete batch."""
    _fields_ = ([("G", I), ("NF", I), ("NC", I), ("F", I)]
                + _ptrs("y", "sc", "sh", "Rs", "Wt1", "Wt2", "bt2", "tmask", "hsum", "agg",
                        "xt", "u", "W1", "b1", "W2", "b2", "gamma", "beta",
                        "Z", "Yp", "rm", "rv", "xt_new", "mu", "var")
                + [("momentum", FL), ("eps", FL)]
                + _ptrs("xs", "gW1", "gb1", "gW2", "gb2", "gw")
                + [("gH", I), ("reps", FL)]
                + _ptrs("means", "gZ", "gV", "unew", "y1", "r1", "r2",
                        "We", "be", "Ws", "bs", "Pt", "Qt"))

_SIGS = {
    "pfsgnn_version": ([], ctypes.c_char_p),
    "pfsgnn_last_error": ([], ctypes.c_char_p),
    "pfsgnn_workspace_bytes": ([I, I, I, I], SZ),
    "pfsgnn_set_edge_path": ([I], I),
    "pfsgnn_sync_bytes": ([], SZ),
    "pfsgnn_set_sync_buffer": ([P, SZ], I),
    "pfsgnn_get_edge_path": ([], I),
    "pfsgnn_edge_grid": ([I, I, I, ctypes.POINTER(ctypes.c_int)], I),
    "pfsgnn_timing_enable": ([I], I),
    "pfsgnn_timing_reset": ([], I),
    "pfsgnn_timing_repeat": ([ctypes.c_char_p, I], I),
    "pfsgnn_timing_query": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_double),
                             ctypes.POINTER(ctypes.c_longlong)], I),
    "pfsgnn_lin": ([P, I, I, I, P, I, P, FL, I, P, I, P], I),
    "pfsgnn_lin_t": ([P, I, I, I, P, I, P, P, I, P], I),
    "pfsgnn_lin_gather": ([P, I, I, I, P, I, P, FL, I, P, I, P, P, I, P, P, I, P], I),
    "pfsgnn_wgrad": ([P, I, P, I, I, I, P, I, P, FL, P, SZ, P], I),
    "pfsgnn_lin_cat": ([P, I, I, SEGP, I, I, P, FL, I, P, I, P], I),
    "pfsgnn_wgrad_cat": ([P, I, SEGP, I, I, I, P, I, P, FL, P, SZ, P], I),
    "pfsgnn_wgrad_part_bytes": ([I, I, I, I], SZ),
    "pfsgnn_wgrad_cat_part": ([P, I, SEGP, I, I, I, P, I, P, FL, P, SZ, REDP,
                               ctypes.POINTER(ctypes.c_int), P], I),
    "pfsgnn_reduce_batch": ([REDP, I, P], I),
    "pfsgnn_wgrad_multi_bytes": ([WGJP, I], SZ),
    "pfsgnn_gemm_multi": ([GMJP, I, P], I),
    "pfsgnn_wgrad_multi": ([WGJP, I, P, SZ, P], I),
    "pfsgnn_defer_begin": ([P, SZ], I),
    "pfsgnn_defer_end": ([P], I),
    "pfsgnn_defer_end_multi": ([WGJP, I, P, SZ, P], I),
    "pfsgnn_defer_need": ([], SZ),
    "pfsgnn_bn_fwd": ([P, I, I, P, P, P, P, FL, FL, P, P, P, P, SZ, P], I),
    "pfsgnn_bn_bwd": ([P, P, P, P, P, FL, I, I, P, P, P, P, SZ, P], I),
    "pfsgnn_mlp_ws_bytes": ([I], SZ),
    "pfsgnn_mlp_fwd": ([SEGP, I, I, P, I, I, P, P, I, P, P, P, P, P, P, P, FL, FL, P, P, P, P,
                        SZ, P], I),
    "pfsgnn_mlp_fwd_epi": ([SEGP, I, I, P, I, I, P, P, I, P, P, P, P, P, P, P, FL, FL, P, P, P,
                            LINMP, I, P, SZ, P], I),
    "pfsgnn_target_global_fwd": ([SEGP, I, I, I, P, I, I, P, P, I, P, P, P, P, P, P, P, FL, FL,
                                  P, P, P, P, I, P, P, I, P, P, P, P, FL] + [P] * 7
                                 + [P] * 6 + [P, SZ, P], I),
    "pfsgnn_mlp_bwd": ([P, I, P, P, P, P, FL, P, P, P, P, I, I, I, P, I, P, P, OSEGP, I, P, SZ,
                        P], I),
    "pfsgnn_mlp_bwd_pre": ([P, I, P, P, P, P, FL, P, P, P, P, I, I, I, P, I, P, P, OSEGP, I, P, I,
                            P, P, I, I, I, P, SZ, P], I),
    "pfsgnn_build_complete": ([I, I, I, I, P, P], I),
    "pfsgnn_graph_reduce": ([P, I, I, I, I, P, P], I),
    "pfsgnn_graph_reduce_add": ([P, I, I, I, I, P, P], I),
    "pfsgnn_graph_bcast_add": ([P, I, I, I, P, FL, P], I),
    "pfsgnn_graph_reduce_multi": ([P, P, I, I, I, P, P], I),
    "pfsgnn_graph_mean2": ([P, I, P, I, I, I, P, P], I),
    "pfsgnn_graph_bcast_add2": ([P, I, FL, P, I, FL, I, I, P, P], I),
    "pfsgnn_rms2_fwd": ([P, I, I, P, FL, P, P, P, P, P], I),
    "pfsgnn_rms2_bwd": ([P, P, P, P, P, P, I, I, FL, P, P, P, SZ, P], I),
    "pfsgnn_global_fwd": ([P, I, P, I, P, I, I, P, I, P, P, P, P, FL] + [P] * 7 + [P], I),
    "pfsgnn_global_bwd": ([P, P, P, P, P, P, I, I, P, I, P, P, P, P, P, P, P, P, I, FL, P, I,
                           FL, P], I),
    "pfsgnn_bn2_finalize": ([P, P, P, P, P, P, I, LL, FL, FL, P, P, P, P, P], I),
    "pfsgnn_bn_eval_coef": ([P, P, P, P, I, FL, I, P, P, P], I),
    "pfsgnn_affine_rows": ([P, I, I, P, P, P, P], I),
    "pfsgnn_bn2_bwd_coef": ([P, P, P, P, P, I, LL, FL, P, P, P, P, P, P], I),
    "pfsgnn_bn2_bwd_coef_part": ([P, I, I, P, P, P, LL, FL, P, P, P, P, P, P], I),
    "pfsgnn_moment_coef": ([P, P, I, I, I, P, P], I),
    "pfsgnn_moment_coef_seg": ([P, P, I, I, P, P, P], I),
    "pfsgnn_sparse_layout_ws_bytes": ([LL], SZ),
    "pfsgnn_sparse_layout": ([P, LL, I, I, I, P, P, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_gather_cols": ([P, I, I, P, LL, P, I, P, P], I),
    "pfsgnn_segment_sum": ([P, I, LL, P, P, I, I, P, I, P], I),
    "pfsgnn_segment_moments": ([P, I, LL, P, I, P, P, P], I),
    "pfsgnn_segment_moment_grad": ([P, I, LL, P, P, P, I, P, P], I),
    "pfsgnn_rows_ws_bytes": ([I, LL], SZ),
    "pfsgnn_rows_stats": ([P, I, LL, P, P, P, SZ, P], I),
    "pfsgnn_rows_bn_sums": ([P, P, I, LL, P, P, P, P, P, SZ, P], I),
    "pfsgnn_rows_axpby": ([P, P, I, LL, P, P, P, P, P], I),
    "pfsgnn_edge_mlp_fwd": ([I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_edge_mlp_fwd_bn": ([I, I, I, I] + [P] * 15 + [FL, FL, P, P, P, P, P, SZ, P], I),
    "pfsgnn_source_fwd": ([I, I, I, I, P, P, P, P, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_target_fwd": ([I, I, I, I, P, P, P, P, P, P, P, P, FL, P, P, P, SZ, P], I),
    "pfsgnn_tmask_bytes": ([I, I, I, I], SZ),
    "pfsgnn_target_bwd": ([I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_target_bwd_bn": ([I, I, I, I] + [P] * 14 + [FL, P, P, SZ, P], I),
    "pfsgnn_source_bwd": ([I, I, I, I] + [P] * 24 + [P, SZ, P], I),
    "pfsgnn_source_bwd_bn": ([I, I, I, I] + [P] * 17 + [LL, FL] + [P] * 12 + [P, SZ, P], I),
    "pfsgnn_msg_bytes": ([I, I, I, I], SZ),
    "pfsgnn_source_fwd_msg": ([I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_source_bwd_msg": ([I, I, I, I] + [P] * 25 + [P, SZ, P], I),
    "pfsgnn_source_bwd_bn_msg": ([I, I, I, I] + [P] * 17 + [LL, FL] + [P] * 13 + [P, SZ, P], I),
    "pfsgnn_edge_bn_grad_sums": ([I, I, I, I, P, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_edge_mlp_bwd": ([I, I, I, I] + [P] * 21 + [P, SZ, P], I),
    "pfsgnn_loss_fwd": ([I, I, I, I, P, P, P, P, P, P, P, P, FL, FL, FL, ULL, P, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_loss_finalize": ([I, I, I, P, P, P, P, FL, FL, FL, FL, FL, FL, P, P, P, P, P, P, P], I),
    "pfsgnn_loss_bwd": ([I, I, I, I, P, P, P, P, P, P, P, P, FL, FL, FL, ULL, P, P, P, P, P, P,
                         P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_loss_bn_parts": ([I, I, I], I),
    "pfsgnn_loss_bwd_bn": ([I, I, I, I, P, P, P, P, P, P, P, P, FL, FL, FL, ULL, P, P, P, P, P,
                            P, P, P, P, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_layout_analyze": ([P, LL, I, I, I, P, P, P, SZ, P], I),
    "pfsgnn_edges_to_canonical": ([P, I, I, I, I, I, P, P, P], I),
    "pfsgnn_edges_from_canonical": ([P, P, P, I, I, I, I, I, P, I, P, P], I),
    "pfsgnn_adam": ([P, P, P, P, LL, I, P, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                     ctypes.c_double, ctypes.c_double, P, P], I),
    "pfsgnn_sliced_max_nc": ([I, ctypes.POINTER(ctypes.c_int)], I),
    "pfsgnn_target_block_fwd": ([ctypes.POINTER(BlockTail), P, SZ, P], I),
    "pfsgnn_sync_faults": ([ctypes.POINTER(ctypes.c_uint)], I),
    "pfsgnn_set_grid_sync_fenced": ([I], I),
    "pfsgnn_block_tail_bytes": ([], SZ),
    "pfsgnn_target_class_bwd": ([ctypes.POINTER(ClassBwd), P, SZ, P], I),
    "pfsgnn_class_bwd_bytes": ([], SZ),
    "pfsgnn_bn_eval_bwd_coef": ([P, P, P, P, I, FL, I, P, P, P, P, P, P, P], I),
    "pfsgnn_sliced_plan_ws_bytes": ([I, I], SZ),
    "pfsgnn_sliced_plan": ([P, I, I, P, P, P, P, P, P, SZ, P], I),
    "pfsgnn_sliced_fill": ([P, P, P, P, LL, I, I, P, P, LL, I, P, P, P, P], I),
    "pfsgnn_edges_to_slots": ([P, LL, LL, I, P, P, P], I),
    "pfsgnn_edges_from_slots": ([P, P, P, LL, LL, I, P, I, P, P], I),
    "pfsgnn_sl_tmask_bytes": ([SLP, I], SZ),
}
# the edge ops on a sliced general batch: the complete op's arguments after the layout
for _op in ("edge_mlp_fwd", "edge_mlp_fwd_bn", "source_fwd", "target_fwd", "target_bwd",
            "source_bwd", "source_bwd_bn", "edge_mlp_bwd"):
    _SIGS["pfsgnn_sl_" + _op] = ([SLP] + _SIGS["pfsgnn_" + _op][0], I)


def lib():
    """Load libpfsgnn.so (once).  Raises NativeUnavailable if it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise NativeUnavailable(
                f"{_LIB_PATH} not found: build it with `make -C pfs-neural-net_amd` "
                "(or __graft_entry__.build()); there is no non-HIP fallback")
        L = ctypes.CDLL(_LIB_PATH)
        for name, (args, ret) in _SIGS.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = ret
        _lib = L
        path = os.environ.get("PFSGNN_EDGE_PATH")
        if path:
            set_edge_path(path)
    return _lib


EDGE_PATHS = {"valu": 0, "mfma": 1, "mfma32": 2, "bf16y": 3, "bf16": 4, "bf16m": 5, "bf16x3": 6,
              "bf16x6": 7}


def set_edge_path(path):
    """Implementation of the per-edge kernels: "mfma" (default; matrix cores,
    exact fp32 forward products, bf16x3 gradient chains), "mfma32" (matrix
    cores, every layer product exact fp32), "valu" (fp32 fmaf chains), "bf16y"
    (mfma32 with the edge state rounded to bf16), "bf16m" (single-bf16 MFMA
    contractions), "bf16" (bf16m + bf16 edge state) or "bf16x3" (every
    per-edge contraction on bf16 MFMAs with split hi + lo operands, forward and
    recompute included; inside the fp32 bar at the bench geometry only) or "bf16x6"
    (the forward contractions and recompute on bf16 MFMAs with three-way split
    operands, fp32-class products; gradient chains as "mfma").  The bf16
    paths are built for Fdim 10; at other Fdims "bf16x6" runs the "mfma"
    arithmetic.
    Read at launch time; env PFSGNN_EDGE_PATH sets it when the library loads."""
    if path not in EDGE_PATHS:
        raise ValueError(f"edge path must be one of {sorted(EDGE_PATHS)}, got {path!r}")
    _check(lib().pfsgnn_set_edge_path(EDGE_PATHS[path]), "pfsgnn_set_edge_path")


def get_edge_path():
    code = lib().pfsgnn_get_edge_path()
    return {v: k for k, v in EDGE_PATHS.items()}[code]


def edge_grid(G, NF, NC):
    """Grid of the current edge path for a batch: dict(KS, CPS, nblocks, NFG)."""
    info = (ctypes.c_int * 4)()
    _check(lib().pfsgnn_edge_grid(int(G), int(NF), int(NC), info), "pfsgnn_edge_grid")
    return dict(KS=info[0], CPS=info[1], nblocks=info[2], NFG=info[3])


def exported_symbols():
    return list(_SIGS.keys())


KERNELS = ["edge_mlp_fwd", "source_fwd", "target_fwd", "target_bwd", "source_bwd",
           "edge_bn_sums", "edge_mlp_bwd", "loss_fwd", "loss_bwd"]


def timing_enable(on=True):
    """on: False / True (events around each launch) / "spin" (the same behind
    a lead-in spin kernel: the kernel's own time in an eager step)."""
    lib().pfsgnn_timing_enable(2 if on == "spin" else (1 if on else 0))


def sync_faults():
    """Device-wide barrier time-outs since the library was loaded (0 when healthy;
    a time-out also traps its launch)."""
    n = ctypes.c_uint(0)
    _check(lib().pfsgnn_sync_faults(ctypes.byref(n)), "pfsgnn_sync_faults")
    return n.value


def set_grid_sync_fenced(fenced):
    """The device-wide barrier's form for later launches: False the sc1 hand-off
    (default), True acq_rel arrival / acquire poll (pfsgnn_set_grid_sync_fenced)."""
    _check(lib().pfsgnn_set_grid_sync_fenced(1 if fenced else 0), "pfsgnn_set_grid_sync_fenced")


def timing_repeat(name, extra):
    """Launch kernel `name` 1 + extra times back to back (pfsgnn_timing_repeat)."""
    _check(lib().pfsgnn_timing_repeat(name.encode(), int(extra)), "pfsgnn_timing_repeat")


def timing_reset():
    lib().pfsgnn_timing_reset()


def timing_query(name):
    """(total milliseconds, launches) of a main kernel since the last reset."""
    ms = ctypes.c_double(0.0)
    n = ctypes.c_longlong(0)
    lib().pfsgnn_timing_query(name.encode(), ctypes.byref(ms), ctypes.byref(n))
    return ms.value, n.value


def _ptr(t):
    if t is None:
        return None
    return t.data_ptr()


def _stream():
    return torch.cuda.current_stream().cuda_stream


def _check(rc, name):
    if rc != 0:
        msg = lib().pfsgnn_last_error().decode()
        raise RuntimeError(f"{name} failed ({rc}): {msg}")


def _call(name, *args):
    _check(getattr(lib(), name)(*args), name)


_SYNC = None


def _ensure_sync(device):
    """The library's in-launch reduction counters (pfsgnn_set_sync_buffer): one
    zeroed device buffer per process, set once.  PFSGNN_NO_HANDOFF=1 leaves it
    unset (the kernels then keep their separate reduce launches: an A/B knob).

    The counters are process-wide, so pfsgnn ops run on ONE device per process
    (the one-process-per-GPU model of torch.distributed) and on one stream at a
    time; a backend on a second device is refused rather than pointed at
    another device's counters."""
    global _SYNC
    if os.environ.get("PFSGNN_NO_HANDOFF", "0") == "1":
        return
    if _SYNC is not None:
        dev = torch.device(device)
        idx = dev.index if dev.index is not None else torch.cuda.current_device()
        if _SYNC.device.index != idx:
            raise RuntimeError(
                f"pfsgnn runs on one device per process: its sync buffer lives on "
                f"{_SYNC.device}, a backend on {dev} was requested (one process per GPU)")
        return
    n = lib().pfsgnn_sync_bytes()
    _SYNC = torch.zeros(n, dtype=torch.uint8, device=device)
    torch.cuda.synchronize(device)
    _call("pfsgnn_set_sync_buffer", _SYNC.data_ptr(), n)


SLOTS = 3   # pfsgnn.gnn.Layout.SLOTS: the positions of a sliced general batch


class SlicedLayout:
    """A sliced general batch's device tensors (pfsgnn_sliced_plan / _fill) and
    the pfsgnn_sliced_t pointing at them, kept alive together.  pos_user [EP]:
    the caller's edge at each position (-1: padding)."""

    def __init__(self, fib, base, ln, slot_of, cls, pos_user, pco, EP, E, maxdeg):
        self.fib, self.base, self.len, self.slot_of = fib, base, ln, slot_of
        self.cls, self.pos_user, self.pco = cls, pos_user, pco
        self.EP, self.E, self.maxdeg = int(EP), int(E), int(maxdeg)
        self.c = Sliced(fib.data_ptr(), base.data_ptr(), ln.data_ptr(), cls.data_ptr(),
                        pco.data_ptr(), self.EP, self.E, self.maxdeg)
        self.ref = ctypes.pointer(self.c)


class HipBackend:
    """The op set of pfsgnn.engine on libpfsgnn.so (fp32, channel-major)."""

    name = "hip"
    fiber_bn_sums = True     # target_bwd(bn_sums=...) / mlp_bwd(bn_part=...)
    loss_bn_part = True      # loss_bwd(bn=...) / bn2_bwd_coef_part

    def __init__(self, device=None):
        if not torch.cuda.is_available():
            raise NativeUnavailable("no HIP device visible: the pfsgnn hot path runs only on "
                                    "an MI355X (gfx950); there is no CPU fallback")
        lib()
        self.device = torch.device(device or "cuda")
        self.dtype = torch.float32
        self._ws = None
        self._ws_key = None
        # buffers replaced by a larger one stay alive: a HIP graph captured
        # while they were current keeps their addresses baked in, and a replay
        # must never write into memory the allocator has handed out again
        self._retired = []
        self._sp = SparseEdgeOps(self)
        _ensure_sync(self.device)

    def edge_path(self):
        """The current edge path's code (pfsgnn_get_edge_path)."""
        return lib().pfsgnn_get_edge_path()

    # ------------------------------------------------------------ memory
    def empty(self, *shape):
        return torch.empty(*shape, dtype=torch.float32, device=self.device)

    def zeros(self, *shape):
        return torch.zeros(*shape, dtype=torch.float32, device=self.device)

    def ones(self, *shape):
        return torch.ones(*shape, dtype=torch.float32, device=self.device)

    def workspace(self, d=None):
        need = lib().pfsgnn_workspace_bytes(d.G, d.NF, d.NC, d.F) if d is not None else 0
        need = max(need, 16 << 20)
        if self._ws is None or self._ws.numel() < need:
            if self._ws is not None:
                self._retired.append(self._ws)
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        return self._ws

    def _wsargs(self, d=None):
        ws = self.workspace(d)
        return ws.data_ptr(), ws.numel()

    @staticmethod
    def _chk(*ts):
        for t in ts:
            if t is not None:
                assert t.dtype == torch.float32 and t.is_cuda and t.is_contiguous(), \
                    (t.dtype, t.device, t.shape, t.stride())

    # ------------------------------------------------------------ node ops
    def lin(self, W, col0, ncol, X, b=None, act_in=False, out=None, add=False, bscale=1.0):
        M, ldw = W.shape
        N = X.shape[1]
        assert X.shape[0] == ncol
        if out is None:
            out = self.empty(M, N)
            add = False
        self._chk(W, X, b, out)
        _call("pfsgnn_lin", W.data_ptr() + 4 * col0, ldw, M, ncol, X.data_ptr(), N, _ptr(b),
              float(bscale), int(act_in), out.data_ptr(), int(add), _stream())
        return out

    def lin_gather(self, W, col0, ncol, X, gathers, b=None):
        """W[:, col0:col0+ncol] . X + b + sum_j G_j[:, idx_j] (up to two
        (G [M, ld], idx int32 [N]) pairs), one launch."""
        M, ldw = W.shape
        N = X.shape[1]
        out = self.empty(M, N)
        self._chk(W, X, b, out)
        g = list(gathers) + [(None, None)] * (2 - len(gathers))
        for G, idx in gathers:
            self._chk(G)
            assert idx.dtype == torch.int32 and idx.numel() == N and G.shape[0] == M
        _call("pfsgnn_lin_gather", W.data_ptr() + 4 * col0, ldw, M, ncol, X.data_ptr(), N, _ptr(b),
              1.0, 0, out.data_ptr(), 0, _ptr(g[0][0]), _ptr(g[0][1]),
              0 if g[0][0] is None else g[0][0].shape[1], _ptr(g[1][0]), _ptr(g[1][1]),
              0 if g[1][0] is None else g[1][0].shape[1], _stream())
        return out

    def lin_t(self, W, col0, ncol, dY, z=None, out=None, add=False):
        M, ldw = W.shape
        N = dY.shape[1]
        if out is None:
            out = self.empty(ncol, N)
            add = False
        self._chk(W, dY, z, out)
        _call("pfsgnn_lin_t", W.data_ptr() + 4 * col0, ldw, M, ncol, dY.data_ptr(), N, _ptr(z),
              out.data_ptr(), int(add), _stream())
        return out

    def linear_batch(self, ops):
        """Independent small products in one launch (pfsgnn_gemm_multi).  ops:
        ("cat", W, segs, N, b) -> Y = W . cat(segs) + b (a new [M, N] tensor), or
        ("t", W, col0, ncol, dY, out, add) -> out (+)= W[:, col0:col0+ncol]^T dY.
        Returns the outputs in order."""
        arr = (GemmJob * len(ops))()
        keep, outs = [], []
        for i, op in enumerate(ops):
            if op[0] == "cat":
                _, W, segs, N, b = op
                M, ldw = W.shape
                Y = self.empty(M, N)
                sg = self._segs(segs, N)
                self._chk(W, b)
                arr[i] = GemmJob(W.data_ptr(), ldw, 0, M, 0, sg, len(segs), N, _ptr(b), 1.0, 0,
                                 None, Y.data_ptr(), 0)
                keep.append(sg)
            else:
                _, W, col0, ncol, dY, Y, add = op
                Mw, ldw = W.shape
                N = dY.shape[1]
                if Y is None:
                    Y, add = self.empty(ncol, N), False
                self._chk(W, dY, Y)
                sg = self._segs([(dY, 0, False)], N)
                arr[i] = GemmJob(W.data_ptr() + 4 * col0, ldw, 1, ncol, Mw, sg, 1, N, None, 1.0,
                                 0, None, Y.data_ptr(), int(add))
                keep.append(sg)
            outs.append(Y)
        _call("pfsgnn_gemm_multi", arr, len(ops), _stream())
        return outs

    # ----------------------------------------------- deferred weight gradients
    # Between defer_begin() and defer_flush(), wgrad/wgrad_cat only record a
    # job; the flush computes them all in a few launches (pfsgnn_wgrad_multi:
    # jobs of one kernel shape share a launch, the reductions are batched).
    # The engine defers over a backward pass: its weight gradients are read
    # only by the optimizer, and the jobs' inputs are activations and
    # gradients that no later op of the pass writes (engine.Engine.backward).
    # The fused edge backward kernels' own weight reductions are deferred the
    # same way inside the library (pfsgnn_defer_begin / _end), their partials
    # in a second arena sized by the previous pass (warm-up sizes it before
    # any graph capture; a pass that does not fit reduces at once).
    def defer_begin(self):
        self._jobs = []
        ea = getattr(self, "_earena", None)
        _call("pfsgnn_defer_begin", None if ea is None else ea.data_ptr(),
              0 if ea is None else ea.numel())

    def defer_flush(self):
        jobs, self._jobs = getattr(self, "_jobs", None), None
        if jobs is None:
            return
        arr, arena = None, None
        if jobs:
            arr = (WgJob * len(jobs))()
            for i, (job, _keep) in enumerate(jobs):
                arr[i] = job
            need = lib().pfsgnn_wgrad_multi_bytes(arr, len(jobs))
            if need == 0:
                raise RuntimeError("pfsgnn_wgrad_multi_bytes: " + lib().pfsgnn_last_error().decode())
            arena = getattr(self, "_arena", None)
            if arena is None or arena.numel() < need:
                # grown during warm-up, before any graph capture; a replaced arena
                # stays alive (see __init__)
                if arena is not None:
                    self._retired.append(arena)
                self._arena = arena = torch.empty(max(need, 64 << 20), dtype=torch.uint8,
                                                  device=self.device)
        # the jobs and every queued reduction of the pass in one flush
        _call("pfsgnn_defer_end_multi", arr, len(jobs), None if arena is None else arena.data_ptr(),
              0 if arena is None else arena.numel(), _stream())
        need = lib().pfsgnn_defer_need()
        ea = getattr(self, "_earena", None)
        if need and (ea is None or ea.numel() < need):
            if ea is not None:
                self._retired.append(ea)
            self._earena = torch.empty(need + (1 << 20), dtype=torch.uint8, device=self.device)

    def _wgrad_job(self, dY, arr, nseg, N, act_in, dW, db, dbscale, keep):
        job = WgJob(dY.data_ptr(), dY.shape[0], arr, nseg, N, int(act_in), dW.data_ptr(),
                    dW.shape[1], _ptr(db), float(dbscale))
        self._jobs.append((job, (arr, dY, dW, db) + tuple(keep)))

    def wgrad(self, dY, X, dW, col0=0, db=None, act_in=False, dbscale=1.0):
        M, N = dY.shape
        K = X.shape[0]
        self._chk(dY, X, dW, db)
        if getattr(self, "_jobs", None) is not None:
            self._wgrad_job(dY, self._segs([(X, col0, False)], N), 1, N, act_in, dW, db, dbscale,
                            (X,))
            return
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        _call("pfsgnn_wgrad", dY.data_ptr(), M, X.data_ptr(), K, N, int(act_in),
              dW.data_ptr() + 4 * col0, dW.shape[1], _ptr(db), float(dbscale), ws, wsb, _stream())

    def _segs(self, segs, N):
        """[(X, col, per_graph)] -> ctypes pfsgnn_seg array; per_graph segments
        are [rows, G] tensors broadcast over the N // G nodes of each graph."""
        arr = (Seg * len(segs))()
        for i, (X, col, bc) in enumerate(segs):
            self._chk(X)
            assert (N % X.shape[1] == 0) if bc else (X.shape[1] == N), (X.shape, N, bc)
            arr[i].x = X.data_ptr()
            arr[i].rows = X.shape[0]
            arr[i].col = int(col)
            arr[i].per_graph = N // X.shape[1] if bc else 0
        return arr

    def lin_cat(self, W, segs, N, b=None, act_in=False, out=None, add=False, bscale=1.0):
        """Y (+)= sum_s W[:, col_s:col_s+rows_s] @ act(X_s[, broadcast per graph]) + bscale*b."""
        M, ldw = W.shape
        if out is None:
            out = self.empty(M, N)
            add = False
        self._chk(W, b, out)
        arr = self._segs(segs, N)
        _call("pfsgnn_lin_cat", W.data_ptr(), ldw, M, arr, len(segs), N, _ptr(b), float(bscale),
              int(act_in), out.data_ptr(), int(add), _stream())
        return out

    def wgrad_cat(self, dY, segs, dW, db=None, act_in=False, dbscale=1.0):
        """dW[:, col_s:col_s+rows_s] += dY @ act(X_s)^T; db += dbscale * dY.sum(1)."""
        M, N = dY.shape
        self._chk(dY, dW, db)
        arr = self._segs(segs, N)
        if getattr(self, "_jobs", None) is not None:
            self._wgrad_job(dY, arr, len(segs), N, act_in, dW, db, dbscale,
                            tuple(X for X, _, _ in segs))
            return
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        _call("pfsgnn_wgrad_cat", dY.data_ptr(), M, arr, len(segs), N, int(act_in), dW.data_ptr(),
              dW.shape[1], _ptr(db), float(dbscale), ws, wsb, _stream())

    # ------------------------------------------------------- fused node MLPs
    def mlp_fwd(self, segs, N, W1, b1, W2, b2, bn=None, save_z=True):
        """MLP (gnn.py:65) over a concatenated node input (+ training BatchNorm1d
        when ``bn`` = (gamma, beta, running_mean, running_var, momentum, eps)).
        Returns (Y, Z, Yp, mu, var): Y the module output, Z the saved
        pre-activation, Yp the pre-norm output (Y itself without bn)."""
        H, ldw1 = W1.shape
        O = W2.shape[0]
        self._chk(W1, b1, W2, b2)
        arr = self._segs(segs, N)
        Z = self.empty(H, N) if save_z else None
        Yp = self.empty(O, N)
        g = bt = rm = rv = None
        mom, eps = 0.0, 0.0
        Y = mu = var = None
        if bn is not None:
            g, bt, rm, rv, mom, eps = bn
            self._chk(g, bt, rm, rv)
            Y, mu, var = self.empty(O, N), self.empty(O), self.empty(O)
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        _call("pfsgnn_mlp_fwd", arr, len(segs), N, W1.data_ptr(), ldw1, H, b1.data_ptr(),
              W2.data_ptr(), O, b2.data_ptr(), _ptr(Z), Yp.data_ptr(), _ptr(g), _ptr(bt), _ptr(rm),
              _ptr(rv), float(mom), float(eps), _ptr(Y), _ptr(mu), _ptr(var), ws, wsb, _stream())
        return (Yp if Y is None else Y), Z, Yp, mu, var

    def mlp_fwd_epi(self, segs, N, W1, b1, W2, b2, bn, epi):
        """mlp_fwd with BatchNorm + up to two linear maps of the normalised output
        done in the normalising pass: ``epi`` = [(W, col0, nk, b)] ->
        W[:, col0:col0+O] . Y + b ([nk, N] each, returned as a 6th item)."""
        H, ldw1 = W1.shape
        O = W2.shape[0]
        self._chk(W1, b1, W2, b2)
        arr = self._segs(segs, N)
        Z, Yp = self.empty(H, N), self.empty(O, N)
        g, bt, rm, rv, mom, eps = bn
        self._chk(g, bt, rm, rv)
        Y, mu, var = self.empty(O, N), self.empty(O), self.empty(O)
        em = (LinMap * len(epi))()
        outs = []
        for i, (W, col0, nk, b) in enumerate(epi):
            self._chk(W, b)
            assert col0 + O <= W.shape[1] and nk <= W.shape[0]
            o = self.empty(nk, N)
            em[i] = LinMap(W.data_ptr(), W.shape[1], int(col0), int(nk), _ptr(b), o.data_ptr())
            outs.append(o)
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        _call("pfsgnn_mlp_fwd_epi", arr, len(segs), N, W1.data_ptr(), ldw1, H, b1.data_ptr(),
              W2.data_ptr(), O, b2.data_ptr(), Z.data_ptr(), Yp.data_ptr(), g.data_ptr(),
              bt.data_ptr(), _ptr(rm), _ptr(rv), float(mom), float(eps), Y.data_ptr(),
              mu.data_ptr(), var.data_ptr(), em, len(epi), ws, wsb, _stream())
        return Y, Z, Yp, mu, var, outs

    def target_block_fwd(self, d, y, sc, sh, Rs, Wt1, Wt2, bt2, tmask, xt, u, W1, b1, W2, b2,
                         bn, xs, gW1, gb1, gW2, gb2, gw, reps, nxt=None):
        """target_fwd (TModel's per-edge layer) + target_global_fwd on a complete
        batch, the class side in one launch (pfsgnn_target_block_fwd).  -> dict
        with target_global_fwd's keys plus hsum and agg."""
        F, G, NC, NT = d.F, d.G, d.NC, d.NT
        H = W1.shape[0]
        assert W1.shape == (4 * F, 4 * F) and W2.shape == (F, 4 * F) and Wt2.shape == (2 * F, 2 * F)
        self._chk(y, sc, sh, Rs, Wt1, Wt2, bt2, xt, u, W1, b1, W2, b2, xs, gW1, gb1, gW2, gb2, gw)
        g, bt, rm, rv, mom, eps = bn
        self._chk(g, bt, rm, rv)
        gH = gW1.shape[0]
        r = dict(hsum=self.empty(2 * F, NT), agg=self.empty(2 * F, NT), Z=self.empty(H, NT),
                 Yp=self.empty(F, NT), xt=self.empty(F, NT), mu=self.empty(F), var=self.empty(F),
                 means=self.empty(2 * F, G), gZ=self.empty(gH, G), gV=self.empty(F, G),
                 u=self.empty(F, G))
        rms = (self.empty(F, G), self.empty(G), self.empty(G)) if gw is not None else None
        y1, r1, r2 = rms if rms is not None else (None, None, None)
        We = be_ = Ws = bs = Pt = Qt = None
        if nxt is not None:
            We, be_, Ws, bs = nxt
            self._chk(We, be_, Ws, bs)
            assert We.shape == (4 * F, 4 * F) and Ws.shape == (2 * F, 2 * F)
            Pt, Qt = self.empty(4 * F, NT), self.empty(2 * F, NT)
        a = BlockTail(G=G, NF=d.NF, NC=NC, F=F, y=y.data_ptr(), sc=_ptr(sc), sh=_ptr(sh),
                      Rs=Rs.data_ptr(), Wt1=Wt1.data_ptr(), Wt2=Wt2.data_ptr(),
                      bt2=bt2.data_ptr(), tmask=_ptr(tmask), hsum=r["hsum"].data_ptr(),
                      agg=r["agg"].data_ptr(), xt=xt.data_ptr(), u=u.data_ptr(),
                      W1=W1.data_ptr(), b1=b1.data_ptr(), W2=W2.data_ptr(), b2=b2.data_ptr(),
                      gamma=g.data_ptr(), beta=bt.data_ptr(), Z=r["Z"].data_ptr(),
                      Yp=r["Yp"].data_ptr(), rm=_ptr(rm), rv=_ptr(rv), xt_new=r["xt"].data_ptr(),
                      mu=r["mu"].data_ptr(), var=r["var"].data_ptr(), momentum=float(mom),
                      eps=float(eps), xs=xs.data_ptr(), gW1=gW1.data_ptr(), gb1=gb1.data_ptr(),
                      gW2=gW2.data_ptr(), gb2=gb2.data_ptr(), gw=_ptr(gw), gH=gH,
                      reps=float(reps), means=r["means"].data_ptr(), gZ=r["gZ"].data_ptr(),
                      gV=r["gV"].data_ptr(), unew=r["u"].data_ptr(), y1=_ptr(y1), r1=_ptr(r1),
                      r2=_ptr(r2), We=_ptr(We), be=_ptr(be_), Ws=_ptr(Ws), bs=_ptr(bs),
                      Pt=_ptr(Pt), Qt=_ptr(Qt))
        ws, wsb = self._wsargs(d)
        _call("pfsgnn_target_block_fwd", ctypes.byref(a), ws, wsb, _stream())
        r["rms"], r["Pt"], r["Qt"] = rms, Pt, Qt
        return r

    def target_class_bwd(self, d, pend, gu_up, V, w, rms, gZ, gW1, gW2, gV, gdZ, dwp, gu, g_xs,
                         g_xt, Yp, mu, var, gamma, eps, dgamma, dbeta, Z, W1, W2, Wt2, gxt_in):
        """The class side of a block's backward in one launch
        (pfsgnn_target_class_bwd): pending u-gradient sums into gu_up, the
        GlobalModel backward, the means broadcast, TModel node_mlp_2 + BatchNorm
        backward and g_hsum = Wt2^T g_agg.  -> dict(dYp, dZ, g_agg, gu_t, g_hsum)."""
        F, NT = d.F, d.NT
        H = W1.shape[0]
        assert len(pend) <= 4 and W1.shape == (4 * F, 4 * F) and W2.shape == (F, 4 * F)
        self._chk(gu_up, V, w, gZ, gW1, gW2, gV, gdZ, dwp, gu, g_xs, g_xt, Yp, mu, var, gamma,
                  dgamma, dbeta, Z, W1, W2, Wt2, gxt_in, *pend)
        r = dict(dYp=self.empty(F, NT), dZ=self.empty(H, NT), g_agg=self.empty(2 * F, NT),
                 gu_t=self.empty(F, NT), g_hsum=self.empty(2 * F, NT))
        y1, r1, r2 = rms if rms is not None else (None, None, None)
        a = ClassBwd(G=d.G, NF=d.NF, NC=d.NC, F=F, npend=len(pend), gH=gW1.shape[0],
                     eps=float(eps))
        for i, X in enumerate(pend):
            a.pend[i] = X.data_ptr()
            a.pend_n[i] = X.shape[1] // d.G
        for k, v in dict(V=V, w=w, y1=y1, r1=r1, r2=r2, gZ=gZ, gW1=gW1, gW2=gW2, gu_up=gu_up,
                         gV=gV, gdZ=gdZ, dwp=dwp, gu=gu, g_xs=g_xs, g_xt=g_xt, Yp=Yp, mu=mu,
                         var=var, gamma=gamma, Z=Z, W1=W1, W2=W2, Wt2=Wt2, dgamma=dgamma,
                         dbeta=dbeta, dYp=r["dYp"], dZ=r["dZ"], gxt_in=gxt_in,
                         g_agg=r["g_agg"], gu_t=r["gu_t"], g_hsum=r["g_hsum"]).items():
            setattr(a, k, _ptr(v))
        ws, wsb = self._wsargs(d)
        _call("pfsgnn_target_class_bwd", ctypes.byref(a), ws, wsb, _stream())
        return r

    def sync_faults(self):
        """Device-wide barrier time-outs since load (pfsgnn_sync_faults; 0 when healthy)."""
        n = ctypes.c_uint(0)
        _call("pfsgnn_sync_faults", ctypes.byref(n))
        return n.value

    def target_global_fwd(self, segs, G, NC, W1, b1, W2, b2, bn, xs, NF, u, gW1, gb1, gW2, gb2,
                          gw, reps, nxt=None):
        """TModel's node_mlp_2 + BatchNorm1d (gnn.py:191-192) and the GlobalModel
        (gnn.py:218-223), + with ``nxt`` = (We, be, Ws, bs) the next block's
        per-class parts Pt, Qt (pfsgnn_target_global_fwd).  -> dict."""
        H, ldw1 = W1.shape
        F = W2.shape[0]
        N = G * NC
        gH = gW1.shape[0]
        self._chk(W1, b1, W2, b2, xs, u, gW1, gb1, gW2, gb2, gw)
        arr = self._segs(segs, N)
        g, bt, rm, rv, mom, eps = bn
        self._chk(g, bt, rm, rv)
        r = dict(Z=self.empty(H, N), Yp=self.empty(F, N), xt=self.empty(F, N), mu=self.empty(F),
                 var=self.empty(F), means=self.empty(2 * F, G), gZ=self.empty(gH, G),
                 gV=self.empty(F, G), u=self.empty(F, G))
        rms = (self.empty(F, G), self.empty(G), self.empty(G)) if gw is not None else None
        y1, r1, r2 = rms if rms is not None else (None, None, None)
        We = be = Ws = bs = Pt = Qt = None
        if nxt is not None:
            We, be, Ws, bs = nxt
            self._chk(We, be, Ws, bs)
            assert We.shape == (4 * F, 4 * F) and Ws.shape == (2 * F, 2 * F)
            Pt, Qt = self.empty(4 * F, N), self.empty(2 * F, N)
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        _call("pfsgnn_target_global_fwd", arr, len(segs), G, NC, W1.data_ptr(), ldw1, H,
              b1.data_ptr(), W2.data_ptr(), F, b2.data_ptr(), r["Z"].data_ptr(),
              r["Yp"].data_ptr(), g.data_ptr(), bt.data_ptr(), _ptr(rm), _ptr(rv), float(mom),
              float(eps), r["xt"].data_ptr(), r["mu"].data_ptr(), r["var"].data_ptr(),
              xs.data_ptr(), NF, u.data_ptr(), gW1.data_ptr(), gH, gb1.data_ptr(), gW2.data_ptr(),
              gb2.data_ptr(), _ptr(gw), float(reps), r["means"].data_ptr(), r["gZ"].data_ptr(),
              r["gV"].data_ptr(), r["u"].data_ptr(), _ptr(y1), _ptr(r1), _ptr(r2), _ptr(We),
              _ptr(be), _ptr(Ws), _ptr(bs), _ptr(Pt), _ptr(Qt), ws, wsb, _stream())
        r["rms"], r["Pt"], r["Qt"] = rms, Pt, Qt
        return r

    def mlp_bwd(self, dY, Z, W1, W2, K, bn=None, outs=(), bn_part=None, mom_coef=None):
        """Input side of the MLP(+BN) backward.  ``bn`` = (Yp, mu, var, gamma, eps,
        dgamma, dbeta) or None; ``outs`` = [(tensor or None, rows, add)] covering
        the K input rows (empty: no input gradient); ``bn_part``: the BatchNorm
        sums' partials the producer of dY already made (target_bwd's
        ``bn_sums``), else they are summed here; ``mom_coef`` = (mom, coef, k0,
        n): input rows [k0, k0 + 4C) are SModel's moment gradients, turned into
        moment_coef(mom, ., n)'s coefficients in coef instead of written.
        Returns (dYp, dZ)."""
        H, ldw1 = W1.shape
        O, N = dY.shape
        dY = dY.contiguous()
        self._chk(dY, Z, W1, W2)
        dZ = self.empty(H, N)
        Yp = mu = var = g = dg = db = None
        eps = 0.0
        dYp = dY
        if bn is not None:
            Yp, mu, var, g, eps, dg, db = bn
            self._chk(Yp, mu, var, g, dg, db)
            dYp = self.empty(O, N)
        arr = (OSeg * max(1, len(outs)))()
        for i, (t, rows, add) in enumerate(outs):
            if t is not None:
                self._chk(t)
                assert t.shape == (rows, N), (t.shape, rows, N)
            arr[i].x = None if t is None else t.data_ptr()
            arr[i].rows = int(rows)
            arr[i].add = int(bool(add))
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        if bn_part is not None or mom_coef is not None:
            nparts = 0
            if bn_part is not None:
                assert bn is not None and bn_part.shape == ((N + 63) // 64, 32), bn_part.shape
                self._chk(bn_part)
                nparts = bn_part.shape[0]
            mom = coef = None
            k0 = C = n = 0
            if mom_coef is not None:
                mom, coef, k0, n = mom_coef
                self._chk(mom, coef)
                C = mom.shape[1]
                assert mom.shape == (4, C, N) and coef.shape == (4, C, N), (mom.shape, coef.shape)
            _call("pfsgnn_mlp_bwd_pre", dY.data_ptr(), N, _ptr(Yp), _ptr(mu), _ptr(var), _ptr(g),
                  float(eps), _ptr(dg), _ptr(db), Z.data_ptr(), W1.data_ptr(), ldw1, H, int(K),
                  W2.data_ptr(), O, None if bn is None else dYp.data_ptr(), dZ.data_ptr(), arr,
                  len(outs), _ptr(bn_part), nparts, _ptr(mom), _ptr(coef), int(k0), int(C),
                  int(n), ws, wsb, _stream())
            return dYp, dZ
        _call("pfsgnn_mlp_bwd", dY.data_ptr(), N, _ptr(Yp), _ptr(mu), _ptr(var), _ptr(g),
              float(eps), _ptr(dg), _ptr(db), Z.data_ptr(), W1.data_ptr(), ldw1, H, int(K),
              W2.data_ptr(), O, None if bn is None else dYp.data_ptr(), dZ.data_ptr(), arr,
              len(outs), ws, wsb, _stream())
        return dYp, dZ

    def bn_fwd(self, X, gamma, beta, rm, rv, momentum, eps):
        C, N = X.shape
        Y, mu, var = self.empty(C, N), self.empty(C), self.empty(C)
        self._chk(X, gamma, beta, rm, rv)
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        _call("pfsgnn_bn_fwd", X.data_ptr(), C, N, gamma.data_ptr(), beta.data_ptr(), _ptr(rm),
              _ptr(rv), float(momentum), float(eps), Y.data_ptr(), mu.data_ptr(), var.data_ptr(),
              ws, wsb, _stream())
        return Y, mu, var

    def bn_bwd(self, dY, X, mu, var, gamma, eps, dgamma, dbeta):
        C, N = X.shape
        dX = self.empty(C, N)
        dY = dY.contiguous()
        self._chk(dY, X, mu, var, gamma, dgamma, dbeta)
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        _call("pfsgnn_bn_bwd", dY.data_ptr(), X.data_ptr(), mu.data_ptr(), var.data_ptr(),
              gamma.data_ptr(), float(eps), C, N, dX.data_ptr(), dgamma.data_ptr(),
              dbeta.data_ptr(), ws, wsb, _stream())
        return dX

    def graph_reduce(self, X, G, mean=False, out=None):
        """Per-graph sum (mean) of a node table; with ``out`` it is accumulated."""
        C, N = X.shape
        self._chk(X)
        if out is not None:
            self._chk(out)
            _call("pfsgnn_graph_reduce_add", X.data_ptr(), C, G, N // G, int(mean),
                  out.data_ptr(), _stream())
            return out
        out = self.empty(C, G)
        _call("pfsgnn_graph_reduce", X.data_ptr(), C, G, N // G, int(mean), out.data_ptr(),
              _stream())
        return out

    def graph_reduce_multi(self, Xs, G, out):
        """out[c][g] += per-graph sums of every X in Xs (one launch)."""
        self._chk(out, *Xs)
        m = len(Xs)
        arr = (ctypes.c_void_p * m)(*[X.data_ptr() for X in Xs])
        ns = (ctypes.c_int * m)(*[X.shape[1] // G for X in Xs])
        for X in Xs:
            assert X.shape[0] == out.shape[0] and X.shape[1] % G == 0
        _call("pfsgnn_graph_reduce_multi", arr, ns, m, out.shape[0], G, out.data_ptr(), _stream())
        return out

    def graph_bcast_add(self, out, src, scale=1.0):
        C, N = out.shape
        G = src.shape[1]
        src = src.contiguous()
        self._chk(out, src)
        _call("pfsgnn_graph_bcast_add", out.data_ptr(), C, G, N // G, src.data_ptr(),
              float(scale), _stream())
        return out

    def graph_mean2(self, X1, X2, G):
        """[2C, G]: per-graph means of X1 (rows 0..C) and X2 (rows C..2C)."""
        C = X1.shape[0]
        self._chk(X1, X2)
        out = self.empty(2 * C, G)
        _call("pfsgnn_graph_mean2", X1.data_ptr(), X1.shape[1] // G, X2.data_ptr(),
              X2.shape[1] // G, C, G, out.data_ptr(), _stream())
        return out

    def graph_bcast_add2(self, out1, s1, out2, s2, src):
        C, G = src.shape[0] // 2, src.shape[1]
        src = src.contiguous()
        self._chk(out1, out2, src)
        _call("pfsgnn_graph_bcast_add2", out1.data_ptr(), out1.shape[1] // G, float(s1),
              out2.data_ptr(), out2.shape[1] // G, float(s2), C, G, src.data_ptr(), _stream())

    def rms2_fwd(self, X, w, eps):
        C, G = X.shape
        Y, y1, r1, r2 = self.empty(C, G), self.empty(C, G), self.empty(G), self.empty(G)
        self._chk(X, w)
        _call("pfsgnn_rms2_fwd", X.data_ptr(), C, G, w.data_ptr(), float(eps), Y.data_ptr(),
              y1.data_ptr(), r1.data_ptr(), r2.data_ptr(), _stream())
        return Y, (y1, r1, r2)

    def rms2_bwd(self, dY, X, w, saved, eps, dw):
        y1, r1, r2 = saved
        C, G = X.shape
        dX = self.empty(C, G)
        dY = dY.contiguous()
        self._chk(dY, X, w, dw)
        ws, wsb = self._wsargs(getattr(self, "_dims", None))
        _call("pfsgnn_rms2_bwd", dY.data_ptr(), X.data_ptr(), w.data_ptr(), y1.data_ptr(),
              r1.data_ptr(), r2.data_ptr(), C, G, float(eps), dX.data_ptr(), dw.data_ptr(), ws,
              wsb, _stream())
        return dX

    def global_fwd(self, xs, xt, u, W1, b1, W2, b2, w, eps, G):
        """The whole GlobalModel forward (gnn.py:208-223), one call (two launches).  w: the
        RMSNorm weight or None (unnormed).  -> (u_new, means [2F, G], Z, V, rms)."""
        F = u.shape[0]
        H = W1.shape[0]
        assert W1.shape[1] == 3 * F and W2.shape == (F, H)
        self._chk(xs, xt, u, W1, b1, W2, b2, w)
        means, Z, V, Y = self.empty(2 * F, G), self.empty(H, G), self.empty(F, G), self.empty(F, G)
        rms = (self.empty(F, G), self.empty(G), self.empty(G)) if w is not None else None
        y1, r1, r2 = rms if rms is not None else (None, None, None)
        _call("pfsgnn_global_fwd", xs.data_ptr(), xs.shape[1] // G, xt.data_ptr(), xt.shape[1] // G,
              u.data_ptr(), F, G, W1.data_ptr(), H, b1.data_ptr(), W2.data_ptr(), b2.data_ptr(),
              _ptr(w), float(eps), means.data_ptr(), Z.data_ptr(), V.data_ptr(), Y.data_ptr(),
              _ptr(y1), _ptr(r1), _ptr(r2), _stream())
        return Y, means, Z, V, rms

    def _ones_row(self, n):
        c = getattr(self, "_ones_cache", None)
        if c is None:
            c = self._ones_cache = {}
        if n not in c:
            c[n] = self.ones(1, n)
        return c[n]

    def global_bwd(self, dY, V, w, rms, eps, dw, Z, W1, W2, g_u, g_xs, s1, g_xt, s2):
        """Backward of global_fwd, one call (two launches; + the RMSNorm weight gradient as a
        deferred weight-gradient job).  Accumulates into g_u, g_xs, g_xt and dw;
        -> (gV, dZ) for the MLP's weight gradients."""
        F, G = V.shape
        H = W1.shape[0]
        dY = dY.contiguous()
        self._chk(dY, V, w, Z, W1, W2, g_u, g_xs, g_xt)
        gV, dZ, gm = self.empty(F, G), self.empty(H, G), self.empty(2 * F, G)
        dwp = self.empty(F, G) if w is not None else None
        y1, r1, r2 = rms if rms is not None else (None, None, None)
        _call("pfsgnn_global_bwd", dY.data_ptr(), V.data_ptr(), _ptr(w), _ptr(y1), _ptr(r1),
              _ptr(r2), F, G, Z.data_ptr(), H, W1.data_ptr(), W2.data_ptr(), gV.data_ptr(),
              dZ.data_ptr(), _ptr(dwp), g_u.data_ptr(), gm.data_ptr(), g_xs.data_ptr(),
              g_xs.shape[1] // G,
              float(s1), g_xt.data_ptr(), g_xt.shape[1] // G, float(s2), _stream())
        if w is not None:
            # dw[c] += sum_g dwp[c][g]: a [F, G] x [1, G]^T weight-gradient job
            self.wgrad(dwp, self._ones_row(G), dw.view(F, 1))
        return gV, dZ

    def bn2_finalize(self, mu1, var1, gamma, beta, rm, rv, n, momentum, eps):
        C = mu1.shape[0]
        sc, sh, inv1, inv2 = self.empty(C), self.empty(C), self.empty(C), self.empty(C)
        _call("pfsgnn_bn2_finalize", mu1.data_ptr(), var1.data_ptr(), gamma.data_ptr(),
              beta.data_ptr(), _ptr(rm), _ptr(rv), C, int(n), float(momentum), float(eps),
              sc.data_ptr(), sh.data_ptr(), inv1.data_ptr(), inv2.data_ptr(), _stream())
        return sc, sh, inv1, inv2

    def bn_eval_coef(self, gamma, beta, rm, rv, eps, times):
        """Eval-mode BatchNorm1d applied ``times`` times as (sc, sh)."""
        C = gamma.shape[0]
        self._chk(gamma, beta, rm, rv)
        sc, sh = self.empty(C), self.empty(C)
        _call("pfsgnn_bn_eval_coef", gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(),
              rv.data_ptr(), C, float(eps), int(times), sc.data_ptr(), sh.data_ptr(), _stream())
        return sc, sh

    def bn_eval_bwd_coef(self, gamma, beta, rm, rv, eps, times, Sg=None, Sgx=None, dgamma=None,
                         dbeta=None):
        """Eval-mode BatchNorm1d backward coefficients (pfsgnn_bn_eval_bwd_coef):
        -> (inv, scale); with the gradient sums (Sg, Sgx) dgamma / dbeta += the
        parameter gradients of the ``times``-fold application."""
        C = gamma.shape[0]
        self._chk(gamma, beta, rm, rv, Sg, Sgx, dgamma, dbeta)
        inv, scale = self.empty(C), self.empty(C)
        _call("pfsgnn_bn_eval_bwd_coef", gamma.data_ptr(), beta.data_ptr(), rm.data_ptr(),
              rv.data_ptr(), C, float(eps), int(times), _ptr(Sg), _ptr(Sgx), inv.data_ptr(),
              scale.data_ptr(), _ptr(dgamma), _ptr(dbeta), _stream())
        return inv, scale

    def affine_rows(self, X, sc, sh):
        C, N = X.shape
        self._chk(X, sc, sh)
        Y = self.empty(C, N)
        _call("pfsgnn_affine_rows", X.data_ptr(), C, N, sc.data_ptr(), sh.data_ptr(),
              Y.data_ptr(), _stream())
        return Y

    def bn2_bwd_coef_part(self, part, mu1, var1, gamma, n, eps, dgamma, dbeta):
        """bn2_bwd_coef from per-block partials [nparts, 2C] (loss_bwd's ``bn``)."""
        C = mu1.shape[0]
        assert part.dim() == 2 and part.shape[1] == 2 * C, part.shape
        self._chk(part)
        a, g0, g1 = self.empty(C), self.empty(C), self.empty(C)
        _call("pfsgnn_bn2_bwd_coef_part", part.data_ptr(), part.shape[0], C, gamma.data_ptr(),
              mu1.data_ptr(), var1.data_ptr(), int(n), float(eps), a.data_ptr(), g0.data_ptr(),
              g1.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), _stream())
        return a, g0, g1

    def bn2_bwd_coef(self, Sg, Sgx, mu1, var1, gamma, n, eps, dgamma, dbeta):
        C = mu1.shape[0]
        a, g0, g1 = self.empty(C), self.empty(C), self.empty(C)
        _call("pfsgnn_bn2_bwd_coef", Sg.data_ptr(), Sgx.data_ptr(), mu1.data_ptr(),
              var1.data_ptr(), gamma.data_ptr(), C, int(n), float(eps), a.data_ptr(),
              g0.data_ptr(), g1.data_ptr(), dgamma.data_ptr(), dbeta.data_ptr(), _stream())
        return a, g0, g1

    def moment_coef(self, mom, gst, n):
        """``n``: the messages per fiber -- an int (complete graphs: NC), or a
        general graph's fiber CSR pointer (int32 [NS+1] device tensor)."""
        _, C, NS = mom.shape
        coef = self.empty(4, C, NS)
        gst = gst.contiguous()
        self._chk(mom, gst)
        if isinstance(n, torch.Tensor):
            assert n.dtype == torch.int32 and n.is_cuda and n.numel() == NS + 1
            _call("pfsgnn_moment_coef_seg", mom.data_ptr(), gst.data_ptr(), C, NS, n.data_ptr(),
                  coef.data_ptr(), _stream())
            return coef
        _call("pfsgnn_moment_coef", mom.data_ptr(), gst.data_ptr(), C, NS, int(n), coef.data_ptr(),
              _stream())
        return coef

    # ------------------------------------------------------------ edge ops
    def _set_dims(self, d):
        self._dims = d

    @staticmethod
    def _composed(d):
        """A general batch without a sliced layout: the composed ops (pfsgnn.sparse)."""
        return d.sp is not None and d.sp.sl is None

    @staticmethod
    def _ecall(op, d, *args):
        """Edge op `op` of the C ABI: pfsgnn_<op> on complete graphs,
        pfsgnn_sl_<op> (same arguments after the layout) on a sliced batch."""
        sl = d.sp.sl if d.sp is not None else None
        if sl is None:
            _call("pfsgnn_" + op, *args)
        else:
            _call("pfsgnn_sl_" + op, sl.ref, *args)

    def edge_mlp_fwd(self, d, xe, xsc, xsh, Ps, Pt, W1, W2, b2):
        if self._composed(d):
            return self._sp.edge_mlp_fwd(d, xe, xsc, xsh, Ps, Pt, W1, W2, b2)
        self._set_dims(d)
        y, mu, var = self.empty(d.F, d.EP), self.empty(d.F), self.empty(d.F)
        self._chk(xe, Ps, Pt, W1, W2, b2)
        ws, wsb = self._wsargs(d)
        self._ecall("edge_mlp_fwd", d, d.G, d.NF, d.NC, d.F, xe.data_ptr(), _ptr(xsc), _ptr(xsh),
              Ps.data_ptr(), Pt.data_ptr(), W1.data_ptr(), W2.data_ptr(), b2.data_ptr(),
              y.data_ptr(), mu.data_ptr(), var.data_ptr(), ws, wsb, _stream())
        return y, mu, var

    def edge_mlp_fwd_bn(self, d, xe, xsc, xsh, Ps, Pt, W1, W2, b2, bn):
        """edge_mlp_fwd + bn2_finalize in one call; ``bn`` = (gamma, beta,
        running_mean, running_var, momentum, eps).  -> y, mu1, var1, sc, sh, inv1."""
        gamma, beta, rm, rv, momentum, eps = bn
        if self._composed(d):
            y, mu, var = self._sp.edge_mlp_fwd(d, xe, xsc, xsh, Ps, Pt, W1, W2, b2)
            sc, sh, inv1, _ = self.bn2_finalize(mu, var, gamma, beta, rm, rv, d.E, momentum, eps)
            return y, mu, var, sc, sh, inv1
        self._set_dims(d)
        F = d.F
        y, mu, var = self.empty(F, d.EP), self.empty(F), self.empty(F)
        sc, sh, inv1, inv2 = self.empty(F), self.empty(F), self.empty(F), self.empty(F)
        self._chk(xe, Ps, Pt, W1, W2, b2, gamma, beta, rm, rv)
        ws, wsb = self._wsargs(d)
        self._ecall("edge_mlp_fwd_bn", d, d.G, d.NF, d.NC, F, xe.data_ptr(), _ptr(xsc), _ptr(xsh),
              Ps.data_ptr(), Pt.data_ptr(), W1.data_ptr(), W2.data_ptr(), b2.data_ptr(),
              y.data_ptr(), mu.data_ptr(), var.data_ptr(), gamma.data_ptr(), beta.data_ptr(),
              _ptr(rm), _ptr(rv), float(momentum), float(eps), sc.data_ptr(), sh.data_ptr(),
              inv1.data_ptr(), inv2.data_ptr(), ws, wsb, _stream())
        return y, mu, var, sc, sh, inv1

    def source_fwd(self, d, y, sc, sh, Qt, Ws1, Ws2, bs2, hs_out, msg=None):
        """-> mom; ``msg`` (from ``msg_cache(d)``) receives the per-edge messages
        for source_bwd (pfsgnn_source_fwd_msg)."""
        if self._composed(d):
            return self._sp.source_fwd(d, y, sc, sh, Qt, Ws1, Ws2, bs2, hs_out)
        mom = self.empty(4, 2 * d.F, d.NS)
        self._chk(y, Qt, Ws1, Ws2, bs2, hs_out)
        ws, wsb = self._wsargs(d)
        args = (d.G, d.NF, d.NC, d.F, y.data_ptr(), _ptr(sc), _ptr(sh), Qt.data_ptr(),
                Ws1.data_ptr(), Ws2.data_ptr(), bs2.data_ptr(), mom.data_ptr(), hs_out.data_ptr())
        if msg is not None:
            _call("pfsgnn_source_fwd_msg", *args, msg.data_ptr(), ws, wsb, _stream())
        else:
            self._ecall("source_fwd", d, *args, ws, wsb, _stream())
        return mom

    def msg_cache(self, d):
        """A buffer for SModel's per-edge messages [2F][E] (pfsgnn_msg_bytes),
        or None when the current path recomputes them in the backward."""
        if self._composed(d) or d.sp is not None:
            return None
        n = lib().pfsgnn_msg_bytes(d.G, d.NF, d.NC, d.F)
        return torch.empty(n // 4, dtype=torch.float32, device=self.device) if n else None

    def tmask(self, d):
        """A buffer for TModel's LeakyReLU mask (pfsgnn_tmask_bytes), or None
        when the current edge path recomputes that layer in the backward."""
        if self._composed(d):
            return None
        if d.sp is not None:
            n = lib().pfsgnn_sl_tmask_bytes(d.sp.sl.ref, d.F)
            return torch.empty(n, dtype=torch.uint8, device=self.device) if n else None
        n = lib().pfsgnn_tmask_bytes(d.G, d.NF, d.NC, d.F)
        return torch.empty(n, dtype=torch.uint8, device=self.device) if n else None

    def target_fwd(self, d, y, sc, sh, Rs, Wt1, agg=None, tmask=None):
        """-> hsum; with ``agg`` = (Wt2, bt2, bscale) -> (hsum, Wt2 hsum + bscale bt2),
        the second Linear done in the class reduction's epilogue.  ``tmask``
        (from ``tmask(d)``) receives TModel's LeakyReLU mask for the backward."""
        if self._composed(d):
            hsum = self._sp.target_fwd(d, y, sc, sh, Rs, Wt1)
            if agg is None:
                return hsum
            Wt2, bt2, bscale = agg
            return hsum, self.lin(Wt2, 0, Wt2.shape[1], hsum, b=bt2, bscale=bscale)
        hsum = self.empty(2 * d.F, d.NT)
        Wt2 = bt2 = A = None
        bscale = 1.0
        if agg is not None:
            Wt2, bt2, bscale = agg
            self._chk(Wt2, bt2)
            assert Wt2.shape == (2 * d.F, 2 * d.F)
            A = self.empty(2 * d.F, d.NT)
        ws, wsb = self._wsargs(d)
        self._ecall("target_fwd", d, d.G, d.NF, d.NC, d.F, y.data_ptr(), _ptr(sc), _ptr(sh),
              Rs.data_ptr(), Wt1.data_ptr(), hsum.data_ptr(), _ptr(Wt2), _ptr(bt2),
              float(bscale), _ptr(A), _ptr(tmask), ws, wsb, _stream())
        return hsum if agg is None else (hsum, A)

    def target_bwd(self, d, y, sc, sh, Rs, Wt1, g_hsum, dWt1, want_gxe=False, g_xs=None,
                   tmask=None, bn_sums=None):
        """-> (GzT, gxe); with ``g_xs``: g_xs += Wt1[:, :F]^T GzT as well;
        ``tmask``: the forward's mask (target_fwd), read instead of recomputed.
        ``bn_sums`` = (Yp, mu, var, eps) of the BatchNorm whose backward reads the
        finished g_xs next (SModel's, gnn.py:154; complete graphs): its sums come
        out of the same call -> (GzT, gxe, partials for mlp_bwd's bn_part)."""
        if bn_sums is not None:
            assert g_xs is not None and not self._composed(d) and d.sp is None
            Yp, mu, var, eps = bn_sums
            self._chk(g_xs, Yp, mu, var)
            GzT = self.empty(2 * d.F, d.NS)
            gxe = self.empty(d.F, d.EP) if want_gxe else None
            part = self.empty((d.NS + 63) // 64, 32)
            g_hsum = g_hsum.contiguous()
            ws, wsb = self._wsargs(d)
            _call("pfsgnn_target_bwd_bn", d.G, d.NF, d.NC, d.F, y.data_ptr(), _ptr(sc), _ptr(sh),
                  Rs.data_ptr(), Wt1.data_ptr(), g_hsum.data_ptr(), GzT.data_ptr(),
                  dWt1.data_ptr(), _ptr(gxe), g_xs.data_ptr(), _ptr(tmask), Yp.data_ptr(),
                  mu.data_ptr(), var.data_ptr(), float(eps), part.data_ptr(), ws, wsb, _stream())
            return GzT, gxe, part
        if self._composed(d):
            out = self._sp.target_bwd(d, y, sc, sh, Rs, Wt1, g_hsum, dWt1, want_gxe=want_gxe)
            if g_xs is not None:
                self.lin_t(Wt1, 0, d.F, out[0], out=g_xs, add=True)
            return out
        self._chk(g_xs)
        GzT = self.empty(2 * d.F, d.NS)
        gxe = self.empty(d.F, d.EP) if want_gxe else None
        g_hsum = g_hsum.contiguous()
        ws, wsb = self._wsargs(d)
        self._ecall("target_bwd", d, d.G, d.NF, d.NC, d.F, y.data_ptr(), _ptr(sc), _ptr(sh),
              Rs.data_ptr(), Wt1.data_ptr(), g_hsum.data_ptr(), GzT.data_ptr(), dWt1.data_ptr(),
              _ptr(gxe), _ptr(g_xs), _ptr(tmask), ws, wsb, _stream())
        return GzT, gxe

    def source_bwd(self, d, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, tpart, g_next, bnstat,
                   dWs1, dWs2, dbs2, bn2=None, g_xt=None, tmask=None, msg=None):
        """-> (g_tot, GzS, Sg, Sgx).  With ``bn2`` = (gamma, var1, n, eps, dgamma,
        dbeta) (and ``bnstat``) the edge BatchNorm's backward is finished in the
        same call: -> (g_tot, GzS, None, None, (alpha, gam0, gam1)).  With
        ``g_xt``: g_xt += Ws1[:, :F]^T GzS as well."""
        if self._composed(d):
            out = self._sp.source_bwd(d, y, sc, sh, Qt, Ws1, Ws2, bs2, mean, coef, tpart, g_next,
                                      bnstat, dWs1, dWs2, dbs2)
            if g_xt is not None:
                self.lin_t(Ws1, 0, d.F, out[1], out=g_xt, add=True)
            if bn2 is None:
                return out
            gamma, var1, n, eps, dg, db = bn2
            cf = self.bn2_bwd_coef(out[2], out[3], bnstat[0], var1, gamma, n, eps, dg, db)
            return out[0], out[1], None, None, cf
        g_tot = self.empty(d.F, d.EP)
        GzS = self.empty(2 * d.F, d.NT)
        Rs = Wt1 = g_hsum = None
        if tpart is not None:
            Rs, Wt1, g_hsum = tpart
            g_hsum = g_hsum.contiguous()
        mu1 = inv1 = Sg = Sgx = None
        if bnstat is not None:
            mu1, inv1 = bnstat
            if bn2 is None:
                Sg, Sgx = self.empty(d.F), self.empty(d.F)
        mean = mean.contiguous()
        if g_next is not None:
            g_next = g_next.contiguous()
        ws, wsb = self._wsargs(d)
        head = (d.G, d.NF, d.NC, d.F, y.data_ptr(), _ptr(sc), _ptr(sh), Qt.data_ptr(),
                Ws1.data_ptr(), Ws2.data_ptr(), bs2.data_ptr(), mean.data_ptr(), coef.data_ptr(),
                _ptr(Rs), _ptr(Wt1), _ptr(g_hsum), _ptr(g_next), _ptr(mu1), _ptr(inv1))
        if bn2 is not None:
            assert bnstat is not None
            gamma, var1, n, eps, dg, db = bn2
            a, g0, g1 = self.empty(d.F), self.empty(d.F), self.empty(d.F)
            tail = (var1.data_ptr(), gamma.data_ptr(), int(n), float(eps), g_tot.data_ptr(),
                    GzS.data_ptr(), dWs1.data_ptr(), dWs2.data_ptr(), dbs2.data_ptr(),
                    a.data_ptr(), g0.data_ptr(), g1.data_ptr(), dg.data_ptr(), db.data_ptr(),
                    _ptr(g_xt), _ptr(tmask))
            if msg is not None:
                _call("pfsgnn_source_bwd_bn_msg", *head, *tail, msg.data_ptr(), ws, wsb, _stream())
            else:
                self._ecall("source_bwd_bn", d, *head, *tail, ws, wsb, _stream())
            return g_tot, GzS, None, None, (a, g0, g1)
        tail = (g_tot.data_ptr(), GzS.data_ptr(), dWs1.data_ptr(), dWs2.data_ptr(),
                dbs2.data_ptr(), _ptr(Sg), _ptr(Sgx), _ptr(g_xt), _ptr(tmask))
        if msg is not None:
            _call("pfsgnn_source_bwd_msg", *head, *tail, msg.data_ptr(), ws, wsb, _stream())
        else:
            self._ecall("source_bwd", d, *head, *tail, ws, wsb, _stream())
        return g_tot, GzS, Sg, Sgx

    def edge_bn_grad_sums(self, d, g, y, mu1, inv1):
        if d.sp is not None:   # (slot tensors hold 0 at padding: the column sums hold)
            return self._sp.edge_bn_grad_sums(d, g, y, mu1, inv1)
        Sg, Sgx = self.empty(d.F), self.empty(d.F)
        ws, wsb = self._wsargs(d)
        _call("pfsgnn_edge_bn_grad_sums", d.G, d.NF, d.NC, d.F, g.data_ptr(), y.data_ptr(),
              mu1.data_ptr(), inv1.data_ptr(), Sg.data_ptr(), Sgx.data_ptr(), ws, wsb, _stream())
        return Sg, Sgx

    def edge_mlp_bwd(self, d, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1, W2,
                     dW1, dW2, db2, want_gxe=True, nodes=None):
        """-> (gxe, GzEs, GzEt); with ``nodes`` = (g_xs, g_xt) the first Linear's
        node-input gradients are added in the reductions' epilogues and the
        result is (gxe, GzEs, GzEt, Vu), Vu = W1[:, 3F:4F]^T GzEt per class."""
        if self._composed(d):
            out = self._sp.edge_mlp_bwd(d, g_tot, alpha, gam0, gam1, y, xe, xsc, xsh, Ps, Pt, W1,
                                        W2, dW1, dW2, db2, want_gxe=want_gxe)
            if nodes is None:
                return out
            F = d.F
            self.lin_t(W1, 0, F, out[1], out=nodes[0], add=True)
            self.lin_t(W1, F, F, out[2], out=nodes[1], add=True)
            return out + (self.lin_t(W1, 3 * F, F, out[2]),)
        gxe = self.empty(d.F, d.EP) if want_gxe else None
        GzEs, GzEt = self.empty(4 * d.F, d.NS), self.empty(4 * d.F, d.NT)
        g_xs = g_xt = Vu = None
        if nodes is not None:
            g_xs, g_xt = nodes
            self._chk(g_xs, g_xt)
            Vu = self.empty(d.F, d.NT)
        ws, wsb = self._wsargs(d)
        self._ecall("edge_mlp_bwd", d, d.G, d.NF, d.NC, d.F, g_tot.data_ptr(), alpha.data_ptr(),
              gam0.data_ptr(), gam1.data_ptr(), y.data_ptr(), xe.data_ptr(), _ptr(xsc), _ptr(xsh),
              Ps.data_ptr(), Pt.data_ptr(), W1.data_ptr(), W2.data_ptr(), dW1.data_ptr(),
              dW2.data_ptr(), db2.data_ptr(), _ptr(gxe), GzEs.data_ptr(), GzEt.data_ptr(),
              _ptr(g_xs), _ptr(g_xt), _ptr(Vu), ws, wsb, _stream())
        return (gxe, GzEs, GzEt) if nodes is None else (gxe, GzEs, GzEt, Vu)

    def edge_apply(self, d, y, sc, sh):
        if d.sp is not None:
            return self._sp.edge_apply(d, y, sc, sh)
        out = self.empty(d.F, d.E)
        _call("pfsgnn_edges_from_canonical", y.data_ptr(), _ptr(sc), _ptr(sh), d.G, d.NF, d.NC,
              d.F, 2, None, 0, out.data_ptr(), _stream())
        return out

    # ------------------------------------------------------------ loss
    def _seed_args(self, seed):
        """(value, device pointer): a device int64 tensor is read by the kernels
        (graph-capturable: each replay sees its current value)."""
        if isinstance(seed, torch.Tensor):
            if not seed.is_cuda or seed.dtype != torch.int64 or seed.numel() != 1:
                raise ValueError("a tensor seed must be one int64 on the device")
            return 0, seed.data_ptr()
        return int(seed) & ((1 << 64) - 1), None

    def loss_fwd(self, d, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sharpness, noiselevel, seed,
                 want_time=False):
        n_prime, fiber_time = self.empty(d.NT), self.empty(d.NS)
        tmean, tvar = self.empty(d.NT), self.empty(d.NT)
        tt = self.empty(d.E) if want_time else None
        ci = ci.contiguous()
        ws, wsb = self._wsargs(d)
        _call("pfsgnn_loss_fwd", d.G, d.NF, d.NC, d.F, y.data_ptr(), _ptr(sc), _ptr(sh),
              Wd1.data_ptr(), bd1.data_ptr(), Wd2.data_ptr(), bd2.data_ptr(), ci.data_ptr(),
              float(scale), float(sharpness), float(noiselevel), *self._seed_args(seed),
              n_prime.data_ptr(), fiber_time.data_ptr(), tmean.data_ptr(), tvar.data_ptr(),
              _ptr(tt), ws, wsb, _stream())
        return n_prime, fiber_time, tmean, tvar, tt

    def loss_finalize(self, d, n_prime, fiber_time, tvar, ci, pclass, pfiber, total_time, nfields,
                      wutils, wvar, gscale=1.0):
        loss, utils, variance = self.empty(d.G), self.empty(d.G), self.empty(d.G)
        Gn, Gf, Gv = self.empty(d.NT), self.empty(d.NS), self.empty(d.NT)
        ci = ci.contiguous()
        _call("pfsgnn_loss_finalize", d.G, d.NF, d.NC, n_prime.data_ptr(), fiber_time.data_ptr(),
              tvar.data_ptr(), ci.data_ptr(), float(pclass), float(pfiber), float(total_time),
              float(nfields), float(wutils), float(wvar), loss.data_ptr(), utils.data_ptr(),
              variance.data_ptr(), Gn.data_ptr(), Gf.data_ptr(), Gv.data_ptr(), _stream())
        return loss, utils, variance, Gn, Gf, Gv

    def loss_bwd(self, d, y, sc, sh, Wd1, bd1, Wd2, bd2, ci, scale, sharpness, noiselevel, seed,
                 Gn, Gf, Gv, tmean, gscale, dWd1, dbd1, dWd2, dbd2, bn=None):
        """-> gxe; with ``bn`` = (mu1, inv1) of the final edge BatchNorm ->
        (gxe, its backward sums' per-block partials) (pfsgnn_loss_bwd_bn)."""
        gxe = self.empty(d.F, d.E)
        gs = None
        if isinstance(gscale, torch.Tensor):
            gs = gscale.reshape(1).to(torch.float32).contiguous()
        elif gscale != 1.0:
            gs = torch.full((1,), float(gscale), dtype=torch.float32, device=self.device)
        ci = ci.contiguous()
        ws, wsb = self._wsargs(d)
        if bn is not None:
            mu1, inv1 = bn
            self._chk(mu1, inv1)
            part = self.empty(lib().pfsgnn_loss_bn_parts(d.G, d.NF, d.NC), 2 * d.F)
            _call("pfsgnn_loss_bwd_bn", d.G, d.NF, d.NC, d.F, y.data_ptr(), _ptr(sc), _ptr(sh),
                  Wd1.data_ptr(), bd1.data_ptr(), Wd2.data_ptr(), bd2.data_ptr(), ci.data_ptr(),
                  float(scale), float(sharpness), float(noiselevel), *self._seed_args(seed),
                  Gn.data_ptr(), Gf.data_ptr(), Gv.data_ptr(), tmean.data_ptr(), _ptr(gs),
                  dWd1.data_ptr(), dbd1.data_ptr(), dWd2.data_ptr(), dbd2.data_ptr(),
                  gxe.data_ptr(), mu1.data_ptr(), inv1.data_ptr(), part.data_ptr(), ws, wsb,
                  _stream())
            return gxe, part
        _call("pfsgnn_loss_bwd", d.G, d.NF, d.NC, d.F, y.data_ptr(), _ptr(sc), _ptr(sh),
              Wd1.data_ptr(), bd1.data_ptr(), Wd2.data_ptr(), bd2.data_ptr(), ci.data_ptr(),
              float(scale), float(sharpness), float(noiselevel), *self._seed_args(seed),
              Gn.data_ptr(), Gf.data_ptr(), Gv.data_ptr(), tmean.data_ptr(), _ptr(gs),
              dWd1.data_ptr(), dbd1.data_ptr(), dWd2.data_ptr(), dbd2.data_ptr(), gxe.data_ptr(),
              ws, wsb, _stream())
        return gxe

    # ------------------------------------------------------------ graph building
    def build_complete(self, G, NF, NC, order=0):
        """edge_index [2, G*NF*NC] int64 of G complete bipartite graphs on the
        device; order 0 fiber-major (train.py:94), 1 class-major (graph.py:41)."""
        ei = torch.empty(2, G * NF * NC, dtype=torch.int64, device=self.device)
        _call("pfsgnn_build_complete", int(G), int(NF), int(NC), int(order), ei.data_ptr(),
              _stream())
        return ei

    # ------------------------------------------------------------ general graphs
    def sparse_layout(self, edge_index, G, NF, NC):
        """CSR layout of a batch that is not complete bipartite (pfsgnn.sparse).
        Raises ValueError if an edge is out of range or crosses graphs."""
        E = int(edge_index.shape[1])
        ei = edge_index.to(device=self.device, dtype=torch.int64).contiguous()
        i32 = dict(dtype=torch.int32, device=self.device)
        src_p, tgt_p, user_of, cls_ord = (torch.empty(E, **i32) for _ in range(4))
        fib_ptr = torch.empty(G * NF + 1, **i32)
        cls_ptr = torch.empty(G * NC + 1, **i32)
        status = torch.empty(1, **i32)
        ws = torch.empty(lib().pfsgnn_sparse_layout_ws_bytes(E), dtype=torch.uint8,
                         device=self.device)
        _call("pfsgnn_sparse_layout", ei.data_ptr(), E, int(G), int(NF), int(NC), src_p.data_ptr(),
              tgt_p.data_ptr(), user_of.data_ptr(), fib_ptr.data_ptr(), cls_ord.data_ptr(),
              cls_ptr.data_ptr(), status.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        if int(status.item()) != 0:
            raise ValueError("edge_index has an edge out of range or joining nodes of different "
                             f"graphs (G={G}, NF={NF}, NC={NC}; gnn.py:32-47 batching)")
        deg_t = (cls_ptr[1:] - cls_ptr[:-1]).to(torch.float32).reshape(1, -1).contiguous()
        return SparseGeo(E, src_p, tgt_p, user_of, fib_ptr, cls_ord, cls_ptr, deg_t)

    def sliced_max_nc(self, F):
        """Classes per graph the fused sliced kernels of the current edge path
        take at Fdim F (pfsgnn_sliced_max_nc: static + per-class LDS <= 160 KB);
        0 when that path has no sliced kernels (the bf16 edge-state paths)."""
        nc = ctypes.c_int(0)
        _call("pfsgnn_sliced_max_nc", int(F), ctypes.byref(nc))
        return nc.value

    def sliced_layout(self, sp, G, NF, NC):
        """Slices of 16 fibers over a sparse layout (pfsgnn_sliced_plan / _fill):
        the fused general-graph edge kernels' layout (pfsgnn_sliced.hip).  One
        host read (the position count EP) per edge_index."""
        i32 = dict(dtype=torch.int32, device=self.device)
        nsl = G * ((NF + 63) // 64) * 4
        fib, base, ln = torch.empty(nsl * 16, **i32), torch.empty(nsl, **i32), torch.empty(nsl, **i32)
        slot_of = torch.empty(G * NF, **i32)
        info = torch.empty(2, dtype=torch.int64, device=self.device)
        ws = torch.empty(lib().pfsgnn_sliced_plan_ws_bytes(int(G), int(NF)), dtype=torch.uint8,
                         device=self.device)
        _call("pfsgnn_sliced_plan", sp.fib_ptr.data_ptr(), int(G), int(NF), fib.data_ptr(),
              base.data_ptr(), ln.data_ptr(), slot_of.data_ptr(), info.data_ptr(), ws.data_ptr(),
              ws.numel(), _stream())
        EP, maxdeg = (int(v) for v in info.tolist())
        cls = torch.empty(EP, dtype=torch.uint8, device=self.device)
        pos_user = torch.empty(EP, **i32)
        pco = torch.empty(8 * max(maxdeg, 1), dtype=torch.float32, device=self.device)
        _call("pfsgnn_sliced_fill", sp.src_p.data_ptr(), sp.tgt_p.data_ptr(),
              sp.user_of.data_ptr(), sp.fib_ptr.data_ptr(), sp.E, int(NF), int(NC),
              slot_of.data_ptr(), base.data_ptr(), EP, maxdeg, cls.data_ptr(), pos_user.data_ptr(),
              pco.data_ptr(), _stream())
        return SlicedLayout(fib, base, ln, slot_of, cls, pos_user, pco, EP, sp.E, maxdeg)

    def gather_cols(self, X, idx, mode=0, out=None, Z=None):
        """out[c][e] (=, +=) X[c][idx[e]]; mode 2: X[c][idx[e]] * lrelu'(Z[c][e])."""
        C, N = X.shape
        E = idx.numel()
        if out is None:
            assert mode != 1
            out = self.empty(C, E)
        self._chk(X, Z, out)
        assert idx.dtype == torch.int32 and out.shape == (C, E)
        _call("pfsgnn_gather_cols", X.data_ptr(), C, N, idx.data_ptr(), E, _ptr(Z), int(mode),
              out.data_ptr(), _stream())
        return out

    def segment_sum(self, X, ord, ptr, nseg, act=False, out=None, add=False):
        C, E = X.shape
        if out is None:
            out, add = self.empty(C, nseg), False
        self._chk(X, out)
        assert ptr.numel() == nseg + 1
        _call("pfsgnn_segment_sum", X.data_ptr(), C, E, _ptr(ord), ptr.data_ptr(), int(nseg),
              int(act), out.data_ptr(), int(add), _stream())
        return out

    def segment_moments(self, M, ptr, nseg, hs_out):
        C, E = M.shape
        mom = self.empty(4, C, nseg)
        self._chk(M, hs_out)
        assert hs_out.shape == (4 * C, nseg)
        _call("pfsgnn_segment_moments", M.data_ptr(), C, E, ptr.data_ptr(), int(nseg),
              mom.data_ptr(), hs_out.data_ptr(), _stream())
        return mom

    def segment_moment_grad(self, M, seg, mean, coef):
        C, E = M.shape
        nseg = mean.shape[1]
        mean, coef = mean.contiguous(), coef.contiguous()
        self._chk(M, mean, coef)
        gm = self.empty(C, E)
        _call("pfsgnn_segment_moment_grad", M.data_ptr(), C, E, seg.data_ptr(), mean.data_ptr(),
              coef.data_ptr(), int(nseg), gm.data_ptr(), _stream())
        return gm

    def _rows_ws(self, C, N):
        nb = lib().pfsgnn_rows_ws_bytes(int(C), int(N))
        ws = self.workspace(getattr(self, "_dims", None))
        if ws.numel() < nb:
            return torch.empty(nb, dtype=torch.uint8, device=self.device)
        return ws

    def rows_stats(self, X):
        C, N = X.shape
        self._chk(X)
        mu, var = self.empty(C), self.empty(C)
        ws = self._rows_ws(C, N)
        _call("pfsgnn_rows_stats", X.data_ptr(), C, N, mu.data_ptr(), var.data_ptr(),
              ws.data_ptr(), ws.numel(), _stream())
        return mu, var

    def rows_bn_sums(self, g, y, mu, inv):
        C, N = y.shape
        self._chk(g, y, mu, inv)
        Sg, Sgx = self.empty(C), self.empty(C)
        ws = self._rows_ws(C, N)
        _call("pfsgnn_rows_bn_sums", g.data_ptr(), y.data_ptr(), C, N, mu.data_ptr(),
              inv.data_ptr(), Sg.data_ptr(), Sgx.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        return Sg, Sgx

    def rows_axpby(self, g, y, alpha, gam1, gam0, out=None):
        """out = alpha*g + gam1*y + gam0 per channel (out may be g or y)."""
        C, N = y.shape
        out = self.empty(C, N) if out is None else out
        self._chk(g, y, alpha, gam1, gam0, out)
        _call("pfsgnn_rows_axpby", g.data_ptr(), y.data_ptr(), C, N, alpha.data_ptr(),
              gam1.data_ptr(), gam0.data_ptr(), out.data_ptr(), _stream())
        return out

    # ------------------------------------------------------------ layout / optim
    def layout_analyze(self, edge_index, G, NF, NC):
        """-> (perm [E] int32, complete, caller order is fiber-major, caller order is canonical)."""
        E = edge_index.shape[1]
        ei = edge_index.to(device=self.device, dtype=torch.int64).contiguous()
        perm = torch.empty(E, dtype=torch.int32, device=self.device)
        status = torch.empty(3, dtype=torch.int32, device=self.device)
        ws = torch.empty(max(4 * E, 256), dtype=torch.uint8, device=self.device)
        _call("pfsgnn_layout_analyze", ei.data_ptr(), E, G, NF, NC, perm.data_ptr(),
              status.data_ptr(), ws.data_ptr(), ws.numel(), _stream())
        st = status.cpu().tolist()
        return perm, bool(st[0]), bool(st[1]), bool(st[2])

    def edges_to_canonical(self, x, lay):
        """Caller-order [E, F] -> canonical channel-major [F, E]; ``lay`` carries
        (G, NF, NC, mode, perm) (pfsgnn.gnn.Layout)."""
        E, F = x.shape
        x = x.to(device=self.device, dtype=torch.float32).contiguous()
        if lay.mode == SLOTS:
            sl = lay.sp.sl
            out = self.empty(F, sl.EP)
            _call("pfsgnn_edges_to_slots", x.data_ptr(), E, sl.EP, F, sl.pos_user.data_ptr(),
                  out.data_ptr(), _stream())
            return out
        out = self.empty(F, E)
        _call("pfsgnn_edges_to_canonical", x.data_ptr(), lay.G, lay.NF, lay.NC, F, lay.mode,
              _ptr(lay.perm), out.data_ptr(), _stream())
        return out

    def edges_from_canonical(self, y, sc, sh, lay, rowmajor=True):
        F, E = y.shape
        if lay.mode == SLOTS:
            sl = lay.sp.sl
            E = sl.E
            out = self.empty(E, F) if rowmajor else self.empty(F, E)
            _call("pfsgnn_edges_from_slots", y.data_ptr(), _ptr(sc), _ptr(sh), E, sl.EP, F,
                  sl.pos_user.data_ptr(), int(rowmajor), out.data_ptr(), _stream())
            return out
        out = self.empty(E, F) if rowmajor else self.empty(F, E)
        _call("pfsgnn_edges_from_canonical", y.data_ptr(), _ptr(sc), _ptr(sh), lay.G, lay.NF,
              lay.NC, F, lay.mode, _ptr(lay.perm), int(rowmajor), out.data_ptr(), _stream())
        return out

    def adam(self, p, g, m, v, step, lr, beta1, beta2, eps, weight_decay, live=None):
        """``step``: int, or a device float tensor holding the (already
        incremented) step count (capturable form).  ``live``: optional device
        uint8 mask; elements with 0 are skipped (parameters without a grad)."""
        self._chk(p, g, m, v)
        if live is not None:
            assert live.dtype == torch.uint8 and live.is_cuda and live.numel() == p.numel()
        if isinstance(step, torch.Tensor):
            if not step.is_cuda or step.dtype != torch.float32 or step.numel() != 1:
                raise ValueError("a tensor step must be one float32 on the device")
            sval, sptr = 0, step.data_ptr()
        else:
            sval, sptr = int(step), None
        _call("pfsgnn_adam", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
              sval, sptr, float(lr), float(beta1), float(beta2), float(eps), float(weight_decay),
              _ptr(live), _stream())
