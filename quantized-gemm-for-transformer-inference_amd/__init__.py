"""qgemm_amd -- host-side mirror of the reference's quantized-GEMM operator over the C-ABI.

The product is ``build/libqgemm.so`` (hand-written gfx950 HIP kernels behind the C-ABI in
``include/qgemm.h``).  This module binds that ABI with ctypes and mirrors the reference's
operator interface for the hot path:

    op_quantized_mm(X, W, O, range)   <- op_mm.cuh:67-101 (same name, argument meaning, asserts)
    op_mm_quantize(A, B, C)           <- the north-star C-ABI op_mm_quantize(A,B,C,M,N,K)
    pack_a / pack_b / mm_packed       <- the chain's stages (op_absmax+op_inv_divide+op_multiply,
                                         op_mm<int8_t,int>+op_dequantize+op_multiply)
    fill_uniform                      <- op_uniform_init (op_elemwise.cuh:728-744), seeded

PyTorch is plumbing here: it owns device memory and streams.  There is NO CPU fallback: if the
HIP library is missing, every compute entry point raises.

Import it by path (the directory name is not a Python identifier)::

    import importlib.util, sys
    spec = importlib.util.spec_from_file_location("qgemm_amd", "<repo>/quantized-gemm-for-transformer-inference_amd/__init__.py")
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import threading

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
REPO_DIR = os.path.dirname(PKG_DIR)
LIB_PATH = os.path.join(PKG_DIR, "build", "libqgemm.so")
HEADER_PATH = os.path.join(REPO_DIR, "include", "qgemm.h")
DIST_LIB_PATH = os.path.join(PKG_DIR, "build", "libqgemm_dist.so")
DIST_HEADER_PATH = os.path.join(REPO_DIR, "include", "qgemm_dist.h")

DEFAULT_RANGE = 127.0  # `range` at every reference call site (test_quantize.cu:76, timing_quantize.cu:43)
ROW_PAD = 256          # packed operand rows are padded to the GEMM macro-tile
K_PAD = 128            # packed operand k is padded to the GEMM k-step

# Every symbol include/qgemm.h declares (checked against the header by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "op_mm_quantize",
    "op_mm_quantize_ex",
    "op_mm_quantize_workspace_size",
    "op_mm_quantize_ws",
    "qgemm_packed_size",
    "qgemm_pack_a",
    "qgemm_pack_b",
    "qgemm_mm_packed",
    "qgemm_mm_packed_i32",
    "qgemm_mm_fp32",
    "qgemm_error_stats",
    "qgemm_linear_workspace_size",
    "qgemm_linear",
    "op_mm_quantize_prepacked",
    "op_mm_quantize_prepacked_workspace_size",
    "op_mm_quantize_prepacked_ws",
    "qgemm_softmax_rows",
    "qgemm_add_layernorm_rows",
    "qgemm_encoder_create",
    "qgemm_encoder_forward",
    "qgemm_encoder_destroy",
    "qgemm_mm_outlier_workspace_size",
    "qgemm_mm_outlier",
    "qgemm_outlier_count",
    "qgemm_set_gemm_events",
    "qgemm_set_event_mode",
    "qgemm_fill_uniform",
    "qgemm_gemm_plan",
    "qgemm_version",
)

# Every symbol include/qgemm_dist.h declares (libqgemm_dist.so: M-shards + RCCL all-gather).
DIST_EXPORTED_SYMBOLS = (
    "qgemm_shard_rows",
    "op_mm_quantize_shard",
    "qgemm_comm_unique_id",
    "qgemm_comm_init_rank",
    "qgemm_comm_init_all",
    "qgemm_comm_destroy",
    "qgemm_comm_count",
    "qgemm_comm_user_rank",
    "qgemm_allgather_rows",
    "qgemm_allgather_plan",
    "qgemm_allgather_chunk_plan",
    "op_mm_quantize_shard_pipelined_workspace_size",
    "op_mm_quantize_shard_pipelined",
    "qgemm_node_allgather_plan",
    "qgemm_node_mm_quantize",
)
COMM_ID_BYTES = 128

HIP_ERROR_INVALID_VALUE = 1

_lock = threading.Lock()
_lib = None
_dist = None


class QGemmError(RuntimeError):
    """A non-zero hipError_t returned through the C-ABI."""

    def __init__(self, fn: str, code: int):
        super().__init__(f"{fn} failed with hipError_t {code}")
        self.code = code


def build(verbose: bool = False) -> str:
    """Compile libqgemm.so and the harness binaries for gfx950 (hipcc; see Makefile)."""
    out = None if verbose else subprocess.DEVNULL
    jobs = str(min(8, os.cpu_count() or 1))
    subprocess.run(["make", "-C", PKG_DIR, "-j", jobs, "all"], check=True, stdout=out)
    return LIB_PATH


def load() -> ctypes.CDLL:
    """Load the HIP library (no fallback: raises if it was not built)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"qgemm HIP library not built: {LIB_PATH} missing (run build())")
        L = ctypes.CDLL(LIB_PATH)
        i64, i32, f32, vp, sz = ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t
        L.op_mm_quantize.argtypes = [vp, vp, vp, i32, i32, i32]
        L.op_mm_quantize.restype = i32
        L.op_mm_quantize_ex.argtypes = [vp, i64, i64, vp, i64, i64, vp, i64, i64, i32, i32, i32, f32, vp]
        L.op_mm_quantize_ex.restype = i32
        L.op_mm_quantize_workspace_size.argtypes = [i32, i32, i32]
        L.op_mm_quantize_workspace_size.restype = sz
        L.op_mm_quantize_ws.argtypes = [vp, i64, i64, vp, i64, i64, vp, i64, i64, i32, i32, i32, f32, vp, sz, vp]
        L.op_mm_quantize_ws.restype = i32
        L.qgemm_packed_size.argtypes = [i32, i32]
        L.qgemm_packed_size.restype = sz
        L.qgemm_pack_a.argtypes = [vp, i64, i64, i32, i32, f32, vp, vp]
        L.qgemm_pack_a.restype = i32
        L.qgemm_pack_b.argtypes = [vp, i64, i64, i32, i32, f32, vp, vp]
        L.qgemm_pack_b.restype = i32
        L.qgemm_mm_packed.argtypes = [vp, vp, vp, i64, i64, i32, i32, i32, f32, vp]
        L.qgemm_mm_packed.restype = i32
        L.qgemm_mm_packed_i32.argtypes = [vp, vp, vp, i32, i32, i32, vp]
        L.qgemm_mm_packed_i32.restype = i32
        L.qgemm_mm_fp32.argtypes = [vp, i64, i64, vp, i64, i64, vp, i64, i64, i32, i32, i32, vp]
        L.qgemm_mm_fp32.restype = i32
        L.qgemm_error_stats.argtypes = [vp, vp, i64, i32, vp, vp]
        L.qgemm_error_stats.restype = i32
        L.qgemm_linear_workspace_size.argtypes = [i32, i32, i32]
        L.qgemm_linear_workspace_size.restype = sz
        L.qgemm_linear.argtypes = [vp, i64, i32, i32, vp, i32, vp, i32, vp, i64, vp, sz, vp]
        L.qgemm_linear.restype = i32
        L.op_mm_quantize_prepacked.argtypes = [vp, vp, vp, i32, i32, i32]
        L.op_mm_quantize_prepacked.restype = i32
        L.op_mm_quantize_prepacked_workspace_size.argtypes = [i32, i32, i32]
        L.op_mm_quantize_prepacked_workspace_size.restype = sz
        L.op_mm_quantize_prepacked_ws.argtypes = [vp, i64, vp, vp, i64, i32, i32, i32, vp, sz, vp]
        L.op_mm_quantize_prepacked_ws.restype = i32
        L.qgemm_softmax_rows.argtypes = [vp, vp, i64, i32, f32, vp]
        L.qgemm_softmax_rows.restype = i32
        L.qgemm_add_layernorm_rows.argtypes = [vp, vp, vp, i64, i32, vp]
        L.qgemm_add_layernorm_rows.restype = i32
        L.qgemm_encoder_create.argtypes = [i32, i32, i32, i32, i32, ctypes.c_uint64, ctypes.POINTER(vp)]
        L.qgemm_encoder_create.restype = i32
        L.qgemm_encoder_forward.argtypes = [vp, vp, vp, i32, vp]
        L.qgemm_encoder_forward.restype = i32
        L.qgemm_encoder_destroy.argtypes = [vp]
        L.qgemm_encoder_destroy.restype = i32
        L.qgemm_mm_outlier_workspace_size.argtypes = [i32, i32, i32]
        L.qgemm_mm_outlier_workspace_size.restype = sz
        L.qgemm_mm_outlier.argtypes = [vp, vp, vp, i32, i32, i32, f32, vp, sz, vp]
        L.qgemm_mm_outlier.restype = i32
        L.qgemm_outlier_count.argtypes = [i32, vp, ctypes.POINTER(i32)]
        L.qgemm_outlier_count.restype = i32
        L.qgemm_fill_uniform.argtypes = [vp, i64, ctypes.c_uint64, f32, f32, vp]
        L.qgemm_fill_uniform.restype = i32
        L.qgemm_set_gemm_events.argtypes = [vp, vp]
        L.qgemm_set_gemm_events.restype = i32
        L.qgemm_set_event_mode.argtypes = [i32]
        L.qgemm_set_event_mode.restype = i32
        L.qgemm_gemm_plan.argtypes = [i32, i32, i32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_char_p)]
        L.qgemm_gemm_plan.restype = i32
        L.qgemm_version.argtypes = []
        L.qgemm_version.restype = ctypes.c_char_p
        _lib = L
        return L


def load_dist() -> ctypes.CDLL:
    """Load libqgemm_dist.so (M-sharded calls + the RCCL all-gather; no fallback)."""
    global _dist
    load()
    with _lock:
        if _dist is not None:
            return _dist
        if not os.path.exists(DIST_LIB_PATH):
            raise RuntimeError(f"qgemm multi-GPU library not built: {DIST_LIB_PATH} missing (run build())")
        D = ctypes.CDLL(DIST_LIB_PATH)
        i32, vp = ctypes.c_int, ctypes.c_void_p
        D.qgemm_shard_rows.argtypes = [i32, i32, i32, ctypes.POINTER(i32), ctypes.POINTER(i32)]
        D.qgemm_shard_rows.restype = i32
        D.op_mm_quantize_shard.argtypes = [vp, vp, vp, i32, i32, i32, i32, i32, vp]
        D.op_mm_quantize_shard.restype = i32
        D.qgemm_comm_unique_id.argtypes = [vp]
        D.qgemm_comm_unique_id.restype = i32
        D.qgemm_comm_init_rank.argtypes = [ctypes.POINTER(vp), i32, vp, i32]
        D.qgemm_comm_init_rank.restype = i32
        D.qgemm_comm_init_all.argtypes = [ctypes.POINTER(vp), i32, ctypes.POINTER(i32)]
        D.qgemm_comm_init_all.restype = i32
        D.qgemm_comm_destroy.argtypes = [vp]
        D.qgemm_comm_destroy.restype = i32
        D.qgemm_comm_count.argtypes = [vp, ctypes.POINTER(i32)]
        D.qgemm_comm_count.restype = i32
        D.qgemm_comm_user_rank.argtypes = [vp, ctypes.POINTER(i32)]
        D.qgemm_comm_user_rank.restype = i32
        D.qgemm_allgather_rows.argtypes = [vp, i32, i32, i32, i32, vp, vp]
        D.qgemm_allgather_rows.restype = i32
        i64p = ctypes.POINTER(ctypes.c_int64)
        D.qgemm_allgather_plan.argtypes = [i32, i32, i32, i64p, i64p, ctypes.POINTER(i32), i32]
        D.qgemm_allgather_plan.restype = i32
        D.qgemm_allgather_chunk_plan.argtypes = [i32, i32, i32, i32, i64p, i64p, ctypes.POINTER(i32), i32]
        D.qgemm_allgather_chunk_plan.restype = i32
        D.op_mm_quantize_shard_pipelined_workspace_size.argtypes = [i32, i32, i32, i32, i32]
        D.op_mm_quantize_shard_pipelined_workspace_size.restype = ctypes.c_size_t
        D.op_mm_quantize_shard_pipelined.argtypes = [vp, vp, vp, i32, i32, i32, i32, i32, i32, vp, vp, ctypes.c_size_t,
                                                     vp, vp]
        D.op_mm_quantize_shard_pipelined.restype = i32
        D.qgemm_node_allgather_plan.argtypes = [i32, i32, i32, ctypes.POINTER(CollOp), i32]
        D.qgemm_node_allgather_plan.restype = i32
        D.qgemm_node_mm_quantize.argtypes = [vp, vp, vp, i32, i32, i32, i32, ctypes.POINTER(i32), vp, vp, i32]
        D.qgemm_node_mm_quantize.restype = i32
        _dist = D
        return D


def shard_rows(m: int, world: int, rank: int) -> tuple:
    """(m0, rows) of rank's contiguous row shard (qgemm_shard_rows)."""
    m0, rows = ctypes.c_int(), ctypes.c_int()
    _check("qgemm_shard_rows", load_dist().qgemm_shard_rows(m, world, rank, ctypes.byref(m0), ctypes.byref(rows)))
    return m0.value, rows.value


class CollOp(ctypes.Structure):
    """qgemm_coll_op (include/qgemm_dist.h): one planned collective of the one-process node path."""
    _fields_ = [("rank", ctypes.c_int), ("root", ctypes.c_int), ("send_off", ctypes.c_int64),
                ("recv_off", ctypes.c_int64), ("count", ctypes.c_int64)]


def node_allgather_plan(m: int, n: int, ndev: int) -> list:
    """The collectives qgemm_node_mm_quantize enqueues in its ONE RCCL group, in issue order, as
    [(rank, root, send_off, recv_off, count)] (root -1: in-place all-gather; else an in-place broadcast)."""
    D = load_dist()
    cnt = D.qgemm_node_allgather_plan(m, n, ndev, None, 0)
    if cnt < 0:
        raise QGemmError("qgemm_node_allgather_plan", -cnt)
    ops = (CollOp * max(1, cnt))()
    got = D.qgemm_node_allgather_plan(m, n, ndev, ops, cnt)
    if got != cnt:
        raise QGemmError("qgemm_node_allgather_plan", -got if got < 0 else 1)
    return [(o.rank, o.root, o.send_off, o.recv_off, o.count) for o in ops[:cnt]]


def allgather_plan(m: int, n: int, world: int) -> list:
    """The collectives qgemm_allgather_rows enqueues for an m x n C over `world` ranks, as
    [(first, count, root)]: root -1 = one in-place all-gather of `count` floats per rank starting at
    element `first`; root >= 0 = an in-place broadcast of [first, first + count) from that rank."""
    cap = max(1, world)
    first, count, root = (ctypes.c_int64 * cap)(), (ctypes.c_int64 * cap)(), (ctypes.c_int * cap)()
    ops = load_dist().qgemm_allgather_plan(m, n, world, first, count, root, cap)
    if ops < 0:
        raise QGemmError("qgemm_allgather_plan", -ops)
    return [(first[i], count[i], root[i]) for i in range(ops)]


def allgather_chunk_plan(m: int, n: int, world: int, chunks: int) -> list:
    """The broadcasts op_mm_quantize_shard_pipelined issues, chunk-major, as [(first, count, root)]
    (qgemm_allgather_chunk_plan): each moves `count` floats at element `first` of C from rank `root`."""
    D = load_dist()
    cnt = D.qgemm_allgather_chunk_plan(m, n, world, chunks, None, None, None, 0)
    if cnt < 0:
        raise QGemmError("qgemm_allgather_chunk_plan", -cnt)
    cap = max(1, cnt)
    first, count, root = (ctypes.c_int64 * cap)(), (ctypes.c_int64 * cap)(), (ctypes.c_int * cap)()
    got = D.qgemm_allgather_chunk_plan(m, n, world, chunks, first, count, root, cap)
    if got != cnt:
        raise QGemmError("qgemm_allgather_chunk_plan", -got if got < 0 else 1)
    return [(first[i], count[i], root[i]) for i in range(cnt)]


def op_mm_quantize_shard_pipelined(A, B, C, world: int, rank: int, chunks: int, comm=None, gather_stream=None,
                                   workspace=None) -> None:
    """op_mm_quantize_shard with the all-gather of C pipelined under the chunks' compute
    (op_mm_quantize_shard_pipelined): on return (stream order) every rank's C holds all rows."""
    import torch
    for t, nm in ((A, "A"), (B, "B"), (C, "C")):
        _require_device_f32(t, nm)
        assert t.is_contiguous(), f"{nm} must be contiguous row-major"
    M, K = A.shape
    N = B.shape[1]
    assert B.shape[0] == K and C.shape == (M, N), "A m x k, B k x n, C m x n"
    D = load_dist()
    need = D.op_mm_quantize_shard_pipelined_workspace_size(M, N, K, world, chunks)
    if workspace is None:
        workspace = torch.empty(need, dtype=torch.uint8, device=A.device)
    assert workspace.numel() >= need, "workspace too small"
    s = _stream(A.device)
    g = ctypes.c_void_p(gather_stream.cuda_stream) if gather_stream is not None else s  # a torch.cuda.Stream
    _check("op_mm_quantize_shard_pipelined",
           D.op_mm_quantize_shard_pipelined(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, world, rank, chunks,
                                            comm.handle if comm is not None else None, workspace.data_ptr(),
                                            workspace.numel(), s, g))


def op_mm_quantize_shard(A, B, C, world: int, rank: int) -> None:
    """Rows [m0, m0 + rows) of C = op_mm_quantize(A, B) on this rank (per-rank pointer offsets into the
    full row-major A and C; bit-identical to those rows of the one-GPU call)."""
    for t, nm in ((A, "A"), (B, "B"), (C, "C")):
        _require_device_f32(t, nm)
        assert t.is_contiguous(), f"{nm} must be contiguous row-major"
    M, K = A.shape
    N = B.shape[1]
    assert B.shape[0] == K and C.shape == (M, N), "A m x k, B k x n, C m x n"
    _check("op_mm_quantize_shard", load_dist().op_mm_quantize_shard(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K,
                                                                    world, rank, _stream(A.device)))


class Comm:
    """An RCCL communicator of libqgemm_dist.so (one rank per process, or world == 1 alone)."""

    def __init__(self, world: int, rank: int, unique_id: bytes):
        assert len(unique_id) == COMM_ID_BYTES
        self.world, self.rank = world, rank
        self._id = ctypes.create_string_buffer(unique_id, COMM_ID_BYTES)
        self.handle = ctypes.c_void_p()
        _check("qgemm_comm_init_rank",
               load_dist().qgemm_comm_init_rank(ctypes.byref(self.handle), world, self._id, rank))

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        _check("qgemm_comm_unique_id", load_dist().qgemm_comm_unique_id(buf))
        return buf.raw

    def allgather_rows(self, C) -> None:
        """In place: every rank's row shard of the full C (m x n) to every rank (qgemm_allgather_rows)."""
        _require_device_f32(C, "C")
        assert C.is_contiguous()
        _check("qgemm_allgather_rows", load_dist().qgemm_allgather_rows(C.data_ptr(), C.shape[0], C.shape[1], self.world,
                                                                        self.rank, self.handle, _stream(C.device)))

    def count(self) -> int:
        """The communicator's size as RCCL reports it (ncclCommCount)."""
        c = ctypes.c_int(-1)
        _check("qgemm_comm_count", load_dist().qgemm_comm_count(self.handle, ctypes.byref(c)))
        return c.value

    def user_rank(self) -> int:
        r = ctypes.c_int(-1)
        _check("qgemm_comm_user_rank", load_dist().qgemm_comm_user_rank(self.handle, ctypes.byref(r)))
        return r.value

    def close(self) -> None:
        if self.handle:
            _check("qgemm_comm_destroy", load_dist().qgemm_comm_destroy(self.handle))
            self.handle = ctypes.c_void_p()


def version() -> str:
    return load().qgemm_version().decode()


def source_hash() -> str:
    """The Makefile's SRC_HASH recomputed from this tree: sha256 of the Makefile, csrc/*.{hip,h,cpp}, include/*.h and
    the harness sources src/*.cpp, src/*/*.{h,cuh}
    concatenated in sorted path order (make's $(sort) of the same relative paths), first 16 hex digits."""
    import glob
    import hashlib
    rel = ["Makefile"]
    for pat in ("csrc/*.hip", "csrc/*.h", "csrc/*.cpp", "../include/*.h", "src/*.cpp", "src/*.hip", "src/*/*.h",
                "src/*/*.cuh"):
        rel += [os.path.relpath(p, PKG_DIR) for p in glob.glob(os.path.join(PKG_DIR, pat))]
    h = hashlib.sha256()
    for r in sorted(rel):
        with open(os.path.join(PKG_DIR, r), "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def binary_hash() -> str:
    """The source hash compiled into the loaded libqgemm.so (the `src=` field of qgemm_version())."""
    for field in version().split():
        if field.startswith("src="):
            return field[4:]
    return "none"


def file_hash(path: str = LIB_PATH) -> str:
    """The source hash tagged inside a built libqgemm.so, read from the file (no dlopen): "" if absent."""
    import re
    try:
        with open(path, "rb") as f:
            m = re.search(rb"QGEMM_SRC_HASH=([0-9a-f]{16})", f.read())
    except OSError:
        return ""
    return m.group(1).decode() if m else ""


def check_binary() -> str:
    """Refuse a libqgemm.so built from other sources than this tree's (a stale build/ shipped with the
    snapshot): returns the hash, raises RuntimeError on a mismatch."""
    want, got = source_hash(), binary_hash()
    if got != want:
        raise RuntimeError(f"{LIB_PATH} was built from sources src={got}, this tree is src={want}: rebuild "
                           "(make -C quantized-gemm-for-transformer-inference_amd all)")
    return got


def _check(fn: str, rc: int) -> None:
    if rc != 0:
        raise QGemmError(fn, rc)


def _stream(device=None):
    import torch
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_device_f32(t, name):
    import torch
    assert isinstance(t, torch.Tensor) and t.dim() == 2, f"{name} must be a 2-D tensor"
    assert t.is_cuda, f"{name}.on_device (op_mm.cuh:72)"
    assert t.dtype == torch.float32, f"{name} must be float32 (op_quantized_mm is instantiated at T=float)"


# ------------------------------------------------------------------------------- the operator
def op_quantized_mm(X, W, O, range: float = DEFAULT_RANGE) -> None:  # noqa: A002 - reference name
    """O = quantized X @ W, in place -- the reference's ``op_quantized_mm<float>`` (op_mm.cuh:67-101).

    Same argument meaning and the same asserts (op_mm.cuh:71-72): ``X.h == O.h && W.w == O.w &&
    X.w == W.h`` and all three on the device.  Strided/transposed views are accepted, as the
    reference's Index() macro accepts them.  Enqueued on torch's current stream.
    """
    for t, nm in ((X, "X"), (W, "W"), (O, "O")):
        _require_device_f32(t, nm)
    assert X.shape[0] == O.shape[0] and W.shape[1] == O.shape[1] and X.shape[1] == W.shape[0], \
        "X.h == O.h && W.w == O.w && X.w == W.h (op_mm.cuh:71)"
    M, K = X.shape
    N = W.shape[1]
    if M == 0 or N == 0:
        return
    rc = load().op_mm_quantize_ex(X.data_ptr(), X.stride(0), X.stride(1), W.data_ptr(), W.stride(0), W.stride(1),
                                  O.data_ptr(), O.stride(0), O.stride(1), M, N, K, float(range), _stream(X.device))
    _check("op_mm_quantize_ex", rc)


def op_mm_quantize(A, B, C=None):
    """The north-star C-ABI op_mm_quantize(A, B, C, M, N, K) on contiguous row-major tensors."""
    import torch
    _require_device_f32(A, "A")
    _require_device_f32(B, "B")
    M, K = A.shape
    N = B.shape[1]
    if C is None:
        C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    op_quantized_mm(A, B, C, DEFAULT_RANGE)
    return C


# ------------------------------------------------------------------------- packed operands
def _round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


class Packed:
    """A packed (quantized, MFMA-ready) operand: [scale f32][reserved u32 partials][q int8, rows_pad x k_pad]."""

    def __init__(self, buf, rows: int, k: int, range_: float):
        self.buf, self.rows, self.k, self.range = buf, rows, k, range_
        self.rows_pad, self.k_pad = _round_up(rows, ROW_PAD), _round_up(k, K_PAD)

    @property
    def scale(self):
        """Cx (for A) or Cw (for B), padded to rows_pad."""
        import torch
        return self.buf[: 4 * self.rows_pad].view(torch.float32)

    @property
    def q_raw(self):
        """The packed bytes as stored: FRAGMENT-MAJOR (csrc/qgemm_internal.h fofs) -- 1-KiB blocks of 16
        rows x 64 k in MFMA lane order, block (rg, kb) at (rg * k_pad / 64 + kb) * 1024."""
        import torch
        parts = -(-(self.k - 1) // 256) if self.k > 1 else 1
        off = _round_up(4 * self.rows_pad * (1 + parts), 256)
        return self.buf[off: off + self.rows_pad * self.k_pad].view(torch.int8)

    @property
    def q(self):
        """X_int8 (rows_pad x k_pad) or W_int8^T (n_pad x k_pad), zero padded, row-major -- a COPY, un-permuted
        from the fragment-major storage ([rg][kb][kc][r][16 B] -> [rg][r][kb][kc][16 B]): writes into it do not
        reach the packed buffer; in-place edits go through q_raw."""
        r16, kb = self.rows_pad // 16, self.k_pad // 64
        return (self.q_raw.view(r16, kb, 4, 16, 16).permute(0, 3, 1, 2, 4).reshape(self.rows_pad, self.k_pad))


def _alloc_packed(rows, k, device):
    import torch
    nbytes = load().qgemm_packed_size(rows, k)
    return torch.empty(nbytes, dtype=torch.uint8, device=device)


def pack_a(A, range: float = DEFAULT_RANGE) -> Packed:  # noqa: A002
    """Cx = absmax rows (op_mm.cuh:76-77) and X_int8 (op_mm.cuh:82-87), fused."""
    _require_device_f32(A, "A")
    M, K = A.shape
    p = Packed(_alloc_packed(M, K, A.device), M, K, range)
    _check("qgemm_pack_a", load().qgemm_pack_a(A.data_ptr(), A.stride(0), A.stride(1), M, K, float(range),
                                              p.buf.data_ptr(), _stream(A.device)))
    return p


def pack_b(B, range: float = DEFAULT_RANGE) -> Packed:  # noqa: A002
    """Cw = absmax columns (op_mm.cuh:78-79) and W_int8 (op_mm.cuh:84-89), stored transposed."""
    _require_device_f32(B, "B")
    K, N = B.shape
    p = Packed(_alloc_packed(N, K, B.device), N, K, range)
    _check("qgemm_pack_b", load().qgemm_pack_b(B.data_ptr(), B.stride(0), B.stride(1), K, N, float(range),
                                              p.buf.data_ptr(), _stream(B.device)))
    return p


def mm_packed(pa: Packed, pb: Packed, C=None):
    """int8 MFMA GEMM + fused dequantize (op_mm.cuh:92-99) on packed operands."""
    import torch
    assert pa.k == pb.k, "X.w == W.h"
    if C is None:
        C = torch.empty((pa.rows, pb.rows), dtype=torch.float32, device=pa.buf.device)
    _require_device_f32(C, "C")
    assert C.shape == (pa.rows, pb.rows)
    _check("qgemm_mm_packed", load().qgemm_mm_packed(pa.buf.data_ptr(), pb.buf.data_ptr(), C.data_ptr(), C.stride(0),
                                                    C.stride(1), pa.rows, pb.rows, pa.k, float(pa.range),
                                                    _stream(C.device)))
    return C


def mm_packed_i32(pa: Packed, pb: Packed):
    """The raw int32 accumulator O_int32 (op_mm.cuh:92-93)."""
    import torch
    acc = torch.empty((pa.rows, pb.rows), dtype=torch.int32, device=pa.buf.device)
    _check("qgemm_mm_packed_i32", load().qgemm_mm_packed_i32(pa.buf.data_ptr(), pb.buf.data_ptr(), acc.data_ptr(),
                                                            pa.rows, pb.rows, pa.k, _stream(acc.device)))
    return acc


def mm_fp32(A, B, C=None):
    """The reference's unquantized op_mm<float,float> (op_mm.cuh:49-65), bit-exact, on the GPU."""
    import torch
    _require_device_f32(A, "A")
    _require_device_f32(B, "B")
    M, K = A.shape
    N = B.shape[1]
    assert B.shape[0] == K
    if C is None:
        C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    _check("qgemm_mm_fp32", load().qgemm_mm_fp32(A.data_ptr(), A.stride(0), A.stride(1), B.data_ptr(), B.stride(0),
                                                B.stride(1), C.data_ptr(), C.stride(0), C.stride(1), M, N, K,
                                                _stream(A.device)))
    return C


def error_stats(C, O, reference_order: bool = False) -> dict:
    """Quantization error of O against the unquantized C, on the device (qgemm_error_stats).

    signed_mean_ref is the reference's printed metric (timing_quantize.cu:67-70 via tensor.cuh:201-211,
    sequential fp32) -- only with reference_order=True (one GPU lane, slow at large sizes)."""
    import torch
    _require_device_f32(C, "C")
    _require_device_f32(O, "O")
    assert C.shape == O.shape and C.is_contiguous() and O.is_contiguous()
    st = torch.empty(5, dtype=torch.float64, device=C.device)
    _check("qgemm_error_stats", load().qgemm_error_stats(C.data_ptr(), O.data_ptr(), C.numel(),
                                                        1 if reference_order else 0, st.data_ptr(),
                                                        _stream(C.device)))
    v = st.cpu().tolist()
    return dict(signed_mean_ref=v[0], signed_mean=v[1], mean_abs=v[2], max_abs=v[3],
                rel=v[2] / v[4] if v[4] else float("nan"))


def linear(X, pw: Packed, bias=None, relu: bool = False, Y=None):
    """LinearLayer.forward on the quantized path (linear.cuh:50-54): quantized_mm(X, W) [+ b] [relu],
    W packed once by pack_b."""
    import torch
    _require_device_f32(X, "X")
    assert X.stride(1) == 1 and X.shape[1] == pw.k
    assert pw.range == DEFAULT_RANGE, f"qgemm_linear needs a weight packed with range {DEFAULT_RANGE}"
    M, K = X.shape
    N = pw.rows
    if Y is None:
        Y = torch.empty((M, N), dtype=torch.float32, device=X.device)
    assert Y.shape == (M, N) and Y.stride(1) == 1
    L = load()
    ws = torch.empty(max(1, L.qgemm_linear_workspace_size(M, N, K)), dtype=torch.uint8, device=X.device)
    b = 0 if bias is None else bias.data_ptr()
    _check("qgemm_linear", L.qgemm_linear(X.data_ptr(), X.stride(0), M, K, pw.buf.data_ptr(), N, b, 1 if relu else 0,
                                          Y.data_ptr(), Y.stride(0), ws.data_ptr(), ws.numel(), _stream(X.device)))
    return Y


def op_mm_quantize_prepacked(A, pb: Packed, C=None):
    """The weight-cache drop-in: C = op_quantized_mm(A, W) with W packed once by
    pack_b; A quantized on every call (op_mm.cuh:76-77, 82-87), then the int8 GEMM + dequantize."""
    import torch
    _require_device_f32(A, "A")
    assert A.stride(1) == 1 and A.shape[1] == pb.k, "X.w == W.h"
    # the C entry point quantizes A with range 127 and dequantizes with 1/127^2: a B packed with another
    # range would silently differ from op_mm_quantize
    assert pb.range == DEFAULT_RANGE, f"op_mm_quantize_prepacked needs a B packed with range {DEFAULT_RANGE}"
    M, K = A.shape
    N = pb.rows
    if C is None:
        C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    assert C.shape == (M, N) and C.stride(1) == 1
    L = load()
    ws = torch.empty(max(1, L.op_mm_quantize_prepacked_workspace_size(M, N, K)), dtype=torch.uint8, device=A.device)
    _check("op_mm_quantize_prepacked_ws",
           L.op_mm_quantize_prepacked_ws(A.data_ptr(), A.stride(0), pb.buf.data_ptr(), C.data_ptr(), C.stride(0), M, N,
                                         K, ws.data_ptr(), ws.numel(), _stream(A.device)))
    return C


def softmax_rows(S, scale: float = 1.0, P=None):
    """op_multiply(S, scale) + op_softmax (attention.cuh:65-68) over the rows of a contiguous S."""
    import torch
    _require_device_f32(S, "S")
    assert S.is_contiguous()
    P = torch.empty_like(S) if P is None else P
    _check("qgemm_softmax_rows", load().qgemm_softmax_rows(S.data_ptr(), P.data_ptr(), S.numel() // S.shape[-1],
                                                          S.shape[-1], float(scale), _stream(S.device)))
    return P


def add_layernorm_rows(A, B, Y=None):
    """op_add(A, B) + op_layernorm (transformer.cu:58-59, op_layernorm.cuh as written)."""
    import torch
    for t, nm in ((A, "A"), (B, "B")):
        _require_device_f32(t, nm)
        assert t.is_contiguous()
    assert A.shape == B.shape
    Y = torch.empty_like(A) if Y is None else Y
    _check("qgemm_add_layernorm_rows", load().qgemm_add_layernorm_rows(A.data_ptr(), B.data_ptr(), Y.data_ptr(),
                                                                      A.numel() // A.shape[-1], A.shape[-1],
                                                                      _stream(A.device)))
    return Y


def mm_outlier(A, B, threshold: float = 6.0, C=None):
    """LLM.int8() decomposition: outlier feature columns in fp32, the rest int8.
    Returns (C, number of outlier columns)."""
    import torch
    _require_device_f32(A, "A")
    _require_device_f32(B, "B")
    assert A.is_contiguous() and B.is_contiguous()
    M, K = A.shape
    N = B.shape[1]
    assert B.shape[0] == K
    if C is None:
        C = torch.empty((M, N), dtype=torch.float32, device=A.device)
    L = load()
    ws = torch.empty(L.qgemm_mm_outlier_workspace_size(M, N, K), dtype=torch.uint8, device=A.device)
    _check("qgemm_mm_outlier", L.qgemm_mm_outlier(A.data_ptr(), B.data_ptr(), C.data_ptr(), M, N, K, float(threshold),
                                                  ws.data_ptr(), ws.numel(), _stream(A.device)))
    cnt = ctypes.c_int()
    torch.cuda.current_stream(A.device).synchronize()
    _check("qgemm_outlier_count", L.qgemm_outlier_count(K, ws.data_ptr(), ctypes.byref(cnt)))
    return C, cnt.value


ENCODER_WEIGHT_KINDS = ("Wq", "Wk", "Wv", "Wo", "W1", "b1", "W2", "b2")


def encoder_weight_seed(base: int, block: int, kind: int, head: int) -> int:
    """Seed of one encoder weight tensor (include/qgemm.h, encoder.hip)."""
    return (base * 1000003 + block * 4099 + kind * 131 + head) & 0xFFFFFFFFFFFFFFFF


class Encoder:
    """transformer.cu:14-77's Encoder with its linears on the quantized path."""

    def __init__(self, d_model: int, n_heads: int, d_ff: int, n_blocks: int, max_seq: int, seed: int = 0):
        self.d_model, self.n_heads, self.d_ff, self.n_blocks, self.max_seq, self.seed = (
            d_model, n_heads, d_ff, n_blocks, max_seq, seed)
        h = ctypes.c_void_p()
        _check("qgemm_encoder_create", load().qgemm_encoder_create(d_model, n_heads, d_ff, n_blocks, max_seq, seed,
                                                                  ctypes.byref(h)))
        self._h = h

    def forward(self, X, Y=None):
        import torch
        _require_device_f32(X, "X")
        assert X.is_contiguous() and X.shape[1] == self.d_model
        Y = torch.empty_like(X) if Y is None else Y
        _check("qgemm_encoder_forward", load().qgemm_encoder_forward(self._h, X.data_ptr(), Y.data_ptr(), X.shape[0],
                                                                    _stream(X.device)))
        return Y

    def close(self):
        if getattr(self, "_h", None):
            load().qgemm_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fill_uniform(t, seed: int, lo: float = -1.0, hi: float = 1.0):
    """Seeded U[lo,hi) fill of a contiguous fp32 device tensor (bit-identical to the oracle's)."""
    assert t.is_contiguous()
    _check("qgemm_fill_uniform", load().qgemm_fill_uniform(t.data_ptr(), t.numel(), seed, lo, hi, _stream(t.device)))
    return t


