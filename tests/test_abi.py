"""The C-ABI library: builds for gfx950, loads, exports exactly what include/qgemm.h declares,
and rejects bad arguments (the reference's asserts, op_mm.cuh:71-72) without touching a GPU."""
import ctypes
import os
import re
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "qgemm.h")


def header_functions():
    text = open(HEADER).read()
    return sorted(re.findall(r"^QGEMM_API\s+[\w\s\*]+?\b((?:op_|qgemm_)\w+)\s*\(", text, flags=re.M))


def exported(lib_path):
    out = subprocess.run(["nm", "-D", "--defined-only", lib_path], check=True, capture_output=True, text=True).stdout
    return sorted(line.split()[-1] for line in out.splitlines() if " T " in line)


def test_header_declares_the_north_star_entry_point():
    fns = header_functions()
    assert "op_mm_quantize" in fns
    # op_mm_quantize(A, B, C, M, N, K): three pointers and three ints, no parameter named N
    text = open(HEADER).read()
    assert re.search(r"int op_mm_quantize\(const float \*A, const float \*B, float \*C, int m, int n, int k\);", text)
    assert not re.search(r"\bint N\b", text), "the reference #defines N (op_elemwise.cuh:10)"


def test_library_exports_every_declared_symbol(qg):
    assert header_functions() == sorted(qg.EXPORTED_SYMBOLS)
    assert exported(qg.LIB_PATH) == header_functions(), "exports must be exactly the C-ABI"


def test_library_carries_gfx950_code_object(qg):
    blob = open(qg.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_version_and_sizes_without_gpu(qg):
    L = qg.load()
    assert "gfx950" in qg.version()
    # packed operand: [scale rows_pad*4][reserved parts*rows_pad*4][rows_pad*k_pad], parts = ceil((k-1)/256)
    def size(rows, k):
        rp = -(-rows // 256) * 256
        kp = -(-k // 128) * 128
        parts = -(-(k - 1) // 256) if k > 1 else 1
        head = -(-(rp * 4 * (1 + parts)) // 256) * 256
        return head + rp * kp
    for rows, k in [(4096, 4096), (1, 1), (257, 129), (2048, 16384), (3, 2)]:
        assert L.qgemm_packed_size(rows, k) == size(rows, k), (rows, k)
    ws = L.op_mm_quantize_workspace_size(4096, 4096, 4096)
    assert ws == 2 * size(4096, 4096)  # 256 tiles: no split-K scratch
    # FFN down (2048 x 16384 -> 4096): 128 tiles, split-K 2, ticket-first -> tickets + ONE int32 256x256 slab per tile
    split = 4096 + 128 * 256 * 256 * 4
    assert L.op_mm_quantize_workspace_size(2048, 4096, 16384) == split + size(2048, 16384) + size(4096, 16384)
    assert L.op_mm_quantize_workspace_size(4, 4, 0) == 0


@pytest.mark.parametrize("args", [
    (None, None, None, 4, 4, 4),
    (8, 8, 8, 4, 4, 0),      # K = 0: no reduction vector
    (8, 8, 8, -1, 4, 4),
])
def test_invalid_arguments_return_hip_error_invalid_value(qg, args):
    L = qg.load()
    a, b, c, m, n, k = args
    assert L.op_mm_quantize(a, b, c, m, n, k) == qg.HIP_ERROR_INVALID_VALUE


def test_invalid_pack_and_workspace_calls(qg):
    L = qg.load()
    assert L.qgemm_pack_a(None, 4, 1, 4, 4, 127.0, 8, None) == 1
    assert L.qgemm_pack_b(8, 4, 1, 0, 4, 127.0, 8, None) == 1
    # too small an explicit workspace is refused before any launch
    assert L.op_mm_quantize_ws(8, 4, 1, 8, 4, 1, 8, 4, 1, 4, 4, 4, 127.0, 8, 16, None) == 1
    assert L.qgemm_mm_packed(None, 8, 8, 4, 1, 4, 4, 4, 127.0, None) == 1


def test_harness_binaries_built(qg):
    for exe in ("test_quantize", "timing_quantize", "transformer"):
        p = os.path.join(qg.PKG_DIR, "build", exe)
        assert os.access(p, os.X_OK), p


def test_missing_library_fails_loudly(qg, monkeypatch, tmp_path):
    """No CPU fallback: without the HIP library every entry point raises."""
    monkeypatch.setattr(qg, "LIB_PATH", str(tmp_path / "libqgemm.so"))
    monkeypatch.setattr(qg, "_lib", None)
    with pytest.raises(RuntimeError, match="not built"):
        qg.load()


def test_reference_side_ctypes_binding_matches(qg):
    """The ctypes stub shown in INTEGRATION.md binds the same signature."""
    L = ctypes.CDLL(qg.LIB_PATH)
    f = L.op_mm_quantize
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int] * 3
    f.restype = ctypes.c_int
    assert f(None, None, None, 1, 1, 1) == 1


DIST_HEADER = os.path.join(REPO, "include", "qgemm_dist.h")


def test_dist_library_exports_every_declared_symbol(qg):
    text = open(DIST_HEADER).read()
    fns = sorted(re.findall(r"^QGEMM_API\s+[\w\s\*]+?\b((?:op_|qgemm_)\w+)\s*\(", text, flags=re.M))
    assert fns == sorted(qg.DIST_EXPORTED_SYMBOLS)
    assert exported(qg.DIST_LIB_PATH) == fns, "libqgemm_dist.so exports must be exactly qgemm_dist.h"
    # the RCCL call sites are real (rccl.h), not a shim
    out = subprocess.run(["nm", "-D", "--undefined-only", qg.DIST_LIB_PATH], check=True, capture_output=True,
                         text=True).stdout
    for sym in ("ncclAllGather", "ncclBroadcast", "ncclCommInitRank", "ncclCommInitAll", "ncclGetUniqueId"):
        assert sym in out, sym


def test_shard_rows_partition_without_gpu(qg):
    """qgemm_shard_rows: contiguous, balanced (sizes differ by <= 1), covering."""
    for m in (0, 1, 7, 255, 4096, 65536, 65537):
        for world in (1, 2, 3, 4, 8):
            nxt, sizes = 0, []
            for r in range(world):
                m0, rows = qg.shard_rows(m, world, r)
                assert m0 == nxt and rows >= 0
                nxt = m0 + rows
                sizes.append(rows)
            assert nxt == m and max(sizes) - min(sizes) <= 1
    D = qg.load_dist()
    a, b = ctypes.c_int(), ctypes.c_int()
    assert D.qgemm_shard_rows(8, 2, 2, ctypes.byref(a), ctypes.byref(b)) == 1  # rank >= world
    assert D.qgemm_shard_rows(8, 0, 0, ctypes.byref(a), ctypes.byref(b)) == 1
    # argument checks before any device work
    assert D.op_mm_quantize_shard(None, None, None, 8, 8, 8, 2, 0, None) == 1
    assert D.qgemm_allgather_rows(None, 8, 8, 2, 0, None, None) == 1


def _simulate_plan(plan, m, n, world, qg):
    """Execute qgemm_allgather_rows' collectives on `world` simulated ranks (numpy buffers), each starting
    with only its own shard's rows set: returns the ranks' buffers afterwards."""
    import numpy as np
    full = np.arange(m * n, dtype=np.float64) + 1
    bufs = []
    for r in range(world):
        b = np.zeros(m * n)
        m0, rows = qg.shard_rows(m, world, r)
        b[m0 * n:(m0 + rows) * n] = full[m0 * n:(m0 + rows) * n]
        bufs.append(b)
    for first, count, root in plan:
        if root < 0:  # in-place all-gather: rank r's send buffer is recv + r * count
            sent = [bufs[r][first + r * count:first + (r + 1) * count].copy() for r in range(world)]
            for b in bufs:
                for r in range(world):
                    b[first + r * count:first + (r + 1) * count] = sent[r]
        else:
            src = bufs[root][first:first + count].copy()
            for b in bufs:
                b[first:first + count] = src
    return full, bufs


@pytest.mark.parametrize("world", [1, 2, 3, 4, 5, 7, 8])
def test_allgather_plan_reassembles_every_rank(qg, world):
    """The collectives qgemm_allgather_rows enqueues (qgemm_allgather_plan), run on simulated ranks: every
    rank ends with all m rows, for m % world == 0 (one in-place all-gather) and != 0 (one broadcast per
    owner; empty owners skipped), including m < world."""
    import numpy as np
    for m in (0, 1, 3, 8, 24, 65, 96, 1001):
        n = 5
        plan = qg.allgather_plan(m, n, world)
        if world == 1 or m == 0:
            assert plan == []
            continue
        if m % world == 0:
            assert plan == [(0, m // world * n, -1)]
        else:
            assert all(root >= 0 for _, _, root in plan) and len(plan) == min(m, world)
        full, bufs = _simulate_plan(plan, m, n, world, qg)
        for r, b in enumerate(bufs):
            assert np.array_equal(b, full), f"m={m} world={world} rank {r}"
    D = qg.load_dist()
    assert D.qgemm_allgather_plan(-1, 4, 2, None, None, None, 0) < 0
    assert D.qgemm_allgather_plan(8, 4, 2, None, None, None, 0) < 0  # one op needed, no room


def _simulate_node_group(ops, m, n, ndev, qg):
    """Run one RCCL group of planned collectives the way RCCL matches them: the i-th collective on every
    communicator forms one operation, so every rank must list the same (kind, root, count, recv_off) sequence;
    then execute them on per-rank numpy buffers that start with only the rank's own shard."""
    import numpy as np
    per = [[o for o in ops if o[0] == r] for r in range(ndev)]
    assert all(len(p) == len(per[0]) for p in per), "every communicator enqueues the same number of ops"
    full = np.arange(m * n, dtype=np.float64) + 1
    bufs = []
    for r in range(ndev):
        b = np.zeros(m * n)
        m0, rows = qg.shard_rows(m, ndev, r)
        b[m0 * n:(m0 + rows) * n] = full[m0 * n:(m0 + rows) * n]
        bufs.append(b)
    for i in range(len(per[0])):
        col = [per[r][i] for r in range(ndev)]
        keys = {(root, count, recv) for (_, root, _, recv, count) in col}
        assert len(keys) == 1, f"op {i}: ranks disagree on the collective {col}"
        root, count, recv = keys.pop()
        if root < 0:  # all-gather: rank r contributes [send_off, send_off + count), which must be its own rows
            sent = []
            for (r, _, send, _, _) in col:
                m0, rows = qg.shard_rows(m, ndev, r)
                assert send == recv + r * count and send == m0 * n and count == rows * n, "in-place send = own rows"
                sent.append(bufs[r][send:send + count].copy())
            for b in bufs:
                for r in range(ndev):
                    b[recv + r * count:recv + (r + 1) * count] = sent[r]
        else:  # broadcast from root, in place: the root's own rows
            m0, rows = qg.shard_rows(m, ndev, root)
            assert recv == m0 * n and count == rows * n, "a broadcast moves exactly its root's rows"
            assert all(send == recv for (_, _, send, _, _) in col), "in place"
            src = bufs[root][recv:recv + count].copy()
            for b in bufs:
                b[recv:recv + count] = src
    return full, bufs


@pytest.mark.parametrize("ndev", [2, 3, 4, 5, 7, 8])
def test_node_allgather_plan_assembles_every_device(qg, ndev):
    """The one-process node path (qgemm_node_mm_quantize mode 1 / 2, the harness's -g) issues exactly
    qgemm_node_allgather_plan's list inside ONE flat RCCL group (no GPU needed to check its
    argument and group logic).  For equal shards (m % ndev == 0) and unequal ones, including m < ndev: every
    communicator lists the same collectives in the same order, every send is the rank's own rows, and running
    them assembles the whole C on every device."""
    import numpy as np
    for m in (1, 3, 8, 24, 65, 96, 1001, 65536 + 3):
        n = 3
        ops = qg.node_allgather_plan(m, n, ndev)
        plan = qg.allgather_plan(m, n, ndev)
        assert len(ops) == ndev * len(plan)
        assert [o[0] for o in ops] == sorted(o[0] for o in ops), "rank by rank, in plan order"
        if m % ndev == 0:
            assert len(plan) == 1 and plan[0][2] == -1
        else:
            assert all(root >= 0 for _, _, root in plan) and len(plan) == min(m, ndev)
        full, bufs = _simulate_node_group(ops, m, n, ndev, qg)
        for r, b in enumerate(bufs):
            assert np.array_equal(b, full), f"m={m} ndev={ndev} device {r}"
    assert qg.node_allgather_plan(0, 4, ndev) == [] and qg.node_allgather_plan(8, 0, ndev) == []
    D = qg.load_dist()
    assert D.qgemm_node_allgather_plan(-1, 4, ndev, None, 0) < 0
    assert D.qgemm_node_allgather_plan(5, 4, ndev, (qg.CollOp * 1)(), 1) < 0  # ndev ops needed, room for one


def test_allgather_plan_has_no_world_cap(qg):
    """qgemm_allgather_rows sizes its plan from the world size (a fixed 64-op cap refused
    communicators above 64 ranks even for the one-all-gather plan)."""
    assert qg.allgather_plan(128 * 4, 2, 128) == [(0, 8, -1)]
    assert len(qg.allgather_plan(129, 2, 128)) == 128
    D = qg.load_dist()
    assert D.qgemm_allgather_rows(None, 512, 2, 128, 0, None, None) == 1  # still the argument check, not a cap


def _copy_tree(qg, dst):
    """The package's hashed sources + its built library, laid out as in the repo (pkg/ beside include/)."""
    import shutil
    pkg = dst / "pkg"
    shutil.copytree(os.path.join(qg.PKG_DIR, "csrc"), pkg / "csrc")
    shutil.copytree(os.path.join(qg.PKG_DIR, "src"), pkg / "src")
    shutil.copy(os.path.join(qg.PKG_DIR, "Makefile"), pkg / "Makefile")
    shutil.copy(os.path.join(qg.PKG_DIR, "__init__.py"), pkg / "__init__.py")
    shutil.copytree(os.path.join(REPO, "include"), dst / "include")
    (pkg / "build").mkdir()
    shutil.copy(qg.LIB_PATH, pkg / "build" / "libqgemm.so")
    return pkg


def _load_copy(pkg, name):
    import importlib.util
    spec = importlib.util.spec_from_file_location(name, str(pkg / "__init__.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_binary_carries_this_trees_source_hash(qg):
    """qgemm_version() names the sources it was built from (Makefile SRC_HASH) and they are this tree's."""
    h = qg.source_hash()
    assert len(h) == 16 and f"src={h}" in qg.version()
    assert qg.check_binary() == h


def test_stale_binary_is_rejected(qg, tmp_path):
    """A build/ compiled from other sources (here: one source edited after the build) is refused by
    check_binary(), which smoke() and bench.py call before any timing."""
    pkg = _copy_tree(qg, tmp_path)
    fresh = _load_copy(pkg, "qgemm_copy_fresh")
    assert fresh.source_hash() == qg.source_hash() and fresh.check_binary() == qg.source_hash()
    with open(pkg / "csrc" / "api.hip", "a") as f:
        f.write("\n// edited after the build\n")
    stale = _load_copy(pkg, "qgemm_copy_stale")
    assert stale.source_hash() != qg.source_hash()
    assert stale.file_hash() == qg.source_hash(), "the binary's own tag names the sources it was built from"
    with pytest.raises(RuntimeError, match="built from sources"):
        stale.check_binary()


@pytest.mark.parametrize("world", [1, 2, 3, 5, 8])
@pytest.mark.parametrize("chunks", [1, 2, 3, 4])
def test_chunked_allgather_plan_assembles_every_rank(qg, world, chunks):
    """op_mm_quantize_shard_pipelined's broadcasts (qgemm_allgather_chunk_plan), executed on per-rank
    buffers: chunk-major, each op is its root's own rows of that chunk, every row is moved exactly once,
    and every rank ends with the whole C -- for m % world != 0, m < world, m % chunks != 0."""
    import numpy as np
    n = 3
    for m in (0, 1, world - 1, 7, 65, 1001, 65536 + 3):
        plan = qg.allgather_chunk_plan(m, n, world, chunks)
        owner = np.full(m, -1)
        for r in range(world):
            m0, rows = qg.shard_rows(m, world, r)
            owner[m0:m0 + rows] = r
        seen = np.zeros(m, dtype=int)
        last_chunk = -1
        bufs = [np.full(m * n, np.nan) for _ in range(world)]
        for r in range(world):  # each rank holds only its own rows before the gather
            m0, rows = qg.shard_rows(m, world, r)
            bufs[r][m0 * n:(m0 + rows) * n] = np.arange(m0 * n, (m0 + rows) * n)
        for first, count, root in plan:
            assert first % n == 0 and count % n == 0 and count > 0
            r0, rr = first // n, count // n
            assert (owner[r0:r0 + rr] == root).all(), "a broadcast moves its root's own rows"
            m0, rows = qg.shard_rows(m, world, root)
            c = [ci for ci in range(chunks) if qg.shard_rows(rows, chunks, ci)[0] + m0 == r0][0]
            assert c >= last_chunk, "chunk-major order"
            last_chunk = c
            seen[r0:r0 + rr] += 1
            for b in bufs:  # in place: receive = send region on every rank
                b[first:first + count] = bufs[root][first:first + count]
        assert (seen == 1).all(), (m, world, chunks)
        for b in bufs:
            assert np.array_equal(b, np.arange(m * n, dtype=float))
        assert len(plan) <= world * chunks


@pytest.mark.parametrize("m,n,k,tile,splits", [
    (4096, 4096, 4096, 256, 1),     # C2: 256 tiles, one per CU
    (2048, 16384, 4096, 256, 1),    # C3 FFN up: 512 tiles
    (2048, 4096, 16384, 256, 2),    # C3 FFN down: 128 tiles, ticket-first 2-way split-K
    (8192, 4096, 4096, 256, 1),     # C4 shard
    (512, 3072, 1024, 64, 1),       # C5 Q/K/V (384 64-tiles)
    (512, 4096, 1024, 64, 1),       # C5 FFN up (512 64-tiles)
    (512, 1024, 1024, 32, 1),       # C5 W_O (512 32-tiles)
    (512, 1024, 4096, 32, 1),       # C5 FFN down (512 32-tiles)
    (128, 128, 128, 64, 1),         # C1: 4 64-tiles (too few 32-tiles to fill the chip)
])
def test_gemm_plan_for_every_baseline_shape(qg, m, n, k, tile, splits):
    """qgemm_gemm_plan (host-only: no GPU) picks, for each BASELINE config's GEMM shapes, the kernel the profiles in
    profiles/r06_kernel_stats_*.csv show running (gemm_i8.hip gemm_plan)."""
    L = qg.load()
    t, name = ctypes.c_int(0), ctypes.c_char_p()
    assert L.qgemm_gemm_plan(m, n, k, ctypes.byref(t), ctypes.byref(name)) == splits
    assert t.value == tile
    expect = "gemm_i8_fm" if tile == 256 else f"gemm_i8_small<{tile}>"
    assert name.value.decode().startswith(expect)
