#!/usr/bin/env python3
"""Benchmark of the hot path: op_mm_quantize (fp32 X[M,K] @ fp32 W[K,N] -> fp32 O via absmax int8).

One "step" = one full drop-in call on inputs already resident in HBM: pack X (Cx + X_int8), pack W
(Cw + W_int8^T), int8 MFMA GEMM with the fused dequantize epilogue -- exactly the reference's
op_quantized_mm chain (op_mm.cuh:67-101), which re-quantizes both operands every call.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 the driver launches it
under torch.distributed.run, one rank per GPU.  Run WITHOUT a launcher (no WORLD_SIZE in the environment)
and N > 1, bench.py launches itself that way: ``python -m torch.distributed.run --nnodes=1
--nproc-per-node N --master-addr 127.0.0.1 ...`` as a CHILD process, before importing torch or touching
the GPU, and exits with the child's code (rank 0's JSON line reaches the same stdout).  A WORLD_SIZE that
differs from --gpus is an error (exit 2): n_gpus always equals --gpus, and `rccl_world` is the size RCCL
itself reports for the product's communicator (ncclCommCount).  Each rank owns its own M-shard (weak
scaling over batched M: every rank runs the BASELINE configs[1] problem, M=N=K=4096, on its own rows
with the replicated W); no data-path collective.  Timed region: barrier + synchronize, K steps,
synchronize + barrier, max over ranks.  Rank 0 prints ONE JSON line.

Extra objects on that line:
  roofline     -- the dominant kernel (the int8 GEMM): algorithmic 2*M*N*K int8 ops per launch over
                  its average launch time, measured with HIP events around each GEMM launch inside
                  the timed region, against the gfx950 dense int8 MFMA peak.
  cpu_baseline -- the CPU oracle (a C restatement of the reference chain, oracle/) timed on the host cores
                  (rank 0, N=1 only): the FULL M=N=K=4096 problem repeated for ~--cpu-seconds (the oracle
                  runs one whole chain in well under a second on 16 threads), plus the unquantized fp32
                  op_mm restatement once on the full problem.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

# gfx950 dense int8 MFMA peak: 256 CU x 4 SIMD x 2048 ops/clk (v_mfma_i32_32x32x32_i8: 65536 ops per
# 32 cycles) x 2.4 GHz = 5.033e15 ops/s (MI355X_MICROARCH.md: i8 = 2x the bf16 2.5 PF dense rate).
# Sustained bare int8-MFMA rate (lab/pp_lab.hip `peak`: v_mfma_i32_16x16x64_i8 back to back, operands in
# registers with no VALU in the loop, every CU, 2 s; PMC MFMA busy 0.957; profiles/r02_mfma_peak.txt):
# the chip holds ~2.03-2.05 GHz under it.  The 32x32x32 form sustains only 3515 TOPS (1.72 GHz).
PRACTICAL_INT8_TOPS = 4116.0
PEAK_INT8_TOPS = 256 * 4 * 2048 * 2.4e9 / 1e12
PEAK_HBM_GBS = 8000.0
OUTLIER_COLS = 8
OUTLIER_THRESHOLD = 6.0

CONFIGS = {
    # name: (M, N, K, description)  -- BASELINE.json configs
    "c2": (4096, 4096, 4096, "M=N=K=4096 single-GPU int8 GEMM (BASELINE configs[1])"),
    "c3_up": (2048, 16384, 4096, "FFN up 2048x4096->16384 (BASELINE configs[2])"),
    "c3_down": (2048, 4096, 16384, "FFN down 2048x16384->4096 (BASELINE configs[2])"),
    "c4_shard": (8192, 4096, 4096, "M=65536 K=N=4096 / 8 GPUs, one 8192-row shard (BASELINE configs[3])"),
    # the LLM.int8() decomposition (qgemm_mm_outlier) at the headline shape, X with
    # OUTLIER_COLS outlier feature columns (|x| 7..60 in every 50th row; threshold 6)
    # the weight-cache drop-in (op_mm_quantize_prepacked) at the headline shape, W packed
    # once before the timed region, X quantized in every step
    "c2_prepacked": (4096, 4096, 4096, "M=N=K=4096 with W prepacked once (op_mm_quantize_prepacked: pack X + "
                     "int8 GEMM/dequant per step)"),
    "c2_outlier": (4096, 4096, 4096, "M=N=K=4096 LLM.int8() outlier decomposition (qgemm_mm_outlier, threshold 6, "
                   "8 outlier feature columns)"),
    # encoder forward: (seq, d_model, n_heads, d_ff, n_blocks)
    "c5_encoder": (512, 1024, 16, 4096, 2, "encoder forward d_model=1024 seq=512 (BASELINE configs[4]), 16 heads, "
                   "d_ff 4096, 2 blocks; quantized Q/K/V, W_O, FFN linears"),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=50)
    p.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample time")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-error-stats", action="store_true", help="skip the post-run quantization-error check")
    p.add_argument("--cold-steps", type=int, default=20,
                   help="after the timed region: calls timed one by one after a 1-GiB read sweep that evicts the "
                        "inputs from the 256-MB Infinity Cache (0 = skip); reported beside the warm steady state")
    p.add_argument("--node-reps", type=int, default=10,
                   help="timed whole-node C4 steps (shard compute + RCCL all-gather, after 2 warm-up steps) for the "
                        "c4_node report (0 = skip); c2 config only")
    p.add_argument("--prewarm-ms", type=float, default=200.0,
                   help="before the W warm-up steps: keep calling the step for this long (wall clock) so the GPU's "
                        "power management leaves its idle clocks before timing; reported as `prewarm` (0 = off)")
    p.add_argument("--gemm-timing-every", type=int, default=5,
                   help="time the GEMM kernel on every n-th timed step (events cost ~4 us per timed step)")
    p.add_argument("--gemm-timing", default="ext", choices=["record", "ext", "none"],
                   help="how the GEMM kernel is timed inside the timed region: hipExtLaunchKernel start/stop "
                        "events (ext, exact kernel bounds), hipEventRecord around its launch (record, includes the "
                        "kernel-boundary gap), or not at all (none)")
    p.add_argument("--node-timeout", type=float, default=120.0,
                   help="seconds the c4_node report may take (its RCCL collectives have never run at N > 1 on this "
                        "pool): past it rank 0 prints the measurement line with c4_node marked as timed out and every "
                        "rank exits (0 = no watchdog)")
    p.add_argument("--node-chunks", type=int, default=0,
                   help="row chunks per rank of the pipelined whole-node C4 step (0 = rows / 4096, at least 1)")
    p.add_argument("--launch-dry-run", action="store_true",
                   help="N > 1 without WORLD_SIZE: print the child launcher command as JSON instead of running it")
    return p.parse_args(argv)


def world_mode(args, env):
    """How this process runs: ("launch", None) -- N > 1 and no launcher: start torch.distributed.run as a
    child; ("run", world) -- run the ranks' body here; ("error", message) -- WORLD_SIZE disagrees with
    --gpus (the driver would otherwise read a 1-rank line as an N-GPU one)."""
    if args.gpus < 1:
        return "error", f"--gpus must be >= 1, got {args.gpus}"
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return ("launch", None) if args.gpus > 1 else ("run", 1)
    try:
        world = int(ws)
    except ValueError:
        return "error", f"WORLD_SIZE={ws!r} is not an integer"
    if world != args.gpus:
        return "error", f"WORLD_SIZE={world} but --gpus {args.gpus}: launch one rank per GPU (torch.distributed.run " \
                        f"--nproc-per-node {args.gpus}) or pass --gpus {world}"
    return "run", world


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(args, argv, port):
    """The child command for N ranks on this node (the driver's own form of the launch)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


class HipEvents:
    """hipEvent_t handles from the HIP runtime torch already loaded (same soname, one runtime)."""

    def __init__(self, n):
        import ctypes
        self.ct = ctypes
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.ev = []
        for _ in range(n):
            h = ctypes.c_void_p()
            if self.hip.hipEventCreate(ctypes.byref(h)) != 0:
                raise RuntimeError("hipEventCreate failed")
            self.ev.append(h)

    def elapsed_ms(self, a, b):
        ms = self.ct.c_float()
        self.hip.hipEventSynchronize(b)
        if self.hip.hipEventElapsedTime(self.ct.byref(ms), a, b) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return ms.value

    def destroy(self):
        for h in self.ev:
            self.hip.hipEventDestroy(h)
        self.ev = []


def pmc_traffic(config):
    """HBM bytes per GEMM launch from the newest committed PMC summary of this config
    (profiles/rNN_pmc_<config>.json, written by scripts/summarize_pmc.py from separate
    FETCH_SIZE / WRITE_SIZE passes with the gfx950 x2 read correction), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"r*_pmc_{config}.json")))
    if not files:
        return None, None
    try:
        d = json.load(open(files[-1]))
        g = d["kernels"]["gemm_i8"]
        return g.get("hbm_bytes"), os.path.relpath(files[-1], REPO)
    except (OSError, KeyError, ValueError):
        return None, None


def load_pkg():
    import _pkg
    qg = _pkg.package(build=False)
    qg.load()  # raises if the HIP library is missing: no fallback
    qg.check_binary()  # raises if build/ was compiled from other sources than this tree's
    return qg


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def outlier_columns(K):
    """The c2_outlier workload's outlier feature columns (spread over K) and their rows (every 50th)."""
    return [(K // OUTLIER_COLS) * c + 7 * c + 3 for c in range(OUTLIER_COLS)], 50


def host_cpu_share():
    """The host cores this process may use, measured: the affinity mask (os.sched_getaffinity), the cgroup
    CPU quota (cpu.max: quota / period), and OMP_NUM_THREADS if the environment pins it; the thread count
    is the smallest of them (the box's CPU share), reported with where it came from."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    cands = [("affinity", aff)]
    if quota:
        cands.append(("cgroup cpu.max", max(1, int(quota))))
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        cands.append(("OMP_NUM_THREADS", int(env)))
    src, n = min(cands, key=lambda c: c[1])
    return {"threads": n, "source": src, "affinity": aff, "quota": quota}


def cpu_baseline(M, N, K, target_s, outlier=False):
    """Time the oracle's quantized chain (and the unquantized fp32 GEMM) on the host cores.

    The sample is the full workload repeated until ~target_s of CPU time (the oracle runs a whole
    M=N=K=4096 chain in well under a second on 16 cores); the fp32 path runs once on the full problem."""
    from oracle import oracle as O
    O.build()
    cpu = host_cpu_share()
    threads = cpu["threads"]
    O.set_threads(threads)
    X, W = O.uniform((M, K), 0), O.uniform((K, N), 1)
    if outlier:
        cols, every = outlier_columns(K)
        for c in cols:
            X[::every, c] = 30.0
        run = lambda: O.mm_outlier(X, W, OUTLIER_THRESHOLD)  # noqa: E731
    else:
        run = lambda: O.quantized_mm(X, W)  # noqa: E731
    O.quantized_mm(X[:64], W)  # warm the pool / pages
    reps, tq = 0, 0.0
    while tq < target_s and reps < 200:
        t0 = time.perf_counter()
        run()
        tq += time.perf_counter() - t0
        reps += 1
    # the unquantized fp32 op_mm on the FULL problem, once (sequential-k fmaf; ~0.6 s at 4096^3 on 16 threads)
    t0 = time.perf_counter()
    O.mm_fp32(X, W)
    tf = time.perf_counter() - t0
    return {
        "value": reps / tq,
        "unit": "GEMMs/s",
        "cores": threads,
        "cores_source": cpu["source"],
        "affinity_cpus": cpu["affinity"],
        "cgroup_cpu_quota": cpu["quota"],
        "cpu_model": cpu_model(),
        "host_cpus_visible": os.cpu_count(),
        "kind": "port",
        "sample": ("oracle/ C restatement of the LLM.int8() decomposition (oracle_mm_outlier)" if outlier else
                   "oracle/ C restatement of the reference chain (op_mm.cuh:67-101)") + f", full {M}x{N}x{K} "
                  f"problem x{reps} = {tq:.1f} s on {threads} OpenMP threads; unquantized fp32 op_mm "
                  f"(the reference's op_mm<float>, sequential-k fmaf) on the full problem once: {tf:.2f} s",
        "unquantized_gemms_per_s": 1.0 / tf,
    }


def prewarm_device(args, step, dev):
    """Untimed calls for --prewarm-ms of wall time before the warm-up steps: a freshly started process
    meets the GPU at idle clocks, and a 20-step timed region (~2 ms) ends before power management has
    raised them (measured: GEMM kernel 66-68 us in the first milliseconds vs 62-65 us after)."""
    import torch
    if args.prewarm_ms <= 0:
        return None
    t0, calls = time.perf_counter(), 0
    while (time.perf_counter() - t0) * 1e3 < args.prewarm_ms:
        for _ in range(10):
            step()
        calls += 10
        torch.cuda.synchronize(dev)
    return {"ms": round((time.perf_counter() - t0) * 1e3, 1), "calls": calls,
            "note": "untimed calls before the W warm-up steps (GPU clock ramp from idle)"}


def ctypes_count(L, K, ws):
    import ctypes
    c = ctypes.c_int(-1)
    if L.qgemm_outlier_count(K, ws.data_ptr(), ctypes.byref(c)) != 0:
        raise RuntimeError("qgemm_outlier_count failed")
    return c.value


def share_comm_id(rank, distributed, make_id, nbytes):
    """Rank 0 draws the communicator id (qgemm_comm_unique_id); every rank receives it over the
    torch.distributed group (broadcast_object_list).  Host-side orchestration of c4_node, tested on
    gloo (tests/test_distributed.py)."""
    uid = make_id() if rank == 0 else bytes(nbytes)
    if distributed:
        import torch.distributed as dist
        box = [uid]
        dist.broadcast_object_list(box, src=0)
        uid = box[0]
    return uid


def node_phase_times(reps, warm, distributed, run_step, dev):
    """`warm` untimed then `reps` timed whole-node steps: barrier, run_step() -> (compute_ms, gather_ms) on this
    rank, then the MAX over ranks of each phase (all_reduce); returns the timed steps' two lists.  Host-side
    orchestration of c4_node, tested on gloo with a stub step (tests/test_distributed.py)."""
    import torch
    comp, gath = [], []
    for it in range(warm + reps):
        if distributed:
            import torch.distributed as dist
            dist.barrier()
        c, g = run_step()
        t = torch.tensor([c, g], device=dev, dtype=torch.float64)
        if distributed:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if it >= warm:
            comp.append(float(t[0]))
            gath.append(float(t[1]))
    return comp, gath


def all_ranks_true(flag, distributed, dev):
    """True when `flag` holds on every rank (MIN all-reduce), e.g. every rank's gathered rows matched."""
    import torch
    t = torch.tensor([1 if flag else 0], device=dev, dtype=torch.int32)
    if distributed:
        import torch.distributed as dist
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(int(t[0]))


def c4_chunks(args, rows):
    """Chunks per rank of the pipelined C4 step: --node-chunks, else one per 4096 rows of the rank's shard."""
    return args.node_chunks if args.node_chunks > 0 else max(1, rows // 4096)


def c4_node_report(args, world, rows, distributed, dev, serial_step, reset, pipe_step, gathered_ok,
                   Mg=65536, N=4096, K=4096):
    """c4_node's host-side orchestration and its JSON: 2 warm-up + args.node_reps timed serial steps (serial_step()
    -> this rank's (compute_ms, allgather_ms)), then the same for the pipelined step (pipe_step() -> ms) after
    reset(); each phase's per-step MAX over ranks, reported as medians; gathered_ok() is AND-ed over the ranks after
    each phase.  The GPU steps are bench.c4_node's; tests/test_distributed.py runs this on gloo with stub steps."""
    import statistics
    chunks = c4_chunks(args, rows)
    comp, gath = node_phase_times(args.node_reps, 2, distributed, serial_step, dev)
    serial_ok = all_ranks_true(gathered_ok(), distributed, dev)
    reset()
    pipe, _ = node_phase_times(args.node_reps, 2, distributed, lambda: (pipe_step(), 0.0), dev)
    pipe_ok = all_ranks_true(gathered_ok(), distributed, dev)
    cm, gm, pm = statistics.median(comp), statistics.median(gath), statistics.median(pipe)
    return {
        "workload": f"BASELINE configs[3]: M={Mg} K=N={N} sharded over {world} GPU(s) ({Mg // world} rows each) + "
                    "in-place RCCL all-gather of C (1 GiB) over xGMI",
        "global_M": Mg, "N": N, "K": K, "world": world, "shard_rows": rows,
        "reps": args.node_reps, "compute_ms_median": round(cm, 4), "allgather_ms_median": round(gm, 4),
        "node_gemms_per_s_compute": round(1e3 / cm, 2),
        "node_gemms_per_s_with_allgather": round(1e3 / (cm + gm), 2),
        "node_tops_compute": round(2.0 * Mg * N * K / (cm * 1e-3) / 1e12, 1),
        "allgather_GBps_recv_per_rank": round(Mg * N * 4 * (world - 1) / world / (gm * 1e-3) / 1e9, 1) if world > 1 else None,
        "gathered_rows_match_one_gpu": serial_ok,
        "pipelined": {
            "chunks_per_rank": chunks, "ms_median": round(pm, 4),
            "node_gemms_per_s_with_allgather": round(1e3 / pm, 2),
            "gathered_rows_match_one_gpu": pipe_ok,
            "note": "op_mm_quantize_shard_pipelined: W packed once, each chunk's rows quantized + GEMM on the "
                    "compute stream, the chunk's per-owner in-place ncclBroadcasts on a second stream behind an "
                    "event (under the next chunk's compute); serial = compute_ms + allgather_ms above"},
        "note": "the compute is a full drop-in call per rank on its row shard (pack + GEMM); world 1: the whole "
                "65536-row problem on one GPU and a no-op gather",
    }


def run_with_deadline(fn, seconds, on_timeout):
    """fn() under a watchdog: if it has not returned after `seconds`, on_timeout() runs on the watchdog thread and the
    process ends with os._exit(0), so a collective that never completes (a peer that never arrives) cannot hold back the
    measurement line that is already complete.  seconds <= 0: no watchdog.  Each rank arms its own."""
    if seconds <= 0:
        return fn()
    lock = threading.Lock()
    state = {"done": False}

    def fire():
        with lock:
            if state["done"]:
                return
            try:
                on_timeout()
            finally:
                sys.stdout.flush()
                os._exit(0)

    timer = threading.Timer(seconds, fire)
    timer.daemon = True
    timer.start()
    try:
        return fn()
    finally:
        with lock:
            state["done"] = True
        timer.cancel()


def c4_node(args, qg, dev, world, rank, distributed, comm):
    """BASELINE configs[3] as a whole-node figure: the global M = 65536 x 4096 x 4096 problem with M sharded
    over the `world` ranks (op_mm_quantize_shard: per-rank pointer offsets into the full A and C), then the
    in-place RCCL all-gather of C over xGMI (qgemm_allgather_rows, libqgemm_dist.so -- our own rccl.h call
    site on `comm`, the product communicator).  Then the PIPELINED step (op_mm_quantize_shard_pipelined): W
    packed once, the rank's rows in chunks, chunk c's broadcasts on a second stream under chunk c + 1's compute.
    Timing and the JSON: c4_node_report.  Kept OUT of `value` (the gather moves 1 GiB of C, ~10x the compute)."""
    import torch
    Mg, N, K = 65536, 4096, 4096
    A = qg.fill_uniform(torch.empty((Mg, K), device=dev), seed=2 * 7)  # the same A on every rank
    B = qg.fill_uniform(torch.empty((K, N), device=dev), seed=2 * 7 + 1)
    C = torch.empty((Mg, N), device=dev)
    m0, rows = qg.shard_rows(Mg, world, rank)
    chunks = c4_chunks(args, rows)
    hip = HipEvents(3)
    gstream = torch.cuda.Stream(dev)
    ws = torch.empty(qg.load_dist().op_mm_quantize_shard_pipelined_workspace_size(Mg, N, K, world, chunks),
                     dtype=torch.uint8, device=dev)
    probe = [qg.shard_rows(Mg, world, r)[0] for r in range(world)]
    Cref = torch.empty((len(probe), N), device=dev)
    for i, r0 in enumerate(probe):  # one row of every shard, by this rank's own one-GPU call
        qg.op_mm_quantize(A[r0:r0 + 1].contiguous(), B, Cref[i:i + 1])

    def gathered_ok():
        torch.cuda.synchronize(dev)
        return bool(torch.equal(C[probe].view(torch.int32), Cref.view(torch.int32)))

    def serial_step():
        torch.cuda.synchronize(dev)
        s = qg._stream(dev)
        hip.hip.hipEventRecord(hip.ev[0], s)
        qg.op_mm_quantize_shard(A, B, C, world, rank)
        hip.hip.hipEventRecord(hip.ev[1], s)
        comm.allgather_rows(C)
        hip.hip.hipEventRecord(hip.ev[2], s)
        return hip.elapsed_ms(hip.ev[0], hip.ev[1]), hip.elapsed_ms(hip.ev[1], hip.ev[2])

    def pipe_step():
        torch.cuda.synchronize(dev)
        s = qg._stream(dev)
        hip.hip.hipEventRecord(hip.ev[0], s)
        qg.op_mm_quantize_shard_pipelined(A, B, C, world, rank, chunks, comm=comm, gather_stream=gstream,
                                          workspace=ws)
        hip.hip.hipEventRecord(hip.ev[1], s)  # the call leaves s waiting for the last broadcast
        return hip.elapsed_ms(hip.ev[0], hip.ev[1])

    try:
        return c4_node_report(args, world, rows, distributed, dev, serial_step, lambda: C.fill_(float("nan")),
                              pipe_step, gathered_ok, Mg, N, K)
    finally:
        hip.destroy()


def gemm_kernel_name(L, M, N, K, outlier):
    """The GEMM kernel this call launches, as the library plans it (qgemm_gemm_plan)."""
    if outlier:
        return ("gemm_i8_fm<kEpiOutlier> (256x256 tiles, 4 waves of 128x128, fragment-major operands straight to "
                "VGPRs, fused dequant + outlier fp32 chain on f32 MFMAs)")
    tile, name = ctypes.c_int(0), ctypes.c_char_p()
    splits = L.qgemm_gemm_plan(M, N, K, ctypes.byref(tile), ctypes.byref(name))
    return f"{name.value.decode()}, plan: {tile.value}-tiles x {splits} K-slice(s)"


def init_distributed(world, backend):
    """This process's rank, local rank, whether it is one of several, and its device.  backend "nccl" (the
    product run: RCCL, one GPU per rank) or "gloo" (the CPU tests of this branch)."""
    import torch
    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    distributed = world > 1
    if backend == "gloo":
        if distributed:
            dist.init_process_group("gloo")
        return rank, local, distributed, torch.device("cpu")
    if distributed:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local if distributed else 0)
    torch.cuda.set_device(dev)
    return rank, local, distributed, dev


def timed_region(step, steps, distributed, sync):
    """The contract's timed region: barrier + synchronize, `steps` steps, synchronize + barrier; this rank's
    wall seconds (the caller takes the max over ranks)."""
    import torch.distributed as dist
    if distributed:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    if distributed:
        dist.barrier()
    return time.perf_counter() - t0


def max_over_ranks(vals, distributed, dev):
    """Element-wise MAX of `vals` over the ranks (all_reduce); the values themselves at world 1."""
    if not distributed:
        return [float(v) for v in vals]
    import torch
    import torch.distributed as dist
    t = torch.tensor(vals, device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t]


def base_result(args, metric, unit, world, rccl_world, elapsed):
    """The fields every line carries; value = all ranks' steps over the max-over-ranks time."""
    return {
        "metric": metric,
        "value": round(world * args.steps / elapsed, 2),
        "unit": unit,
        "n_gpus": world,
        "rccl_world": rccl_world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
    }


METRIC = "int8 GEMMs/sec + achieved int8-MFMA TOPS%, M=N=K=4096, 1/2/4/8 MI355X"


def main(argv=None, backend="nccl", stub_step=None):
    """The contract's entry.  stub_step (tests only): run the ranks' body on `backend` with this CPU step in
    place of the drop-in call -- the launch / world checks, timed region, max over ranks and the base line
    are the product's own; nothing touches a GPU."""
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    mode, info = world_mode(args, os.environ)
    if mode == "error":
        print(f"bench.py: {info}", file=sys.stderr, flush=True)
        return 2
    if mode == "launch":
        # N ranks and no launcher: torch.distributed.run as a CHILD (this process has not imported torch nor
        # touched the GPU); rank 0's JSON line goes to the inherited stdout, the child's code is ours
        cmd = launcher_command(args, argv, free_port())
        if args.launch_dry_run:
            print(json.dumps({"launch": cmd, "nproc": args.gpus}), flush=True)
            return 0
        env = dict(os.environ, MASTER_ADDR="127.0.0.1")
        return subprocess.call(cmd, env=env)
    world = info
    rank, local, distributed, dev = init_distributed(world, backend)
    import torch.distributed as dist
    try:
        if stub_step is not None:
            elapsed = timed_region(stub_step, args.steps, distributed, lambda: None)
            (elapsed,) = max_over_ranks([elapsed], distributed, dev)
            rw = dist.get_world_size() if distributed else 1
            result = base_result(args, METRIC, "GEMMs/s", world, rw, elapsed)
            result["backend"] = backend
            if rank == 0:
                print(json.dumps(result), flush=True)
            return 0
        return run_gpu(args, world, rank, distributed, dev)
    finally:
        if distributed:
            dist.destroy_process_group()


def product_comm(qg, world, rank, distributed):
    """The product's RCCL communicator (libqgemm_dist.so) over every rank, its id shared through the
    torch.distributed group; returns (comm, the size RCCL reports for it)."""
    uid = share_comm_id(rank, distributed, qg.Comm.unique_id, qg.COMM_ID_BYTES)
    comm = qg.Comm(world, rank, uid)
    rw = comm.count()
    if rw != world:
        comm.close()
        raise RuntimeError(f"RCCL communicator has {rw} ranks, expected {world}")
    return comm, rw


def run_gpu(args, world, rank, distributed, dev):
    qg = load_pkg()
    L = qg.load()
    comm, rccl_world = product_comm(qg, world, rank, distributed)
    try:
        if args.config == "c5_encoder":
            return bench_encoder(args, qg, L, dev, world, rank, distributed, rccl_world)
        return bench_gemm(args, qg, L, dev, world, rank, distributed, comm, rccl_world)
    finally:
        comm.close()


def bench_gemm(args, qg, L, dev, world, rank, distributed, comm, rccl_world):
    import torch
    M, N, K, desc = CONFIGS[args.config]

    # inputs resident in HBM before timing; X differs per rank (its M-shard), W is replicated
    X = qg.fill_uniform(torch.empty((M, K), device=dev), seed=2 * (1000 + rank))
    W = qg.fill_uniform(torch.empty((K, N), device=dev), seed=2 * 1000 + 1)
    O = torch.empty((M, N), device=dev)
    outlier = args.config == "c2_outlier"
    prepacked = args.config == "c2_prepacked"
    if outlier:
        cols, every = outlier_columns(K)
        g = torch.Generator(device="cpu").manual_seed(rank)
        for c in cols:
            rows = X[::every, c]
            mag = 7.0 + 53.0 * torch.rand(rows.numel(), generator=g)
            sign = torch.where(torch.rand(rows.numel(), generator=g) < 0.5, -1.0, 1.0)
            X[::every, c] = (mag * sign).to(dev)
        ws = torch.empty(L.qgemm_mm_outlier_workspace_size(M, N, K), dtype=torch.uint8, device=dev)
    elif prepacked:
        pb = qg.pack_b(W)  # the weight cache: quantized once, outside the timed region
        ws = torch.empty(L.op_mm_quantize_prepacked_workspace_size(M, N, K), dtype=torch.uint8, device=dev)
    else:
        ws = torch.empty(L.op_mm_quantize_workspace_size(M, N, K), dtype=torch.uint8, device=dev)
    s = qg._stream(dev)
    range_ = 127.0
    hip = HipEvents(2 * args.steps)
    L.qgemm_set_event_mode(1 if args.gemm_timing == "record" else 0)

    mode = args.gemm_timing
    every = max(1, args.gemm_timing_every)
    timed = [i for i in range(args.steps) if i % every == 0]

    def step(i=None):
        # the drop-in call: op_mm_quantize on caller memory (explicit workspace, torch's stream)
        if i is not None and mode != "none" and i % every == 0:
            L.qgemm_set_gemm_events(hip.ev[2 * i], hip.ev[2 * i + 1])
        if outlier:
            rc = L.qgemm_mm_outlier(X.data_ptr(), W.data_ptr(), O.data_ptr(), M, N, K, OUTLIER_THRESHOLD,
                                    ws.data_ptr(), ws.numel(), s)
        elif prepacked:
            rc = L.op_mm_quantize_prepacked_ws(X.data_ptr(), K, pb.buf.data_ptr(), O.data_ptr(), N, M, N, K,
                                               ws.data_ptr(), ws.numel(), s)
        else:
            rc = L.op_mm_quantize_ws(X.data_ptr(), K, 1, W.data_ptr(), N, 1, O.data_ptr(), N, 1, M, N, K, range_,
                                     ws.data_ptr(), ws.numel(), s)
        if rc:
            raise RuntimeError(f"drop-in call ({args.config}) returned {rc}")

    prewarm = prewarm_device(args, step, dev)
    for _ in range(args.warmup):
        step()

    elapsed = timed_region(step, args.steps, distributed, lambda: torch.cuda.synchronize(dev))

    if mode != "none":
        gemm_ms = sum(hip.elapsed_ms(hip.ev[2 * i], hip.ev[2 * i + 1]) for i in timed) / len(timed)
    else:
        gemm_ms = float("nan")
    hip.destroy()
    elapsed, gemm_ms = max_over_ranks([elapsed, gemm_ms], distributed, dev)

    ops = 2.0 * M * N * K
    traffic, traffic_src = pmc_traffic(args.config)
    achieved = ops / (gemm_ms * 1e-3) / 1e12
    result = base_result(args, METRIC, "GEMMs/s", world, rccl_world, elapsed)
    result.update({
        "dtype": "int8",
        "data": "synthetic U(-1,1) fp32 inputs (seeded counter-based generator, generated in HBM)",
        "config": {
            "workload": (f"qgemm_mm_outlier fp32->fp32, {desc}: outlier flags + index, masked pack of X and W, "
                         "int8 MFMA GEMM/dequant with the outlier columns' fp32 chain in its epilogue, per step"
                         if outlier else
                         f"op_mm_quantize_prepacked fp32->fp32, {desc}" if prepacked else
                         f"op_mm_quantize fp32->fp32, {desc}: pack X + pack W + int8 MFMA GEMM/dequant per step"),
            "M": M, "N": N, "K": K, "global_M": M * world, "range": range_,
            "parallelism": f"M-shard x{world} (replicated W, no collective)",
        },
        "tops_full_path": round(ops * world * args.steps / elapsed / 1e12, 2),
        "tops_pct_full_path": round(100 * ops * args.steps / elapsed / 1e12 / PEAK_INT8_TOPS, 2),
        "gemm_kernel_ms": round(gemm_ms, 5),
        "core_gemms_per_s": round(world * 1e3 / gemm_ms, 2),
        "roofline": {
            "bound": "mfma",
            "achieved": round(achieved, 2),
            "peak": round(PEAK_INT8_TOPS, 1),
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_INT8_TOPS, 4),
            "traffic": traffic,
            "traffic_unit": "bytes per launch (HBM + Infinity Cache fill, FETCH_SIZE x2 + WRITE_SIZE)",
            "traffic_source": traffic_src,
            "alg_bytes": M * K + N * K + 4 * M * N + 4 * (M + N),
            "kernel": gemm_kernel_name(L, M, N, K, outlier),
            "ceiling_measured": {
                "value": PRACTICAL_INT8_TOPS, "frac": round(achieved / PRACTICAL_INT8_TOPS, 4),
                "note": "bare v_mfma_i32_16x16x64_i8 issue, operands in registers, no VALU in the loop, every CU, "
                        "2 s sustained (PMC MFMA busy 0.957 at ~2.03 GHz held clock; lab/pp_lab.hip peak mode; "
                        "profiles/r02_mfma_peak.txt)"},
            "timing": {"record": "hipEventRecord right before/after the GEMM launch (same stream)",
                       "ext": "hipExtLaunchKernel start/stop events on the GEMM launch",
                       "none": "not timed"}[args.gemm_timing] + f" on {len(timed)} of the {args.steps} timed steps",
        },
        "library": qg.version(),
        "prewarm": prewarm,
    })
    if args.config == "c2" and args.node_reps > 0:
        def node_timed_out():
            if rank == 0:
                result["c4_node"] = {"error": f"did not finish within {args.node_timeout:g} s (an RCCL collective "
                                              "that never completed); every other field of this line was measured "
                                              "before it"}
                print(json.dumps(result), flush=True)

        node = run_with_deadline(lambda: c4_node(args, qg, dev, world, rank, distributed, comm), args.node_timeout,
                                 node_timed_out)
        result["c4_node"] = node
        result["allgather_ms_median"] = node["allgather_ms_median"]
    if rank == 0 and args.cold_steps > 0:
        # Steady-state steps re-read the same X and W, which (with O) fit in the 256-MB Infinity Cache;
        # this is the same call with them evicted first (a 1-GiB read sweep between calls), each call timed
        # alone by events on its stream (includes the launch of its first kernel)
        flush = torch.ones(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB, read (not written) per sweep
        ev = HipEvents(2)
        cold = []
        for i in range(args.cold_steps):
            flush.sum()  # clean lines: no write-back of the sweep competes with the call
            torch.cuda.synchronize(dev)
            ev.hip.hipEventRecord(ev.ev[0], s)
            step()
            ev.hip.hipEventRecord(ev.ev[1], s)
            cold.append(ev.elapsed_ms(ev.ev[0], ev.ev[1]))
        ev.destroy()
        del flush
        cold.sort()
        result["cold_cache"] = {
            "ms_per_call_median": round(cold[len(cold) // 2], 5), "ms_per_call_min": round(cold[0], 5),
            "calls": len(cold),
            "note": "each call after a 1-GiB read sweep evicted X, W and O from the Infinity Cache; value above is the "
                    "warm steady state (same inputs every step, as GEMM benchmarks run)"}
    if rank == 0 and not args.no_error_stats:
        # after the timed region: the quantization error of this run's output against the reference's
        # unquantized op_mm (qgemm_mm_fp32, bit-exact sequential-k fmaf), computed on the device
        C = qg.mm_fp32(X, W)
        st = qg.error_stats(C, O, reference_order=M * N <= (1 << 24))  # sequential chain: ~tens of ms
        result["quant_error"] = {k: (None if v != v else float(f"{v:.6g}")) for k, v in st.items()}
        result["quant_error"]["note"] = ("signed_mean_ref = the reference's printed metric (sequential fp32, "
                                         "timing_quantize.cu:67-70); the others fp64 on the device")
        del C
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(M, N, K, args.cpu_seconds, outlier=outlier)
        if prepacked:
            result["cpu_baseline"]["note"] = "the reference chain re-quantizes W every call (it has no weight cache)"
    if outlier and rank == 0:
        cnt = ctypes_count(L, K, ws)
        result["config"]["outlier_columns"] = cnt
    if rank == 0:
        print(json.dumps(result), flush=True)
    return 0


def bench_encoder(args, qg, L, dev, world, rank, distributed, rccl_world):
    """BASELINE config 5: the encoder counterpart's forward (seeded weights packed once, the
    activations' quantize inside every forward); one forward per step, each rank its own sequence."""
    import torch
    seq, d, H, dff, blocks, desc = CONFIGS["c5_encoder"]
    enc = qg.Encoder(d, H, dff, blocks, max_seq=seq, seed=1000)
    X = qg.fill_uniform(torch.empty((seq, d), device=dev), seed=2 * (1000 + rank))
    Y = torch.empty_like(X)
    hip = HipEvents(2 * args.steps)
    L.qgemm_set_event_mode(0)
    every = max(1, args.gemm_timing_every)
    timed = [i for i in range(args.steps) if i % every == 0]
    prewarm = prewarm_device(args, lambda: enc.forward(X, Y), dev)
    for _ in range(args.warmup):
        enc.forward(X, Y)

    def step(i):
        if i % every == 0:  # times the forward's first GEMM: the fused Q/K/V projection
            L.qgemm_set_gemm_events(hip.ev[2 * i], hip.ev[2 * i + 1])
        enc.forward(X, Y)

    elapsed = timed_region(step, args.steps, distributed, lambda: torch.cuda.synchronize(dev))
    gemm_ms = sum(hip.elapsed_ms(hip.ev[2 * i], hip.ev[2 * i + 1]) for i in timed) / len(timed)
    hip.destroy()
    elapsed, gemm_ms = max_over_ranks([elapsed, gemm_ms], distributed, dev)
    qkv_ops = 2.0 * seq * 3 * d * d
    lin_ops = blocks * 2.0 * seq * (3 * d * d + d * d + 2 * d * dff)
    attn_flops = blocks * 2.0 * 2 * H * seq * seq * (d // H)
    achieved = qkv_ops / (gemm_ms * 1e-3) / 1e12
    result = base_result(args, "encoder forwards/s (BASELINE configs[4])", "forwards/s", world, rccl_world, elapsed)
    result.update({
        "dtype": "int8",
        "data": "synthetic U(-1,1) fp32 input, seeded weights (qgemm_fill_uniform streams)",
        "config": {"workload": desc, "seq": seq, "d_model": d, "n_heads": H, "d_ff": dff, "n_blocks": blocks,
                   "parallelism": f"independent sequences x{world}"},
        "tokens_per_s": round(world * args.steps * seq / elapsed, 1),
        "int8_tops_linears": round(lin_ops * args.steps / elapsed / 1e12, 2),
        "fp32_tflops_attention": round(attn_flops * args.steps / elapsed / 1e12, 2),
        "roofline": {
            "bound": "mfma",
            "achieved": round(achieved, 2),
            "peak": round(PEAK_INT8_TOPS, 1),
            "unit": "TFLOP/s",
            "frac": round(achieved / PEAK_INT8_TOPS, 4),
            "traffic": None,
            "kernel": "gemm_i8_small<64, 0, 3> (fused Q/K/V projection, 512 x 3072 x 1024)",
            "timing": f"hipExtLaunchKernel start/stop events on {len(timed)} of the {args.steps} timed forwards",
        },
        "library": qg.version(),
        "prewarm": prewarm,
    })
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        from oracle import oracle as O
        O.build()
        cpu = host_cpu_share()
        O.set_threads(cpu["threads"])
        Xh = O.uniform((seq, d), 2 * 1000)
        O.encoder_forward(Xh, d, H, dff, 1, 1000)  # warm
        reps, tc = 0, 0.0
        while tc < args.cpu_seconds and reps < 100:
            c0 = time.perf_counter()
            O.encoder_forward(Xh, d, H, dff, blocks, 1000)
            tc += time.perf_counter() - c0
            reps += 1
        result["cpu_baseline"] = {
            "value": reps / tc, "unit": "forwards/s",
            "cores": cpu["threads"], "cores_source": cpu["source"], "affinity_cpus": cpu["affinity"], "kind": "port",
            "sample": f"oracle/ C restatement of the encoder (transformer.cu:14-77 with quantized linears), "
                      f"full config-5 forward x{reps} = {tc:.1f} s",
        }
    if rank == 0:
        print(json.dumps(result), flush=True)
    enc.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
