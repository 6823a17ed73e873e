"""Multi-GPU layer on one MI355X: the M-shard entry point (per-rank pointer offsets, bit-identical
to the one-GPU call), the RCCL communicator + all-gather C-ABI (libqgemm_dist.so), and the C++
multi-GPU driver (timing_quantize -g).  The 8-GPU run itself is the driver's scaling bench."""
import json
import os
import subprocess

import numpy as np
import pytest
import torch

from util import assert_bits_equal

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "quantized-gemm-for-transformer-inference_amd", "build")


@pytest.mark.parametrize("world", [2, 3, 8])
def test_shards_assemble_the_one_gpu_result(qg, oracle, device, world):
    M, N, K = 1000, 300, 520
    X, W = oracle.inputs(M, N, K, 77)
    Xd, Wd = torch.from_numpy(X).to(device), torch.from_numpy(W).to(device)
    C = torch.full((M, N), float("nan"), device=device)
    for r in range(world):  # each rank's call in turn, into its rows of the one full C
        qg.op_mm_quantize_shard(Xd, Wd, C, world, r)
    torch.cuda.synchronize()
    assert_bits_equal(C.cpu().numpy(), oracle.quantized_mm(X, W), f"{world} shards")


def test_rccl_comm_and_allgather_one_rank(qg, device):
    comm = qg.Comm(1, 0, qg.Comm.unique_id())
    try:
        C = torch.arange(64 * 48, dtype=torch.float32, device=device).reshape(64, 48)
        before = C.clone()
        comm.allgather_rows(C)  # world 1: every row is already local
        torch.cuda.synchronize()
        assert torch.equal(C, before)
    finally:
        comm.close()


@pytest.mark.parametrize("M,chunks", [(1000, 3), (4096, 2), (96, 5)])
def test_pipelined_shard_gather_one_rank_bit_identical(qg, oracle, device, M, chunks):
    """op_mm_quantize_shard_pipelined at world 1: W packed once, the rows in chunks on the compute stream,
    each chunk's (in-place, one-rank) ncclBroadcast on a second stream behind an event; the caller's stream
    waits for the last one.  C must equal the one-GPU call bit for bit (optional pipelining)."""
    N, K = 300, 520
    X, W = oracle.inputs(M, N, K, 78)
    Xd, Wd = torch.from_numpy(X).to(device), torch.from_numpy(W).to(device)
    C = torch.full((M, N), float("nan"), device=device)
    comm = qg.Comm(1, 0, qg.Comm.unique_id())
    try:
        assert comm.count() == 1 and comm.user_rank() == 0
        g = torch.cuda.Stream(device)
        qg.op_mm_quantize_shard_pipelined(Xd, Wd, C, 1, 0, chunks, comm=comm, gather_stream=g)
        got = C.cpu().numpy()  # on torch's stream, which waits for the gather stream
    finally:
        comm.close()
    assert_bits_equal(got, oracle.quantized_mm(X, W), f"pipelined, {chunks} chunks")


def test_pipelined_shard_rejects_small_workspace_and_missing_comm(qg, device):
    D = qg.load_dist()
    A = torch.zeros((64, 32), device=device)
    B = torch.zeros((32, 16), device=device)
    C = torch.zeros((64, 16), device=device)
    need = D.op_mm_quantize_shard_pipelined_workspace_size(64, 16, 32, 2, 2)
    ws = torch.empty(need, dtype=torch.uint8, device=device)
    s = qg._stream(device)
    assert D.op_mm_quantize_shard_pipelined(A.data_ptr(), B.data_ptr(), C.data_ptr(), 64, 16, 32, 1, 0, 2, None,
                                            ws.data_ptr(), need - 1, s, s) == qg.HIP_ERROR_INVALID_VALUE
    # world 2 without a communicator: nothing to gather with
    assert D.op_mm_quantize_shard_pipelined(A.data_ptr(), B.data_ptr(), C.data_ptr(), 64, 16, 32, 2, 0, 2, None,
                                            ws.data_ptr(), need, s, s) == qg.HIP_ERROR_INVALID_VALUE


def test_cpp_multi_gpu_driver_one_gpu():
    """timing_quantize -g: shard compute + RCCL all-gather timed, every C bit-equal to one-GPU."""
    out = subprocess.run([os.path.join(BUILD, "timing_quantize"), "-m", "1024", "-n", "768", "-k", "512", "-r", "3",
                          "-g", "1"], check=True, capture_output=True, text=True, timeout=120).stdout
    node = json.loads(out.strip().splitlines()[-1])["node"]
    assert node["gpus"] == 1 and node["bit_identical_to_one_gpu"] is True and node["mismatches"] == 0
    assert node["compute_ms"] > 0 and node["sharded_gemms_per_s"] > 0


def test_timing_quantize_prints_the_reference_lines():
    """The reference harness's output format (timing_quantize.cu:33-34,63-64,69-70,108,112-113) at its
    own shape 2048x512x512 (the stashed side of timing_quantize.cu:77-79)."""
    r = 2
    out = subprocess.run([os.path.join(BUILD, "timing_quantize"), "-m", "2048", "-n", "512", "-k", "512", "-r", str(r)],
                         check=True, capture_output=True, text=True, timeout=120).stdout.splitlines()
    i = 0
    for it in range(r):
        assert out[i] == "Time taken for matmul: " and float(out[i + 1]) > 0
        assert out[i + 2] == "Time taken for quantized matmul: " and float(out[i + 3]) > 0
        assert out[i + 4] == "Mean Quantization error: " and abs(float(out[i + 5])) < 1e-2
        t, qt = (float(x) for x in out[i + 6].split())
        assert t == float(out[i + 1]) and qt == float(out[i + 3])
        i += 7
    assert out[i] == "Final times"
    avg = [float(x) for x in out[i + 1].split()]
    assert len(avg) == 2 and all(a > 0 for a in avg)
    js = json.loads(out[i + 2])
    assert js["m"] == 2048 and js["quantized_gemms_per_s"] > 0


def test_one_rccl_with_torch_process_group(qg, device):
    """bench.py --gpus N runs torch's RCCL process group (barriers, MAX all-reduce) beside libqgemm_dist.so's
    own communicator (the C4 all-gather).  Both RCCL builds carry the soname librccl.so.1, so the dynamic
    loader must satisfy libqgemm_dist.so's NEEDED entry with the copy torch already mapped: exactly one
    librccl in the process, the one torch loaded."""
    import socket
    import torch.distributed as dist
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device(device))
    try:
        t = torch.ones(4, device=device)
        dist.all_reduce(t)
        comm = qg.Comm(1, 0, qg.Comm.unique_id())
        try:
            C = torch.arange(16 * 8, dtype=torch.float32, device=device).reshape(16, 8)
            comm.allgather_rows(C)
            torch.cuda.synchronize()
        finally:
            comm.close()
        maps = open("/proc/self/maps").read().splitlines()
        rccl = sorted({ln.split()[-1] for ln in maps if "librccl" in ln.split()[-1]})
        print("mapped RCCL:", rccl)
        assert len(rccl) == 1, f"{len(rccl)} RCCL libraries mapped: {rccl}"
        assert "torch" in rccl[0], rccl
    finally:
        dist.destroy_process_group()


def test_bench_line_names_its_world_and_binary(qg):
    """One short bench.py run on the GPU (the driver's contract at N = 1): the line reports n_gpus 1 and the
    world RCCL itself sees for the product communicator, the library's source hash equal to this tree's, and the
    whole-node C4 figure with the serial and the pipelined gather both leaving the shards' rows bit-identical."""
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline", "--no-error-stats", "--cold-steps", "0", "--node-reps", "1",
                        "--prewarm-ms", "0"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    js = json.loads(r.stdout.strip().splitlines()[-1])
    assert js["n_gpus"] == 1 and js["rccl_world"] == 1
    assert f"src={qg.source_hash()}" in js["library"]
    node = js["c4_node"]
    assert node["gathered_rows_match_one_gpu"] is True and node["pipelined"]["gathered_rows_match_one_gpu"] is True
