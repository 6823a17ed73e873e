"""Multi-process (world_size 2, gloo, CPU) coverage of the M-sharded path through the
product's own pieces:

* the partition is libqgemm_dist.so's qgemm_shard_rows (ctypes; loads without a GPU);
* the whole-node gather executes the product's collective plan (qgemm_allgather_plan -- exactly the
  ncclAllGather / ncclBroadcast calls qgemm_allgather_rows enqueues, with the same in-place offsets) on
  gloo collectives over CPU tensors;
* bench.py's c4_node orchestration (share_comm_id: the communicator id over broadcast_object_list;
  node_phase_times: the per-step barrier + MAX all-reduce; c4_node_report: the whole C4 report a SCALE line
  carries, serial and pipelined phases) runs on gloo with stub compute, gather and pipeline steps.

Each rank's rows are computed by the CPU oracle here (no GPU in this container); the GPU side of the same
partition is tests/test_gpu_dist.py.  Cx is per row and Cw depends only on W, so the sharded result must
equal the single-process one bit for bit.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run_plan(qg, C, m, n, world, rank):
    """qgemm_allgather_rows' collectives on gloo, in place on the flat CPU tensor C."""
    import torch
    import torch.distributed as dist
    flat = C.view(-1)
    for first, count, root in qg.allgather_plan(m, n, world):
        if root < 0:  # ONE in-place all-gather: rank r sends flat[first + r*count : first + (r+1)*count]
            parts = [torch.empty(count, dtype=C.dtype) for _ in range(world)]
            dist.all_gather(parts, flat[first + rank * count: first + (rank + 1) * count].clone())
            flat[first: first + world * count] = torch.cat(parts)
        else:
            seg = flat[first: first + count].clone()
            dist.broadcast(seg, src=root)
            flat[first: first + count] = seg


def _worker(rank, world, port, M, N, K, out_dir):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "tests"))
    import torch
    import torch.distributed as dist

    import _pkg
    import bench
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    qg = _pkg.package()
    X, W = O.inputs(M, N, K, seed=77)
    m0, rows = qg.shard_rows(M, world, rank)
    C = torch.full((M, N), float("nan"))
    C[m0:m0 + rows] = torch.from_numpy(O.quantized_mm(X[m0:m0 + rows], W))
    _run_plan(qg, C, M, N, world, rank)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), C.numpy())

    # bench.py c4_node orchestration: rank 0's id reaches every rank; per step the MAX over ranks
    uid = bench.share_comm_id(rank, True, lambda: bytes(range(7, 7 + qg.COMM_ID_BYTES)), qg.COMM_ID_BYTES)
    steps = iter([(1.0 + rank, 5.0 - rank), (2.0 * (rank + 1), 1.0), (0.5, 0.25 + rank)] * 2)
    comp, gath = bench.node_phase_times(4, 2, True, lambda: next(steps), torch.device("cpu"))
    np.save(os.path.join(out_dir, f"uid{rank}.npy"), np.frombuffer(uid, dtype=np.uint8))
    np.save(os.path.join(out_dir, f"times{rank}.npy"), np.array(comp + gath))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("M", [64, 67])  # even shards (one in-place all-gather) and ragged (broadcasts)
def test_msharded_gather_matches_single_process(oracle, tmp_path, M):
    N, K, world = 48, 96, 2
    mp.spawn(_worker, args=(world, _free_port(), M, N, K, str(tmp_path)), nprocs=world, join=True)
    X, W = oracle.inputs(M, N, K, seed=77)
    want = oracle.quantized_mm(X, W)
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        assert got.shape == want.shape
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"rank {r}"
        uid, times = np.load(tmp_path / f"uid{r}.npy"), np.load(tmp_path / f"times{r}.npy")
        assert uid.tobytes() == bytes(range(7, 7 + 128)), f"rank {r} comm id"
        # steps 2..5 after 2 warm-ups; rank-wise MAX: (1+r, 5-r) -> (2, 5); (2(r+1), 1) -> (4, 1); (0.5, 0.25+r) -> (0.5, 1.25)
        assert list(times) == [0.5, 2.0, 4.0, 0.5, 1.25, 5.0, 1.0, 1.25], f"rank {r} phase maxima"


def _report_worker(rank, world, port, out_dir):
    import json
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "tests"))
    import torch
    import torch.distributed as dist

    import _pkg
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    qg = _pkg.package()
    args = bench.parse(["--gpus", str(world), "--node-reps", "5"])
    m0, rows = qg.shard_rows(65536, world, rank)  # the product's partition (libqgemm_dist.so)
    # stub steps: this rank's (compute, gather) ms per step and pipelined ms; rank 1 is slower in compute, rank 0
    # in the gather, so the per-step MAX over ranks picks from both
    serial = iter([(0.15 + 0.01 * rank, 0.9 - 0.05 * rank + 0.001 * i) for i in range(7)])
    pipe = iter([0.95 + 0.02 * rank + 0.001 * i for i in range(7)])
    ok = iter([True, rank == 0])  # serial rows match everywhere; the pipelined phase fails on rank 1
    resets = []
    rep = bench.c4_node_report(args, world, rows, True, torch.device("cpu"), lambda: next(serial),
                               lambda: resets.append(1), lambda: next(pipe), lambda: next(ok))
    with open(os.path.join(out_dir, f"report{rank}.json"), "w") as f:
        json.dump({"report": rep, "resets": len(resets), "rows": rows}, f)
    dist.barrier()
    dist.destroy_process_group()


def test_c4_node_report_world2_on_gloo(tmp_path):
    """bench.c4_node's orchestration at world 2 with stub compute / gather / pipeline steps --
    the fields a SCALE line's c4_node carries: per-step MAX over ranks then medians, the all-gather GB/s received per
    rank, chunks_per_rank == rows // 4096, and the gathered-rows checks AND-ed over the ranks."""
    import json
    world = 2
    mp.spawn(_report_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    reps = [json.load(open(tmp_path / f"report{r}.json")) for r in range(world)]
    for r, got in enumerate(reps):
        rep = got["report"]
        assert got["rows"] == 32768 and got["resets"] == 1
        assert rep["world"] == 2 and rep["shard_rows"] == 32768 and rep["global_M"] == 65536 and rep["reps"] == 5
        # timed steps i = 2..6: compute max = 0.16, gather max = 0.9 + 0.001 i (rank 0) -> median i = 4: 0.904
        assert rep["compute_ms_median"] == 0.16 and rep["allgather_ms_median"] == 0.904, rep
        assert rep["allgather_GBps_recv_per_rank"] == round(65536 * 4096 * 4 * 0.5 / 0.904e-3 / 1e9, 1)
        assert rep["node_gemms_per_s_compute"] == round(1e3 / 0.16, 2)
        assert rep["node_gemms_per_s_with_allgather"] == round(1e3 / (0.16 + 0.904), 2)
        pipe = rep["pipelined"]
        assert pipe["chunks_per_rank"] == 32768 // 4096 == 8
        assert pipe["ms_median"] == round(0.97 + 0.004, 4)  # rank 1's 0.97 + 0.001 i, median i = 4
        assert rep["gathered_rows_match_one_gpu"] is True
        assert pipe["gathered_rows_match_one_gpu"] is False, "rank 1's failed check must reach every rank"


def test_c4_node_report_world8_shapes():
    """The world-8 branch of c4_node's report, one process: 8192-row shards, 2 chunks per rank (the N = 8 SCALE
    line stays unmeasured on hardware: no 8-GPU node in any round)."""
    import sys
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    import _pkg
    qg = _pkg.package()
    args = bench.parse(["--node-reps", "3"])
    for rank in (0, 7):
        m0, rows = qg.shard_rows(65536, 8, rank)
        assert (m0, rows) == (8192 * rank, 8192)
        it = iter([(0.1, 0.9)] * 5)
        rep = bench.c4_node_report(args, 8, rows, False, torch.device("cpu"), lambda: next(it), lambda: None,
                                   lambda: 1.0, lambda: True)
        assert rep["pipelined"]["chunks_per_rank"] == 2 and rep["shard_rows"] == 8192
        assert rep["allgather_GBps_recv_per_rank"] == round(65536 * 4096 * 4 * 7 / 8 / 0.9e-3 / 1e9, 1)
