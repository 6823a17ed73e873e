"""Multi-process (world_size 2, gloo, CPU) coverage of the M-sharded path through the
product's own pieces:

* the partition is libqgemm_dist.so's qgemm_shard_rows (ctypes; loads without a GPU);
* the whole-node gather executes the product's collective plan (qgemm_allgather_plan -- exactly the
  ncclAllGather / ncclBroadcast calls qgemm_allgather_rows enqueues, with the same in-place offsets) on
  gloo collectives over CPU tensors;
* bench.py's c4_node orchestration (share_comm_id: the communicator id over broadcast_object_list;
  node_phase_times: the per-step barrier + MAX all-reduce) runs on gloo with a stub step.

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
