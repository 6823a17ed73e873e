"""Multi-process (world_size 2, gloo, CPU) coverage of the M-sharded path.

Each rank quantizes-and-multiplies its own row block [row_range(M, world, rank)) with the replicated
W -- here through the CPU oracle, since this runs without a GPU -- and the optional whole-node
gather (shard.gather_rows, all_gather_into_tensor) must reassemble exactly the single-process
result: Cx is per row and Cw depends only on W, so sharding over M is bit-exact.
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


def _worker(rank, world, port, M, N, K, out_dir):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, repo)
    sys.path.insert(0, os.path.join(repo, "tests"))
    import torch
    import torch.distributed as dist

    import _pkg
    from oracle import oracle as O

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    qg = _pkg.package()
    X, W = O.inputs(M, N, K, seed=77)
    lo, hi = qg.shard.row_range(M, world, rank)
    local = torch.from_numpy(O.quantized_mm(X[lo:hi], W))
    full = qg.shard.gather_rows(local, M)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), full.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("M", [64, 67])  # even and ragged shards
def test_msharded_gather_matches_single_process(oracle, tmp_path, M):
    N, K, world = 48, 96, 2
    mp.spawn(_worker, args=(world, _free_port(), M, N, K, str(tmp_path)), nprocs=world, join=True)
    X, W = oracle.inputs(M, N, K, seed=77)
    want = oracle.quantized_mm(X, W)
    for r in range(world):
        got = np.load(tmp_path / f"rank{r}.npy")
        assert got.shape == want.shape
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"rank {r}"
