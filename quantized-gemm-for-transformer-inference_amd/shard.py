"""M-sharding of the quantized GEMM across ranks.

The path is embarrassingly parallel over output rows: Cx is per row and Cw depends only on W, so
rank r computes rows [row_range(M, world, r)) of C from its rows of X and the replicated W, with
results bit-identical to the single-GPU call.  No data-path collective is needed; the optional
whole-node gather of C (the north star's "RCCL all-gather of C over xGMI") is ``gather_rows``.
"""
from __future__ import annotations


def row_range(M: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous, balanced row block [lo, hi) of rank ``rank`` (sizes differ by at most 1)."""
    assert world >= 1 and 0 <= rank < world and M >= 0
    base, extra = divmod(M, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_rows(local, M: int, group=None):
    """All-gather row blocks into the full [M, N] C on every rank (torch.distributed; RCCL on
    GPU tensors, gloo on CPU).  Uneven blocks are padded to the largest and trimmed."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    sizes = [row_range(M, world, r) for r in range(world)]
    maxrows = max(hi - lo for lo, hi in sizes)
    N = local.shape[1]
    buf = local
    if local.shape[0] != maxrows:
        buf = torch.zeros((maxrows, N), dtype=local.dtype, device=local.device)
        buf[: local.shape[0]] = local
    out = torch.empty((world * maxrows, N), dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(out, buf.contiguous(), group=group)
    parts = [out[r * maxrows: r * maxrows + (hi - lo)] for r, (lo, hi) in enumerate(sizes)]
    return torch.cat(parts, 0) if any(hi - lo != maxrows for lo, hi in sizes) else out
