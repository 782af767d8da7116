"""Multi-GPU plumbing for the ballot path: one process per GPU.

Ballots are independent, so ranks own contiguous ballot shards and exchange NOTHING on
the data path except the final per-selection partial tallies (2 x n_real x 512 B per
rank): one all-gather over RCCL/xGMI, then a mod-p fold on rank 0 (RCCL has no
modular-multiply reduction op).  Verdicts are combined with an all-reduce(min).
Trustees are NOT sharded: each remote DecryptingTrustee is its own process with its own
GPU (replicas only, separate trust domains).
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import numpy as np


def shard_range(n_total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous ballot range of `rank` (sizes differ by at most one)."""
    base, extra = divmod(n_total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _host_collectives(dist) -> bool:
    """gloo (CPU tests, single-GPU rehearsals) runs the collectives on host tensors;
    nccl (= RCCL) runs them on the device tensors over xGMI."""
    return dist.get_backend() == "gloo"


def all_valid(dist, ok: bool, device) -> bool:
    import torch

    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        if _host_collectives(dist):
            flag = flag.cpu()
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def gather_fold_tally(dist, local_tally, fold: Callable[[np.ndarray, int, int], np.ndarray],
                      dst: int = 0) -> Optional[np.ndarray]:
    """All-gather (n_real, 2, 512) uint8 partial tallies from every rank and fold them
    mod p on `dst` with fold(elems (groups*world, 512), groups, world) -> (groups, 512)
    (GroupContext.prodP_groups on the GPU in production)."""
    import torch

    world = dist.get_world_size() if (dist is not None and dist.is_initialized()) else 1
    if world == 1:
        return local_tally.cpu().numpy()
    shp = tuple(local_tally.shape)
    if _host_collectives(dist):
        parts_l = [torch.empty(shp, dtype=local_tally.dtype) for _ in range(world)]
        dist.all_gather(parts_l, local_tally.detach().cpu().contiguous())
        gathered = torch.cat(parts_l, 0)
    else:
        gathered = torch.empty((world * shp[0],) + shp[1:], dtype=local_tally.dtype, device=local_tally.device)
        dist.all_gather_into_tensor(gathered, local_tally.contiguous())  # rank-major concatenation
    if dist.get_rank() != dst:
        return None
    parts = gathered.cpu().numpy().reshape((world,) + shp)  # (world, n_real, 2, 512)
    n_real = parts.shape[1]
    g = np.ascontiguousarray(np.transpose(parts, (1, 2, 0, 3))).reshape(-1, 512)
    return fold(g, n_real * 2, world).reshape(n_real, 2, 512)
