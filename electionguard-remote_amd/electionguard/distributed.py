"""Multi-GPU plumbing for the ballot path: one process per GPU.

Ballots are independent, so ranks own contiguous ballot shards and exchange NOTHING on
the data path except the final per-selection partial tallies (2 x n_real x 512 B per
rank): one all-gather over RCCL/xGMI, then a mod-p fold on rank 0 (RCCL has no
modular-multiply reduction op).  Verdicts are combined with an all-reduce(min).
Trustees are NOT sharded: each remote DecryptingTrustee is its own process with its own
GPU (replicas only, separate trust domains).

The exchange runs inside libeg_hip.so (``TallyExchange`` in "rccl" mode: eg_comm_init /
eg_comm_all_valid / eg_tally_allgather_fold on the context's stream and HIP runtime), so a
rank process holds one HIP runtime and never passes device memory to another framework.  A
host process group (torch.distributed over gloo: CPU only, it never touches the GPU) carries
the control traffic: the RCCL unique id, barriers and the max-over-ranks step time.  Mode
"gloo" keeps the whole exchange on the host (every rank may then share one GPU: the
single-GPU rehearsal of the N > 1 path, and the CPU tests).
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


def all_valid(dist, ok: bool, device=None) -> bool:
    """min over ranks of ok through the torch process group (host tensors under gloo)."""
    import torch

    flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    if dist is not None and dist.is_initialized() and dist.get_world_size() > 1:
        if _host_collectives(dist):
            flag = flag.cpu()
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    return bool(flag.item())


def gather_fold_tally(dist, local_tally, fold: Callable[[np.ndarray, int, int], np.ndarray],
                      dst: int = 0) -> Optional[np.ndarray]:
    """All-gather (n_real, 2, 512) uint8 partial tallies (a numpy array or torch tensor) from every
    rank and fold them mod p on `dst` with fold(elems (groups*world, 512), groups, world) ->
    (groups, 512) (GroupContext.prodP_groups on the GPU in production)."""
    import torch

    if isinstance(local_tally, np.ndarray):
        local_tally = torch.from_numpy(np.ascontiguousarray(local_tally))
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


def share_comm_id(dist, rank: int, make_id: Callable[[], bytes], src: int = 0) -> bytes:
    """Rank `src` makes the 128-byte RCCL unique id (eg_comm_unique_id) and every rank of the host
    process group receives it (broadcast over gloo, before any rank touches RCCL)."""
    box = [make_id() if rank == src else None]
    dist.broadcast_object_list(box, src=src)
    uid = box[0]
    if not isinstance(uid, (bytes, bytearray)) or len(uid) != 128:
        raise RuntimeError("bad RCCL unique id from rank %d" % src)
    return bytes(uid)


def max_over_ranks(dist, x: float) -> float:
    """max of a host float over the host process group (the step time every rank measured)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(x)
    import torch

    t = torch.tensor([float(x)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


class TallyExchange:
    """The per-step exchange of the sharded verify + tally for one rank.

    mode "rccl": libeg_hip's RCCL communicator on the group's context (the id travels over
    ``dist``, the host process group); the verdict is an RCCL all-reduce(min) and the tally one
    ncclAllGather plus the k_prod fold on rank 0's GPU (eg_tally_allgather_fold).
    mode "gloo": the tally comes back to the host and travels over ``dist`` (gloo), rank 0 folds
    it on its GPU (prodP_groups); every rank may share one GPU.
    world 1: the local tally, through the same fold entry point (no communicator)."""

    def __init__(self, group, dist, world: int, rank: int, mode: str = "rccl", fallback: bool = True):
        if mode not in ("rccl", "gloo"):
            raise ValueError(f"unknown exchange mode {mode!r}")
        self.group, self.dist, self.world, self.rank, self.mode = group, dist, world, rank, mode
        self.note = None
        if world > 1 and mode == "rccl":
            # 1. readiness vote BEFORE any rank enters the collective eg_comm_init: every
            #    rank opens RCCL (eg_comm_unique_id doubles as the probe; rank 0's id is the one used)
            #    and the world proceeds only if every rank could
            err = None
            try:
                uid = group.comm_unique_id()
            except Exception as e:
                uid, err = b"", e
            ready = all_valid(dist, err is None)
            if ready:
                box = [uid if rank == 0 else None]
                dist.broadcast_object_list(box, src=0)
                uid = box[0]
                # 2. the collective init: a non-blocking communicator with a deadline inside libeg
                #    (EG_COMM_TIMEOUT_S), so a rank whose peers fail returns with an error instead of
                #    hanging, and reaches the vote below
                try:
                    group.comm_init(uid, world, rank)
                except Exception as e:
                    err = e
                ready = all_valid(dist, err is None)
            # every rank learns whether every rank has a communicator; if one failed, the whole
            # world keeps the exchange on the host (the line says so, rccl_ranks = 0) instead of dying
            if not ready:
                if fallback:
                    # every rank drops what it has: a live communicator, or (the rank whose init
                    # failed) the context's sticky aborted-communicator state
                    try:
                        group.comm_destroy()
                    except Exception as e:  # noqa: BLE001 - the host exchange does not need it
                        import sys
                        print(f"rank {rank}: comm_destroy after a failed init: {e}", file=sys.stderr, flush=True)
                    self.mode = "gloo"
                    self.note = f"RCCL communicator unavailable ({err or 'on another rank'}): host exchange"
                    import sys
                    print(f"rank {rank}: {self.note}", file=sys.stderr, flush=True)
                else:  # strict (bench.py --strict-rccl, the default at N > 1): every rank fails
                    raise RuntimeError(f"eg_comm_init failed: {err or 'on another rank'}")

    @property
    def collective(self) -> str:
        if self.world == 1:
            return "no communicator (world 1: local fold)"
        return "RCCL (libeg_hip)" if self.mode == "rccl" else "gloo (host)"

    @property
    def rccl_ranks(self) -> int:
        """Ranks of the RCCL communicator as RCCL itself reports them (eg_comm_info ->
        ncclCommCount); 0 when the exchange runs without one (world 1, or the host fallback)."""
        if self.world == 1 or self.mode != "rccl":
            return 0
        return int(self.group.comm_info()[0])

    def all_valid(self, ok: bool) -> bool:
        if self.world == 1:
            return bool(ok)
        if self.mode == "rccl":
            return self.group.comm_all_valid(ok)
        return all_valid(self.dist, ok)

    def fold(self, d_tally, n_real: int) -> Optional[np.ndarray]:
        """d_tally: this rank's (n_real, 2, 512) partial tally in HBM (a DeviceBuffer) ->
        the folded (n_real, 2, 512) tally on rank 0, None on the others."""
        if self.world == 1 or self.mode == "rccl":
            out = self.group.tally_allgather_fold(d_tally, 1, n_real * 2, 0)
            return None if out is None else out.reshape(n_real, 2, 512)
        local = d_tally.download().reshape(n_real, 2, 512)
        return gather_fold_tally(self.dist, local, self.group.prodP_groups)

    def close(self) -> None:
        if self.world > 1 and self.mode == "rccl":
            self.group.comm_destroy()
