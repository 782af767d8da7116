"""Rank program for tests/test_distributed_gloo.py::test_world8_exchange_* (not a test module): started
by electionguard.launch.run_ranks, it runs electionguard.distributed.TallyExchange the way bench.py
does, over a stand-in group (no GPU: the communicator calls are recorded, the fold is the oracle's
product), in two worlds:
  1. every rank's RCCL probe and init succeed: mode "rccl", rccl_ranks = what the communicator
     reports (here WORLD_SIZE), the verdict and the folded tally over all ranks;
  2. the probe fails on rank EG_TEST_PROBE_FAIL (default 3): the readiness vote keeps EVERY rank
     out of the collective init, the world folds over the host (gloo) with rccl_ranks 0 and a note.
Rank 0 writes the results as JSON to argv[1]."""
import json
import os
import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import eg_oracle as O  # noqa: E402
from electionguard.distributed import TallyExchange, gather_fold_tally, shard_range  # noqa: E402


def ballots(nb, n_real):
    G = O.production_group()
    rng = random.Random(29)
    return [[[rng.randrange(1, G.p) for _ in range(2)] for _ in range(n_real)] for _ in range(nb)]


def fold(elems, groups, length):
    G = O.production_group()
    out = np.zeros((groups, 512), np.uint8)
    for g in range(groups):
        xs = [int.from_bytes(elems[g * length + k].tobytes(), "big") for k in range(length)]
        out[g] = np.frombuffer(G.prodP(xs).to_bytes(512, "big"), np.uint8)
    return out


class Tally:
    """A partial tally 'in HBM' (download() is all TallyExchange needs in host mode)."""

    def __init__(self, a):
        self.a = a

    def download(self):
        return self.a.copy()


class StandInGroup:
    """The communicator calls of GroupContext, recorded; the RCCL collectives stand in over gloo."""

    def __init__(self, rank, world, probe_fail):
        self.rank, self.world, self.probe_fail = rank, world, probe_fail
        self.calls, self.comm = [], None

    def comm_unique_id(self):
        self.calls.append("probe")
        if self.rank == self.probe_fail:
            raise RuntimeError("RCCL unavailable (test)")
        return bytes(range(128))

    def comm_init(self, uid, w, r):
        self.calls.append("init")
        assert uid == bytes(range(128)) and w == self.world and r == self.rank
        self.comm = (w, r)

    def comm_info(self):
        return self.comm if self.comm else (0, 0)

    def comm_destroy(self):
        self.calls.append("destroy")
        self.comm = None

    def comm_all_valid(self, ok):
        t = torch.tensor([1 if ok else 0], dtype=torch.int32)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    def tally_allgather_fold(self, d, nparts, n, root):
        out = gather_fold_tally(dist, d.download().reshape(n // 2, 2, 512), fold)
        return None if out is None else out.reshape(n, 512)

    def prodP_groups(self, elems, groups, length):
        return fold(elems, groups, length)


def run(rank, world, probe_fail, nb, n_real, cts):
    g = StandInGroup(rank, world, probe_fail)
    x = TallyExchange(g, dist, world, rank, "rccl")
    a, b = shard_range(nb, world, rank)
    G = O.production_group()
    part = np.zeros((n_real, 2, 512), np.uint8)
    for s in range(n_real):
        for c in range(2):
            part[s, c] = np.frombuffer(G.prodP([cts[i][s][c] for i in range(a, b)]).to_bytes(512, "big"), np.uint8)
    ok = x.all_valid(True)
    bad = x.all_valid(rank != world - 1)
    tally = x.fold(Tally(part), n_real)
    res = {"mode": x.mode, "collective": x.collective, "rccl_ranks": x.rccl_ranks, "note": x.note,
           "calls": g.calls, "ok": ok, "bad": bad,
           "tally": None if tally is None else [[t.tobytes().hex() for t in sel] for sel in tally]}
    x.close()
    return res


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    nb, n_real = 19, 2  # ragged shards over 8 ranks
    cts = ballots(nb, n_real)
    good = run(rank, world, -1, nb, n_real, cts)
    failed = run(rank, world, int(os.environ.get("EG_TEST_PROBE_FAIL", "3")), nb, n_real, cts)
    calls = [None] * world
    dist.all_gather_object(calls, (good["calls"], failed["calls"], good["rccl_ranks"], failed["rccl_ranks"]))
    if rank == 0:
        Path(sys.argv[1]).write_text(json.dumps({"world": world, "good": good, "failed": failed, "calls": calls}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
