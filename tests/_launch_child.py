"""Rank program for tests/test_distributed_gloo.py::test_launcher_* (not a test module):
started by electionguard.launch.run_ranks with RANK/WORLD_SIZE/MASTER_* set, it shards a
seeded ballot set, all-gathers the partial tallies over gloo and folds them (oracle product
standing in for the GPU fold).  Rank 0 writes {"n_gpus", "tally"} as JSON to argv[1]."""
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
from electionguard.distributed import all_valid, gather_fold_tally, shard_range  # noqa: E402


def ballots(nb, n_real):
    G = O.production_group()
    rng = random.Random(11)
    return [[[rng.randrange(1, G.p) for _ in range(2)] for _ in range(n_real)] for _ in range(nb)]


def fold(elems, groups, length):
    G = O.production_group()
    out = np.zeros((groups, 512), np.uint8)
    for g in range(groups):
        xs = [int.from_bytes(elems[g * length + k].tobytes(), "big") for k in range(length)]
        out[g] = np.frombuffer(G.prodP(xs).to_bytes(512, "big"), np.uint8)
    return out


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo")
    fail = os.environ.get("EG_TEST_FAIL_RANK")  # "r:code": rank r exits with code, the others wait for it
    if fail:
        r, code = (int(x) for x in fail.split(":"))
        if rank == r:
            os._exit(code)
        dist.barrier()  # blocks: the failed rank never arrives (the launcher must end this)
        return
    G = O.production_group()
    nb, n_real = 5, 2
    cts = ballots(nb, n_real)
    a, b = shard_range(nb, world, rank)
    part = np.zeros((n_real, 2, 512), np.uint8)
    for s in range(n_real):
        for c in range(2):
            part[s, c] = np.frombuffer(G.prodP([cts[i][s][c] for i in range(a, b)]).to_bytes(512, "big"), np.uint8)
    ok = all_valid(dist, True, torch.device("cpu"))
    tally = gather_fold_tally(dist, torch.from_numpy(part), fold)
    if rank == 0:
        Path(sys.argv[1]).write_text(json.dumps({"n_gpus": dist.get_world_size(), "ok": ok,
                                                 "tally": [[t.tobytes().hex() for t in sel] for sel in tally]}))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
