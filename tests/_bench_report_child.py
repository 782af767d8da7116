"""Rank program for tests/test_distributed_gloo.py::test_bench_line_at_world_2_has_cpu_baseline (not a
test module): started by electionguard.launch.run_ranks, it runs bench.py's N > 1 reporting tail
(barrier, then rank 0 times the CPU port on its host sample: bench.report) on a few
oracle-encrypted ballots, with a stand-in GPU value.  Rank 0 writes the line to argv[1]."""
import json
import random
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))
sys.path.insert(0, str(ROOT / "oracle"))

import numpy as np  # noqa: E402

import bench  # noqa: E402
import eg_oracle as O  # noqa: E402
from electionguard.ballot import EncryptedBallots, Manifest  # noqa: E402


def main():
    a = bench.parse(["--gpus", "2", "--contests", "2", "--selections", "2", "--cpu-seconds", "0.5"])
    world, rank, _, dist = bench.init_ranks(a)
    G = O.production_group()
    rng = random.Random(3)
    gs, K = O.key_ceremony(G, 3, 3, rng)
    qbar = rng.randrange(G.q)
    man_o, man = O.Manifest(2, 2, 1), Manifest(2, 2, 1)
    sample = None
    if rank == 0:
        ebs = [O.encrypt_ballot(G, K, qbar, man_o, O.ballot_plaintexts(man_o, rng), rng) for _ in range(3)]
        b = lambda x, n: np.frombuffer(int(x).to_bytes(n, "big"), np.uint8)  # noqa: E731
        cts = np.stack([np.stack([np.stack([b(c.pad, 512), b(c.data, 512)]) for c in eb.cts]) for eb in ebs])
        rp = np.stack([np.stack([np.stack([b(v, 32) for v in (p.c0, p.v0, p.c1, p.v1)]) for p in eb.proofs])
                       for eb in ebs])
        cp = np.stack([np.stack([np.stack([b(p.c, 32), b(p.v, 32)]) for p in eb.contest_proofs]) for eb in ebs])
        sample = EncryptedBallots(cts, rp, cp)
    out = {"metric": "ballots verified+tallied/sec (node, 4096-bit group)", "value": 1000.0 * world,
           "n_gpus": world, "vs_baseline": None}
    out = bench.report(a, out, world, rank, dist, man, sample, qbar, K)
    if rank == 0:
        Path(sys.argv[1]).write_text(json.dumps(out))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
