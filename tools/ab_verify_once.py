"""One verify workload (AB_NB ballots of 4x5, AB_WB-bit tables) on the library EG_LIB names,
for per-kernel traces of A/B builds (tools/ab_kernels.sh)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "electionguard-remote_amd"))
from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes  # noqa: E402
from electionguard.core import productionGroup  # noqa: E402
from electionguard.keyceremony import key_ceremony  # noqa: E402

G = productionGroup(0)
_, K = key_ceremony(G, 3, 3, seed=5)
key = ElectionKey(G, K, window_bits=int(os.environ.get("AB_WB", "16")))
man = Manifest(4, 5, 1)
rng = np.random.default_rng(0)
nb = int(os.environ.get("AB_NB", "4000"))
votes = random_votes(rng, man, nb)
eb = batch_encryption(G, key, 77, man, votes, random_scalars(rng, (nb, man.nsel, 4), G.q),
                      random_scalars(rng, (nb, man.n_contests), G.q))
V = Verifier(G, key, 77, man)
for _ in range(3):
    ok_s, ok_c, _ = V.verify(eb)
    assert ok_s.all() and ok_c.all()
print("ok")
