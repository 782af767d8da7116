"""GPU: the trustee's constant-time path (k_pow<F, true>: comb with full 32-entry masked table
scans, g^u from g's shared comb table, branch-free mod-q response) stays bit-exact against the
oracle on edge-case secrets and nonces (0/1 digits everywhere, all-ones rows, q-1), in both
production groups."""
import random

import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", [O.MODE4096, O.MODE4096_V2])
def test_trustee_shares_edge_exponents(mode):
    from electionguard.core import productionGroup
    from electionguard.decrypt import partial_decrypt_batch
    group = productionGroup(0, mode)
    G = O.production_group(mode)
    rng = random.Random(17)
    q = G.q
    texts = [O.encrypt(G, G.gPowP(rng.randrange(1, q)), rng.randrange(3), rng.randrange(1, q)) for _ in range(6)]
    T = np.stack([np.stack([np.frombuffer(t.pad.to_bytes(512, "big"), np.uint8),
                            np.frombuffer(t.data.to_bytes(512, "big"), np.uint8)]) for t in texts])
    nonces = [1, q - 1, 2**52 - 1, 2**255, (2**256 - 1) % q, rng.randrange(1, q)]
    N = np.stack([np.frombuffer(u.to_bytes(32, "big"), np.uint8) for u in nonces])
    qbar = rng.randrange(q)
    for s in (1, 2, q - 1, 2**255 + 12345, rng.randrange(1, q)):
        gd = O.Guardian("g", 1, [s], [G.gPowP(s)])
        want = O.direct_decrypt(G, qbar, gd, texts, nonces)
        M, pr = partial_decrypt_batch(group, s, qbar, T, N)
        for i, (Mw, pw) in enumerate(want):
            assert int.from_bytes(M[i].tobytes(), "big") == Mw, (s, i)
            assert int.from_bytes(pr[i, 0].tobytes(), "big") == pw.c and int.from_bytes(pr[i, 1].tobytes(), "big") == pw.v
