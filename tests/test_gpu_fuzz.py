"""GPU: differential tamper fuzzing of the verifier against the independent OpenSSL-BN
oracle (oracle/eg_oracle_c.c).  Each of 160 ballots gets one random corruption: a byte of
alpha or beta (which usually leaves the ciphertext below p but outside the order-q subgroup,
or at/above p), a byte of one range-proof scalar, a byte of a contest-proof scalar, a whole
ciphertext component replaced by p - x (the order-2 twist of a valid residue, hash-checked
values unchanged otherwise), or nothing.  The GPU's per-selection and per-contest verdicts
must equal the oracle's for every ballot (Verifier.verify, RunRemoteWorkflowTest.java:179-182,
with the EG 1.0 residue checks)."""
import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


def test_random_tampers_match_c_oracle(group):
    from eg_oracle_c import COracle
    from electionguard.ballot import (ElectionKey, EncryptedBallots, Manifest, Verifier, batch_encryption,
                                      random_scalars, random_votes)
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 3, 3, seed=123)
    key = ElectionKey(group, K, window_bits=12)
    man = Manifest(2, 3, 1)
    rng = np.random.default_rng(123)
    nb = 160
    qbar = 99991
    votes = random_votes(rng, man, nb)
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), group.q),
                          random_scalars(rng, (nb, man.n_contests), group.q))
    p = O.production_group().p
    cts, rp, cp = eb.cts.copy(), eb.rproof.copy(), eb.cproof.copy()
    kinds = []
    for b in range(nb):
        kind = int(rng.integers(0, 5))
        s = int(rng.integers(0, man.nsel))
        if kind == 0:    # one byte of alpha or beta
            cts[b, s, int(rng.integers(0, 2)), int(rng.integers(0, 512))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif kind == 1:  # one byte of c0 / v0 / c1 / v1
            rp[b, s, int(rng.integers(0, 4)), int(rng.integers(0, 32))] ^= np.uint8(1 << int(rng.integers(0, 8)))
        elif kind == 2:  # one byte of a contest proof's c or v
            cp[b, int(rng.integers(0, man.n_contests)), int(rng.integers(0, 2)), int(rng.integers(0, 32))] ^= \
                np.uint8(1 << int(rng.integers(0, 8)))
        elif kind == 3:  # x -> p - x: still < p, but (-1)-twisted out of the subgroup
            comp = int(rng.integers(0, 2))
            x = int.from_bytes(cts[b, s, comp].tobytes(), "big")
            cts[b, s, comp] = np.frombuffer((p - x).to_bytes(512, "big"), np.uint8)
        kinds.append(kind)   # kind 4: untouched
    V = Verifier(group, key, qbar, man)
    ok_s, ok_c, _ = V.verify(EncryptedBallots(cts, rp, cp), with_tally=False)
    co = COracle(O.production_group().p, O.Q, O.production_group().g)
    co.set_key(K)
    want_s, want_c, _ = co.verify_ballots(qbar, man.n_contests, man.spc, 1, 1, cts, rp, cp, threads=8, tally=False)
    assert np.array_equal(ok_s.astype(bool), np.asarray(want_s, bool)), np.argwhere(ok_s != want_s).tolist()
    assert np.array_equal(ok_c.astype(bool), np.asarray(want_c, bool)), np.argwhere(ok_c != want_c).tolist()
    # the fuzz must actually exercise rejections of every kind and keep the untouched ballots
    kinds = np.array(kinds)
    bad_ballot = ~(ok_s.all(axis=1) & ok_c.all(axis=1))
    for k in range(4):
        assert bad_ballot[kinds == k].all(), k
    assert not bad_ballot[kinds == 4].any()
