"""The fused GPU verifier on two non-production Schnorr groups (tests/golden/test_groups.json,
made by tests/golden/make_test_groups.py): neither p is Montgomery-friendly, and their
residue-test exponents c = 2^256 - q take both ways the op-program compiler builds
w = x^c -- from the squaring chain's stored powers (sparse c, bits at and past the comb's
table positions) and by the left-to-right ladder (dense c).  Honest oracle-encrypted
ballots verify with the oracle's tally; the alpha * (p-1) forgery with re-made proofs is
rejected for its selection and its contest."""
import json
import random
from pathlib import Path

import numpy as np
import pytest

import eg_oracle as O
from test_oracle_golden import forge_negated_alpha

pytestmark = pytest.mark.gpu

GROUPS = json.loads((Path(__file__).resolve().parent / "golden" / "test_groups.json").read_text())["groups"]


def _group(d):
    h = lambda s: int(s, 16)
    return O.Group(h(d["p"]), h(d["q"]), h(d["g"]))


def _arrays(ebs):
    b = lambda x, n: np.frombuffer(int(x).to_bytes(n, "big"), np.uint8)
    cts = np.stack([np.stack([np.stack([b(ct.pad, 512), b(ct.data, 512)]) for ct in eb.cts]) for eb in ebs])
    rp = np.stack([np.stack([np.stack([b(v, 32) for v in (pr.c0, pr.v0, pr.c1, pr.v1)]) for pr in eb.proofs])
                   for eb in ebs])
    cp = np.stack([np.stack([np.stack([b(pr.c, 32), b(pr.v, 32)]) for pr in eb.contest_proofs]) for eb in ebs])
    return cts, rp, cp


@pytest.mark.parametrize("gd", GROUPS, ids=[g["name"] for g in GROUPS])
def test_verifier_on_test_group(gd):
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
    from electionguard.core import GroupContext
    og = _group(gd)
    rng = random.Random(31)
    _, K = O.key_ceremony(og, 3, 2, rng)
    qbar = rng.randrange(og.q)
    man_o = O.Manifest(2, 3, 1)
    honest = [O.encrypt_ballot(og, K, qbar, man_o, O.ballot_plaintexts(man_o, rng), rng) for _ in range(5)]
    sel = 4  # second contest
    forged = forge_negated_alpha(og, K, qbar, man_o, O.ballot_plaintexts(man_o, rng), rng, sel)
    cts, rp, cp = _arrays(honest + [forged])
    G = GroupContext(og.p, og.q, og.g)
    try:
        man = Manifest(man_o.n_contests, man_o.n_selections, man_o.votes_allowed)
        ok_s, ok_c, _ = Verifier(G, ElectionKey(G, K), qbar, man).verify(EncryptedBallots(cts, rp, cp))
        assert ok_s[:5].all() and ok_c[:5].all()
        assert ok_s[5].tolist() == [i != sel for i in range(man.nsel)]
        assert ok_c[5].tolist() == [True, False]
        # the tally of the honest ballots alone equals the oracle's
        ok_s, ok_c, tally = Verifier(G, ElectionKey(G, K), qbar, man).verify(
            EncryptedBallots(cts[:5], rp[:5], cp[:5]))
        assert ok_s.all() and ok_c.all()
        for i, ct in enumerate(O.accumulate_tally(og, man_o, honest)):
            assert int.from_bytes(tally[i, 0].tobytes(), "big") == ct.pad, i
            assert int.from_bytes(tally[i, 1].tobytes(), "big") == ct.data, i
    finally:
        G.close()
