"""CPU checks of the non-production test groups (tests/golden/test_groups.json) the GPU
verifier is run on in tests/test_gpu_test_groups.py: they are Schnorr groups with the
stated c = 2^256 - q shapes, and both oracles accept honest ballots on them and reject the
alpha * (p-1) forgery (so the GPU test's expectations are the oracles' verdicts)."""
import json
import random
from pathlib import Path

import numpy as np
import pytest

import eg_oracle as O
from test_oracle_golden import forge_negated_alpha

GROUPS = json.loads((Path(__file__).resolve().parent / "golden" / "test_groups.json").read_text())["groups"]
h = lambda s: int(s, 16)


def _mr(n, rounds=4, seed=3):
    rng = random.Random(seed)
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        x = pow(rng.randrange(2, n - 2), d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


@pytest.mark.parametrize("gd", GROUPS, ids=[g["name"] for g in GROUPS])
def test_test_group_is_schnorr(gd):
    p, q, g = h(gd["p"]), h(gd["q"]), h(gd["g"])
    assert p.bit_length() == 4096 and q.bit_length() in (255, 256) and (p - 1) % q == 0
    assert g != 1 and pow(g, q, p) == 1
    assert _mr(q, 16) and _mr(p, 2)
    assert p % (1 << 29) != (1 << 29) - 1          # not Montgomery-friendly: general CIOS path
    c = 2 ** 256 - q
    assert bin(c).count("1") == gd["c_popcount"]
    if gd["name"] == "sparse_c":
        assert gd["c_popcount"] <= 16 and all((c >> b) & 1 for b in (26, 52, 208, 240, 255))
    else:
        assert gd["c_popcount"] > 16                # the ladder fallback


@pytest.mark.parametrize("gd", GROUPS, ids=[g["name"] for g in GROUPS])
def test_oracles_on_test_group(gd):
    from eg_oracle_c import COracle
    og = O.Group(h(gd["p"]), h(gd["q"]), h(gd["g"]))
    rng = random.Random(31)
    _, K = O.key_ceremony(og, 3, 2, rng)
    qbar = rng.randrange(og.q)
    man = O.Manifest(2, 3, 1)
    honest = O.encrypt_ballot(og, K, qbar, man, O.ballot_plaintexts(man, rng), rng)
    assert O.verify_ballot(og, K, qbar, man, honest)
    sel = 4
    forged = forge_negated_alpha(og, K, qbar, man, O.ballot_plaintexts(man, rng), rng, sel)
    assert not O.verify_ballot(og, K, qbar, man, forged)
    b = lambda x, n: np.frombuffer(int(x).to_bytes(n, "big"), np.uint8)
    cts = np.stack([np.stack([np.stack([b(ct.pad, 512), b(ct.data, 512)]) for ct in eb.cts]) for eb in (honest, forged)])
    rp = np.stack([np.stack([np.stack([b(v, 32) for v in (pr.c0, pr.v0, pr.c1, pr.v1)]) for pr in eb.proofs])
                   for eb in (honest, forged)])
    cp = np.stack([np.stack([np.stack([b(pr.c, 32), b(pr.v, 32)]) for pr in eb.contest_proofs])
                   for eb in (honest, forged)])
    co = COracle(og.p, og.q, og.g)
    co.set_key(K)
    ok_s, ok_c, _ = co.verify_ballots(qbar, man.n_contests, man.sel_per_contest, 1, 1, cts, rp, cp, tally=False)
    assert ok_s[0].all() and ok_c[0].all()
    assert ok_s[1].tolist() == [i != sel for i in range(man.sel_per_ballot)]
    assert ok_c[1].tolist() == [True, False]
