"""CPU: pin the oracle.  The reference has no fixtures for this path, so
the golden vectors come from oracle/eg_oracle.py and are cross-checked here against the
independent OpenSSL-BN restatement (oracle/eg_oracle_c.c) and the constants' self-checks."""
import json
import random
from pathlib import Path

import numpy as np
import pytest

import eg_oracle as O

GOLD = Path(__file__).resolve().parent / "golden"


def load(name):
    return json.loads((GOLD / name).read_text())


def h(s):
    return int(s, 16)


def test_constants_derivation_and_selfchecks():
    import sympy
    from electionguard.core import constants as C
    p, q, g, r = O.derive_production_group()
    gold = load("constants.json")
    assert (p, q, g, r) == (h(gold["p"]), h(gold["q"]), h(gold["g"]), h(gold["r"]))
    assert (p, q, g, r) == (C.P, C.Q, C.G, C.R)          # product constants == oracle derivation
    assert q == 2**256 - 189 and p.bit_length() == 4096
    assert (p - 1) % q == 0 and r * q + 1 == p
    assert pow(g, q, p) == 1 and g != 1 and g == pow(2, r, p)
    assert sympy.isprime(q) and sympy.isprime(p)
    assert p % 2**256 == 2**256 - 1                       # Montgomery-friendly: -p^-1 = 1 mod 2^256


def test_python_oracle_reproduces_group_golden(oracle_group):
    G = oracle_group
    d = load("group_ops.json")
    for v in d["powP"]:
        assert G.powP(h(v["b"]), h(v["e"])) == h(v["r"])
    for v in d["gPowP"][:8]:
        assert G.gPowP(h(v["e"])) == h(v["r"])
    for v in d["multP"]:
        assert G.multP(h(v["a"]), h(v["b"])) == h(v["r"])
    for v in d["multInv"]:
        assert G.multInv(h(v["a"])) == h(v["r"])
        assert G.multP(h(v["a"]), h(v["r"])) == 1
    for v in d["prodP"]:
        assert G.prodP([h(x) for x in v["xs"]]) == h(v["r"])


def _arr(hexes, n):
    return np.stack([np.frombuffer(bytes.fromhex(x), np.uint8) for x in hexes]).reshape(-1, n)


def test_c_oracle_agrees_on_group_golden(oracle_group):
    from eg_oracle_c import COracle
    G = oracle_group
    co = COracle(G.p, G.q, G.g)
    d = load("group_ops.json")
    out = co.powp(_arr([v["b"] for v in d["powP"]], 512), _arr([v["e"] for v in d["powP"]], 32))
    assert [x.tobytes().hex() for x in out] == [v["r"] for v in d["powP"]]
    out = co.gpowp(_arr([v["e"] for v in d["gPowP"]], 32))
    assert [x.tobytes().hex() for x in out] == [v["r"] for v in d["gPowP"]]


def golden_ballot_arrays():
    d = load("ballots.json")
    nc, ns, va = d["manifest"]
    spc = ns + va
    nb = len(d["ballots"])
    nsel = nc * spc
    cts = np.zeros((nb, nsel, 2, 512), np.uint8)
    rp = np.zeros((nb, nsel, 4, 32), np.uint8)
    cp = np.zeros((nb, nc, 2, 32), np.uint8)
    for b, bal in enumerate(d["ballots"]):
        cts[b] = _arr([x for ct in bal["cts"] for x in ct], 512).reshape(nsel, 2, 512)
        rp[b] = _arr([x for pr in bal["rproofs"] for x in pr], 32).reshape(nsel, 4, 32)
        cp[b] = _arr([x for pr in bal["cproofs"] for x in pr], 32).reshape(nc, 2, 32)
    return d, (nc, ns, va, spc), cts, rp, cp


def test_c_oracle_verifies_golden_ballots_and_tally(oracle_group):
    from eg_oracle_c import COracle
    G = oracle_group
    d, (nc, ns, va, spc), cts, rp, cp = golden_ballot_arrays()
    co = COracle(G.p, G.q, G.g)
    co.set_key(h(d["K"]))
    ok_s, ok_c, tally = co.verify_ballots(h(d["qbar"]), nc, spc, va, va, cts, rp, cp, threads=2)
    assert ok_s.all() and ok_c.all() and all(b["valid"] for b in d["ballots"])
    assert [[t[0].tobytes().hex(), t[1].tobytes().hex()] for t in tally] == d["tally"]
    bad = rp.copy()
    bad[1, 2, 1, 0] ^= 0x40
    ok_s, _, _ = co.verify_ballots(h(d["qbar"]), nc, spc, va, va, cts, bad, cp, threads=1, tally=False)
    assert not ok_s[1, 2] and ok_s.sum() == ok_s.size - 1


def test_python_oracle_trustee_golden(oracle_group):
    G = oracle_group
    d = load("trustee.json")
    qbar = h(d["qbar"])
    gs = [O.Guardian(f"guardian{g['x']}", g["x"], [h(a) for a in g["coeffs"]], [h(k) for k in g["commitments"]])
          for g in d["guardians"]]
    texts = [O.Ciphertext(h(a), h(b)) for a, b in d["texts"]]
    nonces = [h(u) for u in d["nonces"]]
    for (M, pr), want in zip(O.direct_decrypt(G, qbar, gs[0], texts, nonces), d["direct"]):
        assert (M, pr.c, pr.v) == (h(want["M"]), h(want["c"]), h(want["v"]))
        assert O.verify_share(G, qbar, gs[0].K, texts[0] if False else texts[d["direct"].index(want)], M, pr)


def test_hash_host_matches_oracle():
    from electionguard.core.hashing import hash_elems
    rng = random.Random(9)
    for _ in range(5):
        els = [("Q", rng.randrange(2**256))] + [("P", rng.randrange(2**4096)) for _ in range(3)]
        assert hash_elems(O.Q, *els) == O.hash_elems(O.Q, *els)
