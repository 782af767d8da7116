"""CPU: pin the oracle.  The reference has no fixtures for this path, so
the golden vectors come from oracle/eg_oracle.py and are cross-checked here against the
independent OpenSSL-BN restatement (oracle/eg_oracle_c.c) and the constants' self-checks.
Every fixture exists for both production groups (tests/golden/<ProductionMode>/):
Mode4096 (EG 1.0, the reference's group) and Mode4096_V2 (EG 2.0)."""
import json
import random
from pathlib import Path

import numpy as np
import pytest

import eg_oracle as O

GOLD = Path(__file__).resolve().parent / "golden"
MODES = (O.MODE4096, O.MODE4096_V2)


def load(name, mode=O.MODE4096):
    return json.loads((GOLD / mode / name).read_text())


def h(s):
    return int(s, 16)


@pytest.mark.parametrize("mode", MODES)
def test_constants_derivation_and_selfchecks(mode):
    import sympy
    from electionguard.core import constants as C
    p, q, g, r = O.derive_group(mode)
    gold = load("constants.json", mode)
    assert (p, q, g, r) == (h(gold["p"]), h(gold["q"]), h(gold["g"]), h(gold["r"]))
    c = C.constants_for(mode)
    assert (p, q, g, r) == (c.p, c.q, c.g, c.r)          # product constants == oracle derivation
    assert q == 2**256 - 189 and p.bit_length() == 4096
    assert (p - 1) % q == 0 and r * q + 1 == p
    assert pow(g, q, p) == 1 and g != 1 and g == pow(2, r, p)
    assert sympy.isprime(q) and sympy.isprime(p) and sympy.isprime(r // 2)
    assert p % 2**256 == 2**256 - 1                       # Montgomery-friendly: -p^-1 = 1 mod 2^256


def test_reference_group_is_the_eg1_gamma_group():
    """Mode4096 (the default everywhere) is built from Euler's gamma and reproduces the
    published EG 1.0 generator; the ln 2 group is only the named V2 option."""
    from electionguard.core import constants as C
    assert C.P == C.MODE4096.p and C.G == C.MODE4096.g
    assert f"{C.P:01024X}"[64:96] == "93C467E37DB0C7A4D1BE3F810152CB56"   # gamma = 0.93C467E3...h
    assert f"{C.G:01024X}".startswith(O.EG1_G_PREFIX)
    assert f"{C.MODE4096_V2.p:01024X}"[64:80] == "B17217F7D1CF79AB"        # ln 2 = 0.B17217F7...h
    assert O.production_group().p == C.P


@pytest.mark.parametrize("mode", MODES)
def test_python_oracle_reproduces_group_golden(mode):
    G = O.production_group(mode)
    d = load("group_ops.json", mode)
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


@pytest.mark.parametrize("mode", MODES)
def test_c_oracle_agrees_on_group_golden(mode):
    from eg_oracle_c import COracle
    G = O.production_group(mode)
    co = COracle(G.p, G.q, G.g)
    d = load("group_ops.json", mode)
    out = co.powp(_arr([v["b"] for v in d["powP"]], 512), _arr([v["e"] for v in d["powP"]], 32))
    assert [x.tobytes().hex() for x in out] == [v["r"] for v in d["powP"]]
    out = co.gpowp(_arr([v["e"] for v in d["gPowP"]], 32))
    assert [x.tobytes().hex() for x in out] == [v["r"] for v in d["gPowP"]]


def golden_ballot_arrays(mode=O.MODE4096):
    d = load("ballots.json", mode)
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


@pytest.mark.parametrize("mode", MODES)
def test_c_oracle_verifies_golden_ballots_and_tally(mode):
    from eg_oracle_c import COracle
    G = O.production_group(mode)
    d, (nc, ns, va, spc), cts, rp, cp = golden_ballot_arrays(mode)
    co = COracle(G.p, G.q, G.g)
    co.set_key(h(d["K"]))
    ok_s, ok_c, tally = co.verify_ballots(h(d["qbar"]), nc, spc, va, va, cts, rp, cp, threads=2)
    assert ok_s.all() and ok_c.all() and all(b["valid"] for b in d["ballots"])
    assert [[t[0].tobytes().hex(), t[1].tobytes().hex()] for t in tally] == d["tally"]
    bad = rp.copy()
    bad[1, 2, 1, 0] ^= 0x40
    ok_s, _, _ = co.verify_ballots(h(d["qbar"]), nc, spc, va, va, cts, bad, cp, threads=1, tally=False)
    assert not ok_s[1, 2] and ok_s.sum() == ok_s.size - 1


@pytest.mark.parametrize("mode", MODES)
def test_c_oracle_encrypts_golden_ballots_byte_exact(mode):
    """The C oracle's batchEncryption (known-nonce fake branch, 8-bit radix tables) reproduces the
    golden ballots' bytes from their injected nonces: ciphertexts, range proofs and contest proofs."""
    from eg_oracle_c import COracle
    G = O.production_group(mode)
    d, (nc, ns, va, spc), cts, rp, cp = golden_ballot_arrays(mode)
    co = COracle(G.p, G.q, G.g)
    co.set_key(h(d["K"]))
    votes = np.array([b["votes"] for b in d["ballots"]], np.uint8)
    sn = np.stack([_arr([x for n4 in b["nonces"] for x in n4], 32).reshape(-1, 4, 32) for b in d["ballots"]])
    cn = np.stack([_arr(b["contest_nonces"], 32) for b in d["ballots"]])
    for threads in (1, 2):
        c2, r2, p2 = co.encrypt_ballots(h(d["qbar"]), nc, spc, votes, sn, cn, threads=threads)
        assert np.array_equal(c2, cts) and np.array_equal(r2, rp) and np.array_equal(p2, cp)


@pytest.mark.parametrize("mode", MODES)
def test_c_oracle_trustee_golden(mode):
    """The C oracle's directDecrypt / compensatedDecrypt reproduce the golden shares and proofs."""
    from eg_oracle_c import COracle
    G = O.production_group(mode)
    d = load("trustee.json", mode)
    co = COracle(G.p, G.q, G.g)
    T = np.stack([_arr(t, 512) for t in d["texts"]])
    N = _arr(d["nonces"], 32)
    M, pr = co.trustee_decrypt(h(d["guardians"][0]["coeffs"][0]), h(d["qbar"]), T, N, threads=3)
    assert [(m.tobytes().hex(), p[0].tobytes().hex(), p[1].tobytes().hex()) for m, p in zip(M, pr)] == \
        [(w["M"], w["c"], w["v"]) for w in d["direct"]]
    share = O.poly_eval([h(a) for a in d["guardians"][2]["coeffs"]], 2, O.Q)
    M, pr = co.trustee_decrypt(share, h(d["qbar"]), T, N)
    assert [(m.tobytes().hex(), p[0].tobytes().hex(), p[1].tobytes().hex()) for m, p in zip(M, pr)] == \
        [(w["M"], w["c"], w["v"]) for w in d["compensated_by_x2_for_x3"]]


@pytest.mark.parametrize("mode", MODES)
def test_python_oracle_trustee_golden(mode):
    G = O.production_group(mode)
    d = load("trustee.json", mode)
    qbar = h(d["qbar"])
    gs = [O.Guardian(f"guardian{g['x']}", g["x"], [h(a) for a in g["coeffs"]], [h(k) for k in g["commitments"]])
          for g in d["guardians"]]
    texts = [O.Ciphertext(h(a), h(b)) for a, b in d["texts"]]
    nonces = [h(u) for u in d["nonces"]]
    for i, ((M, pr), want) in enumerate(zip(O.direct_decrypt(G, qbar, gs[0], texts, nonces), d["direct"])):
        assert (M, pr.c, pr.v) == (h(want["M"]), h(want["c"]), h(want["v"]))
        assert O.verify_share(G, qbar, gs[0].K, texts[i], M, pr)


@pytest.mark.parametrize("fmt", ["fixed", "minimal"])
def test_hash_host_matches_oracle(fmt):
    from electionguard.core.hashing import hash_elems, hexP, hexQ
    rng = random.Random(9)
    for _ in range(5):
        els = [("Q", rng.randrange(2**256))] + [("P", rng.randrange(2**4096)) for _ in range(3)] + \
              [("P", rng.randrange(2**100)), ("Q", 0), ("P", 5)]
        with O.hash_format(fmt):
            assert hash_elems(O.Q, *els, fmt=fmt) == O.hash_elems(O.Q, *els)
    # the minimal form is electionguard-python's to_hex: even length, leading zero bytes dropped
    assert (hexQ(0, "minimal"), hexQ(5, "minimal"), hexP(0xABC, "minimal")) == ("00", "05", "0ABC")
    assert len(hexP(5, "fixed")) == 1024 and len(hexQ(5, "fixed")) == 64


# --------------------------------------------------------------------------------------
# Residue (subgroup) validation: a ballot whose alpha is multiplied by p-1 (order 2) while
# its proofs are re-made to match.  Without the x^q == 1 tests every proof verifies.
# --------------------------------------------------------------------------------------

def forge_negated_alpha(G, K, qbar, man, votes, rng, sel):
    """Encrypt a ballot, then replace selection `sel`'s alpha by (p-1)*alpha = -alpha and
    re-make its range proof and its contest's constant proof so that every Fiat-Shamir
    check passes on the forged ciphertext: the real-branch recompute g^v (-alpha)^c equals
    g^u exactly when c is even, so the prover retries its nonces until both challenges are
    even.  Returns (ballot, the honest nonces R per selection)."""
    q = G.q
    spc = man.sel_per_contest
    Rs = [rng.randrange(1, q) for _ in votes]
    cts = [O.encrypt(G, K, m, R) for m, R in zip(votes, Rs)]
    cts[sel] = O.Ciphertext((G.p - 1) * cts[sel].pad % G.p, cts[sel].data)
    proofs, cproofs = [], []
    for i, (ct, m, R) in enumerate(zip(cts, votes, Rs)):
        while True:
            pr = O.make_range_proof(G, K, qbar, ct, m, R, rng.randrange(1, q), rng.randrange(q), rng.randrange(q))
            c_real = pr.c0 if m == 0 else pr.c1
            if i != sel or c_real % 2 == 0:
                break
        proofs.append(pr)
    for c in range(man.n_contests):
        sl = slice(c * spc, (c + 1) * spc)
        A = G.prodP([ct.pad for ct in cts[sl]])
        B = G.prodP([ct.data for ct in cts[sl]])
        R_sum = sum(Rs[sl]) % q
        while True:
            cpr = O.make_constant_proof(G, K, qbar, A, B, R_sum, rng.randrange(1, q))
            if not (c * spc <= sel < (c + 1) * spc) or cpr.c % 2 == 0:
                break
        cproofs.append(cpr)
    return O.EncryptedBallot(cts, proofs, cproofs)


def _proof_checks_without_residues(G, K, qbar, man, eb):
    """The verifier's Fiat-Shamir equations alone (no residue tests)."""
    spc = man.sel_per_contest
    ok = []
    for i, (ct, pr) in enumerate(zip(eb.cts, eb.proofs)):
        a0, b0, a1, b1 = O.range_commitments(G, K, ct, pr)
        ok.append((pr.c0 + pr.c1) % G.q == O.range_challenge(G, qbar, ct, a0, b0, a1, b1))
    for c in range(man.n_contests):
        A = G.prodP([ct.pad for ct in eb.cts[c * spc:(c + 1) * spc]])
        B = G.prodP([ct.data for ct in eb.cts[c * spc:(c + 1) * spc]])
        a, b = O.constant_commitments(G, K, A, B, man.votes_allowed, eb.contest_proofs[c])
        ok.append(eb.contest_proofs[c].c == O.constant_challenge(G, qbar, A, B, a, b))
    return ok


def residue_forgery_case(seed=77):
    G = O.production_group()
    rng = random.Random(seed)
    gs, K = O.key_ceremony(G, 2, 2, rng)
    qbar = rng.randrange(G.q)
    man = O.Manifest(2, 2, 1)
    votes = O.ballot_plaintexts(man, rng)
    sel = 1
    eb = forge_negated_alpha(G, K, qbar, man, votes, rng, sel)
    return G, K, qbar, man, eb, sel


def test_oracle_rejects_non_residue_alpha_with_matching_proofs():
    G, K, qbar, man, eb, sel = residue_forgery_case()
    assert all(_proof_checks_without_residues(G, K, qbar, man, eb))   # the forgery is complete
    assert not O.is_valid_residue(G, eb.cts[sel].pad)
    ok_sel = [O.verify_range_proof(G, K, qbar, ct, pr) for ct, pr in zip(eb.cts, eb.proofs)]
    assert ok_sel == [i != sel for i in range(len(eb.cts))]
    assert not O.verify_ballot(G, K, qbar, man, eb)
    spc = man.sel_per_contest
    A = G.prodP([ct.pad for ct in eb.cts[:spc]])
    assert not O.is_valid_residue(G, A)                                  # the contest is flagged too


def test_c_oracle_rejects_non_residue_alpha():
    from eg_oracle_c import COracle
    G, K, qbar, man, eb, sel = residue_forgery_case()
    b = lambda x, n: np.frombuffer(int(x).to_bytes(n, "big"), np.uint8)
    cts = np.stack([np.stack([b(ct.pad, 512), b(ct.data, 512)]) for ct in eb.cts])[None]
    rp = np.stack([np.stack([b(v, 32) for v in (pr.c0, pr.v0, pr.c1, pr.v1)]) for pr in eb.proofs])[None]
    cp = np.stack([np.stack([b(pr.c, 32), b(pr.v, 32)]) for pr in eb.contest_proofs])[None]
    co = COracle(G.p, G.q, G.g)
    co.set_key(K)
    ok_s, ok_c, _ = co.verify_ballots(qbar, man.n_contests, man.sel_per_contest, 1, 1, cts, rp, cp, tally=False)
    assert ok_s[0].tolist() == [i != sel for i in range(len(eb.cts))]
    assert ok_c[0].tolist() == [False, True]


def twisted_pair_case(seed=78):
    """An honest ballot whose contest 0 has the alphas of its first two selections multiplied by
    p - 1 (order 2): both selections are non-residues, but A = prod alpha is unchanged, so the
    contest's own proof still verifies.  The contest is rejected with its selections."""
    G = O.production_group()
    rng = random.Random(seed)
    gs, K = O.key_ceremony(G, 2, 2, rng)
    qbar = rng.randrange(G.q)
    man = O.Manifest(2, 2, 1)
    eb = O.encrypt_ballot(G, K, qbar, man, O.ballot_plaintexts(man, rng), rng)
    for i in (0, 1):
        eb.cts[i] = O.Ciphertext(eb.cts[i].pad * (G.p - 1) % G.p, eb.cts[i].data)
    return G, K, qbar, man, eb


def ballot_wire_arrays(eb):
    b = lambda x, n: np.frombuffer(int(x).to_bytes(n, "big"), np.uint8)
    cts = np.stack([np.stack([b(ct.pad, 512), b(ct.data, 512)]) for ct in eb.cts])[None]
    rp = np.stack([np.stack([b(v, 32) for v in (pr.c0, pr.v0, pr.c1, pr.v1)]) for pr in eb.proofs])[None]
    cp = np.stack([np.stack([b(pr.c, 32), b(pr.v, 32)]) for pr in eb.contest_proofs])[None]
    return cts, rp, cp


def test_contest_with_two_invalid_selections_is_rejected_by_both_oracles():
    from eg_oracle_c import COracle
    G, K, qbar, man, eb = twisted_pair_case()
    spc = man.sel_per_contest
    A = G.prodP([ct.pad for ct in eb.cts[:spc]])
    B = G.prodP([ct.data for ct in eb.cts[:spc]])
    assert O.is_valid_residue(G, A) and O.is_valid_residue(G, B)     # the aggregate alone passes
    assert O.verify_constant_proof(G, K, qbar, A, B, man.votes_allowed, eb.contest_proofs[0])
    assert not O.verify_ballot(G, K, qbar, man, eb)
    co = COracle(G.p, G.q, G.g)
    co.set_key(K)
    ok_s, ok_c, _ = co.verify_ballots(qbar, man.n_contests, spc, 1, 1, *ballot_wire_arrays(eb), tally=False)
    assert ok_s[0].tolist() == [i > 1 for i in range(len(eb.cts))]
    assert ok_c[0].tolist() == [False, True]


# --------------------------------------------------------------------------------------
# Spoiled ballots (RunRemoteDecryptor.java:264-269): cast-only tally and decryptBallot.
# --------------------------------------------------------------------------------------

def spoiled_case(mode=O.MODE4096):
    d = load("spoiled.json", mode)
    nc, ns, va = d["manifest"]
    spc = ns + va
    nsel = nc * spc
    nb = len(d["ballots"])
    cts = np.zeros((nb, nsel, 2, 512), np.uint8)
    rp = np.zeros((nb, nsel, 4, 32), np.uint8)
    cp = np.zeros((nb, nc, 2, 32), np.uint8)
    for b, bal in enumerate(d["ballots"]):
        cts[b] = _arr([x for ct in bal["cts"] for x in ct], 512).reshape(nsel, 2, 512)
        rp[b] = _arr([x for pr in bal["rproofs"] for x in pr], 32).reshape(nsel, 4, 32)
        cp[b] = _arr([x for pr in bal["cproofs"] for x in pr], 32).reshape(nc, 2, 32)
    gs = [O.Guardian(f"guardian{g['x']}", g["x"], [h(a) for a in g["coeffs"]], [h(k) for k in g["commitments"]])
          for g in d["guardians"]]
    return d, (nc, ns, va, spc), cts, rp, cp, gs


@pytest.mark.parametrize("mode", MODES)
def test_c_oracle_cast_only_tally_and_spoiled_plaintexts(mode):
    """The C oracle's tally of the cast ballots alone equals the fixture's (cast-only) tally, every
    ballot verifies, and each spoiled ballot's plaintext is its real selections' votes."""
    from eg_oracle_c import COracle
    G = O.production_group(mode)
    d, (nc, ns, va, spc), cts, rp, cp, gs = spoiled_case(mode)
    co = COracle(G.p, G.q, G.g)
    co.set_key(h(d["K"]))
    ok_s, ok_c, _ = co.verify_ballots(h(d["qbar"]), nc, spc, va, va, cts, rp, cp, threads=2, tally=False)
    assert ok_s.all() and ok_c.all()
    cast = np.array(d["cast"], bool)
    _, _, tally = co.verify_ballots(h(d["qbar"]), nc, spc, va, va, cts[cast], rp[cast], cp[cast], threads=2)
    assert [[t[0].tobytes().hex(), t[1].tobytes().hex()] for t in tally] == d["tally"]
    for bal, c in zip(d["ballots"], d["cast"]):
        if not c:
            assert bal["plaintext"] == [bal["votes"][k * spc + s] for k in range(nc) for s in range(ns)]
    assert K_of(gs, G) == h(d["K"])


def K_of(gs, G):
    return G.prodP([g.K for g in gs])


def test_python_oracle_reproduces_spoiled_decryption():
    """decryptBallot restated (oracle.decrypt_ballot) reproduces every share, proof, recovery key
    and plaintext of the fixture from the guardians' coefficients and the injected nonces."""
    G = O.production_group()
    d, (nc, ns, va, spc), cts, rp, cp, gs = spoiled_case()
    man = O.Manifest(nc, ns, va)
    qbar = h(d["qbar"])
    avail = [g for g in gs if g.gid in d["available"]]
    missing = [g for g in gs if g.gid in d["missing"]]
    for b, (bal, c) in enumerate(zip(d["ballots"], d["cast"])):
        if c:
            continue
        eb = O.EncryptedBallot([O.Ciphertext(h(a), h(x)) for a, x in bal["cts"]], [], [])
        plain, shares = O.decrypt_ballot(G, qbar, man, eb, avail, missing, [h(u) for u in bal["nonces"]])
        assert plain == bal["plaintext"]
        for gid, lst in shares["direct"].items():
            assert [(hex(M), hex(p.c), hex(p.v)) for M, p in lst] == \
                [(hex(h(w["M"])), hex(h(w["c"])), hex(h(w["v"]))) for w in bal["direct"][gid]]
        for l, by in shares["compensated"].items():
            for gid, lst in by.items():
                assert [(M, p.c, p.v, rk) for M, p, rk in lst] == \
                    [(h(w["M"]), h(w["c"]), h(w["v"]), h(w["recovery"])) for w in bal["compensated"][l][gid]]
