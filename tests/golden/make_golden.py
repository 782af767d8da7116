"""Generate the committed golden fixtures from the CPU oracle (oracle/eg_oracle.py).

The reference (JohnLCaron/electionguard-remote) holds no fixtures or known-answer tests
for this path and its arithmetic dependency cannot run here, so these
vectors are produced by the oracle restatement and cross-checked against the
independent OpenSSL-BN restatement (oracle/eg_oracle_c.c) by tests/test_oracle_golden.py.
Both production groups get a full set (tests/golden/<ProductionMode>/*.json):
Mode4096 (EG 1.0, the reference's group) and Mode4096_V2 (EG 2.0, named option).
Run:  python tests/golden/make_golden.py   (deterministic; seeds below)
"""
import json
import random
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent / "oracle"))
import eg_oracle as O  # noqa: E402


def hx(x, n):
    return int(x).to_bytes(n, "big").hex()


def group_ops(G):
    rng = random.Random(101)
    p, q = G.p, G.q
    bases = [0, 0, 1, p - 1, p, p + 1, 2**4096 - 1, G.g] + [rng.randrange(2**4096) for _ in range(40)]
    exps = [0, 7, 2**256 - 1, 2, 3, q - 1, q, 1] + [rng.randrange(2**256) for _ in range(40)]
    powp = [{"b": hx(b, 512), "e": hx(e, 32), "r": hx(G.powP(b, e), 512)} for b, e in zip(bases, exps)]
    gexps = [0, 1, q - 1, 2**256 - 1] + [rng.randrange(q) for _ in range(28)]
    gpow = [{"e": hx(e, 32), "r": hx(G.gPowP(e), 512)} for e in gexps]
    mul = []
    for _ in range(24):
        a, b = rng.randrange(2**4096), rng.randrange(2**4096)
        mul.append({"a": hx(a, 512), "b": hx(b, 512), "r": hx(G.multP(a, b), 512)})
    inv = []
    for x in [1, 2, p - 1] + [rng.randrange(1, p) for _ in range(5)]:
        inv.append({"a": hx(x, 512), "r": hx(G.multInv(x), 512)})
    prods = []
    for length in (1, 5, 33):
        xs = [rng.randrange(p) for _ in range(length)]
        prods.append({"xs": [hx(x, 512) for x in xs], "r": hx(G.prodP(xs), 512)})
    return {"powP": powp, "gPowP": gpow, "multP": mul, "multInv": inv, "prodP": prods}


def ballots(G):
    rng = random.Random(202)
    gs, K = O.key_ceremony(G, 3, 2, rng)
    qbar = rng.randrange(G.q)
    man = O.Manifest(2, 3, 1)
    out = {"K": hx(K, 512), "qbar": hx(qbar, 32), "manifest": [2, 3, 1], "ballots": []}
    ebs = []
    for b in range(3):
        votes = O.ballot_plaintexts(man, rng)
        state = rng.getstate()
        eb = O.encrypt_ballot(G, K, qbar, man, votes, rng)
        r2 = random.Random()
        r2.setstate(state)
        nonces, cnonces = [], []
        for c in range(man.n_contests):
            for s in range(man.sel_per_contest):
                nonces.append([hx(r2.randrange(1, G.q), 32)] + [hx(r2.randrange(1, G.q), 32)] +
                              [hx(r2.randrange(G.q), 32), hx(r2.randrange(G.q), 32)])
            cnonces.append(hx(r2.randrange(1, G.q), 32))
        ebs.append(eb)
        out["ballots"].append({
            "votes": votes, "nonces": nonces, "contest_nonces": cnonces,
            "cts": [[hx(ct.pad, 512), hx(ct.data, 512)] for ct in eb.cts],
            "rproofs": [[hx(v, 32) for v in (pr.c0, pr.v0, pr.c1, pr.v1)] for pr in eb.proofs],
            "cproofs": [[hx(pr.c, 32), hx(pr.v, 32)] for pr in eb.contest_proofs],
            "valid": O.verify_ballot(G, K, qbar, man, eb),
        })
    tally = O.accumulate_tally(G, man, ebs)
    out["tally"] = [[hx(ct.pad, 512), hx(ct.data, 512)] for ct in tally]
    return out


def trustee(G):
    rng = random.Random(303)
    gs, K = O.key_ceremony(G, 3, 2, rng)
    qbar = rng.randrange(G.q)
    texts = [O.encrypt(G, K, rng.randrange(4), rng.randrange(1, G.q)) for _ in range(4)]
    nonces = [rng.randrange(1, G.q) for _ in texts]
    d = O.direct_decrypt(G, qbar, gs[0], texts, nonces)
    c = O.compensated_decrypt(G, qbar, gs[1], gs[2], texts, nonces)
    return {
        "qbar": hx(qbar, 32),
        "guardians": [{"x": g.x, "coeffs": [hx(a, 32) for a in g.coeffs],
                       "commitments": [hx(k, 512) for k in g.commitments]} for g in gs],
        "texts": [[hx(t.pad, 512), hx(t.data, 512)] for t in texts],
        "nonces": [hx(u, 32) for u in nonces],
        "direct": [{"M": hx(M, 512), "c": hx(p.c, 32), "v": hx(p.v, 32)} for M, p in d],
        "compensated_by_x2_for_x3": [{"M": hx(M, 512), "c": hx(p.c, 32), "v": hx(p.v, 32),
                                       "recovery": hx(rk, 512)} for M, p, rk in c],
    }


def spoiled(G):
    """Cast / spoiled ballots (RunRemoteDecryptor.java:264-269): 5 guardians, quorum 3, guardians
    4 and 5 missing; 4 ballots of which 1 and 3 are spoiled.  The tally covers the cast ballots
    only; each spoiled ballot is decrypted selection by selection with injected proof nonces."""
    rng = random.Random(404)
    gs, K = O.key_ceremony(G, 5, 3, rng)
    qbar = rng.randrange(G.q)
    man = O.Manifest(2, 3, 1)
    cast = [True, False, True, False]
    ebs, votes_all = [], []
    for _ in cast:
        votes = O.ballot_plaintexts(man, rng)
        votes_all.append(votes)
        ebs.append(O.encrypt_ballot(G, K, qbar, man, votes, rng))
    tally = O.accumulate_tally(G, man, ebs, cast)
    avail, missing = gs[:3], gs[3:]
    n_real = man.n_contests * man.n_selections
    out = {"K": hx(K, 512), "qbar": hx(qbar, 32), "manifest": [2, 3, 1], "cast": cast,
           "guardians": [{"x": g.x, "coeffs": [hx(a, 32) for a in g.coeffs],
                          "commitments": [hx(k, 512) for k in g.commitments]} for g in gs],
           "available": [g.gid for g in avail], "missing": [g.gid for g in missing],
           "ballots": [], "tally": [[hx(ct.pad, 512), hx(ct.data, 512)] for ct in tally]}
    for eb, votes, c in zip(ebs, votes_all, cast):
        b = {"votes": votes, "cts": [[hx(ct.pad, 512), hx(ct.data, 512)] for ct in eb.cts],
             "rproofs": [[hx(v, 32) for v in (pr.c0, pr.v0, pr.c1, pr.v1)] for pr in eb.proofs],
             "cproofs": [[hx(pr.c, 32), hx(pr.v, 32)] for pr in eb.contest_proofs]}
        if not c:
            nonces = [rng.randrange(1, G.q) for _ in range(n_real * (len(avail) + len(avail) * len(missing)))]
            plain, shares = O.decrypt_ballot(G, qbar, man, eb, avail, missing, nonces)
            b["nonces"] = [hx(u, 32) for u in nonces]
            b["plaintext"] = plain
            b["direct"] = {gid: [{"M": hx(M, 512), "c": hx(p.c, 32), "v": hx(p.v, 32)} for M, p in d]
                           for gid, d in shares["direct"].items()}
            b["compensated"] = {l: {gid: [{"M": hx(M, 512), "c": hx(p.c, 32), "v": hx(p.v, 32), "recovery": hx(rk, 512)}
                                          for M, p, rk in d] for gid, d in by.items()}
                                for l, by in shares["compensated"].items()}
        out["ballots"].append(b)
    return out


def proof_formats(G):
    """Every unpinned proof convention (eg_ctx_set_proof_format): the response sign x the challenge
    pre-image order.  The same key, ballots, nonces and trustee texts under each variant (so the
    variants differ only in proof bytes): 2 ballots of 2 x (2 + 1) and 3 texts' direct and
    compensated shares (2 of 3 guardians available)."""
    rng = random.Random(505)
    gs, K = O.key_ceremony(G, 3, 2, rng)
    qbar = rng.randrange(G.q)
    man = O.Manifest(2, 2, 1)
    plan = []
    for _ in range(2):
        votes = O.ballot_plaintexts(man, rng)
        plan.append((votes, rng.getstate()))
        O.encrypt_ballot(G, K, qbar, man, votes, rng)  # advance rng past this ballot's nonces
    texts = [O.encrypt(G, K, rng.randrange(4), rng.randrange(1, G.q)) for _ in range(3)]
    nonces = [rng.randrange(1, G.q) for _ in texts]
    out = {"K": hx(K, 512), "qbar": hx(qbar, 32), "manifest": [2, 2, 1],
           "guardians": [{"x": g.x, "coeffs": [hx(a, 32) for a in g.coeffs],
                          "commitments": [hx(k, 512) for k in g.commitments]} for g in gs],
           "texts": [[hx(t.pad, 512), hx(t.data, 512)] for t in texts], "nonces": [hx(u, 32) for u in nonces],
           "variants": []}
    for resp in O.RESPONSES:
        for pre in O.PREIMAGES:
            with O.proof_format(resp, pre):
                v = {"response": resp, "preimage": pre, "ballots": []}
                for votes, state in plan:
                    r = random.Random()
                    r.setstate(state)
                    eb = O.encrypt_ballot(G, K, qbar, man, votes, r)
                    r2 = random.Random()
                    r2.setstate(state)
                    nonces4, cnonces = [], []
                    for c in range(man.n_contests):
                        for s in range(man.sel_per_contest):
                            nonces4.append([hx(r2.randrange(1, G.q), 32)] + [hx(r2.randrange(1, G.q), 32)] +
                                           [hx(r2.randrange(G.q), 32), hx(r2.randrange(G.q), 32)])
                        cnonces.append(hx(r2.randrange(1, G.q), 32))
                    assert O.verify_ballot(G, K, qbar, man, eb)
                    v["ballots"].append({
                        "votes": votes, "nonces": nonces4, "contest_nonces": cnonces,
                        "cts": [[hx(ct.pad, 512), hx(ct.data, 512)] for ct in eb.cts],
                        "rproofs": [[hx(x, 32) for x in (pr.c0, pr.v0, pr.c1, pr.v1)] for pr in eb.proofs],
                        "cproofs": [[hx(pr.c, 32), hx(pr.v, 32)] for pr in eb.contest_proofs]})
                d = O.direct_decrypt(G, qbar, gs[0], texts, nonces)
                c = O.compensated_decrypt(G, qbar, gs[1], gs[2], texts, nonces)
                assert all(O.verify_share(G, qbar, gs[0].K, t, M, p) for t, (M, p) in zip(texts, d))
                assert all(O.verify_share(G, qbar, rk, t, M, p) for t, (M, p, rk) in zip(texts, c))
                v["direct"] = [{"M": hx(M, 512), "c": hx(p.c, 32), "v": hx(p.v, 32)} for M, p in d]
                v["compensated_by_x2_for_x3"] = [{"M": hx(M, 512), "c": hx(p.c, 32), "v": hx(p.v, 32),
                                                  "recovery": hx(rk, 512)} for M, p, rk in c]
                out["variants"].append(v)
    return out


if __name__ == "__main__" and sys.argv[1:] == ["--proof-formats"]:
    G = O.production_group(O.MODE4096)
    (HERE / O.MODE4096 / "proof_formats.json").write_text(json.dumps(proof_formats(G), indent=0))
    print("written proof_formats.json")
elif __name__ == "__main__":
    for mode in (O.MODE4096, O.MODE4096_V2):
        out = HERE / mode
        out.mkdir(exist_ok=True)
        G = O.production_group(mode)
        (out / "group_ops.json").write_text(json.dumps(group_ops(G), indent=0))
        (out / "ballots.json").write_text(json.dumps(ballots(G), indent=0))
        (out / "trustee.json").write_text(json.dumps(trustee(G), indent=0))
        (out / "spoiled.json").write_text(json.dumps(spoiled(G), indent=0))
        if mode == O.MODE4096:
            (out / "proof_formats.json").write_text(json.dumps(proof_formats(G), indent=0))
        p, q, g, r = O.derive_group(mode)
        (out / "constants.json").write_text(json.dumps({"mode": mode, "p": hx(p, 512), "q": hx(q, 32),
                                                        "g": hx(g, 512), "r": hx(r, 512)}, indent=0))
    print("written")
