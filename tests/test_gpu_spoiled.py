"""GPU: spoiled ballots (RunRemoteDecryptor.java:264-269) and the cast-only tally.

* golden (tests/golden/<mode>/spoiled.json, from oracle.decrypt_ballot): the fused verifier with a
  cast mask verifies all 4 ballots and tallies only the 2 cast ones, bit-exact; the GPU trustees
  reproduce every direct and compensated share of the spoiled ballots byte for byte with the
  fixture's injected nonces; Decryption.decryptBallots returns the plaintexts;
* a GPU-encrypted mixed batch (5 guardians, quorum 3, 2 missing): host and device verify with the
  same mask give the same tally, equal to the C oracle's tally of the cast subset, and every
  spoiled ballot decrypts to its exact votes; the record of the spoiled decryption verifies.
The gRPC path (trustees as processes) is tests/test_gpu_workflow.py with -nspoiled."""
import json
from pathlib import Path

import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def h(x):
    return int(x, 16)


def _arr(hexes, n):
    return np.stack([np.frombuffer(bytes.fromhex(x), np.uint8) for x in hexes]).reshape(-1, n)


@pytest.fixture(params=[O.MODE4096, O.MODE4096_V2])
def case(request):
    from electionguard.core import productionGroup
    mode = request.param
    return productionGroup(0, mode), json.loads((GOLD / mode / "spoiled.json").read_text())


def test_golden_cast_mask_and_spoiled_shares(case):
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
    from electionguard.decrypt import DecryptingTrustee, Decryption, spoiled_texts
    from electionguard.keyceremony import GuardianKeys, poly_eval
    G, d = case
    nc, ns, va = d["manifest"]
    man = Manifest(nc, ns, va)
    nb = len(d["ballots"])
    cts = np.stack([_arr([x for ct in b["cts"] for x in ct], 512).reshape(man.nsel, 2, 512) for b in d["ballots"]])
    rp = np.stack([_arr([x for pr in b["rproofs"] for x in pr], 32).reshape(man.nsel, 4, 32) for b in d["ballots"]])
    cp = np.stack([_arr([x for pr in b["cproofs"] for x in pr], 32).reshape(nc, 2, 32) for b in d["ballots"]])
    cast = np.array(d["cast"], bool)
    qbar = h(d["qbar"])
    key = ElectionKey(G, h(d["K"]))
    ok_s, ok_c, tally = Verifier(G, key, qbar, man).verify(EncryptedBallots(cts, rp, cp), cast=cast)
    assert ok_s.all() and ok_c.all()
    assert [[t[0].tobytes().hex(), t[1].tobytes().hex()] for t in tally] == d["tally"]
    # all cast, and none cast, around it
    _, _, t_all = Verifier(G, key, qbar, man).verify(EncryptedBallots(cts, rp, cp))
    assert [[t[0].tobytes().hex(), t[1].tobytes().hex()] for t in t_all] != d["tally"]
    _, _, t_none = Verifier(G, key, qbar, man).verify(EncryptedBallots(cts, rp, cp), cast=np.zeros(nb, bool))
    assert all(int.from_bytes(t.tobytes(), "big") == 1 for t in t_none.reshape(-1, 512))
    # trustees from the fixture's coefficients: every share byte-exact with the injected nonces
    gs = [GuardianKeys(f"guardian{g['x']}", g["x"], [h(a) for a in g["coeffs"]], [h(k) for k in g["commitments"]])
          for g in d["guardians"]]
    for gi in gs:
        for gl in gs:
            if gl.gid != gi.gid:
                gi.shares_from[gl.gid] = poly_eval(gl.coeffs, gi.x, G.q)
    comm = {g.gid: g.commitments for g in gs}
    avail = [DecryptingTrustee(G, g, comm) for g in gs if g.gid in d["available"]]
    missing = [g.gid for g in gs if g.gid in d["missing"]]
    spoiled = [b for b, c in zip(d["ballots"], d["cast"]) if not c]
    sp_cts = cts[~cast]
    for b, bal in enumerate(spoiled):
        T = spoiled_texts(man, sp_cts[b:b + 1])
        nonces = iter(h(u) for u in bal["nonces"])
        for tr in avail:
            res = tr.directDecrypt(G, T, qbar, [next(nonces) for _ in range(len(T))])
            assert [(r.partialDecryption, r.proof.c, r.proof.v) for r in res] == \
                [(h(w["M"]), h(w["c"]), h(w["v"])) for w in bal["direct"][tr.id()]]
        for l in missing:
            for tr in avail:
                res = tr.compensatedDecrypt(G, l, T, qbar, [next(nonces) for _ in range(len(T))])
                assert [(r.partialDecryption, r.proof.c, r.proof.v, r.recoveredPublicKeyShare) for r in res] == \
                    [(h(w["M"]), h(w["c"]), h(w["v"]), h(w["recovery"])) for w in bal["compensated"][l][tr.id()]]
    dec = Decryption(G, qbar, avail, missing, {g.gid: g.public_key for g in gs})
    plain = dec.decryptBallots(sp_cts, man)
    assert plain.tolist() == [bal["plaintext"] for bal in spoiled]
    assert dec.decryptBallot(sp_cts[1], man) == spoiled[1]["plaintext"]


def test_mixed_batch_cast_tally_and_spoiled_decryption(group):
    from electionguard.ballot import (ElectionKey, EncryptedBallots, Manifest, Verifier, accumulate_tally,
                                      batch_encryption, random_scalars, random_votes)
    from electionguard.decrypt import DecryptingTrustee, Decryption, verify_decryption_record
    from electionguard.keyceremony import key_ceremony
    from eg_oracle_c import COracle
    man = Manifest(3, 4, 1)
    nb = 301
    gk, K = key_ceremony(group, 5, 3, seed=41)
    key = ElectionKey(group, K)
    rng = np.random.default_rng(41)
    votes = random_votes(rng, man, nb)
    qbar = 0x5B01ED
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), group.q),
                          random_scalars(rng, (nb, man.n_contests), group.q))
    cast = rng.random(nb) > 0.3
    cast[:2] = (False, True)
    V = Verifier(group, key, qbar, man)
    ok_s, ok_c, tally = V.verify(eb, cast=cast)
    assert ok_s.all() and ok_c.all()
    # C oracle over the cast subset, and the GPU tally helper with the same mask
    co = COracle(group.p, group.q, group.g)
    co.set_key(K)
    _, _, want = co.verify_ballots(qbar, man.n_contests, man.spc, 1, 1, eb.cts[cast], eb.rproof[cast], eb.cproof[cast],
                                   threads=4)
    assert np.array_equal(tally, want)
    assert np.array_equal(accumulate_tally(group, man, eb, cast), want)
    # device path with a device mask: same verdicts and tally
    d = [group.to_device(np.ascontiguousarray(x)) for x in (eb.cts, eb.rproof, eb.cproof)]
    dmask = group.to_device(cast.astype(np.uint8))
    oks = group.device_zeros((nb, man.nsel))
    okc = group.device_zeros((nb, man.n_contests))
    tal = group.device_zeros((man.n_real, 2, 512))
    V.verify_device(d[0].ptr, d[1].ptr, d[2].ptr, nb, oks.ptr, okc.ptr,
                    tal.ptr, dmask.ptr)
    group.sync()
    assert group.all_nonzero(oks) and group.all_nonzero(okc) and np.array_equal(tal.download(), want)
    # the tally decrypts to the cast votes; the spoiled ballots to their own votes
    comm = {g.gid: g.commitments for g in gk}
    avail = [DecryptingTrustee(group, g, comm) for g in gk[:3]]
    dec = Decryption(group, qbar, avail, [g.gid for g in gk[3:]], {g.gid: g.public_key for g in gk})
    real = votes.reshape(nb, man.n_contests, man.spc)[:, :, : man.n_selections].reshape(nb, man.n_real)
    assert dec.decrypt(tally, nb) == [int(x) for x in real[cast].sum(axis=0)]
    spoiled = EncryptedBallots(eb.cts[~cast], eb.rproof[~cast], eb.cproof[~cast])
    rec = dec.decrypt_ballots_record(spoiled, man)
    assert np.array_equal(np.array(rec.counts).reshape(-1, man.n_real), real[~cast])
    checks = verify_decryption_record(group, qbar, rec, {g.gid: g.public_key for g in gk}, comm,
                                      guardian_xs={g.gid: g.x for g in gk}, quorum=3, max_count=man.votes_allowed)
    assert all(checks.values()), checks
