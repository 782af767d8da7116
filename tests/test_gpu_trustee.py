"""Parity of the trustee path (DecryptingTrusteeIF.directDecrypt / compensatedDecrypt,
RunRemoteDecryptingTrustee.java:189-193,227-232) and the mediator combine
(Decryption.decrypt, RunRemoteDecryptor.java:261-262) vs the oracle."""
import random

import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


def test_direct_and_compensated_shares_bitexact(group):
    from electionguard.decrypt import partial_decrypt_batch
    og = O.production_group()
    rng = random.Random(21)
    gs, K = O.key_ceremony(og, 3, 2, rng)
    qbar = rng.randrange(og.q)
    texts = [O.encrypt(og, K, rng.randrange(3), rng.randrange(1, og.q)) for _ in range(5)]
    nonces = [rng.randrange(1, og.q) for _ in texts]
    T = np.zeros((5, 2, 512), np.uint8)
    for i, ct in enumerate(texts):
        T[i, 0] = np.frombuffer(ct.pad.to_bytes(512, "big"), np.uint8)
        T[i, 1] = np.frombuffer(ct.data.to_bytes(512, "big"), np.uint8)
    N = np.stack([np.frombuffer(u.to_bytes(32, "big"), np.uint8) for u in nonces])
    want = O.direct_decrypt(og, qbar, gs[0], texts, nonces)
    M, pr = partial_decrypt_batch(group, gs[0].s, qbar, T, N)
    for i, (Mi, p) in enumerate(want):
        assert int.from_bytes(M[i].tobytes(), "big") == Mi
        assert int.from_bytes(pr[i, 0].tobytes(), "big") == p.c
        assert int.from_bytes(pr[i, 1].tobytes(), "big") == p.v
    wantc = O.compensated_decrypt(og, qbar, gs[1], gs[2], texts, nonces)
    share = O.poly_eval(gs[2].coeffs, gs[1].x, og.q)
    M2, pr2 = partial_decrypt_batch(group, share, qbar, T, N)
    for i, (Mi, p, rk) in enumerate(wantc):
        assert int.from_bytes(M2[i].tobytes(), "big") == Mi
        assert (int.from_bytes(pr2[i, 0].tobytes(), "big"), int.from_bytes(pr2[i, 1].tobytes(), "big")) == (p.c, p.v)


def test_full_threshold_decryption(group):
    """5 guardians, quorum 3, 2 missing (config C4 shape): tally counts recovered exactly."""
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.decrypt import DecryptingTrustee, Decryption
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 5, 3, seed=3)
    key = ElectionKey(group, K)
    man = Manifest(2, 3, 1)
    nr = np.random.default_rng(1)
    nb = 9
    votes = random_votes(nr, man, nb)
    qbar = 12345
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(nr, (nb, man.nsel, 4), group.q),
                          random_scalars(nr, (nb, man.n_contests), group.q))
    ok_s, ok_c, tally = Verifier(group, key, qbar, man).verify(eb)
    assert ok_s.all() and ok_c.all()
    comm = {g.gid: g.commitments for g in gk}
    avail = [DecryptingTrustee(group, g, comm) for g in gk[:3]]
    dec = Decryption(group, qbar, avail, [g.gid for g in gk[3:]], {g.gid: g.public_key for g in gk})
    counts = dec.decrypt(tally, nb)
    expected = votes.reshape(nb, man.n_contests, man.spc)[:, :, : man.n_selections].sum(axis=0).reshape(-1)
    assert counts == [int(x) for x in expected]


def test_decryption_record_verification(group):
    """Record-level decryption checks (verify_decryption_record): an honest record passes
    every check; a tampered share, recovery key, count or a missing quorum member fails
    exactly the check it should.  The tally relation B == M g^t is cross-checked with
    CPython pow on the honest record."""
    import copy
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.decrypt import (CompensatedDecryptionAndProof, DecryptingTrustee, Decryption,
                                       verify_decryption_record)
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 5, 3, seed=8)
    key = ElectionKey(group, K)
    man = Manifest(1, 3, 1)
    nr = np.random.default_rng(8)
    nb = 7
    votes = random_votes(nr, man, nb)
    qbar = 4242
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(nr, (nb, man.nsel, 4), group.q),
                          random_scalars(nr, (nb, man.n_contests), group.q))
    _, _, tally = Verifier(group, key, qbar, man).verify(eb)
    comm = {g.gid: g.commitments for g in gk}
    pks = {g.gid: g.public_key for g in gk}
    avail = [DecryptingTrustee(group, g, comm) for g in (gk[0], gk[2], gk[4])]
    rec = Decryption(group, qbar, avail, [gk[1].gid, gk[3].gid], pks).decrypt_record(tally, nb)
    expected = votes.reshape(nb, man.n_contests, man.spc)[:, :, : man.n_selections].sum(axis=0).reshape(-1)
    assert rec.counts == [int(x) for x in expected]
    assert all(verify_decryption_record(group, qbar, rec, pks, comm).values())
    # CPython cross-check of B = M g^t with M rebuilt from the record's shares
    og = O.production_group()
    xs = list(rec.xs.values())
    for i in range(len(rec.counts)):
        M = 1
        for gid, res in rec.direct.items():
            M = M * res[i].partialDecryption % og.p
        for l, by in rec.compensated.items():
            for gid, res in by.items():
                num = den = 1
                for xj in xs:
                    if xj != rec.xs[gid]:
                        num, den = num * xj % og.q, den * (xj - rec.xs[gid]) % og.q
                M = M * pow(res[i].partialDecryption, num * pow(den, -1, og.q) % og.q, og.p) % og.p
        assert M * pow(og.g, rec.counts[i], og.p) % og.p == int.from_bytes(bytes(rec.texts[i, 1]), "big")

    def check(r):
        return verify_decryption_record(group, qbar, r, pks, comm)

    bad = copy.deepcopy(rec)
    bad.counts[1] += 1
    v = check(bad)
    assert not v["tally"] and v["direct_proofs"] and v["compensated_proofs"]
    bad = copy.deepcopy(rec)
    d = bad.direct[gk[2].gid][2]
    d.partialDecryption = d.partialDecryption * og.g % og.p
    v = check(bad)
    assert not v["direct_proofs"] and not v["tally"] and v["compensated_proofs"] and v["recovery_keys"]
    bad = copy.deepcopy(rec)
    c = bad.compensated[gk[3].gid][gk[4].gid][0]
    bad.compensated[gk[3].gid][gk[4].gid][0] = CompensatedDecryptionAndProof(
        c.partialDecryption, c.proof, c.recoveredPublicKeyShare * og.g % og.p)
    v = check(bad)
    assert not v["recovery_keys"] and not v["compensated_proofs"] and v["direct_proofs"] and v["tally"]
    bad = copy.deepcopy(rec)
    del bad.compensated[gk[1].gid][gk[0].gid]
    v = check(bad)
    assert not v["quorum"] and v["direct_proofs"]


def test_verify_shares_rejects_bad_proof(group):
    from electionguard.decrypt import GenericChaumPedersenProof, verify_shares
    og = O.production_group()
    rng = random.Random(22)
    gs, K = O.key_ceremony(og, 2, 2, rng)
    qbar = rng.randrange(og.q)
    texts = [O.encrypt(og, K, 1, rng.randrange(1, og.q)) for _ in range(3)]
    res = O.direct_decrypt(og, qbar, gs[0], texts, [rng.randrange(1, og.q) for _ in texts])
    proofs = [GenericChaumPedersenProof(p.c, p.v) for _, p in res]
    proofs[1] = GenericChaumPedersenProof(proofs[1].c, (proofs[1].v + 1) % og.q)
    ok = verify_shares(group, qbar, [gs[0].K] * 3, [(t.pad, t.data) for t in texts], [m for m, _ in res], proofs)
    assert list(ok) == [True, False, True]


def test_verify_shares_large_batch_key_table(group):
    """>= 8192 shares of one trustee: eg_verify_shares switches a = g^v K_i^c to a cached
    fixed-base table of K_i; every honest proof verifies, tampered ones (c or v) fail, and a
    batch mixing two keys takes the window path with the same verdicts."""
    import ctypes
    from electionguard.ballot import random_scalars
    from electionguard.core import native
    from electionguard.core.group import p_bytes, q_bytes
    from electionguard.decrypt import partial_decrypt_batch
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 2, 2, seed=77)
    rng = np.random.default_rng(77)
    n = 8200
    R = random_scalars(rng, (n,), group.q)
    T = np.ascontiguousarray(np.stack([group.gPowP_batch(R), group.powP_batch([K] * n, R)], axis=1))
    qbar = 0xABCDEF
    M, pr = partial_decrypt_batch(group, gk[0].secret, qbar, T, random_scalars(rng, (n,), group.q))
    pr = pr.copy()
    pr[17, 1, 31] ^= 1      # v
    pr[8199, 0, 0] ^= 0x40  # c
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)

    def verify(keys):
        ok = np.zeros(n, np.uint8)
        native.check(group._lib, "eg_verify_shares",
                     group._lib.eg_verify_shares(group.handle, native.buf(q_bytes(qbar)), ptr(keys), ptr(T), ptr(M),
                                                 ptr(pr), n, ptr(ok)))
        return np.argwhere(ok == 0).reshape(-1).tolist()

    Ki = np.ascontiguousarray(np.tile(np.frombuffer(p_bytes(gk[0].public_key), np.uint8), (n, 1)))
    assert verify(Ki) == [17, 8199]   # table path
    assert verify(Ki) == [17, 8199]   # cached table
    mixed = Ki.copy()
    mixed[5] = np.frombuffer(p_bytes(gk[1].public_key), np.uint8)  # wrong key for share 5 -> window path
    assert verify(mixed) == [5, 17, 8199]


def test_share_backups_gpu_ceremony_and_trustee(group):
    """GPU key ceremony backups decrypt (oracle, CPython) to P_l(x_i); the trustee's
    share_of() opens them on the GPU; a tampered backup makes compensatedDecrypt fail."""
    from electionguard.decrypt import DecryptingTrustee
    from electionguard.keyceremony import backup_label, key_ceremony
    og = O.production_group()
    gk, K = key_ceremony(group, 4, 3, seed=91)
    for gi in gk:
        for gl in gk:
            if gl.gid == gi.gid:
                continue
            share = O.poly_eval(gl.coeffs, gi.x, og.q)
            assert O.backup_decrypt(og, gi.secret, gi.backups_from[gl.gid], backup_label(gl.gid, gi.gid)) == share
    comm = {g.gid: g.commitments for g in gk}
    t = DecryptingTrustee(group, gk[0], comm)
    assert t.share_of(gk[2].gid) == O.poly_eval(gk[2].coeffs, gk[0].x, og.q)
    c0, c1, c2 = gk[1].backups_from[gk[3].gid]
    gk[1].backups_from[gk[3].gid] = (c0, c1, bytes([c2[0] ^ 0x80]) + c2[1:])
    t1 = DecryptingTrustee(group, gk[1], comm)
    with pytest.raises(ValueError):
        t1.compensatedDecrypt(group, gk[3].gid, np.zeros((1, 2, 512), np.uint8), 5)


def test_trustee_batch_past_one_sublaunch(group):
    """More texts than one k_pow sub-launch holds (2^18 jobs): the constant-time pair jobs
    split into two sub-launches and the g^u jobs ride as the last one's second part. Every
    share proof verifies on the mediator path, and M is checked with CPython pow around the
    sub-launch boundary."""
    import ctypes
    from electionguard.ballot import random_scalars
    from electionguard.core import native
    from electionguard.core.group import p_bytes, q_bytes
    from electionguard.decrypt import partial_decrypt_batch
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 2, 2, seed=91)
    rng = np.random.default_rng(91)
    n = (1 << 18) + 1000
    R = random_scalars(rng, (n,), group.q)
    pads = group.gPowP_batch(R)
    T = np.ascontiguousarray(np.stack([pads, pads], axis=1))
    qbar = 0x5EED
    s = gk[0].secret
    M, pr = partial_decrypt_batch(group, s, qbar, T, random_scalars(rng, (n,), group.q))
    for i in (0, (1 << 18) - 1, 1 << 18, n - 1):
        P = int.from_bytes(pads[i].tobytes(), "big")
        assert int.from_bytes(M[i].tobytes(), "big") == pow(P, s, group.p), i
    ok = np.zeros(n, np.uint8)
    Ki = np.ascontiguousarray(np.tile(np.frombuffer(p_bytes(gk[0].public_key), np.uint8), (n, 1)))
    ptr = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    native.check(group._lib, "eg_verify_shares",
                 group._lib.eg_verify_shares(group.handle, native.buf(q_bytes(qbar)), ptr(Ki), ptr(T), ptr(M),
                                             ptr(pr), n, ptr(ok)))
    assert ok.all()
