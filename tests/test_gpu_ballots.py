"""Parity of the ballot-level path (batchEncryption / Verifier / runAccumulateBallots,
RunRemoteWorkflowTest.java:140-182) on the GPU vs the CPU oracle, with injected nonces."""
import random

import numpy as np
import pytest

import eg_oracle as O
from conftest import be2i

pytestmark = pytest.mark.gpu


def _setup(group, seed=11, n=3, quorum=2):
    from electionguard.ballot import ElectionKey
    og = O.production_group()
    rng = random.Random(seed)
    gs, K = O.key_ceremony(og, n, quorum, rng)
    qbar = rng.randrange(og.q)
    return og, rng, K, qbar, ElectionKey(group, K)


def _oracle_ballots(og, K, qbar, man_o, nb, rng):
    """Encrypt with the oracle, returning arrays in the C-ABI layout + the oracle objects."""
    spc = man_o.sel_per_contest
    nsel = man_o.sel_per_ballot
    cts = np.zeros((nb, nsel, 2, 512), np.uint8)
    rp = np.zeros((nb, nsel, 4, 32), np.uint8)
    cp = np.zeros((nb, man_o.n_contests, 2, 32), np.uint8)
    obs = []
    for b in range(nb):
        votes = O.ballot_plaintexts(man_o, rng)
        eb = O.encrypt_ballot(og, K, qbar, man_o, votes, rng)
        obs.append((votes, eb))
        for i, (ct, pr) in enumerate(zip(eb.cts, eb.proofs)):
            cts[b, i, 0] = np.frombuffer(ct.pad.to_bytes(512, "big"), np.uint8)
            cts[b, i, 1] = np.frombuffer(ct.data.to_bytes(512, "big"), np.uint8)
            for k, v in enumerate((pr.c0, pr.v0, pr.c1, pr.v1)):
                rp[b, i, k] = np.frombuffer(v.to_bytes(32, "big"), np.uint8)
        for c, pr in enumerate(eb.contest_proofs):
            cp[b, c, 0] = np.frombuffer(pr.c.to_bytes(32, "big"), np.uint8)
            cp[b, c, 1] = np.frombuffer(pr.v.to_bytes(32, "big"), np.uint8)
    return cts, rp, cp, obs


def test_verify_oracle_ballots_and_tally(group):
    from electionguard.ballot import EncryptedBallots, Manifest, Verifier
    og, rng, K, qbar, key = _setup(group)
    man = Manifest(2, 3, 1)
    man_o = O.Manifest(2, 3, 1)
    cts, rp, cp, obs = _oracle_ballots(og, K, qbar, man_o, 3, rng)
    v = Verifier(group, key, qbar, man)
    ok_s, ok_c, tally = v.verify(EncryptedBallots(cts, rp, cp))
    assert ok_s.all() and ok_c.all()
    want = O.accumulate_tally(og, man_o, [eb for _, eb in obs])
    for s, ct in enumerate(want):
        assert be2i(tally[s, 0]) == ct.pad and be2i(tally[s, 1]) == ct.data, s


def test_verify_rejects_tampering(group):
    from electionguard.ballot import EncryptedBallots, Manifest, Verifier
    og, rng, K, qbar, key = _setup(group, seed=12)
    man = Manifest(1, 2, 1)
    cts, rp, cp, _ = _oracle_ballots(og, K, qbar, O.Manifest(1, 2, 1), 2, rng)
    rp2 = rp.copy()
    rp2[0, 1, 3, 31] ^= 1          # v1 of selection 1, ballot 0
    cp2 = cp.copy()
    cp2[1, 0, 1, 5] ^= 0x10         # contest response, ballot 1
    cts2 = cts.copy()
    cts2[1, 2, 1] = 0xFF            # data >= p (range check), ballot 1 selection 2
    v = Verifier(group, key, qbar, man)
    ok_s, ok_c, _ = v.verify(EncryptedBallots(cts2, rp2, cp2))
    assert not ok_s[0, 1] and ok_s[0, 0] and ok_s[0, 2]
    assert not ok_s[1, 2] and ok_s[1, 0]
    assert ok_c[0, 0] and not ok_c[1, 0]


def test_encrypt_bitexact_vs_oracle(group):
    """GPU batchEncryption with the oracle's injected nonces reproduces its bytes exactly."""
    from electionguard.ballot import Manifest, batch_encryption
    og, rng, K, qbar, key = _setup(group, seed=13)
    man = Manifest(2, 2, 1)
    man_o = O.Manifest(2, 2, 1)
    nb = 2
    votes = np.zeros((nb, man.nsel), np.uint8)
    sn = np.zeros((nb, man.nsel, 4, 32), np.uint8)
    cn = np.zeros((nb, man.n_contests, 32), np.uint8)
    expect = []
    for b in range(nb):
        vts = O.ballot_plaintexts(man_o, rng)
        votes[b] = vts
        # replay the oracle's nonce draws
        state = rng.getstate()
        eb = O.encrypt_ballot(og, K, qbar, man_o, vts, rng)
        rng2 = random.Random()
        rng2.setstate(state)
        for c in range(man.n_contests):
            for s in range(man.spc):
                i = c * man.spc + s
                R = rng2.randrange(1, og.q)
                u, cf, vf = rng2.randrange(1, og.q), rng2.randrange(og.q), rng2.randrange(og.q)
                for k, x in enumerate((R, u, cf, vf)):
                    sn[b, i, k] = np.frombuffer(x.to_bytes(32, "big"), np.uint8)
            cn[b, c] = np.frombuffer(rng2.randrange(1, og.q).to_bytes(32, "big"), np.uint8)
        expect.append(eb)
    got = batch_encryption(group, key, qbar, man, votes, sn, cn)
    for b, eb in enumerate(expect):
        for i, (ct, pr) in enumerate(zip(eb.cts, eb.proofs)):
            assert be2i(got.cts[b, i, 0]) == ct.pad and be2i(got.cts[b, i, 1]) == ct.data, (b, i)
            assert [be2i(got.rproof[b, i, k]) for k in range(4)] == [pr.c0, pr.v0, pr.c1, pr.v1], (b, i)
        for c, pr in enumerate(eb.contest_proofs):
            assert be2i(got.cproof[b, c, 0]) == pr.c and be2i(got.cproof[b, c, 1]) == pr.v, (b, c)


def test_encrypt_verify_roundtrip_random(group):
    from electionguard.ballot import Manifest, Verifier, batch_encryption, random_scalars, random_votes
    og, rng, K, qbar, key = _setup(group, seed=14)
    man = Manifest(4, 5, 1)
    nr = np.random.default_rng(0)
    nb = 37
    votes = random_votes(nr, man, nb)
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(nr, (nb, man.nsel, 4), og.q),
                          random_scalars(nr, (nb, man.n_contests), og.q))
    ok_s, ok_c, tally = Verifier(group, key, qbar, man).verify(eb)
    assert ok_s.all() and ok_c.all()
    # spot-check one ballot with the oracle verifier
    b = 17
    from conftest import be2i as I
    cts = [O.Ciphertext(I(eb.cts[b, i, 0]), I(eb.cts[b, i, 1])) for i in range(man.nsel)]
    prs = [O.RangeProof(*[I(eb.rproof[b, i, k]) for k in range(4)]) for i in range(man.nsel)]
    cps = [O.GenericProof(I(eb.cproof[b, c, 0]), I(eb.cproof[b, c, 1])) for c in range(man.n_contests)]
    assert O.verify_ballot(og, K, qbar, O.Manifest(4, 5, 1), O.EncryptedBallot(cts, prs, cps))


def test_window_path_context_matches_comb(group, monkeypatch):
    """EG_NO_COMB=1 (read at context creation) runs the gathered contest jobs and the trustee
    shares through the 4-bit fixed-window programs instead of the Lim-Lee comb: a second
    context built that way must give the same verdicts, tally, tamper flags and trustee
    shares as the default one (and the oracle's tally)."""
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
    from electionguard.core import GroupContext
    from electionguard.decrypt import partial_decrypt_batch
    og, rng, K, qbar, key = _setup(group, seed=41)
    man = Manifest(2, 3, 1)
    cts, rp, cp, obs = _oracle_ballots(og, K, qbar, O.Manifest(2, 3, 1), 5, rng)
    eb = EncryptedBallots(cts, rp, cp)
    monkeypatch.setenv("EG_NO_COMB", "1")
    g2 = GroupContext(group.p, group.q, group.g, device=group.device)
    monkeypatch.delenv("EG_NO_COMB")
    try:
        key2 = ElectionKey(g2, K)
        s1, c1, t1 = Verifier(group, key, qbar, man).verify(eb)
        s2, c2, t2 = Verifier(g2, key2, qbar, man).verify(eb)
        assert s1.all() and c1.all() and (s2 == s1).all() and (c2 == c1).all() and (t2 == t1).all()
        want = O.accumulate_tally(og, O.Manifest(2, 3, 1), [e for _, e in obs])
        for s, ct in enumerate(want):
            assert be2i(t2[s, 0]) == ct.pad and be2i(t2[s, 1]) == ct.data, s
        cp2 = cp.copy()
        cp2[3, 1, 1, 7] ^= 0x40
        s3, c3, _ = Verifier(g2, key2, qbar, man).verify(EncryptedBallots(cts, rp, cp2), with_tally=False)
        assert s3.all() and np.argwhere(~c3).tolist() == [[3, 1]]
        texts = np.ascontiguousarray(cts[:, :, :, :].reshape(-1, 2, 512)[:7])
        secret = rng.randrange(og.q)
        nonces = np.stack([np.frombuffer(rng.randrange(og.q).to_bytes(32, "big"), np.uint8) for _ in range(7)])
        Ma, pa = partial_decrypt_batch(group, secret, qbar, texts, nonces)
        Mb, pb = partial_decrypt_batch(g2, secret, qbar, texts, nonces)
        assert np.array_equal(Ma, Mb) and np.array_equal(pa, pb)
        for i in range(7):
            assert be2i(Ma[i]) == pow(be2i(texts[i, 0]), secret, og.p)
    finally:
        g2.close()
