"""GPU: the switchable Fiat-Shamir pre-image (eg_ctx_set_hash_format).  Upstream's hex form is
unpinned, so both candidates are bit-exact against the oracle: ballots made by
the oracle under the minimal-length form verify on the GPU under that form and NOT under the
fixed-width one, the GPU encryptor reproduces them byte for byte, and trustee shares match."""
import random

import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


def _arrays(ebs):
    b = lambda x, n: np.frombuffer(int(x).to_bytes(n, "big"), np.uint8)
    cts = np.stack([np.stack([np.stack([b(ct.pad, 512), b(ct.data, 512)]) for ct in eb.cts]) for eb in ebs])
    rp = np.stack([np.stack([np.stack([b(v, 32) for v in (pr.c0, pr.v0, pr.c1, pr.v1)]) for pr in eb.proofs])
                   for eb in ebs])
    cp = np.stack([np.stack([np.stack([b(pr.c, 32), b(pr.v, 32)]) for pr in eb.contest_proofs]) for eb in ebs])
    return cts, rp, cp


def test_minimal_hash_format_end_to_end(group):
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier, batch_encryption
    from electionguard.decrypt import partial_decrypt_batch
    G = O.production_group()
    rng = random.Random(71)
    gs, K = O.key_ceremony(G, 2, 2, rng)
    # a qbar with leading zero bytes, so the two forms really differ in length
    qbar = rng.randrange(2**200)
    man_o, man = O.Manifest(2, 3, 1), Manifest(2, 3, 1)
    with O.hash_format("minimal"):
        states, ebs, votes = [], [], []
        for _ in range(3):
            v = O.ballot_plaintexts(man_o, rng)
            states.append(rng.getstate())
            ebs.append(O.encrypt_ballot(G, K, qbar, man_o, v, rng))
            votes.append(v)
        assert all(O.verify_ballot(G, K, qbar, man_o, eb) for eb in ebs)
        texts = [O.encrypt(G, K, 1, rng.randrange(1, G.q)) for _ in range(4)]
        nonces = [rng.randrange(1, G.q) for _ in texts]
        want_shares = O.direct_decrypt(G, qbar, gs[0], texts, nonces)
    with O.hash_format("fixed"):
        assert not any(O.verify_ballot(G, K, qbar, man_o, eb) for eb in ebs)
    cts, rp, cp = _arrays(ebs)
    key = ElectionKey(group, K)
    V = Verifier(group, key, qbar, man)
    try:
        group.hash_format = "minimal"
        ok_s, ok_c, _ = V.verify(EncryptedBallots(cts, rp, cp))
        assert ok_s.all() and ok_c.all()
        # the GPU encryptor under the same injected nonces reproduces the oracle's bytes
        sn, cn = [], []
        for st in states:
            r2 = random.Random()
            r2.setstate(st)
            s4, c1 = [], []
            for c in range(man_o.n_contests):
                for s in range(man_o.sel_per_contest):
                    s4.append([r2.randrange(1, G.q), r2.randrange(1, G.q), r2.randrange(G.q), r2.randrange(G.q)])
                c1.append(r2.randrange(1, G.q))
            sn.append(s4)
            cn.append(c1)
        to = lambda xs: np.frombuffer(b"".join(int(x).to_bytes(32, "big") for x in xs), np.uint8)
        SN = np.stack([to([x for s4 in b for x in s4]).reshape(-1, 4, 32) for b in sn])
        CN = np.stack([to(b).reshape(-1, 32) for b in cn])
        eb = batch_encryption(group, key, qbar, man, np.array(votes, np.uint8), SN, CN)
        assert np.array_equal(eb.cts, cts) and np.array_equal(eb.rproof, rp) and np.array_equal(eb.cproof, cp)
        T = np.stack([np.stack([np.frombuffer(t.pad.to_bytes(512, "big"), np.uint8),
                                np.frombuffer(t.data.to_bytes(512, "big"), np.uint8)]) for t in texts])
        N = np.stack([np.frombuffer(u.to_bytes(32, "big"), np.uint8) for u in nonces])
        M, pr = partial_decrypt_batch(group, gs[0].s, qbar, T, N)
        for i, (Mw, pw) in enumerate(want_shares):
            assert int.from_bytes(M[i].tobytes(), "big") == Mw
            assert (int.from_bytes(pr[i, 0].tobytes(), "big"), int.from_bytes(pr[i, 1].tobytes(), "big")) == (pw.c, pw.v)
        group.hash_format = "fixed"
        ok_s, ok_c, _ = V.verify(EncryptedBallots(cts, rp, cp))
        assert not ok_s.any() and not ok_c.any()
    finally:
        group.hash_format = "fixed"
