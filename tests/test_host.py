"""CPU: host-side logic of the path (scalar generation, ballot layout, Lagrange, sharding)."""
import random

import numpy as np

import eg_oracle as O


def test_random_scalars_below_q():
    from electionguard.ballot import random_scalars
    rng = np.random.default_rng(3)
    q = O.Q
    s = random_scalars(rng, (1000, 4), q)
    assert s.shape == (1000, 4, 32)
    assert all(int.from_bytes(x.tobytes(), "big") < q for x in s.reshape(-1, 32))
    tiny_q = 2**255 + 12345  # forces rejections
    s2 = random_scalars(rng, (500,), tiny_q)
    assert all(int.from_bytes(x.tobytes(), "big") < tiny_q for x in s2)


def test_random_votes_one_hot_and_placeholders_zero():
    from electionguard.ballot import Manifest, random_votes
    man = Manifest(4, 5, 1)
    v = random_votes(np.random.default_rng(1), man, 200).reshape(200, 4, 6)
    assert (v.sum(axis=2) == 1).all() and (v[:, :, 5] == 0).all()


def test_manifest_shape():
    from electionguard.ballot import Manifest
    m = Manifest(4, 5, 1)
    assert (m.spc, m.nsel, m.n_real) == (6, 24, 20)


def test_lagrange_matches_oracle_and_interpolates():
    from electionguard.decrypt import lagrange
    q = O.Q
    rng = random.Random(4)
    coeffs = [rng.randrange(q) for _ in range(3)]
    xs = [1, 3, 5]
    ys = [O.poly_eval(coeffs, x, q) for x in xs]
    assert sum(lagrange(xs, x, q) * y for x, y in zip(xs, ys)) % q == coeffs[0]
    assert all(lagrange(xs, x, q) == O.lagrange(xs, x, q) for x in xs)


def test_shard_range_covers_exactly():
    from electionguard.distributed import shard_range
    for n in (0, 1, 7, 10000, 1000003):
        for w in (1, 2, 3, 8):
            spans = [shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            assert max(b - a for a, b in spans) - min(b - a for a, b in spans) <= 1


def test_tally_group_layout_matches_oracle_order():
    """accumulate_tally's (contest, selection, component) x ballots grouping."""
    from electionguard.ballot import Manifest
    man = Manifest(2, 3, 1)
    nb = 4
    cts = np.arange(nb * man.nsel * 2, dtype=np.int64).reshape(nb, man.nsel, 2)
    sel = cts.reshape(nb, man.n_contests, man.spc, 2)[:, :, : man.n_selections]
    g = np.transpose(sel, (1, 2, 3, 0)).reshape(-1, nb)
    # group (k, s, c) must hold element (b, k*spc+s, c) for every ballot b
    for k in range(2):
        for s in range(3):
            for c in range(2):
                row = g[(k * 3 + s) * 2 + c]
                assert list(row) == [cts[b, k * man.spc + s, c] for b in range(nb)]


def test_share_backup_kdf_matches_oracle():
    """The product's backup KDF/MAC (keyceremony.backup_open, host code) opens backups made by
    the oracle restatement, rejects a flipped bit and a wrong recipient (CPU only: k = c0^s by
    CPython pow)."""
    import random
    import eg_oracle as O
    from electionguard.keyceremony import backup_label, backup_open
    G = O.production_group()
    rng = random.Random(31)
    gs, _ = O.key_ceremony(G, 3, 2, rng)
    for l, i in [(0, 1), (2, 0)]:
        share = O.poly_eval(gs[l].coeffs, gs[i].x, G.q)
        label = backup_label(gs[l].gid, gs[i].gid)
        c0, c1, c2 = O.backup_encrypt(G, gs[i].K, share, rng.randrange(1, G.q), label)
        k = pow(c0, gs[i].s, G.p)
        assert backup_open(c0, k, c1, c2, label) == share
        assert O.backup_decrypt(G, gs[i].s, (c0, c1, c2), label) == share
        bad = bytes([c1[0] ^ 1]) + c1[1:]
        assert backup_open(c0, k, bad, c2, label) is None
        wrong = gs[(i + 1) % 3]
        assert backup_open(c0, pow(c0, wrong.s, G.p), c1, c2, label) is None
        assert backup_open(c0, k, c1, c2, backup_label(gs[l].gid, wrong.gid)) is None


def test_oracle_schnorr_and_backup_checks():
    """Oracle restatement of the key-ceremony proofs (CPU, CPython pow): prove -> verify,
    tampering and non-residues rejected; backup shares checked against commitments."""
    import random
    import eg_oracle as O
    G = O.production_group()
    rng = random.Random(8)
    gs, _ = O.key_ceremony(G, 3, 2, rng)
    a, K = gs[1].coeffs[1], gs[1].commitments[1]
    pr = O.schnorr_prove(G, a, K, rng.randrange(1, G.q))
    assert O.schnorr_verify(G, K, pr)
    assert not O.schnorr_verify(G, K, O.GenericProof(pr.c, (pr.v + 1) % G.q))
    assert not O.schnorr_verify(G, G.p - 1, pr)
    assert not O.schnorr_verify(G, gs[0].K, pr)
    share = O.poly_eval(gs[2].coeffs, gs[0].x, G.q)
    assert O.verify_backup_share(G, share, gs[2], gs[0].x)
    assert not O.verify_backup_share(G, share, gs[2], gs[1].x)


def test_oracle_threshold_decryption_round_trip():
    """The oracle's own threshold decryption (the checker the GPU trustee / record tests lean
    on): 4 guardians, quorum 2, guardians 2 and 4 missing.  Every share proof verifies,
    recovery keys match the compensating guardian's share, and combine() recovers the
    encrypted counts; a tampered share breaks its proof."""
    import random

    import eg_oracle as O
    G = O.production_group()
    rng = random.Random(5)
    gs, K = O.key_ceremony(G, 4, 2, rng)
    avail, missing = [gs[0], gs[2]], [gs[1], gs[3]]
    counts = [0, 3, 17]
    texts = [O.encrypt(G, K, m, rng.randrange(1, G.q)) for m in counts]
    qbar = rng.randrange(G.q)
    direct, comp = {}, {}
    for gd in avail:
        res = O.direct_decrypt(G, qbar, gd, texts, [rng.randrange(1, G.q) for _ in texts])
        assert all(O.verify_share(G, qbar, gd.K, t, M, pr) for t, (M, pr) in zip(texts, res))
        direct[gd.gid] = [M for M, _ in res]
    for gl in missing:
        comp[gl.gid] = {}
        for gd in avail:
            res = O.compensated_decrypt(G, qbar, gd, gl, texts, [rng.randrange(1, G.q) for _ in texts])
            for t, (M, pr, rk) in zip(texts, res):
                assert rk == G.gPowP(O.poly_eval(gl.coeffs, gd.x, G.q))
                assert O.verify_share(G, qbar, rk, t, M, pr)
            comp[gl.gid][gd.gid] = [M for M, _, _ in res]
    xs = {g.gid: g.x for g in avail}
    for i, t in enumerate(texts):
        got = O.combine(G, t, {g: v[i] for g, v in direct.items()},
                        {l: {g: v[i] for g, v in by.items()} for l, by in comp.items()}, xs, 20)
        assert got == counts[i]
    M, pr = O.direct_decrypt(G, qbar, avail[0], texts[:1], [7])[0]
    assert not O.verify_share(G, qbar, avail[0].K, texts[0], M * G.g % G.p, pr)
