"""GPU: the launch-splitting paths of the fused verifier (eg_capi_ballot.inc / launch_pow).

* > 2^18 selection jobs in one chunk: k_pow is split into sub-launches and the gathered
  contest-A jobs ride in the LAST sub-launch of the beta jobs (PowPart tail);
* > 16384 ballots: two verify chunks, the running tally is combined across chunks.
Both must give every verdict valid and a tally equal to the product of all ballots'
ciphertexts (checked against the independent C oracle / CPython products); a tampered
proof in the second sub-launch / second chunk must be flagged exactly.
"""
import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


def _encrypt(group, man, nb, seed):
    from electionguard.ballot import ElectionKey, batch_encryption, random_scalars, random_votes
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 3, 3, seed=seed)
    key = ElectionKey(group, K, window_bits=12)
    rng = np.random.default_rng(seed)
    votes = random_votes(rng, man, nb)
    qbar = 777 + seed
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), group.q),
                          random_scalars(rng, (nb, man.n_contests), group.q))
    return key, K, qbar, eb


def _tally_products(man, eb):
    p = O.production_group().p
    out = np.zeros((man.n_real, 2, 512), np.uint8)
    for s in range(man.n_real):
        k, r = divmod(s, man.n_selections)
        i = k * man.spc + r
        for c in range(2):
            acc = 1
            col = eb.cts[:, i, c]
            for b in range(eb.n):
                acc = acc * int.from_bytes(col[b].tobytes(), "big") % p
            out[s, c] = np.frombuffer(acc.to_bytes(512, "big"), np.uint8)
    return out


def test_split_sublaunches_with_contest_tail(group):
    from electionguard.ballot import EncryptedBallots, Manifest, Verifier
    man = Manifest(4, 5, 1)
    nb = 11000  # 264,000 selection jobs > 2^18 -> two k_pow sub-launches per job type
    key, K, qbar, eb = _encrypt(group, man, nb, 31)
    V = Verifier(group, key, qbar, man)
    ok_s, ok_c, tally = V.verify(eb)
    assert ok_s.all() and ok_c.all()
    assert np.array_equal(tally, _tally_products(man, eb))
    # tamper: a selection proof in the second sub-launch and a contest proof near the end
    rp, cp = eb.rproof.copy(), eb.cproof.copy()
    rp[10990, 3, 1, 0] ^= 0x80   # job 10990*24+3 = 263,763 > 2^18
    cp[10500, 2, 0, 31] ^= 0x01
    ok_s, ok_c, _ = V.verify(EncryptedBallots(eb.cts, rp, cp), with_tally=False)
    assert np.argwhere(~ok_s).tolist() == [[10990, 3]]
    assert np.argwhere(~ok_c).tolist() == [[10500, 2]]


def test_two_chunks_tally_combined(group):
    from electionguard.ballot import EncryptedBallots, Manifest, Verifier
    man = Manifest(1, 2, 1)
    nb = 16384 + 700  # two verify chunks (CH = 16384 ballots)
    key, K, qbar, eb = _encrypt(group, man, nb, 47)
    V = Verifier(group, key, qbar, man)
    ok_s, ok_c, tally = V.verify(eb)
    assert ok_s.all() and ok_c.all()
    assert np.array_equal(tally, _tally_products(man, eb))
    # linearity across the chunk boundary
    _, _, t1 = V.verify(eb.slice(0, 16384))
    _, _, t2 = V.verify(eb.slice(16384, nb))
    prod = group.multP_batch(t1.reshape(-1, 512), t2.reshape(-1, 512)).reshape(tally.shape)
    assert np.array_equal(prod, tally)
    rp = eb.rproof.copy()
    rp[17000, 1, 3, 5] ^= 0x02
    ok_s, ok_c, _ = V.verify(EncryptedBallots(eb.cts, rp, eb.cproof), with_tally=False)
    assert np.argwhere(~ok_s).tolist() == [[17000, 1]] and ok_c.all()


def test_encrypt_chunk_boundary(group):
    """eg_encrypt_ballots runs in 16384-ballot chunks: with injected nonces the bytes of a
    ballot must not depend on which chunk it lands in (ballots straddling the boundary are
    re-encrypted alone and compared), and every proof verifies."""
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    from electionguard.keyceremony import key_ceremony
    man = Manifest(1, 2, 1)
    nb = 16384 + 5
    _, K = key_ceremony(group, 3, 3, seed=53)
    key = ElectionKey(group, K, window_bits=12)
    rng = np.random.default_rng(53)
    votes = random_votes(rng, man, nb)
    sn = random_scalars(rng, (nb, man.nsel, 4), group.q)
    cn = random_scalars(rng, (nb, man.n_contests), group.q)
    qbar = 9091
    eb = batch_encryption(group, key, qbar, man, votes, sn, cn)
    a, b = 16380, nb
    part = batch_encryption(group, key, qbar, man, votes[a:b], sn[a:b], cn[a:b])
    assert np.array_equal(part.cts, eb.cts[a:b])
    assert np.array_equal(part.rproof, eb.rproof[a:b])
    assert np.array_equal(part.cproof, eb.cproof[a:b])
    ok_s, ok_c, _ = Verifier(group, key, qbar, man).verify(eb, with_tally=False)
    assert ok_s.all() and ok_c.all()


def test_three_streamed_chunks(group):
    """eg_verify_ballots streams host input through two upload buffers on a copy stream:
    with three chunks the third reuses the first buffer set (waits on chunk 0's kernels).
    Verdicts, the tally and a tamper in the third chunk must all come out exactly."""
    from electionguard.ballot import EncryptedBallots, Manifest, Verifier
    man = Manifest(1, 1, 1)
    nb = 2 * 16384 + 100
    key, K, qbar, eb = _encrypt(group, man, nb, 61)
    V = Verifier(group, key, qbar, man)
    ok_s, ok_c, tally = V.verify(eb)
    assert ok_s.all() and ok_c.all()
    assert np.array_equal(tally, _tally_products(man, eb))
    cts = eb.cts.copy()
    cts[nb - 7, 1, 0, 100] ^= 0x04   # the placeholder's pad in the third chunk
    rp = eb.rproof.copy()
    rp[5, 0, 2, 9] ^= 0x01           # first chunk
    ok_s, ok_c, _ = V.verify(EncryptedBallots(cts, rp, eb.cproof), with_tally=False)
    assert np.argwhere(~ok_s).tolist() == [[5, 0], [nb - 7, 1]]
    assert np.argwhere(~ok_c).tolist() == [[nb - 7, 0]]


def test_device_encryption_matches_host(group):
    """eg_encrypt_ballots_dev (inputs and outputs in HBM, two chunks) writes exactly the
    bytes of the host-pointer eg_encrypt_ballots for the same injected nonces."""
    from electionguard.ballot import (ElectionKey, Manifest, batch_encryption, batch_encryption_device,
                                      random_scalars, random_votes)
    from electionguard.keyceremony import key_ceremony
    man = Manifest(1, 2, 1)
    nb = 16384 + 9
    _, K = key_ceremony(group, 3, 3, seed=71)
    key = ElectionKey(group, K, window_bits=12)
    rng = np.random.default_rng(71)
    votes = random_votes(rng, man, nb)
    sn = random_scalars(rng, (nb, man.nsel, 4), group.q)
    cn = random_scalars(rng, (nb, man.n_contests), group.q)
    eb = batch_encryption(group, key, 555, man, votes, sn, cn)
    dv, dsn, dcn = (group.to_device(np.ascontiguousarray(x)) for x in (votes, sn, cn))
    oc = group.device_empty(eb.cts.shape)
    orp = group.device_empty(eb.rproof.shape)
    ocp = group.device_empty(eb.cproof.shape)
    batch_encryption_device(group, key, 555, man, nb, dv.ptr, dsn.ptr, dcn.ptr, oc.ptr,
                            orp.ptr, ocp.ptr)
    assert np.array_equal(oc.download(), eb.cts)
    assert np.array_equal(orp.download(), eb.rproof)
    assert np.array_equal(ocp.download(), eb.cproof)


def test_host_pointer_encryption_equals_device_resident_with_wide_contests(group):
    """Two encryption chunks (> 16384 ballots) with a contest of more than 32 selections, so
    the contest-aggregate product tree runs several rounds through its scratch buffer while
    chunk 0's outputs are still being copied back (the contest proofs of output
    set 0 used to share that buffer).  The host-pointer bytes must equal the device-resident
    encryption's, which has no copy-back overlap."""
    from electionguard.ballot import (ElectionKey, Manifest, batch_encryption, batch_encryption_device,
                                      random_scalars, random_votes)
    from electionguard.keyceremony import key_ceremony
    man = Manifest(1, 33, 1)          # spc = 34 > 32
    nb = 16384 + 40
    gk, K = key_ceremony(group, 2, 2, seed=8)
    key = ElectionKey(group, K, window_bits=12)
    rng = np.random.default_rng(8)
    votes = random_votes(rng, man, nb)
    sn = random_scalars(rng, (nb, man.nsel, 4), group.q)
    cn = random_scalars(rng, (nb, man.n_contests), group.q)
    eb = batch_encryption(group, key, 99, man, votes, sn, cn)
    dv, dsn, dcn = (group.to_device(np.ascontiguousarray(x)) for x in (votes, sn, cn))
    oc = group.device_empty(eb.cts.shape)
    orp = group.device_empty(eb.rproof.shape)
    ocp = group.device_empty(eb.cproof.shape)
    batch_encryption_device(group, key, 99, man, nb, dv.ptr, dsn.ptr, dcn.ptr,
                            oc.ptr, orp.ptr, ocp.ptr)
    assert np.array_equal(oc.download(), eb.cts)
    assert np.array_equal(orp.download(), eb.rproof)
    assert np.array_equal(ocp.download(), eb.cproof)


def test_wide_manifest_smaller_chunks(group):
    """A 200-selection contest (201 jobs per ballot) lowers the chunk to 2^21 // 201 = 10,433
    ballots (eg_capi_ballot.inc ballot_chunk), so 10,463 ballots run as two verify chunks and
    two encryption chunks: a ballot's bytes must not depend on its chunk, every proof
    verifies, the running tally equals the product of the two halves' tallies (and CPython's
    product for a few selections), and a tamper in the second chunk is flagged exactly."""
    from electionguard.ballot import (ElectionKey, EncryptedBallots, Manifest, Verifier, batch_encryption,
                                      random_scalars, random_votes)
    from electionguard.keyceremony import key_ceremony
    man = Manifest(1, 200, 1)
    chunk = (1 << 21) // man.nsel
    assert chunk == 10433
    nb = chunk + 30
    _, K = key_ceremony(group, 2, 2, seed=83)
    key = ElectionKey(group, K, window_bits=12)
    rng = np.random.default_rng(83)
    votes = random_votes(rng, man, nb)
    sn = random_scalars(rng, (nb, man.nsel, 4), group.q)
    cn = random_scalars(rng, (nb, man.n_contests), group.q)
    eb = batch_encryption(group, key, 4242, man, votes, sn, cn)
    a, b = chunk - 4, chunk + 4
    part = batch_encryption(group, key, 4242, man, votes[a:b], sn[a:b], cn[a:b])
    assert np.array_equal(part.cts, eb.cts[a:b]) and np.array_equal(part.rproof, eb.rproof[a:b])
    assert np.array_equal(part.cproof, eb.cproof[a:b])
    V = Verifier(group, key, 4242, man)
    ok_s, ok_c, tally = V.verify(eb)
    assert ok_s.all() and ok_c.all()
    _, _, t1 = V.verify(eb.slice(0, chunk))
    _, _, t2 = V.verify(eb.slice(chunk, nb))
    prod = group.multP_batch(t1.reshape(-1, 512), t2.reshape(-1, 512)).reshape(tally.shape)
    assert np.array_equal(prod, tally)
    p = O.production_group().p
    for s in (0, 117, 199):
        for comp in range(2):
            acc = 1
            for row in eb.cts[:, s, comp]:
                acc = acc * int.from_bytes(row.tobytes(), "big") % p
            assert int.from_bytes(tally[s, comp].tobytes(), "big") == acc, (s, comp)
    rp = eb.rproof.copy()
    rp[chunk + 11, 150, 0, 7] ^= 0x10
    ok_s, ok_c, _ = V.verify(EncryptedBallots(eb.cts, rp, eb.cproof), with_tally=False)
    assert np.argwhere(~ok_s).tolist() == [[chunk + 11, 150]] and ok_c.all()


def test_oversized_arguments_rejected(group):
    """Batches past the 32-bit device index range and manifests wider than 2^20 selections
    per ballot fail with EG_ERR_ARG before anything is read or allocated."""
    import ctypes
    lib = group._lib
    one = ctypes.create_string_buffer(512)
    rc = lib.eg_powp_batch(group.handle, one, one, one, (1 << 31) + 1)
    assert rc == 1 and b"batch too large" in lib.eg_last_error()
    rc = lib.eg_multp_batch(group.handle, one, one, one, (1 << 31) + 1)
    assert rc == 1
    rc = lib.eg_prod_reduce(group.handle, one, 1 << 16, 1 << 16, one)
    assert rc == 1
    rc = lib.eg_verify_ballots_dev(group.handle, one, one, 1, 1 << 21, 1, 0, 1, one, one, one, None, one, one, None)
    assert rc == 1 and b"manifest" in lib.eg_last_error()
    rc = lib.eg_encrypt_ballots(group.handle, one, one, 1, 1 << 11, 1 << 10, one, one, one, one, one, one)
    assert rc == 1 and b"manifest" in lib.eg_last_error()


@pytest.mark.parametrize("slots,cbe,l3w", [("0", "0", "2"), ("37", "0", "2"), ("100", "0", "2"), ("768", "0", "2"),
                                           ("5000", "0", "2"), ("37", "1", "2"), ("37", "1", "1"), ("100", "1", "3"),
                                           ("768", "1", "2")])
def test_launch_split_independent(group, slots, cbe, l3w, monkeypatch):
    """The verifier sizes its three k_pow launches from the resident-workgroup count (beta
    head in launch 1, every contest-a job in launch 2, contest b in launch 3; with
    EG_CB_EARLY=1 launch 1 takes more betas and launch 2 the contest-b jobs they complete,
    launch 3 keeps EG_L3_WAVES waves per SIMD of them; eg_capi_ballot.inc).  Verdicts and tally
    must not depend on where the splits fall: EG_POW_SLOTS forces other split points (0 = no
    split), against the CPython tally and a tamper in the moved jobs."""
    from electionguard.ballot import EncryptedBallots, Manifest, Verifier
    man = Manifest(4, 5, 1)
    nb = 700  # 16,800 selection jobs = 525 workgroups: every slot count above splits differently
    key, K, qbar, eb = _encrypt(group, man, nb, 91)
    V = Verifier(group, key, qbar, man)
    monkeypatch.setenv("EG_POW_SLOTS", slots)
    monkeypatch.setenv("EG_CB_EARLY", cbe)
    monkeypatch.setenv("EG_L3_WAVES", l3w)  # launch 3's size in waves per SIMD (EG_CB_EARLY=1)
    ok_s, ok_c, tally = V.verify(eb)
    assert ok_s.all() and ok_c.all()
    assert np.array_equal(tally, _tally_products(man, eb))
    rp, cp = eb.rproof.copy(), eb.cproof.copy()
    rp[3, 7, 2, 4] ^= 0x08       # a beta-head job (ballot 3) in launch 1 when split
    cp[10, 2, 1, 3] ^= 0x10      # an early contest (its contest-b job in launch 2 when split)
    cp[650, 1, 1, 9] ^= 0x20     # a late contest (its contest-b job in launch 3 when split)
    ok_s, ok_c, _ = V.verify(EncryptedBallots(eb.cts, rp, cp), with_tally=False)
    assert np.argwhere(~ok_s).tolist() == [[3, 7]]
    assert np.argwhere(~ok_c).tolist() == [[10, 2], [650, 1]]


def test_cast_mask_across_verify_chunks(group):
    """The cast flags follow each ballot across the verifier's 16,384-ballot chunks, on the
    host-pointer path (flags uploaded once, offset per chunk) and the device path: spoiled
    ballots on both sides of the boundary, the tally equals the CPython product over the cast
    ballots only; the verdicts of every ballot are still computed."""
    from electionguard.ballot import EncryptedBallots, Manifest, Verifier
    man = Manifest(1, 2, 1)
    nb = 16384 + 300
    key, K, qbar, eb = _encrypt(group, man, nb, 53)
    rng = np.random.default_rng(53)
    cast = rng.random(nb) > 0.25
    cast[[16383, 16384]] = (False, False)
    V = Verifier(group, key, qbar, man)
    ok_s, ok_c, tally = V.verify(eb, cast=cast)
    assert ok_s.all() and ok_c.all()
    want = _tally_products(man, EncryptedBallots(eb.cts[cast], eb.rproof[cast], eb.cproof[cast]))
    assert np.array_equal(tally, want)
    d = [group.to_device(np.ascontiguousarray(x)) for x in (eb.cts, eb.rproof, eb.cproof)]
    dm = group.to_device(cast.astype(np.uint8))
    oks = group.device_zeros((nb, man.nsel))
    okc = group.device_zeros((nb, man.n_contests))
    tal = group.device_zeros((man.n_real, 2, 512))
    V.verify_device(d[0].ptr, d[1].ptr, d[2].ptr, nb, oks.ptr, okc.ptr,
                    tal.ptr, dm.ptr)
    group.sync()
    assert group.all_nonzero(oks) and group.all_nonzero(okc) and np.array_equal(tal.download(), want)
