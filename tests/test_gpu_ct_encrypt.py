"""GPU: constant-time encryption (eg_ctx_set_ct_encrypt).  The fixed-base terms of the encryptor
read 6-bit radix tables of g and K with masked scans of every window column instead of indexing
the 22-bit tables by nonce digits, and both proof branches are computed and ordered with masks, so
no address depends on a nonce or a vote.  The bytes must not change: the golden ballots (oracle
encryption with injected nonces) and a random batch in both modes, host and device pointers."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_ct_mode_reproduces_golden_ballots(group):
    from test_oracle_golden import golden_ballot_arrays
    from electionguard.ballot import ElectionKey, Manifest, batch_encryption
    d, (nc, ns, va, spc), cts, rp, cp = golden_ballot_arrays()
    man = Manifest(nc, ns, va)
    votes = np.array([b["votes"] for b in d["ballots"]], np.uint8)
    sn = np.stack([np.stack([np.stack([np.frombuffer(bytes.fromhex(x), np.uint8) for x in s4]) for s4 in b["nonces"]])
                   for b in d["ballots"]])
    cn = np.stack([np.stack([np.frombuffer(bytes.fromhex(x), np.uint8) for x in b["contest_nonces"]])
                   for b in d["ballots"]])
    key = ElectionKey(group, int(d["K"], 16), window_bits=12)
    group.ct_encrypt = True
    try:
        eb = batch_encryption(group, key, int(d["qbar"], 16), man, votes, sn, cn)
    finally:
        group.ct_encrypt = False
    assert np.array_equal(eb.cts, cts) and np.array_equal(eb.rproof, rp) and np.array_equal(eb.cproof, cp)


def test_ct_mode_same_bytes_host_and_device(group):
    from electionguard.ballot import (ElectionKey, Manifest, Verifier, batch_encryption, batch_encryption_device,
                                      random_scalars, random_votes)
    from electionguard.keyceremony import key_ceremony
    man = Manifest(4, 5, 1)
    nb = 600
    _, K = key_ceremony(group, 3, 3, seed=61)
    key = ElectionKey(group, K, window_bits=16)
    rng = np.random.default_rng(61)
    votes = random_votes(rng, man, nb)
    sn = random_scalars(rng, (nb, man.nsel, 4), group.q)
    cn = random_scalars(rng, (nb, man.n_contests), group.q)
    qbar = 0xC7E
    ref = batch_encryption(group, key, qbar, man, votes, sn, cn)
    group.ct_encrypt = True
    try:
        ct = batch_encryption(group, key, qbar, man, votes, sn, cn)
        dv, dsn, dcn = (group.to_device(np.ascontiguousarray(x)) for x in (votes, sn, cn))
        oc = group.device_empty(ref.cts.shape)
        orp = group.device_empty(ref.rproof.shape)
        ocp = group.device_empty(ref.cproof.shape)
        batch_encryption_device(group, key, qbar, man, nb, dv.ptr, dsn.ptr, dcn.ptr,
                                oc.ptr, orp.ptr, ocp.ptr)
    finally:
        group.ct_encrypt = False
    assert np.array_equal(ct.cts, ref.cts) and np.array_equal(ct.rproof, ref.rproof)
    assert np.array_equal(ct.cproof, ref.cproof)
    assert np.array_equal(oc.download(), ref.cts) and np.array_equal(orp.download(), ref.rproof)
    assert np.array_equal(ocp.download(), ref.cproof)
    ok_s, ok_c, _ = Verifier(group, key, qbar, man).verify(ct, with_tally=False)
    assert ok_s.all() and ok_c.all()
