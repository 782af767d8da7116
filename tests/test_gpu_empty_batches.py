"""GPU: empty and one-element batches through every batched entry point (the edge cases of the
reference's batch calls: an election with no cast ballots, a trustee RPC with no texts --
decrypting_trustee_rpc.proto:15-18 allows an empty `repeated ElGamalCiphertext text` -- and a
single ballot).  Empty batches return empty results (and the identity tally) without touching the
device; one-element batches go through the latency-shaped layouts and must equal the oracle."""
import random

import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


def _be(x: int, n: int = 512) -> np.ndarray:
    return np.frombuffer(int(x).to_bytes(n, "big"), np.uint8)


def test_empty_group_batches(group):
    z512, z32 = np.empty((0, 512), np.uint8), np.empty((0, 32), np.uint8)
    assert group.powP_batch(z512, z32).shape == (0, 512)
    assert group.gPowP_batch(z32).shape == (0, 512)
    assert group.multP_batch(z512, z512).shape == (0, 512)
    assert group.multInv_batch(z512).shape == (0, 512)
    assert group.prodP_groups(z512, 0, 3).shape[0] == 0


def test_empty_ballot_batches_give_the_identity_tally(group, oracle_group):
    from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
    rng = random.Random(3)
    K = pow(oracle_group.g, rng.randrange(1, oracle_group.q), oracle_group.p)
    key = ElectionKey(group, K, window_bits=8)
    man = Manifest(2, 3, 1)
    nrng = np.random.default_rng(3)
    eb = batch_encryption(group, key, 5, man, random_votes(nrng, man, 0), random_scalars(nrng, (0, man.nsel, 4), group.q),
                          random_scalars(nrng, (0, man.n_contests), group.q))
    assert eb.cts.shape == (0, man.nsel, 2, 512) and eb.rproof.shape[0] == 0 and eb.cproof.shape[0] == 0
    ok_s, ok_c, tally = Verifier(group, key, 5, man).verify(eb)
    assert ok_s.shape == (0, man.nsel) and ok_c.shape == (0, man.n_contests)
    # runAccumulateBallots over no cast ballots: every selection's (pad, data) is the group identity
    assert tally.shape == (man.n_real, 2, 512)
    assert all(int.from_bytes(tally[i, j].tobytes(), "big") == 1 for i in range(man.n_real) for j in range(2))
    # the device-resident form writes the same identity tally
    d_tal = group.device_zeros((man.n_real, 2, 512))
    Verifier(group, key, 5, man).verify_device(0, 0, 0, 0, 0, 0, d_tal.ptr)
    group.sync()
    assert np.array_equal(d_tal.download(), tally)


def test_empty_and_single_trustee_batches(group, oracle_group):
    """A trustee RPC with no texts answers with no shares; one text gives one share the oracle
    verifies (DecryptingTrusteeIF.directDecrypt / compensatedDecrypt, RemoteDecryptingTrusteeProxy.java:48-115)."""
    from electionguard.decrypt import DecryptingTrustee, verify_shares
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 3, 2, seed=11)
    comm = {g.gid: g.commitments for g in gk}
    tr = DecryptingTrustee(group, gk[0], comm)
    qbar = 77
    assert tr.directDecrypt(group, [], qbar) == []
    assert tr.compensatedDecrypt(group, gk[2].gid, [], qbar) == []
    G = oracle_group
    rng = random.Random(12)
    ct = O.encrypt(G, K, 1, rng.randrange(1, G.q))
    res = tr.directDecrypt(group, [(ct.pad, ct.data)], qbar)
    assert len(res) == 1
    assert res[0].partialDecryption == pow(ct.pad, int(gk[0].secret), G.p)
    M, pr = tr.directDecryptArrays(group, [(ct.pad, ct.data)], qbar)
    assert verify_shares(group, qbar, gk[0].public_key, [(ct.pad, ct.data)], M, pr).all()


def test_single_ballot_verify_and_tally_equal_the_oracle(group, oracle_group):
    """One ballot (the smallest ragged batch): the verifier accepts it and its tally is the ballot's
    own ciphertexts, as the oracle encrypts them."""
    from electionguard.ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
    G = oracle_group
    rng = random.Random(13)
    gs, K = O.key_ceremony(G, 2, 2, rng)
    qbar = rng.randrange(G.q)
    man_o, man = O.Manifest(3, 2, 1), Manifest(3, 2, 1)
    eb = O.encrypt_ballot(G, K, qbar, man_o, O.ballot_plaintexts(man_o, rng), rng)
    cts = np.stack([np.stack([_be(ct.pad), _be(ct.data)]) for ct in eb.cts])[None]
    rp = np.stack([np.stack([_be(v, 32) for v in (p.c0, p.v0, p.c1, p.v1)]) for p in eb.proofs])[None]
    cp = np.stack([np.stack([_be(p.c, 32), _be(p.v, 32)]) for p in eb.contest_proofs])[None]
    ok_s, ok_c, tally = Verifier(group, ElectionKey(group, K), qbar, man).verify(EncryptedBallots(cts, rp, cp))
    assert ok_s.all() and ok_c.all()
    for i, ct in enumerate(O.accumulate_tally(G, man_o, [eb])):
        assert int.from_bytes(tally[i, 0].tobytes(), "big") == ct.pad
        assert int.from_bytes(tally[i, 1].tobytes(), "big") == ct.data
