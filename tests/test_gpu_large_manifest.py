"""GPU: the large-manifest shape of BASELINE configs[4] (100 selections per ballot:
20 contests x 5 selections + 1 placeholder each = 120 encrypted selections).

* GPU-encrypted ballots (random nonces) verify on the GPU AND on the independent
  OpenSSL-BN C oracle; the GPU tally equals the C oracle's tally bit-exactly;
* the tally decrypts (3 guardians, quorum 3) to the exact per-selection vote counts;
* tampering one contest proof in a late contest flags exactly that contest.
"""
import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def large(group):
    from electionguard.ballot import ElectionKey, Manifest, batch_encryption, random_scalars, random_votes
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 3, 3, seed=55)
    key = ElectionKey(group, K, window_bits=12)
    man = Manifest(20, 5, 1)
    rng = np.random.default_rng(5)
    nb = 40
    votes = random_votes(rng, man, nb)
    qbar = 0x5EED
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), group.q),
                          random_scalars(rng, (nb, man.n_contests), group.q))
    return gk, key, K, man, qbar, votes, eb


def test_large_manifest_verify_tally_vs_c_oracle(group, large):
    from eg_oracle_c import COracle
    from electionguard.ballot import Verifier
    gk, key, K, man, qbar, votes, eb = large
    assert man.nsel == 120 and man.n_real == 100
    ok_s, ok_c, tally = Verifier(group, key, qbar, man).verify(eb)
    assert ok_s.all() and ok_c.all()
    og = O.production_group()
    co = COracle(og.p, O.Q, og.g)
    co.set_key(K)
    s_ok, c_ok, t_ref = co.verify_ballots(qbar, man.n_contests, man.spc, 1, 1, eb.cts, eb.rproof, eb.cproof,
                                          threads=8, tally=True)
    assert s_ok.all() and c_ok.all()
    assert np.array_equal(t_ref, tally)


def test_large_manifest_decrypts_to_counts(group, large):
    from electionguard.ballot import Verifier
    from electionguard.decrypt import Decryption, DecryptingTrustee
    gk, key, K, man, qbar, votes, eb = large
    _, _, tally = Verifier(group, key, qbar, man).verify(eb)
    comm = {g.gid: g.commitments for g in gk}
    trustees = [DecryptingTrustee(group, g, comm) for g in gk]
    counts = Decryption(group, qbar, trustees, [], {g.gid: g.public_key for g in gk}).decrypt(tally, eb.n)
    want = votes.reshape(eb.n, man.n_contests, man.spc)[:, :, : man.n_selections].sum(axis=0).reshape(-1)
    assert counts == want.tolist()


def test_large_manifest_tamper_late_contest(group, large):
    from electionguard.ballot import EncryptedBallots, Verifier
    gk, key, K, man, qbar, votes, eb = large
    cp = eb.cproof.copy()
    cp[7, 17, 1, 30] ^= 0x10
    ok_s, ok_c, _ = Verifier(group, key, qbar, man).verify(EncryptedBallots(eb.cts, eb.rproof, cp), with_tally=False)
    assert ok_s.all()
    assert np.argwhere(~ok_c).tolist() == [[7, 17]]
