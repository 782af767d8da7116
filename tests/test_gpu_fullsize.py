"""GPU: size-independent checks at bench scale (configs[1]: 4 contests x 5 selections).

* every verdict valid on honest ballots and the GPU tally equals the independent
  OpenSSL-BN oracle's tally over ALL ballots (products only: cheap on the CPU);
* a spot sample (every 97th ballot) is re-verified by the C oracle;
* linearity: tally(A ++ B) = tally(A) * tally(B) componentwise (fold of partial tallies);
* tampering one proof anywhere flips exactly that verdict.
"""
import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def big(group):
    from electionguard.ballot import ElectionKey, Manifest, batch_encryption, random_scalars, random_votes
    from electionguard.keyceremony import key_ceremony
    gk, K = key_ceremony(group, 3, 3, seed=8)
    key = ElectionKey(group, K, window_bits=16)
    man = Manifest(4, 5, 1)
    rng = np.random.default_rng(97)
    nb = 2000
    votes = random_votes(rng, man, nb)
    qbar = 424242
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), group.q),
                          random_scalars(rng, (nb, man.n_contests), group.q))
    return key, K, man, qbar, votes, eb


def test_fullsize_verify_tally_vs_c_oracle(group, big):
    from eg_oracle_c import COracle
    from electionguard.ballot import Verifier
    key, K, man, qbar, votes, eb = big
    ok_s, ok_c, tally = Verifier(group, key, qbar, man).verify(eb)
    assert ok_s.all() and ok_c.all()
    co = COracle(O.production_group().p, O.Q, O.production_group().g)
    co.set_key(K)
    sample = eb.slice(0, eb.n)
    idx = np.arange(0, eb.n, 97)
    s_ok, c_ok, _ = co.verify_ballots(qbar, man.n_contests, man.spc, 1, 1, sample.cts[idx], sample.rproof[idx],
                                      sample.cproof[idx], threads=8, tally=False)
    assert s_ok.all() and c_ok.all()
    # tally of all ballots by the oracle's products (CPython ints)
    G = O.production_group()
    nb = eb.n
    for s in range(man.n_real):
        k, r = divmod(s, man.n_selections)
        i = k * man.spc + r
        for c in range(2):
            want = 1
            for b in range(nb):
                want = want * int.from_bytes(eb.cts[b, i, c].tobytes(), "big") % G.p
            assert int.from_bytes(tally[s, c].tobytes(), "big") == want, (s, c)


def test_tally_linearity_and_tamper(group, big):
    from electionguard.ballot import EncryptedBallots, Verifier
    key, K, man, qbar, votes, eb = big
    V = Verifier(group, key, qbar, man)
    _, _, t_all = V.verify(eb.slice(0, 1000))
    _, _, t_a = V.verify(eb.slice(0, 613))
    _, _, t_b = V.verify(eb.slice(613, 1000))
    prod = group.multP_batch(t_a.reshape(-1, 512), t_b.reshape(-1, 512)).reshape(t_all.shape)
    assert np.array_equal(prod, t_all)
    rp = eb.rproof[:500].copy()
    rp[321, 17, 0, 9] ^= 0x04
    ok_s, ok_c, _ = V.verify(EncryptedBallots(eb.cts[:500], rp, eb.cproof[:500]), with_tally=False)
    bad = np.argwhere(~ok_s)
    assert bad.tolist() == [[321, 17]] and ok_c.all()
