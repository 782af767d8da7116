"""GPU: the exact configuration bench.py times (configs[1]: 10,000 ballots, 4 contests x 5
selections + 1 placeholder, 22-bit g/K radix tables, device-pointer verifier), checked the
way a full-size run can be checked on the CPU:

* every verdict of the honest batch is valid, and the C oracle (OpenSSL BN, an independent
  restatement) re-verifies every 50th ballot;
* the GPU tally equals the CPython product of all 10,000 ballots' ciphertexts per selection;
* the device-pointer path (verify_ballots_dev, what bench.py times) and the host-pointer
  path agree byte for byte on the tally;
* flipping one bit of one proof in the middle of the batch flips exactly that verdict.
"""
import numpy as np
import pytest

import eg_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def bench_batch(group):
    from electionguard.ballot import ElectionKey, Manifest, batch_encryption, random_scalars, random_votes
    from electionguard.keyceremony import key_ceremony
    man = Manifest(4, 5, 1)
    gk, K = key_ceremony(group, 3, 3, seed=20241015)
    key = ElectionKey(group, K, window_bits=22)
    qbar = int.from_bytes(b"electionguard-remote mi355x qbar".ljust(32, b"\0"), "big") % group.q
    rng = np.random.default_rng(1000)
    nb = 10000
    votes = random_votes(rng, man, nb)
    eb = batch_encryption(group, key, qbar, man, votes, random_scalars(rng, (nb, man.nsel, 4), group.q),
                          random_scalars(rng, (nb, man.n_contests), group.q))
    return man, key, K, qbar, votes, eb


def test_bench_config_verdicts_tally_and_device_path(group, bench_batch):
    from eg_oracle_c import COracle
    from electionguard.ballot import Verifier
    man, key, K, qbar, votes, eb = bench_batch
    V = Verifier(group, key, qbar, man)
    ok_s, ok_c, tally = V.verify(eb)
    assert ok_s.all() and ok_c.all()
    # independent re-verification of a sample
    og = O.production_group()
    co = COracle(og.p, O.Q, og.g)
    co.set_key(K)
    idx = np.arange(0, eb.n, 50)
    s_ok, c_ok, _ = co.verify_ballots(qbar, man.n_contests, man.spc, 1, 1, eb.cts[idx], eb.rproof[idx],
                                      eb.cproof[idx], threads=16, tally=False)
    assert s_ok.all() and c_ok.all()
    # tally = product over all ballots (CPython ints)
    p = og.p
    for s in range(man.n_real):
        k, r = divmod(s, man.n_selections)
        i = k * man.spc + r
        for c in range(2):
            acc = 1
            for b in range(eb.n):
                acc = acc * int.from_bytes(eb.cts[b, i, c].tobytes(), "big") % p
            assert int.from_bytes(tally[s, c].tobytes(), "big") == acc, (s, c)
    # the device-pointer path bench.py times
    d_cts, d_rp, d_cp = (group.to_device(a) for a in (eb.cts, eb.rproof, eb.cproof))
    d_oks = group.device_zeros((eb.n, man.nsel))
    d_okc = group.device_zeros((eb.n, man.n_contests))
    d_tal = group.device_zeros((man.n_real, 2, 512))
    V.verify_device(d_cts.ptr, d_rp.ptr, d_cp.ptr, eb.n, d_oks.ptr, d_okc.ptr,
                    d_tal.ptr)
    group.sync()
    assert group.all_nonzero(d_oks) and group.all_nonzero(d_okc)
    assert np.array_equal(d_tal.download(), tally)


def test_bench_config_single_bit_tamper(group, bench_batch):
    from electionguard.ballot import EncryptedBallots, Verifier
    man, key, K, qbar, votes, eb = bench_batch
    rp = eb.rproof.copy()
    rp[5003, 11, 2, 7] ^= 0x10
    ok_s, ok_c, _ = Verifier(group, key, qbar, man).verify(EncryptedBallots(eb.cts, rp, eb.cproof), with_tally=False)
    assert np.argwhere(~ok_s).tolist() == [[5003, 11]] and ok_c.all()
