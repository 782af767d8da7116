"""Concurrent callers on one context.  The reference's verifier and trustees call the
group from a thread pool (Verifier.kt nthreads, RunRemoteWorkflowTest.java:140-182 runs
11 threads); libeg_hip serialises them on the context mutex, and ctypes drops the GIL
around each foreign call, so interleaved batches from many threads must each come back
bit-exact with the oracle."""
import random
import threading

import pytest

import eg_oracle as O
from conftest import be2i
from test_gpu_ballots import _oracle_ballots, _setup

pytestmark = pytest.mark.gpu


def _run_threads(fns):
    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 - re-raised on the main thread
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts), "a caller thread is still running"
    if errs:
        raise errs[0]


def test_concurrent_powp_and_fixed_base(group, oracle_group):
    Og = oracle_group
    results = {}

    def powp(seed):
        def f():
            rng = random.Random(seed)
            n = 29 + seed
            bases = [rng.randrange(Og.p) for _ in range(n)]
            exps = [rng.randrange(Og.q) for _ in range(n)]
            for _ in range(3):
                out = group.powP_batch(bases, exps)
                results.setdefault(seed, []).append(
                    all(be2i(out[i]) == pow(bases[i], exps[i], Og.p) for i in range(n)))
        return f

    def gpow(seed):
        def f():
            rng = random.Random(seed)
            n = 100 + seed
            exps = [rng.randrange(Og.q) for _ in range(n)]
            for _ in range(3):
                out = group.gPowP_batch(exps)
                results.setdefault(seed, []).append(
                    all(be2i(out[i]) == pow(Og.g, exps[i], Og.p) for i in range(n)))
        return f

    _run_threads([powp(s) for s in range(1, 5)] + [gpow(s) for s in range(11, 15)])
    assert len(results) == 8
    assert all(all(v) and len(v) == 3 for v in results.values()), results


def test_concurrent_verifiers_one_context(group):
    """Four verifier threads over the same ballots, plus one with a tampered ballot:
    every thread gets the same accept/reject vector and tally as a lone call."""
    from electionguard.ballot import EncryptedBallots, Manifest, Verifier
    og, rng, K, qbar, key = _setup(group, seed=31)
    man = Manifest(2, 3, 1)
    cts, rp, cp, _ = _oracle_ballots(og, K, qbar, O.Manifest(2, 3, 1), 4, rng)
    ref_s, ref_c, ref_t = Verifier(group, key, qbar, man).verify(EncryptedBallots(cts, rp, cp))
    assert ref_s.all() and ref_c.all()
    rp_bad = rp.copy()
    rp_bad[2, 4, 1, 31] ^= 1
    got = {}

    def run(tag, rp_use):
        def f():
            v = Verifier(group, key, qbar, man)
            for k in range(2):
                got[(tag, k)] = v.verify(EncryptedBallots(cts, rp_use, cp))
        return f

    _run_threads([run(t, rp) for t in range(4)] + [run("bad", rp_bad)])
    for t in range(4):
        for k in range(2):
            s, c, tl = got[(t, k)]
            assert (s == ref_s).all() and (c == ref_c).all() and (tl == ref_t).all()
    for k in range(2):
        s, c, _ = got[("bad", k)]
        assert not s[2, 4] and s.sum() == s.size - 1 and c.all()


def test_two_keys_on_one_context_device_paths(group):
    """Threads using DIFFERENT election keys on the one shared context (productionGroup): every
    device-pointer verify and encryption call passes its own K and the library sets it under the
    ctx lock for that call, so no call can run against another thread's key (the
    ensure()-then-call sequence used to race).  Each thread encrypts on the device, checks the
    bytes against its own host encryption made before the threads start, and verifies on the
    device; a tally under the wrong key would fail the proofs."""
    import numpy as np
    from electionguard.ballot import (ElectionKey, Manifest, Verifier, batch_encryption, batch_encryption_device,
                                      random_scalars, random_votes)
    from electionguard.keyceremony import key_ceremony
    man = Manifest(2, 3, 1)
    jobs = []
    for seed in (101, 202, 303):
        _, K = key_ceremony(group, 2, 2, seed=seed)
        key = ElectionKey(group, K)
        rng = np.random.default_rng(seed)
        nb = 40
        votes = random_votes(rng, man, nb)
        sn = random_scalars(rng, (nb, man.nsel, 4), group.q)
        cn = random_scalars(rng, (nb, man.n_contests), group.q)
        ref = batch_encryption(group, key, seed, man, votes, sn, cn)
        jobs.append((seed, key, nb, votes, sn, cn, ref))
    ok = {}

    def run(seed, key, nb, votes, sn, cn, ref):
        def f():
            dv, dsn, dcn = (group.to_device(np.ascontiguousarray(x)) for x in (votes, sn, cn))
            oc = group.device_empty(ref.cts.shape)
            orp = group.device_empty(ref.rproof.shape)
            ocp = group.device_empty(ref.cproof.shape)
            oks = group.device_zeros((nb, man.nsel))
            okc = group.device_zeros((nb, man.n_contests))
            V = Verifier(group, key, seed, man)
            res = []
            for _ in range(4):
                batch_encryption_device(group, key, seed, man, nb, dv.ptr, dsn.ptr, dcn.ptr,
                                        oc.ptr, orp.ptr, ocp.ptr)
                V.verify_device(oc.ptr, orp.ptr, ocp.ptr, nb, oks.ptr, okc.ptr, None)
                group.sync()
                res.append(bool(np.array_equal(oc.download(), ref.cts)) and group.all_nonzero(oks) and group.all_nonzero(okc))
            ok[seed] = res
        return f

    _run_threads([run(*j) for j in jobs])
    assert ok == {s: [True] * 4 for s, *_ in jobs}, ok
