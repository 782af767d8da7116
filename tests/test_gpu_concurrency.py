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
