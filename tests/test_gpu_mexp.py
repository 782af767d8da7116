"""GPU: the general per-element job (eg_mexp_submit / eg_mexp_one, the per-wave kernel k_wave_job) and
the constant-time exponentiation switch (eg_ctx_set_ct_pow), bit-exact against CPython integers.

Upstream drives the group one element at a time from 11 threads: g^R, K^R (the accelerated election
key), g^v * alpha^c, the contest aggregate (prod alpha)^c (RunRemoteWorkflowTest.java:140-141,
179-181, on the group of KUtils.java:10-12).  Every such call is one job
    out = (prod bases)^e * T0^e0 * T1^e1 mod p,
and a coalesced batch mixes every kind of job in one launch."""
import random
import threading

import pytest

pytestmark = pytest.mark.gpu

def _edges(og):
    return [0, 1, 2, og.q - 1, og.q, 2**256 - 1]


def _want(og, bases, e, fixed):
    prod = 1
    for b in bases:
        prod = prod * b % og.p
    r = 1 if (e is not None and not bases) else (pow(prod, e, og.p) if e is not None else prod % og.p)
    for base, fe in fixed:
        r = r * pow(base, fe, og.p) % og.p
    return r


def _random_job(rng, og, tabs):
    nb = rng.choice([0, 0, 1, 1, 1, 2, 3, 16])
    bases = [rng.choice([rng.randrange(og.p), rng.randrange(2**4096), 0, 1, og.p - 1, og.p]) if rng.random() < 0.2
             else rng.randrange(og.p) for _ in range(nb)]
    e = None
    if rng.random() < 0.7:
        e = rng.choice(_edges(og)) if rng.random() < 0.2 else rng.randrange(og.q)
    nf = rng.choice([0, 1, 1, 2])
    if nb == 0 and e is None and nf == 0:
        nf = 1
    fixed = []
    for _ in range(nf):
        name = rng.choice(list(tabs))
        fe = rng.choice(_edges(og)) if rng.random() < 0.2 else rng.randrange(og.q)
        fixed.append((name, fe))
    return bases, e, fixed


@pytest.fixture(scope="module")
def tables(group, oracle_group):
    """g's table (the context's), an election key K at 12 bits (wider than a constant-time scan takes:
    the companion path) and a second key at 8 bits."""
    og = oracle_group
    rng = random.Random(77)
    K = pow(og.g, rng.randrange(og.q), og.p)
    K2 = pow(og.g, rng.randrange(og.q), og.p)
    t = {"g": (None, og.g), "K12": (group.fixed_base(K, 12), K), "K8": (group.fixed_base(K2, 8), K2)}
    yield t
    for fb, _ in t.values():
        if fb is not None:
            fb.close()


def _run_jobs(group, og, tables, jobs):
    bad = []
    for i, (bases, e, fixed) in enumerate(jobs):
        got = group.mexp_one(bases, e, [(tables[n][0], fe) for n, fe in fixed])
        want = _want(og, bases, e, [(tables[n][1], fe) for n, fe in fixed])
        if int.from_bytes(got, "big") != want:
            bad.append((i, len(bases), e is not None, [n for n, _ in fixed]))
    return bad


@pytest.mark.parametrize("ct", [False, True])
def test_mexp_jobs_eleven_threads_bitexact(group, oracle_group, tables, ct):
    """11 threads submit random jobs of every shape (0-16 bases, with or without an exponent, 0-2
    fixed-base terms over three tables, edge values) through the coalescer: the batches mix kinds in
    one launch; every result equals the CPython product.  ct: the constant-time instantiation."""
    og = oracle_group
    rng = random.Random(101 + ct)
    jobs = [_random_job(rng, og, tables) for _ in range(11 * 24)]
    bad = []
    group.ct_pow = ct
    try:
        ths = [threading.Thread(target=lambda k=k: bad.extend(_run_jobs(group, og, tables, jobs[k::11])))
               for k in range(11)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    finally:
        group.ct_pow = False
    assert not bad, bad[:8]


def test_mexp_fused_forms(group, oracle_group, tables):
    """The fused forms the per-element mirrors build: g^v * alpha^c (one base, an exponent, g's table),
    K^v * beta^c * g^-c, the contest aggregate (alpha_1 ... alpha_5)^c, times (two bases)."""
    og = oracle_group
    rng = random.Random(5)
    al, be = rng.randrange(og.p), rng.randrange(og.p)
    c, v = rng.randrange(og.q), rng.randrange(og.q)
    g_t, k_t = tables["g"][0], tables["K12"][0]
    K = tables["K12"][1]
    assert int.from_bytes(group.mexp_one([al], c, [(g_t, v)]), "big") == pow(og.g, v, og.p) * pow(al, c, og.p) % og.p
    got = group.mexp_one([be], c, [(k_t, v), (g_t, og.q - c)])
    assert int.from_bytes(got, "big") == pow(K, v, og.p) * pow(be, c, og.p) * pow(og.g, og.q - c, og.p) % og.p
    alphas = [rng.randrange(og.p) for _ in range(5)]
    A = 1
    for x in alphas:
        A = A * x % og.p
    assert int.from_bytes(group.mexp_one(alphas, c), "big") == pow(A, c, og.p)
    assert int.from_bytes(group.mexp_one([al, be]), "big") == al * be % og.p
    # an accelerated element's powP (eg_fb_pow_one) and gPowP through the same kernel
    assert int.from_bytes(k_t.pow_one(c), "big") == pow(K, c, og.p)
    assert int.from_bytes(group.gPowP_one(c), "big") == pow(og.g, c, og.p)


def test_mexp_argument_errors(group, tables):
    from electionguard.core import native
    with pytest.raises(native.EgError):
        group.mexp_one([1] * 17, 3)  # at most 16 bases per job
    with pytest.raises(ValueError):
        group.mexp_one([], None, [(tables["K8"][0], 1)] * 3)


@pytest.mark.parametrize("n", [1, 700, 3000, 9000])
def test_ct_pow_batches_bitexact(group, oracle_group, tables, n):
    """eg_ctx_set_ct_pow on the batch entry points: the per-wave (<= one per SIMD: n = 1, 700), 16-lane
    (<= half a resident round, ~6k: n = 3000) and 8-lane (n = 9000) variable-base layouts and
    fixed-base batches over an 8-bit table and a 12-bit table (its 6-bit constant-time companion) are
    bit-exact on edge and random exponents."""
    og = oracle_group
    rng = random.Random(n)
    exps = [_edges(og)[i % 6] if i < 12 else rng.randrange(og.q) for i in range(n)]
    bases = [rng.randrange(og.p) if i % 5 else rng.choice([0, 1, og.p - 1, og.p, 2**4096 - 1]) for i in range(n)]
    group.ct_pow = True
    try:
        out = group.powP_batch(bases, exps)
        for name in ("K8", "K12", "g"):
            fb, base = tables[name]
            fo = fb.pow_batch(exps) if fb is not None else group.gPowP_batch(exps)
            for i in range(0, n, max(1, n // 97)):
                assert int.from_bytes(fo[i].tobytes(), "big") == pow(base, exps[i], og.p), (name, i)
    finally:
        group.ct_pow = False
    for i in range(0, n, max(1, n // 97)):
        assert int.from_bytes(out[i].tobytes(), "big") == pow(bases[i], exps[i], og.p), i
    for i in range(min(n, 12)):
        assert int.from_bytes(out[i].tobytes(), "big") == pow(bases[i], exps[i], og.p), i


def _r2l_exponents(og):
    """Top bits at every residue mod 3 (the chain's rounds take 3 powers), single bits, runs of ones,
    and the edges."""
    es = [0, 1, 2, 3, 4, 5, 6, 7, 8, og.q - 1, og.q, 2**256 - 1, 2**255, 2**254, 2**253]
    es += [2**k for k in (9, 10, 11, 127, 128, 129)]
    es += [2**k - 1 for k in (2, 3, 4, 250, 251, 252)]
    return es


@pytest.mark.parametrize("n", [1, 37, 256])
def test_r2l_powp_batch_bitexact(group, oracle_group, n):
    """Batches of at most one job per CU run the variable part right to left over four waves (wave 0
    squares, waves 1-3 multiply in the set bits from an LDS ring): bit-exact on every top-bit position
    class, edge exponents and edge bases."""
    og = oracle_group
    rng = random.Random(900 + n)
    es = _r2l_exponents(og)
    exps = [es[i % len(es)] if i < len(es) or rng.random() < 0.3 else rng.randrange(og.q) for i in range(n)]
    if n == 1:
        exps = [rng.randrange(og.q)]
    bases = [rng.choice([0, 1, og.p - 1, og.p, og.p + 5, 2**4096 - 1]) if rng.random() < 0.15 else rng.randrange(og.p)
             for _ in range(n)]
    out = group.powP_batch(bases, exps)
    bad = [i for i in range(n) if int.from_bytes(out[i].tobytes(), "big") != pow(bases[i], exps[i], og.p)]
    assert not bad, bad[:8]


def test_r2l_mixed_jobs_bitexact(group, oracle_group, tables):
    """Mixed per-element jobs through the coalescer on the right-to-left shape: a variable part on the
    chain and fixed-base windows on the multiplying waves in the same rounds (g^v * alpha^c,
    K^v * beta^c * g^-c), products of several bases raised to edge exponents, and products without an
    exponent in the same batch."""
    og = oracle_group
    rng = random.Random(4242)
    es = _r2l_exponents(og)
    g_t, k_t, k8 = tables["g"][0], tables["K12"][0], tables["K8"][0]
    K, K2 = tables["K12"][1], tables["K8"][1]
    subs = []
    for i, e in enumerate(es):
        al = rng.randrange(og.p)
        v = rng.randrange(og.q)
        bases = [al] if i % 3 else [al, rng.randrange(og.p), rng.randrange(og.p)]
        prod = 1
        for b in bases:
            prod = prod * b % og.p
        subs.append((group.mexp_submit(bases, e, [(g_t, v)]), pow(prod, e, og.p) * pow(og.g, v, og.p) % og.p))
        subs.append((group.mexp_submit(bases, e, [(k_t, v), (k8, og.q - e % og.q)]),
                     pow(prod, e, og.p) * pow(K, v, og.p) * pow(K2, og.q - e % og.q, og.p) % og.p))
        subs.append((group.mexp_submit(bases, e), pow(prod, e, og.p)))
        subs.append((group.mexp_submit(bases), prod))
    bad = [i for i, (t, want) in enumerate(subs) if int.from_bytes(t.wait(), "big") != want]
    assert not bad, bad[:8]


def test_table_destroyed_with_jobs_queued(group, oracle_group):
    """eg_fixed_base_destroy on a table with per-element jobs still queued waits until their batch
    has run: the jobs complete bit-exact and no batch reads a freed table."""
    og = oracle_group
    rng = random.Random(31)
    K = pow(og.g, rng.randrange(og.q), og.p)
    fb = group.fixed_base(K, 8)
    es = [rng.randrange(og.q) for _ in range(40)]
    import time
    # a FIXED 20 ms window (honoured exactly), and eg_ctx_set_coalescing makes the next batch wait for
    # max_batch jobs or the window: the 40 jobs are still queued at the close
    group.set_coalescing(4096, 20000)
    try:
        t = time.monotonic()
        ts = [group.mexp_submit([], None, [(fb, e)]) for e in es]
        fb.close()
        waited = time.monotonic() - t
        got = [int.from_bytes(t.wait(), "big") for t in ts]
    finally:
        group.set_coalescing(16384, 0)  # the library default (adaptive window)
    assert got == [pow(K, e, og.p) for e in es]
    assert waited >= 0.015, f"close returned after {waited * 1e3:.1f} ms: the jobs were not queued"


@pytest.mark.parametrize("ct", [False, True])
@pytest.mark.parametrize("n", [1, 3, 256])
def test_fixed_base_batches_on_eight_waves(group, oracle_group, tables, n, ct):
    """Batches without a variable exponent, of at most one job per CU, split their fixed-base windows
    over 8 waves (two per SIMD): one and two fixed-base terms, a product of bases times a term (wave 0
    takes the product, seven waves the windows), edge exponents; every result equals CPython's."""
    og = oracle_group
    rng = random.Random(808 + n + 1000 * ct)
    g_t, k_t, k8 = tables["g"][0], tables["K12"][0], tables["K8"][0]
    K, K2 = tables["K12"][1], tables["K8"][1]
    edges = _edges(og)
    group.ct_pow = ct
    try:
        subs = []
        for i in range(n):
            a = edges[i % len(edges)] if i < 2 * len(edges) else rng.randrange(og.q)
            b = rng.randrange(og.q)
            kind = i % 4
            if kind == 0:
                subs.append((group.mexp_submit([], None, [(k8, a)]), pow(K2, a, og.p)))
            elif kind == 1:
                subs.append((group.mexp_submit([], None, [(g_t, a), (k8, b)]), pow(og.g, a, og.p) * pow(K2, b, og.p) % og.p))
            elif kind == 2:  # constant time: the 12-bit table takes its 6-bit companion
                subs.append((group.mexp_submit([], None, [(k_t, a), (g_t, b)]), pow(K, a, og.p) * pow(og.g, b, og.p) % og.p))
            else:
                al = rng.randrange(og.p)
                subs.append((group.mexp_submit([al], None, [(g_t, a)]), al * pow(og.g, a, og.p) % og.p))
        bad = [i for i, (t, want) in enumerate(subs) if int.from_bytes(t.wait(), "big") != want]
    finally:
        group.ct_pow = False
    assert not bad, bad[:8]
