"""Parity of the group-level ops (GroupContext / ElementModP, KUtils.java:10-12) on the
GPU, through the C ABI, against the CPU oracle (CPython int == BigInteger semantics)."""
import random

import numpy as np
import pytest

from conftest import be2i

pytestmark = pytest.mark.gpu


def test_powp_random(group, oracle_group):
    O = oracle_group
    rng = random.Random(1)
    n = 67  # ragged: not a multiple of the 32 elements of a workgroup
    bases = [rng.randrange(2**4096) for _ in range(n)]  # includes values >= p (reduced, like BigInteger)
    exps = [rng.randrange(2**256) for _ in range(n)]    # exponents used as given (not reduced mod q)
    out = group.powP_batch(bases, exps)
    for i in range(n):
        assert be2i(out[i]) == O.powP(bases[i], exps[i]), i


def test_powp_edges(group, oracle_group):
    O = oracle_group
    p, q = O.p, O.q
    bases = [0, 0, 1, p - 1, p, p + 1, 2**4096 - 1, O.g, 2, p - 1]
    exps = [0, 5, 2**256 - 1, 2, 7, 3, 2**256 - 1, q, q - 1, 0]
    out = group.powP_batch(bases, exps)
    for i in range(len(bases)):
        assert be2i(out[i]) == O.powP(bases[i], exps[i]), (i, bases[i] % p, exps[i])


def test_powp_empty(group):
    assert group.powP_batch(np.empty((0, 512), np.uint8), np.empty((0, 32), np.uint8)).shape == (0, 512)


def test_gpowp_fixed_base(group, oracle_group):
    O = oracle_group
    rng = random.Random(2)
    exps = [0, 1, 2, O.q - 1, 2**256 - 1] + [rng.randrange(O.q) for _ in range(40)]
    out = group.gPowP_batch(exps)
    for i, e in enumerate(exps):
        assert be2i(out[i]) == O.gPowP(e), i


@pytest.mark.parametrize("wbits", [4, 11, 16])
def test_fixed_base_windows(group, oracle_group, wbits):
    O = oracle_group
    rng = random.Random(wbits)
    base = rng.randrange(O.p)
    fb = group.fixed_base(base, window_bits=wbits)
    exps = [0, 1, O.q - 1, 2**256 - 1] + [rng.randrange(O.q) for _ in range(20)]
    out = fb.pow_batch(exps)
    for i, e in enumerate(exps):
        assert be2i(out[i]) == O.powP(base, e), i
    fb.close()


def test_multp(group, oracle_group):
    O = oracle_group
    rng = random.Random(3)
    a = [rng.randrange(2**4096) for _ in range(50)] + [0, O.p, O.p - 1]
    b = [rng.randrange(2**4096) for _ in range(50)] + [5, 3, O.p - 1]
    out = group.multP_batch(a, b)
    for i in range(len(a)):
        assert be2i(out[i]) == O.multP(a[i], b[i]), i


def test_prod_reduce(group, oracle_group):
    O = oracle_group
    rng = random.Random(4)
    for groups, length in [(3, 1), (5, 7), (2, 100), (1, 33)]:
        xs = [rng.randrange(O.p) for _ in range(groups * length)]
        out = group.prodP_groups(xs, groups, length)
        for g in range(groups):
            assert be2i(out[g]) == O.prodP(xs[g * length:(g + 1) * length]), (groups, length, g)


def test_multinv(group, oracle_group):
    O = oracle_group
    rng = random.Random(5)
    xs = [1, O.p - 1, 2] + [rng.randrange(1, O.p) for _ in range(5)]
    out = group.multInv_batch(xs)
    for i, x in enumerate(xs):
        assert be2i(out[i]) == O.multInv(x), i


def test_generic_odd_modulus(oracle_group):
    """A non-Montgomery-friendly odd 4096-bit modulus exercises the general CIOS path."""
    from electionguard.core import GroupContext
    rng = random.Random(6)
    p = rng.randrange(2**4095, 2**4096) | 1
    g = 3
    G = GroupContext(p, oracle_group.q, g)
    bases = [rng.randrange(2**4096) for _ in range(20)]
    exps = [rng.randrange(2**256) for _ in range(20)]
    out = G.powP_batch(bases, exps)
    for i in range(20):
        assert be2i(out[i]) == pow(bases[i] % p, exps[i], p), i
    gout = G.gPowP_batch(exps)
    for i in range(20):
        assert be2i(gout[i]) == pow(g, exps[i], p), i
    G.close()


def test_powp_and_fb_dev_pointers(group, oracle_group):
    """eg_powp_batch_dev / eg_fb_pow_batch_dev (operands resident in HBM, libeg_hip device buffers'
    data_ptr()): same results as the host-pointer calls and the oracle, incl. edge cases,
    a ragged size and a second call that reuses the cached job table."""
    O = oracle_group
    rng = random.Random(23)
    p, q = O.p, O.q
    bases = [0, 0, 1, p - 1, p, p + 1, 2**4096 - 1, O.g] + [rng.randrange(2**4096) for _ in range(91)]
    exps = [0, 5, 2**256 - 1, 2, 7, 3, 2**256 - 1, q] + [rng.randrange(2**256) for _ in range(91)]
    n = len(bases)
    B = np.stack([np.frombuffer(b.to_bytes(512, "big"), np.uint8) for b in bases])
    E = np.stack([np.frombuffer(e.to_bytes(32, "big"), np.uint8) for e in exps])
    dB, dE = group.to_device(B), group.to_device(E)
    dO = group.device_zeros((n, 512))
    for _ in range(2):
        dO.zero()
        group.powP_batch_dev(dB.ptr, dE.ptr, dO.ptr, n)
        group.sync()
        out = dO.download()
        for i in range(n):
            assert be2i(out[i]) == O.powP(bases[i], exps[i]), i
    group.gPowP_batch_dev(dE.ptr, dO.ptr, n)
    group.sync()
    out = dO.download()
    for i in range(n):
        assert be2i(out[i]) == O.gPowP(exps[i]), i
    fb = group.fixed_base(bases[20], window_bits=9)
    fb.pow_batch_dev(dE.ptr, dO.ptr, 33)
    group.sync()
    out = dO.download()
    for i in range(33):
        assert be2i(out[i]) == O.powP(bases[20], exps[i]), i
    fb.close()


def test_profile_counts_and_clock(group):
    """eg_ctx_profile_end counts the k_pow work of the window from the op programs, and
    eg_ctx_profile_clock reports the shader clock it ran at (median per-workgroup s_memtime
    over s_memrealtime ticks, every record usable): a 4-bit-window powP is 14 table MMs +
    63 x (4 sq + 1 mul).  Batches up to half a resident 16-lane round run on the latency layouts
    (eg_pow16.hip, not k_pow: nothing to count), so the counted batch is larger (and within one
    8-lane round: one launch)."""
    rng = np.random.default_rng(5)
    small = rng.integers(0, 256, size=(64, 512), dtype=np.uint8)
    group.profile_begin()
    group.powP_batch(small, rng.integers(0, 256, size=(64, 32), dtype=np.uint8))
    assert group.profile_end().launches == 0
    n = 20000
    bases = rng.integers(0, 256, size=(n, 512), dtype=np.uint8)
    bases[:, 0] = 0
    exps = rng.integers(0, 256, size=(n, 32), dtype=np.uint8)
    group.profile_begin()
    group.powP_batch(bases, exps)
    kp = group.profile_end()
    assert kp.launches == 1
    assert kp.mont_ops == n * (14 + 63 * 5) and kp.squarings == n * 63 * 4
    assert kp.ms > 0 and 1.0 <= kp.clock_ghz <= 2.6, kp
    assert kp.clock_records == (n + 31) // 32 and kp.clock_dropped == 0, kp


@pytest.mark.parametrize("n", [1, 9, 3000])
def test_multinv_subgroup_first(group, oracle_group, n):
    """eg_multinv_batch tries a^(q-1) (the inverse inside the order-q subgroup: a 256-bit exponent),
    checks r * a == 1 and sends the rest to a^(p-2): subgroup elements, elements outside it (random
    residues, p - 1 of order 2), unreduced inputs and 0 (-> 0, a^(p-2)) all come back exact, at the
    latency shapes (n = 1, 9) and on the 8-lane batch layout (n = 3000)."""
    O = oracle_group
    rng = random.Random(50 + n)
    xs = []
    for i in range(n):
        k = rng.random()
        if k < 0.5:
            xs.append(pow(O.g, rng.randrange(O.q), O.p))
        elif k < 0.8:
            xs.append(rng.randrange(1, O.p))
        else:
            xs.append(rng.choice([1, O.p - 1, 0, O.p + 1, O.p + 2, 2**4096 - 1]))
    if n == 1:
        xs = [pow(O.g, rng.randrange(O.q), O.p)]
    out = group.multInv_batch(xs)
    for i, x in enumerate(xs):
        want = 0 if x % O.p == 0 else O.multInv(x)
        assert be2i(out[i]) == want, (i, x % O.p == 0)
