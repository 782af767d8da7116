"""CPU: the per-wave kernel's delayed-quotient Montgomery multiply (eg_pow16.hip, egw::mul_d2),
restated on whole columns, against the per-step CIOS (egw::mul) and against x*y*R^-1 mod p.

mul_d2 needs p = -1 mod 2^58: with p~ = p + 1 (low two limbs zero) it adds m_i * p~ two steps
late (p~ shifted down by two limbs) and drops the retiring column's low 29 bits (= m_i, the
"- m_i" of m_i * p = m_i * p~ - m_i).  The quotient digits must come out identical to the
per-step CIOS ones, and so must the product integer.  Checked for the production p (p = -1 mod
2^256) and for a modulus that is -1 mod 2^58 only (p~_2 != 0: the delayed term lands in the
lowest column before its quotient is read)."""
import random

import pytest

B, N = 29, 144
MASK = (1 << B) - 1
R = 1 << (B * N)


def limbs(v, n=N + 3):
    return [(v >> (B * i)) & MASK for i in range(n)]


def value(cols):
    return sum(c << (B * i) for i, c in enumerate(cols))


def cios(x, y, p):
    """per-step quotient (mul<F>): the digits and the result integer"""
    xl, yl, pl = limbs(x), limbs(y), limbs(p)
    T = [0] * (N + 4)
    ms = []
    for i in range(N):
        for j in range(N):
            T[j] += xl[j] * yl[i]
        m = (T[0] * (-pow(p, -1, 1 << B))) & MASK
        ms.append(m)
        for j in range(N):
            T[j] += m * pl[j]
        assert T[0] & MASK == 0
        c = T[0] >> B
        T = T[1:] + [0]
        T[0] += c
    return ms, value(T)


def delayed(x, y, p):
    """mul_d2: m_i applied at step i + 2 against p~ shifted by two limbs, the tail after the loop"""
    xl, yl = limbs(x), limbs(y)
    pt = limbs(p + 1)
    assert pt[0] == 0 and pt[1] == 0, "needs p = -1 mod 2^58"
    pd = [pt[k + 2] if k + 2 < N else 0 for k in range(N)]
    pd1 = [pt[k + 1] if k + 1 < N else 0 for k in range(N)]
    T = [0] * (N + 4)
    ms, m1, m2 = [], 0, 0
    for i in range(N):
        for j in range(N):
            T[j] += xl[j] * yl[i]
        for j in range(N):
            T[j] += pd[j] * m2
        m = T[0] & MASK          # readlane of lane 0's lowest column
        ms.append(m)
        c = T[0] >> B            # the carry; the low bits (= m) are dropped by the lane shift
        T = T[1:] + [0]
        T[0] += c
        m2, m1 = m1, m
    for j in range(N):
        T[j] += pd[j] * m2 + pd1[j] * m1
    return ms, value(T)


@pytest.mark.parametrize("kind", ["production", "minus1_mod_2_58_only"])
def test_delayed_quotient_matches_cios(kind):
    import eg_oracle as O
    rng = random.Random(58)
    if kind == "production":
        p = O.production_group().p
    else:
        # an odd 4096-bit modulus with exactly 58 low one-bits (bit 58 clear): p~_2 != 0
        while True:
            p = (rng.getrandbits(4096 - 59) << 59) | ((1 << 58) - 1) | (1 << 4095)
            if (p >> 58) & 1 == 0 and limbs(p + 1)[2] != 0:
                break
    assert (p + 1) % (1 << 58) == 0
    rinv = pow(R, -1, p)
    for _ in range(6):
        x, y = rng.randrange(2 * p), rng.randrange(2 * p)
        ms_a, a = cios(x, y, p)
        ms_b, b = delayed(x, y, p)
        assert ms_a == ms_b          # the same quotient digits
        assert a == b                # the same integer (xy + M p) / R
        assert a < 2 * p and a % p == x * y * rinv % p
