"""Generate the two non-production Schnorr groups the GPU verifier is tested on
(tests/test_gpu_test_groups.py), written to tests/golden/test_groups.json.

Both are 4096-bit p = k*q + 1 with a prime q < 2^256 (255 bits for sparse c) and
g = 2^((p-1)/q) mod p, so neither p is Montgomery-friendly (the verifier runs its general-p CIOS instantiation). They differ
in c = 2^256 - q, the public exponent of the residue test x^(2^256) == x^c:
  * "sparse_c": c has 12 set bits, some at the comb chain's table positions (26, 52, 208)
    and some past them (240, 255): w = x^c is built from the chain's stored powers;
  * "dense_c": q is a random 256-bit prime, c has ~128 set bits: the op-program compiler
    falls back to a left-to-right ladder for w.
Run:  python tests/golden/make_test_groups.py   (deterministic; about a minute of CPython)
"""
import json
import random
from pathlib import Path

HERE = Path(__file__).resolve().parent
SMALL = [p for p in range(3, 20000) if all(p % d for d in range(2, int(p ** 0.5) + 1))]


def is_probable_prime(n: int, rng: random.Random, rounds: int = 24) -> bool:
    if n < 2:
        return False
    for sp in SMALL[:200]:
        if n % sp == 0:
            return n == sp
    d, s = n - 1, 0
    while d % 2 == 0:
        d //= 2
        s += 1
    for _ in range(rounds):
        a = rng.randrange(2, n - 2)
        x = pow(a, d, n)
        if x in (1, n - 1):
            continue
        for _ in range(s - 1):
            x = x * x % n
            if x == n - 1:
                break
        else:
            return False
    return True


def schnorr_p(q: int, rng: random.Random) -> int:
    """Smallest p = k*q + 1 >= a random 4096-bit start with k even, p prime (sieved)."""
    k = rng.randrange(2 ** 4095 // q, 2 ** 4096 // q) & ~1
    while True:
        p = k * q + 1
        if p.bit_length() == 4096 and all(p % sp for sp in SMALL) and is_probable_prime(p, rng):
            return p
        k += 2


def make(name: str, q: int, rng: random.Random) -> dict:
    p = schnorr_p(q, rng)
    g = pow(2, (p - 1) // q, p)
    assert g != 1 and pow(g, q, p) == 1
    c = 2 ** 256 - q
    return {"name": name, "p": p.to_bytes(512, "big").hex(), "q": q.to_bytes(32, "big").hex(),
            "g": g.to_bytes(512, "big").hex(), "c_popcount": bin(c).count("1")}


def main():
    rng = random.Random(20261017)
    groups = []
    fixed = [0, 3, 26, 52, 99, 131, 160, 208, 240, 255]
    while True:  # sparse c: the fixed bits plus two random ones, q = 2^256 - c prime
        bits = set(fixed) | {rng.randrange(1, 256) for _ in range(2)}
        c = sum(1 << b for b in bits)
        if len(bits) == 12 and is_probable_prime(2 ** 256 - c, rng):
            break
    groups.append(make("sparse_c", 2 ** 256 - c, rng))
    while True:  # dense c: a random 256-bit prime q
        q = rng.randrange(2 ** 255, 2 ** 256) | 1
        if is_probable_prime(q, rng) and bin(2 ** 256 - q).count("1") > 64:
            break
    groups.append(make("dense_c", q, rng))
    (HERE / "test_groups.json").write_text(json.dumps({"groups": groups}, indent=1) + "\n")
    for gr in groups:
        print(gr["name"], "popcount(c) =", gr["c_popcount"])


if __name__ == "__main__":
    main()
