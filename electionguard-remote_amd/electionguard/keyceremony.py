"""Synthetic key ceremony — produces the inputs the hot path needs (joint key K,
guardian secrets and polynomial shares).  The reference's remote key ceremony
(src/main/java/electionguard/keyceremony/, RunRemoteKeyCeremony.java:200-233) is out
of scope; this restates only its outputs: guardian i (x-coordinate
i, RunRemoteKeyCeremony.java:268) holds a degree-(quorum-1) polynomial P_i with
secret s_i = P_i(0), public commitments K_ij = g^{a_ij} (computed on the GPU), and
the shares P_l(x_i) of every other guardian l, both in the clear (``shares_from``, for
tests and callers that hold decrypted shares) and as the key ceremony's encrypted backups
(``backups_from``: HashedElGamal under K_i), which the trustee decrypts
in ``compensatedDecrypt``.  K = prod_i K_i0.
"""
from __future__ import annotations

import hashlib
import hmac
import secrets
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import numpy as np

from .core.group import GroupContext, p_bytes


@dataclass
class GuardianKeys:
    gid: str
    x: int
    coeffs: List[int]
    commitments: List[int]                       # g^{a_j}
    shares_from: Dict[str, int] = field(default_factory=dict)  # l -> P_l(x)
    backups_from: Dict[str, Tuple[int, bytes, bytes]] = field(default_factory=dict)  # l -> (c0, c1, c2)

    @property
    def secret(self) -> int:
        return self.coeffs[0]

    @property
    def public_key(self) -> int:
        return self.commitments[0]


def poly_eval(coeffs: List[int], x: int, q: int) -> int:
    acc = 0
    for a in reversed(coeffs):
        acc = (acc * x + a) % q
    return acc


# Share backups: the upstream HashedElGamalCiphertext layout is not in the container
# (unpinned); this build defines it, identically to oracle/eg_oracle.py (backup_encrypt):
#   c0 = g^r, k = K_i^r = c0^{s_i}, kk = SHA256(c0 || k), stream / mac_key = HMAC(kk, 1|2 ...),
#   c1 = P_l(x_i) XOR stream (32 B), c2 = HMAC-SHA256(mac_key, c0 || c1).
def backup_label(from_gid: str, to_gid: str) -> bytes:
    return from_gid.encode() + b"|" + to_gid.encode()


def backup_keys(c0: int, k: int, label: bytes) -> Tuple[bytes, bytes]:
    kk = hashlib.sha256(p_bytes(c0) + p_bytes(k)).digest()
    return (hmac.new(kk, b"\x01share" + label, hashlib.sha256).digest(),
            hmac.new(kk, b"\x02share" + label, hashlib.sha256).digest())


def backup_open(c0: int, k: int, c1: bytes, c2: bytes, label: bytes) -> Optional[int]:
    """Share from a backup given k = c0^{s_i} (computed on the GPU by the caller); None on a bad MAC."""
    stream, mac_key = backup_keys(c0, k, label)
    if not hmac.compare_digest(c2, hmac.new(mac_key, p_bytes(c0) + c1, hashlib.sha256).digest()):
        return None
    return int.from_bytes(bytes(a ^ b for a, b in zip(c1, stream)), "big")


def key_ceremony(group: GroupContext, n: int, quorum: int, seed: Optional[int] = None):
    """-> (guardians, K).  Coefficients from a seeded RNG (tests) or `secrets`."""
    if not (1 <= quorum <= n):
        raise ValueError("need 1 <= quorum <= n")
    q = group.q
    if seed is None:
        draw = lambda: secrets.randbelow(q - 1) + 1
    else:
        import random

        r = random.Random(seed)
        draw = lambda: r.randrange(1, q)
    coeffs = [[draw() for _ in range(quorum)] for _ in range(n)]
    flat = [a for co in coeffs for a in co]
    comm = group.gPowP_batch(flat)
    gs = []
    for i in range(n):
        cm = [int.from_bytes(comm[i * quorum + j].tobytes(), "big") for j in range(quorum)]
        gs.append(GuardianKeys(f"guardian{i + 1}", i + 1, coeffs[i], cm))
    pairs = [(gl, gi) for gi in gs for gl in gs if gl.gid != gi.gid]
    for gl, gi in pairs:
        gi.shares_from[gl.gid] = poly_eval(gl.coeffs, gi.x, q)
    if pairs:  # encrypted backups: c0 = g^r and k = K_i^r, one GPU batch each
        rs = [draw() for _ in pairs]
        c0s = group.gPowP_batch(rs)
        ks = group.powP_batch([gi.public_key for _, gi in pairs], rs)
        for (gl, gi), c0b, kb in zip(pairs, c0s, ks):
            c0, k = int.from_bytes(c0b.tobytes(), "big"), int.from_bytes(kb.tobytes(), "big")
            label = backup_label(gl.gid, gi.gid)
            stream, mac_key = backup_keys(c0, k, label)
            c1 = bytes(a ^ b for a, b in zip(gi.shares_from[gl.gid].to_bytes(32, "big"), stream))
            gi.backups_from[gl.gid] = (c0, c1, hmac.new(mac_key, p_bytes(c0) + c1, hashlib.sha256).digest())
    Ks = np.stack([np.frombuffer(p_bytes(g.public_key), dtype=np.uint8) for g in gs])
    K = int.from_bytes(group.prodP_groups(Ks, 1, n)[0].tobytes(), "big")
    return gs, K
