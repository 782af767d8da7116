"""Synthetic key ceremony — produces the inputs the hot path needs (joint key K,
guardian secrets and polynomial shares).  The reference's remote key ceremony
(src/main/java/electionguard/keyceremony/, RunRemoteKeyCeremony.java:200-233) is out
of scope; this restates only its outputs: guardian i (x-coordinate
i, RunRemoteKeyCeremony.java:268) holds a degree-(quorum-1) polynomial P_i with
secret s_i = P_i(0), public commitments K_ij = g^{a_ij} (computed on the GPU), and
the shares P_l(x_i) of every other guardian l.  K = prod_i K_i0.
"""
from __future__ import annotations

import secrets
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

from .core.group import GroupContext, p_bytes


@dataclass
class GuardianKeys:
    gid: str
    x: int
    coeffs: List[int]
    commitments: List[int]                       # g^{a_j}
    shares_from: Dict[str, int] = field(default_factory=dict)  # l -> P_l(x)

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
    for gi in gs:
        for gl in gs:
            if gl.gid != gi.gid:
                gi.shares_from[gl.gid] = poly_eval(gl.coeffs, gi.x, q)
    Ks = np.stack([np.frombuffer(p_bytes(g.public_key), dtype=np.uint8) for g in gs])
    K = int.from_bytes(group.prodP_groups(Ks, 1, n)[0].tobytes(), "big")
    return gs, K
