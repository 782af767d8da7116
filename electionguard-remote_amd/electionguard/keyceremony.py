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

from .core.group import GroupContext, as_p_array, p_bytes
from .core.hashing import hash_elems


@dataclass
class GuardianKeys:
    gid: str
    x: int
    coeffs: List[int]
    commitments: List[int]                       # g^{a_j}
    shares_from: Dict[str, int] = field(default_factory=dict)  # l -> P_l(x)
    backups_from: Dict[str, Tuple[int, bytes, bytes]] = field(default_factory=dict)  # l -> (c0, c1, c2)
    proofs: List[Tuple[int, int]] = field(default_factory=list)  # Schnorr (c, v) per commitment

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
    # Schnorr proofs of every coefficient (h = g^u on the GPU, hash on the host)
    us = [draw() for _ in flat]
    hs = group.gPowP_batch(us)
    for i, gi in enumerate(gs):
        for j in range(quorum):
            k = i * quorum + j
            c = hash_elems(q, ("P", gi.commitments[j]), ("P", int.from_bytes(hs[k].tobytes(), "big")),
                           fmt=group.hash_format)
            gi.proofs.append((c, (us[k] - c * gi.coeffs[j]) % q))
    Ks = np.stack([np.frombuffer(p_bytes(g.public_key), dtype=np.uint8) for g in gs])
    K = int.from_bytes(group.prodP_groups(Ks, 1, n)[0].tobytes(), "big")
    return gs, K


def _be(row) -> int:
    return int.from_bytes(row.tobytes(), "big")


def verify_commitment_proofs(group: GroupContext, commitments: List[int], proofs: List[Tuple[int, int]]) -> List[bool]:
    """Schnorr proofs of the public commitments K_ij (what each guardian checks of the others
    in the key ceremony), one GPU batch: K^q == 1, h = g^v K^c, c == H(K, h).  Same
    definition as oracle/eg_oracle.py (schnorr_verify)."""
    n = len(commitments)
    if len(proofs) != n:
        raise ValueError("one proof per commitment")
    if not n:
        return []
    q, p = group.q, group.p
    Ks = as_p_array(commitments)
    res = group.powP_batch(np.concatenate([Ks, Ks]), [q] * n + [c for c, _ in proofs])
    h = group.multP_batch(group.gPowP_batch([v for _, v in proofs]), res[n:])
    out = []
    for k in range(n):
        c, v = proofs[k]
        K = commitments[k]
        ok = 0 < K < p and 0 <= c < q and 0 <= v < q and _be(res[k]) == 1
        out.append(bool(ok and c == hash_elems(q, ("P", K), ("P", _be(h[k])), fmt=group.hash_format)))
    return out


def verify_backups(group: GroupContext, keys: GuardianKeys, all_commitments: Dict[str, List[int]]) -> Dict[str, bool]:
    """A recipient's check of every backup it holds (key ceremony, receiving side): the backup
    opens under its secret (k = c0^{s_i}, one GPU batch) and the share matches the sender's
    commitments, g^{P_l(x_i)} == prod_j K_lj^{x_i^j} (two GPU batches + one product)."""
    ids = sorted(keys.backups_from)
    if not ids:
        return {}
    q = group.q
    ks = group.powP_batch([keys.backups_from[l][0] for l in ids], [keys.secret] * len(ids))
    shares = [backup_open(keys.backups_from[l][0], _be(ks[t]), keys.backups_from[l][1], keys.backups_from[l][2],
                          backup_label(l, keys.gid)) for t, l in enumerate(ids)]
    quorum = len(all_commitments[ids[0]])
    if any(len(all_commitments[l]) != quorum for l in ids):
        raise ValueError("all guardians commit to quorum coefficients")
    xe = [pow(keys.x, j, q) for j in range(quorum)]
    terms = group.powP_batch([K for l in ids for K in all_commitments[l]], xe * len(ids))
    rk = group.prodP_groups(terms, len(ids), quorum)
    gs = group.gPowP_batch([s if s is not None else 0 for s in shares])
    return {l: shares[t] is not None and _be(gs[t]) == _be(rk[t]) for t, l in enumerate(ids)}
