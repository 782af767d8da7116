"""Fiat-Shamir hash (host side, for the few proofs hashed outside the GPU kernels).

EG 1.0-style ``hash_elems``: SHA-256 over "|" + "|".join(fixed-width upper-case hex)
+ "|", big-endian, reduced mod q.  ElementModP -> 1024 hex chars, ElementModQ -> 64
(common.proto:6-16).  Identical to the device implementation in
csrc/eg_sha256.hpp; the upstream pre-image format is not in the container
(unpinned).
"""
from __future__ import annotations

import hashlib

from .constants import P_BYTES, Q_BYTES


def hexP(x: int) -> str:
    return int(x).to_bytes(P_BYTES, "big").hex().upper()


def hexQ(x: int) -> str:
    return int(x).to_bytes(Q_BYTES, "big").hex().upper()


def hash_elems(q: int, *elems) -> int:
    """elems: ("P"|"Q", int) pairs."""
    parts = [hexP(v) if kind == "P" else hexQ(v) for kind, v in elems]
    msg = ("|" + "|".join(parts) + "|").encode("ascii")
    return int.from_bytes(hashlib.sha256(msg).digest(), "big") % q
