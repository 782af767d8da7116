"""Fiat-Shamir hash (host side, for the few proofs hashed outside the GPU kernels).

EG 1.0-style ``hash_elems``: SHA-256 over "|" + "|".join(upper-case hex) + "|", big-endian,
reduced mod q.  The hex form is the context's hash format (eg_ctx_set_hash_format):
  "fixed"   (default) ElementModP -> 1024 hex chars, ElementModQ -> 64 (common.proto:6-16);
  "minimal" the integer's even-length hex (leading zero bytes dropped, 0 -> "00"), as
            electionguard-python 1.x's to_hex.
Identical to the device implementation in csrc/eg_sha256.hpp; the upstream pre-image format
is not in the container (unpinned), hence the switch.
"""
from __future__ import annotations

import hashlib

from .constants import P_BYTES, Q_BYTES

FORMATS = {"fixed": 0, "minimal": 1}  # EG_HASH_FIXED_WIDTH, EG_HASH_MINIMAL (include/eg_hip.h)


def _hex(x: int, width: int, fmt: str) -> str:
    b = int(x).to_bytes(width, "big")
    if fmt == "minimal":
        b = b.lstrip(b"\0") or b"\0"
    elif fmt != "fixed":
        raise ValueError(f"unknown hash format {fmt!r}")
    return b.hex().upper()


def hexP(x: int, fmt: str = "fixed") -> str:
    return _hex(x, P_BYTES, fmt)


def hexQ(x: int, fmt: str = "fixed") -> str:
    return _hex(x, Q_BYTES, fmt)


def hash_elems(q: int, *elems, fmt: str = "fixed") -> int:
    """elems: ("P"|"Q", int) pairs."""
    parts = [hexP(v, fmt) if kind == "P" else hexQ(v, fmt) for kind, v in elems]
    msg = ("|" + "|".join(parts) + "|").encode("ascii")
    return int.from_bytes(hashlib.sha256(msg).digest(), "big") % q
