"""ConvertCommonProto analog (src/main/java/electionguard/util/ConvertCommonProto.java).

The wire layout is the protobuf ``bytes value`` of ElementModP (512 B big-endian,
common.proto:6-10) and ElementModQ (32 B, common.proto:12-16).  Import is unchecked
(``new BigInteger(1, bytes)``, :41-57): values >= p are accepted and reduced by the
group ops.  Export is ``byteArray()`` (:111-121).  Unlike BigInteger.toByteArray the
export here is always fixed width (leading zeros kept), matching the 512/32-byte
fields every GPU batch uses.
"""
from __future__ import annotations

from typing import Optional

from .core.group import ElementModP, ElementModQ, GroupContext, p_bytes, q_bytes


def importElementModP(group: GroupContext, value: Optional[bytes]) -> Optional[ElementModP]:
    if not value:
        return None  # ConvertCommonProto.java:51-53
    return ElementModP(int.from_bytes(value, "big"), group)


def importElementModQ(group: GroupContext, value: Optional[bytes]) -> Optional[ElementModQ]:
    if not value:
        return None  # :42-44
    return ElementModQ(int.from_bytes(value, "big"), group)


def publishElementModP(e: ElementModP) -> bytes:
    return p_bytes(e.value)


def publishElementModQ(e: ElementModQ) -> bytes:
    return q_bytes(e.value)
