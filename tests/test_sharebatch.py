"""CPU: ShareBatch, the trustee result kept in wire form (decrypt.py).  It must behave as the
List<DirectDecryptionAndProof> / List<CompensatedDecryptionAndProof> DecryptingTrusteeIF returns
(RemoteDecryptingTrusteeProxy.java:48-53, 84-90): in-order indexing, field reads, and the edits a
record check is tested with (a share's field rewritten in place, a share replaced), while the
mediator reads its arrays without per-share conversion."""
import copy
import random

import numpy as np
import pytest


def _batch(n, rng, recovery=False):
    from electionguard.decrypt import ShareBatch
    M = [rng.getrandbits(4095) for _ in range(n)]
    cv = [(rng.getrandbits(255), rng.getrandbits(255)) for _ in range(n)]
    Ma = np.frombuffer(b"".join(m.to_bytes(512, "big") for m in M), np.uint8).reshape(n, 512).copy()
    pa = np.frombuffer(b"".join(c.to_bytes(32, "big") + v.to_bytes(32, "big") for c, v in cv),
                       np.uint8).reshape(n, 2, 32).copy()
    rk = rng.getrandbits(4095)
    ra = np.tile(np.frombuffer(rk.to_bytes(512, "big"), np.uint8), (n, 1)) if recovery else None
    return ShareBatch(Ma, pa, ra), M, cv, rk


def test_reads_match_the_share_objects():
    from electionguard.decrypt import (CompensatedDecryptionAndProof, DirectDecryptionAndProof,
                                       GenericChaumPedersenProof)
    rng = random.Random(3)
    b, M, cv, _ = _batch(7, rng)
    assert len(b) == 7
    want = [DirectDecryptionAndProof(m, GenericChaumPedersenProof(c, v)) for m, (c, v) in zip(M, cv)]
    assert [(r.partialDecryption, r.proof.c, r.proof.v) for r in b] == [(m, c, v) for m, (c, v) in zip(M, cv)]
    assert b == want and b[-1] == want[-1] and b[2:4] == want[2:4]
    with pytest.raises(IndexError):
        b[7]
    cb, M2, cv2, rk = _batch(4, rng, recovery=True)
    assert cb == [CompensatedDecryptionAndProof(m, GenericChaumPedersenProof(c, v), rk) for m, (c, v) in zip(M2, cv2)]
    assert all(r.recoveredPublicKeyShare == rk for r in cb)
    with pytest.raises(AttributeError):
        b[0].recoveredPublicKeyShare


def test_edits_write_through_and_deepcopy_isolates():
    from electionguard.decrypt import CompensatedDecryptionAndProof, GenericChaumPedersenProof, share_arrays
    rng = random.Random(4)
    b, M, cv, rk = _batch(5, rng, recovery=True)
    bad = copy.deepcopy(b)
    d = bad[2]
    d.partialDecryption = d.partialDecryption * 3 % (1 << 4095)
    assert bad[2].partialDecryption == M[2] * 3 % (1 << 4095) and b[2].partialDecryption == M[2]
    c = bad[0]
    bad[0] = CompensatedDecryptionAndProof(c.partialDecryption, c.proof, rk + 1)
    assert bad[0].recoveredPublicKeyShare == rk + 1 and b[0].recoveredPublicKeyShare == rk
    bad[1].proof = GenericChaumPedersenProof(5, 6)
    assert (bad[1].proof.c, bad[1].proof.v) == (5, 6)
    Ma, pa, ra = share_arrays(bad)
    assert int.from_bytes(ra[0].tobytes(), "big") == rk + 1 and int.from_bytes(pa[1, 0].tobytes(), "big") == 5
    # the list form packs to the same arrays
    Ml, pl, rl = share_arrays(list(bad))
    assert np.array_equal(Ml, Ma) and np.array_equal(pl, pa) and np.array_equal(rl, ra)
    assert share_arrays([])[0].shape == (0, 512)
