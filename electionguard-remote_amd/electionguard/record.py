"""Election-record verification: the reference's last workflow step,
``new Verifier(record, 11).verify()`` (RunRemoteWorkflowTest.java:179-182; the Verifier is
upstream, electionguard-kotlin-multiplatform-jvm), over the parts of the record the hot
path produces.  Every exponentiation runs on the GPU through the C ABI:

  * ``guardian_proofs``  Schnorr proofs of every guardian's coefficient commitments
                         (keyceremony.verify_commitment_proofs);
  * ``joint_key``        K == prod_i K_i0;
  * ``ballots``          every disjunctive and contest proof of every ballot (eg_verify_ballots);
  * ``tally``            the published encrypted tally == the product of the CAST ballots'
                         ciphertexts per real selection (runAccumulateBallots, :151);
  * ``decryption.*``     decrypt.verify_decryption_record (share proofs, recovery keys,
                         quorum, B == M g^t, counts <= the number of cast ballots);
  * ``spoiled.*``        with spoiled ballots (``cast`` flags): their decryption record covers
                         exactly their real selections (``spoiled.texts``) and passes the same
                         share / quorum / B == M g^t checks with values <= votesAllowed
                         (decryptBallot, RunRemoteDecryptor.java:264-269).

Manifest, hash-chain and protobuf-format checks are record plumbing outside the hot path
 and are not restated.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np

from .ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
from .core.group import GroupContext, as_p_array
from .decrypt import DecryptionRecord, spoiled_texts, verify_decryption_record
from .keyceremony import verify_commitment_proofs


@dataclass
class GuardianRecord:
    gid: str
    x: int
    commitments: List[int]          # K_ij = g^{a_ij}
    proofs: List[Tuple[int, int]]   # Schnorr (c, v) per commitment


@dataclass
class ElectionRecord:
    manifest: Manifest
    qbar: int                       # extended base hash Q-bar
    joint_key: int                  # K
    guardians: List[GuardianRecord]
    ballots: EncryptedBallots
    encrypted_tally: np.ndarray     # (n_real, 2, 512), over the cast ballots
    decryption: DecryptionRecord
    cast: Optional[np.ndarray] = None                   # (nb,) bool; None = every ballot cast
    spoiled_decryption: Optional[DecryptionRecord] = None  # the spoiled ballots' selections


def verify_election_record(group: GroupContext, rec: ElectionRecord, window_bits: int = 8) -> Dict[str, bool]:
    """-> {check name: passed}.  A check that cannot run because an earlier one failed
    structurally (wrong shapes) reports False."""
    out: Dict[str, bool] = {}
    comm = [k for g in rec.guardians for k in g.commitments]
    prf = [p for g in rec.guardians for p in g.proofs]
    # every guardian commits to a polynomial of the same degree: quorum = its coefficient count
    shapes_ok = bool(rec.guardians) and all(g.commitments for g in rec.guardians) and \
        len({len(g.commitments) for g in rec.guardians}) == 1
    out["guardian_proofs"] = shapes_ok and len(comm) == len(prf) and all(verify_commitment_proofs(group, comm, prf))
    if shapes_ok:
        k0 = as_p_array([g.commitments[0] for g in rec.guardians])
        K = int.from_bytes(group.prodP_groups(k0, 1, len(rec.guardians))[0].tobytes(), "big")
        out["joint_key"] = K == rec.joint_key
    else:
        out["joint_key"] = False
    man = rec.manifest
    key = ElectionKey(group, rec.joint_key, window_bits=window_bits)
    nb = rec.ballots.n
    cast = np.ones(nb, bool) if rec.cast is None else np.asarray(rec.cast, bool).reshape(-1)
    cast_ok = cast.shape == (nb,)
    if not cast_ok:
        cast = np.ones(nb, bool)
    ok_s, ok_c, tally = Verifier(group, key, rec.qbar, man).verify(rec.ballots, cast=cast)
    out["ballots"] = bool(ok_s.all() and ok_c.all()) and cast_ok
    et = np.ascontiguousarray(rec.encrypted_tally, dtype=np.uint8).reshape(-1, 2, 512)
    out["tally"] = et.shape == tally.shape and bool(np.array_equal(et, tally))
    dtexts = np.ascontiguousarray(rec.decryption.texts, dtype=np.uint8).reshape(-1, 2, 512)
    same_texts = dtexts.shape == et.shape and bool(np.array_equal(dtexts, et))
    pks = {g.gid: g.commitments[0] for g in rec.guardians if g.commitments}
    commitments = {g.gid: g.commitments for g in rec.guardians if g.commitments}
    dv = verify_decryption_record(group, rec.qbar, rec.decryption, pks, commitments,
                                  guardian_xs={g.gid: g.x for g in rec.guardians},
                                  quorum=len(rec.guardians[0].commitments) if shapes_ok else None,
                                  max_count=int(cast.sum()))
    out["decryption.texts"] = same_texts
    for name, ok in dv.items():
        out[f"decryption.{name}"] = ok
    if (~cast).any() or rec.spoiled_decryption is not None:
        sp = rec.spoiled_decryption
        want = spoiled_texts(man, rec.ballots.cts[~cast])
        got = None if sp is None else np.ascontiguousarray(sp.texts, dtype=np.uint8).reshape(-1, 2, 512)
        out["spoiled.texts"] = got is not None and got.shape == want.shape and bool(np.array_equal(got, want))
        if sp is None or not len(want):
            out["spoiled.decryption"] = sp is None and not len(want)
        else:
            sv = verify_decryption_record(group, rec.qbar, sp, pks, commitments,
                                          guardian_xs={g.gid: g.x for g in rec.guardians},
                                          quorum=len(rec.guardians[0].commitments) if shapes_ok else None,
                                          max_count=man.votes_allowed)
            for name, ok in sv.items():
                out[f"spoiled.{name}"] = ok
    return out
