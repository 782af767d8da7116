"""Trustee partial decryption and the mediator's combine — GPU-backed.

Reference boundary: ``DecryptingTrusteeIF``, implemented remotely by
``RemoteDecryptingTrusteeProxy`` (src/main/java/electionguard/decrypt/RemoteDecryptingTrusteeProxy.java:30,48-115)
and served by ``RunRemoteDecryptingTrustee.directDecrypt`` / ``compensatedDecrypt``
(RunRemoteDecryptingTrustee.java:180-208, 217-247).  Contract kept here:

  * ``id()``, ``xCoordinate()``, ``electionPublicKey()``  (RemoteDecryptingTrusteeProxy.java:33-46)
  * ``directDecrypt(group, texts, extendedBaseHash, nonce)`` -> list of
    DirectDecryptionAndProof in text order (decrypting_trustee_rpc.proto:20-28)
  * ``compensatedDecrypt(group, missingGuardianId, texts, extendedBaseHash, nonce)`` ->
    list of CompensatedDecryptionAndProof (decrypting_trustee_rpc.proto:36-45)
  * the whole text list is ONE batch (one GPU call), as the RPC is batched
    (decrypting_trustee_rpc.proto:15-18).

The mediator side restates ``Decryption.decrypt`` (RunRemoteDecryptor.java:261-262):
verify each share's proof, Lagrange-combine compensated shares, M = prod M_i,
T = B / M, t = dLog_g(T) (baby-step giant-step on the GPU), and ``decryptBallot`` for the
spoiled ballots (RunRemoteDecryptor.java:264-269): the same shares, combine and dLog per
selection, with every spoiled ballot's selections in ONE trustee batch per guardian.
"""
from __future__ import annotations

import ctypes
import math
import secrets
from collections.abc import Sequence as _SequenceABC
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .core import native
from .core.group import GroupContext, as_p_array, as_q_array, p_bytes, q_bytes
from .keyceremony import GuardianKeys, backup_label, backup_open, poly_eval


@dataclass
class GenericChaumPedersenProof:
    c: int
    v: int


@dataclass
class DirectDecryptionAndProof:
    partialDecryption: int
    proof: GenericChaumPedersenProof


@dataclass
class CompensatedDecryptionAndProof:
    partialDecryption: int
    proof: GenericChaumPedersenProof
    recoveredPublicKeyShare: int


class _ShareView:
    """Share i of a ShareBatch: the fields of Direct/CompensatedDecryptionAndProof, read from and
    written to the batch's arrays."""
    __slots__ = ("_b", "_i")

    def __init__(self, b: "ShareBatch", i: int):
        self._b, self._i = b, i

    @property
    def partialDecryption(self) -> int:
        return int.from_bytes(self._b.M[self._i].tobytes(), "big")

    @partialDecryption.setter
    def partialDecryption(self, v: int) -> None:
        self._b.M[self._i] = np.frombuffer(p_bytes(v), dtype=np.uint8)

    @property
    def proof(self) -> GenericChaumPedersenProof:
        pr = self._b.proofs[self._i]
        return GenericChaumPedersenProof(int.from_bytes(pr[0].tobytes(), "big"), int.from_bytes(pr[1].tobytes(), "big"))

    @proof.setter
    def proof(self, p: GenericChaumPedersenProof) -> None:
        self._b.proofs[self._i, 0] = np.frombuffer(q_bytes(p.c), dtype=np.uint8)
        self._b.proofs[self._i, 1] = np.frombuffer(q_bytes(p.v), dtype=np.uint8)

    @property
    def recoveredPublicKeyShare(self) -> int:
        if self._b.recovery is None:
            raise AttributeError("a direct share has no recovery key")
        return int.from_bytes(self._b.recovery[self._i].tobytes(), "big")

    @recoveredPublicKeyShare.setter
    def recoveredPublicKeyShare(self, v: int) -> None:
        self._b.recovery[self._i] = np.frombuffer(p_bytes(v), dtype=np.uint8)

    def _fields(self):
        f = (self.partialDecryption, self.proof)
        return f + (self.recoveredPublicKeyShare,) if self._b.recovery is not None else f

    def __eq__(self, other) -> bool:
        if isinstance(other, _ShareView):
            return self._fields() == other._fields()
        if isinstance(other, (DirectDecryptionAndProof, CompensatedDecryptionAndProof)):
            return self._fields() == tuple(getattr(other, k) for k in (
                ("partialDecryption", "proof", "recoveredPublicKeyShare") if self._b.recovery is not None
                else ("partialDecryption", "proof")))
        return NotImplemented

    def __repr__(self) -> str:
        return f"ShareView({self._fields()!r})"


class ShareBatch(_SequenceABC):
    """The n shares one trustee returns for a batch of texts, kept in their wire form: M (n, 512),
    proofs (n, 2, 32) = (c, v) and, for compensated shares, the recovery keys (n, 512).  It is the
    list DecryptingTrusteeIF.directDecrypt / compensatedDecrypt return (indexing yields share
    objects whose fields read and write the arrays), and the mediator and the record checks take
    the arrays directly (share_arrays), with no per-share conversion."""

    def __init__(self, M: np.ndarray, proofs: np.ndarray, recovery: Optional[np.ndarray] = None):
        self.M = np.ascontiguousarray(M, dtype=np.uint8).reshape(-1, 512)
        self.proofs = np.ascontiguousarray(proofs, dtype=np.uint8).reshape(-1, 2, 32)
        self.recovery = None if recovery is None else np.ascontiguousarray(recovery, dtype=np.uint8).reshape(-1, 512)

    def __len__(self) -> int:
        return len(self.M)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return ShareBatch(self.M[i], self.proofs[i], None if self.recovery is None else self.recovery[i])
        n = len(self.M)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("share index out of range")
        return _ShareView(self, i)

    def __setitem__(self, i: int, share) -> None:
        v = self[i]
        v.partialDecryption = share.partialDecryption
        v.proof = share.proof
        if self.recovery is not None:
            v.recoveredPublicKeyShare = share.recoveredPublicKeyShare

    def __eq__(self, other) -> bool:
        if isinstance(other, ShareBatch):
            return (np.array_equal(self.M, other.M) and np.array_equal(self.proofs, other.proofs) and
                    (self.recovery is None) == (other.recovery is None) and
                    (self.recovery is None or np.array_equal(self.recovery, other.recovery)))
        if isinstance(other, (list, tuple)):
            return len(self) == len(other) and all(a == b for a, b in zip(self, other))
        return NotImplemented


def share_arrays(res) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
    """(M (n, 512), proofs (n, 2, 32), recovery keys (n, 512) or None) of a trustee's result: the
    arrays of a ShareBatch, or packed from a list of share objects."""
    if isinstance(res, ShareBatch):
        return res.M, res.proofs, res.recovery
    res = list(res)
    pr = np.empty((len(res), 2, 32), dtype=np.uint8)
    pr[:, 0] = as_q_array([r.proof.c for r in res])
    pr[:, 1] = as_q_array([r.proof.v for r in res])
    rk = (as_p_array([r.recoveredPublicKeyShare for r in res])
          if res and hasattr(res[0], "recoveredPublicKeyShare") else None)
    return as_p_array([r.partialDecryption for r in res]), pr, rk


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _texts_array(texts) -> np.ndarray:
    """texts: (n, 2, 512) uint8 array or a sequence of (pad, data) int pairs."""
    if isinstance(texts, np.ndarray):
        return np.ascontiguousarray(texts, dtype=np.uint8).reshape(-1, 2, 512)
    out = np.empty((len(texts), 2, 512), dtype=np.uint8)
    for i, (a, b) in enumerate(texts):
        out[i, 0] = np.frombuffer(p_bytes(a), dtype=np.uint8)
        out[i, 1] = np.frombuffer(p_bytes(b), dtype=np.uint8)
    return out


def _nonces(group: GroupContext, n: int, nonces) -> np.ndarray:
    if nonces is None:
        return np.stack([np.frombuffer(q_bytes(secrets.randbelow(group.q - 1) + 1), dtype=np.uint8)
                         for _ in range(n)]) if n else np.empty((0, 32), np.uint8)
    a = np.empty((n, 32), dtype=np.uint8)
    for i, u in enumerate(nonces):
        a[i] = np.frombuffer(q_bytes(int(u)), dtype=np.uint8)
    return a


def _be_int(row: np.ndarray) -> int:
    return int.from_bytes(row.tobytes(), "big")


def partial_decrypt_batch(group: GroupContext, secret: int, qbar: int, texts: np.ndarray,
                          nonces: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """One GPU batch: M_i = pad_i^secret and proofs (c, v).  -> (M (n,512), proof (n,2,32))."""
    n = texts.shape[0]
    M = np.empty((n, 512), dtype=np.uint8)
    pr = np.empty((n, 2, 32), dtype=np.uint8)
    if n:
        sb, qb = q_bytes(secret), q_bytes(qbar)
        native.check(group._lib, "eg_trustee_decrypt_batch",
                     group._lib.eg_trustee_decrypt_batch(group.handle, native.buf(sb), native.buf(qb), _ptr(texts),
                                                         _ptr(nonces), n, _ptr(M), _ptr(pr)))
    return M, pr


class DecryptingTrustee:
    """GPU-backed DecryptingTrusteeIF (one process per trustee, one GPU each)."""

    accepts_arrays = True  # texts may be an (n, 2, 512) wire-form array (the gRPC server passes one)

    def __init__(self, group: GroupContext, keys: GuardianKeys, commitments: Dict[str, List[int]]):
        self.group = group
        self.keys = keys
        self.commitments = commitments  # every guardian's public commitments (for recovery keys)
        self._shares: Dict[str, int] = {}  # decrypted backups, by missing guardian id

    def id(self) -> str:
        return self.keys.gid

    def xCoordinate(self) -> int:
        return self.keys.x

    def electionPublicKey(self) -> int:
        return self.keys.public_key

    def directDecrypt(self, group: GroupContext, texts, extendedBaseHash: int,
                      nonce: Optional[Sequence[int]] = None) -> ShareBatch:
        """-> the n DirectDecryptionAndProof, in text order (a ShareBatch)."""
        return ShareBatch(*self.directDecryptArrays(group, texts, extendedBaseHash, nonce))

    # Array forms for the gRPC server (remote.DecryptingTrusteeServer): the same shares and proofs
    # as directDecrypt / compensatedDecrypt, kept in their wire bytes.
    def directDecryptArrays(self, group: GroupContext, texts, extendedBaseHash: int, nonce=None):
        """-> (M (n, 512), proofs (n, 2, 32)) uint8."""
        T = _texts_array(texts)
        return partial_decrypt_batch(group, self.keys.secret, extendedBaseHash, T, _nonces(group, len(T), nonce))

    def compensatedDecryptArrays(self, group: GroupContext, missingGuardianId: str, texts, extendedBaseHash: int,
                                 nonce=None):
        """-> (M (n, 512), proofs (n, 2, 32), recovery key (512,)) uint8."""
        share = self.share_of(missingGuardianId)
        T = _texts_array(texts)
        M, pr = partial_decrypt_batch(group, share, extendedBaseHash, T, _nonces(group, len(T), nonce))
        rk = np.frombuffer(p_bytes(self.recovery_public_key(missingGuardianId)), dtype=np.uint8)
        return M, pr, rk

    def recovery_public_key(self, missing_id: str) -> int:
        """g^{P_l(x_i)} = prod_j K_{l,j}^{x_i^j} (GPU powP batch + product)."""
        comm = self.commitments[missing_id]
        q = self.group.q
        exps = [pow(self.keys.x, j, q) for j in range(len(comm))]
        pw = self.group.powP_batch(comm, exps)
        return _be_int(self.group.prodP_groups(pw, 1, len(comm))[0])

    def share_of(self, missing_id: str) -> int:
        """P_l(x_i): decrypt guardian l's key-ceremony backup with this trustee's secret
        (k = c0^{s_i} on the GPU, then the KDF / MAC of keyceremony.backup_open); callers that
        only hold decrypted shares fall back to ``shares_from``."""
        cached = self._shares.get(missing_id)
        if cached is not None:
            return cached
        if missing_id in self.keys.backups_from:
            c0, c1, c2 = self.keys.backups_from[missing_id]
            k = _be_int(self.group.powP_batch([c0], [self.keys.secret])[0])
            share = backup_open(c0, k, c1, c2, backup_label(missing_id, self.keys.gid))
            if share is None:
                raise ValueError(f"share backup from {missing_id} fails its MAC")
        elif missing_id in self.keys.shares_from:
            share = self.keys.shares_from[missing_id]
        else:
            raise KeyError(f"no share of {missing_id}")
        self._shares[missing_id] = share
        return share

    def compensatedDecrypt(self, group: GroupContext, missingGuardianId: str, texts, extendedBaseHash: int,
                           nonce: Optional[Sequence[int]] = None) -> ShareBatch:
        """-> the n CompensatedDecryptionAndProof, in text order (a ShareBatch)."""
        M, pr, rk = self.compensatedDecryptArrays(group, missingGuardianId, texts, extendedBaseHash, nonce)
        return ShareBatch(M, pr, np.tile(rk, (len(M), 1)))


def verify_shares(group: GroupContext, qbar: int, Ki, texts, M, proofs) -> np.ndarray:
    """a = g^v K_i^c, b = pad^v M^c; c == H(qbar, pad, data, a, b, M).  -> bool (n,)
    Ki: one key (int) for every share or one per share; M: ints or an (n, 512) array; proofs:
    GenericChaumPedersenProof objects or an (n, 2, 32) array of (c, v)."""
    T = _texts_array(texts)
    n = len(T)
    ok = np.zeros(n, dtype=np.uint8)
    if n:
        if isinstance(Ki, (int, np.integer)):
            K = np.ascontiguousarray(np.broadcast_to(np.frombuffer(p_bytes(Ki), dtype=np.uint8), (n, 512)))
        else:
            K = as_p_array(Ki if isinstance(Ki, np.ndarray) else list(Ki))
        Mm = as_p_array(M if isinstance(M, np.ndarray) else list(M))
        if isinstance(proofs, np.ndarray):
            pr = np.ascontiguousarray(proofs, dtype=np.uint8).reshape(-1, 2, 32)
        else:
            pr = np.empty((n, 2, 32), dtype=np.uint8)
            pr[:, 0] = as_q_array([p.c for p in proofs])
            pr[:, 1] = as_q_array([p.v for p in proofs])
        if len(K) != n or len(Mm) != n or len(pr) != n:
            raise ValueError("verify_shares: keys, shares and proofs must match the texts")
        qb = q_bytes(qbar)
        native.check(group._lib, "eg_verify_shares",
                     group._lib.eg_verify_shares(group.handle, native.buf(qb), _ptr(K), _ptr(T), _ptr(Mm), _ptr(pr),
                                                 n, _ptr(ok)))
    return ok.astype(bool)


def _concurrently(fn, items) -> list:
    """[fn(x) for x in items], the calls made from one thread each (the first exception is
    raised after every call has returned)."""
    items = list(items)
    if len(items) <= 1:
        return [fn(x) for x in items]
    with ThreadPoolExecutor(max_workers=len(items)) as ex:
        return list(ex.map(fn, items))


def lagrange(xs: Sequence[int], xi: int, q: int) -> int:
    num, den = 1, 1
    for xj in xs:
        if xj != xi:
            num = num * xj % q
            den = den * (xj - xi) % q
    return num * pow(den, -1, q) % q


def dlog_g_batch(group: GroupContext, ys, max_result: int) -> List[Optional[int]]:
    """Baby-step giant-step on the GPU: t with g^t = y, 0 <= t <= max_result."""
    Y = as_p_array(list(ys)) if not isinstance(ys, np.ndarray) else np.ascontiguousarray(ys).reshape(-1, 512)
    n = len(Y)
    if n == 0:
        return []
    m = math.isqrt(max_result) + 1
    baby = group.gPowP_batch(list(range(m)))
    table = {baby[j].tobytes(): j for j in range(m)}
    q = group.q
    giants = group.gPowP_batch([(q - (m * i) % q) % q for i in range(m + 1)])  # g^{-m i}
    a = np.repeat(Y, m + 1, axis=0)
    b = np.tile(giants, (n, 1))
    prod = group.multP_batch(a, b).reshape(n, m + 1, 512)
    out: List[Optional[int]] = []
    for k in range(n):
        res = None
        for i in range(m + 1):
            j = table.get(prod[k, i].tobytes())
            if j is not None:
                t = i * m + j
                if t <= max_result:
                    res = t
                    break
        out.append(res)
    return out


@dataclass
class DecryptionRecord:
    """What the mediator publishes for a decrypted tally (the EG 1.0 DecryptionShare data the
    reference's ``Verifier.verify`` re-checks, RunRemoteWorkflowTest.java:179-182):
    per text, every available guardian's direct share, every (missing, available) pair's
    compensated share with its recovery key, and the plaintext counts."""
    texts: np.ndarray                                            # (n, 2, 512) encrypted tally
    xs: Dict[str, int]                                           # available guardian -> x coordinate
    direct: Dict[str, List[DirectDecryptionAndProof]]            # available guardian -> n shares
    compensated: Dict[str, Dict[str, List[CompensatedDecryptionAndProof]]]  # missing -> available -> n
    counts: List[Optional[int]]


def spoiled_texts(man, cts: np.ndarray) -> np.ndarray:
    """The real selections' ciphertexts of spoiled ballots, ballot-major: (nb * n_real, 2, 512)
    from the wire layout (nb, nsel, 2, 512) (placeholders are not part of a decrypted ballot)."""
    nb = cts.shape[0]
    sel = np.asarray(cts).reshape(nb, man.n_contests, man.spc, 2, 512)[:, :, : man.n_selections]
    return np.ascontiguousarray(sel).reshape(nb * man.n_real, 2, 512)


class Decryption:
    """Mediator combine (``new Decryption(group, init, trustees, missing).decrypt(tally)``)."""

    def __init__(self, group: GroupContext, qbar: int, trustees: Sequence, missing: Sequence[str],
                 public_keys: Dict[str, int]):
        self.group, self.qbar = group, qbar
        self.trustees = list(trustees)
        self.missing = list(missing)
        self.public_keys = public_keys

    def decrypt(self, tally: np.ndarray, max_count: int) -> List[Optional[int]]:
        """tally: (n, 2, 512) encrypted per-selection totals -> plaintext counts."""
        return self.decrypt_record(tally, max_count).counts

    def decrypt_record(self, tally: np.ndarray, max_count: int) -> DecryptionRecord:
        """decrypt() keeping every share and proof (the published decryption record)."""
        G = self.group
        T = _texts_array(tally)
        n = len(T)
        xs = [t.xCoordinate() for t in self.trustees]
        rec = DecryptionRecord(T, {t.id(): t.xCoordinate() for t in self.trustees}, {}, {}, [])
        parts = []  # (n,512) arrays to multiply together
        # every trustee's batch is requested at once (remote trustees are separate processes,
        # one GPU each); the checks and the combine below run in trustee order
        direct = _concurrently(lambda tr: tr.directDecrypt(G, T, self.qbar), self.trustees)
        pairs = [(l, tr) for l in self.missing for tr in self.trustees]
        comp = iter(_concurrently(lambda lt: lt[1].compensatedDecrypt(G, lt[0], T, self.qbar), pairs))
        for tr, res in zip(self.trustees, direct):
            if len(res) != n:  # remote proxies return [] on failure (RemoteDecryptingTrusteeProxy.java:64-66)
                raise ValueError(f"trustee {tr.id()} returned {len(res)} of {n} direct decryptions")
            Md, prd, _ = share_arrays(res)
            ok = verify_shares(G, self.qbar, tr.electionPublicKey(), T, Md, prd)
            if not ok.all():
                raise ValueError(f"invalid direct decryption proof from {tr.id()}")
            rec.direct[tr.id()] = res
            parts.append(Md)
        for l in self.missing:
            rec.compensated[l] = {}
            for tr in self.trustees:
                res = next(comp)
                if len(res) != n:
                    raise ValueError(f"trustee {tr.id()} returned {len(res)} of {n} compensated decryptions for {l}")
                Ml, prl, rkl = share_arrays(res)
                ok = verify_shares(G, self.qbar, rkl, T, Ml, prl)
                if not ok.all():
                    raise ValueError(f"invalid compensated decryption proof from {tr.id()} for {l}")
                rec.compensated[l][tr.id()] = res
                w = lagrange(xs, tr.xCoordinate(), G.q)
                parts.append(G.powP_batch(Ml, [w] * n))
        k = len(parts)
        stacked = np.ascontiguousarray(np.stack(parts, axis=1)).reshape(n * k, 512)
        M = G.prodP_groups(stacked, n, k)
        Tv = G.multP_batch(np.ascontiguousarray(T[:, 1]), G.multInv_batch(M))
        rec.counts = dlog_g_batch(G, Tv, max_count)
        return rec

    # ---- spoiled ballots: decryptBallot (RunRemoteDecryptor.java:264-269) ----
    def decrypt_ballots_record(self, ballots, man) -> DecryptionRecord:
        """decryptBallot over a batch of spoiled ballots keeping every share and proof: the texts
        are the ballots' real selections, ballot-major, in ONE trustee batch per guardian (and
        per missing guardian), so the record's counts are the plaintext selections in that
        order, each in [0, votesAllowed]."""
        cts = ballots.cts if hasattr(ballots, "cts") else np.asarray(ballots)
        return self.decrypt_record(spoiled_texts(man, cts), man.votes_allowed)

    def decryptBallots(self, ballots, man) -> np.ndarray:
        """-> (nb, n_real) decrypted selections of the spoiled ballots (EncryptedBallots or their
        (nb, nsel, 2, 512) ciphertexts); -1 where a value is not a valid selection count, which
        an honest ballot never has."""
        cts = ballots.cts if hasattr(ballots, "cts") else np.asarray(ballots)
        nb = cts.shape[0]
        if nb == 0:
            return np.zeros((0, man.n_real), dtype=np.int64)
        counts = self.decrypt_ballots_record(cts, man).counts
        return np.array([-1 if c is None else int(c) for c in counts], dtype=np.int64).reshape(nb, man.n_real)

    def decryptBallot(self, ballot, man) -> List[int]:
        """``decryptBallot(spoiled)`` for ONE ballot (its (nsel, 2, 512) ciphertexts); a batch
        of spoiled ballots should go through decryptBallots (one trustee batch for all)."""
        return [int(x) for x in self.decryptBallots(np.asarray(ballot).reshape(1, man.nsel, 2, 512), man)[0]]


def verify_decryption_record(group: GroupContext, qbar: int, rec: DecryptionRecord, public_keys: Dict[str, int],
                             commitments: Dict[str, List[int]], guardian_xs: Optional[Dict[str, int]] = None,
                             quorum: Optional[int] = None, max_count: Optional[int] = None) -> Dict[str, bool]:
    """Record-level checks of the tally decryption (the decryption part of the reference's
    ``Verifier(record, 11).verify()``, RunRemoteWorkflowTest.java:179-182; EG 1.0 spec
    verification steps for partial / compensated decryptions and the plaintext tally),
    independent of the mediator that produced ``rec``; every exponentiation runs on the GPU:

      * ``direct_proofs``      every direct share's proof against the guardian's key K_i;
      * ``recovery_keys``      every recovery key g^{P_l(x_i)} == prod_j K_{l,j}^{x_i^j},
                               from the missing guardian's public commitments;
      * ``compensated_proofs`` every compensated share's proof against its recovery key;
      * ``quorum``             the shares come from one quorum: for every missing guardian
                               the same set of available guardians, each with a direct share;
      * ``tally``              B == M * g^t per text with M = prod_i M_i * prod_l prod_i
                               M_{l,i}^{w_i} (Lagrange w_i over the available x's) and t
                               the published count (an integer in [0, max_count]).
    With the key ceremony's view (``guardian_xs``: every guardian's x-coordinate, ``quorum``)
    the quorum check also requires the record's x's to be the ceremony's, at least ``quorum``
    available guardians, and available + missing = all guardians.
    """
    G = group
    T = rec.texts
    n = len(T)
    out = {"direct_proofs": True, "recovery_keys": True, "compensated_proofs": True, "quorum": True, "tally": True}
    avail = list(rec.direct)
    if guardian_xs is not None:
        out["quorum"] &= all(rec.xs.get(g) == x for g, x in guardian_xs.items() if g in rec.xs)
        out["quorum"] &= all(g in guardian_xs for g in rec.xs)
        out["quorum"] &= sorted(avail + list(rec.compensated)) == sorted(guardian_xs)
    if quorum is not None:
        out["quorum"] &= len(avail) >= quorum
    for gid in avail:
        res = rec.direct[gid]
        if gid not in public_keys or gid not in rec.xs:
            out["direct_proofs"] = out["quorum"] = False
            continue
        if len(res) != n:
            out["direct_proofs"] = False
            continue
        Md, prd, _ = share_arrays(res)
        out["direct_proofs"] &= bool(verify_shares(G, qbar, public_keys[gid], T, Md, prd).all())
    if len(rec.counts) != n or any(
            c is None or not isinstance(c, (int, np.integer)) or c < 0 or (max_count is not None and c > max_count)
            for c in rec.counts):
        out["tally"] = False
    for l, by_avail in rec.compensated.items():
        out["quorum"] &= sorted(by_avail) == sorted(avail)
        comm = commitments.get(l)
        if comm is None:  # a "missing guardian" the key ceremony never had
            out["recovery_keys"] = out["compensated_proofs"] = False
            continue
        for gid, res in by_avail.items():
            if gid not in rec.xs:
                out["quorum"] = False
                continue
            x = rec.xs[gid]
            exps = [pow(x, j, G.q) for j in range(len(comm))]
            want = _be_int(G.prodP_groups(G.powP_batch(comm, exps), 1, len(comm))[0])
            if len(res) != n:
                out["recovery_keys"] = out["compensated_proofs"] = False
                continue
            Ml, prl, rkl = share_arrays(res)
            out["recovery_keys"] &= rkl is not None and bool(
                (rkl == np.frombuffer(p_bytes(want), dtype=np.uint8)).all())
            out["compensated_proofs"] &= rkl is not None and bool(verify_shares(G, qbar, rkl, T, Ml, prl).all())
    lengths_ok = all(len(rec.direct[g]) == n for g in avail) and all(
        len(res) == n for by in rec.compensated.values() for res in by.values())
    if not lengths_ok:
        out["tally"] = False
    if not (out["quorum"] and out["tally"] and n):
        return out
    xs = [rec.xs[g] for g in avail]
    parts = [share_arrays(rec.direct[g])[0] for g in avail]
    for l, by_avail in rec.compensated.items():
        for gid in avail:
            w = lagrange(xs, rec.xs[gid], G.q)
            parts.append(G.powP_batch(share_arrays(by_avail[gid])[0], [w] * n))
    k = len(parts)
    M = G.prodP_groups(np.ascontiguousarray(np.stack(parts, axis=1)).reshape(n * k, 512), n, k)
    lhs = G.multP_batch(M, G.gPowP_batch([int(c) for c in rec.counts]))
    out["tally"] = bool(np.array_equal(lhs, np.ascontiguousarray(T[:, 1])))
    return out
