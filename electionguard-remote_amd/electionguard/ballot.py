"""Batched ballot encryption, verification and tally accumulation on the GPU.

Replaces the three in-process hot loops of the reference's end-to-end driver
(src/test/java/electionguard/workflow/RunRemoteWorkflowTest.java):

  * ``batchEncryption(group, ..., true, 11, "createdBy", CheckType.None)``   :140-141
  * ``runAccumulateBallots(group, ...)``                                     :151
  * ``new Verifier(record, 11).verify()``                                   :179-182

Data layout (device and host, big-endian bytes, ballot-major; see include/eg_hip.h):
  cts    (nb, nsel, 2, 512)  ElGamal (pad alpha, data beta) per selection
  rproof (nb, nsel, 4, 32)   disjunctive 0/1 proof (c0, v0, c1, v1), compact form
  cproof (nb, nc, 2, 32)     contest selection-limit proof (c, v)
Selections are contest-major with the placeholder selection(s) last in each contest.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np

from .core import native
from .core.group import GroupContext, p_bytes, q_bytes


@dataclass(frozen=True)
class Manifest:
    """Synthetic manifest shape (RandomBallotProvider input, RunRemoteWorkflowTest.java:133)."""
    n_contests: int = 4
    n_selections: int = 5     # real selections per contest
    votes_allowed: int = 1    # = number of placeholder selections per contest

    @property
    def spc(self) -> int:
        return self.n_selections + self.votes_allowed

    @property
    def nsel(self) -> int:
        return self.n_contests * self.spc

    @property
    def n_real(self) -> int:
        return self.n_contests * self.n_selections


@dataclass
class EncryptedBallots:
    cts: np.ndarray     # (nb, nsel, 2, 512) uint8
    rproof: np.ndarray  # (nb, nsel, 4, 32) uint8
    cproof: np.ndarray  # (nb, nc, 2, 32) uint8

    @property
    def n(self) -> int:
        return self.cts.shape[0]

    def slice(self, a: int, b: int) -> "EncryptedBallots":
        return EncryptedBallots(self.cts[a:b], self.rproof[a:b], self.cproof[a:b])


def random_scalars(rng: np.random.Generator, shape, q: int) -> np.ndarray:
    """Uniform 256-bit big-endian scalars in [0, q) (q = 2^256 - 189 for EG)."""
    out = rng.integers(0, 256, size=tuple(shape) + (32,), dtype=np.uint8)
    flat = out.reshape(-1, 32)
    qb = np.frombuffer(q_bytes(q), dtype=np.uint8)
    q_top = int.from_bytes(bytes(qb[:8]), "big")
    # rows >= q are re-drawn (probability ~2^-248 for the EG q).  The top 64 bits decide every
    # row except those equal to q's top word, which are compared byte by byte.
    while True:
        top = flat[:, :8].copy().view(">u8").ravel()
        ge = top > q_top
        for i in np.flatnonzero(top == q_top):
            ge[i] = bytes(flat[i]) >= bytes(qb)
        if not ge.any():
            return out
        flat[ge] = rng.integers(0, 256, size=(int(ge.sum()), 32), dtype=np.uint8)


def random_votes(rng: np.random.Generator, man: Manifest, nb: int) -> np.ndarray:
    """One-hot vote over the real selections of each contest (placeholders 0)."""
    v = np.zeros((nb, man.n_contests, man.spc), dtype=np.uint8)
    pick = rng.integers(0, man.n_selections, size=(nb, man.n_contests))
    np.put_along_axis(v, pick[..., None], 1, axis=2)
    return v.reshape(nb, man.nsel)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


class ElectionKey:
    """The joint election key K: registers its fixed-base table (window_bits wide) on a
    GroupContext.  Every ballot call passes K itself, and the library sets it under the ctx lock
    for that call, so threads using different keys on one shared context cannot mix them up."""

    def __init__(self, group: GroupContext, K: int, window_bits: int = 8):
        self.group, self.K, self.window_bits = group, int(K), window_bits
        self._K_be = p_bytes(K)
        self.ensure()

    @property
    def K_be(self) -> bytes:
        return self._K_be

    def ensure(self) -> None:
        """(Re)build K's table at this key's width (a no-op when the ctx already holds it)."""
        native.check(self.group._lib, "eg_set_election_key",
                     self.group._lib.eg_set_election_key(self.group.handle, native.buf(self._K_be),
                                                         self.window_bits))


def batch_encryption(group: GroupContext, key: ElectionKey, qbar: int, man: Manifest, votes: np.ndarray,
                     sel_nonces: np.ndarray, contest_nonces: np.ndarray) -> EncryptedBallots:
    """Encrypt nb ballots with injected nonces (batchEncryption, RunRemoteWorkflowTest.java:140-141).

    votes (nb, nsel) in {0,1}; sel_nonces (nb, nsel, 4, 32) = (R, u, c_fake, v_fake);
    contest_nonces (nb, nc, 32).  Deterministic given the nonces.
    """
    nb = votes.shape[0]
    votes = np.ascontiguousarray(votes, dtype=np.uint8).reshape(nb, man.nsel)
    sn = np.ascontiguousarray(sel_nonces, dtype=np.uint8).reshape(nb, man.nsel, 4, 32)
    cn = np.ascontiguousarray(contest_nonces, dtype=np.uint8).reshape(nb, man.n_contests, 32)
    cts = np.empty((nb, man.nsel, 2, 512), dtype=np.uint8)
    rp = np.empty((nb, man.nsel, 4, 32), dtype=np.uint8)
    cp = np.empty((nb, man.n_contests, 2, 32), dtype=np.uint8)
    if nb:
        qb = q_bytes(qbar)
        native.check(group._lib, "eg_encrypt_ballots",
                     group._lib.eg_encrypt_ballots(group.handle, native.buf(key.K_be), native.buf(qb), nb,
                                                   man.n_contests, man.spc, _ptr(votes), _ptr(sn), _ptr(cn), _ptr(cts),
                                                   _ptr(rp), _ptr(cp)))
    return EncryptedBallots(cts, rp, cp)


def batch_encryption_device(group: GroupContext, key: ElectionKey, qbar: int, man: Manifest, nb: int, d_votes: int,
                            d_sel_nonces: int, d_contest_nonces: int, d_cts: int, d_rproof: int,
                            d_cproof: int) -> None:
    """batch_encryption on device pointers (e.g. torch tensors' data_ptr()): the same
    layouts, inputs and outputs resident in HBM (eg_encrypt_ballots_dev)."""
    if nb:
        native.check(group._lib, "eg_encrypt_ballots_dev",
                     group._lib.eg_encrypt_ballots_dev(group.handle, native.buf(key.K_be), native.buf(q_bytes(qbar)),
                                                       nb, man.n_contests, man.spc, d_votes, d_sel_nonces,
                                                       d_contest_nonces, d_cts, d_rproof, d_cproof))


class Verifier:
    """Ballot-proof verification + homomorphic tally (Verifier.verify / runAccumulateBallots)."""

    def __init__(self, group: GroupContext, key: ElectionKey, qbar: int, man: Manifest):
        self.group, self.key, self.qbar, self.man = group, key, int(qbar), man
        self._qb = q_bytes(qbar)

    def verify(self, eb: EncryptedBallots, with_tally: bool = True,
               cast: Optional[np.ndarray] = None) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
        """-> ok_sel (nb, nsel) bool, ok_contest (nb, nc) bool, tally (n_real, 2, 512) or None.

        cast (nb,) bool (None = all cast): every ballot is verified, only the cast ones are
        tallied (runAccumulateBallots counts cast ballots; spoiled ones are decrypted one by one,
        RunRemoteDecryptor.java:264-269)."""
        man, g = self.man, self.group
        nb = eb.n
        cts = np.ascontiguousarray(eb.cts, dtype=np.uint8)
        rp = np.ascontiguousarray(eb.rproof, dtype=np.uint8)
        cp = np.ascontiguousarray(eb.cproof, dtype=np.uint8)
        cm = None if cast is None else np.ascontiguousarray(np.asarray(cast).reshape(nb) != 0, dtype=np.uint8)
        ok_s = np.zeros((nb, man.nsel), dtype=np.uint8)
        ok_c = np.zeros((nb, man.n_contests), dtype=np.uint8)
        tally = np.empty((man.n_real, 2, 512), dtype=np.uint8) if with_tally else None
        native.check(g._lib, "eg_verify_ballots",
                     g._lib.eg_verify_ballots(g.handle, native.buf(self.key.K_be), native.buf(self._qb), nb,
                                              man.n_contests, man.spc, man.votes_allowed, man.votes_allowed, _ptr(cts),
                                              _ptr(rp), _ptr(cp), _ptr(cm) if cm is not None else None, _ptr(ok_s),
                                              _ptr(ok_c), _ptr(tally) if tally is not None else None))
        return ok_s.astype(bool), ok_c.astype(bool), tally

    def verify_device(self, d_cts: int, d_rproof: int, d_cproof: int, nb: int, d_ok_sel: int, d_ok_con: int,
                      d_tally: Optional[int], d_cast: Optional[int] = None) -> None:
        """Asynchronous verify on device pointers (e.g. torch CUDA tensors' data_ptr()); d_cast
        (nb bytes, 0 = spoiled) as verify's cast."""
        man, g = self.man, self.group
        native.check(g._lib, "eg_verify_ballots_dev",
                     g._lib.eg_verify_ballots_dev(g.handle, native.buf(self.key.K_be), native.buf(self._qb), nb,
                                                  man.n_contests, man.spc, man.votes_allowed, man.votes_allowed, d_cts,
                                                  d_rproof, d_cproof, d_cast, d_ok_sel, d_ok_con, d_tally))


def accumulate_tally(group: GroupContext, man: Manifest, eb: EncryptedBallots,
                     cast: Optional[np.ndarray] = None) -> np.ndarray:
    """runAccumulateBallots without verification: per real selection, prod pad / prod data over the
    cast ballots (cast (nb,) bool, None = all)."""
    if cast is not None:
        eb = EncryptedBallots(eb.cts[np.asarray(cast, bool)], eb.rproof[np.asarray(cast, bool)],
                              eb.cproof[np.asarray(cast, bool)])
    nb = eb.n
    sel = eb.cts.reshape(nb, man.n_contests, man.spc, 2, 512)[:, :, : man.n_selections]
    # groups ordered (contest, selection, component), elements over ballots
    g = np.ascontiguousarray(np.transpose(sel, (1, 2, 3, 0, 4))).reshape(-1, 512)
    out = group.prodP_groups(g, man.n_real * 2, nb)
    return out.reshape(man.n_real, 2, 512)
