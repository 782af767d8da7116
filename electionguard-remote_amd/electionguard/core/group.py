"""GroupContext / ElementModP / ElementModQ — host mirror of the upstream group layer.

Reference boundary: the reference builds its one GroupContext in
``KUtils.productionGroup()`` (src/main/java/electionguard/util/KUtils.java:10-12) and
moves elements as fixed-width big-endian bytes (common.proto:6-16), importing them
unchecked via ``new BigInteger(1, bytes)`` (ConvertCommonProto.java:41-57).

Every mod-p operation here runs on the GPU through libeg_hip.so (batched C ABI);
mod-q scalar arithmetic (256-bit, a few ops per proof) is host integer arithmetic.
The per-element methods exist for API compatibility and are batches of one; the
``*_batch`` methods are the intended drop-in entry points.
"""
from __future__ import annotations

import ctypes
import threading
from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Union

import numpy as np

from . import native
from .constants import P_BYTES, Q_BYTES, ProductionMode, constants_for

BytesLike = Union[bytes, bytearray, memoryview]


def p_bytes(x: int) -> bytes:
    return int(x).to_bytes(P_BYTES, "big")


def q_bytes(x: int) -> bytes:
    return int(x).to_bytes(Q_BYTES, "big")


def as_p_array(elems: Union[np.ndarray, Sequence["ElementModP"], Sequence[int]]) -> np.ndarray:
    """-> contiguous uint8 array of shape (n, 512)."""
    if isinstance(elems, np.ndarray):
        a = np.ascontiguousarray(elems, dtype=np.uint8)
        return a.reshape(-1, P_BYTES)
    raw = bytearray().join(e.byteArray() if isinstance(e, ElementModP) else int(e).to_bytes(P_BYTES, "big")
                           for e in elems)
    return np.frombuffer(raw, dtype=np.uint8).reshape(-1, P_BYTES)


def as_q_array(elems: Union[np.ndarray, Sequence["ElementModQ"], Sequence[int]]) -> np.ndarray:
    if isinstance(elems, np.ndarray):
        a = np.ascontiguousarray(elems, dtype=np.uint8)
        return a.reshape(-1, Q_BYTES)
    raw = bytearray().join(e.byteArray() if isinstance(e, ElementModQ) else int(e).to_bytes(Q_BYTES, "big")
                           for e in elems)
    return np.frombuffer(raw, dtype=np.uint8).reshape(-1, Q_BYTES)


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _p_be(x) -> bytes:
    if isinstance(x, ElementModP):
        return x.byteArray()
    if isinstance(x, (bytes, bytearray)):
        if len(x) != P_BYTES:
            raise ValueError("ElementModP bytes must be 512 long")
        return bytes(x)
    return p_bytes(int(x))


def _q_be(x) -> bytes:
    if isinstance(x, ElementModQ):
        return x.byteArray()
    if isinstance(x, (bytes, bytearray)):
        if len(x) != Q_BYTES:
            raise ValueError("ElementModQ bytes must be 32 long")
        return bytes(x)
    return q_bytes(int(x))


# Algorithmic 32-bit MACs of one 4096-bit (128-word) Montgomery operation:
# product 128^2 (a square needs only 128*129/2) + reduction 128^2.
MAC_PER_MUL = 2 * 128 * 128
MAC_PER_SQR = 128 * 129 // 2 + 128 * 128


@dataclass
class KernelProfile:
    """Device time and work of the k_pow launches between profile_begin / profile_end."""
    ms: float          # summed HIP-event milliseconds on the ctx stream
    mont_ops: float    # Montgomery multiplies + squarings
    squarings: float   # of which squarings
    launches: int
    clock_ghz: float = 0.0  # shader clock the launches ran at (median per-workgroup s_memtime / s_memrealtime)
    clock_records: int = 0  # workgroup clock records behind clock_ghz
    clock_dropped: int = 0  # records dropped as unset, wrapped or out of range (eg_clock_median)

    @property
    def macs(self) -> float:
        return (self.mont_ops - self.squarings) * MAC_PER_MUL + self.squarings * MAC_PER_SQR


class MexpTicket:
    """A queued per-element job (GroupContext.mexp_submit): wait() returns its 512 output bytes.  The
    library writes `out` until the ticket is waited, so an unwaited ticket waits when collected."""

    def __init__(self, lib):
        self._lib = lib
        self.out = bytearray(P_BYTES)
        self.ticket = ctypes.c_void_p()
        self._done = False

    def wait(self) -> bytes:
        if not self._done:
            self._done = True
            native.check(self._lib, "eg_ticket_wait", self._lib.eg_ticket_wait(self.ticket))
        return bytes(self.out)

    def __del__(self):
        if not self._done and self.ticket:
            self._done = True
            self._lib.eg_ticket_wait(self.ticket)


class GroupContext:
    """GPU-backed GroupContext (one per device; calls are thread-safe)."""

    def __init__(self, p: int, q: int, g: int, device: int = 0, fb_window_bits: int = 8):
        self.p, self.q, self.g = p, q, g
        self.r = (p - 1) // q if q and (p - 1) % q == 0 else None
        self.device = device
        self.mode = None  # ProductionMode name when made by productionGroup
        self._lib = native.load()
        self._p_be, self._q_be, self._g_be = p_bytes(p), q_bytes(q), p_bytes(g)
        h = ctypes.c_void_p()
        native.check(self._lib, "eg_ctx_create",
                     self._lib.eg_ctx_create(native.buf(self._p_be), native.buf(self._q_be),
                                             native.buf(self._g_be), device, ctypes.byref(h)))
        self._ctx = h
        self._lock = threading.Lock()
        self._fb_window_bits = fb_window_bits
        self.ONE_MOD_P = ElementModP(1, self)
        self.ZERO_MOD_P = ElementModP(0, self)
        self.G_MOD_P = ElementModP(g, self)
        self.ZERO_MOD_Q = ElementModQ(0, self)
        self.ONE_MOD_Q = ElementModQ(1, self)

    # ---- lifetime ----
    def close(self) -> None:
        if getattr(self, "_ctx", None):
            self._lib.eg_ctx_destroy(self._ctx)
            self._ctx = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._ctx

    # ---- element construction (ConvertCommonProto.importElementModP/Q semantics) ----
    def binaryToElementModP(self, b: BytesLike) -> ElementModP:
        return ElementModP(int.from_bytes(bytes(b), "big"), self)

    def binaryToElementModQ(self, b: BytesLike) -> ElementModQ:
        return ElementModQ(int.from_bytes(bytes(b), "big"), self)

    def uIntToElementModQ(self, x: int) -> ElementModQ:
        return ElementModQ(x % self.q, self)

    # ---- batched group ops (the drop-in entry points) ----
    def powP_batch(self, bases, exps) -> np.ndarray:
        """out[i] = bases[i]^exps[i] mod p  (ElementModP.powP)."""
        B, E = as_p_array(bases), as_q_array(exps)
        if len(B) != len(E):
            raise ValueError("bases/exps length mismatch")
        out = np.empty_like(B)
        if len(B):
            native.check(self._lib, "eg_powp_batch",
                         self._lib.eg_powp_batch(self._ctx, _ptr(B), _ptr(E), _ptr(out), len(B)))
        return out

    def gPowP_batch(self, exps) -> np.ndarray:
        """out[i] = g^exps[i] mod p via the fixed-base table (GroupContext.gPowP)."""
        E = as_q_array(exps)
        out = np.empty((len(E), P_BYTES), dtype=np.uint8)
        if len(E):
            fb = self._lib.eg_ctx_g_table(self._ctx)
            native.check(self._lib, "eg_fb_pow_batch",
                         self._lib.eg_fb_pow_batch(fb, _ptr(E), _ptr(out), len(E)))
        return out

    def powP_batch_dev(self, d_bases: int, d_exps: int, d_out: int, n: int) -> None:
        """Asynchronous powP on device pointers (n x 512 B bases, n x 32 B exponents, n x 512 B
        out, big-endian rows in HBM, e.g. torch CUDA tensors' data_ptr()); ``sync()`` waits."""
        if n:
            native.check(self._lib, "eg_powp_batch_dev",
                         self._lib.eg_powp_batch_dev(self._ctx, d_bases, d_exps, d_out, n))

    def gPowP_batch_dev(self, d_exps: int, d_out: int, n: int) -> None:
        """Asynchronous gPowP on device pointers (see powP_batch_dev)."""
        if n:
            fb = self._lib.eg_ctx_g_table(self._ctx)
            native.check(self._lib, "eg_fb_pow_batch_dev", self._lib.eg_fb_pow_batch_dev(fb, d_exps, d_out, n))

    def multP_batch(self, a, b) -> np.ndarray:
        A, B = as_p_array(a), as_p_array(b)
        if len(A) != len(B):
            raise ValueError("length mismatch")
        out = np.empty_like(A)
        if len(A):
            native.check(self._lib, "eg_multp_batch",
                         self._lib.eg_multp_batch(self._ctx, _ptr(A), _ptr(B), _ptr(out), len(A)))
        return out

    def prodP_groups(self, elems, groups: int, length: int) -> np.ndarray:
        """out[g] = prod_k elems[g*length + k] (Iterable<ElementModP>.multP())."""
        A = as_p_array(elems)
        if len(A) != groups * length:
            raise ValueError("elems must hold groups*length elements")
        out = np.empty((groups, P_BYTES), dtype=np.uint8)
        if groups:
            native.check(self._lib, "eg_prod_reduce",
                         self._lib.eg_prod_reduce(self._ctx, _ptr(A), groups, length, _ptr(out)))
        return out

    def multInv_batch(self, a) -> np.ndarray:
        A = as_p_array(a)
        out = np.empty_like(A)
        if len(A):
            native.check(self._lib, "eg_multinv_batch",
                         self._lib.eg_multinv_batch(self._ctx, _ptr(A), _ptr(out), len(A)))
        return out

    # ---- per-element API: coalesced across calling threads (eg_*_one, include/eg_hip.h) ----
    # The reference calls the group element by element from 11 threads (RunRemoteWorkflowTest.java:
    # 140,180); concurrent calls join one GPU batch (eg_ctx_set_coalescing sets its window).
    def powP_one(self, base, e) -> bytes:
        b, x = _p_be(base), _q_be(e)
        out = bytearray(P_BYTES)
        native.check(self._lib, "eg_powp_one",
                     self._lib.eg_powp_one(self._ctx, native.buf(b), native.buf(x), native.buf(out)))
        return bytes(out)

    def gPowP_one(self, e) -> bytes:
        x = _q_be(e)
        out = bytearray(P_BYTES)
        native.check(self._lib, "eg_gpowp_one", self._lib.eg_gpowp_one(self._ctx, native.buf(x), native.buf(out)))
        return bytes(out)

    def multP_one(self, a, b) -> bytes:
        x, y = _p_be(a), _p_be(b)
        out = bytearray(P_BYTES)
        native.check(self._lib, "eg_multp_one",
                     self._lib.eg_multp_one(self._ctx, native.buf(x), native.buf(y), native.buf(out)))
        return bytes(out)

    def mexp_one(self, bases=(), e=None, fixed=()) -> bytes:
        """One general per-element job (eg_mexp_one): (prod bases)^e * prod_t fb_t^e_t mod p.
        bases: up to 16 elements; e: None = exponent 1; fixed: up to two (FixedBase, exponent) terms,
        e.g. g^v * alpha^c = mexp_one([alpha], c, [(g_table, v)])."""
        bs = b"".join(_p_be(b) for b in bases)
        x = _q_be(e) if e is not None else None
        fixed = list(fixed)
        if len(fixed) > 2:
            raise ValueError("at most two fixed-base terms")
        fbs = [f[0]._fb if f[0] is not None else self._g_table() for f in fixed] + [None] * (2 - len(fixed))
        fes = [_q_be(f[1]) for f in fixed] + [None] * (2 - len(fixed))
        out = bytearray(P_BYTES)
        keep = [bs, x, *fes]  # alive across the call
        native.check(self._lib, "eg_mexp_one",
                     self._lib.eg_mexp_one(self._ctx, native.buf(bs) if bs else None, len(bases),
                                           native.buf(x) if x is not None else None, fbs[0],
                                           native.buf(fes[0]) if fes[0] is not None else None, fbs[1],
                                           native.buf(fes[1]) if fes[1] is not None else None, native.buf(out)))
        del keep
        return bytes(out)

    def mexp_submit(self, bases=(), e=None, fixed=()) -> "MexpTicket":
        """The job of mexp_one, queued (eg_mexp_submit: inputs are copied, the output buffer is held by the
        ticket); jobs submitted before a wait share the coalescer's next batch.  ticket.wait() -> bytes."""
        bs = b"".join(_p_be(b) for b in bases)
        x = _q_be(e) if e is not None else None
        fixed = list(fixed)
        if len(fixed) > 2:
            raise ValueError("at most two fixed-base terms")
        fbs = [f[0]._fb if f[0] is not None else self._g_table() for f in fixed] + [None] * (2 - len(fixed))
        fes = [_q_be(f[1]) for f in fixed] + [None] * (2 - len(fixed))
        t = MexpTicket(self._lib)
        native.check(self._lib, "eg_mexp_submit",
                     self._lib.eg_mexp_submit(self._ctx, native.buf(bs) if bs else None, len(bases),
                                              native.buf(x) if x is not None else None, fbs[0],
                                              native.buf(fes[0]) if fes[0] is not None else None, fbs[1],
                                              native.buf(fes[1]) if fes[1] is not None else None,
                                              native.buf(t.out), ctypes.byref(t.ticket)))
        return t

    def _g_table(self):
        return self._lib.eg_ctx_g_table(self._ctx)

    def set_coalescing(self, max_batch: int, window_us: int) -> None:
        native.check(self._lib, "eg_ctx_set_coalescing",
                     self._lib.eg_ctx_set_coalescing(self._ctx, max_batch, window_us))

    def gPowP(self, e: Union["ElementModQ", int]) -> "ElementModP":
        return ElementModP.from_bytes(self.gPowP_one(e), self)

    def multP(self, *elems: "ElementModP") -> "ElementModP":
        if not elems:
            return self.ONE_MOD_P
        if len(elems) == 2:
            return ElementModP.from_bytes(self.multP_one(elems[0], elems[1]), self)
        return ElementModP.from_bytes(self.prodP_groups(list(elems), 1, len(elems))[0], self)

    def dLogG(self, y: "ElementModP", max_result: int) -> Optional[int]:
        """t with g^t = y, 0 <= t <= max_result (baby-step giant-step on the GPU)."""
        from ..decrypt import dlog_g_batch

        return dlog_g_batch(self, [y], max_result)[0]

    def fixed_base(self, base: Union["ElementModP", int], window_bits: int = 8) -> "FixedBase":
        return FixedBase(self, base, window_bits)

    # ---- Fiat-Shamir pre-image format (unpinned upstream: switchable) ----
    @property
    def hash_format(self) -> str:
        return getattr(self, "_hash_format", "fixed")

    @hash_format.setter
    def hash_format(self, fmt: str) -> None:
        from .hashing import FORMATS
        if fmt not in FORMATS:
            raise ValueError(f"unknown hash format {fmt!r} (have {', '.join(FORMATS)})")
        native.check(self._lib, "eg_ctx_set_hash_format", self._lib.eg_ctx_set_hash_format(self._ctx, FORMATS[fmt]))
        self._hash_format = fmt

    # ---- response convention and challenge pre-image order (unpinned upstream, eg_ctx_set_proof_format) ----
    RESPONSES = {"minus": 0, "plus": 1}
    PREIMAGES = {"message_first": 0, "commitments_first": 1, "with_key": 2}

    @property
    def proof_format(self) -> tuple:
        """(response, preimage): ("minus", "message_first") by default -- v = u - c x with a = g^v X^c,
        and the hashed elements after Q-bar message first; see include/eg_hip.h for the variants."""
        return getattr(self, "_proof_format", ("minus", "message_first"))

    @proof_format.setter
    def proof_format(self, fmt) -> None:
        resp, pre = fmt
        if resp not in self.RESPONSES or pre not in self.PREIMAGES:
            raise ValueError(f"unknown proof format {fmt!r} (responses {list(self.RESPONSES)}, "
                             f"pre-images {list(self.PREIMAGES)})")
        native.check(self._lib, "eg_ctx_set_proof_format",
                     self._lib.eg_ctx_set_proof_format(self._ctx, self.RESPONSES[resp], self.PREIMAGES[pre]))
        self._proof_format = (resp, pre)

    # ---- constant-time encryption (eg_ctx_set_ct_encrypt) ----
    @property
    def ct_encrypt(self) -> bool:
        """Encryption with masked scans of small radix tables: no address or schedule depends on
        a nonce or a vote (the default indexes the wide tables by nonce digits).  Same bytes."""
        return getattr(self, "_ct_encrypt", False)

    @ct_encrypt.setter
    def ct_encrypt(self, on: bool) -> None:
        native.check(self._lib, "eg_ctx_set_ct_encrypt", self._lib.eg_ctx_set_ct_encrypt(self._ctx, 1 if on else 0))
        self._ct_encrypt = bool(on)

    # ---- constant-time exponentiation for secret exponents (eg_ctx_set_ct_pow) ----
    @property
    def ct_pow(self) -> bool:
        """Variable-base and fixed-base exponentiation (batches and per-element jobs) on a fixed
        window schedule with masked table scans: no address or schedule depends on the exponent (a
        trustee's share s_i through the per-element API).  Same results."""
        return getattr(self, "_ct_pow", False)

    @ct_pow.setter
    def ct_pow(self, on: bool) -> None:
        native.check(self._lib, "eg_ctx_set_ct_pow", self._lib.eg_ctx_set_ct_pow(self._ctx, 1 if on else 0))
        self._ct_pow = bool(on)

    # ---- profiling of the dominant kernel ----
    def profile_begin(self) -> None:
        native.check(self._lib, "eg_ctx_profile_begin", self._lib.eg_ctx_profile_begin(self._ctx))

    def profile_end(self) -> "KernelProfile":
        ms, mm, sq, n = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_int()
        native.check(self._lib, "eg_ctx_profile_end",
                     self._lib.eg_ctx_profile_end(self._ctx, ctypes.byref(ms), ctypes.byref(mm), ctypes.byref(sq),
                                                  ctypes.byref(n)))
        ghz, used, dropped = ctypes.c_double(), ctypes.c_uint32(), ctypes.c_uint32()
        native.check(self._lib, "eg_ctx_profile_clock",
                     self._lib.eg_ctx_profile_clock(self._ctx, ctypes.byref(ghz), ctypes.byref(used),
                                                    ctypes.byref(dropped)))
        return KernelProfile(ms.value, mm.value, sq.value, n.value, ghz.value, used.value, dropped.value)

    def sync(self) -> None:
        native.check(self._lib, "eg_ctx_sync", self._lib.eg_ctx_sync(self._ctx))

    # ---- device memory through this library's own HIP runtime (eg_dev_alloc, include/eg_hip.h) ----
    def device_buffer(self, nbytes: int) -> "DeviceBuffer":
        """``nbytes`` of HBM on this context's device (no other GPU framework in the process)."""
        return DeviceBuffer(self, nbytes)

    def device_empty(self, shape, dtype=np.uint8) -> "DeviceBuffer":
        """An uninitialised device array of ``shape`` (bytes = prod(shape) x itemsize)."""
        shape = (shape,) if isinstance(shape, int) else tuple(shape)
        return DeviceBuffer(self, int(np.prod(shape)) * np.dtype(dtype).itemsize, shape, dtype)

    def device_zeros(self, shape, dtype=np.uint8) -> "DeviceBuffer":
        d = self.device_empty(shape, dtype)
        d.zero()
        return d

    def to_device(self, a: np.ndarray) -> "DeviceBuffer":
        """A device copy of the contiguous array ``a`` (its shape and dtype kept for download())."""
        a = np.ascontiguousarray(a)
        d = DeviceBuffer(self, a.nbytes, a.shape, a.dtype)
        d.upload(a)
        return d

    def all_nonzero(self, d_flags: "DeviceBuffer", n: Optional[int] = None) -> bool:
        """Every one of the first n flag bytes in HBM is non-zero (the verifier's ok_sel / ok_contest)."""
        out = ctypes.c_int()
        native.check(self._lib, "eg_all_nonzero_dev",
                     self._lib.eg_all_nonzero_dev(self._ctx, d_flags.ptr, d_flags.nbytes if n is None else n,
                                                  ctypes.byref(out)))
        return bool(out.value)

    # ---- the multi-GPU tally exchange on this context (RCCL inside libeg_hip) ----
    @staticmethod
    def comm_unique_id() -> bytes:
        lib = native.load()
        b = bytearray(128)
        native.check(lib, "eg_comm_unique_id", lib.eg_comm_unique_id(native.buf(b)))
        return bytes(b)

    def comm_init(self, uid: bytes, world: int, rank: int) -> None:
        if len(uid) != 128:
            raise ValueError("the RCCL unique id is 128 bytes")
        native.check(self._lib, "eg_comm_init", self._lib.eg_comm_init(self._ctx, native.buf(uid), world, rank))
        self._rank = rank

    def comm_destroy(self) -> None:
        native.check(self._lib, "eg_comm_destroy", self._lib.eg_comm_destroy(self._ctx))
        self._rank = 0

    def comm_all_valid(self, ok: bool) -> bool:
        out = ctypes.c_int()
        native.check(self._lib, "eg_comm_all_valid",
                     self._lib.eg_comm_all_valid(self._ctx, 1 if ok else 0, ctypes.byref(out)))
        return bool(out.value)

    def tally_allgather_fold(self, d_parts: "DeviceBuffer", nparts: int, n: int, root: int = 0) -> Optional[np.ndarray]:
        """Fold every rank's nparts x n partial-tally elements (512-B rows in HBM) mod p on ``root``
        (eg_tally_allgather_fold: one RCCL all-gather + the k_prod tree); -> (n, 512) on root, None
        elsewhere.  Without comm_init the local parts are folded."""
        if nparts < 1 or n < 1:
            raise ValueError("empty tally")
        if d_parts.nbytes < nparts * n * P_BYTES:  # the all-gather reads nparts x n rows
            raise ValueError(f"d_parts holds {d_parts.nbytes} B, need nparts * n * 512 = {nparts * n * P_BYTES}")
        out = np.empty((n, P_BYTES), dtype=np.uint8)
        native.check(self._lib, "eg_tally_allgather_fold",
                     self._lib.eg_tally_allgather_fold(self._ctx, d_parts.ptr, nparts, n, root, _ptr(out)))
        return out if self._comm_rank() == root else None

    def comm_info(self) -> tuple:
        """(ranks, rank) as the RCCL communicator reports them (ncclCommCount / ncclCommUserRank);
        (0, 0) without one (eg_comm_info)."""
        n, r = ctypes.c_int(), ctypes.c_int()
        native.check(self._lib, "eg_comm_info", self._lib.eg_comm_info(self._ctx, ctypes.byref(n), ctypes.byref(r)))
        return n.value, r.value

    def _comm_rank(self) -> int:
        return getattr(self, "_rank", 0)


class DeviceBuffer:
    """HBM allocated through libeg_hip (eg_dev_alloc): ``ptr`` is the device address the *_dev
    entry points take.  Freed by ``free()`` (after the ctx stream drains) or on collection."""

    def __init__(self, group: GroupContext, nbytes: int, shape=None, dtype=np.uint8):
        self.group = group
        self.nbytes = int(nbytes)
        self.shape = tuple(shape) if shape is not None else (self.nbytes,)
        self.dtype = np.dtype(dtype)
        h = ctypes.c_void_p()
        native.check(group._lib, "eg_dev_alloc", group._lib.eg_dev_alloc(group.handle, self.nbytes, ctypes.byref(h)))
        self._h = h

    @property
    def ptr(self) -> int:
        return (self._h.value or 0) + getattr(self, "_off", 0)

    def __getitem__(self, sl: slice) -> "DeviceBuffer":
        """A view of rows [start, stop) along the first axis (shares the memory; never frees it)."""
        if not isinstance(sl, slice) or sl.step not in (None, 1):
            raise TypeError("device buffers slice contiguous rows only")
        start, stop, _ = sl.indices(self.shape[0])
        stop = max(start, stop)
        row = self.nbytes // max(self.shape[0], 1)
        v = DeviceBuffer.__new__(DeviceBuffer)
        v.group, v.dtype = self.group, self.dtype
        v.shape = (stop - start,) + self.shape[1:]
        v.nbytes = row * (stop - start)
        v._h, v._off, v._owner = self._h, getattr(self, "_off", 0) + row * start, self
        return v

    def upload(self, a: np.ndarray) -> None:
        a = np.ascontiguousarray(a)
        if a.nbytes != self.nbytes:
            raise ValueError(f"upload of {a.nbytes} B into a {self.nbytes}-B buffer")
        native.check(self.group._lib, "eg_memcpy_htod",
                     self.group._lib.eg_memcpy_htod(self.group.handle, self.ptr, _ptr(a), a.nbytes))

    def download(self) -> np.ndarray:
        out = np.empty(self.shape, dtype=self.dtype)
        native.check(self.group._lib, "eg_memcpy_dtoh",
                     self.group._lib.eg_memcpy_dtoh(self.group.handle, _ptr(out), self.ptr, self.nbytes))
        return out

    def zero(self) -> None:
        native.check(self.group._lib, "eg_memset_dev", self.group._lib.eg_memset_dev(self.group.handle, self.ptr, 0,
                                                                                     self.nbytes))

    def free(self) -> None:
        if getattr(self, "_owner", None) is not None:  # a view: the owner frees the memory
            return
        if getattr(self, "_h", None) and self._h.value and getattr(self.group, "_ctx", None):
            self.group._lib.eg_dev_free(self.group.handle, self._h)
        self._h = ctypes.c_void_p()

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.free()
        except Exception:
            pass


class FixedBase:
    """Accelerated base (``acceleratePow`` / PowRadix): radix table on the device."""

    def __init__(self, group: GroupContext, base, window_bits: int = 8):
        self.group = group
        b = base.value if isinstance(base, ElementModP) else int(base)
        self._be = p_bytes(b)
        h = ctypes.c_void_p()
        native.check(group._lib, "eg_fixed_base_create",
                     group._lib.eg_fixed_base_create(group.handle, native.buf(self._be), window_bits,
                                                     ctypes.byref(h)))
        self._fb = h

    def pow_batch(self, exps) -> np.ndarray:
        E = as_q_array(exps)
        out = np.empty((len(E), P_BYTES), dtype=np.uint8)
        if len(E):
            native.check(self.group._lib, "eg_fb_pow_batch",
                         self.group._lib.eg_fb_pow_batch(self._fb, _ptr(E), _ptr(out), len(E)))
        return out

    def pow_batch_dev(self, d_exps: int, d_out: int, n: int) -> None:
        """Asynchronous base^exps[i] on device pointers (see GroupContext.powP_batch_dev)."""
        if n:
            native.check(self.group._lib, "eg_fb_pow_batch_dev",
                         self.group._lib.eg_fb_pow_batch_dev(self._fb, d_exps, d_out, n))

    def pow_one(self, e) -> bytes:
        """base^e, one coalesced per-element job (eg_fb_pow_one: an accelerated element's powP)."""
        x = _q_be(e)
        out = bytearray(P_BYTES)
        native.check(self.group._lib, "eg_fb_pow_one", self.group._lib.eg_fb_pow_one(self._fb, native.buf(x),
                                                                                     native.buf(out)))
        return bytes(out)

    def close(self) -> None:
        if getattr(self, "_fb", None):
            self.group._lib.eg_fixed_base_destroy(self._fb)
            self._fb = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


@dataclass(frozen=True)
class ElementModP:
    """A member of Z_p (value unchecked on import, as upstream; ops reduce mod p)."""
    value: int
    group: GroupContext

    @staticmethod
    def from_bytes(b, group: GroupContext) -> "ElementModP":
        return ElementModP(int.from_bytes(bytes(b), "big"), group)

    def byteArray(self) -> bytes:
        return p_bytes(self.value)

    def powP(self, e: Union["ElementModQ", int]) -> "ElementModP":
        return ElementModP.from_bytes(self.group.powP_one(self, e), self.group)

    def times(self, other: "ElementModP") -> "ElementModP":
        return ElementModP.from_bytes(self.group.multP_one(self, other), self.group)

    def multInv(self) -> "ElementModP":
        return ElementModP.from_bytes(self.group.multInv_batch([self])[0], self.group)

    def div(self, other: "ElementModP") -> "ElementModP":
        return self.times(other.multInv())

    def inBounds(self) -> bool:
        return 0 <= self.value < self.group.p

    def __int__(self) -> int:
        return self.value


@dataclass(frozen=True)
class ElementModQ:
    """A member of Z_q; 256-bit scalar arithmetic on the host."""
    value: int
    group: GroupContext

    def byteArray(self) -> bytes:
        return q_bytes(self.value)

    def _q(self) -> int:
        return self.group.q

    def __add__(self, o: "ElementModQ") -> "ElementModQ":
        return ElementModQ((self.value + int(o)) % self._q(), self.group)

    def __sub__(self, o: "ElementModQ") -> "ElementModQ":
        return ElementModQ((self.value - int(o)) % self._q(), self.group)

    def __mul__(self, o: "ElementModQ") -> "ElementModQ":
        return ElementModQ((self.value * int(o)) % self._q(), self.group)

    def __neg__(self) -> "ElementModQ":
        return ElementModQ((-self.value) % self._q(), self.group)

    def inBounds(self) -> bool:
        return 0 <= self.value < self._q()

    def __int__(self) -> int:
        return self.value


_PRODUCTION: dict = {}
_PRODUCTION_LOCK = threading.Lock()


def productionGroup(device: int = 0, mode: str = ProductionMode.Mode4096) -> GroupContext:
    """``KUtils.productionGroup()`` (KUtils.java:10-12): ``Mode4096`` is the EG 1.0 4096-bit group
    the reference's upstream 1.0-SNAPSHOT uses; ``ProductionMode.Mode4096_V2`` selects the EG 2.0
    group.  One context per (mode, device), even when first requested from several threads."""
    with _PRODUCTION_LOCK:
        g = _PRODUCTION.get((mode, device))
        if g is None:
            C = constants_for(mode)
            g = GroupContext(C.p, C.q, C.g, device=device)
            g.mode = mode
            _PRODUCTION[(mode, device)] = g
        return g
