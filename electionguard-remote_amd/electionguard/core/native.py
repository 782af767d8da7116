"""ctypes binding of libeg_hip.so (the C ABI in include/eg_hip.h).

The shared library is built in-tree by ``__graft_entry__.build()`` (hipcc,
``--offload-arch=gfx950``) into ``electionguard-remote_amd/electionguard/lib/``.
There is deliberately NO CPU fallback: if the library (or a GPU) is missing,
every group operation raises :class:`NativeUnavailable`.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
from typing import Optional

LIB_DIR = Path(__file__).resolve().parent.parent / "lib"
LIB_PATH = LIB_DIR / "libeg_hip.so"

# Every symbol declared in include/eg_hip.h (tests check the library exports them).
EXPORTED = [
    "eg_last_error", "eg_version", "eg_ctx_create", "eg_ctx_destroy", "eg_ctx_sync",
    "eg_ctx_profile_begin", "eg_ctx_profile_end", "eg_ctx_profile_clock", "eg_ctx_g_table", "eg_ctx_set_hash_format",
    "eg_fixed_base_create", "eg_fixed_base_destroy", "eg_powp_batch", "eg_fb_pow_batch",
    "eg_powp_batch_dev", "eg_fb_pow_batch_dev",
    "eg_multp_batch", "eg_prod_reduce", "eg_multinv_batch", "eg_verify_ballots",
    "eg_set_election_key", "eg_verify_ballots_dev", "eg_encrypt_ballots", "eg_encrypt_ballots_dev",
    "eg_trustee_decrypt_batch", "eg_verify_shares", "eg_clock_median",
    "eg_ctx_set_coalescing", "eg_powp_submit", "eg_gpowp_submit", "eg_multp_submit", "eg_ticket_wait",
    "eg_powp_one", "eg_gpowp_one", "eg_multp_one", "eg_ctx_set_ct_encrypt",
    "eg_dev_alloc", "eg_dev_free", "eg_memcpy_htod", "eg_memcpy_dtoh", "eg_memset_dev", "eg_all_nonzero_dev",
    "eg_comm_unique_id", "eg_comm_init", "eg_comm_destroy", "eg_comm_all_valid", "eg_tally_allgather_fold",
    "eg_ctx_set_proof_format",
    "eg_mexp_submit", "eg_mexp_one", "eg_fb_pow_submit", "eg_fb_pow_one", "eg_ctx_set_ct_pow", "eg_comm_info",
]


class NativeUnavailable(RuntimeError):
    pass


class EgError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed (status {code}): {msg}")
        self.code = code


_lib: Optional[ctypes.CDLL] = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_vp = ctypes.c_void_p
c_sz = ctypes.c_size_t


def _sig(lib: ctypes.CDLL) -> None:
    I = ctypes.c_int
    P = c_vp
    S = c_sz
    U32 = ctypes.c_uint32
    D = ctypes.POINTER(ctypes.c_double)
    sigs = {
        "eg_last_error": ([], ctypes.c_char_p),
        "eg_version": ([ctypes.c_char_p, S], I),
        "eg_ctx_create": ([P, P, P, I, ctypes.POINTER(c_vp)], I),
        "eg_ctx_destroy": ([P], I),
        "eg_ctx_sync": ([P], I),
        "eg_ctx_profile_begin": ([P], I),
        "eg_ctx_profile_end": ([P, D, D, D, ctypes.POINTER(I)], I),
        "eg_ctx_profile_clock": ([P, D, ctypes.POINTER(U32), ctypes.POINTER(U32)], I),
        "eg_clock_median": ([P, S, D, ctypes.POINTER(U32), ctypes.POINTER(U32)], I),
        "eg_ctx_g_table": ([P], P),
        "eg_ctx_set_hash_format": ([P, I], I),
        "eg_ctx_set_proof_format": ([P, I, I], I),
        "eg_fixed_base_create": ([P, P, I, ctypes.POINTER(c_vp)], I),
        "eg_fixed_base_destroy": ([P], I),
        "eg_powp_batch": ([P, P, P, P, S], I),
        "eg_fb_pow_batch": ([P, P, P, S], I),
        "eg_powp_batch_dev": ([P, P, P, P, S], I),
        "eg_fb_pow_batch_dev": ([P, P, P, S], I),
        "eg_multp_batch": ([P, P, P, P, S], I),
        "eg_prod_reduce": ([P, P, S, S, P], I),
        "eg_multinv_batch": ([P, P, P, S], I),
        "eg_verify_ballots": ([P, P, P, S, S, S, S, U32, P, P, P, P, P, P, P], I),
        "eg_set_election_key": ([P, P, I], I),
        "eg_verify_ballots_dev": ([P, P, P, S, S, S, S, U32, P, P, P, P, P, P, P], I),
        "eg_encrypt_ballots": ([P, P, P, S, S, S, P, P, P, P, P, P], I),
        "eg_encrypt_ballots_dev": ([P, P, P, S, S, S, P, P, P, P, P, P], I),
        "eg_ctx_set_ct_encrypt": ([P, I], I),
        "eg_ctx_set_coalescing": ([P, S, U32], I),
        "eg_powp_submit": ([P, P, P, P, ctypes.POINTER(c_vp)], I),
        "eg_gpowp_submit": ([P, P, P, ctypes.POINTER(c_vp)], I),
        "eg_multp_submit": ([P, P, P, P, ctypes.POINTER(c_vp)], I),
        "eg_ticket_wait": ([P], I),
        "eg_powp_one": ([P, P, P, P], I),
        "eg_gpowp_one": ([P, P, P], I),
        "eg_multp_one": ([P, P, P, P], I),
        "eg_trustee_decrypt_batch": ([P, P, P, P, P, S, P, P], I),
        "eg_verify_shares": ([P, P, P, P, P, P, S, P], I),
        "eg_dev_alloc": ([P, S, ctypes.POINTER(c_vp)], I),
        "eg_dev_free": ([P, P], I),
        "eg_memcpy_htod": ([P, P, P, S], I),
        "eg_memcpy_dtoh": ([P, P, P, S], I),
        "eg_memset_dev": ([P, P, I, S], I),
        "eg_all_nonzero_dev": ([P, P, S, ctypes.POINTER(I)], I),
        "eg_comm_unique_id": ([P], I),
        "eg_comm_init": ([P, P, I, I], I),
        "eg_comm_destroy": ([P], I),
        "eg_comm_all_valid": ([P, I, ctypes.POINTER(I)], I),
        "eg_tally_allgather_fold": ([P, P, S, S, I, P], I),
        "eg_comm_info": ([P, ctypes.POINTER(I), ctypes.POINTER(I)], I),
        "eg_mexp_submit": ([P, P, S, P, P, P, P, P, P, ctypes.POINTER(c_vp)], I),
        "eg_mexp_one": ([P, P, S, P, P, P, P, P, P], I),
        "eg_fb_pow_submit": ([P, P, P, ctypes.POINTER(c_vp)], I),
        "eg_fb_pow_one": ([P, P, P], I),
        "eg_ctx_set_ct_pow": ([P, I], I),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res


def load(path: Optional[os.PathLike] = None) -> ctypes.CDLL:
    """Load libeg_hip.so (no GPU needed to load; compute calls need one)."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    if path is None and os.environ.get("EG_LIB"):
        path = os.environ["EG_LIB"]  # A/B builds (tools/ab_mm.py); production uses the in-tree default
    p = Path(path) if path else LIB_PATH
    if not p.exists():
        raise NativeUnavailable(
            f"{p} not built — run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the HIP extension is required; there is no CPU fallback)")
    lib = ctypes.CDLL(str(p))
    _sig(lib)
    if path is None:
        _lib = lib
    return lib


def check(lib: ctypes.CDLL, fn: str, rc: int) -> None:
    if rc != 0:
        raise EgError(fn, rc, lib.eg_last_error().decode(errors="replace"))


def buf(b: bytes | bytearray | memoryview):
    """Pointer to the bytes of b (kept alive by the caller)."""
    if isinstance(b, (bytes,)):
        return ctypes.cast(ctypes.c_char_p(b), c_vp)
    arr = (ctypes.c_uint8 * len(b)).from_buffer(b)
    return ctypes.cast(arr, c_vp)


def out_buf(n: int) -> bytearray:
    return bytearray(max(n, 1))


def version() -> str:
    """Build string of the loaded library, e.g. 'eg_hip gfx950 radix2^29 limbs=144 ...'."""
    lib = load()
    b = ctypes.create_string_buffer(160)
    check(lib, "eg_version", lib.eg_version(b, len(b)))
    return b.value.decode()


def lib_path() -> Path:
    """Path of the library load() uses (EG_LIB override or the in-tree build)."""
    return Path(os.environ["EG_LIB"]) if os.environ.get("EG_LIB") else LIB_PATH
