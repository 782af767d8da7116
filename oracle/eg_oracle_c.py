"""ctypes wrapper of oracle/_build/libegoracle.so (eg_oracle_c.c) — TEST INFRASTRUCTURE
ONLY (tests/ and bench.py's cpu_baseline leg).  Built by __graft_entry__.build_oracle()."""
from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np

LIB = Path(__file__).resolve().parent / "_build" / "libegoracle.so"
_lib = None


def load():
    global _lib
    if _lib is None:
        if not LIB.exists():
            import sys
            sys.path.insert(0, str(LIB.parent.parent.parent))
            import __graft_entry__
            __graft_entry__.build_oracle()
        _lib = ctypes.CDLL(str(LIB))
        P = ctypes.c_void_p
        S = ctypes.c_size_t
        _lib.ego_init.argtypes = [P, P, P]
        _lib.ego_set_key.argtypes = [P]
        _lib.ego_verify_ballots.argtypes = [P, S, S, S, S, ctypes.c_uint32, P, P, P, P, P, P, ctypes.c_int]
        _lib.ego_powp.argtypes = [P, P, P, S]
        _lib.ego_gpowp.argtypes = [P, P, S]
        _lib.ego_encrypt_ballots.argtypes = [P, S, S, S, P, P, P, P, P, P, ctypes.c_int]
        _lib.ego_trustee_decrypt.argtypes = [P, P, P, P, S, P, P, ctypes.c_int]
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _b(x: int, n: int) -> np.ndarray:
    return np.frombuffer(int(x).to_bytes(n, "big"), dtype=np.uint8).copy()


class COracle:
    def __init__(self, p: int, q: int, g: int):
        self.lib = load()
        self._keep = [_b(p, 512), _b(q, 32), _b(g, 512)]
        assert self.lib.ego_init(*[_p(a) for a in self._keep]) == 0

    def set_key(self, K: int) -> None:
        self._K = _b(K, 512)
        self.lib.ego_set_key(_p(self._K))

    def powp(self, bases: np.ndarray, exps: np.ndarray) -> np.ndarray:
        bases = np.ascontiguousarray(bases, np.uint8).reshape(-1, 512)
        exps = np.ascontiguousarray(exps, np.uint8).reshape(-1, 32)
        out = np.empty_like(bases)
        self.lib.ego_powp(_p(bases), _p(exps), _p(out), len(bases))
        return out

    def gpowp(self, exps: np.ndarray) -> np.ndarray:
        exps = np.ascontiguousarray(exps, np.uint8).reshape(-1, 32)
        out = np.empty((len(exps), 512), np.uint8)
        self.lib.ego_gpowp(_p(exps), _p(out), len(exps))
        return out

    def verify_ballots(self, qbar: int, nc: int, spc: int, ph: int, limit: int, cts, rproof, cproof,
                       threads: int = 1, tally: bool = True):
        nb = cts.shape[0]
        cts = np.ascontiguousarray(cts, np.uint8)
        rproof = np.ascontiguousarray(rproof, np.uint8)
        cproof = np.ascontiguousarray(cproof, np.uint8)
        ok_s = np.zeros((nb, nc * spc), np.uint8)
        ok_c = np.zeros((nb, nc), np.uint8)
        t = np.zeros((nc * (spc - ph), 2, 512), np.uint8) if tally else None
        qb = _b(qbar, 32)
        rc = self.lib.ego_verify_ballots(_p(qb), nb, nc, spc, ph, limit, _p(cts), _p(rproof), _p(cproof),
                                         _p(ok_s), _p(ok_c), _p(t), threads)
        assert rc == 0
        return ok_s.astype(bool), ok_c.astype(bool), t

    def encrypt_ballots(self, qbar: int, nc: int, spc: int, votes, sel_nonces, contest_nonces, threads: int = 1):
        """batchEncryption with injected nonces (eg_oracle.py:encrypt_ballot's algorithm, the
        known-nonce fake branch); -> (cts, rproof, cproof) in the eg_encrypt_ballots layout."""
        votes = np.ascontiguousarray(votes, np.uint8)
        nb = votes.shape[0]
        sn = np.ascontiguousarray(sel_nonces, np.uint8).reshape(nb, nc * spc, 4, 32)
        cn = np.ascontiguousarray(contest_nonces, np.uint8).reshape(nb, nc, 32)
        cts = np.zeros((nb, nc * spc, 2, 512), np.uint8)
        rp = np.zeros((nb, nc * spc, 4, 32), np.uint8)
        cp = np.zeros((nb, nc, 2, 32), np.uint8)
        qb = _b(qbar, 32)
        rc = self.lib.ego_encrypt_ballots(_p(qb), nb, nc, spc, _p(votes), _p(sn), _p(cn), _p(cts), _p(rp), _p(cp),
                                          threads)
        assert rc == 0, "set_key first"
        return cts, rp, cp

    def trustee_decrypt(self, secret: int, qbar: int, texts, nonces, threads: int = 1):
        """directDecrypt (or compensatedDecrypt with secret = P_l(x_i)): -> (M (n, 512), proof (n, 2, 32))."""
        texts = np.ascontiguousarray(texts, np.uint8).reshape(-1, 2, 512)
        n = texts.shape[0]
        nonces = np.ascontiguousarray(nonces, np.uint8).reshape(n, 32)
        M = np.zeros((n, 512), np.uint8)
        pr = np.zeros((n, 2, 32), np.uint8)
        sb, qb = _b(secret, 32), _b(qbar, 32)
        assert self.lib.ego_trustee_decrypt(_p(sb), _p(qb), _p(texts), _p(nonces), n, _p(M), _p(pr), threads) == 0
        return M, pr
