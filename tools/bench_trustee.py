"""Trustee-side throughput (BASELINE configs[3] shape): one GPU per DecryptingTrustee.

5 guardians, quorum 3, guardians 4 and 5 missing.  Each available trustee answers ONE
directDecrypt RPC over the whole tally and ONE compensatedDecrypt RPC per missing guardian
(decrypting_trustee_rpc.proto:15-18: the RPC is already batched), i.e. per text
  direct      : M = A^s (comb pair with the proof nonce: A^s, A^u) + g^u + challenge/response
  compensated : the same with s = P_l(x_i), plus the recovery key (once per RPC)
and the mediator verifies every share proof (eg_verify_shares).

Reports shares/s for one trustee on one GPU (device time of the whole RPC batch, texts
already on the host as wire bytes: the H2D copy is included, as an RPC handler would see
it) and the CPU port (OpenSSL BN: 2 variable-base + 1 fixed-base exponentiation per share,
the JVM algorithm classes) on a bounded sample.

    python tools/bench_trustee.py --texts 100000
"""
import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))
sys.path.insert(0, str(ROOT / "oracle"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--texts", type=int, default=100000, help="tally texts per RPC (selections)")
    ap.add_argument("--cpu-sample", type=int, default=256)
    ap.add_argument("--cpu-threads", type=int, default=0)
    a = ap.parse_args()
    from electionguard.core import productionGroup
    from electionguard.decrypt import DecryptingTrustee, partial_decrypt_batch
    from electionguard.keyceremony import key_ceremony
    from electionguard.ballot import random_scalars

    G = productionGroup(0)
    gk, K = key_ceremony(G, 5, 3, seed=4242)
    comm = {g.gid: g.commitments for g in gk}
    tr = DecryptingTrustee(G, gk[0], comm)
    rng = np.random.default_rng(3)
    n = a.texts
    # synthetic tally texts (pad, data) = (g^R, g^t K^R): built on the GPU
    R = random_scalars(rng, (n,), G.q)
    pads = G.gPowP_batch(R)
    datas = G.multP_batch(G.gPowP_batch([int(t) for t in rng.integers(0, 1000, n)]), G.powP_batch([K] * n, R))
    texts = np.ascontiguousarray(np.stack([pads, datas], axis=1))
    nonces = random_scalars(rng, (n,), G.q)
    qbar = 0xC0FFEE

    # warm-up at the full batch size: kernel load, tables, and the workspaces a 100k-text batch
    # grows to (allocated on first use; a timed first call would include those hipMallocs)
    partial_decrypt_batch(G, gk[0].secret, qbar, texts, nonces)
    G.sync()
    t = time.perf_counter()
    M, pr = partial_decrypt_batch(G, gk[0].secret, qbar, texts, nonces)
    direct_s = time.perf_counter() - t

    share = gk[0].shares_from[gk[3].gid]
    t = time.perf_counter()
    Mc, prc = partial_decrypt_batch(G, share, qbar, texts, nonces)
    rk = tr.recovery_public_key(gk[3].gid)
    comp_s = time.perf_counter() - t

    # mediator: eg_verify_shares on the wire arrays (what Decryption.decrypt calls per trustee)
    import ctypes
    from electionguard.core import native
    from electionguard.core.group import p_bytes, q_bytes
    Ki = np.tile(np.frombuffer(p_bytes(gk[0].public_key), np.uint8), (n, 1))
    ok = np.zeros(n, np.uint8)
    ptr = lambda x: x.ctypes.data_as(ctypes.c_void_p)
    qb = q_bytes(qbar)
    t = time.perf_counter()
    native.check(G._lib, "eg_verify_shares",
                 G._lib.eg_verify_shares(G.handle, native.buf(qb), ptr(Ki), ptr(texts), ptr(M), ptr(pr), n, ptr(ok)))
    ver_s = time.perf_counter() - t
    assert ok.all(), "share proofs must verify"

    out = {
        "metric": "trustee decryption shares with proofs / s (one DecryptingTrustee on one GPU)",
        "texts_per_rpc": n,
        "direct_shares_per_s": round(n / direct_s, 1),
        "compensated_shares_per_s": round(n / comp_s, 1),
        "mediator_share_verifications_per_s": round(n / ver_s, 1),
        "config": "configs[3] shape: 5 guardians, quorum 3, guardians 4,5 missing; EG 1.0 4096-bit group",
    }
    if a.cpu_sample > 0:
        from eg_oracle_c import COracle
        from electionguard.core import constants as C
        co = COracle(C.P, C.Q, C.G)
        s = min(a.cpu_sample, n)
        thr = a.cpu_threads or len(os.sched_getaffinity(0))  # every core this process may use
        try:  # ... capped by a cgroup CPU quota (more threads than the quota only time-slice)
            qq = open("/sys/fs/cgroup/cpu.max").read().split()
            if not a.cpu_threads and qq[0] != "max":
                thr = max(1, min(thr, int(int(qq[0]) / int(qq[1]) + 0.5)))
        except (OSError, ValueError, IndexError):
            pass
        secret = np.frombuffer(int(gk[0].secret).to_bytes(32, "big"), np.uint8)
        from concurrent.futures import ThreadPoolExecutor

        def work(lo, hi):  # ctypes drops the GIL: one slice per host thread
            co.powp(texts[lo:hi, 0], np.tile(secret, (hi - lo, 1)))
            co.powp(texts[lo:hi, 0], nonces[lo:hi])
            co.gpowp(nonces[lo:hi])

        co.gpowp(nonces[:1])  # builds the radix table once, before the threads share it
        edges = np.linspace(0, s, thr + 1).astype(int)
        t = time.perf_counter()
        # per share: A^s, A^u (variable base) + g^u (fixed base), as the JVM trustee does
        with ThreadPoolExecutor(thr) as ex:
            list(ex.map(lambda i: work(edges[i], edges[i + 1]), range(thr)))
        dt = time.perf_counter() - t
        out["cpu_baseline"] = {"value": round(s / dt, 2), "unit": "direct shares/s", "cores": thr, "kind": "port",
                               "sample": f"{s} texts: 2 BN_mod_exp_mont + 1 8-bit radix fixed base each"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
