"""Which proof conventions does a record use?  (The upstream ones are unpinned: the reference's
arithmetic lives in electionguard-kotlin-multiplatform-jvm 1.0-SNAPSHOT, absent here, and its wire
format common.proto:23-28 pins only the field names "c" and "v".)

``pin_formats`` verifies the wire-layout ballots and trustee shares of a record (common.proto byte
layouts: 512-byte ElementModP, 32-byte ElementModQ, big-endian) on the GPU under every combination
of the three switchable conventions -- the hash pre-image's hex form (eg_ctx_set_hash_format), the
response sign and the challenge pre-image order (eg_ctx_set_proof_format) -- and reports the
combinations under which everything verifies.  Proofs made under one response / pre-image order
fail under every other (a different challenge or a different commitment), so an honest record pins
both; the two hex forms hash the same text unless a hashed element has a leading zero byte (about
1 element in 256 for random 4096-bit values), so a small record may leave the hex form open.

Record (JSON, hex strings; tools/pin_format.py):
  {"K": ..., "qbar": ..., "manifest": [contests, selections, votes_allowed],
   "ballots": [{"cts": [[alpha, beta], ...], "rproofs": [[c0, v0, c1, v1], ...],
                "cproofs": [[c, v], ...]}, ...],                      # optional
   "shares": [{"text": [pad, data], "key": K_i, "M": ..., "c": ..., "v": ...}, ...]}   # optional
"""
from __future__ import annotations

import itertools
from typing import Dict, List

import numpy as np

HASH_FORMATS = ("fixed", "minimal")
RESPONSES = ("minus", "plus")
PREIMAGES = ("message_first", "commitments_first", "with_key")


def _h(s: str, n: int) -> np.ndarray:
    return np.frombuffer(bytes.fromhex(s).rjust(n, b"\0")[-n:], np.uint8)


def record_arrays(rec: dict):
    """-> (ballot arrays or None, share arrays or None) in the C ABI layouts."""
    ballots = shares = None
    if rec.get("ballots"):
        nc, ns, va = rec["manifest"]
        nsel = nc * (ns + va)
        bs = rec["ballots"]
        cts = np.stack([np.stack([_h(x, 512) for ct in b["cts"] for x in ct]).reshape(nsel, 2, 512) for b in bs])
        rp = np.stack([np.stack([_h(x, 32) for pr in b["rproofs"] for x in pr]).reshape(nsel, 4, 32) for b in bs])
        cp = np.stack([np.stack([_h(x, 32) for pr in b["cproofs"] for x in pr]).reshape(nc, 2, 32) for b in bs])
        ballots = (cts, rp, cp)
    if rec.get("shares"):
        sh = rec["shares"]
        T = np.stack([np.stack([_h(s["text"][0], 512), _h(s["text"][1], 512)]) for s in sh])
        Ki = np.stack([_h(s["key"], 512) for s in sh])
        M = np.stack([_h(s["M"], 512) for s in sh])
        pr = np.stack([np.stack([_h(s["c"], 32), _h(s["v"], 32)]) for s in sh])
        shares = (T, Ki, M, pr)
    return ballots, shares


def pin_formats(group, rec: dict) -> List[Dict]:
    """Verify the record's ballots and shares under every (hash form, response, pre-image order)
    on ``group``'s GPU; -> one entry per combination with the fraction of ballots and shares that
    verify (the context's settings are restored afterwards)."""
    from .ballot import ElectionKey, EncryptedBallots, Manifest, Verifier
    from .decrypt import verify_shares

    ballots, shares = record_arrays(rec)
    qbar = int(rec["qbar"], 16)
    saved = (group.hash_format, group.proof_format)
    V = None
    if ballots is not None:
        nc, ns, va = rec["manifest"]
        V = Verifier(group, ElectionKey(group, int(rec["K"], 16)), qbar, Manifest(nc, ns, va))
    out = []
    try:
        for hf, resp, pre in itertools.product(HASH_FORMATS, RESPONSES, PREIMAGES):
            group.hash_format = hf
            group.proof_format = (resp, pre)
            r = {"hash_format": hf, "response": resp, "preimage": pre}
            ok = True
            if V is not None:
                ok_s, ok_c, _ = V.verify(EncryptedBallots(*ballots), with_tally=False)
                valid = ok_s.all(axis=1) & ok_c.all(axis=1)
                r["ballots_valid"] = f"{int(valid.sum())}/{len(valid)}"
                ok &= bool(valid.all())
            if shares is not None:
                T, Ki, M, pr = shares
                v = verify_shares(group, qbar, Ki, T, M, pr)
                r["shares_valid"] = f"{int(np.sum(v))}/{len(v)}"
                ok &= bool(np.all(v))
            r["all_valid"] = ok
            out.append(r)
    finally:
        group.hash_format, group.proof_format = saved
    return out


def summarize(results: List[Dict]) -> Dict:
    """-> {"response", "preimage", "hash_format"}: each a name when every combination that verifies
    everything agrees on it, None when nothing verifies, "undetermined" when several values do."""
    hits = [r for r in results if r["all_valid"]]
    out = {}
    for k in ("response", "preimage", "hash_format"):
        vals = sorted({r[k] for r in hits})
        out[k] = vals[0] if len(vals) == 1 else (None if not vals else "undetermined")
    return out
