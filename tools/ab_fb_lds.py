"""A/B of the north_star's LDS-staged fixed-base tables against the HBM radix tables.

Fixed-base exponentiation is the whole of the encryptor's k_pow work (g^R, K^R, the proof commitments:
eg_encrypt_ballots_dev) and the fixed-base half of the verifier's.  Four ways to compute base^e for
n device-resident 256-bit exponents (one base, the election key K), all through eg_fb_pow_batch_dev:
  hbm22   k_pow over the 22-bit radix table in HBM (the production choice: 12 windows, 11 multiplies)
  hbm8    k_pow over an 8-bit table in HBM (LOW_MEMORY_USE's width: 32 windows, 31 multiplies)
  hbm7    k_pow over a 7-bit table in HBM (37 windows, 36 multiplies)
  lds7    k_fb_lds over the same 7-bit table, batch-major: each workgroup stages every window's
          table slice (128 entries, 80 KiB) in LDS and its 96 elements multiply straight out of it
          (EG_FB_LDS=1; SURVEY §7.5's plan -- 8-bit slices of 640-B entries would fill the whole LDS)
Interleaved rounds in one process on one box (the clock drifts between boxes, not between adjacent
launches), every variant bit-exact against CPython on a sample.  Prints one JSON object.

    python tools/ab_fb_lds.py [n=262144] [rounds=4]
Under rocprofv3 --pmc FETCH_SIZE (one round: AB_ROUNDS=1) the dispatch order hbm22, hbm8, hbm7, lds7
gives each variant's HBM bytes."""
import json
import os
import random
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
    rounds = int(os.environ.get("AB_ROUNDS", sys.argv[2] if len(sys.argv) > 2 else "4"))
    os.environ["EG_FB_LDS"] = "0"
    from electionguard.core import constants
    from electionguard.core.group import GroupContext
    p, q, g = constants.P, constants.Q, constants.G
    G = GroupContext(p, q, g, 0)
    os.environ["EG_FB_LDS"] = "1"  # read at context creation: the second context runs k_fb_lds for 7-bit tables
    GL = GroupContext(p, q, g, 0)
    rng = random.Random(11)
    K = pow(g, rng.randrange(q), p)
    tabs = {"hbm22": G.fixed_base(K, 22), "hbm8": G.fixed_base(K, 8), "hbm7": G.fixed_base(K, 7),
            "lds7": GL.fixed_base(K, 7)}
    mm = {"hbm22": 11, "hbm8": 31, "hbm7": 36, "lds7": 36}
    exps = [rng.randrange(q) for _ in range(n)]
    E = np.frombuffer(b"".join(e.to_bytes(32, "big") for e in exps), np.uint8).reshape(n, 32)
    dev = {}
    for name, fb in tabs.items():
        grp = fb.group
        dev[name] = (grp, grp.to_device(E), grp.device_empty((n, 512)))
    res = {k: [] for k in tabs}
    for r in range(rounds + 1):  # round 0 warms up (code objects, workspaces)
        for name, fb in tabs.items():
            grp, d_e, d_o = dev[name]
            grp.sync()
            t = time.perf_counter()
            fb.pow_batch_dev(d_e.ptr, d_o.ptr, n)
            grp.sync()
            dt = time.perf_counter() - t
            if r:
                res[name].append(n / dt)
            if r == 1:
                out = d_o.download()
                for i in range(0, n, max(1, n // 64)):
                    assert int.from_bytes(out[i].tobytes(), "big") == pow(K, exps[i], p), (name, i)
            print(json.dumps({"round": r, "variant": name, "exps_per_s": round(n / dt, 1)}), file=sys.stderr, flush=True)
    summary = {}
    for name, v in res.items():
        if not v:
            continue
        best = max(v)
        summary[name] = {"exps_per_s_best": round(best, 1), "exps_per_s_all": [round(x, 1) for x in v],
                         "mont_ops_per_exp": mm[name], "mm_per_s_best": round(best * mm[name], 1)}
    out = {"n": n, "rounds": rounds, "bitexact_sample": 64, "variants": summary}
    if "hbm22" in summary and "lds7" in summary:
        out["lds7_over_hbm22"] = round(summary["lds7"]["exps_per_s_best"] / summary["hbm22"]["exps_per_s_best"], 4)
        out["lds7_over_hbm7_mm_rate"] = round(summary["lds7"]["mm_per_s_best"] / summary["hbm7"]["mm_per_s_best"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
