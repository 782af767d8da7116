"""Latency of one per-element exponentiation on the per-wave kernel (the shape upstream's per-element
callers wait on), for the A/Bs of its multiply variants (env read at context creation, e.g.
EG_WAVE_R2L=0, EG_POWWAVE_D2=0).  Every result is checked against CPython.

    python tools/ab_wave_latency.py [calls=200]
Prints one JSON line: blocking powP (eg_powp_one, one thread), a one-element eg_powp_batch, and a
blocking g^v * alpha^c job (eg_mexp_one), median and best microseconds per call."""
import json
import os
import random
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    from electionguard.core import constants
    from electionguard.core.group import GroupContext
    p, q, g = constants.P, constants.Q, constants.G
    G = GroupContext(p, q, g, 0)
    rng = random.Random(3)
    xs = [(rng.randrange(p), rng.randrange(q), rng.randrange(q)) for _ in range(calls)]

    def timed(f, check):
        ts = []
        for i, (b, e, v) in enumerate(xs):
            t = time.perf_counter()
            r = f(b, e, v)
            ts.append(time.perf_counter() - t)
            if i % 7 == 0:
                assert int.from_bytes(bytes(r), "big") == check(b, e, v), i
        ts = ts[5:]  # warm-up calls
        return {"median_us": round(statistics.median(ts) * 1e6, 1), "best_us": round(min(ts) * 1e6, 1)}

    out = {"env": {k: os.environ[k] for k in ("EG_COOP", "EG_POWWAVE_CYL", "EG_WAVE_R2L", "EG_POWWAVE_D2")
                   if k in os.environ},
           "calls": calls}
    out["powp_one"] = timed(lambda b, e, v: G.powP_one(b, e), lambda b, e, v: pow(b, e, p))
    out["powp_batch1"] = timed(lambda b, e, v: G.powP_batch([b], [e])[0].tobytes(), lambda b, e, v: pow(b, e, p))
    out["g_v_alpha_c"] = timed(lambda b, e, v: G.mexp_one([b], e, [(None, v)]),
                               lambda b, e, v: pow(b, e, p) * pow(g, v, p) % p)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
