"""Per-element powP through the coalescer on its three layouts (verdict r03 item 5): one element per
wave (eg_pow16.hip egw, the default for batches up to one element per SIMD), the 16-lane groups
(EG_LATENCY_POW=16: small batches up to one resident round on eg16) and the 8-lane layout
(EG_LATENCY_POW=0), for 11 and 1 blocking caller threads and a one-batch latency
sweep, next to the host CPU's variable-base rate (the bench line's cpu_baseline
var_base_modexp_per_s_per_core, OpenSSL BN_mod_exp_mont on one core) x 11 threads and x the lease's
cores.  Expected results come from CPython pow (every result is checked by coalesce_bench).

    python tools/coalesce_shapes.py [--n 12288] [--per-core 1686] [--cores 16] > profiles/<tag>_coalesce_shapes.json
"""
import argparse
import json
import os
import random
import struct
import subprocess
import sys
import tempfile
from multiprocessing import Pool
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "electionguard-remote_amd" / "host" / "_build" / "coalesce_bench"
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))


def _rec(args):
    i, seed = args
    from electionguard.core import constants as C
    rng = random.Random(seed * 1_000_003 + i)
    b, e, b2 = rng.randrange(C.P), rng.randrange(C.Q), rng.randrange(C.P)
    return (b.to_bytes(512, "big") + e.to_bytes(32, "big") + pow(b, e, C.P).to_bytes(512, "big") +
            b2.to_bytes(512, "big") + (b * b2 % C.P).to_bytes(512, "big") + pow(C.G, e, C.P).to_bytes(512, "big"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=12288)
    ap.add_argument("--n-single", type=int, default=1024, help="elements of the one-caller runs")
    ap.add_argument("--per-core", type=float, default=1686.0, help="host variable-base powP/s on one core")
    ap.add_argument("--cores", type=int, default=16, help="the lease's usable host cores")
    a = ap.parse_args()
    with Pool(min(16, os.cpu_count() or 1)) as pool:
        recs = pool.map(_rec, [(i, 7) for i in range(a.n)], chunksize=64)
    with tempfile.TemporaryDirectory() as d:
        vec = Path(d) / "v.bin"
        vec.write_bytes(struct.pack("<I", a.n) + b"".join(recs))
        # one blocking caller pays the whole latency per element: a smaller set keeps each run short
        n1 = min(a.n, a.n_single)
        vec1 = Path(d) / "v1.bin"
        vec1.write_bytes(struct.pack("<I", n1) + b"".join(recs[:n1]))
        res = {}
        for shape, env in (("per-wave", {}), ("per-wave-cios", {"EG_POWWAVE_D2": "0"}), ("16-lane", {"EG_LATENCY_POW": "16"}),
                           ("8-lane", {"EG_LATENCY_POW": "0"})):
            for threads in (11, 1):
                r = subprocess.run([str(BIN), str(vec if threads > 1 else vec1), str(threads)], capture_output=True,
                                   text=True, timeout=900, env=dict(os.environ, **env))
                if r.returncode:
                    sys.exit(r.stdout + r.stderr)
                res[f"{shape}/{threads}"] = json.loads(r.stdout.strip().splitlines()[-1])
                print(f"{shape}/{threads}: {res[f'{shape}/{threads}']['powp_one_blocking_per_s']} powP/s blocking",
                      file=sys.stderr, flush=True)
    cpu11 = a.per_core * 11
    cpu_all = a.per_core * a.cores
    out = {"n": a.n, "n_single_caller": min(a.n, a.n_single), "host_per_core_powp_per_s": a.per_core, "host_cores": a.cores,
           "host_11_threads_powp_per_s": cpu11, "host_all_cores_powp_per_s": cpu_all, "runs": res}
    # the batch size above which one GPU batch beats the host's cores on the same elements
    for shape in ("per-wave", "per-wave-cios", "16-lane", "8-lane"):
        sweep = res[f"{shape}/11"]["sweep"]
        out[f"crossover_vs_{a.cores}_cores_{shape}"] = next(
            (s["m"] for s in sweep if s["m"] / (s["coalesced_ms"] / 1e3) > cpu_all), None)
        out[f"blocking_11_threads_{shape}_per_s"] = res[f"{shape}/11"]["powp_one_blocking_per_s"]
        out[f"blocking_1_thread_{shape}_per_s"] = res[f"{shape}/1"]["powp_one_blocking_per_s"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
