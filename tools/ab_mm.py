"""A/B timing of Montgomery-multiply variants: builds (or reuses) libraries compiled with
different -D flags and measures k_pow throughput on a large powP batch (device time via
HIP events on the ctx stream).  Usage on the GPU box:
    python tools/ab_mm.py VARIANT=flags ...   e.g.  t8="-DEG_T=8" t4="-DEG_T=4"
"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))
BUILD = ROOT / "tools" / "_ab"


def build(name, flags):
    BUILD.mkdir(exist_ok=True)
    out = BUILD / f"libeg_{name}.so"
    if not out.exists():
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
               "-Wno-unused-result", "-Wno-pass-failed", *flags.split(), "-I", str(ROOT / "include"), "-o", str(out),
               str(ROOT / "electionguard-remote_amd" / "csrc" / "eg_capi.hip")]
        subprocess.run(cmd, check=True)
    return out


def measure(lib, n, reps):
    code = f"""
import sys, json, numpy as np
sys.path.insert(0, {str(ROOT / 'electionguard-remote_amd')!r})
from electionguard.core import productionGroup
G = productionGroup(0)
rng = np.random.default_rng(0)
B = rng.integers(0, 256, size=({n}, 512), dtype=np.uint8); B[:, 0] = 0
E = rng.integers(0, 256, size=({n}, 32), dtype=np.uint8)
G.powP_batch(B[:1024], E[:1024])
best = None
for _ in range({reps}):
    G.profile_begin(); G.powP_batch(B, E); ms, mm, nl = G.profile_end()
    r = mm / (ms / 1e3)
    best = r if best is None or r > best else best
print(json.dumps({{"mm_per_s": best, "tmac": best * 32768 / 1e12}}))
"""
    env = dict(os.environ, EG_LIB=str(lib))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return {"error": out.stderr[-800:]}
    return json.loads(out.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    n = int(os.environ.get("AB_N", "131072"))
    res = {}
    for arg in sys.argv[1:]:
        name, flags = arg.split("=", 1)
        lib = build(name, flags)
        res[name] = measure(lib, n, 3)
        print(name, res[name], flush=True)
    print(json.dumps(res))
