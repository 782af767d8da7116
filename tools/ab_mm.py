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
    if not flags.strip():  # no -D flags: the in-tree library (run-time switches only, e.g. name@sel42)
        return ROOT / "electionguard-remote_amd" / "electionguard" / "lib" / "libeg_hip.so"
    BUILD.mkdir(exist_ok=True)
    out = BUILD / f"libeg_{name}.so"
    if not out.exists():  # both translation units (the 8-lane core and the 16-lane eg_pow16.hip)
        csrc = ROOT / "electionguard-remote_amd" / "csrc"
        cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-fno-slp-vectorize",
               "-Wno-unused-result", "-Wno-pass-failed", *flags.split(), "-I", str(ROOT / "include"), "-o", str(out),
               str(csrc / "eg_capi.hip"), str(csrc / "eg_pow16.hip")]
        subprocess.run(cmd, check=True)
    return out


VERIFY_CODE = """
import sys, json, time, numpy as np
sys.path.insert(0, {root!r})
from electionguard.ballot import ElectionKey, Manifest, Verifier, batch_encryption, random_scalars, random_votes
from electionguard.core import productionGroup
from electionguard.keyceremony import key_ceremony
G = productionGroup(0)
gk, K = key_ceremony(G, 3, 3, seed=5)
key = ElectionKey(G, K, window_bits={wb})
man = Manifest(4, 5, 1)
rng = np.random.default_rng(0)
nb = {nb}
votes = random_votes(rng, man, nb)
eb = batch_encryption(G, key, 77, man, votes, random_scalars(rng, (nb, man.nsel, 4), G.q), random_scalars(rng, (nb, man.n_contests), G.q))
V = Verifier(G, key, 77, man)
ok_s, ok_c, _ = V.verify(eb)
assert ok_s.all() and ok_c.all()
best = None
for _ in range({reps}):
    G.profile_begin(); t = time.perf_counter(); V.verify(eb); dt = time.perf_counter() - t; kp = G.profile_end(); ms, mm = kp.ms, kp.mont_ops
    # MM per shader clock (the in-kernel clock of the same launches) takes the box's DVFS out
    r = (nb / dt, mm / (ms / 1e3), mm / nb, kp.clock_ghz, mm / (ms / 1e3) / (kp.clock_ghz * 1e9) if kp.clock_ghz else 0.0)
    best = r if best is None or r[1] > best[1] else best
print(json.dumps({{"ballots_per_s": best[0], "mm_per_s": best[1], "mm_per_ballot": best[2], "clock_ghz": best[3],
                  "mm_per_kclock": best[4] * 1e3}}))
"""


ENCRYPT_CODE = """
import sys, json, time, numpy as np
sys.path.insert(0, {root!r})
from electionguard.ballot import ElectionKey, Manifest, batch_encryption, random_scalars, random_votes
from electionguard.core import productionGroup
from electionguard.keyceremony import key_ceremony
G = productionGroup(0)
gk, K = key_ceremony(G, 3, 3, seed=5)
key = ElectionKey(G, K, window_bits={wb})
man = Manifest(4, 5, 1)
rng = np.random.default_rng(0)
nb = {nb}
votes = random_votes(rng, man, nb)
sn, cn = random_scalars(rng, (nb, man.nsel, 4), G.q), random_scalars(rng, (nb, man.n_contests), G.q)
ref = batch_encryption(G, key, 77, man, votes, sn, cn)
best = None
for _ in range({reps}):
    G.profile_begin(); t = time.perf_counter(); eb = batch_encryption(G, key, 77, man, votes, sn, cn); dt = time.perf_counter() - t; kp = G.profile_end(); ms, mm = kp.ms, kp.mont_ops
    assert (eb.cts == ref.cts).all() and (eb.rproof == ref.rproof).all()
    r = (nb / dt, mm / (ms / 1e3), mm / nb, ms)
    best = r if best is None or r[0] > best[0] else best
print(json.dumps({{"ballots_per_s": best[0], "kpow_mm_per_s": best[1], "mm_per_ballot": best[2], "kpow_ms": best[3]}}))
"""


def measure_verify(lib, nb, reps, env_extra=None, code_tmpl=VERIFY_CODE):
    env = dict(os.environ, EG_LIB=str(lib), **(env_extra or {}))
    code = code_tmpl.format(root=str(ROOT / "electionguard-remote_amd"), nb=nb, reps=reps,
                            wb=int(os.environ.get("AB_WB", "16")))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return {"error": out.stderr[-800:]}
    return json.loads(out.stdout.strip().splitlines()[-1])


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
    G.profile_begin(); G.powP_batch(B, E); kp = G.profile_end()
    r = (kp.mont_ops / (kp.ms / 1e3), kp.macs / (kp.ms / 1e3) / 1e12)
    best = r if best is None or r[0] > best[0] else best
print(json.dumps({{"mm_per_s": best[0], "tmac": best[1]}}))
"""
    env = dict(os.environ, EG_LIB=str(lib))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        return {"error": out.stderr[-800:]}
    return json.loads(out.stdout.strip().splitlines()[-1])


if __name__ == "__main__":
    n = int(os.environ.get("AB_N", "131072"))
    mode = os.environ.get("AB_MODE", "powp")
    res = {}
    for arg in sys.argv[1:]:
        name, flags = arg.split("=", 1)
        env_extra = {}
        if name.endswith("@nocomb"):
            env_extra["EG_NO_COMB"] = "1"
        if name.endswith("@notail"):
            env_extra["EG_TAIL_SPLIT"] = "0"
        if name.endswith("@cbl3"):  # every contest-b job in launch 3 (the default schedule)
            env_extra["EG_CB_EARLY"] = "0"
        if "@cbe" in name:  # early contest-b jobs in launch 2 (opt-in schedule)
            env_extra["EG_CB_EARLY"] = "1"
        for sel in ("43", "42", "44", "52"):  # verifier selection jobs' comb: rows x column blocks
            if f"@sel{sel}" in name:
                env_extra["EG_SEL_COMB"] = sel
        if "@l3w" in name:  # with @cbe: launch 3 sized to 1..3 waves per SIMD (default 2)
            env_extra["EG_CB_EARLY"] = "1"
            env_extra["EG_L3_WAVES"] = name.split("@l3w")[1][:1]
        lib = build(name.split("@")[0], flags)
        nb = int(os.environ.get("AB_NB", "4000"))
        if mode == "verify":
            res[name] = measure_verify(lib, nb, 3, env_extra)
        elif mode == "encrypt":
            res[name] = measure_verify(lib, nb, 3, env_extra, ENCRYPT_CODE)
        else:
            res[name] = measure(lib, n, 3)
        print(name, res[name], flush=True)
    print(json.dumps(res))
