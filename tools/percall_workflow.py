"""Rates of the reference's per-element call pattern through the L1 drop-in:
tests/cpp/percall_workflow.cpp on 11 threads against the CPU port on 11 threads, same ballots, same
run; the deferred per-element API (default), the same calls blocking one at a time (eager), and the
constant-time schedules (ct); and the deferred run with the per-wave kernel's variable parts on one wave
(EG_WAVE_R2L=0: the left-to-right sliding window) against the default right-to-left chain over four
waves.  Prints one JSON object (commit it under profiles/).

    python tools/percall_workflow.py [nballots=1100]"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "electionguard-remote_amd" / "host" / "_build" / "percall_workflow"


def run(n, *mode, env=None):
    t = time.time()
    r = subprocess.run([str(BIN), str(n), "11", *mode], capture_output=True, text=True, timeout=900,
                       env={**os.environ, **(env or {})})
    if r.returncode != 0:
        sys.exit(f"percall_workflow {n} {mode} failed:\n{r.stdout}\n{r.stderr}")
    d = json.loads(r.stdout.strip().splitlines()[-1])
    d["wall_s"] = round(time.time() - t, 2)
    print(f"{mode or 'deferred'}: {d}", file=sys.stderr, flush=True)
    return d


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1100
    out = {"deferred": run(n), "deferred_var_one_wave": run(n, env={"EG_WAVE_R2L": "0"}),
           "constant_time": run(n, "ct"), "eager": run(max(22, n // 10), "eager")}
    d = out["deferred"]
    out["summary"] = {
        "encrypt_gpu_over_cpu_port": round(d["encrypt_ballots_per_s"]["gpu_per_element"] /
                                           d["encrypt_ballots_per_s"]["cpu_port"], 3),
        "verify_gpu_over_cpu_port": round(d["verify_ballots_per_s"]["gpu_per_element"] /
                                          d["verify_ballots_per_s"]["cpu_port"], 3),
        "tally_gpu_over_cpu_port": round(d["tally_ballots_per_s_one_thread"]["gpu_per_element"] /
                                         d["tally_ballots_per_s_one_thread"]["cpu_port"], 3),
        "verify_r2l_over_one_wave": round(d["verify_ballots_per_s"]["gpu_per_element"] /
                                          out["deferred_var_one_wave"]["verify_ballots_per_s"]["gpu_per_element"], 3),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
