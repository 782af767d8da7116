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
    rounds = int(os.environ.get("PERCALL_ROUNDS", "2"))
    # the right-to-left / one-wave A/B interleaved over `rounds` (the per-element rates move with the
    # host's thread scheduling from run to run); the summary quotes the first deferred run
    ab = []
    for _ in range(rounds):
        ab.append({"deferred": run(n), "deferred_var_one_wave": run(n, env={"EG_WAVE_R2L": "0"})})
    out = dict(ab[0])
    out["ab_rounds"] = [{k: {"encrypt": v["encrypt_ballots_per_s"]["gpu_per_element"],
                             "verify": v["verify_ballots_per_s"]["gpu_per_element"]} for k, v in r.items()} for r in ab]
    out["constant_time"] = run(n, "ct")
    out["eager"] = run(max(22, n // 10), "eager")
    d = out["deferred"]

    def best(kind, key):
        return max(r[kind][key]["gpu_per_element"] for r in ab)

    out["summary"] = {
        "encrypt_gpu_over_cpu_port": round(d["encrypt_ballots_per_s"]["gpu_per_element"] /
                                           d["encrypt_ballots_per_s"]["cpu_port"], 3),
        "verify_gpu_over_cpu_port": round(d["verify_ballots_per_s"]["gpu_per_element"] /
                                          d["verify_ballots_per_s"]["cpu_port"], 3),
        "tally_gpu_over_cpu_port": round(d["tally_ballots_per_s_one_thread"]["gpu_per_element"] /
                                         d["tally_ballots_per_s_one_thread"]["cpu_port"], 3),
        "trustee_gpu_ct_over_cpu_port_one_thread": round(
            d["trustee_shares_per_s_one_thread"]["gpu_per_element_constant_time"] /
            d["trustee_shares_per_s_one_thread"]["cpu_port"], 3),
        "verify_r2l_over_one_wave_best": round(best("deferred", "verify_ballots_per_s") /
                                               best("deferred_var_one_wave", "verify_ballots_per_s"), 3),
        "encrypt_r2l_over_one_wave_best": round(best("deferred", "encrypt_ballots_per_s") /
                                                best("deferred_var_one_wave", "encrypt_ballots_per_s"), 3),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
