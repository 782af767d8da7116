"""The one knob the reference's caller owns: the thread count of batchEncryption(..., nthreads = 11, ...)
and new Verifier(record, nthreads) (RunRemoteWorkflowTest.java:140,180).  Runs the per-element
workflow driver (tests/cpp/percall_workflow.cpp: upstream's per-selection call order through the L1
drop-in's per-element API, every byte and verdict checked against the CPU port) at several caller
thread counts, and the batch path (bench.py) once in the same call for the rates the per-element
path is compared with.  Prints one JSON object (commit it under profiles/).

    python tools/percall_threads.py [threads=11,32,64,128,256,512]"""
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "electionguard-remote_amd" / "host" / "_build" / "percall_workflow"


def run_percall(threads: int, nb: int) -> dict:
    t = time.time()
    r = subprocess.run([str(BIN), str(nb), str(threads)], capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        sys.exit(f"percall_workflow {nb} {threads} failed:\n{r.stdout[-2000:]}\n{r.stderr[-2000:]}")
    d = json.loads(r.stdout.strip().splitlines()[-1])
    d["wall_s"] = round(time.time() - t, 2)
    print(f"threads {threads}: encrypt {d['encrypt_ballots_per_s']['gpu_per_element']:.0f}/s, verify "
          f"{d['verify_ballots_per_s']['gpu_per_element']:.0f}/s ({d['wall_s']} s)", file=sys.stderr, flush=True)
    return d


def batch_rates() -> dict:
    """bench.py's configs[1] line (10k ballots, batch API): verify + tally and encryption rates."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--steps", "3", "--warmup", "1", "--cpu-sample", "0",
                        "--modexp-n", "0", "--ct-encrypt", "0"], capture_output=True, text=True, timeout=900)
    if r.returncode != 0:
        sys.exit(f"bench.py failed:\n{r.stderr[-2000:]}")
    line = json.loads(r.stdout.strip().splitlines()[-1])
    return {"verify_ballots_per_s": line["value"], "encrypt_ballots_per_s_host_pointer": line["encrypt_ballots_per_s_per_gpu"],
            "encrypt_ballots_per_s_device_resident": line["encrypt_ballots_per_s_per_gpu_device_resident"],
            "build": line.get("build"), "clock_ghz": line.get("roofline", {}).get("clock_ghz")}


def main():
    threads = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "11,32,64,128,256,512").split(",")]
    batch = batch_rates()
    print(f"batch: {batch}", file=sys.stderr, flush=True)
    rows = []
    for T in threads:
        # enough ballots that every thread walks >= 4 of them (the driver strides ballots over threads)
        nb = max(1100, 8 * T)
        d = run_percall(T, nb)
        mism = sum(d[k] for k in ("encrypt_mismatched_arrays", "verify_flag_mismatches", "invalid_flags",
                                  "tamper_not_rejected", "tally_mismatch", "errors", "trustee_mismatched_arrays"))
        enc, ver = d["encrypt_ballots_per_s"], d["verify_ballots_per_s"]
        rows.append({"threads": T, "ballots": nb, "bit_exact": mism == 0,
                     "encrypt_per_s": enc["gpu_per_element"], "encrypt_cpu_port_per_s": enc["cpu_port"],
                     "verify_per_s": ver["gpu_per_element"], "verify_cpu_port_per_s": ver["cpu_port"],
                     "encrypt_frac_of_batch": round(enc["gpu_per_element"] / batch["encrypt_ballots_per_s_host_pointer"], 4),
                     "verify_frac_of_batch": round(ver["gpu_per_element"] / batch["verify_ballots_per_s"], 4),
                     "wall_s": d["wall_s"], "raw": d})
    out = {"what": "per-element L1 drop-in (tests/cpp/percall_workflow.cpp) at caller thread counts, against the "
                   "batch API on the same box (bench.py configs[1]); CPU port on the same thread count",
           "cpu_threads_available": len(os.sched_getaffinity(0)), "batch": batch, "rows": rows}
    print(json.dumps(out, indent=1))
    return 0 if all(r["bit_exact"] for r in rows) else 1


if __name__ == "__main__":
    sys.exit(main())
