"""Fold the rocprofv3 CSVs written by tools/profile_round.sh into profiles/<tag>_*.

Timed-region selection: bench.py's timed steps are the LAST `roofline.launches` k_pow
dispatches of each run (nothing launches k_pow after the timed region), so the
kernel-trace average over exactly those dispatches is the number that must agree with
bench.py's HIP-event `kernel_ms_per_launch`, and the PMC sums over the same dispatches
give per-launch HBM bytes and VALU issue counts.

Corrections (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE and WRITE_SIZE are
KB; on gfx950 FETCH_SIZE counts half the bytes of wide streaming reads, so it is
doubled; WRITE_SIZE is taken as is.
"""
import argparse
import csv
import glob
import json
import os
import shutil
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
KPOW = "eg::k_pow<"


def bench_line(path):
    for line in reversed(Path(path).read_text().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no bench JSON in {path}")


def one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"missing {pattern}")
    return hits[0]


def kpow_trace(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if KPOW in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    return [(e - s) for s, e in rows]


def kpow_counters(path):
    """-> list (dispatch order) of {counter: summed value} for k_pow dispatches."""
    per = defaultdict(lambda: defaultdict(float))
    order = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if KPOW not in r["Kernel_Name"]:
                continue
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            order.setdefault(d, int(r["Start_Timestamp"]))
    return [per[d] for d in sorted(per, key=lambda k: order[k])]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--tag", default="r01")
    a = ap.parse_args()
    d = Path(a.dir)
    prof = ROOT / "profiles"
    prof.mkdir(exist_ok=True)

    bl = bench_line(d / "bench_trace.log")
    n = int(bl["roofline"]["launches"])
    ops_total = bl["roofline"]["mont_ops_per_launch"] * n

    stats = one(str(d / "trace" / "**" / "*kernel_stats.csv"))
    shutil.copy(stats, prof / f"{a.tag}_rocprof_kernel_stats.csv")
    durs = kpow_trace(one(str(d / "trace" / "**" / "*kernel_trace.csv")))
    timed = durs[-n:]
    out = {
        "source": "tools/profile_round.sh: rocprofv3 --kernel-trace --stats, then separate --pmc passes "
                  "(FETCH_SIZE | WRITE_SIZE | SQ_*+GRBM_GUI_ACTIVE) of `python3 bench.py` (defaults); "
                  "timed region = last `launches` k_pow dispatches; FETCH_SIZE x2 (gfx950)",
        "bench": {k: bl[k] for k in ("value", "unit", "ms_per_step", "steps", "warmup")},
        "bench_config": bl["config"],
        "bench_build": bl.get("build"),
        "bench_roofline": bl["roofline"],
        "rocprof": {
            "kpow_dispatches_all": len(durs),
            "kpow_avg_ms_all": sum(durs) / len(durs) / 1e6 if durs else None,
            "kpow_timed_dispatches": len(timed),
            "kpow_avg_ms_timed": sum(timed) / len(timed) / 1e6 if timed else None,
            "bench_hip_event_ms_per_launch": bl["roofline"]["kernel_ms_per_launch"],
        },
    }
    r = out["rocprof"]
    if r["kpow_avg_ms_timed"]:
        r["agreement"] = r["bench_hip_event_ms_per_launch"] / r["kpow_avg_ms_timed"]

    fetch = kpow_counters(one(str(d / "fetch" / "**" / "*counter_collection.csv")))[-n:]
    write = kpow_counters(one(str(d / "write" / "**" / "*counter_collection.csv")))[-n:]
    fb = sum(c["FETCH_SIZE"] for c in fetch) * 1024 * 2
    wb = sum(c["WRITE_SIZE"] for c in write) * 1024
    out["traffic"] = {
        "fetch_bytes_timed": fb,
        "write_bytes_timed": wb,
        "hbm_bytes_per_launch": (fb + wb) / n,
        "hbm_bytes_per_mont_op": (fb + wb) / ops_total,
        "hbm_GBps_at_kernel_rate": (fb + wb) / n / (r["kpow_avg_ms_timed"] / 1e3) / 1e9,
    }
    sq = kpow_counters(one(str(d / "sq" / "**" / "*counter_collection.csv")))[-n:]
    insts = sum(c["SQ_INSTS_VALU"] for c in sq)
    grbm = sum(c["GRBM_GUI_ACTIVE"] for c in sq)
    xcds = 8
    out["valu"] = {
        "SQ_INSTS_VALU_timed": insts,
        "GRBM_GUI_ACTIVE_per_xcd_timed": grbm / xcds,
        # VALU wave-instructions per CU per cycle (1.0 = every SIMD issues every 4 cycles)
        "valu_issue_util": insts / (grbm / xcds * 256),
        # one wave runs 64/8 = 8 elements' Montgomery ops in lockstep
        "valu_instr_per_mont_op_per_lane": insts * 8 / ops_total,
        "SQ_ACTIVE_INST_VALU_timed": sum(c["SQ_ACTIVE_INST_VALU"] for c in sq),
        "SQ_WAVE_CYCLES_timed": sum(c["SQ_WAVE_CYCLES"] for c in sq),
    }
    (prof / f"{a.tag}_pmc_kpow.json").write_text(json.dumps(out, indent=1))
    shutil.copy(d / "bench_trace.log", prof / f"{a.tag}_bench_profiled.log")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
