"""Summarise a tools/ct_schedule.py run under rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES: per batch (layout x
constant-time switch x exponent class) the VALU instructions of its exponentiation dispatch (k_pow /
k_wave_job), and per layout the spread over the exponent classes.

    python tools/ct_schedule_summary.py OUTDIR ct_schedule.log > profiles/r05x_ct_schedule.txt"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path


def main():
    out, logf = Path(sys.argv[1]), Path(sys.argv[2])
    batches = [json.loads(l) for l in logf.read_text().splitlines() if l.startswith("{")]
    rows = []
    for f in out.rglob("*counter_collection.csv"):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for r in rows:
        k = r.get("Kernel_Name", "")
        if "k_wave_job" not in k and "k_pow" not in k:
            continue
        d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
        per[d][r["Counter_Name"]] += float(r["Counter_Value"])
        names[d] = k
    disp = sorted(per)
    print(f"{len(disp)} exponentiation dispatches for {len(batches)} batches")
    if len(disp) != len(batches):
        print("WARNING: dispatch count differs from the batch count; matching in order anyway")
    groups = defaultdict(list)
    for b, d in zip(batches, disp):
        valu = per[d].get("SQ_INSTS_VALU", 0.0)
        b["valu"] = valu
        b["kernel"] = names[d].split("(")[0][:60]
        groups[(b["layout"], b["ct"])].append(b)
        print(f"  {b['layout']:28s} ct={int(b['ct'])} {b['exponents']:7s} n={b['n']:5d} VALU {valu:14.0f} "
              f"({valu / b['n']:10.1f} per element)  {b['per_s']:10.1f} /s  {b['kernel']}")
    print()
    for (layout, ct), bs in sorted(groups.items()):
        v = [b["valu"] for b in bs]
        spread = (max(v) - min(v)) / max(v) if max(v) else 0.0
        print(f"{layout:28s} {'constant-time' if ct else 'variable-time':14s} VALU spread over exponent classes "
              f"{spread:8.3%}   rate (random) {next(b['per_s'] for b in bs if b['exponents'] == 'random'):10.1f} /s")


if __name__ == "__main__":
    main()
