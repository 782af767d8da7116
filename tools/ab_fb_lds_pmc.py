"""Per-variant HBM bytes of tools/ab_fb_lds.py from a rocprofv3 --pmc FETCH_SIZE pass (AB_ROUNDS=1): the
last four exponentiation dispatches (k_pow x 3, k_fb_lds) are round 1's hbm22, hbm8, hbm7, lds7.
FETCH_SIZE is KB and, on gfx950, half the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM /
rocprofv3 section): both the raw and the doubled figure are printed.

    python tools/ab_fb_lds_pmc.py OUTDIR n"""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def main():
    out, n = Path(sys.argv[1]), int(sys.argv[2])
    per, names = defaultdict(float), {}
    for f in out.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if ("k_pow" in k or "k_fb_lds" in k) and r["Counter_Name"] == "FETCH_SIZE":
                d = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
                per[d] += float(r["Counter_Value"])
                names[d] = k.split("(")[0]
    disp = sorted(per)[-4:]
    print(f"FETCH_SIZE of round 1's exponentiation dispatches (n = {n} exponents each)")
    for v, d in zip(("hbm22", "hbm8", "hbm7", "lds7"), disp):
        kb = per[d]
        print(f"  {v:6s} {names[d]:32s} FETCH_SIZE {kb:14.0f} KB raw, x2 = {2 * kb * 1024 / 1e9:8.3f} GB, "
              f"{2 * kb * 1024 / n:10.0f} B per exponentiation")


if __name__ == "__main__":
    main()
