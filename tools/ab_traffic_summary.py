"""Fold tools/ab_traffic.sh's runs into one JSON: per variant the bench rate, kernel ms per
launch, held clock and MACs/s of every interleaved run; HBM bytes per timed k_pow launch from
its FETCH_SIZE (x2 on gfx950) and WRITE_SIZE passes (the corrections of tools/prof_summary.py);
VALU instructions per Montgomery op per lane and the VALU issue rate from its SQ pass; and each
variant's ratios against the first one."""
import argparse
import glob
import json
from pathlib import Path

from prof_summary import bench_line, kpow_counters


def counters(d, lib, tag):
    hits = glob.glob(str(d / f"{lib}_{tag}" / "**" / "*counter_collection.csv"), recursive=True)
    if not hits:
        return None, None
    bl = bench_line(d / f"bench_{lib}_{tag}.log")
    n = int(bl["roofline"]["launches"])
    return kpow_counters(hits[0])[-n:], bl


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--variants", nargs="+", default=["base", "x2"])
    a = ap.parse_args()
    d = Path(a.dir)
    out = {}
    for lib in a.variants:
        runs = []
        for log in sorted(glob.glob(str(d / f"bench_{lib}_[0-9].log"))):
            bl = bench_line(log)
            r = bl["roofline"]
            runs.append({"ballots_per_s": bl["value"], "kernel_ms_per_launch": r["kernel_ms_per_launch"],
                         "clock_ghz": r.get("clock_ghz"), "tmac_s": r["achieved"], "frac": r["frac"],
                         "tmac_s_per_ghz": r["achieved"] / r["clock_ghz"] if r.get("clock_ghz") else None})
        v = {"runs": runs, "hbm_bytes_per_launch": 0.0}
        for ctr, scale in (("FETCH_SIZE", 2048), ("WRITE_SIZE", 1024)):
            per, bl = counters(d, lib, ctr)
            if per:
                b = sum(c[ctr] for c in per) * scale / len(per)
                v[f"{ctr.lower()}_bytes_per_launch"] = b
                v["hbm_bytes_per_launch"] += b
        per, bl = counters(d, lib, "SQ")
        if per:
            ops = bl["roofline"]["mont_ops_per_launch"] * len(per)
            insts = sum(c["SQ_INSTS_VALU"] for c in per)
            grbm = sum(c["GRBM_GUI_ACTIVE"] for c in per) / 8  # per XCD
            v["valu_instr_per_mont_op_per_lane"] = insts * 8 / ops
            v["valu_issue_util"] = insts / (grbm * 256)
        out[lib] = v
    mean = lambda rs, k: sum(r[k] for r in rs) / len(rs)
    b = out[a.variants[0]]
    for lib in a.variants[1:]:
        x = out[lib]
        if not (b["runs"] and x["runs"]):
            continue
        rel = {
            "ballots_per_s_ratio": mean(x["runs"], "ballots_per_s") / mean(b["runs"], "ballots_per_s"),
            "kernel_ms_ratio": mean(x["runs"], "kernel_ms_per_launch") / mean(b["runs"], "kernel_ms_per_launch"),
        }
        if all(r["tmac_s_per_ghz"] for r in b["runs"] + x["runs"]):
            rel["tmac_s_per_ghz_ratio"] = mean(x["runs"], "tmac_s_per_ghz") / mean(b["runs"], "tmac_s_per_ghz")
            rel["clock_ratio"] = mean(x["runs"], "clock_ghz") / mean(b["runs"], "clock_ghz")
        if b["hbm_bytes_per_launch"] and x["hbm_bytes_per_launch"]:
            rel["hbm_bytes_ratio"] = x["hbm_bytes_per_launch"] / b["hbm_bytes_per_launch"]
        if "valu_instr_per_mont_op_per_lane" in b and "valu_instr_per_mont_op_per_lane" in x:
            rel["valu_per_mm_ratio"] = x["valu_instr_per_mont_op_per_lane"] / b["valu_instr_per_mont_op_per_lane"]
        out[f"{lib}_vs_{a.variants[0]}"] = rel
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
