"""Where a per-element round trip goes: reads a `rocprofv3 --kernel-trace --hip-runtime-trace
--output-format csv` run of tests/cpp/percall_workflow (one thread) and prints, per kernel name, the
launches and their mean duration, the idle time between consecutive kernels (what the host adds per
batch), the HIP runtime calls by total time, and one batch's timeline on the dispatcher thread
(hipMemcpyAsync of the inputs -> hipLaunchKernel -> hipStreamSynchronize, matched to the copy and
job kernels by correlation id), split into short (< 200 us: fixed-base) and long batches.

    python tools/roundtrip_trace.py gpurun_out/r05zo_prof
"""
import collections
import csv
import sys
from pathlib import Path


def rows(d, suffix):
    fs = sorted(Path(d).rglob(f"*{suffix}"))
    if not fs:
        sys.exit(f"no *{suffix} under {d}")
    with open(fs[0]) as f:
        return list(csv.DictReader(f))


def main(d):
    ks = rows(d, "kernel_trace.csv")
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    by = collections.defaultdict(list)
    for r in ks:
        by[r["Kernel_Name"][:90]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("kernels (name, launches, mean us, total ms):")
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1]))[:12]:
        print(f"  {len(v):7d} {sum(v) / len(v):10.1f} {sum(v) / 1e3:10.1f}  {k}")
    # gaps between consecutive per-wave job kernels (the per-element batches)
    wj = [r for r in ks if "k_wave_job" in r["Kernel_Name"]]
    gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(wj, wj[1:])]
    gaps = [g for g in gaps if g < 5000]  # phase boundaries (host-only work) excluded
    if gaps:
        gaps.sort()
        print(f"k_wave_job gaps (us): n {len(gaps)} median {gaps[len(gaps) // 2]:.1f} "
              f"p10 {gaps[len(gaps) // 10]:.1f} p90 {gaps[9 * len(gaps) // 10]:.1f}")
    durs = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in wj)
    if durs:
        print(f"k_wave_job durations (us): median {durs[len(durs) // 2]:.1f} p10 {durs[len(durs) // 10]:.1f} "
              f"p90 {durs[9 * len(durs) // 10]:.1f}")
    try:
        hs = rows(d, "hip_api_trace.csv")
    except SystemExit:
        return
    hb = collections.defaultdict(list)
    for r in hs:
        hb[r["Function"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("HIP runtime calls (name, calls, mean us, total ms):")
    for k, v in sorted(hb.items(), key=lambda kv: -sum(kv[1]))[:14]:
        print(f"  {len(v):8d} {sum(v) / len(v):9.1f} {sum(v) / 1e3:10.1f}  {k}")
    timeline(hs, ks)


def timeline(hs, ks):
    kc = {r["Correlation_Id"]: r for r in ks}
    launches = collections.Counter(r["Thread_Id"] for r in hs if r["Function"] == "hipLaunchKernel")
    disp = launches.most_common(1)[0][0]  # the coalescer's dispatcher issues nearly every launch
    keep = {"hipMemcpyAsync", "hipLaunchKernel", "hipStreamSynchronize"}
    a = sorted((r for r in hs if r["Thread_Id"] == disp and r["Function"] in keep), key=lambda r: int(r["Start_Timestamp"]))
    t = lambda r, f: int(r[f + "_Timestamp"])  # noqa: E731
    seqs = []
    i = 0
    while i + 2 < len(a):
        m, l, s = a[i], a[i + 1], a[i + 2]
        if (m["Function"], l["Function"], s["Function"]) == ("hipMemcpyAsync", "hipLaunchKernel", "hipStreamSynchronize"):
            k = kc.get(l["Correlation_Id"])
            if k and "k_wave_job" in k["Kernel_Name"]:
                seqs.append((m, l, s, k, kc.get(m["Correlation_Id"])))
                i += 3
                continue
        i += 1
    parts = collections.defaultdict(list)
    for j, (m, l, s, k, cp) in enumerate(seqs):
        dur = (t(k, "End") - t(k, "Start")) / 1e3
        kind = "short" if dur < 200 else "long"
        parts[(kind, "1 host: previous sync returned -> inputs copy called")] += (
            [(t(seqs[j + 1][0], "Start") - t(s, "End")) / 1e3] if j + 1 < len(seqs) and
            t(seqs[j + 1][0], "Start") - t(s, "End") < 5e6 else [])
        parts[(kind, "2 hipMemcpyAsync call")].append((t(m, "End") - t(m, "Start")) / 1e3)
        parts[(kind, "3 -> hipLaunchKernel call")].append((t(l, "Start") - t(m, "End")) / 1e3)
        parts[(kind, "4 hipLaunchKernel call")].append((t(l, "End") - t(l, "Start")) / 1e3)
        parts[(kind, "5 launch returned -> kernel start")].append((t(k, "Start") - t(l, "End")) / 1e3)
        if cp:
            parts[(kind, "  (the copy kernel's run)")].append((t(cp, "End") - t(cp, "Start")) / 1e3)
        parts[(kind, "6 kernel")].append(dur)
        parts[(kind, "7 kernel end -> sync returns")].append((t(s, "End") - t(k, "End")) / 1e3)
    print(f"per-batch timeline on the dispatcher thread ({len(seqs)} batches; median / p10 / p90 us):")
    for (kind, name), v in sorted(parts.items()):
        v.sort()
        if v:
            print(f"  {kind:5s} {name:55s} {v[len(v) // 2]:9.1f} {v[len(v) // 10]:9.1f} {v[9 * len(v) // 10]:9.1f}")


if __name__ == "__main__":
    main(sys.argv[1])
