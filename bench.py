"""Benchmark: ballots verified+tallied per second on the EG 1.0 4096-bit group.

Workload: synthetic ballots of 4 contests x 5 selections (+1 placeholder each, 24 encrypted
selections per ballot), batch-encrypted on the GPU in setup (untimed, reported separately),
then ONE step = verify every ballot's disjunctive and contest proofs + homomorphic tally of all
ballots, with the encrypted ballots already resident in HBM.
  * N = 1: BASELINE.json configs[1], 10k ballots on one GPU.
  * N > 1 (torch.distributed.run or self-launched, one rank per GPU): configs[2]'s per-GPU shard,
    125,000 contiguous ballots per rank (weak scaling; N = 8 is configs[2] itself, 1M ballots over
    the node); the per-rank partial tallies are all-gathered over RCCL and folded mod p on rank 0.
  * --manifest large: the configs[4] manifest (20 contests x 5 selections, 120 encrypted
    selections per ballot), same ballot counts unless --ballots is given.
  * --pipeline full: configs[4]'s full pipeline per step (device encryption, verify + tally, the
    all-gather fold and, on rank 0, the threshold decryption through 5 DecryptingTrustees with
    exact counts); see full_pipeline().

Every device buffer, kernel and collective runs through libeg_hip.so (its own HIP runtime and
its own RCCL communicator, include/eg_hip.h): torch is imported only for its CPU process group
(gloo), which carries the RCCL id, barriers and the max-over-ranks time, and never initialises
the GPU.  The step is bracketed by a barrier + a device synchronisation of the library's stream
(group.sync(), the eg_ctx_sync of every kernel the step queued) on both sides.

Prints ONE JSON line (rank 0).  See DESIGN.md §6 for the roofline definition.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))

PEAK_TMAC = 256 * 64 * 2.4e9 / 1e12   # 256 CUs x 64 v_mad_u64_u32 lanes/clk/CU x 2.4 GHz (profiles/r01_ubench_isa.txt)
# measured v_mad_u64_u32 issue ceiling at 3 waves/SIMD (k_pow's occupancy): 58.4 lane-MAC/clk/CU,
# 4.4 cycles per wave-instruction (profiles/r01_ubench_banks.txt)
ISSUE_TMAC = 256 * 58.4 * 2.4e9 / 1e12
SHARD = 125_000  # ballots per GPU at N > 1: configs[2]'s 1M ballots over 8 GPUs


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--ballots", type=int, default=0,
                    help="ballots per GPU (0 = the config's: 10k at N = 1 (configs[1]), 125k per GPU at N > 1 "
                         "(configs[2]'s shard) and for --pipeline full (configs[4]'s shard))")
    ap.add_argument("--manifest", choices=("small", "large"), default=None,
                    help="small = 4 contests x 5 selections (configs[1-2]); large = 20 x 5 (configs[4]; the "
                         "default of --pipeline full)")
    ap.add_argument("--contests", type=int, default=0, help="override the manifest's contests")
    ap.add_argument("--selections", type=int, default=5)
    ap.add_argument("--pipeline", choices=("verify", "full"), default="verify",
                    help="verify = verify + tally (the metric); full = encrypt + verify + tally + fold + "
                         "threshold decryption per step (configs[4])")
    ap.add_argument("--guardians", type=int, default=5, help="--pipeline full: guardians (configs[3-4]: 5)")
    ap.add_argument("--quorum", type=int, default=3)
    ap.add_argument("--available", type=int, default=3, help="--pipeline full: guardians present at decryption")
    ap.add_argument("--dist-timeout", type=float, default=600.0,
                    help="seconds a host (gloo) collective may wait before failing")
    ap.add_argument("--strict-rccl", type=int, choices=(0, 1), default=None,
                    help="1 = a rank that cannot open its RCCL communicator fails the run (non-zero exit) "
                         "instead of falling back to a host exchange; default 1 at --gpus N > 1 in RCCL mode")
    ap.add_argument("--fb-window", type=int, default=22, help="fixed-base radix window bits for g and K")
    ap.add_argument("--cpu-sample", type=int, default=1, help="run the CPU baseline (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=8.0, help="target wall time of the CPU baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0 = the affinity count)")
    ap.add_argument("--cpu-max-ballots", type=int, default=2000,
                    help="ballots rank 0 keeps on the host for the CPU baseline at N > 1")
    ap.add_argument("--modexp-n", type=int, default=1 << 20,
                    help="modexp microbenchmark batch (SURVEY 8(d): 2^20; rank 0 only; 0 = skip)")
    ap.add_argument("--ct-encrypt", type=int, default=1,
                    help="also time the constant-time encryption mode (eg_ctx_set_ct_encrypt; 0 = skip)")
    a = ap.parse_args(argv)
    if a.manifest is None:
        a.manifest = "large" if a.pipeline == "full" else "small"
    if not a.contests:
        a.contests = 20 if a.manifest == "large" else 4
    if not a.ballots:
        a.ballots = default_ballots(a.gpus, a.pipeline)
    if a.strict_rccl is None:
        a.strict_rccl = 1 if a.gpus > 1 and exchange_mode() == "rccl" else 0
    return a


COMM_TIMEOUT_S = 120.0  # EG_COMM_TIMEOUT_S the ranks get unless the caller set one


def comm_timeout_s() -> float:
    """The deadline libeg gives every RCCL init and collective (eg_capi_comm.inc comm_wait_locked)."""
    try:
        v = float(os.environ.get("EG_COMM_TIMEOUT_S", COMM_TIMEOUT_S))
    except ValueError:
        v = COMM_TIMEOUT_S
    return v if v > 0 else COMM_TIMEOUT_S


def launch_budget_s(a) -> float:
    """How long the self-launcher lets N ranks run before it kills them (returns 124): the work the
    run is sized for, with room, plus one communicator deadline -- a rank stuck in a collective
    fails on its own after comm_timeout_s() (and the launcher then ends the others at once), so
    this is only the backstop for a rank stuck anywhere else.  Per-step allowance: 30 us per
    4 x (5+1) ballot on one MI355X (3.8 s per 125k-ballot step) scaled by selections, times 4;
    the full pipeline adds its encryption and decryption; setup covers the first `import torch`
    on a fresh box, the 22-bit tables, the ballots' encryption and the CPU baseline."""
    nsel = a.contests * (a.selections + 1)
    per_step = 4 * 30e-6 * a.ballots * nsel / 24 * (1.5 if a.pipeline == "full" else 1.0)
    setup = 300.0 + 4 * a.cpu_seconds + (60.0 if a.modexp_n else 0.0) + 4 * 30e-6 * a.ballots * nsel / 24
    return setup + (a.steps + a.warmup) * per_step + comm_timeout_s()


def default_ballots(gpus: int, pipeline: str = "verify") -> int:
    """Ballots per GPU of the BASELINE config bench.py measures at N GPUs: configs[1] (10k on one
    GPU) at N = 1; configs[2]'s per-GPU shard (125k = 1M / 8) at N > 1, so every N runs the same
    per-GPU work (weak scaling) and N = 8 is configs[2] exactly; --pipeline full: configs[4]'s
    per-GPU shard (125k ballots of 20 x (5+1)) at every N."""
    if pipeline == "full":
        return SHARD
    return 10_000 if gpus <= 1 else SHARD


def config_name(contests: int, selections: int, nb: int, world: int) -> str:
    """BASELINE.json config this run measures: configs[1] = 10k ballots of 4 x 5 on ONE GPU;
    configs[2] = 1M ballots of 4 x 5 over the node (125k per GPU at N = 8); configs[4] = 1M
    ballots of the 100-selection manifest (20 x 5) at 1/2/4/8 GPUs."""
    total = nb * world
    gpus = f"{world} GPU{'s' if world > 1 else ''}"
    if (contests, selections) == (4, 5):
        if total == 1_000_000:
            return f"configs[2] (1M ballots over {gpus})"
        if world == 1 and nb == 10_000:
            return "configs[1]"
        if nb == SHARD:
            return f"configs[2] per-GPU shard ({SHARD} ballots per GPU x {gpus})"
        return f"configs[1] shape (4x5), {nb} ballots per GPU x {gpus}"
    if (contests, selections) == (20, 5):
        if total == 1_000_000:
            return f"configs[4] (1M ballots of 20x5 over {gpus})"
        if nb == SHARD:
            return f"configs[4] per-GPU shard ({SHARD} ballots of 20x5 per GPU x {gpus})"
        return f"configs[4] shape (20x5), {nb} ballots per GPU x {gpus}"
    return f"custom manifest {contests}x{selections}, {nb} ballots per GPU x {gpus}"


def exchange_mode() -> str:
    """EG_DIST_BACKEND=gloo rehearses N > 1 with host collectives (every rank may share one GPU);
    the default is libeg_hip's RCCL communicator ("nccl" is accepted for it)."""
    m = os.environ.get("EG_DIST_BACKEND", "rccl").lower()
    return "gloo" if m == "gloo" else "rccl"


def note(rank, msg):
    """Progress on stderr (rank 0; outside the timed region): stdout keeps the one JSON line."""
    if rank == 0:
        print(f"bench: {msg}", file=sys.stderr, flush=True)


def init_ranks(a):
    """-> (world, rank, device, dist): the host process group (gloo, CPU only) at N > 1."""
    from electionguard.launch import launched_world
    lw = launched_world()
    if lw is not None and lw != a.gpus:
        sys.exit(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={lw} ranks")
    world = lw or 1
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if exchange_mode() == "gloo" or os.environ.get("EG_RANKS_SHARE_GPU") == "1":
        # the gloo rehearsal puts every rank on one GPU; EG_RANKS_SHARE_GPU=1 does the same in RCCL
        # mode, where RCCL refuses two ranks on one device: the failure path of --strict-rccl on a
        # one-GPU box (every rank must exit non-zero within seconds, none may hang)
        local = 0
    dist = None
    if world > 1:
        import datetime

        import torch.distributed as dist
        # a dead peer fails the collective instead of hanging it
        dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=a.dist_timeout))
    return world, rank, local, dist


def main(argv=None):
    a = parse(argv)
    from electionguard.launch import launched_world, run_ranks
    if launched_world() is None and a.gpus > 1:
        # no launcher: start one rank process per GPU (RANK/LOCAL_RANK/WORLD_SIZE/MASTER_*) before
        # anything touches HIP; rank 0 prints the JSON line; the first rank to fail ends the run
        # (the others are killed) and its status is this process's
        env = dict(os.environ)
        env.setdefault("EG_COMM_TIMEOUT_S", str(COMM_TIMEOUT_S))
        sys.exit(run_ranks(str(Path(__file__).resolve()), sys.argv[1:], a.gpus, timeout=launch_budget_s(a), env=env))
    if a.gpus > 1:
        os.environ.setdefault("EG_COMM_TIMEOUT_S", str(COMM_TIMEOUT_S))  # ranks started by torch.distributed.run
    world, rank, local, dist = init_ranks(a)
    if a.pipeline == "full":
        out = full_pipeline(a, world, rank, local, dist)
    else:
        out = verify_tally(a, world, rank, local, dist)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def setup_election(a, group, rank):
    """Synthetic election shared by every rank (3 guardians, quorum 3: configs[0]'s shape; or the
    --pipeline full trustees) and this rank's ballots (votes, nonces)."""
    from electionguard.ballot import ElectionKey, Manifest, random_scalars, random_votes
    from electionguard.keyceremony import key_ceremony
    man = Manifest(a.contests, a.selections, 1)
    n_g, quorum = (a.guardians, a.quorum) if a.pipeline == "full" else (3, 3)
    gk, K = key_ceremony(group, n_g, quorum, seed=20241015)
    key = ElectionKey(group, K, window_bits=a.fb_window)
    qbar = int.from_bytes(b"electionguard-remote mi355x qbar".ljust(32, b"\0"), "big") % group.q
    rng = np.random.default_rng(1000 + rank)
    nb = a.ballots
    votes = random_votes(rng, man, nb)
    sn = random_scalars(rng, (nb, man.nsel, 4), group.q)
    cn = random_scalars(rng, (nb, man.n_contests), group.q)
    return man, gk, K, key, qbar, votes, sn, cn


def verify_tally(a, world, rank, local, dist):
    """configs[1] / configs[2] (--manifest large: configs[4]): one step = verify + tally of the
    rank's resident ballots, the verdict all-reduce and the tally all-gather + fold."""
    from electionguard.ballot import Verifier, batch_encryption
    from electionguard.core import productionGroup
    from electionguard.distributed import TallyExchange, max_over_ranks

    group = productionGroup(local)
    man, _, K, key, qbar, votes, sn, cn = setup_election(a, group, rank)
    nb = a.ballots
    eb = batch_encryption(group, key, qbar, man, votes, sn, cn)  # the ballots the step verifies
    # The encryption rates are N = 1 figures (at N > 1 a rank keeps only its device copy).
    enc_s = None
    if world == 1:
        for _ in range(2):  # host-pointer encryption rate: best of two warm calls (same nonces, same bytes)
            t = time.perf_counter()
            batch_encryption(group, key, qbar, man, votes, sn, cn)
            dt = time.perf_counter() - t
            enc_s = dt if enc_s is None else min(enc_s, dt)
    d_cts, d_rp, d_cp = (group.to_device(x) for x in (eb.cts, eb.rproof, eb.cproof))
    d_oks = group.device_buffer(nb * man.nsel)
    d_okc = group.device_buffer(nb * man.n_contests)
    d_tal = group.device_buffer(man.n_real * 2 * 512)
    enc_dev = enc_dev_ct = None
    if world == 1:
        enc_dev = encrypt_device_rate(group, key, qbar, man, votes, sn, cn, d_cts, d_rp, d_cp)
        if a.ct_encrypt:  # constant-time mode (masked table scans, no secret-indexed address): same bytes
            group.ct_encrypt = True
            try:
                enc_dev_ct = encrypt_device_rate(group, key, qbar, man, votes, sn, cn, d_cts, d_rp, d_cp, reps=2)
            finally:
                group.ct_encrypt = False
    # rank 0 keeps a bounded host sample of its ballots for the CPU baseline (at N = 1 the whole
    # batch stays: the sample is sized from a calibration run); the other ranks keep none
    sample = eb if world == 1 else (eb.slice(0, min(nb, a.cpu_max_ballots)) if rank == 0 else None)
    if sample is not None and world > 1:
        sample = type(eb)(sample.cts.copy(), sample.rproof.copy(), sample.cproof.copy())
    del eb, sn, cn
    # modexp/sec/GPU microbenchmark on rank 0, before the verify step so the verify
    # launches stay the last k_pow dispatches of the process (tools/prof_summary.py)
    modexp = modexp_ubench(group, a.modexp_n, rank) if a.modexp_n > 0 and rank == 0 else None
    xch = TallyExchange(group, dist, world, rank, exchange_mode(), fallback=not a.strict_rccl)
    ver = Verifier(group, key, qbar, man)
    final_tally = None

    def step():
        nonlocal final_tally
        ver.verify_device(d_cts.ptr, d_rp.ptr, d_cp.ptr, nb, d_oks.ptr, d_okc.ptr, d_tal.ptr)
        ok = xch.all_valid(group.all_nonzero(d_oks) and group.all_nonzero(d_okc))
        final_tally = xch.fold(d_tal, man.n_real)
        if not ok:
            raise RuntimeError("verification failed on honest synthetic ballots")

    note(rank, f"setup done ({nb} ballots per rank resident); {a.warmup} warmup steps")
    for _ in range(a.warmup):
        step()
    if dist:
        dist.barrier()
    note(rank, f"warmup done; {a.steps} timed steps")
    group.sync()
    group.profile_begin()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    group.sync()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    note(rank, f"timed steps done in {el:.2f} s")
    kp = group.profile_end()
    el = max_over_ranks(dist, el)
    rccl_ranks = xch.rccl_ranks  # what RCCL itself reports (ncclCommCount), before the communicator closes
    xch.close()

    value = nb * world * a.steps / el
    out = line_common(a, world, el, value, kp, nb, man, "ballots verified+tallied/sec (node, 4096-bit group)",
                      xch.collective)
    out["config"]["rccl_ranks"] = rccl_ranks
    if xch.note:
        out["config"]["exchange_note"] = xch.note
    attach_traffic(out)
    out["modexp_per_s_per_gpu"] = {"var_base": modexp.get("var_base_per_s"),
                                   "fixed_base_g": modexp.get("fixed_base_g_per_s")} if modexp else None
    # a derived count, not a measurement: the verify step's work expressed in 256-bit
    # exponentiations (4 variable-base + 5 fixed-base per selection, 2 + 3 per contest; comb-
    # shared pairs and fused fixed-base terms counted as whole exponentiations)
    out["modexp_equivalents_per_s_per_gpu"] = round((9 * man.nsel + 5 * man.n_contests) * value / world, 1)
    out["encrypt_ballots_per_s_per_gpu"] = round(nb / enc_s, 2) if enc_s else None
    out["encrypt_ballots_per_s_per_gpu_device_resident"] = enc_dev
    out["encrypt_ballots_per_s_per_gpu_device_resident_constant_time"] = enc_dev_ct
    out["modexp_ubench"] = modexp
    return report(a, out, world, rank, dist, man, sample, qbar, K)


def report(a, out, world, rank, dist, man, sample, qbar, K):
    """After the timed steps: every rank meets at a barrier, then rank 0 alone times the CPU port
    on its host sample (the other ranks are done, so it has the host's cores) and the line gets
    cpu_baseline and vs_baseline at every N."""
    if world > 1:
        dist.barrier()
    if rank == 0 and a.cpu_sample > 0 and sample is not None:
        out["cpu_baseline"] = cpu_baseline(a, man, sample, qbar, K)
        attach_ratio(out)
    return out


def line_common(a, world, el, value, kp, nb, man, metric, collective):
    """The bench line's fields every mode shares (value, roofline of k_pow, config)."""
    from electionguard.core import native
    radix = native.version().split("radix2^")[1].split()[0]
    build_id = hashlib.md5(Path(native.lib_path()).read_bytes()).hexdigest()[:12]
    cfg_name = config_name(a.contests, a.selections, nb, world)
    kms, kmm, klaunch = kp.ms, kp.mont_ops, kp.launches
    clock = kp.clock_ghz if kp.clock_ghz and 1.0 <= kp.clock_ghz <= 2.6 else None
    clock_note = (f"median of {kp.clock_records} workgroup records, {kp.clock_dropped} dropped" if clock else
                  f"null: median {kp.clock_ghz:.3f} GHz outside [1.0, 2.6] ({kp.clock_records} records used, "
                  f"{kp.clock_dropped} dropped as unset, wrapped or out of range)")
    # algorithmic work of the dominant kernel (k_pow), from its own launch schedule:
    # 2*128^2 u32 MACs per multiply, 128*129/2 + 128^2 per squaring (group.MAC_PER_*)
    achieved = kp.macs / (kms / 1e3) / 1e12 if kms > 0 else None
    mm_per_ballot = kmm / (nb * a.steps) if a.steps else None
    what = ("encrypt + verify + tally + fold + threshold decryption" if a.pipeline == "full"
            else "verify + homomorphic tally")
    out = {
        "metric": metric,
        "value": round(value, 2),
        "unit": "ballots/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(el / a.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": f"u32xu32->u64 (radix-2^{radix} limbs)",
        "data": "synthetic (seeded random one-hot ballots, GPU-encrypted with random nonces)",
        "config": {
            "workload": f"{cfg_name}: {what} of {nb} ballots per GPU ({nb * world} in total), {a.contests} contests "
                        f"x {a.selections} selections (+1 placeholder), EG 1.0 4096-bit production group",
            "ballots_per_gpu": nb,
            "selections_per_ballot": man.nsel,
            "fb_window_bits": a.fb_window,
            "parallelism": (f"ballot-sharded x{world}, {collective} all-gather of partial tallies" if world > 1 else
                            f"ballot-sharded x1, {collective}"),
        },
        "roofline": {
            "bound": "valu-int",
            "kernel": "k_pow (windowed Montgomery exponentiation + fused fixed-base terms)",
            "achieved": round(achieved, 3) if achieved else None,
            "peak": round(PEAK_TMAC, 2),
            "unit": "TMAC/s (u32xu32+u64 v_mad_u64_u32)",
            "frac": round(achieved / PEAK_TMAC, 4) if achieved else None,
            "measured_issue_peak": round(ISSUE_TMAC, 2),
            "frac_of_measured_issue_peak": round(achieved / ISSUE_TMAC, 4) if achieved else None,
            # the shader clock the timed k_pow launches ran at (boxes run 2.1-2.3 GHz under this
            # load) and `frac` re-based on the peak at that clock (peak is quoted at 2.4 GHz)
            "clock_ghz": round(clock, 3) if clock else None,
            "clock_source": f"in-kernel s_memtime / s_memrealtime x 100 MHz, {clock_note}",
            "frac_at_measured_clock": round(achieved / (PEAK_TMAC * clock / 2.4), 4) if achieved and clock else None,
            "traffic": None,
            "kernel_ms_per_launch": round(kms / max(klaunch, 1), 3),
            "launches": klaunch,
            "mont_ops_per_launch": round(kmm / max(klaunch, 1)),
            "squaring_frac": round(kp.squarings / kmm, 4) if kmm else None,
        },
        "mont_ops_per_ballot": round(mm_per_ballot, 1) if mm_per_ballot else None,
        "build": build_id,
    }
    if a.pipeline == "full":
        out["config"]["pipeline"] = "full"
    return out


def attach_traffic(out):
    """HBM traffic of k_pow from the committed PMC passes of this same command
    (tools/profile_round.sh); only quoted when the profiled workload (the finished config, exchange
    fields included) AND the library build (md5 of libeg_hip.so) match this run's."""
    for prof in sorted((ROOT / "profiles").glob("r*_pmc_kpow.json"), reverse=True):  # newest round first
        try:
            pm = json.loads(prof.read_text())
            if pm.get("bench_config") == out["config"] and pm.get("bench_build") == out.get("build"):
                out["roofline"]["traffic"] = round(pm["traffic"]["hbm_bytes_per_launch"])
                out["roofline"]["traffic_source"] = f"profiles/{prof.name}"
                break
        except (KeyError, ValueError, TypeError):
            pass
    return out


def attach_ratio(out):
    """vs_baseline = value / cpu_baseline.value: BASELINE.json publishes no number for this metric,
    and the north_star's target (>= 50x on 8 GPUs) is defined against the host-CPU path timed on the
    box's cores in the same run, which cpu_baseline is (same workload shape, cores stated)."""
    cb = out.get("cpu_baseline")
    if cb and cb.get("value"):
        out["vs_baseline"] = round(out["value"] / cb["value"], 2)
        out["vs_baseline_basis"] = (f"value / cpu_baseline.value: the CPU port of the same step on {cb['cores']} "
                                    f"host cores in this run (BASELINE.json publishes no number)")


def encrypt_device_rate(group, key, qbar, man, votes, sn, cn, d_cts, d_rp, d_cp, reps=5):
    """batch-encrypt with votes, nonces and outputs resident in HBM (eg_encrypt_ballots_dev),
    best of `reps` timed runs; the outputs must equal the host-pointer encryption's bytes
    (same injected nonces) already resident in d_cts / d_rp / d_cp."""
    from electionguard.ballot import batch_encryption_device

    nb = votes.shape[0]
    dv, dsn, dcn = (group.to_device(x) for x in (votes, sn, cn))
    oc, orp, ocp = (group.device_buffer(x.nbytes) for x in (d_cts, d_rp, d_cp))

    def run():
        batch_encryption_device(group, key, qbar, man, nb, dv.ptr, dsn.ptr, dcn.ptr, oc.ptr, orp.ptr, ocp.ptr)

    run()
    best = None
    for _ in range(reps):
        t = time.perf_counter()
        run()
        dt = time.perf_counter() - t
        best = dt if best is None else min(best, dt)
    same = all(np.array_equal(x.download().ravel(), y.download().ravel()) for x, y in ((oc, d_cts), (orp, d_rp), (ocp, d_cp)))
    for b in (dv, dsn, dcn, oc, orp, ocp):
        b.free()
    if not same:
        raise RuntimeError("device-resident encryption differs from the host-pointer encryption")
    return round(nb / best, 2)


def modexp_ubench(group, n, rank, reps=2):
    """SURVEY 8(d) modexp microbenchmark on one GPU: n variable-base powP (bases g^x, x and the
    exponents uniform in [1, q)) and n fixed-base gPowP, operands resident in HBM
    (eg_powp_batch_dev / eg_fb_pow_batch_dev); a few results are spot-checked with CPython pow."""
    rng = np.random.default_rng(7 + rank)
    q, p, g = group.q, group.p, group.g

    def scalars(m):  # uniform 256-bit: in [1, q) except with probability 2^-248 (used as given)
        return rng.integers(0, 256, size=(m, 32), dtype=np.uint8)

    xs_h, es_h = scalars(n), scalars(n)
    xs, es = group.to_device(xs_h), group.to_device(es_h)
    bases = group.device_buffer(n * 512)
    out = group.device_buffer(n * 512)
    group.gPowP_batch_dev(xs.ptr, bases.ptr, n)  # bases g^x (subgroup elements)
    group.powP_batch_dev(bases.ptr, es.ptr, out.ptr, n)  # warm-up (job table)
    group.sync()
    res = {"n": n, "exponent_bits": 256, "reps": reps}
    for name, run in (("var_base", lambda: group.powP_batch_dev(bases.ptr, es.ptr, out.ptr, n)),
                      ("fixed_base_g", lambda: group.gPowP_batch_dev(es.ptr, out.ptr, n))):
        run()
        group.sync()
        group.profile_begin()
        t = time.perf_counter()
        for _ in range(reps):
            run()
        group.sync()
        el = time.perf_counter() - t
        kp = group.profile_end()
        res[f"{name}_per_s"] = round(n * reps / el, 1)
        res[f"{name}_mont_ops_per_exp"] = round(kp.mont_ops / (n * reps), 1)
        res[f"{name}_kpow_tmac_s"] = round(kp.macs / (kp.ms / 1e3) / 1e12, 3) if kp.ms > 0 else None
        # spot check the last run's first and last results (CPython pow; not the oracle)
        ob = out.download().reshape(n, 512)
        for i in (0, n - 1):
            e = int.from_bytes(es_h[i].tobytes(), "big")
            b = pow(g, int.from_bytes(xs_h[i].tobytes(), "big"), p) if name == "var_base" else g
            if int.from_bytes(ob[i].tobytes(), "big") != pow(b, e, p):
                raise RuntimeError(f"modexp microbenchmark {name}: result {i} differs from pow()")
    res["spot_checked"] = True
    for b in (xs, es, bases, out):
        b.free()
    return res


def cpu_threads(a):
    """Threads of the CPU baseline: every core the lease lets this process use -- the affinity set,
    capped by the cgroup CPU quota (more threads than the quota only time-slice: 256 threads under
    a 16-CPU quota ran 38% slower)."""
    affinity = len(os.sched_getaffinity(0))
    quota_cpus = None
    try:  # a cgroup CPU quota caps the useful parallelism below the affinity count
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        if q and q[0] != "max":
            quota_cpus = int(q[0]) / int(q[1])
    except (OSError, ValueError, IndexError):
        pass
    threads = a.cpu_threads or max(1, min(affinity, int(quota_cpus + 0.5) if quota_cpus else affinity))
    return threads, affinity, quota_cpus


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return ""


def cpu_baseline(a, man, eb, qbar, K):
    """C restatement of the JVM path (OpenSSL BN Montgomery sliding window, 8-bit radix
    fixed base = LOW_MEMORY_USE) on a bounded sample of the same ballots, on every host core
    this process may run on, sized to about --cpu-seconds of work.  At N > 1 it runs on rank 0
    after the timed steps and the final barrier, on rank 0's host sample (--cpu-max-ballots)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from eg_oracle_c import COracle
    from electionguard.core import constants as C

    threads, affinity, quota_cpus = cpu_threads(a)
    co = COracle(C.P, C.Q, C.G)
    co.set_key(K)

    def run(n):
        sub = eb.slice(0, n)
        t = time.perf_counter()
        ok_s, ok_c, _ = co.verify_ballots(qbar, man.n_contests, man.spc, 1, 1, sub.cts, sub.rproof, sub.cproof,
                                          threads=threads)
        return time.perf_counter() - t, bool(ok_s.all() and ok_c.all())

    n0 = min(eb.n, 2 * threads)
    dt0, _ = run(n0)  # calibration (also warms the radix tables' caches)
    s = max(n0, min(eb.n, int(n0 / dt0 * a.cpu_seconds)))
    dt, valid = run(s)
    # per-core variable-base modexp rate (256-bit exponents, BN_mod_exp_mont, one thread)
    rng = np.random.default_rng(11)
    nb_pow = 256
    bases = np.stack([np.frombuffer(pow(C.G, int(x), C.P).to_bytes(512, "big"), np.uint8)
                      for x in rng.integers(1, 2**62, size=nb_pow)])
    exps = rng.integers(0, 256, size=(nb_pow, 32), dtype=np.uint8)
    t = time.perf_counter()
    co.powp(bases, exps)
    per_core_modexp = nb_pow / (time.perf_counter() - t)
    quota = f", cgroup CPU quota {quota_cpus:.1f}" if quota_cpus else ", no cgroup CPU quota"
    model = cpu_model()
    return {
        "value": round(s / dt, 3),
        "unit": "ballots/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{s} of the same ballots (verify incl. residue tests + tally, {man.nsel} selections each), "
                  f"{threads} threads = the lease's usable CPUs (affinity {affinity} of {os.cpu_count()}{quota}) on "
                  f"{model or 'host CPU'}; OpenSSL BN_mod_exp_mont + 8-bit radix fixed base; "
                  f"verdicts all valid: {valid}; wall {dt:.2f} s",
        "cpu_model": model,
        "affinity_cpus": affinity,
        "cgroup_quota_cpus": quota_cpus,
        "var_base_modexp_per_s_per_core": round(per_core_modexp, 1),
    }


def full_pipeline(a, world, rank, local, dist, keep=None):
    """configs[4]'s full pipeline (RunRemoteWorkflowTest.java:140-182), ONE step per rank =
      1 encrypt the rank's ballots on the device (batchEncryption :140-141; eg_encrypt_ballots_dev:
        votes and injected nonces resident in HBM, ciphertexts and proofs written in HBM);
      2 verify every proof + tally (Verifier :179-182, runAccumulateBallots :151;
        eg_verify_ballots_dev on the ciphertexts step 1 wrote);
      3 the verdict all-reduce and the partial-tally all-gather + mod-p fold;
      4 on rank 0: decryption of the folded tally through the DecryptingTrustees (the remote
        decryption :164-172: each available guardian's direct shares, every (missing, available)
        pair's compensated shares with recovery keys, every share proof checked, Lagrange combine,
        BSGS dLog) -> counts, which must equal the vote totals over every rank exactly.
    value = ballots through the whole pipeline per second over the node.  Per-phase times are
    summed over the timed steps (max over ranks for phases 1-3).  keep (tests): a dict that
    receives the step's artifacts."""
    from electionguard.ballot import Verifier, batch_encryption_device
    from electionguard.core import productionGroup
    from electionguard.decrypt import DecryptingTrustee, Decryption
    from electionguard.distributed import TallyExchange, max_over_ranks

    if not 1 <= a.quorum <= a.available <= a.guardians:
        raise SystemExit("--pipeline full needs quorum <= available <= guardians")
    group = productionGroup(local)
    man, gk, K, key, qbar, votes, sn, cn = setup_election(a, group, rank)
    nb = a.ballots
    want = votes.reshape(nb, man.n_contests, man.spc)[:, :, :man.n_selections].sum(axis=0).reshape(-1).astype(np.int64)
    if dist is not None:  # the expected counts: the vote totals over every rank's shard
        import torch
        tw = torch.from_numpy(want.copy())
        dist.all_reduce(tw)
        want = tw.numpy()
    dv, dsn, dcn = (group.to_device(x) for x in (votes, sn, cn))
    d_cts = group.device_empty((nb, man.nsel, 2, 512))
    d_rp = group.device_empty((nb, man.nsel, 4, 32))
    d_cp = group.device_empty((nb, man.n_contests, 2, 32))
    d_oks = group.device_buffer(nb * man.nsel)
    d_okc = group.device_buffer(nb * man.n_contests)
    d_tal = group.device_buffer(man.n_real * 2 * 512)
    ver = Verifier(group, key, qbar, man)
    dec = None
    if rank == 0:
        comm = {g.gid: g.commitments for g in gk}
        dec = Decryption(group, qbar, [DecryptingTrustee(group, g, comm) for g in gk[:a.available]],
                         [g.gid for g in gk[a.available:]], {g.gid: g.public_key for g in gk})
    xch = TallyExchange(group, dist, world, rank, exchange_mode(), fallback=not a.strict_rccl)
    ph = {"encrypt": 0.0, "verify_tally": 0.0, "exchange": 0.0, "decrypt": 0.0}
    counts = None
    last = {}

    def step(acc):
        nonlocal counts
        t0 = time.perf_counter()
        batch_encryption_device(group, key, qbar, man, nb, dv.ptr, dsn.ptr, dcn.ptr, d_cts.ptr, d_rp.ptr, d_cp.ptr)
        t1 = time.perf_counter()  # (returns when the outputs are written)
        ver.verify_device(d_cts.ptr, d_rp.ptr, d_cp.ptr, nb, d_oks.ptr, d_okc.ptr, d_tal.ptr)
        ok = group.all_nonzero(d_oks) and group.all_nonzero(d_okc)  # (synchronises the stream)
        t2 = time.perf_counter()
        ok = xch.all_valid(ok)
        T = xch.fold(d_tal, man.n_real)
        t3 = time.perf_counter()
        if not ok:
            raise RuntimeError("verification failed on honest synthetic ballots")
        if rank == 0:
            last["tally"] = T
            counts = dec.decrypt(T, nb * world)
            if [int(x) if x is not None else None for x in counts] != [int(x) for x in want]:
                raise RuntimeError("decrypted counts differ from the vote totals")
            if keep is not None:
                keep["tally"], keep["counts"] = T, counts
        t4 = time.perf_counter()
        if acc:
            ph["encrypt"] += t1 - t0
            ph["verify_tally"] += t2 - t1
            ph["exchange"] += t3 - t2
            ph["decrypt"] += t4 - t3

    note(rank, f"setup done ({nb} ballots per rank); {a.warmup} warmup steps")
    for _ in range(a.warmup):
        step(False)
    if dist:
        dist.barrier()
    note(rank, f"warmup done; {a.steps} timed steps")
    group.sync()
    group.profile_begin()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step(True)
    group.sync()
    if dist:
        dist.barrier()
    el = time.perf_counter() - t0
    note(rank, f"timed steps done in {el:.2f} s")
    kp = group.profile_end()
    el = max_over_ranks(dist, el)
    phases = {k: max_over_ranks(dist, v) for k, v in ph.items()}
    rccl_ranks = xch.rccl_ranks
    xch.close()
    value = nb * world * a.steps / el
    out = line_common(a, world, el, value, kp, nb, man,
                      "ballots encrypted+verified+tallied+decrypted/sec (node, 4096-bit group, full pipeline)",
                      xch.collective)
    out["config"]["rccl_ranks"] = rccl_ranks
    if xch.note:
        out["config"]["exchange_note"] = xch.note
    attach_traffic(out)
    tot = nb * world * a.steps
    out["phases"] = {
        "encrypt": {"s": round(phases["encrypt"], 3), "ballots_per_s": round(tot / phases["encrypt"], 1)},
        "verify_tally": {"s": round(phases["verify_tally"], 3),
                         "ballots_per_s": round(tot / phases["verify_tally"], 1)},
        "exchange": {"s": round(phases["exchange"], 4)},
        "decrypt": {"s": round(phases["decrypt"], 3), "texts": man.n_real,
                    "trustees": f"{a.available} of {a.guardians} available, quorum {a.quorum}, "
                                f"{a.guardians - a.available} missing (direct + compensated shares with proofs)",
                    "note": "rank 0 only; the other ranks wait at the next exchange"},
        "counts_exact": True,
    }
    sample = None
    if rank == 0 and a.cpu_sample > 0:
        ns = min(nb, a.cpu_max_ballots)
        sample = (votes[:ns], sn[:ns], cn[:ns], d_cts[0:ns].download(), d_rp[0:ns].download(), d_cp[0:ns].download())
    if keep is not None:
        keep["group"], keep["K"], keep["qbar"], keep["man"], keep["gk"] = group, K, qbar, man, gk
        keep["want"], keep["cts"], keep["rproof"], keep["cproof"] = want, d_cts.download(), d_rp.download(), d_cp.download()
    if world > 1:
        dist.barrier()
    if sample is not None:
        out["cpu_baseline"] = cpu_baseline_pipeline(a, man, sample, qbar, K, gk, nb * world, phases, last["tally"])
        attach_ratio(out)
    return out


def cpu_baseline_pipeline(a, man, sample, qbar, K, gk, nb_total, gpu_phases, tally):
    """The CPU port (oracle/eg_oracle_c.c: OpenSSL BN, 8-bit radix fixed base) on the pipeline's
    phases, on the lease's cores: batchEncryption and verify + tally on a calibrated sample of the
    same ballots (the encryption must reproduce the GPU's bytes), and the trustees' direct +
    compensated shares of one tally (the mediator's share-proof checks and the dLog are not timed on
    the CPU: a lower bound for its decrypt phase).  value = the node's ballots per CPU step time
    projected from the per-phase rates: nb_total / (nb_total / encrypt + nb_total / verify + decrypt)."""
    sys.path.insert(0, str(ROOT / "oracle"))
    from eg_oracle_c import COracle
    from electionguard.core import constants as C
    from electionguard.keyceremony import poly_eval

    votes, sn, cn, cts, rp, cp = sample
    threads, affinity, quota_cpus = cpu_threads(a)
    co = COracle(C.P, C.Q, C.G)
    co.set_key(K)
    per = a.cpu_seconds / 3

    def enc(n):
        t = time.perf_counter()
        c2, r2, p2 = co.encrypt_ballots(qbar, man.n_contests, man.spc, votes[:n], sn[:n], cn[:n], threads=threads)
        dt = time.perf_counter() - t
        if not (np.array_equal(c2, cts[:n]) and np.array_equal(r2, rp[:n]) and np.array_equal(p2, cp[:n])):
            raise RuntimeError("the CPU port's encryption differs from the GPU's bytes")
        return dt

    def ver(n):
        t = time.perf_counter()
        ok_s, ok_c, _ = co.verify_ballots(qbar, man.n_contests, man.spc, 1, 1, cts[:n], rp[:n], cp[:n], threads=threads)
        dt = time.perf_counter() - t
        if not (ok_s.all() and ok_c.all()):
            raise RuntimeError("the CPU port rejects the GPU's ballots")
        return dt

    n_all = len(votes)
    rates = {}
    for name, fn in (("encrypt", enc), ("verify_tally", ver)):
        n0 = min(n_all, 2 * threads)
        dt0 = fn(n0)
        s = max(n0, min(n_all, int(n0 / dt0 * per)))
        rates[name] = (s, s / fn(s))
    # the decrypt phase: every share of one tally (n_real texts) on the CPU
    rng = np.random.default_rng(5)
    texts = np.ascontiguousarray(tally, np.uint8).reshape(man.n_real, 2, 512)
    nonces = rng.integers(0, 256, size=(man.n_real, 32), dtype=np.uint8)
    avail, missing = gk[:a.available], gk[a.available:]
    t = time.perf_counter()
    for g in avail:
        co.trustee_decrypt(g.secret, qbar, texts, nonces, threads=threads)
    for l in missing:
        for g in avail:
            co.trustee_decrypt(poly_eval(l.coeffs, g.x, C.Q), qbar, texts, nonces, threads=threads)
    t_dec = time.perf_counter() - t
    enc_rate, ver_rate = rates["encrypt"][1], rates["verify_tally"][1]
    value = nb_total / (nb_total / enc_rate + nb_total / ver_rate + t_dec)
    quota = f", cgroup CPU quota {quota_cpus:.1f}" if quota_cpus else ", no cgroup CPU quota"
    model = cpu_model()
    nshares = man.n_real * len(avail) * (1 + len(missing))
    return {
        "value": round(value, 3),
        "unit": "ballots/s",
        "cores": threads,
        "kind": "port",
        "sample": f"encrypt {rates['encrypt'][0]} and verify + tally {rates['verify_tally'][0]} of the same ballots "
                  f"(the CPU encryption reproduced the GPU's bytes; every verdict valid), and the {nshares} trustee "
                  f"shares of one {man.n_real}-text tally (share checks and dLog not timed on the CPU); projected to "
                  f"{nb_total} ballots per step; {threads} threads = the lease's usable CPUs (affinity {affinity} of "
                  f"{os.cpu_count()}{quota}) on {model or 'host CPU'}; OpenSSL BN_mod_exp_mont + 8-bit radix fixed base",
        "phases": {"encrypt_ballots_per_s": round(enc_rate, 3), "verify_tally_ballots_per_s": round(ver_rate, 3),
                   "decrypt_shares_s": round(t_dec, 3)},
        "gpu_over_cpu_by_phase": {
            "encrypt": round(nb_total * a.steps / gpu_phases["encrypt"] / enc_rate, 1) if gpu_phases["encrypt"] else None,
            "verify_tally": round(nb_total * a.steps / gpu_phases["verify_tally"] / ver_rate, 1)
            if gpu_phases["verify_tally"] else None,
        },
        "cpu_model": model,
        "affinity_cpus": affinity,
        "cgroup_quota_cpus": quota_cpus,
    }


if __name__ == "__main__":
    main()
