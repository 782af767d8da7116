"""CPU: the N>1 path with world_size 2, 4 and 8 over gloo — ballot shards, verdict all-reduce and
the all-gather + mod-p fold of partial tallies (the fold is the oracle's product here;
on the GPU it is GroupContext.prodP_groups)."""
import os
import random
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import eg_oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fold_oracle(elems, groups, length):
    G = O.production_group()
    out = np.zeros((groups, 512), np.uint8)
    for g in range(groups):
        xs = [int.from_bytes(elems[g * length + k].tobytes(), "big") for k in range(length)]
        out[g] = np.frombuffer(G.prodP(xs).to_bytes(512, "big"), np.uint8)
    return out


def _worker(rank, world, port, data, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from electionguard.distributed import all_valid, gather_fold_tally, shard_range
    cts, n_real = data
    a, b = shard_range(cts.shape[0], world, rank)
    G = O.production_group()
    # partial tally of this shard (oracle product stands in for the GPU reduction)
    part = np.zeros((n_real, 2, 512), np.uint8)
    for s in range(n_real):
        for c in range(2):
            part[s, c] = np.frombuffer(G.prodP([int.from_bytes(cts[i, s, c].tobytes(), "big")
                                               for i in range(a, b)]).to_bytes(512, "big"), np.uint8)
    ok = all_valid(dist, rank != 1 or True, torch.device("cpu"))
    bad = all_valid(dist, rank == 0, torch.device("cpu"))
    tally = gather_fold_tally(dist, torch.from_numpy(part), _fold_oracle)
    if rank == 0:
        q.put((ok, bad, tally.tobytes()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4, 8])
def test_n_rank_tally_fold_equals_global_tally(world):
    G = O.production_group()
    rng = random.Random(5)
    nb, n_real = 7, 3  # ragged shards: 4 + 3 (2 ranks), 2 + 2 + 2 + 1 (4 ranks), 1 x 7 + 0 (8 ranks)
    cts = np.zeros((nb, n_real, 2, 512), np.uint8)
    for i in range(nb):
        for s in range(n_real):
            for c in range(2):
                cts[i, s, c] = np.frombuffer(rng.randrange(1, G.p).to_bytes(512, "big"), np.uint8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, (cts, n_real), q)) for r in range(world)]
    for p in procs:
        p.start()
    ok, bad, tally = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok is True and bad is False
    t = np.frombuffer(tally, np.uint8).reshape(n_real, 2, 512)
    for s in range(n_real):
        for c in range(2):
            want = G.prodP([int.from_bytes(cts[i, s, c].tobytes(), "big") for i in range(nb)])
            assert int.from_bytes(t[s, c].tobytes(), "big") == want


def test_launcher_runs_n_ranks_and_folds_the_global_tally(tmp_path):
    """bench.py --gpus N without a launcher starts N rank processes through
    electionguard.launch.run_ranks; the ranks see WORLD_SIZE = N and the folded tally equals
    the tally over all ballots."""
    import json
    import sys
    from pathlib import Path
    from electionguard.launch import run_ranks
    child = Path(__file__).resolve().parent / "_launch_child.py"
    out = tmp_path / "rank0.json"
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    assert run_ranks(str(child), [str(out)], 2, timeout=240, env=env) == 0
    d = json.loads(out.read_text())
    assert d["n_gpus"] == 2 and d["ok"] is True
    sys.path.insert(0, str(child.parent))
    import _launch_child as L
    G = O.production_group()
    cts = L.ballots(5, 2)
    for s in range(2):
        for c in range(2):
            assert int(d["tally"][s][c], 16) == G.prodP([cts[i][s][c] for i in range(5)])


def test_bench_rejects_a_world_size_other_than_gpus():
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parent.parent
    env = dict(os.environ, WORLD_SIZE="3", RANK="0")
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2"], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_bench_config_names():
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from bench import config_name
    assert config_name(4, 5, 10_000, 1) == "configs[1]"
    assert config_name(4, 5, 125_000, 8).startswith("configs[2] (1M ballots over 8 GPUs")
    assert config_name(4, 5, 125_000, 2).startswith("configs[2] per-GPU shard")
    assert config_name(4, 5, 1_000_000, 1).startswith("configs[2]")
    assert config_name(4, 5, 10_000, 8) == "configs[1] shape (4x5), 10000 ballots per GPU x 8 GPUs"
    assert config_name(4, 5, 2_000, 2).startswith("configs[1] shape")
    assert config_name(20, 5, 10_000, 4).startswith("configs[4] shape")
    assert config_name(20, 5, 250_000, 4).startswith("configs[4] (1M ballots")
    assert config_name(20, 5, 125_000, 1).startswith("configs[4] per-GPU shard")


def test_bench_default_workload_per_gpu_count():
    """N = 1 measures configs[1] (10k ballots); N > 1 measures configs[2]'s per-GPU shard (125k
    ballots per rank: weak scaling, N = 8 is configs[2]'s 1M ballots) without any flag;
    --pipeline full runs configs[4]'s 125k-ballot shard of the 20 x (5+1) manifest at every N."""
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    from bench import config_name, default_ballots, parse
    assert default_ballots(1) == 10_000 and config_name(4, 5, default_ballots(1), 1) == "configs[1]"
    for n in (2, 4, 8):
        assert default_ballots(n) == 125_000
    assert config_name(4, 5, default_ballots(8), 8) == "configs[2] (1M ballots over 8 GPUs)"
    a = parse(["--pipeline", "full"])
    assert (a.contests, a.ballots) == (20, 125_000)
    assert config_name(a.contests, a.selections, a.ballots, 8).startswith("configs[4] (1M ballots")


def test_bench_line_at_world_2_has_cpu_baseline(tmp_path):
    """bench.py's N > 1 tail (bench.report) on 2 gloo ranks: after the barrier rank 0 times the CPU
    port on its host sample, and its line carries cpu_baseline (kind port, cores stated) and a
    non-null vs_baseline = value / cpu_baseline.value."""
    import json
    from pathlib import Path
    from electionguard.launch import run_ranks
    child = Path(__file__).resolve().parent / "_bench_report_child.py"
    out = tmp_path / "line.json"
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    assert run_ranks(str(child), [str(out)], 2, timeout=240, env=env) == 0
    d = json.loads(out.read_text())
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] >= 1 and cb["value"] > 0 and "verdicts all valid: True" in cb["sample"]
    assert d["vs_baseline"] is not None and abs(d["vs_baseline"] - d["value"] / cb["value"]) < 0.01 * d["vs_baseline"] + 0.01
    assert "cpu_baseline.value" in d["vs_baseline_basis"]


def test_comm_id_rendezvous_over_gloo():
    """The RCCL unique id (eg_comm_unique_id on rank 0) reaches every rank of the host process
    group unchanged (electionguard.distributed.share_comm_id, the rendezvous TallyExchange uses
    before eg_comm_init); a stand-in id is used here (no GPU)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_id_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(3))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = bytes(range(128))
    assert [r for r, _ in got] == [0, 1, 2] and all(uid == want for _, uid in got)


def _id_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from electionguard.distributed import share_comm_id

    def make():
        assert rank == 0, "only rank 0 makes the id"
        return bytes(range(128))

    q.put((rank, share_comm_id(dist, rank, make)))
    dist.destroy_process_group()


def test_launcher_fails_fast_when_a_rank_dies(tmp_path):
    """run_ranks (bench.py's self-launch) polls every rank: rank 1 exits 3 while rank 0 waits in
    a collective for it, and the launcher returns 3 within seconds (killing rank 0) instead of
    waiting for the collective's timeout."""
    import sys
    import time
    from pathlib import Path
    from electionguard.launch import run_ranks
    child = Path(__file__).resolve().parent / "_launch_child.py"
    env = dict(os.environ, EG_TEST_FAIL_RANK="1:3")
    env.pop("WORLD_SIZE", None)
    t = time.monotonic()
    rc = run_ranks(str(child), [str(tmp_path / "unused.json")], 2, timeout=240, env=env)
    assert rc == 3
    assert time.monotonic() - t < 60


def _fallback_worker(rank, world, port, q):
    """TallyExchange in "rccl" mode where rank 1 cannot create its communicator: every rank
    learns it and the whole world falls back to the host exchange (no rank dies, no rank hangs)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from electionguard.distributed import TallyExchange

    class FakeGroup:
        destroyed = False

        @staticmethod
        def comm_unique_id():
            return bytes(range(128))

        comm = None

        def comm_init(self, uid, w, r):
            assert uid == bytes(range(128)) and w == world and r == rank
            if rank == 1:
                raise RuntimeError("no RCCL here")
            self.comm = (w, r)

        def comm_info(self):
            return self.comm or (0, 0)

        def comm_destroy(self):
            FakeGroup.destroyed = True

    g = FakeGroup()
    x = TallyExchange(g, dist, world, rank, "rccl")
    q.put((rank, x.mode, x.collective, FakeGroup.destroyed, x.note is not None))
    dist.destroy_process_group()


def test_rccl_init_failure_falls_back_to_the_host_exchange():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fallback_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # both ranks drop their communicator state: rank 0 its live one, rank 1 its failed init's
    assert got == [(0, "gloo", "gloo (host)", True, True), (1, "gloo", "gloo (host)", True, True)]


def _strict_worker(rank, world, port, q):
    """TallyExchange(fallback=False) -- bench.py --strict-rccl, its default at N > 1 -- where rank 1
    cannot create its communicator: EVERY rank raises (the run exits non-zero instead of printing a
    scaling number for a host exchange)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from electionguard.distributed import TallyExchange

    class FakeGroup:
        comm = None

        @staticmethod
        def comm_unique_id():
            return bytes(range(128))

        def comm_init(self, uid, w, r):
            if rank == 1:
                raise RuntimeError("no RCCL here")
            self.comm = (w, r)

        def comm_info(self):
            return self.comm or (0, 0)

        def comm_destroy(self):
            self.comm = None

    try:
        TallyExchange(FakeGroup(), dist, world, rank, "rccl", fallback=False)
        q.put((rank, "no error"))
    except RuntimeError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_strict_rccl_fails_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_strict_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
    assert got[0] == (0, "eg_comm_init failed: on another rank")
    assert got[1][0] == 1 and "no RCCL here" in got[1][1]


def test_bench_strict_rccl_default_and_launch_budget(monkeypatch):
    """bench.py: --strict-rccl is on by default at N > 1 in RCCL mode (off for the gloo rehearsal and
    at N = 1); the self-launcher's kill deadline is the run's own budget plus ONE communicator
    deadline (EG_COMM_TIMEOUT_S), not 4 x --dist-timeout."""
    import importlib
    import sys
    from pathlib import Path
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    bench = importlib.import_module("bench")
    monkeypatch.delenv("EG_DIST_BACKEND", raising=False)
    monkeypatch.delenv("EG_COMM_TIMEOUT_S", raising=False)
    assert bench.parse(["--gpus", "8"]).strict_rccl == 1
    assert bench.parse(["--gpus", "1"]).strict_rccl == 0
    assert bench.parse(["--gpus", "8", "--strict-rccl", "0"]).strict_rccl == 0
    monkeypatch.setenv("EG_DIST_BACKEND", "gloo")
    assert bench.parse(["--gpus", "8"]).strict_rccl == 0
    monkeypatch.delenv("EG_DIST_BACKEND")
    a = bench.parse(["--gpus", "8", "--steps", "20", "--warmup", "5"])
    budget = bench.launch_budget_s(a)
    assert bench.comm_timeout_s() == bench.COMM_TIMEOUT_S
    assert 600 < budget < 1200 < 4 * a.dist_timeout, budget
    monkeypatch.setenv("EG_COMM_TIMEOUT_S", "30")
    assert bench.launch_budget_s(a) == pytest.approx(budget - bench.COMM_TIMEOUT_S + 30)


def test_world8_exchange_rccl_ranks_and_fallback(tmp_path):
    """bench.py's exchange at world 8 (run_ranks, the driver's N = 8 shape) over gloo with a stand-in
    communicator: when every rank's RCCL probe and init succeed the exchange runs in "rccl" mode and
    reports rccl_ranks = 8 on every rank (what the communicator says, eg_comm_info); the verdict is
    the min over ranks and the folded tally equals the tally over all ballots.  When one rank's probe
    fails, the readiness vote keeps EVERY rank out of the collective init (no rank can be left
    waiting in it), the world folds over the host with rccl_ranks 0 and a note, and the tally is
    still exact."""
    import json
    import sys
    from pathlib import Path
    from electionguard.launch import run_ranks
    child = Path(__file__).resolve().parent / "_exchange_child.py"
    out = tmp_path / "rank0.json"
    env = dict(os.environ, EG_TEST_PROBE_FAIL="3")
    env.pop("WORLD_SIZE", None)
    assert run_ranks(str(child), [str(out)], 8, timeout=300, env=env) == 0
    d = json.loads(out.read_text())
    assert d["world"] == 8
    good, failed = d["good"], d["failed"]
    assert good["mode"] == "rccl" and good["collective"] == "RCCL (libeg_hip)" and good["note"] is None
    assert good["ok"] is True and good["bad"] is False
    assert failed["mode"] == "gloo" and failed["collective"] == "gloo (host)" and failed["note"]
    assert failed["ok"] is True and failed["bad"] is False
    for r, (gc, fc, gr, fr) in enumerate(d["calls"]):
        assert gc == ["probe", "init", "destroy"] and gr == 8, (r, gc, gr)
        assert "init" not in fc and fr == 0, (r, fc, fr)  # the vote came before anyone's init
    sys.path.insert(0, str(child.parent))
    import _exchange_child as X
    G = O.production_group()
    cts = X.ballots(19, 2)
    for res in (good, failed):
        for s in range(2):
            for c in range(2):
                assert int(res["tally"][s][c], 16) == G.prodP([cts[i][s][c] for i in range(19)])


def test_world1_exchange_is_labelled_local():
    """At N = 1 there is no communicator: the line says so instead of naming RCCL."""
    from electionguard.distributed import TallyExchange
    x = TallyExchange(None, None, 1, 0, "rccl")
    assert x.collective == "no communicator (world 1: local fold)" and x.rccl_ranks == 0 and x.note is None
