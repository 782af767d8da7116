"""bench.py quotes roofline.traffic only from a committed PMC profile of the same finished config
(exchange fields included) and the same library build (tools/profile_round.sh writes them)."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "electionguard-remote_amd"))

import bench  # noqa: E402


def _newest_profile():
    profs = sorted((ROOT / "profiles").glob("r*_pmc_kpow.json"), reverse=True)
    assert profs, "no committed PMC profile"
    return json.loads(profs[0].read_text()), profs[0].name


def test_traffic_quoted_for_the_profiled_config_and_build():
    pm, name = _newest_profile()
    out = {"config": dict(pm["bench_config"]), "build": pm["bench_build"], "roofline": {"traffic": None}}
    bench.attach_traffic(out)
    assert out["roofline"]["traffic"] == round(pm["traffic"]["hbm_bytes_per_launch"])
    assert out["roofline"]["traffic_source"].startswith("profiles/r")


def test_traffic_not_quoted_for_another_build_or_config():
    pm, _ = _newest_profile()
    other_build = {"config": dict(pm["bench_config"]), "build": "000000000000", "roofline": {"traffic": None}}
    bench.attach_traffic(other_build)
    assert other_build["roofline"]["traffic"] is None
    cfg = dict(pm["bench_config"])
    cfg["rccl_ranks"] = 8
    other_cfg = {"config": cfg, "build": pm["bench_build"], "roofline": {"traffic": None}}
    bench.attach_traffic(other_cfg)
    assert other_cfg["roofline"]["traffic"] is None
