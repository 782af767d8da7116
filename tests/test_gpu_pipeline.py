"""bench.py --pipeline full (configs[4]'s full pipeline: device encryption, verify + tally, the
fold, threshold decryption through 5 DecryptingTrustees with 2 missing) at a small size on one
MI355X: the decrypted counts equal the vote totals, the folded tally equals the C oracle's tally of
the GPU's ciphertexts (which the oracle verifies), and the CPU port reproduces the GPU's encryption
bytes inside the line's cpu_baseline."""
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


def test_full_pipeline_small_against_the_oracle():
    sys.path.insert(0, str(ROOT))
    import bench
    from eg_oracle_c import COracle
    from electionguard.core import constants as C
    a = bench.parse(["--pipeline", "full", "--ballots", "257", "--contests", "3", "--selections", "4",
                     "--steps", "1", "--warmup", "1", "--fb-window", "12", "--cpu-seconds", "1",
                     "--cpu-max-ballots", "257", "--modexp-n", "0"])
    keep = {}
    out = bench.full_pipeline(a, 1, 0, 0, None, keep=keep)
    man = keep["man"]
    assert out["phases"]["counts_exact"] and [int(x) for x in keep["counts"]] == [int(x) for x in keep["want"]]
    assert sum(int(x) for x in keep["counts"]) == 257 * 3  # one vote per contest
    co = COracle(C.P, C.Q, C.G)
    co.set_key(keep["K"])
    ok_s, ok_c, tally = co.verify_ballots(keep["qbar"], man.n_contests, man.spc, 1, 1, keep["cts"], keep["rproof"],
                                          keep["cproof"], threads=8)
    assert ok_s.all() and ok_c.all()
    assert np.array_equal(tally, keep["tally"])
    cb = out["cpu_baseline"]
    assert cb["kind"] == "port" and "reproduced the GPU's bytes" in cb["sample"] and out["vs_baseline"] > 0
    assert out["metric"].startswith("ballots encrypted+verified+tallied+decrypted/sec")
    assert out["config"]["pipeline"] == "full"
