"""GPU: the reference's per-element call pattern end to end (tests/cpp/percall_workflow.cpp).

Upstream encrypts and verifies ballots one group operation at a time from 11 threads and tallies in
one thread (RunRemoteWorkflowTest.java:140-141,151,179-181) on the group KUtils.productionGroup()
makes (KUtils.java:10-12).  The C++ driver restates that call order through the mirror's
per-element API only (deferred elements merged into coalesced library jobs, host/electionguard.hpp
Deferred) and checks every ciphertext and proof byte against the C oracle's encryption of the same
nonces, every verdict against its verifier, a tampered proof's rejection and the one-thread tally
against a BN_mod_mul loop.  Rates are recorded by tools/percall_workflow.py (profiles/), not
asserted here: this suite gates on bit-exactness."""
import json
import subprocess
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parent.parent
BIN = ROOT / "electionguard-remote_amd" / "host" / "_build" / "percall_workflow"


@pytest.mark.parametrize("mode", [[], ["eager"], ["ct"]])
def test_percall_workflow_bitexact(mode):
    assert BIN.exists(), "run __graft_entry__.build() first"
    n = 22 if mode == ["eager"] else 44
    r = subprocess.run([str(BIN), str(n), "11", *mode], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    print(d)
    assert d["ballots"] == n and d["threads"] == 11
    assert d["deferred"] is (mode != ["eager"]) and d["constant_time"] is (mode == ["ct"])
    for k in ("encrypt_mismatched_arrays", "verify_flag_mismatches", "invalid_flags", "tamper_not_rejected",
              "tally_mismatch", "errors"):
        assert d[k] == 0, (k, d)
