"""GPU: the remote workflow end to end (RunRemoteWorkflowTest.java:83-192 shape) with
separate trustee processes over gRPC on localhost, including compensated decryption."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,quorum,avail,nb,spoiled", [(3, 3, 3, 25, 0), (5, 3, 3, 40, 6)])
def test_remote_workflow(n, quorum, avail, nb, spoiled):
    """(5, 3, 3, 40, 6): 5 guardians, quorum 3, 2 missing; 6 of the 40 ballots spoiled -- the tally
    counts the 34 cast ones and each spoiled ballot decrypts through the gRPC trustees (direct and
    compensated shares) to its exact votes (RunRemoteDecryptor.java:264-269)."""
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "run_workflow.py"), "-nguardians", str(n), "-quorum",
                        str(quorum), "-navailable", str(avail), "-nballots", str(nb), "-nspoiled", str(spoiled)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert '"match": true' in r.stdout
    if spoiled:
        assert '"spoiled_match": true' in r.stdout
