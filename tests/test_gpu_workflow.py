"""GPU: the remote workflow end to end (RunRemoteWorkflowTest.java:83-192 shape) with
separate trustee processes over gRPC on localhost, including compensated decryption."""
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,quorum,avail,nb", [(3, 3, 3, 25), (5, 3, 3, 40)])
def test_remote_workflow(n, quorum, avail, nb):
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "run_workflow.py"), "-nguardians", str(n), "-quorum",
                        str(quorum), "-navailable", str(avail), "-nballots", str(nb)],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert '"match": true' in r.stdout
