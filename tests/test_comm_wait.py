"""CPU: the deadline-bounded wait libeg_hip.so runs after every RCCL collective
(electionguard-remote_amd/csrc/eg_comm_wait.hpp; eg_capi_comm.inc comm_wait_locked), driven by
fake communicators (tests/cpp/comm_wait_test.cpp): a completion that never arrives -- a peer that
died after the collective was enqueued -- returns "timed out" at the deadline instead of hanging;
an asynchronous communicator error returns at once; a healthy completion is seen as done."""
import json
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_collective_wait_with_fake_communicators(tmp_path):
    exe = tmp_path / "comm_wait_test"
    subprocess.run(["g++", "-std=c++17", "-O2", "-pthread", "-I", str(ROOT / "electionguard-remote_amd" / "csrc"),
                    "-o", str(exe), str(ROOT / "tests" / "cpp" / "comm_wait_test.cpp")], check=True)
    r = subprocess.run([str(exe), "0.4"], capture_output=True, text=True, timeout=30)
    res = json.loads(r.stdout)
    assert r.returncode == 0 and res["failures"] == 0, res
    nc = res["never_completes"]
    assert nc["result"] == "timed out" and 0.4 <= nc["seconds"] < 3.0
    assert res["async_error"]["result"] == "communicator error" and res["async_error"]["code"] == 6
    assert res["completes"]["result"] == "done" and res["stream_error"]["result"] == "stream error"
