"""C++ host mirror (electionguard-remote_amd/host/electionguard.hpp) over the C ABI.

CPU: the mirror builds, its mod-q scalar arithmetic and constants self-check, and the
generated constants header matches electionguard/core/constants.py.
GPU: the golden vectors of both groups (tests/golden/<mode>/*.json) through the C++ GroupContext /
GpuDecryptingTrustee API, bit-exact, then a 5-guardian quorum-3 decryption with two
missing guardians recovering exact counts (tests/cpp/host_parity.cpp).
"""
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
GOLD = ROOT / "tests" / "golden"


def _bin():
    sys.path.insert(0, str(ROOT))
    import __graft_entry__ as ge
    if not ge.LIB.exists():
        pytest.skip("libeg_hip.so not built")
    return ge.build_host_cpp()


def test_constants_header_is_current():
    sys.path.insert(0, str(ROOT / "tools"))
    import gen_constants_hpp as gen
    assert gen.OUT.read_text() == gen.render(), "run python tools/gen_constants_hpp.py"


def test_cpp_host_cpu_selfcheck():
    r = subprocess.run([str(_bin()), "cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK")


def write_vectors(path: Path, mode: str = "Mode4096") -> int:
    g = json.loads((GOLD / mode / "group_ops.json").read_text())
    t = json.loads((GOLD / mode / "trustee.json").read_text())
    lines = []
    lines += [f"powP {v['b']} {v['e']} {v['r']}" for v in g["powP"]]
    lines += [f"gPowP {v['e']} {v['r']}" for v in g["gPowP"]]
    lines += [f"multP {v['a']} {v['b']} {v['r']}" for v in g["multP"]]
    lines += [f"multInv {v['a']} {v['r']}" for v in g["multInv"]]
    lines += [f"prodP {v['r']} " + " ".join(v["xs"]) for v in g["prodP"]]
    for gd in t["guardians"]:
        lines.append(f"guardian {gd['x']} {len(gd['coeffs'])} " + " ".join(gd["coeffs"]) + " " +
                     " ".join(gd["commitments"]))
    lines.append(f"qbar {t['qbar']}")
    lines += [f"text {a} {b}" for a, b in t["texts"]]
    lines += [f"nonce {u}" for u in t["nonces"]]
    lines += [f"direct {d['M']} {d['c']} {d['v']}" for d in t["direct"]]
    lines += [f"compensated {d['M']} {d['c']} {d['v']} {d['recovery']}" for d in t["compensated_by_x2_for_x3"]]
    path.write_text("\n".join(lines) + "\n")
    return len(lines)


def test_vector_file_covers_golden(tmp_path):
    assert write_vectors(tmp_path / "v.txt") > 100


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["Mode4096", "Mode4096_V2"])
def test_cpp_host_gpu_parity(tmp_path, mode):
    v = tmp_path / "vectors.txt"
    write_vectors(v, mode)
    args = [str(_bin()), "gpu", str(v)] + (["V2"] if mode == "Mode4096_V2" else [])
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("OK")


def write_format_vectors(path: Path, variant: dict, fx: dict) -> None:
    """The trustee lines of one proof-format variant (tests/golden/Mode4096/proof_formats.json)."""
    resp = {"minus": 0, "plus": 1}[variant["response"]]
    pre = {"message_first": 0, "commitments_first": 1, "with_key": 2}[variant["preimage"]]
    lines = [f"format {resp} {pre}"]
    for gd in fx["guardians"]:
        lines.append(f"guardian {gd['x']} {len(gd['coeffs'])} " + " ".join(gd["coeffs"]) + " " +
                     " ".join(gd["commitments"]))
    lines.append(f"qbar {fx['qbar']}")
    lines += [f"text {a} {b}" for a, b in fx["texts"]]
    lines += [f"nonce {u}" for u in fx["nonces"]]
    lines += [f"direct {d['M']} {d['c']} {d['v']}" for d in variant["direct"]]
    lines += [f"compensated {d['M']} {d['c']} {d['v']} {d['recovery']}" for d in variant["compensated_by_x2_for_x3"]]
    path.write_text("\n".join(lines) + "\n")


@pytest.mark.gpu
def test_cpp_host_proof_formats(tmp_path):
    """GroupContext::setProofFormat: the C++ trustee reproduces every variant's shares and proofs, and
    the 5-guardian decryption (proofs made and checked under that variant) recovers its counts."""
    fx = json.loads((GOLD / "Mode4096" / "proof_formats.json").read_text())
    for v in fx["variants"]:
        f = tmp_path / f"{v['response']}_{v['preimage']}.txt"
        write_format_vectors(f, v, fx)
        r = subprocess.run([str(_bin()), "gpu", str(f)], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (v["response"], v["preimage"], r.stdout + r.stderr)
        assert r.stdout.startswith("OK")
