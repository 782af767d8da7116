"""CPU: GpuDecryptingTrustee.java against the reference's DecryptingTrusteeIF, without a JDK.

tools/java_signatures.py parses Java method signatures from source; the reference's side
(RemoteDecryptingTrusteeProxy.java:32-115 implementing DecryptingTrusteeIF, and the delegate calls
of RunRemoteDecryptingTrustee.java:189-193,227-232 that pass a null nonce) is committed as data in
tests/golden/reference_signatures.json.  Every interface method of the GPU trustee must have the
reference's return type, parameter types in order and @Nullable markers, and accept the reference's
own call sites; a deliberately swapped parameter must be caught."""
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import java_signatures as J  # noqa: E402

TRUSTEE = ROOT / "electionguard-remote_amd" / "jvm" / "src" / "main" / "java" / "electionguard" / "gpu" / \
    "GpuDecryptingTrustee.java"


def _fixture():
    return json.loads(J.FIXTURE.read_text())


def test_gpu_trustee_matches_the_reference_interface():
    fx = _fixture()
    impl = J.override_methods(TRUSTEE.read_text())
    assert set(fx["DecryptingTrusteeIF"]) == {"id", "xCoordinate", "electionPublicKey", "directDecrypt",
                                              "compensatedDecrypt"}
    assert fx["delegate_calls"]["directDecrypt"] == [{"nargs": 4, "null_args": [3]}]
    assert fx["delegate_calls"]["compensatedDecrypt"] == [{"nargs": 5, "null_args": [4]}]
    assert J.compare(impl, fx["DecryptingTrusteeIF"], fx["delegate_calls"]) == []


@pytest.mark.parametrize("mutation", ["swap", "nullable", "return", "drop"])
def test_checker_catches_a_broken_signature(mutation):
    src = TRUSTEE.read_text()
    if mutation == "swap":  # missingGuardianId and texts swapped
        bad = src.replace("compensatedDecrypt(GroupContext group, String missingGuardianId,\n"
                          "                                                                List<ElGamalCiphertext> texts,",
                          "compensatedDecrypt(GroupContext group, List<ElGamalCiphertext> texts,\n"
                          "                                                                String missingGuardianId,")
    elif mutation == "nullable":  # the nonce loses @Nullable (the reference passes null)
        bad = src.replace("ElementModQ extendedBaseHash, @Nullable ElementModQ nonce) {",
                          "ElementModQ extendedBaseHash, ElementModQ nonce) {", 1)
    elif mutation == "return":
        bad = src.replace("public List<DirectDecryptionAndProof> directDecrypt(",
                          "public List<CompensatedDecryptionAndProof> directDecrypt(")
    else:  # the nonce parameter dropped
        bad = src.replace("ElementModQ extendedBaseHash, @Nullable ElementModQ nonce) {",
                          "ElementModQ extendedBaseHash) {", 1)
    assert bad != src, "mutation did not apply"
    fx = _fixture()
    assert J.compare(J.override_methods(bad), fx["DecryptingTrusteeIF"], fx["delegate_calls"]) != []


@pytest.mark.skipif(not J.REF.exists(), reason="the reference checkout is not present")
def test_fixture_is_current_with_the_reference():
    assert J.make_fixture() == _fixture()
