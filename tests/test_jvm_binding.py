"""CPU: the JVM binding sources (electionguard-remote_amd/jvm) cover the C ABI.

No JDK exists in this image, so the Java / JNI sources cannot be compiled here; these tests
check them structurally: every export of include/eg_hip.h is called by the JNI C file, every
`native` method of EgHip.java has its JNIEXPORT function (and no orphan exists), the adapters
implement the reference's interfaces, and the generated EgConstants.java is current."""
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
JVM = ROOT / "electionguard-remote_amd" / "jvm" / "src" / "main"
JNI_C = JVM / "c" / "eg_hip_jni.c"
EGHIP = JVM / "java" / "electionguard" / "gpu" / "EgHip.java"


def _exports():
    h = (ROOT / "include" / "eg_hip.h").read_text()
    return set(re.findall(r"^\s*(?:int|const char\*|eg_fixed_base\*)\s+(eg_[a-z0-9_]+)\s*\(", h, re.M))


def test_jni_calls_every_c_abi_export():
    called = set(re.findall(r"\b(eg_[a-z0-9_]+)\s*\(", JNI_C.read_text()))
    exports = _exports()
    assert len(exports) == 54
    assert exports <= called, sorted(exports - called)


def test_every_native_method_has_its_jni_function():
    natives = set(re.findall(r"public static native [\w\[\]]+ (\w+)\(", EGHIP.read_text()))
    jni = set(re.findall(r"Java_electionguard_gpu_EgHip_(\w+)\(", JNI_C.read_text()))
    assert natives and natives == jni, (sorted(natives - jni), sorted(jni - natives))


def test_adapters_implement_the_reference_interfaces():
    t = (JVM / "java" / "electionguard" / "gpu" / "GpuDecryptingTrustee.java").read_text()
    assert "implements DecryptingTrusteeIF" in t
    for sig in ("public String id()", "public int xCoordinate()", "public ElementModP electionPublicKey()",
                "public List<DirectDecryptionAndProof> directDecrypt(GroupContext group, List<ElGamalCiphertext> texts",
                "public List<CompensatedDecryptionAndProof> compensatedDecrypt(GroupContext group, String missingGuardianId"):
        assert sig in t, sig
    g = (JVM / "java" / "electionguard" / "gpu" / "GpuGroupContext.java").read_text()
    for m in ("powP(", "gPowP(", "multP(", "prodP(", "multInv(", "verifyBallots(", "encryptBallots(", "powPAsync("):
        assert f" {m}" in g, m


def test_java_constants_are_current():
    sys.path.insert(0, str(ROOT / "tools"))
    import gen_constants_hpp as gen
    assert gen.OUT_JAVA.read_text() == gen.render_java(), "run python tools/gen_constants_hpp.py"
