"""CPU: execute the JNI wrappers (electionguard-remote_amd/jvm/src/main/c/eg_hip_jni.c) once.

No JDK exists in this image, so tests/jni/jni_harness.c compiles the JNI C file unchanged against a
stand-in jni.h (tests/jni/jni.h, test infrastructure) and calls every Java_electionguard_gpu_EgHip_*
function through a minimal JNIEnv: short arrays and negative counts must raise
IllegalArgumentException before the library is reached, a null handle must surface the library's
status as ArithmeticException(eg_last_error()), a failed array pin must not reach the library nor
leak, and clockMedian must return the median of its records."""
import re
import subprocess
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
LIBDIR = ROOT / "electionguard-remote_amd" / "electionguard" / "lib"
JNI_C = ROOT / "electionguard-remote_amd" / "jvm" / "src" / "main" / "c" / "eg_hip_jni.c"


def test_jni_wrappers_execute(tmp_path):
    exe = tmp_path / "jni_harness"
    subprocess.run(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-Wno-unused-variable", "-Wno-unused-parameter",
                    "-I", ROOT / "include", "-I", ROOT / "tests" / "jni", "-o", exe, ROOT / "tests" / "jni" / "jni_harness.c",
                    "-L", LIBDIR, "-leg_hip", f"-Wl,-rpath,{LIBDIR}", "-Wl,--allow-shlib-undefined"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    m = re.search(r"(\d+) checks, 0 errors", r.stdout)
    assert m and int(m.group(1)) >= 70, r.stdout


def test_harness_calls_every_jni_function():
    defined = set(re.findall(r"Java_electionguard_gpu_EgHip_(\w+)\(", JNI_C.read_text()))
    called = set(re.findall(r"Java_electionguard_gpu_EgHip_(\w+)\(", (ROOT / "tests" / "jni" / "jni_harness.c").read_text()))
    assert defined and defined <= called, sorted(defined - called)
