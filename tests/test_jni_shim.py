"""The JVM side of the boundary, on CPU: the JNI shim (jni/src/main/native/l5dh_jni.c)
must keep compiling against include/l5dhist.h (checked with a declarations-only
JNI stub, tests/jni_stub/jni.h: this image has no JDK), and the C caller of the ABI
(tests/c/abi_test.c, built by build()) links and runs without a GPU."""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(REPO, "jni", "src", "main", "native", "l5dh_jni.c")
JAVA = os.path.join(REPO, "jni", "src", "main", "java", "io", "buoyant", "telemetry", "gpu", "Native.java")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_jni_shim_compiles_against_the_header():
    r = subprocess.run(["gcc", "-fsyntax-only", "-std=c11", "-Wall", "-Wextra", "-Werror",
                        "-I", os.path.join(REPO, "tests", "jni_stub"), "-I", os.path.join(REPO, "include"), SHIM],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_every_native_method_has_a_shim_function():
    natives = set(re.findall(r"public static native \S+ (\w+)\(", open(JAVA).read()))
    shims = set(re.findall(r"Java_io_buoyant_telemetry_gpu_Native_(\w+)\(", open(SHIM).read()))
    assert natives and natives == shims


def test_c_caller_links_the_library():
    exe = os.path.join(REPO, "linkerd_amd", "lib", "l5dh_abi_test")
    if not os.path.exists(exe):
        pytest.skip("not built (run build())")
    r = subprocess.run([exe, "--version"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and r.stdout.strip() == "2"
