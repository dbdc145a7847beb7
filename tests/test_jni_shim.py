"""The JVM side of the boundary, on CPU: the JNI shim (jni/src/main/native/l5dh_jni.c)
must keep compiling against include/l5dhist.h (checked with a declarations-only
JNI stub, tests/jni_stub/jni.h: this image has no JDK), and the C caller of the ABI
(tests/c/abi_test.c) and the fake-JNIEnv driver of the shim (tests/c/jni_fake_env.c,
run on the GPU by tests/test_gpu_jni.py) link and start without a GPU."""
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
    assert r.returncode == 0 and r.stdout.strip() == "3"


def test_fake_jnienv_driver_links_the_shim():
    """tests/c/jni_fake_env.c (built by build()): the shim and the library link into one
    program; without arguments it prints its usage and touches no device."""
    exe = os.path.join(REPO, "linkerd_amd", "lib", "l5dh_jni_fake_env")
    if not os.path.exists(exe):
        pytest.skip("not built (run build())")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr
