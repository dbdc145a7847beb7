"""Sanitizer runs of host code (no sanitizers exist in the reference;
the build runs them on the CPU oracle and the C-ABI's host side):

the oracle's multithreaded ingest (per-series mutexes, the restatement of the
per-Stat monitor) under ThreadSanitizer and under AddressSanitizer + UBSan
(tests/c/oracle_threads.c).  GPU AddressSanitizer is not available on this pool; device code is covered by the
parity tests."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")


def _build_run(tmp_path, name, flags, srcs, env=None):
    exe = tmp_path / name
    cmd = ["gcc", "-O1", "-g", "-std=c11", "-ffp-contract=off", *flags, "-I", os.path.join(REPO, "oracle"),
           "-o", str(exe), *srcs, "-lm", "-lpthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    e = dict(os.environ)
    e.update(env or {})
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0 and r.stdout.strip() == "ok", r.stdout + r.stderr[-4000:]
    return r


SRCS = [os.path.join(REPO, "tests", "c", "oracle_threads.c"), os.path.join(REPO, "oracle", "hist_oracle.c")]


def test_oracle_threaded_ingest_tsan(tmp_path):
    r = _build_run(tmp_path, "tsan", ["-fsanitize=thread"], SRCS, {"TSAN_OPTIONS": "halt_on_error=1"})
    assert "ThreadSanitizer" not in r.stderr


def test_oracle_threaded_ingest_asan_ubsan(tmp_path):
    r = _build_run(tmp_path, "asan", ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"], SRCS,
                   {"ASAN_OPTIONS": "detect_leaks=1"})
    assert "runtime error" not in r.stderr
