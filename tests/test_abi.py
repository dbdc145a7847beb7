"""The drop-in boundary on CPU: libl5dhist.so loads and exports every entry point
include/l5dhist.h declares, the ctypes binding covers exactly those, and the
header's constants agree with the host code.  No compute call is made (there is
no GPU here); l5dh_limits and argument validation in l5dh_open are host-only.
"""
import ctypes
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

from linkerd_amd import _native as N

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(N.LIB_PATH):
        if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
            pytest.skip("libl5dhist.so not built and no hipcc to build it")
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "linkerd_amd", "csrc")], check=True)
    return N.load()


def _header():
    return open(N.HEADER_PATH).read()


def test_exports_every_header_symbol(lib):
    declared = N.header_symbols()
    assert len(declared) >= 18
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing
    # the same check with the dynamic symbol table, as a JNI/cgo linker sees it
    nm = shutil.which("nm")
    if nm:
        out = subprocess.run([nm, "-D", "--defined-only", N.LIB_PATH], capture_output=True, text=True).stdout
        exported = set(re.findall(r"\bT (l5dh_\w+)", out))
        assert set(declared) <= exported, sorted(set(declared) - exported)
        # nothing beyond the header leaks as a public l5dh_ symbol
        assert exported <= set(declared), sorted(exported - set(declared))


def test_binding_covers_header_exactly():
    assert set(N.SIGNATURES) == set(N.header_symbols())


def test_header_constants_match_host():
    h = _header()

    def define(name):
        return int(re.search(rf"#define {name} \(?(\d+)", h).group(1))

    assert define("L5DH_NLIMITS") == N.NLIMITS == 1797
    assert define("L5DH_NBUCKETS") == N.NBUCKETS == 1798
    assert define("L5DH_ABI_VERSION") == 3
    enum = dict((k, int(v)) for k, v in re.findall(r"(L5DH_(?:PARAM|K)_[A-Z0-9_]+) = (\d+)", h))
    assert enum["L5DH_PARAM_TIMING"] == N.PARAM_TIMING
    assert enum["L5DH_PARAM_COLD_LIMIT"] == N.PARAM_COLD_LIMIT
    assert enum["L5DH_PARAM_HOT_CHUNK"] == N.PARAM_HOT_CHUNK
    assert enum["L5DH_PARAM_MAX_SEGMENTS"] == N.PARAM_MAX_SEGMENTS
    assert enum["L5DH_PARAM_REGION_PCT"] == N.PARAM_REGION_PCT
    assert "L5DH_PARAM_BIN_MODE" not in enum and "L5DH_PARAM_SPLIT_MIN" not in enum  # removed in ABI 3
    assert [enum[f"L5DH_K_{n}"] for n in ("COUNT", "SCAN", "BIN", "ACCUM", "HOT", "COPY", "BIN2")] == \
        [N.K_COUNT, N.K_SCAN, N.K_BIN, N.K_ACCUM, N.K_HOT, N.K_COPY, N.K_BIN2]
    assert enum["L5DH_K_NKERNELS"] == len(N.KERNEL_NAMES)
    # l5dh_summary is Metric.HistogramSummary: 10 int64 + 1 double, 88 bytes
    assert N.SUMMARY_DTYPE.itemsize == 88 and N.SUMMARY_DTYPE.names == N.SUMMARY_FIELDS
    assert N.BUCKET_COUNT_DTYPE.itemsize == 12


def test_abi_version_and_limits(lib, oracle):
    assert lib.l5dh_abi_version() == 3
    lim = N.limits()
    assert lim.dtype == np.int32 and lim.shape == (N.NLIMITS,)
    np.testing.assert_array_equal(lim, oracle.limits())
    assert lim[0] == 1 and lim[-1] < 2**31 - 1 and np.all(np.diff(lim) > 0)


def test_open_rejects_bad_arguments_without_device(lib):
    ctx = ctypes.c_void_p()
    assert lib.l5dh_open(ctypes.byref(ctx), 0, 1) == -22          # max_series == 0
    assert lib.l5dh_open(ctypes.byref(ctx), (1 << 20) + 1, 1) == -22
    assert lib.l5dh_open(ctypes.byref(ctx), 10, 0) == -22         # no device
    assert lib.l5dh_open(ctypes.byref(ctx), 10, 3) == -22         # two devices
    assert lib.l5dh_open(None, 10, 1) == -22
    assert lib.l5dh_close(None) in (0, -22)


def test_no_development_switches_in_the_shipped_library(lib):
    """The shipped library reads no environment (no L5DH_DBG-style switches that
    would let a host silently skip work) and carries no such string."""
    data = open(N.LIB_PATH, "rb").read()
    assert b"L5DH_DBG" not in data
    nm = shutil.which("nm")
    if nm:
        undef = subprocess.run([nm, "-D", "--undefined-only", N.LIB_PATH], capture_output=True, text=True).stdout
        assert not re.search(r"\b(secure_)?getenv\b", undef), "libl5dhist.so imports getenv"
    src = os.path.join(REPO, "linkerd_amd", "csrc")
    for f in os.listdir(src):
        if f.endswith((".cpp", ".hip", ".hpp")):
            text = open(os.path.join(src, f)).read()
            assert "getenv" not in text and "g_dbg" not in text, f
