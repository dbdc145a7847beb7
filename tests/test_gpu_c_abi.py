"""A C program (tests/c/abi_test.c, no Python in between) drives the C-ABI on the
GPU the way the JNI shim does -- open, limits, pinned staging, ingest in small calls,
sync, snapshot, peek, 1-rank RCCL merge, close -- and its outputs are compared with
the oracle."""
import os
import subprocess

import numpy as np
import pytest

from linkerd_amd import _native as N
from linkerd_amd import synth

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_c_program_matches_oracle(oracle, tmp_path):
    S, n = 2500, 600_000
    series, vals = synth.c3(S=S, N=n, seed=91)
    inp, out = tmp_path / "in.bin", tmp_path / "out.bin"
    with open(inp, "wb") as f:
        f.write(np.array([S, n], np.uint64).tobytes() + series.tobytes() + vals.tobytes())
    exe = os.path.join(REPO, "linkerd_amd", "lib", "l5dh_abi_test")
    r = subprocess.run([exe, str(inp), str(out), "65536"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    buf = open(out, "rb").read()
    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    want_counts = o.counts()
    want = o.snapshot(reset=False)
    off = 0
    summ = np.frombuffer(buf, N.SUMMARY_DTYPE, S, off); off += 88 * S
    counts = np.frombuffer(buf, np.int32, S * N.NBUCKETS, off).reshape(S, N.NBUCKETS); off += 4 * S * N.NBUCKETS
    npeek = int(np.frombuffer(buf, np.uint64, 1, off)[0]); off += 8
    peek = np.frombuffer(buf, N.BUCKET_COUNT_DTYPE, npeek, off); off += 12 * npeek
    merged = np.frombuffer(buf, N.SUMMARY_DTYPE, S, off); off += 88 * S
    first, count, after = (int(x) for x in np.frombuffer(buf, np.uint64, 3, off))
    np.testing.assert_array_equal(counts, want_counts)
    assert summ.tobytes() == want.tobytes()
    assert merged.tobytes() == want.tobytes()
    assert (first, count, after) == (0, S, 0)
    nz = np.flatnonzero(want_counts[0])
    np.testing.assert_array_equal(peek["count"], want_counts[0][nz])
