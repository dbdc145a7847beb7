"""The JNI shim executed on the GPU without a JVM (SURVEY.md §8(b) "JNI shim";
reference boundary io.buoyant.telemetry.Metric.Stat, Metric.scala:22-70).

tests/c/jni_fake_env.c links jni/src/main/native/l5dh_jni.c with libl5dhist.so and
drives every Java_io_buoyant_telemetry_gpu_Native_* function through a fake JNIEnv
function table, in the call sequence of GpuEngine.scala: open, limits, setParam,
pinAlloc, ingestAsync / ingestWait (double-buffered pinned staging), ingest, sync
(the deferred invalid-id report), lastError, peek, snapshot (summaries + counts,
with reset), commUniqueId / commInitRank / merge (one rank, the RCCL collective
forced), a second context through commInitAll + merge (all-reduce), pinFree, close.
Its outputs are compared with the CPU oracle here, bit for bit."""
import os
import subprocess

import numpy as np
import pytest

from linkerd_amd import _native as N
from linkerd_amd import synth

pytestmark = pytest.mark.gpu

EXE = os.path.join(N.PKG_DIR, "lib", "l5dh_jni_fake_env")


def _summ(path):
    return np.fromfile(path, dtype=N.SUMMARY_DTYPE)


def _eq(got, want, label):
    for f in N.SUMMARY_FIELDS:
        assert np.array_equal(got[f], want[f]), f"{label}: field {f} differs"


def test_every_jni_entry_point_on_the_gpu(oracle, tmp_path):
    S, n, piece = 3000, 600_000, 65_536
    series, vals = synth.c3(S=S, N=n, seed=123)
    vals[::211] = np.float32(3e9)   # escapes (overflow bucket) through the shim too
    vals[5::307] = np.float32(-7.0)
    series.astype(np.uint32).tofile(tmp_path / "series.bin")
    vals.astype(np.float32).tofile(tmp_path / "values.bin")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([EXE, str(tmp_path), str(S), str(n), str(piece)], capture_output=True, text=True, timeout=240,
                       env=env)
    assert r.returncode == 0, f"rc={r.returncode}\n{r.stdout}\n{r.stderr}"
    log = (tmp_path / "log.txt").read_text()
    assert "lastError after invalid ids: series id" in log, log
    calls = [int(x) for x in log.strip().splitlines()[-1].split(":")[1].split()]
    assert len(calls) == 10 and all(c > 0 for c in calls), f"every JNIEnv function is exercised: {calls}"

    o = oracle.OracleHistograms(S)
    o.ingest(series, vals)
    want_counts, want_tot = o.counts(), o.totals()
    want = o.snapshot(reset=False)
    np.testing.assert_array_equal(np.fromfile(tmp_path / "limits.bin", dtype=np.int32), oracle.limits())
    # snapshot(reset) through the shim
    np.testing.assert_array_equal(np.fromfile(tmp_path / "counts.bin", dtype=np.int32).reshape(S, N.NBUCKETS),
                                  want_counts)
    _eq(_summ(tmp_path / "summ.bin"), want, "snapshot")
    assert not _summ(tmp_path / "summ2.bin")["count"].any(), "the reset cleared every series"
    # peek of series 0..3 (BucketAndCount lower/upper/count of the non-empty buckets)
    L = oracle.limits()
    raw = (tmp_path / "peek.bin").read_bytes()
    off = 0
    for s in range(4):
        k = int(np.frombuffer(raw, np.uint32, 1, off)[0])
        off += 4
        pk = np.frombuffer(raw, N.BUCKET_COUNT_DTYPE, k, off)
        off += 12 * k
        nz = np.flatnonzero(want_counts[s] > 0)
        assert k == nz.size
        np.testing.assert_array_equal(pk["count"], want_counts[s][nz])
        np.testing.assert_array_equal(pk["lower"], np.where(nz == 0, 0, L[np.maximum(nz - 1, 0)]))
        np.testing.assert_array_equal(pk["upper"], np.where(nz < 1797, L[np.minimum(nz, 1796)], 2147483647))
    # merge at one rank (reduce-scatter) and through commInitAll (all-reduce): one copy of the data each
    for tag in ("rs", "ar"):
        np.testing.assert_array_equal(
            np.fromfile(tmp_path / f"merge_{tag}_counts.bin", dtype=np.int32).reshape(S, N.NBUCKETS), want_counts)
        _eq(_summ(tmp_path / f"merge_{tag}_summ.bin"), want, f"merge {tag}")
    np.testing.assert_array_equal(np.fromfile(tmp_path / "merge_rs_totals.bin", dtype=np.int64), want_tot)
