"""Golden vectors for the histogram path, produced by the CPU oracle
(oracle/hist_oracle.c, pinned by P1-P5 in tests/test_oracle.py).

The reference (Scala + finagle-stats jar) cannot run in this image, so these
vectors freeze the oracle's restatement; tests/test_oracle.py re-derives them
and tests/test_gpu_parity.py checks the HIP engine against them on the GPU box.
Output: tests/golden/golden_<case>.npz (inputs, dense counts, totals, summaries).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from linkerd_amd import synth  # noqa: E402
from oracle import oracle as O  # noqa: E402

EDGE = np.array([0.0, 0.5, 1.0, 112.99, 113.0, 114.0, 3030.0, 2323.0, 65535.0, 1e6, 1.3e7, 1e9,
                 2137204091.0, 2147483520.0, 2147483648.0, 3e9, np.inf, -0.5, -1.0, -3e9, -np.inf, np.nan],
                dtype=np.float32)


def cases():
    rng = np.random.default_rng(1234)
    # a: 64 series, lognormal + edge values
    S = 64
    s = rng.integers(0, S, 20000, dtype=np.uint32)
    v = np.exp(rng.uniform(0, 7, S)[s] + 0.8 * rng.standard_normal(s.size)).astype(np.float32)
    v[::50] = rng.choice(EDGE, v[::50].size)
    yield "mixed64", S, s, v
    # b: C1 recipe, first 100k samples (one series)
    s, v = synth.c1(n=100_000)
    yield "c1_100k", 1, s, v
    # c: C2 recipe at 200 series x 500 samples
    s, v = synth.c2(S=200, K=500)
    yield "c2_200x500", 200, s, v
    # d: Zipf series (C3 recipe) 1000 series, 50k samples
    s, v = synth.c3(S=1000, N=50_000)
    yield "c3_zipf1000", 1000, s, v


def main():
    for name, S, s, v in cases():
        h = O.OracleHistograms(S)
        assert h.ingest(s, v) == 0
        counts, totals = h.counts(), h.totals()
        summ = h.snapshot(reset=True)
        path = os.path.join(HERE, f"golden_{name}.npz")
        np.savez_compressed(path, nseries=np.int64(S), series=s, values=v, counts=counts, totals=totals,
                            summaries=summ.view(np.uint8).reshape(S, 88))
        print(f"{path}: {s.size} samples, {S} series, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
