"""Simulation of k_rplan1's level-1 capacity plan (linkerd_amd/csrc/l5dh_ingest.hip,
rcap) on C3: 1M series, 1e9 Zipf samples per batch, 2^18 sampled draws, the previous
batch's exact counts as `kprev`.  Counts are Poisson around the Zipf expectation; the
sample is a multinomial draw of the same law.  Reports, per step, the planned super-tile
and direct half-bin space and the bins whose exact records exceed their region (a
level-1 redo on the GPU).

  python tools/plan_sim.py [--rule r05|r06] [--steady] [--steps N]

--steady: every batch has the same law; default: the hot set moves by a third of the
series space per batch (bench.py --hot-shift).  r05: round 5's rule (previous count
when the sample is within 4 sigma above it, else e + 4 sigma); r06: the kernel's rule.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from linkerd_amd.synth import zipf_cdf  # noqa: E402

S, N, R = 1_000_000, 1_000_000_000, 3
F = (S + 31) // 32
K = 2 * F
FS = (F + 63) // 64
M = 1 << 18
SC = N / M


def rcap(prev, e, pad, align, rule, z, floor_sample):
    e0 = prev / SC
    sg = np.sqrt(e0 + 1)
    if rule == "r05":
        ok = (prev > 0) & (e <= e0 + 4 * sg)
        c = np.where(ok, np.ceil(prev * 1.0625 + 4 * np.sqrt(prev)), np.ceil((e + 4 * np.sqrt(e + 1)) * SC))
    else:
        sb = np.ceil((np.sqrt(e + 1) + z / 2) ** 2 * SC)
        ok = (prev > 0) & (e >= e0 - 6 * sg) & (floor_sample | (e <= e0 + 4 * sg))
        pb = np.ceil(prev * 1.0625 + 4 * np.sqrt(prev))
        c = np.where(ok, np.maximum(pb, sb) if floor_sample else pb, sb)
    return np.ceil(np.minimum(c + pad, 2 ** 30) / align) * align


def keys_of(per_series):
    c = np.zeros(K)
    np.add.at(c, np.arange(S) // 16, per_series)
    return c


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rule", default="r06", choices=["r05", "r06"])
    ap.add_argument("--steady", action="store_true")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    rng = np.random.default_rng(a.seed)
    pmf = np.diff(np.concatenate([[0.0], zipf_cdf(S)]))
    cap32 = N + N // 2 + (1 << 19)
    cap16 = 2 * N + N // 8 + 128 * F + 4096
    dlim16 = (cap16 - (N + 16 * F + 1024)) // 8 * 8
    kprev = np.zeros(K)
    bad = 0
    for step in range(a.steps):
        sh = 0 if a.steady else (step % R) * S // R
        lam = np.roll(pmf, sh)
        exact = keys_of(rng.poisson(lam * N).astype(float))
        samp = keys_of(rng.multinomial(M, lam).astype(float))
        tile_e = samp[0::2] + samp[1::2]
        est = tile_e * SC
        thr_min, dmax = N // 8192, 255
        cand = est[(est >= thr_min) & (est > 0)]
        lh = np.bincount(np.floor(np.log2(cand)).astype(int), minlength=33)
        cum, kbest = 0, 32
        for b in range(31, -1, -1):
            cum += lh[b]
            if cum > dmax:
                break
            kbest = b
        thr = max(thr_min, 1 << kbest) if kbest < 32 else np.inf
        direct = est >= thr
        dt = np.flatnonzero(direct)
        nd = ~direct
        st = np.arange(F)[nd] // 64
        P, E, C = (np.bincount(st, w[nd], minlength=FS) for w in
                   (kprev[0::2] + kprev[1::2], tile_e, exact[0::2] + exact[1::2]))
        capS = rcap(P, E, 256, 4, a.rule, 6.0, True)
        dk = np.stack([2 * dt, 2 * dt + 1], 1).ravel()
        capD = rcap(kprev[dk], samp[dk], 256, 8, a.rule, 5.0, False)

        def clamp(cap, lim):
            base = np.concatenate([[0], np.cumsum(cap)[:-1]])
            return np.where(base + cap + 16 > lim, np.maximum(0, lim - 16 - base), cap)

        ovS = np.flatnonzero(C > clamp(capS, cap32))
        ovD = np.flatnonzero(exact[dk] > clamp(capD, dlim16))
        bad += bool(len(ovS) or len(ovD))
        print(f"step {step} shift {sh} direct tiles {len(dt)} super-tile space {capS.sum() / N:.3f}N "
              f"(buffer {cap32 / N:.2f}N) direct space {capD.sum() / N:.3f}N (buffer {dlim16 / N:.3f}N) "
              f"overflowing super-tile bins {len(ovS)} direct half-bins {len(ovD)}")
        kprev = exact
    print(f"{a.rule} {'steady' if a.steady else 'hot-shift'}: {bad} of {a.steps} steps would redo level 1")


if __name__ == "__main__":
    main()
