"""Synthetic workloads of BASELINE.md (C1-C4), counter-based so any slice can be
regenerated independently (numpy here; linkerd_amd/csrc/l5dh_synth.hip is the
same recipe on the GPU for the full-size bench inputs).

Recipe:
  rand(seed, stream, i) = mix64(((seed << 48) ^ (stream << 40) ^ i) + 1) * GOLD),
  where mix64 is the SplitMix64 finalizer; uniform = (r >> 11) * 2^-53.
  Normal by Box-Muller on two uniforms; value = float32(exp(mu + sigma*z))
  clamped to [0, 1e9].
  C1: one series, mu = ln 20, sigma = 1.0, seed 1.
  C2: S series x K samples; mu_s = ln U[1,1000] (stream 1, index s), sigma 0.8;
      COO position i holds sample j = (i*A + B) mod N of series j // K.
  C3: series = Zipf(s=1) rank (inverse CDF over 1/r), values as C2.
"""
from __future__ import annotations

import numpy as np

GOLD = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
PERM_A = 2654435761  # prime, coprime with every N = S*K used here (2^a 5^b)
PERM_B = 40503
VMAX = 1e9


def mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z ^= z >> np.uint64(30)
        z *= M1
        z ^= z >> np.uint64(27)
        z *= M2
        z ^= z >> np.uint64(31)
    return z


def rand_u64(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    x = (np.uint64(seed) << np.uint64(48)) ^ (np.uint64(stream) << np.uint64(40)) ^ idx.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (x + np.uint64(1)) * GOLD
    return mix64(z)


def uniform(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    return (rand_u64(seed, stream, idx) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def normal(seed: int, stream: int, idx: np.ndarray) -> np.ndarray:
    idx = idx.astype(np.uint64)
    u1 = uniform(seed, stream, idx * np.uint64(2)) + 2.0 ** -53  # (0, 1]
    u2 = uniform(seed, stream, idx * np.uint64(2) + np.uint64(1))
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def lognormal_f32(mu, sigma: float, z: np.ndarray) -> np.ndarray:
    v = np.exp(mu + sigma * z)
    return np.clip(v, 0.0, VMAX).astype(np.float32)


def series_mu(seed: int, series: np.ndarray) -> np.ndarray:
    """mu_s = ln(U[1, 1000]) per series (stream 1)."""
    u = uniform(seed, 1, series.astype(np.uint64))
    return np.log(1.0 + 999.0 * u)


def c1(n: int = 10_000_000, seed: int = 1):
    idx = np.arange(n, dtype=np.uint64)
    vals = lognormal_f32(np.log(20.0), 1.0, normal(seed, 2, idx))
    return np.zeros(n, dtype=np.uint32), vals


def c2(S: int = 100_000, K: int = 1_000, seed: int = 2, sigma: float = 0.8):
    N = S * K
    i = np.arange(N, dtype=np.uint64)
    j = (i * np.uint64(PERM_A) + np.uint64(PERM_B)) % np.uint64(N)
    series = (j // np.uint64(K)).astype(np.uint32)
    mu = series_mu(seed, series)
    vals = lognormal_f32(mu, sigma, normal(seed, 2, j))
    return series, vals


def zipf_cdf(S: int, s: float = 1.0) -> np.ndarray:
    w = 1.0 / np.power(np.arange(1, S + 1, dtype=np.float64), s)
    c = np.cumsum(w)
    return c / c[-1]


def c3(S: int = 1_000_000, N: int = 1_000_000_000, seed: int = 3, sigma: float = 0.8, base_index: int = 0):
    idx = np.arange(base_index, base_index + N, dtype=np.uint64)
    u = uniform(seed, 3, idx)
    cdf = zipf_cdf(S)
    series = np.minimum(np.searchsorted(cdf, u, side="right"), S - 1).astype(np.uint32)
    mu = series_mu(seed, series)
    vals = lognormal_f32(mu, sigma, normal(seed, 2, idx))
    return series, vals
