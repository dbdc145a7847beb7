// l5dh_ingest.hip -- ingest-side kernels (Metric.Stat.add, batched): a two-level
// partition of the COO batch into capacity-planned regions, with no counting pass.
//
//   k_rsample  ids of 2^18 evenly spaced samples (every sample of a smaller batch)
//              counted per (tile, half) key
//   k_rplan1   this batch's direct tiles (the biggest estimated) and the level-1 bin
//              regions (super-tiles; two half-bins per direct tile), sized from the
//              previous batch's exact key counts and this batch's sample
//   k_rbin1w   level 1: LDS counting sort of 16K-sample sub-chunks by bin; each run's
//              place in its bin's region comes from ONE returning global atomic per
//              (sub-chunk, bin) on the bin's cursor (order inside a region is free:
//              integer sums do not depend on it); direct tiles' samples bucketized
//              into their final u16 records, their value sums folded in LDS
//   k_rfix1    a run that did not fit its region -> exact regions from the cursors
//              and a second k_rbin1w pass (launched always, it exits unless needed);
//              the direct keys' ranges; the invalid-id count to the host
//   k_rplan2a/b level-2 regions of the other keys (with the level-1 plan; k_rfix1
//              plans the level-2 items: 6K records of a super-tile's level-1 region)
//   k_rbin2    level 2: an item LDS-sorted by key into 16-bit records (series in
//              tile | bucket) in its keys' regions; value sums folded into sumfix
//   k_rfix2a/b exact key counts -> kprev (the next batch's prediction); overflow ->
//              exact regions and a second k_rbin2 pass
//
// Level-1 record of a super-tile bin (rec32): [31:26] tile in super-tile | [25:21]
//   series in tile | [20:0] payload = v (0 <= v < V_ESC) or V_ESC + bucket (escaped:
//   the exact sum contribution went to sumfix[series], integer atomics, order free).
// Final record (rec16, direct tiles at level 1, the others at level 2): [15:11]
//   series in tile | [10:0] bucket.
#include <algorithm>
#include <type_traits>

#include "l5dh_device.hpp"

namespace l5dh {
namespace {

// sampled ids per batch: 2^18 against 2^20 (fewer draws and flush atomics) -- the sample
// and plan phase 0.138 -> 0.097 ms; C2 -0.02 ms, the smallest 8-way C3 shard -5 %
// (profiles/r04z_ab.txt)
constexpr uint32_t RSAMPLE = 1u << 18;
#ifndef L5DH_RS_WG
#define L5DH_RS_WG 64
#endif
constexpr int RS_WG = L5DH_RS_WG;  // k_rsample workgroups (<= 65535 draws each: u16 LDS counters)
constexpr uint32_t INVALID = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t round_up(uint32_t x, uint32_t m) { return (x + m - 1) / m * m; }

// Region capacity of a bin or key from the previous batch's exact records `prev`
// and this batch's sampled ids `e` (scale s = samples per draw).  The sample's bound
// is a Poisson upper bound on the mean, (sqrt(e + 1) + z / 2)^2 draws: e + z sigma
// alone is short for the few draws of a tail bin (C3: 20-80).  When the sample is
// consistent with the previous batch (e within 4 sigma above and 6 sigma below
// prev / s) the previous count +1/16 + 4 sigma, and for a level-1 super-tile bin
// (`floor_sample`) at least the sample's bound; otherwise (a key that grew or shrank,
// or one never seen) the sample's bound; exact when the sample was the whole batch.
// Plus a pad.  A region that still overflows is redone with exact sizes (k_rfix1 /
// k_rfix2), so this only has to be right almost always -- but the sample's bound for
// every level-2 key would oversize each by ~z sigma (C2: 1.3x, past the region buffer).
// Round 6 (C3 --hot-shift, a moved hot set: every level-1 pass was redone,
// profiles/r06fin1_c3hot_bench.json; simulated in tools/plan_sim.py): a super-tile bin
// whose load doubled, sampled at ~80 draws, still fell within 4 sigma of its previous
// count -- hence the sample floor for those bins, whose buffer has room (C3 uses a
// third of it); a bin that lost its hot series kept the old count's region and the
// plan outgrew the buffer -- hence the lower test.  (6 sigma below: at 4, ~3000 well
// sampled C3 keys would take a sample-sized region, about their true count, by chance
// in ~10 % of steady-state batches.)  `pct` scales the result (L5DH_PARAM_REGION_PCT;
// below 100 forces the redo path).
__device__ __forceinline__ uint32_t rcap(double prev, double e, double s, bool exact, double pad, uint32_t align,
                                         uint32_t pct, double z, bool floor_sample) {
  double c;
  if (exact) {
    c = e;
  } else {
    const double e0 = prev / s, sg = sqrt(e0 + 1.0);
    const double r = sqrt(e + 1.0) + 0.5 * z;
    // (a level-2 key neither sampled nor seen before keeps round 5's 4 samples per draw: a
    // sparse space has tens of thousands of them, and (1 + z / 2)^2 draws each outgrew the
    // buffer -- a counting pass every batch, tests/test_gpu_parity.py::
    // test_sparse_key_space_steady_state; a super-tile bin keeps its larger bound)
    const double sb = !floor_sample && prev == 0.0 && e == 0.0 ? ceil(4.0 * s) : ceil(r * r * s);
    if (prev > 0.0 && e >= e0 - 6.0 * sg && (floor_sample || e <= e0 + 4.0 * sg)) {
      c = ceil(prev * 1.0625 + 4.0 * sqrt(prev));
      if (floor_sample) c = fmax(c, sb);
    } else {
      c = sb;
    }
    c += pad;
  }
  if (pct != 100) c = floor(c * (double)pct / 100.0);
  return round_up((uint32_t)fmin(c, 1073741824.0), align);
}

// Exclusive block scan of u64 values (one per thread), NT = 1024.
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t* lds /*[17]*/, uint64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan(v);
  if (lane == 63) lds[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t acc = 0;
    for (int k = 0; k < 16; ++k) {
      const uint64_t q = lds[k];
      lds[k] = acc;
      acc += q;
    }
    lds[16] = acc;
  }
  __syncthreads();
  const uint64_t r = lds[w] + incl - v;
  *total = lds[16];
  __syncthreads();
  return r;
}

#ifdef L5DH_PHASES
__device__ unsigned long long g_phase_plan[16];  // the plans: wall clock at their phase ends (thread 0)
#define RP_MARK(k) \
  if (threadIdx.x == 0) g_phase_plan[k] = wall_clock64();  // (k_rplan1: one workgroup)
#define RS_MARK(k) \
  if (threadIdx.x == 0 && blockIdx.x == 0) g_phase_plan[k] = wall_clock64();
#else
#define RP_MARK(k)
#define RS_MARK(k)
#endif

// ------------------------------------------------------------------------
// Sample: key = series >> 4 = 2 tile + half.  LDS: u16 pairs of keys.
__global__ __launch_bounds__(1024) void k_rsample(const uint32_t* __restrict__ series, size_t n, uint32_t S, uint32_t K,
                                                  uint32_t* __restrict__ kest) {
  extern __shared__ uint32_t c[];  // [(K + 1) / 2]
  RS_MARK(8)
  for (uint32_t i = threadIdx.x; i < (K + 1) / 2; i += 1024) c[i] = 0;
  __syncthreads();
  RS_MARK(9)
  const uint64_t m = n < RSAMPLE ? n : RSAMPLE;
  const uint64_t per = (m + RS_WG - 1) / RS_WG;
  const uint64_t k0 = blockIdx.x * per, k1 = k0 + per < m ? k0 + per : m;
  // evenly spaced single draws (runs of consecutive ids misjudge a structured stream,
  // e.g. C2's affine permutation), four per thread with their loads in flight together
  for (uint64_t kb = k0; kb < k1; kb += 4 * 1024) {
    uint32_t sv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t k = kb + threadIdx.x + 1024u * u;
      const uint64_t i = m == n ? k : k * n / m;
      sv[u] = k < k1 ? series[i < n ? i : 0] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (sv[u] < S) {
        const uint32_t key = sv[u] >> 4;
        atomicAdd(&c[key >> 1], (key & 1u) ? 0x10000u : 1u);
      }
  }
  __syncthreads();
  RS_MARK(10)
  for (uint32_t i = threadIdx.x; i < (K + 1) / 2; i += 1024) {
    const uint32_t x = c[i];
    if (x & 0xFFFFu) atomicAdd(&kest[2 * i], x & 0xFFFFu);
    if ((x >> 16) && 2 * i + 1 < K) atomicAdd(&kest[2 * i + 1], x >> 16);
  }
  RS_MARK(11)
}

// ------------------------------------------------------------------------
// Level-1 plan, one workgroup; thread j owns direct-bitmap word j -- tiles [32 j,
// 32 j + 32), F <= 32768 -- and bin j.  The key arrays are read coalesced (thread j
// loads tiles 2 q, 2 q + 1 for q = j + 1024 i) and turned around through LDS, one tile
// per word, each thread reading its 32 tiles from a rotated start (no bank
// conflicts).  (Round 5 loaded each thread's own 32 tiles: every wave-wide 16-B load
// touched 64 cache lines, and the loads took most of the kernel's 35 us.)  Direct
// tiles: the <= dmax tiles with the most estimated records, at least max(thr_min,
// 2^k), k the smallest power keeping <= dmax of them.
constexpr size_t RPLAN1_LDS = 32768 * 4;  // one word per tile
// Up to this many keys (C2, the smaller shards) the level-2 fix-up is one workgroup
// (k_rfix2s): 6 us against 2 x 5 us on C2.  (Planning their level-2 regions in k_rplan1
// too cost it 13 us, more than the two launches it saved: profiles/r06_plan_kernels.txt.)
constexpr uint32_t RFIX2_ONE_WG_MAX = 16384;
__global__ __launch_bounds__(1024) void k_rplan1(size_t n, uint32_t F, const uint32_t* __restrict__ kest,
                                                 const uint32_t* __restrict__ kprev, uint32_t* __restrict__ meta,
                                                 size_t cap32, size_t dlim16, uint32_t thr_min, uint32_t dmax,
                                                 uint32_t pct) {
  __shared__ uint32_t lh[33];
  __shared__ uint32_t sthr;
  __shared__ uint4 lds4[17];
  __shared__ uint64_t l64[17];
  __shared__ uint32_t dl[DIRECT_MAX + 1];
  __shared__ uint32_t capl[BIN1_BINS];
  extern __shared__ uint32_t tw[];  // [32768] a value per tile
  const MetaLayout L = meta_layout(F);
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t NW = (F + 31) / 32;
  const uint64_t m = n < RSAMPLE ? n : RSAMPLE;
  const bool exact = m == n;
  const double s = m ? (double)n / (double)m : 1.0;
  const uint32_t j = threadIdx.x, t0 = j * 32;
  const int lane = lane_id();
  RP_MARK(0)
  if (j < 33) lh[j] = 0;
  capl[j] = 0;
  // both key arrays, one 16-B load per tile pair (a ragged end word by word): the
  // estimates, then (once they are in LDS) the previous counts
  auto load_pairs = [&](const uint32_t* __restrict__ kw, uint4 (&x)[16]) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t t = 2u * (j + 1024u * (uint32_t)i);
      x[i] = make_uint4(0u, 0u, 0u, 0u);
      if (t + 1 < F) {
        x[i] = *reinterpret_cast<const uint4*>(kw + 2 * t);
      } else if (t < F) {
        x[i].x = kw[2 * t];
        x[i].y = kw[2 * t + 1];
      }
    }
  };
  uint2 te[16];  // tiles 2 q, 2 q + 1
  {
    uint4 x[16];
    load_pairs(kest, x);
#pragma unroll
    for (int i = 0; i < 16; ++i) te[i] = make_uint2(x[i].x + x[i].y, x[i].z + x[i].w);
  }
  auto scaled = [&](uint32_t v) -> uint32_t { return (uint32_t)fmin((double)v * s, 4294967295.0); };
  __syncthreads();  // lh cleared
  RP_MARK(1)
  // log2 histogram of the estimates; a wave whose counted tiles share one bin (C2: all
  // of them) adds once instead of 64 lanes on one LDS word
  auto hist = [&](uint32_t v) {
    const uint32_t e = scaled(v);
    const bool ok = dmax > 0 && e >= thr_min && e > 0;
    const int bin = ok ? 31 - __clz((int)e) : 0;
    const uint64_t act = __ballot(ok);
    if (!act) return;
    const int b0 = __builtin_amdgcn_readlane(bin, __builtin_ctzll(act));
    if (__ballot(ok && bin == b0) == act) {
      if (lane == 0) atomicAdd(&lh[b0], (uint32_t)__popcll(act));
    } else if (ok) {
      atomicAdd(&lh[bin], 1u);
    }
  };
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    hist(te[i].x);
    hist(te[i].y);
  }
  __syncthreads();
  if (j < 64) {  // the lowest k whose tiles of >= 2^k estimated records number <= dmax
    const uint32_t c = j < 32 ? lh[31 - j] : 0u;  // lane l: bin 31 - l
    const uint32_t cum = wave_incl_scan32(c);     // tiles in bins >= 31 - l
    const uint64_t ok = __ballot(dmax > 0 && j < 32 && cum <= dmax);
    // ok is a prefix of lanes (cum only grows): its length is the number of bins taken
    const int nb = __popcll(ok);
    if (j == 0) sthr = nb ? max(max(thr_min, 1u), 1u << (32 - nb)) : 0xFFFFFFFFu;
  }
  // the estimates turned around: thread j's 32 tiles from LDS
#pragma unroll
  for (int i = 0; i < 16; ++i) reinterpret_cast<uint2*>(tw)[j + 1024u * (uint32_t)i] = te[i];
  uint4 xp[16];
  load_pairs(kprev, xp);
  __syncthreads();
  const uint32_t thr = sthr;
  RP_MARK(2)
  uint32_t dbits = 0, E = 0;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const uint32_t kk = (uint32_t)(k + (int)j) & 31u;
    const uint32_t v = tw[t0 + kk];
    if (t0 + kk < F && scaled(v) >= thr) dbits |= 1u << kk;
    else E += v;
  }
  __syncthreads();  // every estimate read
#pragma unroll
  for (int i = 0; i < 16; ++i)
    reinterpret_cast<uint2*>(tw)[j + 1024u * (uint32_t)i] = make_uint2(xp[i].x + xp[i].y, xp[i].z + xp[i].w);
  __syncthreads();
  uint64_t P = 0;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const uint32_t kk = (uint32_t)(k + (int)j) & 31u;
    if (!((dbits >> kk) & 1u)) P += tw[t0 + kk];
  }
  RP_MARK(3)
  uint32_t cv[4] = {(uint32_t)__popc(dbits), 0u, 0u, 0u}, ct[4];
  block_excl_scan4<1024>(cv, lds4, ct);
  const uint32_t ND = ct[0];
  meta[L.dbits() + j] = j < NW ? dbits : 0u;
  meta[L.dpre() + j] = cv[0];
  {
    uint32_t x = dbits, di = cv[0];
    while (x) {
      const uint32_t k = (uint32_t)(__ffs((int)x) - 1);
      x &= x - 1u;
      dl[di] = t0 + k;
      meta[L.dlist() + di] = t0 + k;
      ++di;
    }
  }
  // a super-tile's two words are lanes j, j ^ 1 of one wave
  P += __shfl_xor(P, 1, 64);
  E += __shfl_xor(E, 1, 64);
  RP_MARK(4)
  // super-tile bins
  if ((j & 1u) == 0 && (j >> 1) < FS) {
    const uint32_t b = j >> 1;
    capl[b] = rcap((double)P, (double)E, s, exact, 256.0, 4, pct, 6.0, true);
    meta[L.btot() + b] = (uint32_t)min(P, (uint64_t)0xFFFFFFFFu);  // the bin's previous load, for k_rfix1
  }
  __syncthreads();  // dl complete
  RP_MARK(5)
  const uint32_t TB = FS + 2 * ND;
  if (j >= FS && j < TB) {  // direct half-bins
    const uint32_t t = dl[(j - FS) >> 1], h = (j - FS) & 1u;
    const double p = (double)kprev[2 * t + h], e = (double)kest[2 * t + h];
    capl[j] = rcap(p, e, s, exact, 256.0, 8, pct, 5.0, false);  // (u16 records: 16-B aligned regions)
  }
  __syncthreads();
  // two address spaces: super-tile bins in rec32, the direct half-bins in rec16 below
  // dlim16 (the rest of rec16 stays free for level 2's exact worst case)
  const bool stb = j < FS, dj = j >= FS && j < TB;
  uint64_t tot32, tot16;
  const uint64_t base32 = block_excl_scan64(stb ? (uint64_t)capl[j] : 0ull, l64, &tot32);
  const uint64_t base16 = block_excl_scan64(dj ? (uint64_t)capl[j] : 0ull, l64, &tot16);
  const uint64_t base = stb ? base32 : base16;
  const uint64_t lim = stb ? cap32 : dlim16;
  if (base + capl[j] + 16 > lim)  // past the space's end: clamped (its runs overflow; level 1 is redone exactly)
    capl[j] = base + 16 < lim ? (uint32_t)(lim - 16 - base) & (stb ? ~3u : ~7u) : 0u;
  meta[L.bbase() + j] = (uint32_t)base;
  meta[L.bcap() + j] = j < TB ? capl[j] : 0u;
  meta[L.bcnt() + j] = 0u;
  if (j == 0) {
    uint32_t* hdr = meta + L.hdr();
    hdr[H_ND] = ND;
    hdr[H_OV1] = 0;
    hdr[H_REDO1] = 0;
    hdr[H_OV2] = 0;
    hdr[H_REDO2] = 0;
    hdr[H_COUNT2] = 0;
    hdr[H_EXACT] = exact ? 1u : 0u;
    hdr[H_D16] = (uint32_t)min(tot16, (uint64_t)dlim16);  // level 2's regions follow the direct keys' (8-aligned)
  }
  RP_MARK(6)
}




// ------------------------------------------------------------------------
// Level 1, one 1024-thread workgroup per CU walking its slab in 16K-slot sub-chunks.
// Bins: the FS super-tiles (u32 records with the value, for level 2), two half-bins
// per direct tile (final u16 records: the sample is bucketized here, and its value
// added to an LDS sum of its series), and a trash bin (slots with no valid sample:
// the batch's ragged end, ids >= S) that is never written.  Per sub-chunk: one LDS
// atomic ranks each slot in its bin, one returning global atomic per non-empty bin
// reserves the sub-chunk's run in the bin's region, a block scan (one bin per thread)
// gives stage offsets and run ranks, the records are staged sorted (4 B each), and the stage is
// written out in order: each entry's run is the number of run heads at or before
// it -- a per-64-entry group prefix (gpre) plus a popcount of the group's bits of
// the run-head bitmap -- indexing the runs' destination deltas (rdelta[run] = run
// base - stage offset, or NODEST).  Runs below the first direct bin's rank are u32
// records (rec32), the others u16 (rec16).  The next sub-chunk's first half is loaded
// after B2, in flight through the scatter and write-out (bin1 3.89 -> 3.65 ms on C3,
// profiles/r04r_ab.txt, r04s_ab.txt).  A run that does not fit is dropped and flagged; pass 1 (the redo) exits unless k_rfix1 asked for it and adds nothing to
// sumfix or the error counter.
//
// Direct value sums: u64 per direct series in LDS, added to sumfix by each workgroup at
// the end of its slab.
//
// No LDS atomic of the ranking loop is under a branch that its return value or a
// uniform flag decides: the compiler then waits for each return before the next slot
// (s_waitcnt lgkmcnt(0) after every atomic).  Unconditional rank atomics and return-less
// u64 value sums keep a group's 8 atomics in flight together: bin1 3.56 -> 3.36 ms on C3
// (profiles/r05k_level1_atomics_ab.txt).  16 K-slot sub-chunks (16 slots per thread)
// leave the VGPRs for that (24 K spills the prefetch: 3.94 ms) and the LDS for the u64 sums.
//
// LDS (u32 words): stage[CH], cnt[1024], offr[1024] {offset | run rank << 16},
// rdelta[1024], heads[CH / 32], gpre[CH / 64] (u16), direct words [1024] uint2,
// lut2 [1024] uint2, direct sums [255 x 32] u64.
#ifdef L5DH_PHASES  // development (tools/mk_var.sh, tools/time_lib.py): per-workgroup phase times
__device__ unsigned long long g_phase1[1024 * 8];
__device__ unsigned long long g_phase3[1024 * 8];  // level 2
#define PH_INIT unsigned long long ph_acc[7] = {0, 0, 0, 0, 0, 0, 0}, ph_t = wall_clock64();
#define PH_VWAIT asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#define PH_MARK(k)                                 \
  if (threadIdx.x == 0) {                          \
    const unsigned long long ph_n = wall_clock64(); \
    ph_acc[k] += ph_n - ph_t;                      \
    ph_t = ph_n;                                   \
  }
#define PH_FLUSH                                                                   \
  if (threadIdx.x == 0 && pass == 0) {                                             \
    for (int k = 0; k < 7; ++k) g_phase1[blockIdx.x * 8 + k] += ph_acc[k];          \
    g_phase1[blockIdx.x * 8 + 7] += 1;                                             \
  }
#else
#define PH_INIT
#define PH_MARK(k)
#define PH_VWAIT
#define PH_FLUSH
#endif
// (nontemporal batch loads measured slower: bin2 +0.04 ms, round 5)
__device__ __forceinline__ uint4 ld_stream(const uint32_t* p) { return *reinterpret_cast<const uint4*>(p); }
constexpr int CHW = 16384;
using dsum_t = unsigned long long;
// rdelta of a dropped run: a valid delta (run base - stage offset) lies in (-CHW, cap16),
// cap16 < 2^32 - CHW - 1, so -(CHW + 1) never is one (0xFFFFFFFF is: base 0 at offset 1)
constexpr uint32_t NODEST = 0xFFFFFFFFu - (uint32_t)CHW;
constexpr int NT1 = 1024;  // 16 slots per thread
constexpr int DSUM_N = DIRECT_MAX * TILE;
constexpr size_t rbin1w_lds() {
  return (size_t)CHW * 4 + BIN1_BINS * 12 + CHW / 8 + CHW / 32 + 1024 * 8 + LUT2_N * 8 + DSUM_N * sizeof(dsum_t);
}

template <int NT, int CH>
__global__ __launch_bounds__(NT) void k_rbin1w(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                                  size_t n, size_t per, uint32_t S, uint32_t F, Tables tb,
                                                  uint32_t* __restrict__ meta, uint32_t* __restrict__ rec32,
                                                  uint16_t* __restrict__ rec16, int64_t* __restrict__ sumfix,
                                                  uint32_t* __restrict__ err, int vec, int pass) {
  constexpr int PT = CH / NT;  // slots per thread, loaded and ranked in halves
  constexpr int PH = PT / 2;
  constexpr int GS = 4;  // slots per group (a group's LDS lookups go out together)
  static_assert(PH % 4 == 0 && PH % GS == 0 && GS % 4 == 0 && CH <= 32768, "halves of whole 16-B groups; 15-bit ranks");
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* stage = smem;                                        // [CH] records, sorted by bin
  uint32_t* cnt = stage + CH;                                    // [BIN1_BINS]
  uint32_t* offr = cnt + BIN1_BINS;                              // [BIN1_BINS] stage offset | run rank << 16
  uint32_t* rdelta = offr + BIN1_BINS;                           // [BIN1_BINS] by run rank
  uint32_t* heads = rdelta + BIN1_BINS;                          // [CH / 32] run heads
  uint16_t* gpre = reinterpret_cast<uint16_t*>(heads + CH / 32);  // [CH / 64] runs before each 64-entry group
  uint2* dw = reinterpret_cast<uint2*>(gpre + CH / 64);          // [1024] {direct bits, direct tiles before}
  uint2* lut2 = dw + 1024;                                       // [LUT2_N]
  __shared__ uint32_t wsum[NT / 64];
  dsum_t* dsum = reinterpret_cast<dsum_t*>(lut2 + LUT2_N);       // [DSUM_N] direct series value sums
  const MetaLayout L = meta_layout(F);
  uint32_t* hdr = meta + L.hdr();
  if (pass == 1 && __builtin_amdgcn_readfirstlane(hdr[H_REDO1]) == 0u) return;
  uint32_t* bcnt = meta + L.bcnt();
  const uint32_t* bbase = meta + L.bbase();
  const uint32_t* bcap = meta + L.bcap();
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t NW = (F + 31) / 32;
  const uint32_t ND = hdr[H_ND];
  const uint32_t TB = FS + 2 * ND;
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  for (uint32_t w = threadIdx.x; w < NW; w += NT) dw[w] = make_uint2(meta[L.dbits() + w], meta[L.dpre() + w]);
  for (uint32_t b = threadIdx.x; b < BIN1_BINS; b += NT) cnt[b] = 0;
  for (uint32_t i = threadIdx.x; i < LUT2_N; i += NT) lut2[i] = tb.lut2[i];
  for (uint32_t i = threadIdx.x; i < ND * TILE; i += NT) dsum[i] = 0;
  __syncthreads();
  // (a batch piece holds < 2^30 samples: 32-bit sample indices)
  const uint32_t lo = (uint32_t)((size_t)blockIdx.x * per);
  const uint32_t hi = (uint32_t)min((size_t)lo + per, n);
  bool bad = false;
  // this thread's bins' regions (fixed for the launch): loaded once, not per sub-chunk
  constexpr int RB0 = (BIN1_BINS + NT - 1) / NT;
  uint32_t my_base[RB0], my_cap[RB0];
#pragma unroll
  for (int j = 0; j < RB0; ++j) {
    const uint32_t b = threadIdx.x + (uint32_t)j * NT;
    my_base[j] = b < TB ? bbase[b] : 0u;
    my_cap[j] = b < TB ? bcap[b] : 0u;
  }
  PH_INIT
  // the next sub-chunk's first half loaded during this one's scatter / write-out
  constexpr int PFG = PH / 4;  // prefetched 16-B groups per array
  uint4 pfs[PFG], pfv[PFG];
  auto prefetch = [&](uint32_t c) {
#pragma unroll
    for (int k = 0; k < PFG; ++k) {
      const uint32_t base = c + 4u * ((uint32_t)k * NT + threadIdx.x);
      pfs[k] = ld_stream(series + base);
      pfv[k] = ld_stream(reinterpret_cast<const uint32_t*>(values) + base);
    }
  };
  if (vec && lo + (uint32_t)CH <= hi) prefetch(lo);
  for (uint32_t c0 = lo; c0 < hi; c0 += CH) {
    for (uint32_t wd = threadIdx.x; wd < CH / 32; wd += NT) heads[wd] = 0u;
    // records are staged in slot order first (the stage is free until the scatter), so
    // only their ranks and bins stay in registers while the sub-chunk is ranked
    uint32_t pk[PT];  // [14:0] rank | [24:15] bin
    const bool full = vec && c0 + (uint32_t)CH <= hi;
    const uint32_t cl = c0;
    // the second half, issued once the first half's first group is ranked (in flight through
    // the rest of its ranking): bin1 3.25-3.30 -> 3.18 ms on C3 (issued before the first group,
    // or at the second half's start as in round 4, 3.36 / 3.25; profiles/r05w_second_half_ab.txt)
    uint4 hs[PH / 4], hv[PH / 4];
    auto load_second = [&]() {
      if (full) {
#pragma unroll
        for (int k = 0; k < PH / 4; ++k) {
          const uint32_t base = cl + 4u * ((uint32_t)(PH / 4 + k) * NT + threadIdx.x);
          hs[k] = ld_stream(series + base);
          hv[k] = ld_stream(reinterpret_cast<const uint32_t*>(values) + base);
        }
      }
    };
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1) { PH_MARK(1) }
      uint32_t sv[PH];
      float fv[PH];
      if (full) {
#pragma unroll
        for (int k = 0; k < PH / 4; ++k) {
          uint4 s4, u4;
          if (h == 0) {
            s4 = pfs[h * (PH / 4) + k];
            u4 = pfv[h * (PH / 4) + k];
          } else {
            s4 = hs[k];
            u4 = hv[k];
          }
          const float4 f4 = make_float4(__uint_as_float(u4.x), __uint_as_float(u4.y), __uint_as_float(u4.z),
                                        __uint_as_float(u4.w));
          sv[4 * k] = s4.x; sv[4 * k + 1] = s4.y; sv[4 * k + 2] = s4.z; sv[4 * k + 3] = s4.w;
          fv[4 * k] = f4.x; fv[4 * k + 1] = f4.y; fv[4 * k + 2] = f4.z; fv[4 * k + 3] = f4.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < PH; ++k) {
          const uint32_t i = c0 + 4u * ((uint32_t)(h * (PH / 4) + (k >> 2)) * NT + threadIdx.x) + (uint32_t)(k & 3);
          const bool in = i < hi;
          sv[k] = in ? series[i] : 0xFFFFFFFFu;
          fv[k] = in ? values[i] : 0.0f;
          bad |= in && sv[k] >= S;
        }
      }
      if (full) {  // (phase stamps: the half's loads -- and, on gfx9, every older store -- done)
        PH_VWAIT
        if (h == 0) { PH_MARK(0) } else { PH_MARK(2) }
      }
#pragma unroll
      for (int g = 0; g < PH; g += GS) {
        if (h == 0 && g == GS) load_second();
        uint32_t pl[GS];
        uint32_t escm = 0;
#pragma unroll
        for (int q = 0; q < GS; ++q) {
          // fast: +0 <= f < V_ESC, one integer compare of the bit pattern (-0, NaN and
          // (-1, 0) take the exact slow path, which also truncates them to 0)
          const float f = fv[g + q];
          const bool fast = __float_as_uint(f) < 0x49FFC000u;  // bits of (float)V_ESC
          pl[q] = fast ? (uint32_t)f : 0u;
          escm |= (!fast && sv[g + q] < S) ? (1u << q) : 0u;
          if (full) bad |= sv[g + q] >= S;
        }
        if (__ballot(escm != 0u)) {
          // one copy of the full search in the loop's code: slot q's sample is re-read
          // from the batch (an L2 hit; the 4 slots of a group are consecutive samples).
          // Picking it from the registers by a dynamic q made the compiler keep sv / fv
          // in scratch: 24 scratch stores per thread per sub-chunk, each behind a wait
          // for its load, on every sub-chunk (round 5).
#pragma unroll 1
          for (int q = 0; q < GS; ++q) {
            if ((escm >> q) & 1u) {
              const uint32_t i = cl + 4u * ((uint32_t)(h * (PH / 4) + (g + q) / 4) * NT + threadIdx.x) + (uint32_t)(q & 3);
              const uint32_t r = payload1_slow(series[i], values[i], tb, pass == 0 ? sumfix : nullptr);
#pragma unroll
              for (int u = 0; u < GS; ++u) pl[u] = q == u ? r : pl[u];
            }
          }
        }
        uint2 dv[GS], lv[GS];
#pragma unroll
        for (int q = 0; q < GS; ++q) dv[q] = dw[(sv[g + q] >> (TILE_SHIFT + 5)) & 1023u];  // (any word when s >= S)
#pragma unroll
        // the bucket LUT, read by every slot: issued with the dw reads instead of behind them
        // (only a direct slot uses it; reading it under the direct bit waited for dw first:
        // bin1 3.31 -> 3.25 ms on C3, C2 unchanged, round 5)
        for (int q = 0; q < GS; ++q) lv[q] = lut2[lut2_index(pl[q])];
        uint32_t rc4[GS];
#pragma unroll
        for (int q = 0; q < GS; ++q) {
          const uint32_t s = sv[g + q];
          const uint32_t tw = __builtin_amdgcn_ubfe(s, TILE_SHIFT, 5);
          const bool direct = s < S && __builtin_amdgcn_ubfe(dv[q].x, tw, 1) != 0u;
          const uint32_t di = dv[q].y + (uint32_t)__popc(__builtin_amdgcn_ubfe(dv[q].x, 0, tw));
          const uint32_t p = pl[q];
          uint32_t o;
          const uint32_t bk = lut2_decode(p, lv[q], o);
          const bool esc = p >= V_ESC;
          const uint32_t bucket = sel_u32(esc, p - V_ESC, bk);
          rc4[q] = sel_u32(direct, ((s & (TILE - 1)) << 11) | bucket, ((s & (ST_TILES * TILE - 1)) << 21) | p);
          const uint32_t dbin = FS + 2u * di + ((s >> 4) & 1u);
          const uint32_t bn = sel_u32(s < S, sel_u32(direct, dbin, s >> ST_SHIFT), TB);
          pk[h * PH + g + q] = atomicAdd(cnt + bn, 1u) | (bn << 15);
          // the direct series' value sum (u64: no wrap to check, so nothing reads the return)
          if (direct && !esc && pass == 0 && p) atomicAdd(&dsum[di * TILE + (s & (TILE - 1))], (dsum_t)p);
        }
        // slots 4 (kk NT + thread) + q of the 16-B group kk, as loaded
#pragma unroll
        for (int j = 0; j < GS / 4; ++j)
          *reinterpret_cast<uint4*>(stage + 4u * ((uint32_t)(h * (PH / 4) + g / 4 + j) * NT + threadIdx.x)) =
              make_uint4(rc4[4 * j], rc4[4 * j + 1], rc4[4 * j + 2], rc4[4 * j + 3]);
        asm volatile("" ::: "memory");  // keep the groups apart (bounded register pressure)
      }
    }
    __syncthreads();  // B1: counts complete
    PH_MARK(3)
    // run reservations: thread t -> bins t, t + NT, ... (the trash bin TB gets none)
    constexpr int RB = (BIN1_BINS + NT - 1) / NT;
    uint32_t rn[RB], rold[RB], rbase[RB], rcapv[RB];
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const uint32_t rb_bin = threadIdx.x + (uint32_t)j * NT;
      rn[j] = rb_bin <= TB ? cnt[rb_bin] : 0u;  // records of the bin in this sub-chunk
      rold[j] = 0;
      rbase[j] = my_base[j];
      rcapv[j] = my_cap[j];
      if (rb_bin < TB && rn[j]) rold[j] = atomicAdd(&bcnt[rb_bin], rn[j]);
    }
    {  // stage offsets and run ranks: a block scan of {count, non-empty} (one bin per thread), run heads
      static_assert(NT == BIN1_BINS && RB == 1, "one bin per thread");
      const uint32_t pv = rn[0] | ((rn[0] ? 1u : 0u) << 16);  // (counts sum to <= CH < 2^16: no carry)
      const uint32_t wi = wave_incl_scan32(pv);
      if (lane == 63) wsum[wv] = wi;
      __syncthreads();  // B1b: wave totals
      uint32_t pre = 0;
      for (int q = 0; q < wv; ++q) pre += wsum[q];
      const uint32_t ex = pre + wi - pv;
      offr[threadIdx.x] = ex;  // offset | run rank << 16
      if (rn[0]) atomicOr(&heads[(ex & 0xFFFFu) >> 5], 1u << (ex & 31u));
    }
    uint32_t rec[PT];  // this thread's records, in slot order (read before any is scattered)
#pragma unroll
    for (int kk = 0; kk < PT / 4; ++kk) {
      const uint4 v = *reinterpret_cast<const uint4*>(stage + 4u * ((uint32_t)kk * NT + threadIdx.x));
      rec[4 * kk] = v.x; rec[4 * kk + 1] = v.y; rec[4 * kk + 2] = v.z; rec[4 * kk + 3] = v.w;
    }
    __syncthreads();  // B2: offsets, run ranks, heads; every slot-order record read
    PH_MARK(4)
    // (after B2: the run reservations' returns and the scan never wait behind these loads)
    if (vec && c0 + 2u * (uint32_t)CH <= hi) prefetch(c0 + (uint32_t)CH);
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t bin = (pk[k] >> 15) & 1023u;
      stage[(offr[bin] & 0xFFFFu) + (pk[k] & 0x7FFFu)] = rec[k];
    }
    if (wv == 0) {  // runs before group g = run heads in the groups before it (one wave: a scan of popcounts)
      constexpr int GPL = CH / 64 / 64;  // groups per lane
      static_assert(GPL % 2 == 0, "two groups per 16-B read");
      uint32_t pc[GPL], t = 0;
#pragma unroll
      for (int k = 0; k < GPL; k += 2) {
        const uint4 w = *reinterpret_cast<const uint4*>(heads + 2u * (GPL * (uint32_t)lane + (uint32_t)k));
        pc[k] = (uint32_t)(__popc(w.x) + __popc(w.y));
        pc[k + 1] = (uint32_t)(__popc(w.z) + __popc(w.w));
        t += pc[k] + pc[k + 1];
      }
      uint32_t ex = wave_incl_scan32(t) - t;
#pragma unroll
      for (int k = 0; k < GPL; ++k) {
        gpre[GPL * (uint32_t)lane + (uint32_t)k] = (uint16_t)ex;
        ex += pc[k];
      }
    }
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const uint32_t rb_bin = threadIdx.x + (uint32_t)j * NT;
      if (rn[j]) {
        uint32_t d = NODEST;
        if (rb_bin < TB) {
          if (rold[j] + rn[j] <= rcapv[j]) d = rbase[j] + rold[j] - (offr[rb_bin] & 0xFFFFu);
          else hdr[H_OV1] = 1u;  // this run is dropped; k_rfix1 has the batch redone with exact regions
        }
        rdelta[offr[rb_bin] >> 16] = d;
      }
    }
    __syncthreads();  // B3: stage, group prefixes, deltas (every count read: cleared below)
    PH_MARK(5)
    const uint32_t nst = offr[FS] >> 16;  // runs of super-tile bins (u32 records); the later runs are u16
#pragma unroll
    for (int j = 0; j < RB; ++j)
      if (threadIdx.x + (uint32_t)j * NT < BIN1_BINS) cnt[threadIdx.x + (uint32_t)j * NT] = 0;
#pragma unroll 4
    for (int k = 0; k < PT; ++k) {  // all CH entries, in sorted order (each wave a contiguous PT x 64 range)
      const uint32_t i = (uint32_t)wv * (PT * 64) + (uint32_t)k * 64 + (uint32_t)lane;
      const uint32_t g = i >> 6;  // (wave-uniform)
      const unsigned long long hw = *reinterpret_cast<const unsigned long long*>(heads + 2 * g);
      // run heads at or before this lane: those below it (mbcnt) + its own bit
      const uint32_t run = (uint32_t)gpre[g] + mask_below(hw) + (uint32_t)((hw >> lane) & 1ull) - 1u;
      const uint32_t d = rdelta[run];
      if (d != NODEST) {
        if (run < nst)
          rec32[i + d] = stage[i];
        else
          rec16[i + d] = (uint16_t)stage[i];
      }
    }
    __syncthreads();  // B4
    PH_MARK(6)
  }
  PH_FLUSH
  if (pass == 0) {
    // the slab's direct value sums (every wave's adds are in: the last barrier) into sumfix
    const uint32_t* dl = meta + L.dlist();
    for (uint32_t i = threadIdx.x; i < ND * TILE; i += NT) {
      const unsigned long long v = dsum[i];
      const uint32_t s = dl[i / TILE] * TILE + (i & (TILE - 1));
      if (v && s < S) atomicAdd(reinterpret_cast<unsigned long long*>(&sumfix[s]), (unsigned long long)v);
    }
    if (bad) atomicAdd(err, 1u);  // monotonic: the host compares it with the count it already reported
  }
}

// lut3: byte offset of key v's entry (v < 2^21; the lut2 intervals), and its bucket
__device__ __forceinline__ uint32_t lut3_byte(uint32_t v) {
  const uint32_t sh = 25u - (uint32_t)__builtin_clz(v | 64u);
  return ((v >> sh) + (sh << 6)) << 3;
}
__device__ __forceinline__ uint32_t lut3_bucket(uint32_t v, uint2 x) {
  return (x.x & 0x7FFu) + (((v << 11) | 0x7FFu) >= x.x ? 1u : 0u) + (v >= x.y ? 1u : 0u);
}

// ------------------------------------------------------------------------
// After level 1 (one workgroup, thread = bin): exact bin totals, the direct keys'
// ranges, and on an overflow exact regions for the redo pass (super-tile bins in
// rec32, direct half-bins in rec16 from 0), and the level-2 items per super-tile.
__global__ __launch_bounds__(1024) void k_rfix1(uint32_t F, uint32_t* __restrict__ meta, const uint32_t* __restrict__ err,
                                                uint32_t* __restrict__ err_host) {
  __shared__ uint32_t lds[17];
  const MetaLayout L = meta_layout(F);
  uint32_t* hdr = meta + L.hdr();
  if (threadIdx.x == 0) *reinterpret_cast<volatile uint32_t*>(err_host) = *err;  // to the host's mapped word
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t ND = hdr[H_ND];
  const uint32_t TB = FS + 2 * ND;
  const uint32_t ov = hdr[H_OV1];
  const uint32_t b = threadIdx.x;
  const bool stb = b < FS, dj = b >= FS && b < TB;
  const uint32_t c = b < TB ? meta[L.bcnt() + b] : 0u;
  // A super-tile whose records outgrew the bound its keys' level-2 regions were sized
  // by (their previous counts +1/16 + 4 sigma; k_rplan1 left that count in btot): its
  // load moved, or this is a first interval.  Its keys' regions (sampled at ~1 draw
  // per key) would overflow, so level 2's first pass only counts, and the second
  // writes into exact regions -- not a whole pass written, dropped and redone.
  if (stb && !hdr[H_EXACT]) {
    const double P = (double)meta[L.btot() + b];
    if ((double)c > P * 1.0625 + 4.0 * sqrt(P) + 256.0) hdr[H_COUNT2] = 1u;
  }
  meta[L.btot() + b] = c;
  uint32_t t32, t16;
  const uint32_t nb32 = block_excl_scan<1024>(stb ? round_up(c, 4) : 0u, lds, &t32);
  const uint32_t nb16 = block_excl_scan<1024>(dj ? round_up(c, 8) : 0u, lds, &t16);
  const uint32_t nb = stb ? nb32 : nb16;
  const uint32_t base = ov ? nb : meta[L.bbase() + b];
  if (dj) {
    const uint32_t t = meta[L.dlist() + ((b - FS) >> 1)], h = (b - FS) & 1u;
    meta[L.kbase() + 2 * t + h] = base;
    meta[L.kcnt() + 2 * t + h] = c;
  }
  if (ov) {
    meta[L.bbase() + b] = nb;
    meta[L.bcap() + b] = round_up(c, stb ? 4 : 8);
    meta[L.bcnt() + b] = 0u;
  }
  // A redo lays the direct keys out exactly from 0; past the space planned for them
  // (H_D16) they overlap level 2's planned regions: then level 2's first pass only
  // counts (every region emptied: its runs overflow) and its redo lays the regions
  // out exactly above the direct keys' new end.
  const uint32_t d16 = hdr[H_D16];
  if (ov && t16 > d16) {
    for (uint32_t k = b; k < L.K; k += 1024)
      if (!((meta[L.dbits() + (k >> 6)] >> ((k >> 1) & 31u)) & 1u)) meta[L.kcap() + k] = 0u;
  }
  // level-2 items: ITEM2 level-1 records of a super-tile's region (k_rbin2 finds an
  // item's super-tile in istart); the totals are exact either way
  uint32_t all;
  const uint32_t is = block_excl_scan<1024>(stb ? (c + ITEM2 - 1) / ITEM2 : 0u, lds, &all);
  if (stb) meta[L.istart() + b] = is;
  __syncthreads();  // every thread has read H_OV1
  if (b == 0) {
    meta[L.istart() + FS] = all;
    hdr[H_ITEMS] = all;
    if (ov && t16 > d16) {
      hdr[H_D16] = t16;
      hdr[H_COUNT2] = 1u;
    }
    hdr[H_OV2] = 0u;
    hdr[H_REDO2] = 0u;
    hdr[H_REDO1] = ov;
    hdr[H_OV1] = 0u;
    if (ov) hdr[H_NOVR1] += 1u;
  }
}

// ------------------------------------------------------------------------
__device__ __forceinline__ bool tile_direct(const uint32_t* __restrict__ meta, const MetaLayout& L, uint32_t t) {
  return (meta[L.dbits() + (t >> 5)] >> (t & 31u)) & 1u;
}

// The sum of the u64 per-workgroup partials before workgroup b (b <= 64).
__device__ __forceinline__ uint64_t wsum_before(const uint64_t* __restrict__ ws, uint32_t b, uint64_t* red /*[16]*/) {
  uint64_t v = threadIdx.x < b ? ws[threadIdx.x] : 0ull;
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t r = 0;
  for (int q = 0; q < 16; ++q) r += red[q];
  __syncthreads();
  return r;
}

// Level-2 regions over ceil(2F / 1024) workgroups, key k = 1024 b + thread (coalesced):
// k_rplan2a sizes the regions of the non-direct keys (the previous batch's exact
// counts and this batch's sample; zeroes the sample for the next batch) and sums them
// per workgroup; k_rplan2b adds the earlier workgroups' sums, scans, and clamps a region
// that would pass the buffer's end (its runs overflow; level 2 is redone exactly).
// Regions start at H_D16 (above the direct keys' space), so they are planned with the
// direct tiles, before level 1.
__global__ __launch_bounds__(1024) void k_rplan2a(size_t n, uint32_t F, uint32_t* __restrict__ kest,
                                                  const uint32_t* __restrict__ kprev, uint32_t* __restrict__ meta,
                                                  uint32_t pct) {
  __shared__ uint64_t red[16];
  const MetaLayout L = meta_layout(F);
  const uint64_t m = n < RSAMPLE ? n : RSAMPLE;
  const bool exact = m == n;
  const double s = m ? (double)n / (double)m : 1.0;
  const uint32_t k = blockIdx.x * 1024u + threadIdx.x;
  uint32_t cap = 0;
  if (k < L.K) {
    const uint32_t e = kest[k];
    if (e) kest[k] = 0;  // ready for the next batch
    if (!tile_direct(meta, L, k >> 1)) {
      cap = rcap((double)kprev[k], (double)e, s, exact, 32.0, 8, pct, 5.0, false);
      meta[L.kcap() + k] = cap;
    }
  }
  const uint64_t w = wave_sum((uint64_t)cap);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int q = 0; q < 16; ++q) t += red[q];
    reinterpret_cast<uint64_t*>(meta + L.wsum())[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(1024) void k_rplan2b(uint32_t F, uint32_t* __restrict__ meta, size_t cap16) {
  __shared__ uint64_t red[16];
  __shared__ uint64_t l64[17];
  const MetaLayout L = meta_layout(F);
  uint32_t* hdr = meta + L.hdr();
  const uint64_t before = wsum_before(reinterpret_cast<const uint64_t*>(meta + L.wsum()), blockIdx.x, red);
  const uint32_t k = blockIdx.x * 1024u + threadIdx.x;
  const bool mine = k < L.K && !tile_direct(meta, L, k >> 1);
  uint32_t cap = mine ? meta[L.kcap() + k] : 0u;
  uint64_t total;
  const uint64_t base = hdr[H_D16] + before + block_excl_scan64((uint64_t)cap, l64, &total);
  if (mine) {
    if (base + cap + 64 > cap16) {  // clamped: level 2's first pass only counts (k_rbin2)
      cap = base + 64 < cap16 ? (uint32_t)(cap16 - 64 - base) & ~7u : 0u;
      hdr[H_COUNT2] = 1u;
    }
    meta[L.kbase() + k] = (uint32_t)base;
    meta[L.kcap() + k] = cap;
    meta[L.kcnt() + k] = 0u;
  }
}

// ------------------------------------------------------------------------
// Level 2 (persistent, two 512-thread workgroups per CU): workgroup w walks items
// [w I / G, (w + 1) I / G) -- item order is super-tile order, so a workgroup sees
// few super-tiles and folds the value sums of one super-tile's 2048 series in LDS
// (u64), flushed to sumfix when it moves on.  Per item (<= ITEM2 level-1 records,
// 12 per thread): bucket (LUT), 16-bit record, key = 2 tile-in-ST + half; LDS
// counting sort by key, one returning global atomic per non-empty key on its
// cursor, stage {rec16 | key << 16}, written in order to run base + position.
// Software pipeline, so no global latency is waited for in the item loop: the
// next item's records are loaded while this one is processed, and the stage and
// run offsets are double-buffered -- item i's cursor atomics are issued before its
// scatter and the write-out of item i - 1, and read after them.
constexpr int B2_KEYS = 2 * ST_TILES;
// two 512-thread workgroups per CU (74.5 KB of LDS each), so one's barrier-separated
// phases overlap the other's: level 2 -1.4 % on C3, -10 % on C2 against one 1024-thread
// workgroup with 16 K-record items (profiles/r04p_ab.txt)
constexpr int B2_NT = 512, B2_PER_CU = 2;
constexpr size_t rbin2_lds() {
  return 2048 * 8 + LUT2_N * 8 + 2 * B2_KEYS * 8 + (B2_KEYS + 64) * 4 + 2 * (size_t)ITEM2 * 4;
}

template <int NT>
__global__ __launch_bounds__(NT, B2_PER_CU * NT / 256) void k_rbin2(uint32_t S, uint32_t F, Tables tb, uint32_t* __restrict__ meta,
                                                 const uint32_t* __restrict__ m_is, const uint32_t* __restrict__ m_bb,
                                                 const uint32_t* __restrict__ m_bt,
                                                 const uint32_t* __restrict__ rec32, uint16_t* __restrict__ rec16,
                                                 int64_t* __restrict__ sumfix, int pass) {
  // m_is [FS + 1] first item of each super-tile, m_bb level-1 region base, m_bt
  // level-1 records: words of `meta` this kernel only reads (wave-uniform: scalar loads)
  constexpr int PT = (int)ITEM2 / NT;
  constexpr int PG = PT / 4;  // 16-B groups per thread
  __shared__ __attribute__((aligned(16))) uint32_t smem[rbin2_lds() / 4];  // (static: constant LDS addresses)
  unsigned long long* lsum = reinterpret_cast<unsigned long long*>(smem);  // [2048]
  uint2* lut3 = reinterpret_cast<uint2*>(lsum + 2048);                     // [LUT2_N]
  uint2* ocx = lut3 + LUT2_N;                                              // [2][B2_KEYS] {stage offset, run base}
  uint32_t* cnt = reinterpret_cast<uint32_t*>(ocx + 2 * B2_KEYS);          // [B2_KEYS + 64]: a spare per lane
  uint32_t* stage = cnt + B2_KEYS + 64;                                    // [2][ITEM2] {rec16 | key << 16}, sorted
  const MetaLayout L = meta_layout(F);
  uint32_t* hdr = meta + L.hdr();
  if (pass == 1 && __builtin_amdgcn_readfirstlane(hdr[H_REDO2]) == 0u) return;
  const uint32_t nitems = hdr[H_ITEMS];
  const uint32_t i0 = (uint32_t)(((uint64_t)blockIdx.x * nitems) / gridDim.x);
  const uint32_t i1 = (uint32_t)(((uint64_t)(blockIdx.x + 1) * nitems) / gridDim.x);
  if (i0 >= i1) return;
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  uint32_t* kcnt = meta + L.kcnt();
  const uint32_t* kbase = meta + L.kbase();
  const uint32_t* kcap = meta + L.kcap();
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < LUT2_N; i += NT) lut3[i] = tb.lut3[i];
  for (int i = threadIdx.x; i < 2048; i += NT) lsum[i] = 0ull;
  for (int i = threadIdx.x; i < B2_KEYS; i += NT) cnt[i] = 0u;
  // super-tile of the first item: the last j with istart[j] <= i0 (empty super-tiles
  // share their successor's start)
  uint32_t jl = 0, jh = FS;  // istart[jl] <= i0 < istart[jh]
  while (jh - jl > 1) {
    const uint32_t mid = (jl + jh) >> 1;
    if (m_is[mid] <= i0) jl = mid; else jh = mid;
  }
  __syncthreads();
  // item -> [a, e) of its super-tile's level-1 region (a is 4-aligned)
  uint32_t jn = jl;
  auto item_range = [&](uint32_t item, uint32_t& j, uint32_t& a, uint32_t& e) {
    while (m_is[jn + 1] <= item) jn = __builtin_amdgcn_readfirstlane(jn + 1);
    j = jn;
    const uint32_t bb = m_bb[jn];
    a = bb + (item - m_is[jn]) * ITEM2;
    e = min(a + ITEM2, bb + m_bt[jn]);
  };
  // unconditional loads (a group past the item's end reloads its first group), so all
  // of them stay in flight; records past the end are masked where they are used
  auto load = [&](uint32_t a, uint32_t e, uint4 (&x)[PG]) {
#pragma unroll
    for (int g = 0; g < PG; ++g) {
      const uint32_t idx = a + 4u * ((uint32_t)g * NT + threadIdx.x);
      x[g] = *reinterpret_cast<const uint4*>(rec32 + (idx < e ? idx : a));
    }
  };
  uint32_t cur_j = 0xFFFFFFFFu;
  auto flush = [&](uint32_t jj) {  // the super-tile's value sums into sumfix (one atomic per nonzero series)
    for (int i = threadIdx.x; i < 2048; i += NT) {
      const unsigned long long v = lsum[i];
      const uint32_t s = jj * 2048u + (uint32_t)i;
      if (v && s < S) atomicAdd(reinterpret_cast<unsigned long long*>(&sumfix[s]), v);
      lsum[i] = 0ull;
    }
  };
  // Count-only first pass (H_COUNT2: k_rplan2b clamped a region, or k_rfix1 saw a
  // super-tile outgrow its keys' regions): the keys' exact counts and the value sums --
  // no bucket, stage or write-out, non-returning atomics; k_rfix2 then lays the regions
  // out exactly and the second pass writes them.
  if (pass == 0 && __builtin_amdgcn_readfirstlane(hdr[H_COUNT2]) != 0u) {
    uint32_t j, a, e;
    item_range(i0, j, a, e);
    uint4 x[PG];
    load(a, e, x);
    for (uint32_t item = i0; item < i1; ++item) {
      const uint32_t cj = j, ctot = e - a;
      uint4 xn[PG];
      if (item + 1 < i1) item_range(item + 1, j, a, e);
      load(a, e, xn);
      if (cj != cur_j) {
        if (cur_j != 0xFFFFFFFFu) {
          __syncthreads();
          flush(cur_j);
        }
        cur_j = cj;
        __syncthreads();
      }
#pragma unroll
      for (int g = 0; g < PG; ++g) {
        const uint32_t rr[4] = {x[g].x, x[g].y, x[g].z, x[g].w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t p = rr[q] & 0x1FFFFFu;
          const bool valid = 4u * ((uint32_t)g * NT + threadIdx.x) + (uint32_t)q < ctot;
          atomicAdd(&cnt[valid ? rr[q] >> 25 : (uint32_t)B2_KEYS + (uint32_t)lane], 1u);
          atomicAdd(&lsum[(rr[q] >> 21) & 2047u], (unsigned long long)((valid && p < V_ESC) ? p : 0u));
        }
      }
      __syncthreads();
      if (wv < 2) {
        const uint32_t rk = (uint32_t)wv * 64u + (uint32_t)lane;
        const uint32_t rc = cnt[rk];
        if (rc) atomicAdd(&kcnt[cj * (uint32_t)B2_KEYS + rk], rc);
        cnt[rk] = 0u;
      }
      __syncthreads();
#pragma unroll
      for (int g = 0; g < PG; ++g) x[g] = xn[g];
    }
    __syncthreads();
    flush(cur_j);
    return;
  }
  // write-out of a sorted stage (each wave a contiguous range)
  // (in batches of 4 entries whose LDS reads go out together: entries past the end are
  // read too -- stale stage words, their key masked into range -- and not stored)
  auto write_out = [&](int bb, uint32_t total) {
    const uint32_t* st = stage + bb * ITEM2;
    const uint2* oc = ocx + bb * B2_KEYS;
    constexpr int WB = 4;
#pragma unroll
    for (int k0 = 0; k0 < PT; k0 += WB) {
      uint32_t x[WB];
      uint2 o[WB];
#pragma unroll
      for (int j = 0; j < WB; ++j) x[j] = st[(uint32_t)wv * (PT * 64) + (uint32_t)(k0 + j) * 64 + (uint32_t)lane];
#pragma unroll
      for (int j = 0; j < WB; ++j) o[j] = oc[(x[j] >> 16) & (B2_KEYS - 1)];
#pragma unroll
      for (int j = 0; j < WB; ++j) {
        const uint32_t i = (uint32_t)wv * (PT * 64) + (uint32_t)(k0 + j) * 64 + (uint32_t)lane;
        if (i < total && o[j].y != INVALID) rec16[o[j].y + (i - o[j].x)] = (uint16_t)(x[j] & 0xFFFFu);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  uint32_t j, a, e;
  item_range(i0, j, a, e);
  uint4 x[PG];
  load(a, e, x);
  uint32_t prev_total = 0;
#ifdef L5DH_PHASES
  unsigned long long ph2[5] = {0, 0, 0, 0, 0}, ph2_t = wall_clock64();
#define PH2_MARK(k)                                  \
  if (threadIdx.x == 0) {                            \
    const unsigned long long ph_n = wall_clock64();  \
    ph2[k] += ph_n - ph2_t;                          \
    ph2_t = ph_n;                                    \
  }
#else
#define PH2_MARK(k)
#endif
  for (uint32_t item = i0; item < i1; ++item) {
    const int b = (int)(item & 1u);
    const uint32_t cj = j, ctot = e - a;
    // (A) the next item's records in flight (after the last item: this item's again,
    // unconditionally, so that no copy of the registers waits for the loads)
    uint4 xn[PG];
    if (item + 1 < i1) item_range(item + 1, j, a, e);
    load(a, e, xn);
    if (cj != cur_j) {
      if (pass == 0 && cur_j != 0xFFFFFFFFu) {
        __syncthreads();  // every lane's sums of the previous super-tile are in
        flush(cur_j);
      }
      cur_j = cj;
      __syncthreads();
    }
    // (B) bucket, 16-bit record, key; rank in the key's count; value sums
    uint32_t kr[PT], rank[PT];
    {
      uint32_t r[PT];
#pragma unroll
      for (int g = 0; g < PG; ++g) {
        r[4 * g] = x[g].x; r[4 * g + 1] = x[g].y; r[4 * g + 2] = x[g].z; r[4 * g + 3] = x[g].w;
      }
      // A whole item with no escaped record in the wave (nearly every item) takes the lean
      // form: key = r >> 25 (tile in super-tile, half), lsum index = r >> 21 (tile, series),
      // the bucket from lut3, no validity or escape selects (round 5's form issued ~45 VALU
      // instructions per record).  The careful form (the item's ragged end, escapes, the
      // redo pass): the rank and value-sum atomics carry no control flow -- an invalid slot
      // counts into a spare word of its lane and every slot adds to a sum (0 when it has
      // nothing to add) -- so the atomics of consecutive slots stay in flight together.
      bool escq = false;
#pragma unroll
      for (int k = 0; k < PT; ++k) escq |= (r[k] & 0x1FFFFFu) >= V_ESC;
      const bool lean = ctot == ITEM2 && pass == 0 && !__ballot(escq);
      constexpr int H = PT / 2;  // LUT reads batched per half
      if (lean) {
#pragma unroll
        for (int k = 0; k < PT; ++k) {
          uint2 lv[H];
          if (k % H == 0) {
#pragma unroll
            for (int q = 0; q < H; ++q) lv[q] = lut3[lut3_byte(r[k + q] & 0x1FFFFFu) >> 3];
          }
          const uint32_t p = r[k] & 0x1FFFFFu;
          kr[k] = ((r[k] >> 25) << 16) | ((r[k] >> 10) & 0xF800u) | lut3_bucket(p, lv[k % H]);
          rank[k] = atomicAdd(&cnt[r[k] >> 25], 1u);
          atomicAdd(&lsum[(r[k] >> 21) & 2047u], (unsigned long long)p);
        }
      } else {
#pragma unroll
        for (int k = 0; k < PT; ++k) {
          uint2 lv[H];
          if (k % H == 0) {
#pragma unroll
            for (int q = 0; q < H; ++q) lv[q] = lut3[lut3_byte(r[k + q] & 0x1FFFFFu) >> 3];
          }
          const uint32_t p = r[k] & 0x1FFFFFu;
          const bool esc = p >= V_ESC;
          const uint32_t bucket = sel_u32(esc, p - V_ESC, lut3_bucket(p, lv[k % H]));
          const bool valid = 4u * ((uint32_t)(k >> 2) * NT + threadIdx.x) + (uint32_t)(k & 3) < ctot;
          kr[k] = valid ? (((r[k] >> 25) << 16) | ((r[k] >> 10) & 0xF800u) | bucket) : NOKEY;
          rank[k] = atomicAdd(&cnt[valid ? r[k] >> 25 : (uint32_t)B2_KEYS + (uint32_t)lane], 1u);
          atomicAdd(&lsum[(r[k] >> 21) & 2047u], (unsigned long long)((pass == 0 && valid && !esc) ? p : 0u));
        }
      }
    }
    __syncthreads();  // B1: counts complete
    PH2_MARK(0)
    // (C) run reservations (waves 0 and 1, lane = key; results read in (F)); wave 2
    // scans the counts into this item's stage offsets
    uint32_t rc = 0, rold = 0, rbase = 0, rcapv = 0;
    const uint32_t rk = (uint32_t)wv * 64u + (uint32_t)lane;
    if (wv < 2) {
      const uint32_t gk = cj * (uint32_t)B2_KEYS + rk;
      rc = cnt[rk];
      if (rc) {
        rold = atomicAdd(&kcnt[gk], rc);
        rbase = kbase[gk];
        rcapv = kcap[gk];
      }
    } else if (wv == 2) {
      const uint32_t c0 = cnt[2 * lane], c1 = cnt[2 * lane + 1];
      const uint32_t ex = wave_incl_scan32(c0 + c1) - (c0 + c1);
      ocx[b * B2_KEYS + 2 * lane].x = ex;
      ocx[b * B2_KEYS + 2 * lane + 1].x = ex + c0;
    }
    __syncthreads();  // B2: stage offsets visible; every count read
    PH2_MARK(1)
    // (D) scatter this item into its stage
    {
      uint32_t* st = stage + b * ITEM2;
      const uint2* oc = ocx + b * B2_KEYS;
      // (offset reads of 4 slots together, then their stores: the compiler cannot move a
      // read of ocx above a store to the stage, so a read-store pair per slot waited on
      // every read)
#pragma unroll
      for (int k0 = 0; k0 < PT; k0 += 4) {
        uint32_t o[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = oc[(kr[k0 + j] >> 16) & (B2_KEYS - 1)].x;
        // (an invalid slot's record goes to its lane's spare counter word -- written by
        // nothing else in this phase, read by nothing -- instead of a branch per slot)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          *(kr[k0 + j] != NOKEY ? &st[o[j] + rank[k0 + j]] : &cnt[B2_KEYS + lane]) = kr[k0 + j];
      }
    }
    PH2_MARK(2)
    // (E) write-out of the previous item (its stage and run offsets are complete)
    if (item > i0) write_out(b ^ 1, prev_total);
    PH2_MARK(3)
    // (F) this item's run bases; counts cleared for the next item
    if (wv < 2) {
      uint32_t rb = INVALID;
      if (rc) {
        if (rold + rc <= rcapv) rb = rbase + rold;
        else hdr[H_OV2] = 1u;  // dropped; k_rfix2 has level 2 redone with exact regions
      }
      ocx[b * B2_KEYS + rk].y = rb;
      cnt[rk] = 0u;
    }
    __syncthreads();  // B3
    PH2_MARK(4)
    prev_total = ctot;
#pragma unroll
    for (int g = 0; g < PG; ++g) x[g] = xn[g];
  }
  write_out((int)((i1 - 1) & 1u), prev_total);
  __syncthreads();
  if (pass == 0) flush(cur_j);
#ifdef L5DH_PHASES
  if (threadIdx.x == 0 && pass == 0) {
    for (int k = 0; k < 5; ++k) g_phase3[blockIdx.x * 8 + k] += ph2[k];
    g_phase3[blockIdx.x * 8 + 7] += 1;
  }
#endif
}

// After level 2, over the key workgroups: k_rfix2a copies the exact key counts to
// kprev (the next batch's prediction; a cursor counts on past an overflow, so they
// are exact either way), sums their 8-rounded sizes per workgroup and passes the
// overflow flag on as the redo flag; on a redo, k_rfix2b lays the regions out exactly.
__global__ __launch_bounds__(1024) void k_rfix2a(uint32_t F, uint32_t* __restrict__ meta, uint32_t* __restrict__ kprev) {
  __shared__ uint64_t red[16];
  const MetaLayout L = meta_layout(F);
  uint32_t* hdr = meta + L.hdr();
  const uint32_t k = blockIdx.x * 1024u + threadIdx.x;
  uint32_t r8 = 0;
  if (k < L.K) {
    const uint32_t c = meta[L.kcnt() + k];
    kprev[k] = c;
    if (!tile_direct(meta, L, k >> 1)) r8 = round_up(c, 8);
  }
  const uint64_t w = wave_sum((uint64_t)r8);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = w;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int q = 0; q < 16; ++q) t += red[q];
    reinterpret_cast<uint64_t*>(meta + L.wsum())[blockIdx.x] = t;
    if (blockIdx.x == 0) hdr[H_REDO2] = hdr[H_OV2] | hdr[H_COUNT2];
  }
}

__global__ __launch_bounds__(1024) void k_rfix2b(uint32_t F, uint32_t* __restrict__ meta) {
  __shared__ uint64_t red[16];
  __shared__ uint64_t l64[17];
  const MetaLayout L = meta_layout(F);
  uint32_t* hdr = meta + L.hdr();
  if (hdr[H_REDO2] == 0u) return;  // (grid-uniform)
  const uint64_t before = wsum_before(reinterpret_cast<const uint64_t*>(meta + L.wsum()), blockIdx.x, red);
  const uint32_t k = blockIdx.x * 1024u + threadIdx.x;
  const bool mine = k < L.K && !tile_direct(meta, L, k >> 1);
  const uint32_t c8 = mine ? round_up(meta[L.kcnt() + k], 8) : 0u;
  uint64_t total;
  const uint64_t base = hdr[H_D16] + before + block_excl_scan64((uint64_t)c8, l64, &total);
  if (mine) {
    meta[L.kbase() + k] = (uint32_t)base;
    meta[L.kcap() + k] = c8;
    meta[L.kcnt() + k] = 0u;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (hdr[H_COUNT2]) hdr[H_NCNT2] += 1u;  // a counting first pass, not a redo
    else hdr[H_NOVR2] += 1u;
    hdr[H_OV2] = 0u;
  }
}

// k_rfix2a + k_rfix2b in one workgroup for <= RFIX2_ONE_WG_MAX keys (thread j: keys
// [KP j, KP j + KP), in key order across threads): the exact counts to kprev, and on a
// redo the exact regions.
__global__ __launch_bounds__(1024) void k_rfix2s(uint32_t F, uint32_t* __restrict__ meta, uint32_t* __restrict__ kprev) {
  __shared__ uint64_t l64[17];
  const MetaLayout L = meta_layout(F);
  uint32_t* hdr = meta + L.hdr();
  constexpr uint32_t KPM = RFIX2_ONE_WG_MAX / 1024;
  const uint32_t KP = (L.K + 1023) / 1024, k0 = threadIdx.x * KP;
  const uint32_t redo = hdr[H_OV2] | hdr[H_COUNT2];
  const uint32_t counted = hdr[H_COUNT2];
  uint32_t c8[KPM], dm = 0;
  uint64_t mine = 0;
#pragma unroll
  for (uint32_t q = 0; q < KPM; ++q) {
    const uint32_t k = k0 + q;
    c8[q] = 0;
    if (q < KP && k < L.K) {
      const uint32_t c = meta[L.kcnt() + k];
      kprev[k] = c;
      if (tile_direct(meta, L, k >> 1)) {
        dm |= 1u << q;
      } else {
        c8[q] = round_up(c, 8);
        mine += c8[q];
      }
    }
  }
  __syncthreads();  // every thread has read the header
  if (threadIdx.x == 0) hdr[H_REDO2] = redo;
  if (!redo) return;  // (workgroup-uniform)
  uint64_t total;
  uint64_t kb = (uint64_t)hdr[H_D16] + block_excl_scan64(mine, l64, &total);
#pragma unroll
  for (uint32_t q = 0; q < KPM; ++q) {
    const uint32_t k = k0 + q;
    if (q < KP && k < L.K && !((dm >> q) & 1u)) {
      meta[L.kbase() + k] = (uint32_t)kb;
      meta[L.kcap() + k] = c8[q];
      meta[L.kcnt() + k] = 0u;
      kb += c8[q];
    }
  }
  if (threadIdx.x == 0) {
    if (counted) hdr[H_NCNT2] += 1u;  // a counting first pass, not a redo
    else hdr[H_NOVR2] += 1u;
    hdr[H_OV2] = 0u;
  }
}

// Small host batches into the staging ring: the GPU reads pinned host memory
// directly (zero-copy over PCIe) -- one kernel for both arrays, instead of two
// DMA copies whose setup dominates at 64K samples (35 us per pair measured).
__global__ __launch_bounds__(256) void k_fetch_host(const uint32_t* __restrict__ hs, const uint32_t* __restrict__ hv,
                                                    uint32_t* __restrict__ ds, uint32_t* __restrict__ dv, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t s = hs[i], v = hv[i];
    ds[i] = s;
    dv[i] = v;
  }
}

}  // namespace

#ifdef L5DH_PHASES
extern "C" __attribute__((visibility("default"))) int l5dh_dev_phases3(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase3), sizeof(g_phase3), 0, hipMemcpyDeviceToHost);
}
extern "C" __attribute__((visibility("default"))) int l5dh_dev_phases_plan(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase_plan), sizeof(g_phase_plan), 0, hipMemcpyDeviceToHost);
}
extern "C" __attribute__((visibility("default"))) int l5dh_dev_phases1(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase1), sizeof(g_phase1), 0, hipMemcpyDeviceToHost);
}
#endif

hipError_t launch_fetch_host(const uint32_t* hs, const uint32_t* hv, uint32_t* ds, uint32_t* dv, size_t n,
                             hipStream_t st) {
  if (n == 0) return hipSuccess;
  const size_t blocks = std::min<size_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_fetch_host, dim3((unsigned)blocks), dim3(256), 0, st, hs, hv, ds, dv, n);
  return hipGetLastError();
}

hipError_t set_ingest_attributes() {
  hipError_t e;
  if ((e = hipFuncSetAttribute((const void*)k_rsample, hipFuncAttributeMaxDynamicSharedMemorySize, 32768 * 4)))
    return e;
  if ((e = hipFuncSetAttribute((const void*)k_rplan1, hipFuncAttributeMaxDynamicSharedMemorySize, (int)RPLAN1_LDS)))
    return e;
  return hipFuncSetAttribute((const void*)k_rbin1w<NT1, CHW>, hipFuncAttributeMaxDynamicSharedMemorySize,
                             (int)rbin1w_lds());
}

hipError_t launch_ingest(const IngestArgs& a, int stage, hipStream_t st) {
  const uint32_t K = 2 * a.F;
  switch (stage) {
    case 0:  // sample + level-1 plan
      hipLaunchKernelGGL(k_rsample, dim3(RS_WG), dim3(1024), (size_t)((K + 1) / 2) * 4, st, a.series, a.n, a.S, K,
                         a.kest);
      hipLaunchKernelGGL(k_rplan1, dim3(1), dim3(1024), RPLAN1_LDS, st, a.n, a.F, a.kest, a.kprev, a.meta, a.cap32,
                         a.dlim16, a.thr_min, a.dmax, a.pct);
      {  // level-2 regions of the non-direct keys
        const uint32_t B = (K + 1023) / 1024;  // <= 64 (wsum)
        hipLaunchKernelGGL(k_rplan2a, dim3(B), dim3(1024), 0, st, a.n, a.F, a.kest, a.kprev, a.meta, a.pct);
        hipLaunchKernelGGL(k_rplan2b, dim3(B), dim3(1024), 0, st, a.F, a.meta, a.cap16);
      }
      break;
    case 1:  // level 1, its fix-up, the redo pass (exits at once unless needed)
      for (int pass = 0; pass < 2; ++pass) {
        hipLaunchKernelGGL((k_rbin1w<NT1, CHW>), dim3(a.G), dim3(NT1), rbin1w_lds(), st, a.series, a.values, a.n,
                           a.per, a.S, a.F, a.tb, a.meta, a.rec32, a.rec16, a.sumfix, a.err, a.vec ? 1 : 0, pass);
        if (pass == 0) hipLaunchKernelGGL(k_rfix1, dim3(1), dim3(1024), 0, st, a.F, a.meta, a.err, a.err_host);
      }
      break;
    case 2:  // (the level-2 plan is made by k_rplan1 and k_rfix1)
      break;
    default: {  // level 2, its fix-up, the redo pass
      const uint32_t B = (K + 1023) / 1024;
      for (int pass = 0; pass < 2; ++pass) {
        const MetaLayout L = meta_layout(a.F);
        hipLaunchKernelGGL(k_rbin2<B2_NT>, dim3(a.num_cu * B2_PER_CU), dim3(B2_NT), 0, st, a.S, a.F, a.tb, a.meta,
                           a.meta + L.istart(), a.meta + L.bbase(), a.meta + L.btot(), a.rec32, a.rec16, a.sumfix,
                           pass);
        if (pass == 0 && K <= RFIX2_ONE_WG_MAX) {
          hipLaunchKernelGGL(k_rfix2s, dim3(1), dim3(1024), 0, st, a.F, a.meta, a.kprev);
        } else if (pass == 0) {
          hipLaunchKernelGGL(k_rfix2a, dim3(B), dim3(1024), 0, st, a.F, a.meta, a.kprev);
          hipLaunchKernelGGL(k_rfix2b, dim3(B), dim3(1024), 0, st, a.F, a.meta);
        }
      }
      break;
    }
  }
  return hipGetLastError();
}

}  // namespace l5dh
