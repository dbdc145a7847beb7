// l5dh_paged.hip -- paged ingest (L5DH_PARAM_BIN_MODE 3): the level-1 partition
// writes into CU-private page pools, so no counting pass precedes it (DESIGN.md
// §6c; the layouts measured in profiles/r02m_pages).
//
//   k_psample     this batch's tile sizes estimated from 2^20 sampled ids
//   k_pselect     this batch's direct tiles (the biggest estimated, as k_stplan picks)
//   k_pbin1       level 1: LDS counting sort of 16K-sample sub-chunks by bin (FS
//                 super-tiles, two half-bins per direct tile, a trash bin); a bin's run
//                 fills its current page and spills into consecutive fresh pages of
//                 the slab's pool, logged as (first page, bin, pages)
//   k_pdir_count  per bin: pages and records (from the slabs' logs and last pages)
//   k_pdir_scan   per-bin page bases; direct items and level-2 items (KP pages each)
//   k_pdir_fill   the page directory: per bin, {page, records in it}
//   k_pdir_init   clean direct tiles' state rows zeroed (they are folded at ingest)
//   k_pfold       direct half-tiles folded into their state rows: u32 LDS bins of
//                 16 series per item, flushed with global atomics (as k_accum_split)
//   k_p2count     level-2 items: records per tile of the super-tile
//   k_p2scan_a    per super-tile: exclusive prefixes over its items, tile totals
//   k_p2scan_b    tile_base of the final layout
//   k_p2place     level 2: items re-read, LDS-sorted by tile, written to the final layout
//
// The direct tiles of a batch are chosen from a sample of its own ids; their records never reach the final layout (the snapshot sees them
// as dirty tiles).  All other tiles' records are laid out per tile exactly as the
// two-level path lays them out (split tiles: none), so the snapshot is unchanged.
#include "l5dh_device.hpp"

namespace l5dh {
namespace {

constexpr int ST_TILES = 64;
constexpr int ST_SHIFT = 11;

// payload of a sample outside [0, V_ESC): exact contribution to sumfix, V_ESC + bucket
__device__ __forceinline__ uint32_t ppayload_slow(uint32_t s, float f, Tables tb, int64_t* __restrict__ sumfix) {
  int64_t c;
  const uint32_t b = bucketize(f, tb.lut, tb.lim_pad, c);
  if (c >= 0 && c < (int64_t)V_ESC) return (uint32_t)c;
  atomicAdd(reinterpret_cast<unsigned long long*>(&sumfix[s]), (unsigned long long)c);
  return V_ESC + b;
}

// LDS of k_pbin1: stage[CH1] uint2 | cnt (low 16: records, high 16: stage offset) |
// dA | dB | pg | fr (low 16: fill, high 16: room) [PG_BINS] | dw[1024] uint2 | cursors
constexpr size_t pbin1_lds(int ch) { return (size_t)ch * 8 + 5 * PG_BINS * 4 + 1024 * 8 + 16; }

template <int CH1, int NT>
__global__ __launch_bounds__(NT, 1) void k_pbin1(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                                 size_t n, size_t per, uint32_t S, uint32_t F,
                                                 const uint32_t* __restrict__ plan, Tables tb,
                                                 int64_t* __restrict__ sumfix, uint32_t* __restrict__ err,
                                                 uint32_t pool_pages, uint32_t* __restrict__ pool,
                                                 uint2* __restrict__ plog, uint32_t* __restrict__ nlog,
                                                 uint2* __restrict__ tailpg, int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint2* stage = reinterpret_cast<uint2*>(smem);
  uint32_t* cnt = smem + 2 * CH1;
  uint32_t* dA = cnt + PG_BINS;
  uint32_t* dB = dA + PG_BINS;
  uint32_t* pg = dB + PG_BINS;
  uint32_t* fr = pg + PG_BINS;
  uint2* dw = reinterpret_cast<uint2*>(fr + PG_BINS);
  uint32_t* cur = reinterpret_cast<uint32_t*>(dw + 1024);  // [0] next free page, [1] log entries
  constexpr uint32_t P = PAGE;
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t NW = (F + 31) / 32;
  const uint32_t ND = plan[PLAN_ND];
  const uint32_t TB = FS + 2 * ND;
  const uint32_t g = blockIdx.x;
  const uint32_t pool0 = g * pool_pages;
  uint2* mylog = plog + (size_t)g * pool_pages;
  for (uint32_t b = threadIdx.x; b < PG_BINS; b += NT) {
    cnt[b] = 0;
    pg[b] = 0xFFFFFFFFu;  // no page yet
    fr[b] = P;            // full: the first run allocates
  }
  for (uint32_t w = threadIdx.x; w < NW; w += NT) dw[w] = make_uint2(plan[PLAN_DBITS + w], plan[PLAN_DPRE + w]);
  if (threadIdx.x == 0) cur[0] = cur[1] = 0;
  __syncthreads();
  const size_t lo = (size_t)g * per;
  const size_t hi = lo + per < n ? lo + per : n;
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  constexpr int PT = CH1 / NT;
  bool bad = false;
  for (size_t c0 = lo; c0 < hi; c0 += CH1) {
    uint32_t sv[PT];
    float fv[PT];
    uint32_t inm = 0xFFFFFFFFu;  // slots holding a sample (the batch tail has fewer)
    if (vec && c0 + CH1 <= hi) {
#pragma unroll
      for (int k = 0; k < PT / 4; ++k) {
        const size_t base = c0 + 4 * ((size_t)k * NT + threadIdx.x);
        const uint4 s4 = *reinterpret_cast<const uint4*>(series + base);
        const float4 f4 = *reinterpret_cast<const float4*>(values + base);
        sv[4 * k] = s4.x; sv[4 * k + 1] = s4.y; sv[4 * k + 2] = s4.z; sv[4 * k + 3] = s4.w;
        fv[4 * k] = f4.x; fv[4 * k + 1] = f4.y; fv[4 * k + 2] = f4.z; fv[4 * k + 3] = f4.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < PT; ++k) {
        const size_t i = c0 + 4 * ((size_t)(k >> 2) * NT + threadIdx.x) + (k & 3);
        const bool in = i < hi;
        sv[k] = in ? series[i] : 0xFFFFFFFFu;
        fv[k] = in ? values[i] : 0.0f;
        if (!in) inm &= ~(1u << k);
      }
    }
    // payloads: +0 <= f < V_ESC by one compare of the bit pattern; the rare rest exactly,
    // from a non-unrolled loop over this thread's escaped slots staged in its own part
    // of the (still free) stage -- one inlined copy of the full search
    uint32_t rec[PT], pk[PT];
    uint32_t escm = 0;
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t s = sv[k];
      const bool ok = s < S;
      bad |= !ok && ((inm >> k) & 1u);
      const bool fast = __float_as_uint(fv[k]) < 0x49FFC000u;
      escm |= (ok && !fast) ? (1u << k) : 0u;
      rec[k] = ((s & (ST_TILES * TILE - 1)) << 21) | (fast ? (uint32_t)fv[k] : 0u);
    }
    if (__ballot(escm != 0u)) {
      uint2* tmp = stage + threadIdx.x * PT;
#pragma unroll
      for (int k = 0; k < PT; ++k) tmp[k] = make_uint2(sv[k], __float_as_uint(fv[k]));
#pragma unroll 1
      for (int k = 0; k < PT; ++k)
        if ((escm >> k) & 1u) tmp[k].x = ppayload_slow(tmp[k].x, __uint_as_float(tmp[k].y), tb, sumfix);
#pragma unroll
      for (int k = 0; k < PT; ++k)
        if ((escm >> k) & 1u) rec[k] = ((sv[k] & (ST_TILES * TILE - 1)) << 21) | tmp[k].x;
    }
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t s = sv[k];
      const bool ok = s < S;
      const uint2 d = dw[(s >> (TILE_SHIFT + 5)) & 1023u];
      const uint32_t tw = __builtin_amdgcn_ubfe(s, TILE_SHIFT, 5);
      const bool direct = __builtin_amdgcn_ubfe(d.x, tw, 1) != 0u;
      const uint32_t dbin = FS + 2u * (d.y + (uint32_t)__popc(__builtin_amdgcn_ubfe(d.x, 0, tw))) + ((s >> 4) & 1u);
      const uint32_t b = sel_u32(ok, sel_u32(direct, dbin, s >> ST_SHIFT), TB);
      pk[k] = atomicAdd(cnt + b, 1u) | (b << 14);
    }
    __syncthreads();
    if (wv == 0) {  // stage offsets into the high halves: lane l scans bins [16 l, 16 l + 16)
      uint32_t c[16], tl = 0;
#pragma unroll
      for (int q = 0; q < 16; ++q) tl += (c[q] = cnt[16 * lane + q]);
      uint32_t e = wave_incl_scan32(tl) - tl;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        cnt[16 * lane + q] = c[q] | (e << 16);
        e += c[q];
      }
    }
    // pages: a bin's run fills its current page, then continues in consecutive new
    // pages of the slab's pool (reads cnt's low halves only: no race with the scan)
    for (uint32_t b = threadIdx.x; b <= TB; b += NT) {
      const uint32_t c = cnt[b] & 0xFFFFu;
      if (!c) continue;
      const uint32_t fill = fr[b] & 0xFFFFu, rm = P - fill;
      dA[b] = pg[b] + fill;
      if (c <= rm) {
        fr[b] = (fill + c) | (rm << 16);
      } else {
        const uint32_t need = (c - rm + P - 1) / P;
        const uint32_t np = atomicAdd(&cur[0], need);
        const uint32_t li = atomicAdd(&cur[1], 1u);
        mylog[li] = make_uint2(pool0 + np, b | (need << 16));
        dB[b] = (pool0 + np) * P;
        pg[b] = (pool0 + np + need - 1) * P;
        fr[b] = (c - rm - (need - 1) * P) | (rm << 16);
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PT; ++k) {
      const uint32_t b = pk[k] >> 14, r = pk[k] & 16383u;
      const uint32_t rm = fr[b] >> 16;
      stage[(cnt[b] >> 16) + r] = make_uint2(rec[k], r < rm ? dA[b] + r : dB[b] + (r - rm));
    }
    __syncthreads();
    for (uint32_t b = threadIdx.x; b <= TB; b += NT) cnt[b] = 0;
#pragma unroll
    for (int k = 0; k < PT; ++k) {  // all CH1 entries in sorted order (each wave a contiguous PT x 64 range)
      const uint2 e = stage[(uint32_t)wv * (PT * 64) + (uint32_t)k * 64 + (uint32_t)lane];
      pool[e.y] = e.x;
    }
    __syncthreads();
  }
  if (bad) atomicAdd(err, 1u);  // monotonic, like k_count's
  for (uint32_t b = threadIdx.x; b < PG_BINS; b += NT)
    tailpg[(size_t)g * PG_BINS + b] = make_uint2(pg[b], fr[b] & 0xFFFFu);  // pg ~0u: no page
  if (threadIdx.x == 0) nlog[g] = cur[1];
}

// pd layout (u32): [0 .. PG_BINS) pages per bin | [PG_BINS ..) records per bin |
// [2 PG_BINS ..] page base per bin (PG_BINS + 1) | [3 PG_BINS + 1 ..] fill cursors |
// [4 PG_BINS + 1 ..] direct item base per half-bin (257) | then level-2 item base per
// super-tile (513) | header: direct items, level-2 items
constexpr int PD_PAGES = 0, PD_RECS = PG_BINS, PD_BASE = 2 * PG_BINS, PD_CUR = 3 * PG_BINS + 1,
              PD_DITEM = 4 * PG_BINS + 1, PD_LITEM = PD_DITEM + 2 * DIRECT_MAX + 2, PD_HDR = PD_LITEM + 514;
static_assert(PD_HDR + 2 <= PD_WORDS, "page directory header");

// Per slab (one workgroup): pages and records per bin summed in LDS, then one global
// atomic per (slab, bin) -- a hot bin gets hundreds of log entries per slab, and
// same-address global atomics serialize.
__global__ __launch_bounds__(256) void k_pdir_count(const uint2* __restrict__ plog, const uint32_t* __restrict__ nlog,
                                                    const uint2* __restrict__ tailpg, uint32_t pool_pages,
                                                    uint32_t* __restrict__ pd) {
  __shared__ uint32_t lp[PG_BINS], lr[PG_BINS];
  const uint32_t g = blockIdx.x;
  const uint32_t ne = nlog[g];
  for (uint32_t b = threadIdx.x; b < PG_BINS; b += 256) lp[b] = lr[b] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ne; i += 256) {
    const uint2 e = plog[(size_t)g * pool_pages + i];
    atomicAdd(&lp[e.y & 0xFFFFu], e.y >> 16);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < PG_BINS; b += 256) {
    const uint32_t np = lp[b];
    if (!np) continue;
    const uint2 t = tailpg[(size_t)g * PG_BINS + b];
    atomicAdd(&pd[PD_PAGES + b], np);
    atomicAdd(&pd[PD_RECS + b], np * PAGE - (PAGE - t.y));  // the last page's unused slots
  }
}

// One workgroup: page bases per bin, items of KPD pages per direct half-bin and of
// KP pages per super-tile (the trash bin has none).
__global__ __launch_bounds__(1024) void k_pdir_scan(uint32_t F, const uint32_t* __restrict__ plan,
                                                    uint32_t* __restrict__ pd) {
  __shared__ uint4 lds4[17];
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t ND = plan[PLAN_ND];
  const uint32_t b = threadIdx.x;  // PG_BINS == 1024
  const uint32_t np = pd[PD_PAGES + b];
  uint32_t v[4] = {np, (b >= FS && b < FS + 2 * ND) ? (np + KPD - 1) / KPD : 0u, b < FS ? (np + KP - 1) / KP : 0u, 0u},
           tot[4];
  block_excl_scan4<1024>(v, lds4, tot);
  pd[PD_BASE + b] = v[0];
  pd[PD_CUR + b] = 0;
  if (b >= FS && b < FS + 2 * ND) pd[PD_DITEM + (b - FS)] = v[1];
  if (b < FS) pd[PD_LITEM + b] = v[2];
  if (b == 0) {
    pd[PD_BASE + PG_BINS] = tot[0];
    pd[PD_DITEM + 2 * ND] = tot[1];
    pd[PD_LITEM + FS] = tot[2];
    pd[PD_HDR] = tot[1];
    pd[PD_HDR + 1] = tot[2];
  }
}

// The page directory: dir[base[b] ..) = {page, records in it} of bin b, any order.
// Per slab: its pages per bin (LDS), one global reservation per (slab, bin), then
// the entries placed through LDS cursors.
__global__ __launch_bounds__(256) void k_pdir_fill(const uint2* __restrict__ plog, const uint32_t* __restrict__ nlog,
                                                   const uint2* __restrict__ tailpg, uint32_t pool_pages,
                                                   uint32_t* __restrict__ pd, uint2* __restrict__ dir) {
  __shared__ uint32_t lp[PG_BINS];
  const uint32_t g = blockIdx.x;
  const uint32_t ne = nlog[g];
  for (uint32_t b = threadIdx.x; b < PG_BINS; b += 256) lp[b] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ne; i += 256) {
    const uint2 e = plog[(size_t)g * pool_pages + i];
    atomicAdd(&lp[e.y & 0xFFFFu], e.y >> 16);
  }
  __syncthreads();
  for (uint32_t b = threadIdx.x; b < PG_BINS; b += 256)
    if (lp[b]) lp[b] = pd[PD_BASE + b] + atomicAdd(&pd[PD_CUR + b], lp[b]);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ne; i += 256) {
    const uint2 e = plog[(size_t)g * pool_pages + i];
    const uint32_t b = e.y & 0xFFFFu, np = e.y >> 16;
    const uint32_t at = atomicAdd(&lp[b], np);
    const uint2 t = tailpg[(size_t)g * PG_BINS + b];
    for (uint32_t q = 0; q < np; ++q) {
      const uint32_t page = e.x + q;
      dir[at + q] = make_uint2(page, page * PAGE == t.x ? t.y : PAGE);
    }
  }
}

// Clean direct tiles start from zero rows; all become dirty (their counts live in
// the state rows from now on).  The exact contributions k_pbin1 added to sumfix for
// their escaped samples move into `total` here: no snapshot kernel visits a tile
// without pending records before a range snapshot or export reads its total.
__global__ __launch_bounds__(256) void k_pdir_init(const uint32_t* __restrict__ plan, State st) {
  const uint32_t ND = plan[PLAN_ND];
  for (uint32_t d = blockIdx.x; d < ND; d += gridDim.x) {
    const uint32_t t = plan[PLAN_DLIST + d];
    const uint32_t s0 = t * TILE, s1 = min(st.S, s0 + TILE);
    const bool clean = !st.dirty[t];
    if (clean) {
      uint4* p = reinterpret_cast<uint4*>(st.counts + (size_t)s0 * ROW);
      const size_t n4 = (size_t)(s1 - s0) * ROW / 4;
      for (size_t k = threadIdx.x; k < n4; k += 256) p[k] = make_uint4(0, 0, 0, 0);
    }
    if (threadIdx.x < s1 - s0) {
      const uint32_t s = s0 + threadIdx.x;
      const int64_t f = st.sumfix[s];
      st.total[s] = (clean ? 0 : st.total[s]) + f;
      if (f) st.sumfix[s] = 0;
    }
    __syncthreads();  // (the dirty flag is read by later kernels only)
    if (threadIdx.x == 0) st.dirty[t] = 1;
  }
}

// Last entry e of base[0..n] (ascending) with base[e] <= x.
__device__ __forceinline__ uint32_t upper_index(const uint32_t* __restrict__ base, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t m = (lo + hi) >> 1;
    if (base[m] <= x) lo = m; else hi = m;
  }
  return lo;
}

// Records of an item's pages (<= KP pages of PAGE records = IR groups of 4 per
// thread): thread t takes groups t, t + WG, ...; the page entries are wave-uniform
// (scalar loads), and every load is issued before any record is used (no branches:
// a group past the item or past its page's fill reads a valid page and is masked).
constexpr int IR = (int)(KP * PAGE / 4 / WG);
template <class Fn>
__device__ __forceinline__ void item_records(const uint32_t* __restrict__ pool, const uint2* __restrict__ dir,
                                             uint32_t p0, uint32_t p1, Fn&& fn) {
  static_assert(KP * PAGE % (4 * WG) == 0 && (PAGE / 4) % 64 == 0, "whole waves per page");
  p0 = __builtin_amdgcn_readfirstlane(p0);
  p1 = __builtin_amdgcn_readfirstlane(p1);
  uint4 x[IR];
  uint32_t m[IR];
#pragma unroll
  for (int q = 0; q < IR; ++q) {
    const uint32_t gi = (uint32_t)q * WG + threadIdx.x;
    const uint32_t pi = p0 + gi / (PAGE / 4);  // wave-uniform: a wave's 64 groups are in one page
    const uint2 e = dir[pi < p1 ? pi : p0];
    const uint32_t o = 4u * (gi % (PAGE / 4));
    m[q] = (pi < p1 && e.y > o) ? min(4u, e.y - o) : 0u;  // valid records of this group
    x[q] = *reinterpret_cast<const uint4*>(pool + (size_t)e.x * PAGE + o);
  }
#pragma unroll
  for (int q = 0; q < IR; ++q) fn(x[q], m[q]);
}

// Direct half-tiles folded into their state rows: item = (half-bin, KPD pages);
// u32 LDS bins of the half's 16 series, lane-private u64 value sums, flushed with
// global atomics (k_pdir_init prepared the rows).  Persistent.
__global__ __launch_bounds__(WG) void k_pfold(const uint32_t* __restrict__ pool, const uint2* __restrict__ dir,
                                              const uint32_t* __restrict__ pd, const uint32_t* __restrict__ plan,
                                              uint32_t F, State st, Tables tb) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* hist = smem;                                                              // [16][HROW]
  unsigned long long* vsl = reinterpret_cast<unsigned long long*>(smem + 16 * HROW);  // [16][64]
  uint2* lut2 = reinterpret_cast<uint2*>(vsl + 16 * 64);                              // [LUT2_N]
  uint32_t* ib = reinterpret_cast<uint32_t*>(lut2 + LUT2_N);                          // [2 DIRECT_MAX + 1]
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t ND = plan[PLAN_ND];
  const uint32_t nitems = pd[PD_HDR];
  const int lane = lane_id(), w = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < LUT2_N; i += WG) lut2[i] = tb.lut2[i];
  for (uint32_t i = threadIdx.x; i <= 2 * ND; i += WG) ib[i] = pd[PD_DITEM + i];
  for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
    {
      uint4* q = reinterpret_cast<uint4*>(smem);
      for (int i = threadIdx.x; i < (16 * HROW + 16 * 64 * 2) / 4; i += WG) q[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const uint32_t h = upper_index(ib, 2 * ND, item);  // half-bin h = 2 d + half
    const uint32_t b = FS + h;
    const uint32_t p0 = pd[PD_BASE + b] + (item - ib[h]) * KPD;
    const uint32_t p1 = min(p0 + KPD, pd[PD_BASE + b + 1]);
    // (a direct item is KPD / KP batches of pages: the LDS clear and the 16-row
    // global flush are paid per 2^18 records, as k_accum_split's items)
    for (uint32_t pb = p0; pb < p1; pb += KP) item_records(pool, dir, pb, min(pb + KP, p1), [&](uint4 x, uint32_t m) {
      const uint32_t r[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if ((uint32_t)k >= m) continue;
        uint32_t v;
        const uint32_t bk = record_bucket(r[k], lut2, v);
        const uint32_t loc = (r[k] >> 21) & 15u;
        atomicAdd(&hist[loc * HROW + bk], 1u);
        atomicAdd(&vsl[loc * 64 + lane], (unsigned long long)v);
      }
    });
    __syncthreads();
    const uint32_t t = plan[PLAN_DLIST + (h >> 1)];
    const uint32_t s = t * TILE + 16 * (h & 1u) + w;
    const uint64_t vsum = wave_sum(vsl[w * 64 + lane]);
    if (s < st.S) {
      uint32_t* grow = st.counts + (size_t)s * ROW;
      const uint32_t* hrow = hist + w * HROW;
      for (int b0 = 0; b0 < NB; b0 += 64) {  // 64 consecutive bins per wave atomic
        const int bb = b0 + lane;
        const uint32_t v = bb < NB ? hrow[bb] : 0u;
        if (__ballot(v != 0u)) {
          if (v) atomicAdd(&grow[bb], v);
        }
      }
      if (lane == 0 && vsum) atomicAdd(reinterpret_cast<unsigned long long*>(&st.total[s]), (unsigned long long)vsum);
    }
    __syncthreads();  // the LDS rows are read: the next item may clear them
  }
}

// LDS counter add (RANK: returning the rank) where many lanes of the wave may share
// a key (a hot tile of a super-tile; no plan names it here): twice, the first
// pending lane's key is peeled off -- one atomic for all the lanes holding it, ranks
// by mask_below -- and the remaining lanes add for themselves.  Convergent: every
// lane calls it (valid = false: no record).
template <bool RANK>
__device__ __forceinline__ uint32_t peel_add(uint32_t* ctr, uint32_t key, bool valid) {
  uint32_t rank = 0;
  bool done = !valid;
#pragma unroll
  for (int round = 0; round < 2; ++round) {
    const unsigned long long act = __ballot(!done);
    if (!act) break;  // wave-uniform
    const int leader = __ffsll((long long)act) - 1;
    const uint32_t k0 = __builtin_amdgcn_readlane(key, leader);
    const bool mine = !done && key == k0;
    const unsigned long long m = __ballot(mine);
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(&ctr[k0], (uint32_t)__popcll(m));
    if (RANK) base = __builtin_amdgcn_readlane(base, leader);
    if (mine) {
      rank = base + mask_below(m);
      done = true;
    }
  }
  if (!done) {
    if (RANK)
      rank = atomicAdd(&ctr[key], 1u);
    else
      atomicAdd(&ctr[key], 1u);
  }
  return rank;
}

// Level-2 item = (super-tile j, KP of its pages): records per tile of the super-tile.
__global__ __launch_bounds__(WG) void k_p2count(const uint32_t* __restrict__ pool, const uint2* __restrict__ dir,
                                                const uint32_t* __restrict__ pd, uint32_t F,
                                                uint32_t* __restrict__ cnt2) {
  __shared__ uint32_t c[ST_TILES];
  __shared__ uint32_t ib[513];
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t nitems = pd[PD_HDR + 1];
  for (uint32_t i = threadIdx.x; i <= FS; i += WG) ib[i] = pd[PD_LITEM + i];
  for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
    if (threadIdx.x < ST_TILES) c[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t j = upper_index(ib, FS, item);
    const uint32_t p0 = pd[PD_BASE + j] + (item - ib[j]) * KP;
    const uint32_t p1 = min(p0 + KP, pd[PD_BASE + j + 1]);
    item_records(pool, dir, p0, p1, [&](uint4 x, uint32_t m) {
      const uint32_t r[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        peel_add<false>(c, r[k] >> 26, (uint32_t)k < m);
    });
    __syncthreads();
    if (threadIdx.x < ST_TILES) cnt2[(size_t)item * ST_TILES + threadIdx.x] = c[threadIdx.x];
    __syncthreads();
  }
}

// Per super-tile (one 1024-thread workgroup each, lane = tile of the super-tile):
// exclusive prefixes of its items' tile counts (in place) and the tile totals.  The
// 16 waves take consecutive blocks of the items (a hot super-tile has thousands):
// block sums, prefixes over the waves, then the in-place pass.
__global__ __launch_bounds__(1024) void k_p2scan_a(const uint32_t* __restrict__ pd, uint32_t F,
                                                   uint32_t* __restrict__ cnt2, uint32_t* __restrict__ tot) {
  __shared__ uint32_t part[16][ST_TILES];
  const uint32_t j = blockIdx.x, k = (uint32_t)lane_id(), w = threadIdx.x >> 6;
  const uint32_t i0 = pd[PD_LITEM + j], i1 = pd[PD_LITEM + j + 1];
  const uint32_t n = i1 - i0, per = (n + 15) / 16;
  const uint32_t a = i0 + min(n, w * per), b = i0 + min(n, (w + 1) * per);
  constexpr int U = 16;  // a batch of items' loads at once
  uint32_t acc = 0;
  for (uint32_t i = a; i < b; i += U) {
    uint32_t v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) v[q] = i + q < b ? cnt2[(size_t)(i + q) * ST_TILES + k] : 0u;
#pragma unroll
    for (int q = 0; q < U; ++q) acc += v[q];
  }
  part[w][k] = acc;
  __syncthreads();
  uint32_t off = 0, all = 0;
  for (uint32_t q = 0; q < 16; ++q) {
    const uint32_t x = part[q][k];
    off += q < w ? x : 0u;
    all += x;
  }
  acc = off;
  for (uint32_t i = a; i < b; i += U) {
    uint32_t v[U];
#pragma unroll
    for (int q = 0; q < U; ++q) v[q] = i + q < b ? cnt2[(size_t)(i + q) * ST_TILES + k] : 0u;
#pragma unroll
    for (int q = 0; q < U; ++q)
      if (i + q < b) {
        cnt2[(size_t)(i + q) * ST_TILES + k] = acc;
        acc += v[q];
      }
  }
  const uint32_t t = j * ST_TILES + k;
  if (w == 0 && t < F) tot[t] = all;
}

// One workgroup: tile_base of the final layout (direct tiles hold no records in it).
__global__ __launch_bounds__(1024) void k_p2scan_b(uint32_t F, const uint32_t* __restrict__ tot,
                                                   uint32_t* __restrict__ tile_base, const uint32_t* __restrict__ err,
                                                   uint32_t* __restrict__ err_host) {
  // k_pbin1's invalid-id count, to the host's mapped pinned word (no copy launch)
  if (threadIdx.x == 0) *reinterpret_cast<volatile uint32_t*>(err_host) = *err;
  __shared__ uint32_t lds[17];
  constexpr int PF = 32;  // F <= 32768 tiles: a thread's tiles [32 j, 32 j + 32)
  const uint32_t t0 = threadIdx.x * PF;
  uint32_t v[PF], s = 0;
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    v[k] = t0 + k < F ? tot[t0 + k] : 0u;
    s += v[k];
  }
  uint32_t total;
  uint32_t acc = block_excl_scan<1024>(s, lds, &total);
#pragma unroll
  for (int k = 0; k < PF; ++k)
    if (t0 + k < F) {
      tile_base[t0 + k] = acc;
      acc += v[k];
    }
  if (threadIdx.x == 0) tile_base[F] = total;
}

// This batch's direct tiles from a sample of its ids (before k_pbin1): PSAMPLE ids
// at an even stride, counted per tile in LDS (u16 pairs) by PS_WG workgroups and
// flushed with one global atomic per (workgroup, tile).  A direct tile only chooses
// the path its records take, so an estimate is enough.
constexpr uint32_t PSAMPLE = 1u << 20;
constexpr int PS_WG = 64;
__global__ __launch_bounds__(1024) void k_psample(const uint32_t* __restrict__ series, size_t n, uint32_t S,
                                                  uint32_t F, uint32_t* __restrict__ pcount) {
  __shared__ uint32_t c[16384];  // u16 pairs: tiles 2 i, 2 i + 1 (<= PSAMPLE / PS_WG = 16384 each)
  for (uint32_t i = threadIdx.x; i < (F + 1) / 2; i += 1024) c[i] = 0;
  __syncthreads();
  const uint32_t per = PSAMPLE / PS_WG;
  for (uint32_t k = threadIdx.x; k < per; k += 1024) {
    const uint64_t i = (uint64_t)(blockIdx.x * per + k) * n / PSAMPLE;
    const uint32_t s = series[i];
    if (s < S) {
      const uint32_t t = s >> TILE_SHIFT;
      atomicAdd(&c[t >> 1], (t & 1u) ? 0x10000u : 1u);
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < (F + 1) / 2; i += 1024) {
    const uint32_t x = c[i];
    if (x & 0xFFFFu) atomicAdd(&pcount[2 * i], x & 0xFFFFu);
    if ((x >> 16) && 2 * i + 1 < F) atomicAdd(&pcount[2 * i + 1], x >> 16);
  }
}

// One workgroup: the direct set -- the <= dmax tiles with the biggest estimated
// records (>= max(thr_min, 2^k), k the smallest power keeping <= dmax tiles).
__global__ __launch_bounds__(1024) void k_pselect(uint32_t F, size_t n, uint32_t* __restrict__ pcount,
                                                  uint32_t* __restrict__ plan, uint32_t thr_min, uint32_t dmax) {
  __shared__ uint32_t lh[33];
  __shared__ uint32_t sthr;
  __shared__ uint4 lds4[17];
  constexpr int PF = 32;
  const uint32_t t0 = threadIdx.x * PF;
  uint32_t est[PF];
  if (threadIdx.x < 33) lh[threadIdx.x] = 0;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    uint32_t e = 0;
    if (t0 + k < F) {
      const uint32_t x = pcount[t0 + k];
      if (x) pcount[t0 + k] = 0;  // ready for the next batch
      e = (uint32_t)min((uint64_t)x * n / PSAMPLE, (uint64_t)0xFFFFFFFFu);  // each draw stands for n / PSAMPLE
    }
    est[k] = e;
    if (dmax > 0 && e >= thr_min && e > 0) atomicAdd(&lh[31 - __clz((int)e)], 1u);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t cum = 0, thr = 0xFFFFFFFFu;
    int kbest = 32;
    if (dmax > 0)
      for (int k = 31; k >= 0; --k) {
        cum += lh[k];
        if (cum > dmax) break;
        kbest = k;
      }
    if (kbest < 32) thr = max(max(thr_min, 1u), 1u << kbest);
    sthr = thr;
  }
  __syncthreads();
  const uint32_t thr = sthr;
  uint32_t nb = 0;
#pragma unroll
  for (int k = 0; k < PF; ++k)
    if (t0 + k < F && est[k] >= thr) nb |= 1u << k;
  uint32_t cv[4] = {(uint32_t)__popc(nb), 0u, 0u, 0u}, ct[4];
  block_excl_scan4<1024>(cv, lds4, ct);
  if (t0 < F) {
    plan[PLAN_DBITS + threadIdx.x] = nb;
    plan[PLAN_DPRE + threadIdx.x] = cv[0];
    uint32_t x = nb, di = cv[0];
    while (x) {
      const uint32_t k = (uint32_t)(__ffs((int)x) - 1);
      x &= x - 1u;
      plan[PLAN_DLIST + di] = t0 + k;
      plan[PLAN_DSI + di] = 0xFFFFFFFFu;
      ++di;
    }
  }
  if (threadIdx.x == 0) plan[PLAN_ND] = ct[0];
}

// Level 2: items re-read, 8K-record sub-chunks (two pages) LDS-sorted by tile and
// written in sorted order to tile_base[t] + prefix(item, t) + running rank.
constexpr int P2_CH = 8192;  // records per sub-chunk: P2_CH / PAGE pages
static_assert(P2_CH % PAGE == 0, "whole pages per sub-chunk");
constexpr int P2_NT = 512;
__global__ __launch_bounds__(P2_NT) void k_p2place(const uint32_t* __restrict__ pool, const uint2* __restrict__ dir,
                                                   const uint32_t* __restrict__ pd, uint32_t F,
                                                   const uint32_t* __restrict__ pre2,
                                                   const uint32_t* __restrict__ tile_base,
                                                   uint32_t* __restrict__ records) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint2* stage = reinterpret_cast<uint2*>(smem);  // [P2_CH]
  uint32_t* cnt = smem + 2 * P2_CH;               // [64]
  uint32_t* off = cnt + ST_TILES;                 // [64]
  uint32_t* cur = off + ST_TILES;                 // [64]
  uint32_t* ib = cur + ST_TILES;                  // [513]
  const uint32_t FS = (F + ST_TILES - 1) / ST_TILES;
  const uint32_t nitems = pd[PD_HDR + 1];
  const int lane = lane_id(), wv = threadIdx.x >> 6;
  for (uint32_t i = threadIdx.x; i <= FS; i += P2_NT) ib[i] = pd[PD_LITEM + i];
  __syncthreads();
  for (uint32_t item = blockIdx.x; item < nitems; item += gridDim.x) {
    const uint32_t j = __builtin_amdgcn_readfirstlane(upper_index(ib, FS, item));
    const uint32_t p0 = __builtin_amdgcn_readfirstlane(pd[PD_BASE + j] + (item - ib[j]) * KP);
    const uint32_t p1 = __builtin_amdgcn_readfirstlane(min(p0 + KP, pd[PD_BASE + j + 1]));
    if (threadIdx.x < ST_TILES) {
      const uint32_t t = j * ST_TILES + threadIdx.x;
      cnt[threadIdx.x] = 0;
      cur[threadIdx.x] = t < F ? tile_base[t] + pre2[(size_t)item * ST_TILES + threadIdx.x] : 0u;
    }
    __syncthreads();
    // this thread's records: 16-B groups of a sub-chunk's pages, branch-free, all loads
    // issued at once; the next sub-chunk's are in flight while this one is sorted
    constexpr int G4 = P2_CH / 4 / P2_NT;  // 4 groups per thread
    auto load = [&](uint32_t pp, uint4 (&x)[G4], uint32_t (&m)[G4]) {
#pragma unroll
      for (int q = 0; q < G4; ++q) {
        const uint32_t gi = (uint32_t)q * P2_NT + threadIdx.x;  // group in the sub-chunk
        const uint32_t page = pp + gi / (PAGE / 4);
        const uint32_t o = 4u * (gi % (PAGE / 4));
        const uint2 e = dir[page < p1 ? page : p0];
        m[q] = (page < p1 && e.y > o) ? min(4u, e.y - o) : 0u;
        x[q] = *reinterpret_cast<const uint4*>(pool + (size_t)e.x * PAGE + o);
      }
    };
    uint4 xn[G4];
    uint32_t mn[G4];
    load(p0, xn, mn);
    for (uint32_t pp = p0; pp < p1; pp += P2_CH / PAGE) {
      uint4 x[G4];
      uint32_t m[G4];
#pragma unroll
      for (int q = 0; q < G4; ++q) {
        x[q] = xn[q];
        m[q] = mn[q];
      }
      if (pp + P2_CH / PAGE < p1) load(pp + P2_CH / PAGE, xn, mn);
      uint32_t rk[4 * G4];
#pragma unroll
      for (int q = 0; q < G4; ++q) {
        const uint32_t r[4] = {x[q].x, x[q].y, x[q].z, x[q].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) rk[4 * q + k] = peel_add<true>(cnt, r[k] >> 26, (uint32_t)k < m[q]);
      }
      __syncthreads();
      if (threadIdx.x < 64) {
        const uint32_t a = cnt[threadIdx.x];
        off[threadIdx.x] = wave_incl_scan32(a) - a;
      }
      __syncthreads();
      const uint32_t total = off[ST_TILES - 1] + cnt[ST_TILES - 1];
#pragma unroll
      for (int q = 0; q < G4; ++q) {
        const uint32_t r[4] = {x[q].x, x[q].y, x[q].z, x[q].w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if ((uint32_t)k < m[q]) {
            const uint32_t key = r[k] >> 26;
            const uint32_t pos = off[key] + rk[4 * q + k];
            stage[pos] = make_uint2(r[k], cur[key] - off[key]);
          }
      }
      __syncthreads();
      {
        const uint32_t w0 = (uint32_t)wv * (P2_CH / (P2_NT / 64)) + (uint32_t)lane;  // each wave a contiguous range
#pragma unroll
        for (int k = 0; k < P2_CH / P2_NT; ++k) {
          const uint32_t i = w0 + (uint32_t)k * 64;
          if (i < total) {
            const uint2 e = stage[i];
            records[e.y + i] = e.x;
          }
        }
      }
      if (threadIdx.x < ST_TILES) {
        cur[threadIdx.x] += cnt[threadIdx.x];
        cnt[threadIdx.x] = 0;
      }
      __syncthreads();
    }
  }
}

}  // namespace

size_t paged_pool_pages(size_t per) { return (per + PAGE - 1) / PAGE + PG_BINS + 1; }

hipError_t set_paged_attributes() {
  hipError_t e = hipFuncSetAttribute((const void*)k_pbin1<16384, 1024>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)pbin1_lds(16384));
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_p2place, hipFuncAttributeMaxDynamicSharedMemorySize, (int)P2PLACE_LDS);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)k_pfold, hipFuncAttributeMaxDynamicSharedMemorySize, (int)PFOLD_LDS);
}

hipError_t launch_paged_ingest(const PagedArgs& a, int phase, hipStream_t st) {
  const int ncu = a.num_cu;
  const uint32_t FS = (a.F + ST_TILES - 1) / ST_TILES;
  hipError_t e = hipSuccess;
  switch (phase) {
    case 0:  // this batch's direct tiles (a sample), then level 1 into the page pools
      hipLaunchKernelGGL(k_psample, dim3(PS_WG), dim3(1024), 0, st, a.series, a.n, a.S, a.F, a.pcount);
      hipLaunchKernelGGL(k_pselect, dim3(1), dim3(1024), 0, st, a.F, a.n, a.pcount, a.plan, a.thr_min, a.dmax);
      hipLaunchKernelGGL((k_pbin1<16384, 1024>), dim3(a.G), dim3(1024), pbin1_lds(16384), st, a.series, a.values, a.n,
                         a.per, a.S, a.F, a.plan, a.tb, a.state.sumfix, a.err, a.pool_pages, a.pool, a.plog, a.nlog,
                         a.tailpg, a.vec ? 1 : 0);
      break;
    case 1:  // the page directory and the items
      if ((e = hipMemsetAsync(a.pd, 0, 2 * PG_BINS * 4, st)) != hipSuccess) return e;
      hipLaunchKernelGGL(k_pdir_count, dim3(a.G), dim3(256), 0, st, a.plog, a.nlog, a.tailpg, a.pool_pages, a.pd);
      hipLaunchKernelGGL(k_pdir_scan, dim3(1), dim3(1024), 0, st, a.F, a.plan, a.pd);
      hipLaunchKernelGGL(k_pdir_fill, dim3(a.G), dim3(256), 0, st, a.plog, a.nlog, a.tailpg, a.pool_pages, a.pd,
                         a.dir);
      break;
    case 2:  // direct half-tiles folded into the state rows
      hipLaunchKernelGGL(k_pdir_init, dim3(DIRECT_MAX), dim3(256), 0, st, a.plan, a.state);
      hipLaunchKernelGGL(k_pfold, dim3(ncu), dim3(WG), PFOLD_LDS, st, a.pool, a.dir, a.pd, a.plan, a.F, a.state,
                         a.tb);
      break;
    default:  // level 2 of the other tiles into the final layout; the next batch's direct set
      hipLaunchKernelGGL(k_p2count, dim3(2 * ncu), dim3(WG), 0, st, a.pool, a.dir, a.pd, a.F, a.cnt2);
      hipLaunchKernelGGL(k_p2scan_a, dim3(FS), dim3(1024), 0, st, a.pd, a.F, a.cnt2, a.tot);
      hipLaunchKernelGGL(k_p2scan_b, dim3(1), dim3(1024), 0, st, a.F, a.tot, a.tile_base, a.err, a.err_host);
      hipLaunchKernelGGL(k_p2place, dim3(4 * ncu), dim3(P2_NT), P2PLACE_LDS, st, a.pool, a.dir, a.pd, a.F, a.cnt2,
                         a.tile_base, a.records);
      break;
  }
  return hipGetLastError();
}

}  // namespace l5dh
