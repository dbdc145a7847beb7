// l5dh_snapshot.hip -- snapshot-side kernels (Metric.Stat.snapshot/reset/summary,
// batched as AdminMetricsExportTelemeter.snapshotHistograms drives them).
//
//   k_plan_a/b     per tile: records over pending segments, cold/big, work items
//   k_hot_init     zero the rows big tiles accumulate into
//   k_accum_cold_h cold half-tile: 16 series in u16-packed LDS bins, fused summary +
//                  dense flush, or the sparse export's encoding (persistent, two
//                  workgroups per CU)
//   k_accum_split  big half-tile: (half, chunk) partial in u32 LDS bins, flushed
//                  with global atomics (persistent)
//   k_hot_finish   summaries of big tiles from their merged rows
//   k_rows         summaries / dense copies of state rows or external rows
//   k_fold1        one-tile series spaces folded into state rows at ingest
//
// Every (tile, half) key of a segment is one contiguous range of rec16 records
// (l5dh_kernels.hpp: series in tile | bucket; their value sums are in sumfix).
#include "l5dh_device.hpp"

namespace l5dh {
namespace {

// Records of key (t, h) in segment j.
struct KeyRange {
  const uint16_t* r16;
  uint32_t a, e;
};
__device__ __forceinline__ KeyRange seg_key(const Segs& sg, int j, uint32_t F, uint32_t t, uint32_t h) {
  const MetaLayout L = meta_layout(F);
  const uint32_t* m = sg.meta[j];
  const uint32_t k = 2 * t + h;
  const uint32_t a = m[L.kbase() + k], c = m[L.kcnt() + k];
  return KeyRange{sg.rec16[j], a, a + c};
}
__device__ __forceinline__ uint32_t seg_key_count(const Segs& sg, int j, uint32_t F, uint32_t k) {
  return sg.meta[j][meta_layout(F).kcnt() + k];
}

// k_plan_a / k_plan_b (ceil(F / 1024) workgroups each): k_plan_a classifies tile
// t = 1024 b + thread (cold: <= cold_limit records; else big, accumulated per half
// in chunks of hot_chunk records) and stores its workgroup's item counts in
// header[4 + k B + b]; k_plan_b scans those and writes the lists in tile order.
struct PlanCls {
  uint32_t ci, hot, si, h0, ec;  // ec: the tile's words in the unpacked encoding (sparse export)
};
__device__ __forceinline__ PlanCls plan_classify(const Segs& segs, uint32_t F, uint32_t t, uint32_t& tot,
                                                 int final_mode, uint32_t cold_limit, uint32_t hot_chunk) {
  uint32_t h0 = 0, h1 = 0;
  for (int j = 0; j < segs.n; ++j) {
    h0 += seg_key_count(segs, j, F, 2 * t);
    h1 += seg_key_count(segs, j, F, 2 * t + 1);
  }
  tot = h0 + h1;
  PlanCls r{0u, 0u, 0u, h0, 0u};
  if (tot > cold_limit) {
    r.hot = 1;
    r.si = (h0 + hot_chunk - 1) / hot_chunk + (h1 + hot_chunk - 1) / hot_chunk;
  } else if (final_mode || tot > 0) {
    r.ci = 1;
  }
  return r;
}

// (ENC_HALF_CAP's comment) the tile's words; h0w: those reserved for half 0 of a big or
// dirty tile
__device__ __forceinline__ uint32_t enc_half(uint32_t recs, bool dirty, uint32_t state_words) {
  const uint32_t w = dirty ? state_words + 2u * min(recs, 16u * NB) : min(recs, 16u * NB) + recs / MERGE_CMAX;
  return min(w + 16u, ENC_HALF_CAP);
}
__device__ __forceinline__ uint32_t enc_cap(const PlanCls& c, uint32_t tot, bool dirty, const Plan& plan, uint32_t t,
                                            uint32_t& h0w) {
  if (!c.hot && !dirty) return tot + TILE;
  const uint32_t dw0 = dirty ? plan.enc_dw[2 * t] : 0u, dw1 = dirty ? plan.enc_dw[2 * t + 1] : 0u;
  h0w = enc_half(c.h0, dirty, dw0);
  return h0w + enc_half(tot - c.h0, dirty, dw1);
}

__global__ __launch_bounds__(1024) void k_plan_a(Segs segs, uint32_t F, int final_mode, uint32_t cold_limit,
                                                 uint32_t hot_chunk, const uint8_t* __restrict__ dirty, int encode,
                                                 Plan plan) {
  __shared__ uint32_t red[4][17];
  const uint32_t t = blockIdx.x * 1024u + threadIdx.x;
  PlanCls c{0u, 0u, 0u, 0u, 0u};
  if (t < F) {
    uint32_t tot;
    c = plan_classify(segs, F, t, tot, final_mode, cold_limit, hot_chunk);
    uint32_t h0w = 0;
    if (encode) c.ec = enc_cap(c, tot, dirty[t] != 0, plan, t, h0w);
    plan.tile_tot[t] = tot;
  }
  const uint32_t v[4] = {c.ci, c.hot, c.si, c.ec};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t x = wave_sum((uint64_t)v[k]);
    if (lane == 0) red[k][w] = x;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    uint32_t x = 0;
    for (int q = 0; q < 16; ++q) x += red[threadIdx.x][q];
    plan.header[4 + threadIdx.x * gridDim.x + blockIdx.x] = x;
  }
}

__global__ __launch_bounds__(1024) void k_plan_b(Segs segs, uint32_t F, int final_mode, uint32_t cold_limit,
                                                 uint32_t hot_chunk, const uint8_t* __restrict__ dirty, int direct_out,
                                                 int encode, Plan plan) {
  __shared__ uint4 lds4[17];
  __shared__ uint32_t base[4];
  __shared__ uint32_t nbig;
  __shared__ uint4 big[64];  // {tile, first item, half-0 records, records}
  if (threadIdx.x == 0) nbig = 0;  // (visible after the scans' barriers)
  const uint32_t B = gridDim.x;
  {
    uint32_t x[4], tx[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) x[k] = threadIdx.x < blockIdx.x ? plan.header[4 + k * B + threadIdx.x] : 0u;
    block_excl_scan4<1024>(x, lds4, tx);
    if (threadIdx.x < 4) base[threadIdx.x] = tx[threadIdx.x];
    if (blockIdx.x == 0) {
      uint32_t y[4], ty[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = threadIdx.x < B ? plan.header[4 + k * B + threadIdx.x] : 0u;
      block_excl_scan4<1024>(y, lds4, ty);
      if (threadIdx.x == 0) {  // header: cold items, big tiles, cold-item counter, split items
        plan.header[0] = ty[0];
        plan.header[1] = ty[1];
        plan.header[2] = 0u;
        plan.header[3] = ty[2];
        plan.header[4 + 4 * B] = 0u;   // split-item counter
        plan.header[5 + 4 * B] = ty[3];  // the unpacked encoding's words
        if (plan.big_hint) *reinterpret_cast<volatile uint32_t*>(plan.big_hint) = ty[1];
      }
    }
  }
  __syncthreads();
  const uint32_t t = blockIdx.x * 1024u + threadIdx.x;
  PlanCls c{0u, 0u, 0u, 0u, 0u};
  uint32_t tot = 0, eh0 = 0;
  if (t < F) {
    c = plan_classify(segs, F, t, tot, final_mode, cold_limit, hot_chunk);
    if (encode) c.ec = enc_cap(c, tot, dirty[t] != 0, plan, t, eh0);
  }
  uint32_t pv[4] = {c.ci, c.hot, c.si, c.ec}, ptot[4];
  block_excl_scan4<1024>(pv, lds4, ptot);
  if (encode && t < F) {
    plan.enc_base[t] = base[3] + pv[3];
    plan.enc_h0[t] = eh0;
  }
  const uint32_t ca = base[0] + pv[0];
  const uint32_t xa = base[1] + pv[1];
  uint32_t sa = base[2] + pv[2];
  // a tile with many chunk items (C3's tile 0: ~1000) has them written by the whole
  // workgroup below, not by its one thread
  bool coop = false;
  if (t < F && c.hot && c.si > 32) {
    const uint32_t k = atomicAdd(&nbig, 1u);
    if (k < 64) {
      big[k] = make_uint4(t, sa, c.h0, tot);
      coop = true;
    }
  }
  if (t < F) {
    uint8_t flags = dirty[t] ? TF_DIRTY : 0;
    if (c.hot) {
      flags |= TF_SPLIT;
      // both halves one item each, clean, whole-range resetting snapshot into dense rows:
      // the items own their 16 output rows (no zeroing, no atomics, no finish pass)
      const uint32_t h1 = tot - c.h0;
      if (direct_out && !dirty[t] && c.h0 > 0 && c.h0 <= hot_chunk && h1 > 0 && h1 <= hot_chunk) flags |= TF_SOLO;
      for (uint32_t h = 0; !coop && h < 2; ++h) {
        const uint32_t nh = ((h ? tot - c.h0 : c.h0) + hot_chunk - 1) / hot_chunk;
        for (uint32_t q = 0; q < nh; ++q) plan.split_item[sa++] = make_uint2(t | (h << 15), q);
      }
      plan.hot_list[xa] = t;
    } else if (c.ci) {
      uint4 ci = make_uint4(t | (dirty[t] ? CI_DIRTY : 0u), 0u, 0u, 0u);
      if (segs.n > 0) {  // segment 0's key ranges (the cold kernel prefetches them with one load)
        const KeyRange r0 = seg_key(segs, 0, F, t, 0), r1 = seg_key(segs, 0, F, t, 1);
        ci.y = r0.a;
        ci.z = r1.a;
        ci.w = (r0.e - r0.a) | ((r1.e - r1.a) << 16);
      }
      plan.cold_item[ca] = ci;
    }
    plan.tile_flags[t] = flags;
  }
  __syncthreads();
  const uint32_t nb = min(nbig, 64u);
  for (uint32_t k = 0; k < nb; ++k) {
    const uint4 e = big[k];
    const uint32_t n0 = (e.z + hot_chunk - 1) / hot_chunk, n1 = (e.w - e.z + hot_chunk - 1) / hot_chunk;
    for (uint32_t i = threadIdx.x; i < n0 + n1; i += 1024) {
      const uint32_t h = i >= n0 ? 1u : 0u;
      plan.split_item[e.y + i] = make_uint2(e.x | (h << 15), h ? i - n0 : i);
    }
  }
}

// Where a big tile's counts accumulate: its state rows (stride ROW), or -- a clean
// tile of a resetting full-range snapshot with dense outputs (`direct`) -- its output
// rows (stride NB), so that k_hot_finish summarizes them in place instead of copying
// the state rows out (the state rows of a reset clean tile are never read again).
struct BigRows {
  uint32_t* base;
  uint32_t stride;
};
__device__ __forceinline__ BigRows big_rows(const State& st, const Outputs& out, const Plan& plan, uint32_t t,
                                            int direct_out) {
  if (direct_out && !(plan.tile_flags[t] & TF_DIRTY))
    return BigRows{reinterpret_cast<uint32_t*>(out.counts + ((size_t)t * TILE - out.first) * NB), (uint32_t)NB};
  return BigRows{st.counts + (size_t)t * TILE * ROW, (uint32_t)ROW};
}

// k_hot_init: big tiles accumulate with global atomics, so clean ones start from
// zero.  Persistent (the number of big tiles, header[1], is read on the device).
__global__ __launch_bounds__(256) void k_hot_init(Plan plan, State st, Outputs out, int direct_out) {
  const uint32_t nh = plan.header[1];
  for (uint32_t i = blockIdx.x; i < nh; i += gridDim.x) {
    const uint32_t t = plan.hot_list[i];
    if (plan.tile_flags[t] & (TF_DIRTY | TF_SOLO)) continue;
    const uint32_t s0 = t * TILE;
    const uint32_t s1 = min(st.S, s0 + TILE);
    if (direct_out) {  // the output rows: (s1 - s0) x 1798 int32, 8-B aligned
      uint2* p = reinterpret_cast<uint2*>(out.counts + (size_t)(s0 - out.first) * NB);
      const size_t n2 = (size_t)(s1 - s0) * NB / 2;
      for (size_t k = threadIdx.x; k < n2; k += 256) p[k] = make_uint2(0, 0);
    } else {
      uint4* p = reinterpret_cast<uint4*>(st.counts + (size_t)s0 * ROW);
      const size_t n4 = (size_t)(s1 - s0) * ROW / 4;
      for (size_t k = threadIdx.x; k < n4; k += 256) p[k] = make_uint4(0, 0, 0, 0);
    }
    if (threadIdx.x < s1 - s0) st.total[s0 + threadIdx.x] = 0;
  }
}

// One series of a tile whose new-record counts sit in LDS (`lds`, u16-packed or
// u32 row) and whose new samples sum to `vsum` (+ sumfix): merge with the old state if the
// tile is dirty, write the dense row(s), fold sumfix into the total and, in a
// final snapshot, emit the HistogramSummary.  One wave.
template <class SrcL>
__device__ __forceinline__ void emit_series(const SrcL& lds, uint32_t s, uint64_t vsum, int64_t fix, bool dirty,
                                            bool keep, int final_mode, State st, Tables tb, Outputs out) {
  const int lane = lane_id();
  const int ng = lane_groups(lane);
  const uint32_t oi = s - out.first;
  const bool emit = final_mode && s >= out.first && oi < out.count;
  int32_t* orow = (emit && out.counts) ? out.counts + (size_t)oi * NB : nullptr;
  uint32_t* srow = st.counts + (size_t)s * ROW;
  uint32_t g[9], nw = 0;
  if (!dirty) {
    // coalesced pass: lane l handles groups q = l + 64k (bins 4q..4q+3; 1798/1799 are
    // padding); even output rows are 16-B aligned and take one 16-B store per group
    const bool al16 = (oi & 1u) == 0u;
#pragma unroll 2
    for (int k = 0; k < 8; ++k) {
      const int q = lane + 64 * k;
      if (q < NB4) {
        const int b0 = 4 * q;
        const uint4 v = lds.get4(b0);
        if (orow) {
          if (al16 && b0 != 1796)
            *reinterpret_cast<uint4*>(orow + b0) = v;
          else
            store4_1798(orow, b0, v);
        }
        if (keep) store4_state(srow, b0, v);
      }
    }
    // blocked group sums for the summary scan (and the merge-encoding words)
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      g[q] = 0u;
      if (q < ng) {
        const uint4 v = lds.get4(28 * lane + 4 * q);
        g[q] = sum4(v);
        nw += merge_words4(v);
      }
    }
  } else {
    const SrcRow32 old{srow};
#pragma unroll
    for (int q = 0; q < 9; ++q) {
      g[q] = 0;
      if (q < ng) {
        const int b0 = 28 * lane + 4 * q;
        const uint4 v = lds.get4(b0);
        const uint4 o = old.get4(b0);
        const uint4 cmb = make_uint4(v.x + o.x, v.y + o.y, v.z + o.z, v.w + o.w);
        g[q] = sum4(cmb);
        nw += merge_words4(cmb);
        if (orow) store4_1798(orow, b0, cmb);
        store4_state(srow, b0, cmb);  // the merged row is also the summary source
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  }
  int64_t total = (int64_t)vsum + fix;  // fix = sumfix[s], read (and cleared) by the caller
  if (dirty) total += st.total[s];
  if (lane == 0 && keep) st.total[s] = total;
  if (lane == 0 && emit && out.totals) out.totals[oi] = total;
  if (emit) {
    Summary88* so = out.summ ? out.summ + oi : nullptr;
    put_words(nw, out.words ? out.words + oi : nullptr);
    if (dirty)
      wave_summary(g, SrcRow32{srow}, total, tb.mid, so);
    else
      wave_summary(g, lds, total, tb.mid, so);
  }
}

// Count a batch of K level-1 records per lane (~0u: no record): all bucket-LUT
// reads are issued before any LDS atomic (the compiler cannot move a read above an
// atomic it may alias), then per record one histogram atomic and one lane-private sum.
template <int K, class Hist, class Sum>
__device__ __forceinline__ void count_batch(const uint32_t (&rec)[K], const uint2* __restrict__ lut2, Hist&& hist_add,
                                            Sum&& sum_add) {
  uint2 lv[K];
#pragma unroll
  for (int k = 0; k < K; ++k) lv[k] = lut2[lut2_index(rec[k] & 0x1FFFFFu)];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    if (rec[k] == 0xFFFFFFFFu) continue;
    const uint32_t p = rec[k] & 0x1FFFFFu;
    uint32_t o;
    const uint32_t b = lut2_decode(p, lv[k], o);
    const bool esc = p >= V_ESC;
    hist_add((rec[k] >> 21) & 31u, sel_u32(esc, p - V_ESC, b));
    sum_add((rec[k] >> 21) & 31u, sel_u32(esc, 0u, p));
  }
}

// Level-2 records of one 16-B group (8 u16; m = valid records): bins only.
template <class Hist>
__device__ __forceinline__ void count16(uint4 x, uint32_t m, Hist&& hist_add) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if ((uint32_t)k >= m) continue;
    const uint32_t r = (w[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
    hist_add(r >> 11, r & 2047u);
  }
}

// The records of both halves of tile t in every segment: per segment, the two
// ranges are walked together (a thread's loads of both halves in flight at once).
// Ranges start 16-B aligned (rec16 regions at multiples of 8).
template <int NT, class Hist>
__device__ __forceinline__ void count_tile(const Segs& sg, uint32_t F, uint32_t t, Hist&& hist_add) {
  for (int j = 0; j < sg.n; ++j) {
    const KeyRange r0 = seg_key(sg, j, F, t, 0), r1 = seg_key(sg, j, F, t, 1);
    const uint32_t n0 = r0.e - r0.a, n1 = r1.e - r1.a;
    const uint32_t g0 = (n0 + 7) / 8, g1 = (n1 + 7) / 8, gm = max(g0, g1);
    const uint4* p0 = reinterpret_cast<const uint4*>(r0.r16 + r0.a);
    const uint4* p1 = reinterpret_cast<const uint4*>(r1.r16 + r1.a);
    for (uint32_t g = threadIdx.x; g < gm; g += NT) {
      const uint4 x = g < g0 ? p0[g] : make_uint4(0u, 0u, 0u, 0u);
      const uint4 y = g < g1 ? p1[g] : make_uint4(0u, 0u, 0u, 0u);
      count16(x, g < g0 ? min(8u, n0 - 8 * g) : 0u, hist_add);
      count16(y, g < g1 ? min(8u, n1 - 8 * g) : 0u, hist_add);
    }
  }
}


// k_accum_cold_h: the cold tiles as half-tile items -- 16 series in one u16-packed LDS
// histogram (57.6 KB), 512-thread workgroups, two per CU, so one workgroup counts
// while the other emits its rows (round 4: -0.12 ms of accumulate against one whole
// tile per 1024-thread workgroup, which held one tile in flight per CU).
// Item i is half i & 1 of cold item i >> 1.  ENCODE: the fleet merge's sparse export
// (row encodings, no rows or summaries); half 1's rows start past half 0's room in
// the tile's encoding range (h0 + 16 words for a clean tile: a row's words never
// exceed its records; Plan::enc_h0 for a dirty one).
#ifdef L5DH_PHASES  // development: per-workgroup phase times of k_accum_cold_h
__device__ unsigned long long g_phase2[1024 * 8];
#define PH_INIT unsigned long long ph_acc[4] = {0, 0, 0, 0}, ph_t = wall_clock64();
#define PH_MARK(k)                                 \
  if (threadIdx.x == 0) {                          \
    const unsigned long long ph_n = wall_clock64(); \
    ph_acc[k] += ph_n - ph_t;                      \
    ph_t = ph_n;                                   \
  }
#define PH_FLUSH                                                          \
  if (threadIdx.x == 0) {                                                 \
    for (int k = 0; k < 4; ++k) g_phase2[blockIdx.x * 8 + k] += ph_acc[k]; \
    g_phase2[blockIdx.x * 8 + 7] += 1;                                    \
  }
#else
#define PH_INIT
#define PH_MARK(k)
#define PH_FLUSH
#endif
constexpr int HSER = 16;
template <bool ENCODE>
__global__ __launch_bounds__(512, 2) void k_accum_cold_h(Segs segs, Plan plan, State st, Tables tb, Outputs out,
                                                         uint32_t cold_arg, int final_mode, int reset) {
  constexpr int NT = 512;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t cold_tiles = cold_arg != DEV_COUNT ? cold_arg : plan.header[0];
  const uint32_t nitems = 2u * cold_tiles;
  uint32_t* hist = smem;                                             // [16][900] u16 pairs
  int64_t* fixl = reinterpret_cast<int64_t*>(smem + HSER * CROW);    // [16] sumfix of the item's series
  int32_t* midl = reinterpret_cast<int32_t*>(fixl + HSER);           // [NB] bucket midpoints
  const int w = threadIdx.x >> 6;
  const int lane = lane_id();
  const bool keep = !(final_mode && reset);
  const uint32_t F = st.F;
  Tables tbl = tb;
  tbl.mid = midl;
  auto hist_add = [&](uint32_t loc, uint32_t b) {
    atomicAdd(&hist[(loc & (HSER - 1)) * CROW + (b >> 1)], (b & 1u) ? 0x10000u : 1u);
  };
  // (sparse export) per row, the buckets in the order they were first touched: the
  // returning add tells a first touch; tcnt[par][row] counts them (= the row's words:
  // a cold row's counts stay below the escape), the first ENC_LIST are listed
  uint32_t* tcnt = reinterpret_cast<uint32_t*>(midl + ROW);      // [2][HSER] (double-buffered by item parity)
  uint16_t* tlist = reinterpret_cast<uint16_t*>(tcnt + 2 * HSER);  // [HSER][ENC_LIST]
  int par = 0;
  // (batching the 8 adds of a group and listing the first touches after them measured
  // +0.02 ms per C4 rank, round 5)
  auto hist_add_enc = [&](uint32_t loc, uint32_t b) {
    const uint32_t l = loc & (HSER - 1);
    const uint32_t old = atomicAdd(&hist[l * CROW + (b >> 1)], (b & 1u) ? 0x10000u : 1u);
    if ((((b & 1u) ? old >> 16 : old) & 0xFFFFu) == 0u) {
      const uint32_t k = atomicAdd(&tcnt[par * HSER + l], 1u);
      if (k < (uint32_t)ENC_LIST) tlist[l * ENC_LIST + k] = (uint16_t)b;
    }
  };
  {
    uint4* p = reinterpret_cast<uint4*>(smem);
    for (int i = threadIdx.x; i < HSER * CROW / 4; i += NT) p[i] = make_uint4(0, 0, 0, 0);
    for (int i = threadIdx.x; i < NB; i += NT) midl[i] = tb.mid[i];
    if (ENCODE && threadIdx.x < 2 * HSER) tcnt[threadIdx.x] = 0u;
  }
  // the next item's entry is loaded one item ahead; its sumfix and (one pending
  // segment) each thread's first 16-B group during this item's emission
  const bool one = segs.n == 1;
  uint32_t t = 0, a = 0, nn = 0, hf = 0, eb = 0, h0e = 0;
  bool dirty = false;
  int64_t fraw = 0;
  uint4 x0 = make_uint4(0u, 0u, 0u, 0u);
  const uint16_t* const b16 = segs.rec16[0];
  auto fetch = [&](uint4 ci, uint32_t half) {
    asm volatile("" : "+v"(ci.x), "+v"(ci.y), "+v"(ci.z), "+v"(ci.w));
    const uint32_t cx = __builtin_amdgcn_readfirstlane(ci.x), cw = __builtin_amdgcn_readfirstlane(ci.w);
    t = cx & 0x7FFFu;
    hf = half;
    dirty = (cx & CI_DIRTY) != 0u;
    a = __builtin_amdgcn_readfirstlane(half ? ci.z : ci.y);
    nn = half ? cw >> 16 : cw & 0xFFFFu;
    h0e = cw & 0xFFFFu;  // (sparse export) half 0's records in segment 0: the whole count with one segment
    if (one) {
      const uint32_t g = threadIdx.x;
      x0 = *reinterpret_cast<const uint4*>(b16 + (8 * g < nn ? a + 8 * g : a));
    }
    fraw = st.sumfix[min(t * TILE + HSER * half + (threadIdx.x & (HSER - 1)), st.S - 1)];
    if (ENCODE) eb = plan.enc_base[t];
  };
  __shared__ uint32_t rwl[HSER];  // (sparse export) words of the item's rows
  const uint4* __restrict__ citem = plan.cold_item;
  const uint32_t last = cold_tiles ? cold_tiles - 1u : 0u;
  // items: blockIdx.x, blockIdx.x + G, then from the counter, asked two items ahead (the
  // sparse export: blockIdx.x + k G)
  __shared__ uint32_t s_next[2];
  uint32_t* const ctr = plan.header + 2;  // zeroed by k_plan_b
  const uint32_t G2 = 2u * gridDim.x;
  if (!ENCODE && threadIdx.x == 0) s_next[0] = G2 + atomicAdd(ctr, 1u);
  uint32_t item = blockIdx.x, item1 = blockIdx.x + gridDim.x;
  if (item < nitems) fetch(citem[item >> 1], item & 1u);
  uint4 cn = citem[min(item1 >> 1, last)];
  __syncthreads();
  PH_INIT
  for (; item < nitems; par ^= 1) {
    const uint32_t tc = t, hc = hf, ebc = eb, h0c = h0e, ac = a, nc = nn;
    const bool dc = dirty;
    const uint4 xc = x0;
    const int64_t fc = fraw;
    uint32_t item2 = 0, asked = 0;
    if (ENCODE) {
      // (sparse items emit little: the next item's entry fields and loads, its successor's
      // entry and the counter ask go in flight here, ahead of this item's count)
      // static item order: the counter's returning atomic, waited for inside every short
      // item, cost the sparse export 0.80 -> 0.56 ms per C4 rank (profiles/r04r_ab.txt)
      item2 = item1 + gridDim.x;
      fetch(cn, item1 & 1u);
      cn = citem[min(item2 >> 1, last)];
    }
    if (threadIdx.x < HSER) {
      const uint32_t s = tc * TILE + HSER * hc + threadIdx.x;
      const int64_t f = s < st.S ? fc : 0;
      fixl[threadIdx.x] = f;
      if (f) st.sumfix[s] = 0;
    }
    if (one) {
      const uint32_t g0 = (nc + 7) / 8;
      const uint4* p0 = reinterpret_cast<const uint4*>(b16 + ac);
      uint4 x = xc;
      for (uint32_t g = threadIdx.x; g < g0; g += NT) {
        const uint4 cx = x;
        const uint32_t gn = g + NT;
        x = gn < g0 ? p0[gn] : make_uint4(0u, 0u, 0u, 0u);
        if (ENCODE && !dc)
          count16(cx, min(8u, nc - 8 * g), hist_add_enc);
        else
          count16(cx, min(8u, nc - 8 * g), hist_add);
      }
    } else {
      for (int j = 0; j < segs.n; ++j) {
        const KeyRange r = seg_key(segs, j, F, tc, hc);
        const uint32_t n = r.e - r.a, g0 = (n + 7) / 8;
        const uint4* p = reinterpret_cast<const uint4*>(r.r16 + r.a);
        for (uint32_t g = threadIdx.x; g < g0; g += NT) {
          if (ENCODE && !dc)
            count16(p[g], min(8u, n - 8 * g), hist_add_enc);
          else
            count16(p[g], min(8u, n - 8 * g), hist_add);
        }
      }
    }
    __syncthreads();  // counts complete; fixl visible
    PH_MARK(0)
    if (ENCODE && threadIdx.x < HSER) tcnt[(par ^ 1) * HSER + threadIdx.x] = 0u;  // the next item's (counted after the end barrier)
    if (!ENCODE) {
      fetch(cn, item1 & 1u);  // (past the last item: a harmless refetch)
      item2 = s_next[par];
      if (threadIdx.x == 0) asked = G2 + atomicAdd(ctr, 1u);
      cn = citem[min(item2 >> 1, last)];
    }
    const uint32_t s0 = tc * TILE + HSER * hc;
    const uint32_t oi0 = s0 - out.first;
    const bool linear = !keep && !dc && out.counts != nullptr && s0 >= out.first && oi0 + HSER <= out.count &&
                        s0 + HSER <= st.S && (oi0 & 1u) == 0u;
    if (ENCODE && !dc) {
      // a clean item: each row's words = its first touches; entries in touch order (the
      // decoder adds a source's entries in any order) with the counts from the bins;
      // only the touched bins are cleared.  A row with more than ENC_LIST touches is
      // encoded and cleared from its whole bin row.
      const uint32_t* tc16 = tcnt + par * HSER;
      uint32_t hb = ebc;
      if (hc) {
        uint32_t h0 = h0c;
        if (!one)
          for (int j = 1; j < segs.n; ++j) h0 += seg_key_count(segs, j, F, 2 * tc);
        hb += h0 + HSER;
      }
      PH_MARK(3)
      for (int loc = w; loc < HSER; loc += NT / 64) {
        const uint32_t s = s0 + loc;
        const uint32_t n = tc16[loc];
        uint32_t at = hb;
        for (int l = 0; l < loc; ++l) at += tc16[l];
        uint32_t* row = hist + loc * CROW;
        if (s < st.S) {
          if (n <= (uint32_t)ENC_LIST) {
            for (uint32_t i = (uint32_t)lane; i < n; i += 64) {
              const uint32_t b = tlist[loc * ENC_LIST + i];
              const uint32_t c = (row[b >> 1] >> ((b & 1u) * 16)) & 0xFFFFu;
              out.enc[at + i] = (b << 21) | c;
            }
          } else {
            row_encode(SrcLds16{row}, out.enc, at);
          }
          if (lane == 0) {
            const uint32_t oi = s - out.first;
            out.roff[oi] = at;
            out.words[oi] = n;
            if (out.totals) out.totals[oi] = fixl[loc];
          }
        }
        if (n <= (uint32_t)ENC_LIST) {  // (a wave's LDS ops stay in order: the reads above come first)
          for (uint32_t i = (uint32_t)lane; i < n; i += 64) row[tlist[loc * ENC_LIST + i] >> 1] = 0u;
        } else {
          uint4* hr = reinterpret_cast<uint4*>(row);
          for (int i = lane; i < CROW / 4; i += 64) hr[i] = make_uint4(0u, 0u, 0u, 0u);
        }
      }
      PH_MARK(1)
    } else if (ENCODE) {
      for (int loc = w; loc < HSER; loc += NT / 64) {
        const uint32_t s = s0 + loc;
        uint32_t nw = 0;
        if (s < st.S)
          nw = dc ? row_words(SrcSum2<SrcLds16, SrcRow32>{SrcLds16{hist + loc * CROW}, SrcRow32{st.counts + (size_t)s * ROW}})
                  : row_words(SrcLds16{hist + loc * CROW});
        if (lane == 0) rwl[loc] = nw;
      }
      uint32_t hb = ebc;  // this half's first word
      if (hc) {
        if (dc) {
          hb += plan.enc_h0[tc];
        } else {
          uint32_t h0 = h0c;
          for (int j = 1; j < segs.n; ++j) h0 += seg_key_count(segs, j, F, 2 * tc);
          hb += h0 + HSER;
        }
      }
      __syncthreads();  // rwl complete
      for (int loc = w; loc < HSER; loc += NT / 64) {
        const uint32_t s = s0 + loc;
        if (s < st.S) {
          uint32_t at = hb;
          for (int l = 0; l < loc; ++l) at += rwl[l];
          if (dc)
            row_encode(SrcSum2<SrcLds16, SrcRow32>{SrcLds16{hist + loc * CROW}, SrcRow32{st.counts + (size_t)s * ROW}},
                       out.enc, at);
          else
            row_encode(SrcLds16{hist + loc * CROW}, out.enc, at);
          if (lane == 0) {
            const uint32_t oi = s - out.first;
            out.roff[oi] = at;
            out.words[oi] = rwl[loc];
            if (out.totals) out.totals[oi] = fixl[loc] + (dc ? st.total[s] : 0);
          }
        }
        uint4* hr = reinterpret_cast<uint4*>(hist + loc * CROW);  // cleared for the next item
        for (int i = lane; i < CROW / 4; i += 64) hr[i] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    // (two series' summaries interleaved per wave, unrolled: accumulate +0.02 ms, round 5)
    for (int loc = w; !ENCODE && loc < HSER; loc += NT / 64) {
      const uint32_t s = s0 + loc;
      const uint32_t* row = hist + loc * CROW;
      if (s < st.S) {
        if (linear) {
          const int ng = lane_groups(lane);
          uint32_t g[9], nw = 0;
          if (out.words) {  // (the merge encoding's words: the all-reduce export only)
#pragma unroll
            for (int q = 0; q < 9; ++q) {
              g[q] = 0u;
              if (q < ng) {
                const uint4 v = SrcLds16{row}.get4(28 * lane + 4 * q);
                g[q] = sum4(v);
                nw += merge_words4(v);
              }
            }
            put_words(nw, out.words + (s - out.first));
          } else {
#pragma unroll
            for (int q = 0; q < 9; ++q) g[q] = q < ng ? SrcLds16{row}.sum4(28 * lane + 4 * q) : 0u;
          }
          wave_summary<SrcLds16, true>(g, SrcLds16{row}, fixl[loc], midl, out.summ ? out.summ + (s - out.first) : nullptr);
          if (lane == 0 && out.totals) out.totals[s - out.first] = fixl[loc];
        } else {
          emit_series(SrcLds16{row}, s, 0, fixl[loc], dc, keep, final_mode, st, tbl, out);
        }
      }
      if (!linear) {
        uint4* hr = reinterpret_cast<uint4*>(hist + loc * CROW);
        for (int i = lane; i < CROW / 4; i += 64) hr[i] = make_uint4(0u, 0u, 0u, 0u);
      }
    }
    if (linear) {
      __syncthreads();  // the summaries have read the rows
      PH_MARK(1)
      uint4* o = reinterpret_cast<uint4*>(out.counts + (size_t)oi0 * NB);
      constexpr int NCH = HSER * NB / 4;
      for (int c = threadIdx.x; c < NCH; c += NT) {
        const int e0 = 4 * c;
        const int r0 = e0 / NB, b0 = e0 - r0 * NB;
        uint32_t* p0 = hist + r0 * CROW + (b0 >> 1);
        uint32_t* p1 = b0 == NB - 2 ? hist + (r0 + 1) * CROW : p0 + 1;
        const uint32_t x = *p0, y = *p1;
        *p0 = 0u;
        *p1 = 0u;
        // (nontemporal: the dense rows are the step's output, not read again by it: C3 -0.03 ms;
        // nontemporal record stores in level 1 took it from 3.3 to 5.7 ms, round 5)
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v4 = {x & 0xFFFFu, x >> 16, y & 0xFFFFu, y >> 16};
        __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(o + c));
      }
    }
    if (threadIdx.x == 0) {
      st.dirty[tc] = keep ? 1 : 0;
      if (!ENCODE) s_next[par ^ 1] = asked;
    }
    __syncthreads();
    PH_MARK(2)
    item = item1;
    item1 = item2;
  }
  PH_FLUSH
}

// One-tile series spaces (S <= 32: C1, the head shard of a many-way C3) fold each
// batch into the tile's state rows at ingest -- no records, no partition, no
// segment.  k_fold1_init clears the rows of a clean tile and marks it dirty;
// k_fold1 items are chunks of the batch: u16-packed LDS bins of the 32 series with a
// 2^15 hand-off to the state row (or u32 bins for <= 16 series), nonzero bins flushed
// with global atomics, lane-private u64 value sums into total; escapes go to sumfix
// as at ingest.  Invalid ids are dropped and counted.
__global__ __launch_bounds__(256) void k_fold1_init(State st) {
  const bool clean = st.dirty[0] == 0;
  if (clean) {
    uint4* p = reinterpret_cast<uint4*>(st.counts);
    const size_t n4 = (size_t)st.S * ROW / 4;
    for (size_t k = threadIdx.x; k < n4; k += 256) p[k] = make_uint4(0, 0, 0, 0);
    if (threadIdx.x < st.S) st.total[threadIdx.x] = 0;
  }
  __syncthreads();  // every thread has read the flag
  if (clean && threadIdx.x == 0) st.dirty[0] = 1;
}

template <bool W32>
__global__ __launch_bounds__(WG) void k_fold1(const uint32_t* __restrict__ series, const float* __restrict__ values,
                                              size_t n, uint32_t chunk, State st, Tables tb, uint32_t* __restrict__ err,
                                              int vec) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  constexpr int NSER = W32 ? 16 : TILE;
  constexpr int RW = W32 ? HROW : CROW;                                                 // LDS words per series row
  uint32_t* hist = smem;                                                                // [NSER][RW] u32 / u16 pairs
  unsigned long long* vsl = reinterpret_cast<unsigned long long*>(smem + NSER * RW);    // [NSER][64]
  uint2* lut2 = reinterpret_cast<uint2*>(vsl + NSER * 64);                              // [LUT2_N]
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  const uint32_t S = st.S;
  for (int i = threadIdx.x; i < LUT2_N; i += WG) lut2[i] = tb.lut2[i];
  bool bad = false;
  auto enc = [&](uint32_t s, float f) -> uint32_t {
    if (s >= S) {
      bad = true;
      return 0xFFFFFFFFu;
    }
    return ((s & (TILE - 1)) << 21) | payload1(s, f, tb, st.sumfix);
  };
  auto hist_add = [&](uint32_t loc, uint32_t b) {
    if (W32) {
      atomicAdd(&hist[(loc & (NSER - 1)) * RW + b], 1u);
      return;
    }
    const uint32_t sh = (b & 1u) * 16u;
    uint32_t* wd = &hist[(loc & 31u) * CROW + (b >> 1)];
    const uint32_t old = atomicAdd(wd, 1u << sh);
    if (((old >> sh) & 0xFFFFu) == 0x7FFFu) {  // this add made it 2^15: hand 2^15 over
      atomicSub(wd, 0x8000u << sh);
      atomicAdd(&st.counts[(size_t)(loc & 31u) * ROW + b], 0x8000u);
    }
  };
  auto sum_add = [&](uint32_t loc, uint32_t v) {
    atomicAdd(&vsl[(loc & (NSER - 1)) * 64 + lane], (unsigned long long)v);
  };
  const size_t nitems = (n + chunk - 1) / chunk;
  for (size_t item = blockIdx.x; item < nitems; item += gridDim.x) {
    {
      uint4* q = reinterpret_cast<uint4*>(smem);
      for (int i = threadIdx.x; i < (NSER * RW + NSER * 64 * 2) / 4; i += WG) q[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const size_t lo = item * chunk, hi = lo + chunk < n ? lo + chunk : n;
    if (vec) {  // 16-B loads (lo is a multiple of chunk, itself of 4); one group ahead in flight
      // whole groups [lo, hi4) with unconditional loads (a group past the end reloads the
      // last whole one; masked where used), so the next groups stay in flight; then the
      // batch's ragged end, at most 3 samples
      const size_t hi4 = lo + ((hi - lo) & ~(size_t)3);
      if (hi4 > lo) {
        auto ld = [&](size_t g, uint4& sv, uint4& vv) {
          const size_t gc = g < hi4 ? g : hi4 - 4;
          sv = *reinterpret_cast<const uint4*>(series + gc);
          vv = *reinterpret_cast<const uint4*>(values + gc);
        };
        size_t g = lo + 4u * threadIdx.x;
        uint4 s0, v0, s1, v1;
        ld(g, s0, v0);
        ld(g + 4u * WG, s1, v1);
        for (size_t c = lo; c < hi4; c += 8u * WG, g += 8u * WG) {
          const uint4 cs0 = s0, cv0 = v0, cs1 = s1, cv1 = v1;
          ld(g + 8u * WG, s0, v0);
          ld(g + 12u * WG, s1, v1);
          const uint32_t ss[8] = {cs0.x, cs0.y, cs0.z, cs0.w, cs1.x, cs1.y, cs1.z, cs1.w};
          const uint32_t vv[8] = {cv0.x, cv0.y, cv0.z, cv0.w, cv1.x, cv1.y, cv1.z, cv1.w};
          uint32_t x[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const size_t gk = g + (k >> 2) * 4u * WG + (k & 3);
            x[k] = gk < hi4 ? enc(ss[k], __uint_as_float(vv[k])) : 0xFFFFFFFFu;
          }
          count_batch<8>(x, lut2, hist_add, sum_add);
        }
      }
      if (threadIdx.x < hi - hi4) {
        const size_t g = hi4 + threadIdx.x;
        const uint32_t x[1] = {enc(series[g], values[g])};
        count_batch<1>(x, lut2, hist_add, sum_add);
      }
    } else {
      for (size_t g = lo + threadIdx.x; g < hi; g += WG) {
        const uint32_t x[1] = {enc(series[g], values[g])};
        count_batch<1>(x, lut2, hist_add, sum_add);
      }
    }
    __syncthreads();
    for (int loc = w; loc < NSER; loc += WG / 64) {
      if ((uint32_t)loc >= S) continue;
      const uint64_t vsum = wave_sum(vsl[loc * 64 + lane]);
      uint32_t* grow = st.counts + (size_t)loc * ROW;
      const uint32_t* hrow = hist + loc * RW;
      for (int b0 = 0; b0 < NB; b0 += 64) {  // 64 consecutive bins per wave atomic
        const int b = b0 + lane;
        const uint32_t v = b >= NB ? 0u : W32 ? hrow[b] : (hrow[b >> 1] >> ((b & 1) * 16)) & 0xFFFFu;
        if (__ballot(v != 0u)) {
          if (v) atomicAdd(&grow[b], v);
        }
      }
      if (lane == 0 && vsum) atomicAdd(reinterpret_cast<unsigned long long*>(&st.total[loc]), (unsigned long long)vsum);
    }
    __syncthreads();  // the LDS rows are read: the next item may clear them
  }
  if (bad) atomicAdd(err, 1u);  // monotonic: the host compares it with the count it already reported
}

// Big tiles: item = (tile, half, chunk of hot_chunk records of that half across the
// pending segments; each segment holds the half as one contiguous range).  u32 LDS
// bins for the half's 16 series, flushed with global atomics (k_hot_init cleared the
// rows; k_hot_finish summarizes them); the exact sums are already in sumfix.
__global__ __launch_bounds__(WG) void k_accum_split(Segs segs, Plan plan, State st, Tables tb, Outputs out,
                                                    int direct_out, uint32_t hot_chunk) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  const uint32_t nitems = plan.header[3];  // persistent: items blockIdx.x, + gridDim.x, ...
  const uint32_t F = st.F;
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  uint32_t* hist = smem;  // [16][1800]
  auto hist_add = [&](uint32_t loc, uint32_t b) { atomicAdd(&hist[(loc & 15u) * HROW + b], 1u); };
  // items: blockIdx.x first, then from a counter (G, G + 1, ...) as workgroups finish
  __shared__ uint32_t s_item;
  uint32_t* const ctr = plan.header + 4 + 4 * ((F + 1023) / 1024);  // zeroed by k_plan_b
  for (uint32_t item = blockIdx.x; item < nitems; item = s_item) {
    const uint2 it = plan.split_item[item];
    const uint32_t t = it.x & 0x7FFFu, half = (it.x >> 15) & 1u;
    {
      uint4* q = reinterpret_cast<uint4*>(smem);
      for (int i = threadIdx.x; i < 16 * HROW / 4; i += WG) q[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    const uint64_t vlo = (uint64_t)it.y * hot_chunk, vhi = vlo + hot_chunk;
    uint64_t vbase = 0;
    for (int j = 0; j < segs.n; ++j) {
      const KeyRange r = seg_key(segs, j, F, t, half);
      const uint64_t len = r.e - r.a;
      const uint64_t lo = vlo > vbase ? vlo : vbase;
      const uint64_t hi = vhi < vbase + len ? vhi : vbase + len;
      const uint64_t skip = lo - vbase;
      vbase += len;
      if (lo >= hi) continue;
      // [a, e) of this range; hot_chunk is a multiple of 1024, so a chunk starts 16-B aligned
      const uint32_t a = r.a + (uint32_t)skip, e = a + (uint32_t)(hi - lo);
      // loads are unconditional (a group past the range reloads the first one; records
      // outside [a, e) are masked where they are used), so the next groups stay in flight
      // while this one is counted
      {
        const uint32_t a8 = a & ~7u;
        auto ld = [&](uint32_t g) { return *reinterpret_cast<const uint4*>(r.r16 + (g < e ? g : a8)); };
        uint32_t g = a8 + 8u * threadIdx.x;
        uint4 n0 = ld(g), n1 = ld(g + 8u * WG);
        for (uint32_t c = a8; c < e; c += 16u * WG, g += 16u * WG) {
          const uint4 x0 = n0, x1 = n1;
          n0 = ld(g + 16u * WG);
          n1 = ld(g + 24u * WG);
          const uint4 xs[2] = {x0, x1};
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const uint32_t wd[4] = {xs[q].x, xs[q].y, xs[q].z, xs[q].w};
            const uint32_t gq = g + (uint32_t)q * 8u * WG;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const uint32_t gk = gq + (uint32_t)k;
              if (gk < a || gk >= e) continue;
              const uint32_t rr = (wd[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
              hist_add(rr >> 11, rr & 2047u);
            }
          }
        }
      }
    }
    __syncthreads();
    const uint32_t s = t * TILE + 16 * half + w;
    if (plan.tile_flags[t] & TF_SOLO) {
      // this item holds every record of the half: wave w writes series w's output row,
      // total and summary (direct_out: out.first == 0, the tile is clean, reset)
      if (s < st.S) {
        const SrcLds32 src{hist + w * HROW};
        const int64_t total = st.sumfix[s];
        uint32_t g[9];
        row_pass(src, g, out.counts + (size_t)s * NB, out.words ? out.words + s : nullptr);
        wave_summary(g, src, total, tb.mid, out.summ ? out.summ + s : nullptr);
        if (lane == 0) {
          st.sumfix[s] = 0;
          st.total[s] = total;
          if (out.totals) out.totals[s] = total;
        }
      }
      if (threadIdx.x == 0 && half == 0) st.dirty[t] = 0;
    } else if (s < st.S) {
      const BigRows br = big_rows(st, out, plan, t, direct_out);
      uint32_t* grow = br.base + (size_t)(16 * half + w) * br.stride;
      const uint32_t* hrow = hist + w * HROW;
      for (int b0 = 0; b0 < NB; b0 += 64) {  // 64 consecutive bins per wave atomic
        const int b = b0 + lane;
        const uint32_t v = b < NB ? hrow[b] : 0u;
        if (__ballot(v != 0u)) {
          if (v) atomicAdd(&grow[b], v);
        }
      }
    }
    if (threadIdx.x == 0) s_item = gridDim.x + atomicAdd(ctr, 1u);
    __syncthreads();  // the LDS rows are read: the next item may clear them; the next index visible
  }
}

// k_hot_finish: per (big tile, half): fold sumfix, summarize the merged rows,
// write outputs, update state/dirty.
__global__ __launch_bounds__(WG) void k_hot_finish(Plan plan, State st, Tables tb, Outputs out, int final_mode,
                                                   int reset, int direct_out) {
  const uint32_t nv = 2 * plan.header[1];  // persistent: (big tile, half) pairs
  __shared__ uint32_t rw16[16];  // (sparse export) words of the half's rows
  for (uint32_t vb = blockIdx.x; vb < nv; vb += gridDim.x) {
    const uint32_t t = plan.hot_list[vb >> 1];
    const uint32_t half = vb & 1u;
    if (plan.tile_flags[t] & TF_SOLO) continue;  // written by its k_accum_split items
    const int lane = lane_id();
    const int w = threadIdx.x >> 6;
    const uint32_t s = t * TILE + 16 * half + w;
    if (out.enc) {
      // sparse export (the rows are the state rows: no direct_out): each row's words, then
      // its entries in the half's range of the tile's unpacked encoding
      const SrcRow32 src{st.counts + (size_t)s * ROW};
      const uint32_t nw = s < st.S ? row_words(src) : 0u;
      if (lane == 0) rw16[w] = nw;
      __syncthreads();
      if (s < st.S) {
        uint32_t at = plan.enc_base[t] + (half ? plan.enc_h0[t] : 0u);
        for (int l = 0; l < w; ++l) at += rw16[l];
        row_encode(src, out.enc, at);
        if (lane == 0) {
          const uint32_t oi = s - out.first;
          out.roff[oi] = at;
          out.words[oi] = nw;
          if (out.totals) out.totals[oi] = st.total[s] + st.sumfix[s];
          st.sumfix[s] = 0;
        }
      }
      if (threadIdx.x == 0 && half == 0) st.dirty[t] = 0;
      __syncthreads();  // rw16 read before the next pair's
      continue;
    }
    if (s < st.S) {
      int64_t total = st.total[s] + st.sumfix[s];
      if (final_mode) {
        const uint32_t oi = s - out.first;
        if (s >= out.first && oi < out.count) {
          uint32_t g[9];
          uint32_t* wo = out.words ? out.words + oi : nullptr;
          if (direct_out && !(plan.tile_flags[t] & TF_DIRTY)) {  // counted in the output row itself
            const SrcExt src{out.counts + (size_t)oi * NB};
            row_pass(src, g, nullptr, wo);
            wave_summary(g, src, total, tb.mid, out.summ ? out.summ + oi : nullptr);
          } else {
            const SrcRow32 src{st.counts + (size_t)s * ROW};
            row_pass(src, g, out.counts ? out.counts + (size_t)oi * NB : nullptr, wo);
            wave_summary(g, src, total, tb.mid, out.summ ? out.summ + oi : nullptr);
          }
          if (lane == 0 && out.totals) out.totals[oi] = total;
        }
      }
      if (lane == 0) {
        st.sumfix[s] = 0;
        st.total[s] = total;
      }
    }
    if (threadIdx.x == 0 && half == 0) st.dirty[t] = (final_mode && reset) ? 0 : 1;
  }
}

// k_rows: one wave per series: summary / dense copy of state rows (range
// snapshot, export) or of external dense rows (fleet merge).
__global__ __launch_bounds__(256) void k_rows(State st, const int32_t* __restrict__ ext,
                                              const int64_t* __restrict__ ext_total, Tables tb, Outputs out, int reset,
                                              int64_t* __restrict__ totals_out) {
  const uint32_t i = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= out.count) return;
  const int lane = lane_id();
  uint32_t g[9];
  int32_t* orow = out.counts ? out.counts + (size_t)i * NB : nullptr;
  if (ext) {
    const SrcExt src{ext + (size_t)i * NB};
    const int64_t total = ext_total ? ext_total[i] : 0;
    row_pass(src, g, orow);
    if (out.summ) wave_summary(g, src, total, tb.mid, out.summ + i);
    if (totals_out && lane == 0) totals_out[i] = total;
    return;
  }
  const uint32_t s = out.first + i;
  const bool dirty = st.dirty[s >> TILE_SHIFT] != 0;
  if (dirty) {
    const SrcRow32 src{st.counts + (size_t)s * ROW};
    // + sumfix: a one-tile space's fold leaves its escaped samples' sums there (a fold of
    // segments into the state has moved them into `total` already: 0 then)
    const int64_t total = st.total[s] + st.sumfix[s];
    row_pass(src, g, orow, out.words ? out.words + i : nullptr);
    if (out.summ) wave_summary(g, src, total, tb.mid, out.summ + i);
    if (totals_out && lane == 0) totals_out[i] = total;
    if (reset) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      uint32_t* row = st.counts + (size_t)s * ROW;
      const int ng = lane_groups(lane);
#pragma unroll
      for (int q = 0; q < 9; ++q)
        if (q < ng) store4_state(row, 28 * lane + 4 * q, make_uint4(0u, 0u, 0u, 0u));
      if (lane == 0) {
        st.total[s] = 0;
        st.sumfix[s] = 0;
      }
    }
  } else {
#pragma unroll
    for (int q = 0; q < 9; ++q) g[q] = 0;
    if (orow) {
      const int ng = lane_groups(lane);
#pragma unroll
      for (int q = 0; q < 9; ++q)
        if (q < ng) store4_1798(orow, 28 * lane + 4 * q, make_uint4(0u, 0u, 0u, 0u));
    }
    if (out.summ) wave_summary(g, SrcRow32{st.counts}, 0, tb.mid, out.summ + i);  // num == 0: no bin is read
    if (totals_out && lane == 0) totals_out[i] = 0;
    if (out.words && lane == 0) out.words[i] = 0;
  }
}

int num_cus() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        ncu <= 0)
      ncu = 256;
  }
  return ncu;
}

}  // namespace

#ifdef L5DH_PHASES
extern "C" __attribute__((visibility("default"))) int l5dh_dev_phases2(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_phase2), sizeof(g_phase2), 0, hipMemcpyDeviceToHost);
}
#endif

hipError_t set_snapshot_attributes() {
  hipError_t e = hipSuccess;
  e = hipFuncSetAttribute((const void*)k_accum_cold_h<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)ACC_COLDH_LDS);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_accum_cold_h<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                          (int)ACC_COLDHE_LDS);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_accum_split, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ACC_SPLIT_LDS);
  if (e != hipSuccess) return e;
  e = hipFuncSetAttribute((const void*)k_fold1<true>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)FOLD16_LDS);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute((const void*)k_fold1<false>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)FOLD32_LDS);
}

// Sparse export: the words of each half of a dirty tile's state rows (one wave per
// row, 8 rows per wave), so k_plan_a/b size the tile's encoding from them instead of
// the dense worst case (a merge after a non-resetting snapshot made every
// touched tile dirty, and the encoding twice the dense rows).
__global__ __launch_bounds__(256) void k_enc_dirty(State st, Plan plan) {
  __shared__ uint32_t hw[2];
  const uint32_t t = blockIdx.x;
  if (!st.dirty[t]) return;  // (workgroup-uniform; clean tiles' words are never read)
  if (threadIdx.x < 2) hw[threadIdx.x] = 0u;
  __syncthreads();
  const int lane = lane_id(), w = threadIdx.x >> 6;
  for (int r = w; r < TILE; r += 4) {
    const uint32_t s = t * TILE + (uint32_t)r;
    const uint32_t nw = s < st.S ? row_words(SrcRow32{st.counts + (size_t)s * ROW}) : 0u;
    if (lane == 0 && nw) atomicAdd(&hw[r >> 4], nw);
  }
  __syncthreads();
  if (threadIdx.x < 2) plan.enc_dw[2 * t + threadIdx.x] = hw[threadIdx.x];
}

hipError_t launch_enc_dirty(State st, Plan plan, hipStream_t s) {
  hipLaunchKernelGGL(k_enc_dirty, dim3(st.F), dim3(256), 0, s, st, plan);
  return hipGetLastError();
}

hipError_t launch_plan(Segs segs, uint32_t F, int final_mode, uint32_t cold_limit, uint32_t hot_chunk,
                       const uint8_t* dirty, int direct_out, int encode, Plan plan, hipStream_t st) {
  const uint32_t B = (F + 1023) / 1024;  // header holds plan_header_words(F) words
  hipLaunchKernelGGL(k_plan_a, dim3(B), dim3(1024), 0, st, segs, F, final_mode, cold_limit, hot_chunk, dirty, encode,
                     plan);
  hipLaunchKernelGGL(k_plan_b, dim3(B), dim3(1024), 0, st, segs, F, final_mode, cold_limit, hot_chunk, dirty,
                     direct_out, encode, plan);
  return hipGetLastError();
}

hipError_t launch_hot_init(Plan plan, uint32_t max_hot, State state, Outputs out, int direct_out, hipStream_t st) {
  if (max_hot == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hot_init, dim3(std::min<uint32_t>(max_hot, 4u * num_cus())), dim3(256), 0, st, plan, state,
                     out, direct_out);
  return hipGetLastError();
}

hipError_t launch_accum_cold(Segs segs, Plan plan, uint32_t cold_items, State state, Tables tb, Outputs out,
                             int final_mode, int reset, hipStream_t st) {
  if (cold_items == 0) return hipSuccess;
  // persistent: half-tile items, two 512-thread workgroups per CU; cold_items may be
  // DEV_COUNT (read on the device)
  const uint32_t g2 = std::min<uint32_t>(cold_items == DEV_COUNT ? 0xFFFFFFFFu : 2u * cold_items, 2u * (uint32_t)num_cus());
  if (out.enc)
    hipLaunchKernelGGL(k_accum_cold_h<true>, dim3(g2), dim3(512), ACC_COLDHE_LDS, st, segs, plan, state, tb, out,
                       cold_items, final_mode, reset);
  else
    hipLaunchKernelGGL(k_accum_cold_h<false>, dim3(g2), dim3(512), ACC_COLDH_LDS, st, segs, plan, state, tb, out,
                       cold_items, final_mode, reset);
  return hipGetLastError();
}

hipError_t launch_fold1(const uint32_t* series, const float* values, size_t n, uint32_t chunk, State state, Tables tb,
                        uint32_t* err, bool vec, bool wide, hipStream_t st) {
  hipLaunchKernelGGL(k_fold1_init, dim3(1), dim3(256), 0, st, state);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const size_t items = (n + chunk - 1) / chunk;
  const dim3 grid((uint32_t)std::min<size_t>(items, (size_t)num_cus()));
  if (state.S <= 16 && !wide)
    hipLaunchKernelGGL(k_fold1<true>, grid, dim3(WG), FOLD16_LDS, st, series, values, n, chunk, state, tb, err,
                       vec ? 1 : 0);
  else
    hipLaunchKernelGGL(k_fold1<false>, grid, dim3(WG), FOLD32_LDS, st, series, values, n, chunk, state, tb, err,
                       vec ? 1 : 0);
  return hipGetLastError();
}

hipError_t launch_accum_split(Segs segs, Plan plan, uint32_t max_split_items, State state, Tables tb,
                              Outputs out, int direct_out, uint32_t hot_chunk, hipStream_t st) {
  if (max_split_items == 0) return hipSuccess;
  // at most 3/8 of the CUs: launched first, it leaves the rest to the cold tiles' kernel
  // (k_accum_split takes 115 KB of LDS: the two cannot share a CU), and its workgroups and
  // the cold ones take items until both queues are empty (accumulate phase on C3: 1.67 ms
  // with every CU first, 1.63 with half, 1.61 with 3/8; 1/4: 1.85, 5/8: 1.65;
  // profiles/r05ab_split_fraction_ab.txt).  Alone on its stream too (the last plan had no
  // big tiles): every CU there measured the same on the split-heavy 8-way shards and cost
  // C2 10 us for the launch of 256 idle workgroups (profiles/r06_split_grid_ab.txt).
  const uint32_t g = std::max<uint32_t>(1u, (uint32_t)num_cus() * 3 / 8);
  hipLaunchKernelGGL(k_accum_split, dim3(std::min<uint32_t>(max_split_items, g)), dim3(WG), ACC_SPLIT_LDS, st, segs,
                     plan, state, tb, out, direct_out, hot_chunk);
  return hipGetLastError();
}

hipError_t launch_hot_finish(Plan plan, uint32_t max_hot, State state, Tables tb, Outputs out, int final_mode,
                             int reset, int direct_out, hipStream_t st) {
  if (max_hot == 0) return hipSuccess;
  hipLaunchKernelGGL(k_hot_finish, dim3(std::min<uint32_t>(2 * max_hot, 2u * num_cus())), dim3(WG), 0, st, plan, state,
                     tb, out, final_mode, reset, direct_out);
  return hipGetLastError();
}

hipError_t launch_rows(State state, const int32_t* ext, const int64_t* ext_total, Tables tb, Outputs out, int reset,
                       int64_t* totals_out, hipStream_t st) {
  if (out.count == 0) return hipSuccess;
  hipLaunchKernelGGL(k_rows, dim3((out.count + 3) / 4), dim3(256), 0, st, state, ext, ext_total, tb, out, reset,
                     totals_out);
  return hipGetLastError();
}

}  // namespace l5dh
