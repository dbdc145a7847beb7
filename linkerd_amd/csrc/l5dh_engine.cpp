// l5dh_engine.cpp -- host side of the MI355X histogram engine and the C-ABI
// declared in include/l5dhist.h.
//
// One context = one GPU = one shard of the series space.  The context owns:
//   * dense state    counts[S][1800] u32, total[S] i64, sumfix[S] i64, dirty[F]
//   * a log of binned ingest segments (records u32[n] + tile offsets [F+1])
//   * scratch for the per-(slab, tile) offset table and the snapshot plan
// Ingest bins a batch immediately (count -> scans -> bin); snapshot aggregates
// every pending segment into LDS-private tile histograms and emits summaries
// in the same pass (the fused path) or folds into state first (range path).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/l5dhist.h"
#include "l5dh_kernels.hpp"
#include "l5dh_merge.hpp"

using namespace l5dh;

namespace {

// BucketedHistogram.scala:25-40 (makeLimitsFor), error 0.005.  Host copy used
// to build the device tables; the oracle's independent restatement checks it.
struct HostLimits {
  int32_t L[NL];
  bool ok = false;
  HostLimits() {
    const double maxValue = 2147483647.0;
    const double factor = 1.0 + (0.005 * 2);
    int n = 0;
    L[n++] = 1;
    int32_t last = -1;
    volatile double cur = 1.0;  // volatile: no contraction / excess precision
    for (;;) {
      volatile double next = cur * factor;
      if (next >= maxValue) break;
      const int32_t v = (int32_t)next + 1;
      if (v != last) {
        if (n >= NL) return;
        L[n++] = v;
        last = v;
      }
      cur = next;
    }
    ok = (n == NL);
  }
};

const HostLimits& host_limits() {
  static HostLimits h;
  return h;
}

constexpr size_t MAX_BATCH = ((size_t)1 << 30) - 65536;  // samples per binned piece (k_bin1 tags bit 31)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

}  // namespace

namespace l5dh {
// bucket(v) = number of limits <= v (upper bound), for the LUT builder.
static int host_bucket(const int32_t* L, int64_t v) {
  int lo = 0, hi = NL;
  while (lo < hi) {
    const int m = (lo + hi) / 2;
    if ((int64_t)L[m] <= v) lo = m + 1; else hi = m;
  }
  return lo;
}

int build_bucket_lut(const int32_t* L, uint32_t* lut) {
  // entry = b0 | off1 << 11 | off2 << 21 (offsets of the limits inside the
  // interval from its start, 0 = none) or off1 = 0x3FF for intervals wider
  // than 1024 (the device then compares against the limits).
  int maxin = 0, k = 0;
  for (int v = 0; v < 64; ++v) lut[k++] = (uint32_t)host_bucket(L, v);
  for (int e = 6; e <= 30; ++e)
    for (int m = 0; m < 64; ++m) {
      const int64_t start = (int64_t)(64 + m) << (e - 6);
      int64_t end = ((int64_t)(64 + m + 1) << (e - 6)) - 1;
      if (end > 2147483646) end = 2147483646;
      const int b0 = host_bucket(L, start);
      const int nin = host_bucket(L, end) - b0;
      maxin = std::max(maxin, nin);
      uint32_t x = (uint32_t)b0;
      if (end - start + 1 <= 1024) {
        for (int i = 0; i < nin && i < 2; ++i) {
          const int64_t off = (int64_t)L[b0 + i] - start;  // >= 1: L[b0] > start
          if (off < 1 || off > 1023) return 99;
          x |= (uint32_t)off << (11 + 10 * i);
        }
      } else {
        x |= 0x3FFu << 11;
      }
      lut[k++] = x;
    }
  return k == LUT_N ? maxin : 99;
}

int build_bucket_lut2(const int32_t* L, uint32_t* lut2) {
  int k = 0;
  auto entry = [&](int64_t start, int64_t end) {
    const int b0 = host_bucket(L, start);
    uint32_t o[2] = {0xFFFFu, 0xFFFFu};
    for (int i = 0; i < 2 && b0 + i < NL && L[b0 + i] <= end; ++i) {
      const int64_t off = (int64_t)L[b0 + i] - start;
      if (off < 1 || off >= 0xFFFF) return false;
      o[i] = (uint32_t)off;
    }
    if (b0 + 2 < NL && L[b0 + 2] <= end) return false;  // at most two limits per interval
    const int64_t p = start - (b0 ? (int64_t)L[b0 - 1] : 0);
    if (p < 0 || p > 0xFFFF) return false;
    lut2[2 * k] = o[0] | o[1] << 16;
    lut2[2 * k + 1] = (uint32_t)b0 | (uint32_t)p << 16;
    ++k;
    return true;
  };
  for (int v = 0; v < 64; ++v)
    if (!entry(v, v)) return 1;
  for (int e = 6; e <= 20; ++e)
    for (int m = 0; m < 64; ++m)
      if (!entry((int64_t)(64 + m) << (e - 6), ((int64_t)(64 + m + 1) << (e - 6)) - 1)) return 1;
  if (k != LUT2_N) return 1;
  // exhaustive check of the device decode (bucket_lut2) against upper_bound
  for (uint32_t v = 0; v < (1u << 21); ++v) {
    const uint32_t sh = v < 64 ? 0u : (uint32_t)(25 - __builtin_clz(v));
    const uint32_t idx = v < 64 ? v : 64u + sh * 64u + ((v >> sh) & 63u);
    const uint32_t start = (v >> sh) << sh;
    const uint32_t d = v - start, x0 = lut2[2 * idx], x1 = lut2[2 * idx + 1];
    const uint32_t o1 = x0 & 0xFFFFu, o2 = x0 >> 16;
    const bool k1 = d >= o1, k2 = d >= o2;
    const uint32_t off = k2 ? d - o2 : (k1 ? d - o1 : d + (x1 >> 16));
    const uint32_t b = (x1 & 0xFFFFu) + k1 + k2;
    const int hb = host_bucket(L, v);
    if ((int)b != hb || off != v - (hb ? (uint32_t)L[hb - 1] : 0u)) return 2;
  }
  return 0;
}

// Level 1's LUT (same intervals and index as lut2): entry {b0 | lim1 << 11, lim2}, the
// absolute limits inside the interval (lim1 = 0x1FFFFF, lim2 = 0xFFFFFFFF: none), so
// bucket = b0 + (v << 11 | 0x7FF >= x0) + (v >= x1) for v < V_ESC -- no interval start
// or offset arithmetic on the device.  Verified exhaustively against upper_bound.
int build_bucket_lut3(const int32_t* L, uint32_t* lut3) {
  int k = 0;
  auto entry = [&](int64_t start, int64_t end) {
    const int b0 = host_bucket(L, start);
    uint32_t lim[2] = {0x1FFFFFu, 0xFFFFFFFFu};
    for (int i = 0; i < 2 && b0 + i < NL && L[b0 + i] <= end; ++i) {
      if (L[b0 + i] <= start || L[b0 + i] >= 0x1FFFFF) return false;
      lim[i] = (uint32_t)L[b0 + i];
    }
    if (b0 + 2 < NL && L[b0 + 2] <= end) return false;  // at most two limits per interval
    if (b0 > 0x7FF) return false;
    lut3[2 * k] = (uint32_t)b0 | lim[0] << 11;
    lut3[2 * k + 1] = lim[1];
    ++k;
    return true;
  };
  for (int v = 0; v < 64; ++v)
    if (!entry(v, v)) return 1;
  for (int e = 6; e <= 20; ++e)
    for (int m = 0; m < 64; ++m)
      if (!entry((int64_t)(64 + m) << (e - 6), ((int64_t)(64 + m + 1) << (e - 6)) - 1)) return 1;
  if (k != LUT2_N) return 1;
  for (uint32_t v = 0; v < V_ESC; ++v) {  // the device index (lut3_index) and decode
    const uint32_t sh = (uint32_t)(25 - __builtin_clz(v | 64u));
    const uint32_t idx = (v >> sh) + (sh << 6);
    const uint32_t x0 = lut3[2 * idx], x1 = lut3[2 * idx + 1];
    const uint32_t b = (x0 & 0x7FFu) + ((v << 11 | 0x7FFu) >= x0 ? 1u : 0u) + (v >= x1 ? 1u : 0u);
    if ((int)b != host_bucket(L, v)) return 2;
  }
  return 0;
}
}  // namespace l5dh

struct l5dh_ctx {
  std::mutex mu;
  int device = 0;
  int num_cu = 256;
  uint32_t S = 0, F = 0;
  hipStream_t own_stream = nullptr;
  hipStream_t side = nullptr;       // cold-tile accumulation runs here beside the hot tiles
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  hipStream_t stream = nullptr;
  std::string last_error;

  // tables
  int32_t* d_lim_pad = nullptr;
  int32_t* d_mid = nullptr;
  int32_t* d_base = nullptr;
  uint32_t* d_lut = nullptr;
  uint2* d_lut2 = nullptr;
  // state
  uint32_t* d_counts = nullptr;
  int64_t* d_total = nullptr;
  int64_t* d_sumfix = nullptr;
  uint8_t* d_dirty = nullptr;
  uint32_t* d_err = nullptr;
  // scratch
  uint32_t* d_tile_tot = nullptr;  // [F] tile totals (snapshot plan)
  uint4* d_cold_item = nullptr;
  DevBuf split_item;  // big-tile half chunk items (sized per snapshot)
  uint32_t* d_hot_list = nullptr;
  uint8_t* d_tile_flags = nullptr;
  uint32_t* d_header = nullptr;
  uint32_t* d_enc_base = nullptr;  // [F] sparse export: each tile's first word of the unpacked encoding
  uint32_t* d_enc_h0 = nullptr;    // [F] sparse export: words reserved for half 0 of a big or dirty tile
  uint32_t* d_enc_dw = nullptr;    // [2F] sparse export: words of each half of a dirty tile's state rows
  uint32_t* h_header = nullptr;      // pinned: [4] ingest error count (written by k_rfix1), [5] big tiles of the last plan
  uint32_t* h_header_dev = nullptr;  // its device-side address
  uint32_t* d_kest = nullptr;   // [2F] sampled ids per (tile, half) key of the batch being binned
  uint32_t* d_kprev = nullptr;  // [2F] exact records per key of the previous batch (region sizes)
  int G_max = 256;
  // segments: binned batches awaiting the snapshot
  struct Seg {
    DevBuf rec32, rec16;
    uint32_t* meta = nullptr;  // [meta_layout(F).words()]
    size_t n = 0;
  };
  Seg segs[MAX_SEG];
  int nseg = 0;
  int max_seg = 4;
  uint32_t direct_max = DIRECT_MAX;  // direct tiles per batch (0: none)
  uint32_t direct_div = 1;           // direct tiles average >= 1/direct_div records per 8K samples
  uint32_t region_pct = 100;         // region capacity scale (L5DH_PARAM_REGION_PCT)
  uint64_t fold_last = 0;            // samples of the last batch folded at ingest (one-tile spaces)
  DevBuf stage_series, stage_values, stage_summ, stage_counts, stage_totals, stage_in_counts, stage_in_totals;
  // staging ring: small ingest batches are concatenated on the device and binned together
  DevBuf ring_series, ring_values;
  size_t ring_fill = 0;
  size_t ring_cap = 0;  // samples (0: every batch is binned at once)
  hipEvent_t ev_copy = nullptr;
  // asynchronous ingest: ticket t's inputs are consumed when tick_ev[t % NTICK] (recorded
  // for a ticket >= t, stream order) completes
  static constexpr int NTICK = 64;
  hipEvent_t tick_ev[NTICK] = {};
  uint64_t tick_of[NTICK] = {};
  uint64_t tick_next = 0, tick_done = 0;
  uint32_t err_reported = 0;  // invalid-id reports already returned (h_header[4] is the device's count)
  // fleet merge (RCCL)
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  DevBuf merge_counts, merge_totals, recv_counts, recv_totals;
  // sparse reduce-scatter (l5dh_merge.hip): this rank's encoding, the received slices
  DevBuf m_words, m_offs, m_enc, m_tmp, m_sizes, r_words, r_offs, r_enc;
  DevBuf m_unpacked, m_roff;  // the sparse export: rows' encodings at their tiles' places, each row's first word
  size_t m_unpacked_words = 0;  // (the unpacked encoding's size: a bound of the packed one)
  bool m_sparse = false;      // the last export was sparse (reduce-scatter through the collective)
  size_t m_tmp_bytes = 0;
  std::vector<uint64_t> m_to, m_from;  // words to / from every rank
  uint64_t m_dense_bytes = 0, m_encoded_bytes = 0, m_sent_bytes = 0;
  bool rccl_1rank = false;  // run the collective in a 1-rank communicator too (an identity otherwise skipped)
  bool loopback = false;    // l5dh_comm_init_loopback: the collectives are device copies among the group's contexts
  uint32_t variant = 0;  // L5DH_PARAM_VARIANT: result-preserving kernel variants (A/B timing)
  // params
  uint32_t cold_limit = COLD_LIMIT_MAX;
  uint32_t hot_chunk = 1u << 18;  // records per big-tile item (u32 LDS bins, one half-tile per workgroup)
  bool timing = false;
  struct Ev {
    int kid;
    hipEvent_t a, b;
  };
  std::vector<Ev> pending_ev;
  std::vector<hipEvent_t> ev_pool;
  double k_ms[L5DH_K_NKERNELS] = {0};
  int64_t k_n[L5DH_K_NKERNELS] = {0};
};

namespace {

int fail(l5dh_ctx* c, int code, const std::string& msg) {
  c->last_error = msg;
  return code;
}

int hipfail(l5dh_ctx* c, hipError_t e, const char* what) {
  c->last_error = std::string(what) + ": " + hipGetErrorString(e);
  return -EIO;
}

#define HIPCHK(c, expr)                                \
  do {                                                 \
    hipError_t _e = (expr);                            \
    if (_e != hipSuccess) return hipfail((c), _e, #expr); \
  } while (0)

hipEvent_t ev_get(l5dh_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  hipEventCreate(&e);
  return e;
}

struct KTimer {
  l5dh_ctx* c;
  int kid;
  hipEvent_t a = nullptr;
  KTimer(l5dh_ctx* c_, int kid_) : c(c_), kid(kid_) {
    if (c->timing) {
      a = ev_get(c);
      hipEventRecord(a, c->stream);
    }
  }
  ~KTimer() {
    if (a) {
      hipEvent_t b = ev_get(c);
      hipEventRecord(b, c->stream);
      c->pending_ev.push_back({kid, a, b});
    }
  }
};

void collect_timing(l5dh_ctx* c) {
  for (auto& e : c->pending_ev) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, e.a, e.b) == hipSuccess) {
      c->k_ms[e.kid] += ms;
      c->k_n[e.kid] += 1;
    }
    c->ev_pool.push_back(e.a);
    c->ev_pool.push_back(e.b);
  }
  c->pending_ev.clear();
}

int sync_stream(l5dh_ctx* c) {
  HIPCHK(c, hipStreamSynchronize(c->stream));
  collect_timing(c);
  return 0;
}

bool is_device_ptr(const void* p) {
  if (!p) return false;
  hipPointerAttribute_t a;
  hipError_t e = hipPointerGetAttributes(&a, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

// Device-visible address of page-locked host memory (hipHostMalloc / registered),
// or nullptr for device or pageable memory.
const void* host_mapped_ptr(const void* p) {
  if (!p) return nullptr;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type != hipMemoryTypeHost || !a.devicePointer) return nullptr;
  return static_cast<const char*>(a.devicePointer) + (static_cast<const char*>(p) - static_cast<const char*>(a.hostPointer));
}

int ensure(l5dh_ctx* c, DevBuf& b, size_t bytes) {
  if (b.cap >= bytes) return 0;
  if (b.p) {
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipFree(b.p));
    b.p = nullptr;
    b.cap = 0;
  }
  size_t cap = std::max(bytes, (size_t)4096);
  cap = (cap + 4095) & ~(size_t)4095;
  hipError_t e = hipMalloc(&b.p, cap);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(c, -ENOMEM, std::string("hipMalloc staging: ") + hipGetErrorString(e));
  }
  b.cap = cap;
  return 0;
}

Tables tables(l5dh_ctx* c) { return Tables{c->d_lim_pad, c->d_mid, c->d_base, c->d_lut, c->d_lut2, c->d_lut2 + LUT2_N}; }

State state(l5dh_ctx* c) { return State{c->d_counts, c->d_total, c->d_sumfix, c->d_dirty, c->S, c->F}; }

Plan plan(l5dh_ctx* c) {
  return Plan{c->d_tile_tot, c->d_enc_base, c->d_enc_h0, c->d_enc_dw, c->d_cold_item,
              static_cast<uint2*>(c->split_item.p), c->d_hot_list, c->d_tile_flags, c->d_header,
              c->h_header_dev + 5};
}

Segs segs_view(l5dh_ctx* c) {
  Segs s{};
  s.n = c->nseg;
  for (int j = 0; j < c->nseg; ++j) {
    s.rec16[j] = static_cast<const uint16_t*>(c->segs[j].rec16.p);
    s.meta[j] = c->segs[j].meta;
  }
  return s;
}

// Aggregate every pending segment.  final_mode: emit summaries/counts for the
// whole series space into `out` (fused path); otherwise fold into state.  encode: the
// fleet merge's sparse export (out.words / out.roff / out.totals; out.enc is set here).
int aggregate(l5dh_ctx* c, int final_mode, int reset, Outputs out, bool encode = false) {
  if (!final_mode && c->nseg == 0) return 0;
  Segs sv = segs_view(c);
  size_t recs = 0;
  for (int j = 0; j < c->nseg; ++j) recs += c->segs[j].n;
  // big-tile items: hot_chunk records, fewer when the pending records would leave CUs
  // idle (>= 2 items per CU when the records allow)
  uint32_t hc = c->hot_chunk;
  {
    const size_t fill = recs / (2 * (size_t)std::max(1, c->num_cu));
    hc = (uint32_t)std::min<size_t>(hc, std::max<size_t>(16384, (fill + 1023) & ~(size_t)1023));
  }
  if (int r = ensure(c, c->split_item, (recs / hc + 2 * (size_t)c->F + 2) * 8)) return r;
  Plan pl = plan(c);
  // a resetting snapshot of every series into dense rows: clean big tiles count
  // straight into their output rows (no copy of state rows in k_hot_finish), and those
  // whose halves are one item each are written by their items alone (TF_SOLO)
  const int direct_out = final_mode && reset && out.counts && out.first == 0 && out.count == (uint32_t)c->S;
  // the sparse export (the fleet merge's reduce-scatter): row encodings, no dense rows
  if (encode && !(final_mode && reset && out.first == 0 && out.count == (uint32_t)c->S && !out.counts && !out.summ))
    return fail(c, -EINVAL, "internal: the sparse export is a whole-range resetting export");
  {
    KTimer kt(c, L5DH_K_SCAN);
    // (the sparse export: the dirty tiles' state-row words first, for their encoding ranges)
    if (encode) HIPCHK(c, launch_enc_dirty(state(c), pl, c->stream));
    HIPCHK(c, launch_plan(sv, c->F, final_mode, c->cold_limit, hc, c->d_dirty, direct_out, encode ? 1 : 0, pl,
                          c->stream));
  }
  if (encode) {  // the unpacked encoding's size comes from the plan (one host wait)
    uint32_t words = 0;
    HIPCHK(c, hipMemcpyAsync(&words, c->d_header + 5 + 4 * ((c->F + 1023) / 1024), 4, hipMemcpyDeviceToHost,
                             c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (int r = ensure(c, c->m_unpacked, (size_t)words * 4 + 16)) return r;
    c->m_unpacked_words = words;
    out.enc = static_cast<uint32_t*>(c->m_unpacked.p);
  }
  // The accumulate kernels are persistent and read their item counts from the plan
  // header on the device, so no host round trip separates them from the plan: the
  // launches get upper bounds (a big tile holds > cold_limit records).
  const uint32_t hot = (uint32_t)std::min<size_t>(c->F, recs / ((size_t)c->cold_limit + 1));
  const uint32_t split_items = (uint32_t)std::min<size_t>(0xFFFFFFF0u, recs / hc + 2 * (size_t)hot);
  State st = state(c);
  Tables tb = tables(c);
  if (hot) {
    KTimer kt(c, L5DH_K_HOT);
    HIPCHK(c, launch_hot_init(pl, hot, st, out, direct_out, c->stream));
  }
  bool joined = true;
  {
    // the big tiles first (on at most half the CUs), the cold tiles on the side stream
    // concurrently (disjoint tiles and series; the side stream joins back after
    // k_hot_finish, which touches only big tiles: it runs under the cold kernel)
    KTimer kt(c, L5DH_K_ACCUM);
    // The two streams cost ~20 us of idle GPU (the fork's and the join's barrier packets);
    // they pay only when there are big tiles, so the last plan the host has seen picks the
    // order (a hint: either order is correct; k_plan_b writes it to a mapped host word)
    const bool big_seen = __atomic_load_n(c->h_header + 5, __ATOMIC_RELAXED) != 0u;
    if (split_items && big_seen) {
      HIPCHK(c, hipEventRecord(c->ev_fork, c->stream));
      HIPCHK(c, hipStreamWaitEvent(c->side, c->ev_fork, 0));
      HIPCHK(c, launch_accum_split(sv, pl, split_items, st, tb, out, direct_out, hc, c->stream));
      HIPCHK(c, launch_accum_cold(sv, pl, DEV_COUNT, st, tb, out, final_mode, reset, c->side));
      HIPCHK(c, hipEventRecord(c->ev_join, c->side));
      joined = false;
    } else {
      if (split_items) HIPCHK(c, launch_accum_split(sv, pl, split_items, st, tb, out, direct_out, hc, c->stream));
      HIPCHK(c, launch_accum_cold(sv, pl, DEV_COUNT, st, tb, out, final_mode, reset, c->stream));
    }
    // (timed with the accumulate: with two streams it runs under the cold kernel)
    if (hot) HIPCHK(c, launch_hot_finish(pl, hot, st, tb, out, final_mode, reset, direct_out, c->stream));
    if (!joined) HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_join, 0));
  }
  c->nseg = 0;
  return 0;
}

int fold(l5dh_ctx* c) {
  Outputs none{nullptr, nullptr, 0, 0, nullptr};
  return aggregate(c, 0, 0, none);
}

// Invalid series ids: k_rbin1 (k_fold1) adds to the device counter d_err (never
// reset); k_rfix1 (a copy, after k_fold1) puts it into the pinned, mapped h_header[4].  The host value only grows, so comparing it with the number of
// reports already returned needs no synchronization.
int check_err(l5dh_ctx* c) {
  const uint32_t seen = __atomic_load_n(c->h_header + 4, __ATOMIC_ACQUIRE);
  if (seen != c->err_reported) {
    c->err_reported = seen;
    return fail(c, -EINVAL, "series id >= max_series in an ingest batch (those samples were dropped)");
  }
  return 0;
}

int do_ingest(l5dh_ctx* c, const uint32_t* series, const float* values, size_t n) {
  if (n == 0) return 0;
  if (n > MAX_BATCH) return fail(c, -EINVAL, "batch piece larger than 2^30 samples");
  if (c->nseg >= c->max_seg) {
    int r = fold(c);
    if (r) return r;
  }
  const uint32_t* ds = series;
  const float* dv = values;
  if (!is_device_ptr(series) || !is_device_ptr(values)) {
    int r;
    if ((r = ensure(c, c->stage_series, n * 4))) return r;
    if ((r = ensure(c, c->stage_values, n * 4))) return r;
    KTimer kt(c, L5DH_K_COPY);
    HIPCHK(c, hipMemcpyAsync(c->stage_series.p, series, n * 4, hipMemcpyDefault, c->stream));
    HIPCHK(c, hipMemcpyAsync(c->stage_values.p, values, n * 4, hipMemcpyDefault, c->stream));
    ds = static_cast<const uint32_t*>(c->stage_series.p);
    dv = static_cast<const float*>(c->stage_values.p);
  }
  const bool vec = ((uintptr_t)ds % 16 == 0) && ((uintptr_t)dv % 16 == 0);
  if (c->F == 1) {  // one tile: fold the batch into its state rows now (no records, no segment)
    KTimer kt(c, L5DH_K_BIN);
    // one item per CU when the batch allows (each item clears and flushes its LDS rows:
    // C1's fold 0.040 ms at two items per CU, 0.033 at one, 0.044 at four;
    // profiles/r06_fold_items_ab.txt)
    const size_t fill = n / (size_t)std::max(1, c->num_cu);
    const uint32_t chunk =
        (uint32_t)std::min<size_t>(c->hot_chunk & ~3u, std::max<size_t>(16384, (fill + 1023) & ~(size_t)1023));
    HIPCHK(c, launch_fold1(ds, dv, n, chunk, state(c), tables(c), c->d_err, vec, (c->variant & 1) != 0, c->stream));
    c->fold_last = n;
    HIPCHK(c, hipMemcpyAsync(c->h_header + 4, c->d_err, 4, hipMemcpyDeviceToHost, c->stream));
    return 0;
  }
  auto& sg = c->segs[c->nseg];
  // region buffers: the plan sizes the regions from the previous batch and a sample
  // of this one, with slack; a plan that does not fit is scaled to these sizes (an
  // overflowing region is then redone with exact sizes, which always fit)
  // rec32: the super-tile bins' records; rec16: the direct keys' regions in [0, dlim16)
  // (planned, so possibly oversized) and level 2's regions after them, with room for
  // level 2's exact layout in any case (N + 7 per key of padding)
  const size_t cap32 = n + n / 2 + ((size_t)1 << 19);
  const size_t cap16 = 2 * n + n / 8 + (size_t)128 * c->F + 4096;
  const size_t dlim16 = (cap16 - (n + (size_t)16 * c->F + 1024)) & ~(size_t)7;  // (level-2 regions 16-B aligned)
  {
    int r = ensure(c, sg.rec32, (cap32 + 16) * 4);  // readers load whole 16-B groups
    if (!r) r = ensure(c, sg.rec16, (cap16 + 16) * 2);
    if (r) return r;
  }
  // slabs: one workgroup per CU at most, >= 8K samples each, 16-B aligned starts
  int G = (int)std::min<size_t>((size_t)c->G_max, (n + 8191) / 8192);
  if (G < 1) G = 1;
  size_t per = (n + G - 1) / G;
  per = (per + 3) & ~(size_t)3;
  G = (int)((n + per - 1) / per);
  IngestArgs a{};
  a.series = ds;
  a.values = dv;
  a.n = n;
  a.per = per;
  a.G = G;
  a.num_cu = c->num_cu;
  a.S = c->S;
  a.F = c->F;
  a.tb = tables(c);
  a.sumfix = c->d_sumfix;
  a.err = c->d_err;
  a.err_host = c->h_header_dev + 4;
  a.kest = c->d_kest;
  a.kprev = c->d_kprev;
  a.meta = sg.meta;
  a.rec32 = static_cast<uint32_t*>(sg.rec32.p);
  a.rec16 = static_cast<uint16_t*>(sg.rec16.p);
  a.cap32 = cap32;
  a.cap16 = cap16;
  a.dlim16 = dlim16;
  a.thr_min = (uint32_t)std::min<uint64_t>(std::max<uint64_t>(1, n / (8192ull * c->direct_div)), 0xFFFFFFFFull);
  const uint32_t FS = (c->F + 63) / 64;
  // + the trash bin (and 8 spare bins)
  a.dmax = std::min<uint32_t>(c->direct_max, ((uint32_t)BIN1_BINS - 9 - FS) / 2);
  a.pct = c->region_pct;
  a.vec = vec;
  {
    KTimer kt(c, L5DH_K_SCAN);
    // variant bit 2 (measurement): forget the previous batch's exact key counts, so every
    // batch is planned as a first interval is -- from its sample alone
    if (c->variant & 4) HIPCHK(c, hipMemsetAsync(c->d_kprev, 0, (size_t)2 * c->F * 4, c->stream));
    HIPCHK(c, launch_ingest(a, 0, c->stream));
  }
  {
    KTimer kt(c, L5DH_K_BIN);
    HIPCHK(c, launch_ingest(a, 1, c->stream));
  }
  {
    KTimer kt(c, L5DH_K_BIN2);
    HIPCHK(c, launch_ingest(a, 3, c->stream));
  }
  sg.n = n;
  c->nseg++;
  return 0;  // (k_rfix1 wrote the invalid-id count to h_header[4])
}

// Bin the staging ring as one batch.
int flush_ring(l5dh_ctx* c) {
  if (!c->ring_fill) return 0;
  const size_t n = c->ring_fill;
  c->ring_fill = 0;
  return do_ingest(c, static_cast<const uint32_t*>(c->ring_series.p), static_cast<const float*>(c->ring_values.p), n);
}

// Wait until the caller's buffers of this call have been read by the device.
int wait_inputs(l5dh_ctx* c) {
  HIPCHK(c, hipEventRecord(c->ev_copy, c->stream));
  HIPCHK(c, hipEventSynchronize(c->ev_copy));
  return 0;
}

// Asynchronous ingest: the inputs of ticket t are consumed once its event completes.
int issue_ticket(l5dh_ctx* c, uint64_t* ticket) {
  const uint64_t t = ++c->tick_next;
  const int slot = (int)(t % l5dh_ctx::NTICK);
  if (!c->tick_ev[slot]) HIPCHK(c, hipEventCreateWithFlags(&c->tick_ev[slot], hipEventDisableTiming));
  HIPCHK(c, hipEventRecord(c->tick_ev[slot], c->stream));
  c->tick_of[slot] = t;
  *ticket = t;
  return 0;
}

int wait_ticket(l5dh_ctx* c, uint64_t t) {
  if (t <= c->tick_done) return 0;
  if (t > c->tick_next) return fail(c, -EINVAL, "unknown ingest ticket");
  const int slot = (int)(t % l5dh_ctx::NTICK);
  // the slot holds t or a later ticket (recorded later on the same stream)
  HIPCHK(c, hipEventSynchronize(c->tick_ev[slot]));
  c->tick_done = std::max(c->tick_done, c->tick_of[slot]);
  return 0;
}

int ingest_impl(l5dh_ctx* c, const uint32_t* series, const float* values, size_t n, uint64_t* ticket = nullptr) {
  if (ticket) *ticket = c->tick_next;  // nothing new to wait for (n == 0)
  if (n == 0) return 0;
  const bool dev = is_device_ptr(series) && is_device_ptr(values);
  // caller-stream contexts are stream ordered for device inputs; otherwise the
  // call returns once nothing of the caller's memory is still to be read, or, in
  // the asynchronous form, with a ticket to wait for
  const bool wait = (!dev || c->stream == c->own_stream) && !ticket;
  if (c->ring_cap && n <= c->ring_cap / 2) {
    int r;
    if (c->ring_fill + n > c->ring_cap && (r = flush_ring(c))) return r;
    if ((r = ensure(c, c->ring_series, c->ring_cap * 4 + 64)) || (r = ensure(c, c->ring_values, c->ring_cap * 4 + 64)))
      return r;
    {
      KTimer kt(c, L5DH_K_COPY);
      uint32_t* rs = static_cast<uint32_t*>(c->ring_series.p) + c->ring_fill;
      float* rv = static_cast<float*>(c->ring_values.p) + c->ring_fill;
      // pinned host batches: one zero-copy kernel (variant bit 1: DMA copies instead)
      const void* hs = dev || (c->variant & 2) ? nullptr : host_mapped_ptr(series);
      const void* hv = hs ? host_mapped_ptr(values) : nullptr;
      if (hs && hv) {
        HIPCHK(c, launch_fetch_host(static_cast<const uint32_t*>(hs), static_cast<const uint32_t*>(hv), rs,
                                    reinterpret_cast<uint32_t*>(rv), n, c->stream));
      } else {
        HIPCHK(c, hipMemcpyAsync(rs, series, n * 4, hipMemcpyDefault, c->stream));
        HIPCHK(c, hipMemcpyAsync(rv, values, n * 4, hipMemcpyDefault, c->stream));
      }
    }
    c->ring_fill += n;
    if (ticket) return issue_ticket(c, ticket);
    return wait ? wait_inputs(c) : 0;
  }
  int r = flush_ring(c);
  if (r) return r;
  // batches are binned in pieces below 2^30 samples (k_bin1 tags direct-tile
  // destinations in bit 31)
  for (size_t o = 0; o < n; o += MAX_BATCH) {
    const size_t m = std::min(n - o, MAX_BATCH);
    if ((r = do_ingest(c, series + o, values + o, m))) return r;
  }
  if (ticket) return issue_ticket(c, ticket);
  return wait ? wait_inputs(c) : 0;
}

bool full_range(l5dh_ctx* c, uint32_t first, uint32_t count) { return first == 0 && count == c->S; }

int do_snapshot(l5dh_ctx* c, uint32_t first, uint32_t count, l5dh_summary* out, int32_t* counts_out, int reset) {
  if ((uint64_t)first + count > c->S) return fail(c, -EINVAL, "series range out of bounds");
  if (count == 0) return 0;
  int r = flush_ring(c);
  if (r) return r;
  // outputs: device pointers are written directly, host pointers via staging
  Summary88* d_summ = nullptr;
  int32_t* d_counts = nullptr;
  const bool out_dev = out && is_device_ptr(out) && ((uintptr_t)out % 8 == 0);
  const bool cnt_dev = counts_out && is_device_ptr(counts_out) && ((uintptr_t)counts_out % 8 == 0);
  if (out) {
    if (out_dev)
      d_summ = reinterpret_cast<Summary88*>(out);
    else {
      if ((r = ensure(c, c->stage_summ, (size_t)count * 88))) return r;
      d_summ = static_cast<Summary88*>(c->stage_summ.p);
    }
  }
  if (counts_out) {
    if (cnt_dev)
      d_counts = counts_out;
    else {
      if ((r = ensure(c, c->stage_counts, (size_t)count * NB * 4))) return r;
      d_counts = static_cast<int32_t*>(c->stage_counts.p);
    }
  }
  Outputs o{d_summ, d_counts, first, count, nullptr};
  // (a one-tile space folds every batch into its state rows at ingest: no segments, so its
  // snapshot is the state rows' -- one k_rows launch instead of the plan and accumulate
  // kernels; C1 in profiles/r06_one_tile_snapshot_ab.txt)
  if (full_range(c, first, count) && c->F > 1) {
    if ((r = aggregate(c, 1, reset, o))) return r;
  } else {
    if ((r = fold(c))) return r;
    KTimer kt(c, L5DH_K_HOT);
    HIPCHK(c, launch_rows(state(c), nullptr, nullptr, tables(c), o, reset, nullptr, c->stream));
  }
  {
    KTimer kt(c, L5DH_K_COPY);
    if (out && !out_dev) HIPCHK(c, hipMemcpyAsync(out, d_summ, (size_t)count * 88, hipMemcpyDefault, c->stream));
    if (counts_out && !cnt_dev)
      HIPCHK(c, hipMemcpyAsync(counts_out, d_counts, (size_t)count * NB * 4, hipMemcpyDefault, c->stream));
  }
  // device outputs on a caller stream are stream ordered (as device inputs of
  // l5dh_ingest): the caller's later work on that stream sees them; no host wait
  if ((!out || out_dev) && (!counts_out || cnt_dev) && c->stream != c->own_stream) return 0;
  return sync_stream(c);
}

// ---- fleet merge (RCCL) ------------------------------------------------------
int ncclfail(l5dh_ctx* c, ncclResult_t e, const char* what) {
  c->last_error = std::string(what) + ": " + ncclGetErrorString(e);
  return -EIO;
}

#define NCCLCHK(c, expr)                                     \
  do {                                                       \
    ncclResult_t _e = (expr);                                \
    if (_e != ncclSuccess) return ncclfail((c), _e, #expr);  \
  } while (0)

uint32_t merge_per(const l5dh_ctx* c) { return (c->S + c->nranks - 1) / c->nranks; }

// Phase 1: pending samples + state -> dense rows [Sp][1798] and totals [Sp] (the
// fused whole-range export with reset), pad rows zero.
bool merge_skips_collective(const l5dh_ctx* c);

int merge_export(l5dh_ctx* c, int mode) {
  if (!c->comm && !c->loopback)
    return fail(c, -EINVAL, "no communicator: call l5dh_comm_init_rank or l5dh_comm_init_all first");
  int r = flush_ring(c);
  if (r) return r;
  const size_t Sp = (size_t)merge_per(c) * c->nranks;
  // the reduce-scatter through the collective exports SPARSE: each row's encoding straight
  // from the accumulate kernels' bins (no dense rows, no re-read), words and first word per
  // row; the all-reduce and a 1-rank communicator that skips the collective export dense rows
  c->m_sparse = mode == L5DH_MERGE_REDUCE_SCATTER && !merge_skips_collective(c);
  if ((r = ensure(c, c->merge_totals, Sp * 8)) || (r = ensure(c, c->m_words, (Sp + 1) * 4))) return r;
  int64_t* tot = static_cast<int64_t*>(c->merge_totals.p);
  uint32_t* words = static_cast<uint32_t*>(c->m_words.p);
  if (Sp > c->S) HIPCHK(c, hipMemsetAsync(tot + c->S, 0, (Sp - c->S) * 8, c->stream));
  HIPCHK(c, hipMemsetAsync(words + c->S, 0, (Sp + 1 - c->S) * 4, c->stream));
  if (c->m_sparse) {
    if ((r = ensure(c, c->m_roff, Sp * 4))) return r;
    Outputs o{nullptr, nullptr, 0, c->S, tot, words, nullptr, static_cast<uint32_t*>(c->m_roff.p)};
    return aggregate(c, 1, 1, o, true);
  }
  if ((r = ensure(c, c->merge_counts, Sp * NB * 4))) return r;
  int32_t* cnt = static_cast<int32_t*>(c->merge_counts.p);
  if (Sp > c->S) HIPCHK(c, hipMemsetAsync(cnt + (size_t)c->S * NB, 0, (Sp - c->S) * NB * 4, c->stream));
  return aggregate(c, 1, 1, Outputs{nullptr, cnt, 0, c->S, tot, words, nullptr, nullptr});
}

// Phase 2 (reduce-scatter): the rows are exchanged sparse (l5dh_merge.hip) -- per
// destination rank, the non-empty buckets of its slice plus the words per row --
// and the totals by one int64 reduce-scatter.  A 1-rank communicator skips it (an
// identity) unless L5DH_PARAM_MERGE_RCCL_1RANK forces it, with the encoding sent to
// itself through RCCL.  Steps: encode (local, one host wait for the slice sizes),
// sizes (collective: an all-gather of the words-to matrix), receive buffers (local,
// one host wait), payload (collective).  l5dh_merge_all groups each collective step
// over its contexts.  The forcing parameter applies to an RCCL communicator only: a
// 1-rank loopback group has no transport that could carry the slice to itself (its
// copies skip p == q), so it always takes the identity.
bool merge_skips_collective(const l5dh_ctx* c) { return c->nranks == 1 && (!c->rccl_1rank || c->loopback); }

int merge_encode_step(l5dh_ctx* c) {
  const uint32_t per = merge_per(c);
  const uint32_t Sp = per * (uint32_t)c->nranks;
  const int W = c->nranks;
  int r;
  KTimer kt(c, L5DH_K_MERGE);
  c->m_tmp_bytes = 0;  // (the scans of every slice fit the storage of this, the longest one)
  HIPCHK(c, merge_count(nullptr, Sp, nullptr, nullptr, nullptr, &c->m_tmp_bytes, c->stream));
  if ((r = ensure(c, c->m_words, ((size_t)Sp + 1) * 4)) || (r = ensure(c, c->m_offs, ((size_t)Sp + 1) * 8)) ||
      (r = ensure(c, c->m_tmp, c->m_tmp_bytes)) || (r = ensure(c, c->m_sizes, (size_t)W * W * 8)))
    return r;
  uint32_t* words = static_cast<uint32_t*>(c->m_words.p);
  uint64_t* offs = static_cast<uint64_t*>(c->m_offs.p);
  HIPCHK(c, merge_count(nullptr, Sp, words, offs, c->m_tmp.p, &c->m_tmp_bytes, c->stream));  // (words: the export's)
  // this rank's row of the size matrix (for the all-gather) written on the device: the
  // slice sizes reach the host with the matrix, in the receive step's one host wait
  HIPCHK(c, merge_sizes_row(offs, per, W, static_cast<uint64_t*>(c->m_sizes.p) + (size_t)c->rank * W, c->stream));
  size_t cap = c->m_unpacked_words;  // the packed encoding is no larger than the unpacked one
  if (!c->m_sparse) {  // (dense rows encoded: the exact size, one host wait)
    uint64_t total = 0;
    HIPCHK(c, hipMemcpyAsync(&total, offs + Sp, 8, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    cap = total;
  }
  if ((r = ensure(c, c->m_enc, cap * 4 + 16))) return r;
  if (c->m_sparse)  // the export's row encodings packed in row order (one contiguous slice per destination)
    HIPCHK(c, merge_pack(static_cast<const uint32_t*>(c->m_unpacked.p), static_cast<const uint32_t*>(c->m_roff.p), offs,
                         (uint32_t)std::min<size_t>(Sp, c->S), static_cast<uint32_t*>(c->m_enc.p), c->stream));
  else
    HIPCHK(c, merge_encode(static_cast<const int32_t*>(c->merge_counts.p), Sp, offs,
                           static_cast<uint32_t*>(c->m_enc.p), c->stream));
  c->m_dense_bytes = (uint64_t)Sp * (NB * 4 + 8);
  return 0;
}

int merge_sizes_step(l5dh_ctx* c) {
  const int W = c->nranks;
  uint64_t* m = static_cast<uint64_t*>(c->m_sizes.p);
  NCCLCHK(c, ncclAllGather(m + (size_t)c->rank * W, m, (size_t)W, ncclUint64, c->comm, c->stream));
  return 0;
}

int merge_recv_step(l5dh_ctx* c) {
  const uint32_t per = merge_per(c);
  const int W = c->nranks;
  std::vector<uint64_t> mat((size_t)W * W);
  HIPCHK(c, hipMemcpyAsync(mat.data(), c->m_sizes.p, mat.size() * 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  c->m_from.assign(W, 0);
  c->m_to.assign(W, 0);
  uint64_t all = 0, mine = 0;
  for (int s = 0; s < W; ++s) all += (c->m_from[s] = mat[(size_t)s * W + c->rank]);
  for (int q = 0; q < W; ++q) mine += (c->m_to[q] = mat[(size_t)c->rank * W + q]);
  c->m_encoded_bytes = mine * 4 + (uint64_t)per * W * (4 + 8);  // entries + words per row + totals
  int r;
  if ((r = ensure(c, c->r_enc, (size_t)all * 4 + 16)) || (r = ensure(c, c->r_words, (size_t)W * per * 4)) ||
      (r = ensure(c, c->r_offs, (size_t)W * per * 8)) || (r = ensure(c, c->recv_totals, (size_t)per * 8)))
    return r;
  uint64_t sent = 0;
  for (int q = 0; q < W; ++q)
    if (q != c->rank) sent += 4 * c->m_to[q] + 4ull * per + 8ull * per;
  c->m_sent_bytes = sent;
  return 0;
}

int merge_payload_step(l5dh_ctx* c) {
  const uint32_t per = merge_per(c);
  const int W = c->nranks;
  const uint32_t* enc = static_cast<const uint32_t*>(c->m_enc.p);
  const uint32_t* words = static_cast<const uint32_t*>(c->m_words.p);
  uint32_t* renc = static_cast<uint32_t*>(c->r_enc.p);
  uint32_t* rwords = static_cast<uint32_t*>(c->r_words.p);
  KTimer kt(c, L5DH_K_MERGE);
  uint64_t at = 0, rat = 0;
  for (int q = 0; q < W; ++q) {
    // (the local slice is read in place, except in a forced 1-rank exchange)
    if (q != c->rank || W == 1) {
      if (c->m_to[q]) NCCLCHK(c, ncclSend(enc + at, c->m_to[q], ncclUint32, q, c->comm, c->stream));
      NCCLCHK(c, ncclSend(words + (size_t)q * per, per, ncclUint32, q, c->comm, c->stream));
      if (c->m_from[q]) NCCLCHK(c, ncclRecv(renc + rat, c->m_from[q], ncclUint32, q, c->comm, c->stream));
      NCCLCHK(c, ncclRecv(rwords + (size_t)q * per, per, ncclUint32, q, c->comm, c->stream));
    }
    at += c->m_to[q];
    rat += c->m_from[q];
  }
  NCCLCHK(c, ncclReduceScatter(c->merge_totals.p, c->recv_totals.p, per, ncclInt64, ncclSum, c->comm, c->stream));
  return 0;
}

int merge_dense_allreduce(l5dh_ctx* c) {
  const size_t Sp = (size_t)merge_per(c) * c->nranks;
  KTimer kt(c, L5DH_K_MERGE);
  c->m_dense_bytes = c->m_encoded_bytes = Sp * (NB * 4 + 8);
  c->m_sent_bytes = c->nranks > 1 ? 2 * c->m_dense_bytes * (c->nranks - 1) / c->nranks : 0;
  NCCLCHK(c, ncclAllReduce(c->merge_counts.p, c->merge_counts.p, Sp * NB, ncclInt32, ncclSum, c->comm, c->stream));
  NCCLCHK(c, ncclAllReduce(c->merge_totals.p, c->merge_totals.p, Sp, ncclInt64, ncclSum, c->comm, c->stream));
  return 0;
}

// Phase 3: the rows this rank receives -- decoded from every source and summarized
// (reduce-scatter), or the all-reduced dense rows summarized -- and the copies.
int merge_finish(l5dh_ctx* c, int mode, l5dh_summary* out, int32_t* counts_out, int64_t* totals_out, uint32_t* first,
                 uint32_t* count) {
  const uint32_t per = merge_per(c);
  const bool rs = mode == L5DH_MERGE_REDUCE_SCATTER;
  const bool sparse = rs && !merge_skips_collective(c);
  const uint32_t f = rs ? (uint32_t)std::min<uint64_t>((uint64_t)c->rank * per, c->S) : 0u;
  const uint32_t n = rs ? std::min<uint32_t>(per, c->S - f) : c->S;
  if (first) *first = f;
  if (count) *count = n;
  if (n == 0) return sync_stream(c);
  int r;
  Summary88* d_summ = nullptr;
  const bool out_dev = out && is_device_ptr(out) && ((uintptr_t)out % 8 == 0);
  if (out) {
    if (out_dev)
      d_summ = reinterpret_cast<Summary88*>(out);
    else {
      if ((r = ensure(c, c->stage_summ, (size_t)n * 88))) return r;
      d_summ = static_cast<Summary88*>(c->stage_summ.p);
    }
  }
  const int32_t* rows = static_cast<const int32_t*>(c->merge_counts.p);
  const int64_t* tots = static_cast<const int64_t*>(c->merge_totals.p);
  if (sparse) {
    const int W = c->nranks;
    if (W > MERGE_MAX_RANKS) return fail(c, -EINVAL, "fleet merge: more than 64 ranks");
    const bool cnt_dev = counts_out && is_device_ptr(counts_out) && ((uintptr_t)counts_out % 8 == 0);
    int32_t* drows = nullptr;
    if (counts_out) {
      if (cnt_dev)
        drows = counts_out;
      else {
        if ((r = ensure(c, c->recv_counts, (size_t)per * NB * 4))) return r;
        drows = static_cast<int32_t*>(c->recv_counts.p);
      }
    }
    // the received slices are contiguous in r_enc / r_words, source by source; this
    // rank's own slice (not sent) is copied to its place there, and one scan of the
    // [W][per] word counts gives every source's row offsets
    KTimer kt(c, L5DH_K_MERGE);
    uint32_t* renc = static_cast<uint32_t*>(c->r_enc.p);
    uint32_t* rwords = static_cast<uint32_t*>(c->r_words.p);
    if (W > 1) {
      uint64_t a0 = 0, rat = 0;
      for (int k = 0; k < c->rank; ++k) {
        a0 += c->m_to[k];
        rat += c->m_from[k];
      }
      if (c->m_to[c->rank])
        HIPCHK(c, hipMemcpyAsync(renc + rat, static_cast<const uint32_t*>(c->m_enc.p) + a0, c->m_to[c->rank] * 4,
                                 hipMemcpyDeviceToDevice, c->stream));
      HIPCHK(c, hipMemcpyAsync(rwords + (size_t)c->rank * per, static_cast<const uint32_t*>(c->m_words.p) + (size_t)c->rank * per,
                               (size_t)per * 4, hipMemcpyDeviceToDevice, c->stream));
    }
    uint64_t* roffs = static_cast<uint64_t*>(c->r_offs.p);
    HIPCHK(c, merge_offsets(rwords, (uint32_t)((size_t)W * per), roffs, c->m_tmp.p, c->m_tmp_bytes, c->stream));
    const MergeRecv src{renc, rwords, roffs, per, W};
    HIPCHK(c, merge_decode(src, n, static_cast<const int64_t*>(c->recv_totals.p), tables(c), drows, d_summ, c->stream));
    rows = drows;
    tots = static_cast<const int64_t*>(c->recv_totals.p);
    KTimer kc(c, L5DH_K_COPY);
    if (out && !out_dev) HIPCHK(c, hipMemcpyAsync(out, d_summ, (size_t)n * 88, hipMemcpyDefault, c->stream));
    if (counts_out && !cnt_dev)
      HIPCHK(c, hipMemcpyAsync(counts_out, rows, (size_t)n * NB * 4, hipMemcpyDefault, c->stream));
    if (totals_out) HIPCHK(c, hipMemcpyAsync(totals_out, tots, (size_t)n * 8, hipMemcpyDefault, c->stream));
    return sync_stream(c);
  }
  if (rs) {  // a 1-rank communicator, collective skipped: the exported rows are the sums
    c->m_dense_bytes = (uint64_t)per * (NB * 4 + 8);
    c->m_encoded_bytes = c->m_dense_bytes;
    c->m_sent_bytes = 0;
  }
  if (out) {
    KTimer kt(c, L5DH_K_HOT);
    HIPCHK(c, launch_rows(state(c), rows, tots, tables(c), Outputs{d_summ, nullptr, 0, n, nullptr}, 0, nullptr,
                          c->stream));
  }
  {
    KTimer kt(c, L5DH_K_COPY);
    if (out && !out_dev) HIPCHK(c, hipMemcpyAsync(out, d_summ, (size_t)n * 88, hipMemcpyDefault, c->stream));
    if (counts_out) HIPCHK(c, hipMemcpyAsync(counts_out, rows, (size_t)n * NB * 4, hipMemcpyDefault, c->stream));
    if (totals_out) HIPCHK(c, hipMemcpyAsync(totals_out, tots, (size_t)n * 8, hipMemcpyDefault, c->stream));
  }
  return sync_stream(c);
}

// The loopback group's collectives (l5dh_comm_init_loopback: n contexts on one device):
// the same encode / size / receive / payload steps as over RCCL, with each exchange
// done by device copies (all streams drained first) and the reductions by one kernel
// reading every rank's buffer.
int sync_all(l5dh_ctx** cs, int n) {
  for (int i = 0; i < n; ++i) HIPCHK(cs[i], hipStreamSynchronize(cs[i]->stream));
  return 0;
}

int loop_collectives(l5dh_ctx** cs, int n, int mode) {
  int r;
  const int W = n;
  const uint32_t per = merge_per(cs[0]);
  if (mode != L5DH_MERGE_REDUCE_SCATTER) {  // dense all-reduce: the sum into rank 0's rows, copied to the others
    const size_t Sp = (size_t)per * W;
    if ((r = sync_all(cs, n))) return r;
    std::vector<const int32_t*> rows(W);
    std::vector<const int64_t*> tots(W);
    for (int i = 0; i < W; ++i) {
      rows[i] = static_cast<const int32_t*>(cs[i]->merge_counts.p);
      tots[i] = static_cast<const int64_t*>(cs[i]->merge_totals.p);
    }
    l5dh_ctx* c0 = cs[0];
    HIPCHK(c0, merge_loop_sum_i32(rows.data(), W, static_cast<int32_t*>(c0->merge_counts.p), Sp * NB, c0->stream));
    HIPCHK(c0, merge_loop_sum_i64(tots.data(), W, static_cast<int64_t*>(c0->merge_totals.p), Sp, c0->stream));
    HIPCHK(c0, hipStreamSynchronize(c0->stream));
    for (int i = 1; i < W; ++i) {
      HIPCHK(cs[i], hipMemcpyAsync(cs[i]->merge_counts.p, c0->merge_counts.p, Sp * NB * 4, hipMemcpyDeviceToDevice,
                                   cs[i]->stream));
      HIPCHK(cs[i], hipMemcpyAsync(cs[i]->merge_totals.p, c0->merge_totals.p, Sp * 8, hipMemcpyDeviceToDevice,
                                   cs[i]->stream));
    }
    for (int i = 0; i < W; ++i) {
      cs[i]->m_dense_bytes = cs[i]->m_encoded_bytes = Sp * (NB * 4 + 8);
      cs[i]->m_sent_bytes = 2 * cs[i]->m_dense_bytes * (W - 1) / W;
    }
    return sync_all(cs, n);
  }
  for (int i = 0; i < n; ++i)
    if ((r = merge_encode_step(cs[i]))) return r;
  if ((r = sync_all(cs, n))) return r;
  {  // all-gather of the size rows: one copy launch per destination
    for (int j = 0; j < n; ++j) {
      LoopCopies l{};
      for (int i = 0; i < n; ++i)
        if (i != j) {
          l.src[l.n] = reinterpret_cast<const uint32_t*>(static_cast<const uint64_t*>(cs[i]->m_sizes.p) + (size_t)i * W);
          l.dst[l.n] = reinterpret_cast<uint32_t*>(static_cast<uint64_t*>(cs[j]->m_sizes.p) + (size_t)i * W);
          l.words[l.n++] = (uint64_t)W * 2;
        }
      HIPCHK(cs[j], merge_loop_copy(l, cs[j]->stream));
    }
  }
  for (int i = 0; i < n; ++i)
    if ((r = merge_recv_step(cs[i]))) return r;
  if ((r = sync_all(cs, n))) return r;
  for (int q = 0; q < W; ++q) {  // destination q receives every other source's slice q (one copy launch)
    l5dh_ctx* d = cs[q];
    uint64_t rat = 0;
    LoopCopies l{};
    for (int p = 0; p < W; ++p) {
      l5dh_ctx* sp = cs[p];
      if (p != q) {
        uint64_t at = 0;
        for (int k = 0; k < q; ++k) at += sp->m_to[k];
        if (sp->m_to[q]) {
          l.src[l.n] = static_cast<const uint32_t*>(sp->m_enc.p) + at;
          l.dst[l.n] = static_cast<uint32_t*>(d->r_enc.p) + rat;
          l.words[l.n++] = sp->m_to[q];
        }
        l.src[l.n] = static_cast<const uint32_t*>(sp->m_words.p) + (size_t)q * per;
        l.dst[l.n] = static_cast<uint32_t*>(d->r_words.p) + (size_t)p * per;
        l.words[l.n++] = per;
      }
      rat += d->m_from[p];
    }
    HIPCHK(d, merge_loop_copy(l, d->stream));
    std::vector<const int64_t*> tots(W);  // the totals' reduce-scatter: slice q summed over the sources
    for (int p = 0; p < W; ++p) tots[p] = static_cast<const int64_t*>(cs[p]->merge_totals.p) + (size_t)q * per;
    HIPCHK(d, merge_loop_sum_i64(tots.data(), W, static_cast<int64_t*>(d->recv_totals.p), per, d->stream));
  }
  return sync_all(cs, n);
}

// The collective steps of one merge over contexts `cs` (one, or every context of an
// l5dh_comm_init_all communicator): each collective step is grouped over them.
int merge_collectives(l5dh_ctx** cs, int n, int mode) {
  if (cs[0]->loopback) return loop_collectives(cs, n, mode);
  int r = 0;
  if (mode != L5DH_MERGE_REDUCE_SCATTER) {
    NCCLCHK(cs[0], ncclGroupStart());
    for (int i = 0; i < n && !r; ++i) {
      hipSetDevice(cs[i]->device);
      if (!merge_skips_collective(cs[i])) r = merge_dense_allreduce(cs[i]);
    }
    const ncclResult_t ge = ncclGroupEnd();
    if (r) return r;
    return ge == ncclSuccess ? 0 : ncclfail(cs[0], ge, "ncclGroupEnd");
  }
  if (merge_skips_collective(cs[0])) return 0;
  for (int i = 0; i < n; ++i) {
    hipSetDevice(cs[i]->device);
    if ((r = merge_encode_step(cs[i]))) return r;
  }
  NCCLCHK(cs[0], ncclGroupStart());
  for (int i = 0; i < n && !r; ++i) {
    hipSetDevice(cs[i]->device);
    r = merge_sizes_step(cs[i]);
  }
  ncclResult_t ge = ncclGroupEnd();
  if (r) return r;
  if (ge != ncclSuccess) return ncclfail(cs[0], ge, "ncclGroupEnd");
  for (int i = 0; i < n; ++i) {
    hipSetDevice(cs[i]->device);
    if ((r = merge_recv_step(cs[i]))) return r;
  }
  NCCLCHK(cs[0], ncclGroupStart());
  for (int i = 0; i < n && !r; ++i) {
    hipSetDevice(cs[i]->device);
    r = merge_payload_step(cs[i]);
  }
  ge = ncclGroupEnd();
  if (r) return r;
  return ge == ncclSuccess ? 0 : ncclfail(cs[0], ge, "ncclGroupEnd");
}

}  // namespace

// ============================================================================
// C-ABI
// ============================================================================
extern "C" {

int l5dh_abi_version(void) { return L5DH_ABI_VERSION; }

const int32_t* l5dh_limits(size_t* n) {
  const HostLimits& h = host_limits();
  if (n) *n = h.ok ? NL : 0;
  return h.ok ? h.L : nullptr;
}

int l5dh_open(l5dh_ctx** out, uint32_t max_series, uint32_t device_mask) {
  if (!out) return -EINVAL;
  *out = nullptr;
  if (max_series == 0 || max_series > L5DH_MAX_SERIES) return -EINVAL;
  if (device_mask == 0 || (device_mask & (device_mask - 1))) return -EINVAL;  // exactly one device
  const HostLimits& hl = host_limits();
  if (!hl.ok) return -EIO;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    (void)hipGetLastError();
    return -ENODEV;
  }
  int dev = __builtin_ctz(device_mask);
  if (dev >= ndev) return -ENODEV;
  auto* c = new (std::nothrow) l5dh_ctx();
  if (!c) return -ENOMEM;
  c->device = dev;
  c->S = max_series;
  // staging ring: 64 samples per series, between 2^20 and 2^26 samples (4 MB .. 256 MB per array)
  c->ring_cap = std::min<size_t>(std::max<size_t>((size_t)max_series * 64, (size_t)1 << 20), (size_t)1 << 26);
  c->F = (max_series + TILE - 1) / TILE;
  auto bail = [&](int code) {
    l5dh_close(c);
    return code;
  };
  if (hipSetDevice(dev) != hipSuccess) return bail(-EIO);
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) c->num_cu = prop.multiProcessorCount;
  // one slab per CU: the level-1 kernel holds one 1024-thread workgroup per CU (LDS-bound)
  c->G_max = std::max(1, std::min(c->num_cu, 512));
  if (set_ingest_attributes() != hipSuccess || set_snapshot_attributes() != hipSuccess) return bail(-EIO);
  if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) return bail(-EIO);
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess) return bail(-EIO);
  if (hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_copy, hipEventDisableTiming) != hipSuccess)
    return bail(-EIO);
  c->stream = c->own_stream;
  const size_t S = c->S, F = c->F;
  auto mal = [&](void** p, size_t bytes) { return hipMalloc(p, std::max<size_t>(bytes, 256)) == hipSuccess; };
  bool ok = mal((void**)&c->d_lim_pad, LIM_PAD * 4) && mal((void**)&c->d_mid, NB * 4) &&
            mal((void**)&c->d_base, ROW * 4) && mal((void**)&c->d_lut, LUT_N * 4) && mal((void**)&c->d_lut2, LUT2_N * 16) && mal((void**)&c->d_counts, S * ROW * 4) &&
            mal((void**)&c->d_total, S * 8) && mal((void**)&c->d_sumfix, S * 8) && mal((void**)&c->d_dirty, F) &&
            mal((void**)&c->d_err, 4) && mal((void**)&c->d_tile_tot, F * 4) &&
            mal((void**)&c->d_cold_item, (F + 1) * 16) && mal((void**)&c->d_hot_list, F * 4) &&
            mal((void**)&c->d_header, plan_header_words((uint32_t)F) * 4) && mal((void**)&c->d_tile_flags, F) &&
            mal((void**)&c->d_enc_base, F * 4) && mal((void**)&c->d_enc_h0, F * 4) &&
            mal((void**)&c->d_enc_dw, 2 * F * 4) &&
            mal((void**)&c->d_kest, 2 * F * 4) && mal((void**)&c->d_kprev, 2 * F * 4);
  const size_t meta_bytes = (size_t)meta_layout((uint32_t)F).words() * 4;
  for (int j = 0; ok && j < MAX_SEG; ++j)  // (zeroed: the header's redo counters only grow)
    ok = mal((void**)&c->segs[j].meta, meta_bytes) && hipMemset(c->segs[j].meta, 0, meta_bytes) == hipSuccess;
  if (!ok) {
    (void)hipGetLastError();
    return bail(-ENOMEM);
  }
  if (hipHostMalloc((void**)&c->h_header, 32, hipHostMallocMapped) != hipSuccess) return bail(-ENOMEM);  // [4]: err count
  memset(c->h_header, 0, 32);
  if (hipHostGetDevicePointer((void**)&c->h_header_dev, c->h_header, 0) != hipSuccess) return bail(-ENOMEM);
  // constant tables
  int32_t lim_pad[LIM_PAD], mid[NB], base[ROW] = {0};
  for (int i = 0; i < LIM_PAD; ++i) lim_pad[i] = i < NL ? hl.L[i] : INT_MAXV;
  for (int b = 0; b < NB; ++b) {
    mid[b] = b == 0 ? 0 : (b >= NL ? INT_MAXV : (int32_t)(((int64_t)hl.L[b - 1] + hl.L[b]) / 2));
    base[b] = b == 0 ? 0 : hl.L[b - 1];
  }
  uint32_t lut[LUT_N];
  if (build_bucket_lut(hl.L, lut) > 2) return bail(-EIO);
  static uint32_t lut2[4 * LUT2_N];  // lut2, then lut3 (d_lut2 holds both)
  static int lut2_rc = build_bucket_lut2(hl.L, lut2) | build_bucket_lut3(hl.L, lut2 + 2 * LUT2_N);  // once per process
  if (lut2_rc != 0) return bail(-EIO);
  if (hipMemcpy(c->d_lut, lut, sizeof(lut), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_lut2, lut2, sizeof(lut2), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_lim_pad, lim_pad, sizeof(lim_pad), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_mid, mid, sizeof(mid), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(c->d_base, base, sizeof(base), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemset(c->d_dirty, 0, F) != hipSuccess || hipMemset(c->d_sumfix, 0, S * 8) != hipSuccess ||
      hipMemset(c->d_err, 0, 4) != hipSuccess || hipMemset(c->d_kest, 0, 2 * F * 4) != hipSuccess ||
      hipMemset(c->d_kprev, 0, 2 * F * 4) != hipSuccess || hipDeviceSynchronize() != hipSuccess)
    return bail(-EIO);
  *out = c;
  return 0;
}

int l5dh_close(l5dh_ctx* c) {
  if (!c) return -EINVAL;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  for (auto& e : c->pending_ev) {
    hipEventDestroy(e.a);
    hipEventDestroy(e.b);
  }
  for (auto e : c->ev_pool) hipEventDestroy(e);
  void* ptrs[] = {c->d_lim_pad, c->d_mid,      c->d_base,     c->d_lut,       c->d_lut2,     c->d_counts,
                  c->d_total,   c->d_sumfix,   c->d_dirty,    c->d_err,       c->d_tile_tot, c->d_cold_item,
                  c->d_hot_list, c->d_header,  c->d_tile_flags, c->d_kest,    c->d_kprev, c->d_enc_base,
                  c->d_enc_h0,  c->d_enc_dw};
  for (void* p : ptrs)
    if (p) hipFree(p);
  for (auto& s : c->segs) {
    if (s.meta) hipFree(s.meta);
    if (s.rec32.p) hipFree(s.rec32.p);
    if (s.rec16.p) hipFree(s.rec16.p);
  }
  if (c->comm) ncclCommDestroy(c->comm);
  DevBuf* bufs[] = {&c->split_item,      &c->stage_series, &c->stage_values,  &c->stage_summ,
                    &c->stage_counts,    &c->stage_totals, &c->stage_in_counts, &c->stage_in_totals,
                    &c->ring_series,     &c->ring_values,  &c->merge_counts,   &c->merge_totals,
                    &c->recv_counts,     &c->recv_totals,  &c->m_words,        &c->m_offs,
                    &c->m_enc,           &c->m_tmp,        &c->m_sizes,        &c->r_words,
                    &c->r_offs,          &c->r_enc,        &c->m_unpacked,     &c->m_roff};
  for (DevBuf* b : bufs)
    if (b->p) hipFree(b->p);
  if (c->h_header) hipHostFree(c->h_header);
  if (c->side) hipStreamDestroy(c->side);
  if (c->ev_fork) hipEventDestroy(c->ev_fork);
  if (c->ev_join) hipEventDestroy(c->ev_join);
  if (c->ev_copy) hipEventDestroy(c->ev_copy);
  for (hipEvent_t e : c->tick_ev)
    if (e) hipEventDestroy(e);
  if (c->own_stream) hipStreamDestroy(c->own_stream);
  delete c;
  return 0;
}

int l5dh_ingest(l5dh_ctx* c, const uint32_t* series, const float* values, size_t n) {
  if (!c) return -EINVAL;
  if (n && (!series || !values)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  // 0 = the batch was accepted; a deferred invalid-id report never rides on a later
  // batch's status (l5dh_sync returns it), so a caller never re-sends an accepted batch
  return ingest_impl(c, series, values, n);
}

int l5dh_ingest_async(l5dh_ctx* c, const uint32_t* series, const float* values, size_t n, uint64_t* ticket) {
  if (!c || !ticket) return -EINVAL;
  if (n && (!series || !values)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  return ingest_impl(c, series, values, n, ticket);  // (deferred id errors: l5dh_sync)
}

int l5dh_ingest_wait(l5dh_ctx* c, uint64_t ticket) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  return wait_ticket(c, ticket);
}

int l5dh_snapshot(l5dh_ctx* c, uint32_t first, uint32_t count, l5dh_summary* out, int32_t* counts_out, int reset) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  return do_snapshot(c, first, count, out, counts_out, reset);
}

int l5dh_export_state(l5dh_ctx* c, uint32_t first, uint32_t count, int32_t* counts, int64_t* totals, int reset) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  if ((uint64_t)first + count > c->S) return fail(c, -EINVAL, "series range out of bounds");
  if (count == 0) return 0;
  int r = flush_ring(c);
  if (r) return r;
  const bool fused = full_range(c, first, count) && reset;  // the fleet merge's export: one aggregate pass
  if (!fused && (r = fold(c))) return r;
  const bool cnt_dev = counts && is_device_ptr(counts) && ((uintptr_t)counts % 8 == 0);
  const bool tot_dev = totals && is_device_ptr(totals) && ((uintptr_t)totals % 8 == 0);
  int32_t* d_counts = nullptr;
  int64_t* d_totals = nullptr;
  if (counts) {
    if (cnt_dev)
      d_counts = counts;
    else {
      if ((r = ensure(c, c->stage_counts, (size_t)count * NB * 4))) return r;
      d_counts = static_cast<int32_t*>(c->stage_counts.p);
    }
  }
  if (totals) {
    if (tot_dev)
      d_totals = totals;
    else {
      if ((r = ensure(c, c->stage_totals, (size_t)count * 8))) return r;
      d_totals = static_cast<int64_t*>(c->stage_totals.p);
    }
  }
  if (fused) {
    // pending records and state go straight into the caller's dense rows and
    // totals (no fold into state, no second pass), and the state is left clean
    if ((r = aggregate(c, 1, 1, Outputs{nullptr, d_counts, first, count, d_totals}))) return r;
  } else {
    Outputs o{nullptr, d_counts, first, count, nullptr};
    KTimer kt(c, L5DH_K_HOT);
    HIPCHK(c, launch_rows(state(c), nullptr, nullptr, tables(c), o, reset, d_totals, c->stream));
  }
  if (counts && !cnt_dev)
    HIPCHK(c, hipMemcpyAsync(counts, d_counts, (size_t)count * NB * 4, hipMemcpyDefault, c->stream));
  if (totals && !tot_dev) HIPCHK(c, hipMemcpyAsync(totals, d_totals, (size_t)count * 8, hipMemcpyDefault, c->stream));
  return sync_stream(c);
}

int l5dh_summarize_dense(l5dh_ctx* c, const int32_t* counts, const int64_t* totals, size_t n, l5dh_summary* out) {
  if (!c || (n && (!counts || !out))) return -EINVAL;
  if (n == 0) return 0;
  if (n > 0xFFFFFFFFull) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  int r;
  const int32_t* d_counts = counts;
  const int64_t* d_totals = totals;
  if (!(is_device_ptr(counts) && (uintptr_t)counts % 8 == 0)) {
    if ((r = ensure(c, c->stage_in_counts, n * NB * 4))) return r;
    HIPCHK(c, hipMemcpyAsync(c->stage_in_counts.p, counts, n * NB * 4, hipMemcpyDefault, c->stream));
    d_counts = static_cast<const int32_t*>(c->stage_in_counts.p);
  }
  if (totals && !is_device_ptr(totals)) {
    if ((r = ensure(c, c->stage_in_totals, n * 8))) return r;
    HIPCHK(c, hipMemcpyAsync(c->stage_in_totals.p, totals, n * 8, hipMemcpyDefault, c->stream));
    d_totals = static_cast<const int64_t*>(c->stage_in_totals.p);
  }
  const bool out_dev = is_device_ptr(out) && ((uintptr_t)out % 8 == 0);
  Summary88* d_summ;
  if (out_dev)
    d_summ = reinterpret_cast<Summary88*>(out);
  else {
    if ((r = ensure(c, c->stage_summ, n * 88))) return r;
    d_summ = static_cast<Summary88*>(c->stage_summ.p);
  }
  Outputs o{d_summ, nullptr, 0, (uint32_t)n, nullptr};
  {
    KTimer kt(c, L5DH_K_HOT);
    HIPCHK(c, launch_rows(state(c), d_counts, d_totals, tables(c), o, 0, nullptr, c->stream));
  }
  if (!out_dev) HIPCHK(c, hipMemcpyAsync(out, d_summ, n * 88, hipMemcpyDefault, c->stream));
  return sync_stream(c);
}

int l5dh_peek(l5dh_ctx* c, uint32_t series, l5dh_bucket_count* out, size_t cap, size_t* n_out) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  if (series >= c->S) return fail(c, -EINVAL, "series id out of range");
  int r;
  if ((r = flush_ring(c)) || (r = fold(c))) return r;
  uint8_t dirty = 0;
  std::vector<uint32_t> row(ROW, 0);
  HIPCHK(c, hipMemcpyAsync(&dirty, c->d_dirty + (series >> TILE_SHIFT), 1, hipMemcpyDeviceToHost, c->stream));
  if ((r = sync_stream(c))) return r;
  if (dirty) {
    HIPCHK(c, hipMemcpyAsync(row.data(), c->d_counts + (size_t)series * ROW, NB * 4, hipMemcpyDeviceToHost,
                             c->stream));
    if ((r = sync_stream(c))) return r;
  }
  const HostLimits& hl = host_limits();
  size_t k = 0;
  for (int b = 0; b < NB; ++b) {
    const int32_t cnt = (int32_t)row[b];
    if (cnt > 0) {
      if (out && k < cap) {
        out[k].lower = b == 0 ? 0 : hl.L[b - 1];
        out[k].upper = b < NL ? hl.L[b] : INT_MAXV;
        out[k].count = cnt;
      }
      ++k;
    }
  }
  if (n_out) *n_out = k;
  return 0;
}

int l5dh_sync(l5dh_ctx* c) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  int r;
  if ((r = flush_ring(c)) || (r = sync_stream(c))) return r;
  return check_err(c);
}

int l5dh_set_stream(l5dh_ctx* c, void* s) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  int r = sync_stream(c);
  if (r) return r;
  c->stream = s == L5DH_OWN_STREAM ? c->own_stream : static_cast<hipStream_t>(s);
  return 0;
}

int l5dh_wait_event(l5dh_ctx* c, void* ev) {
  if (!c || !ev) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  HIPCHK(c, hipStreamWaitEvent(c->stream, static_cast<hipEvent_t>(ev), 0));
  return 0;
}

int l5dh_set_param(l5dh_ctx* c, int param, int64_t v) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  switch (param) {
    case L5DH_PARAM_TIMING:
      c->timing = v != 0;
      return 0;
    case L5DH_PARAM_COLD_LIMIT:
      if (v < 0 || v > (int64_t)COLD_LIMIT_MAX) return fail(c, -EINVAL, "cold limit must be in [0, 65535]");
      c->cold_limit = (uint32_t)v;
      return 0;
    case L5DH_PARAM_HOT_CHUNK:
      // <= 2^20: an item's records index LDS bins in u32 (and stay far below 2^32)
      if (v < 1024 || v > (1ll << 20)) return fail(c, -EINVAL, "hot chunk must be in [1024, 2^20]");
      c->hot_chunk = (uint32_t)v;
      return 0;
    case L5DH_PARAM_MAX_SEGMENTS:
      if (v < 1 || v > MAX_SEG) return fail(c, -EINVAL, "max segments must be in [1, 8]");
      if (c->nseg > v) {
        hipSetDevice(c->device);
        int r = fold(c);
        if (r) return r;
      }
      c->max_seg = (int)v;
      return 0;
    case L5DH_PARAM_DIRECT_MAX:
      if (v < 0 || v > DIRECT_MAX) return fail(c, -EINVAL, "direct tiles must be in [0, 255]");
      c->direct_max = (uint32_t)v;
      return 0;
    case L5DH_PARAM_DIRECT_DIV:
      if (v < 1 || v > 65536) return fail(c, -EINVAL, "direct divisor must be in [1, 65536]");
      c->direct_div = (uint32_t)v;
      return 0;
    case L5DH_PARAM_STAGE_SAMPLES: {
      if (v < 0 || v > (int64_t)MAX_BATCH) return fail(c, -EINVAL, "staging ring must be in [0, 2^30 - 65536] samples");
      hipSetDevice(c->device);
      int r = flush_ring(c);  // staged samples are binned before the ring changes size
      if (r) return r;
      if ((size_t)v * 4 + 64 > c->ring_series.cap) {  // the next small batch allocates the new size
        if ((r = sync_stream(c))) return r;
        for (DevBuf* b : {&c->ring_series, &c->ring_values}) {
          if (b->p) hipFree(b->p);
          b->p = nullptr;
          b->cap = 0;
        }
      }
      c->ring_cap = ((size_t)v + 3) & ~(size_t)3;
      return 0;
    }
    case L5DH_PARAM_VARIANT:
      if (v < 0 || v > 31) return fail(c, -EINVAL, "variant bits must be in [0, 31]");
      c->variant = (uint32_t)v;
      return 0;
    case L5DH_PARAM_REGION_PCT:
      if (v < 1 || v > 1000) return fail(c, -EINVAL, "region capacity percent must be in [1, 1000]");
      c->region_pct = (uint32_t)v;
      return 0;
    case L5DH_PARAM_MERGE_RCCL_1RANK:
      c->rccl_1rank = v != 0;
      return 0;
    case L5DH_PARAM_MAX_SLABS:
      if (v < 1 || v > 512) return fail(c, -EINVAL, "slabs must be in [1, 512]");
      c->G_max = (int)v;
      return 0;
    default:
      return fail(c, -EINVAL, "unknown parameter");
  }
}

int l5dh_kernel_time(l5dh_ctx* c, int kid, double* ms, int64_t* launches, int reset_after) {
  if (!c || kid < 0 || kid >= L5DH_K_NKERNELS) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  int r = sync_stream(c);
  if (r) return r;
  if (ms) *ms = c->k_ms[kid];
  if (launches) *launches = c->k_n[kid];
  if (reset_after) {
    c->k_ms[kid] = 0;
    c->k_n[kid] = 0;
  }
  return 0;
}

int l5dh_device(l5dh_ctx* c, int* dev) {
  if (!c || !dev) return -EINVAL;
  *dev = c->device;
  return 0;
}

uint32_t l5dh_max_series(l5dh_ctx* c) { return c ? c->S : 0; }

int l5dh_pin_alloc(size_t bytes, void** out) {
  if (!out || bytes == 0) return -EINVAL;
  if (hipHostMalloc(out, bytes, 0) != hipSuccess) {
    (void)hipGetLastError();
    *out = nullptr;
    return -ENOMEM;
  }
  return 0;
}

int l5dh_pin_free(void* p) {
  if (!p) return -EINVAL;
  return hipHostFree(p) == hipSuccess ? 0 : -EINVAL;
}

const char* l5dh_last_error(l5dh_ctx* c) { return c ? c->last_error.c_str() : "null context"; }

int l5dh_comm_unique_id(void* id_out) {
  if (!id_out) return -EINVAL;
  static_assert(sizeof(ncclUniqueId) == L5DH_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -EIO;
  memcpy(id_out, &id, sizeof(id));
  return 0;
}

int l5dh_comm_init_rank(l5dh_ctx* c, const void* id, int nranks, int rank) {
  if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->comm || c->loopback) return fail(c, -EINVAL, "context already has a communicator");
  // (the sparse reduce-scatter holds one source per rank: checked before any merge runs)
  if (nranks > MERGE_MAX_RANKS) return fail(c, -EINVAL, "fleet merge: more than 64 ranks");
  hipSetDevice(c->device);
  ncclUniqueId uid;
  memcpy(&uid, id, sizeof(uid));
  ncclComm_t comm = nullptr;
  NCCLCHK(c, ncclCommInitRank(&comm, nranks, uid, rank));
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  return 0;
}

int l5dh_comm_init_all(l5dh_ctx** ctxs, int n) {
  if (!ctxs || n < 1 || n > MERGE_MAX_RANKS) return -EINVAL;
  std::vector<int> devs(n);
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i] || ctxs[i]->comm || ctxs[i]->loopback || ctxs[i]->S != ctxs[0]->S) return -EINVAL;
    devs[i] = ctxs[i]->device;
  }
  std::vector<ncclComm_t> comms(n, nullptr);
  const ncclResult_t e = ncclCommInitAll(comms.data(), n, devs.data());
  if (e != ncclSuccess) {
    ctxs[0]->last_error = std::string("ncclCommInitAll: ") + ncclGetErrorString(e);
    return -EIO;
  }
  for (int i = 0; i < n; ++i) {
    std::lock_guard<std::mutex> g(ctxs[i]->mu);
    ctxs[i]->comm = comms[i];
    ctxs[i]->nranks = n;
    ctxs[i]->rank = i;
  }
  return 0;
}

int l5dh_comm_init_loopback(l5dh_ctx** ctxs, int n) {
  if (!ctxs || n < 1 || n > MERGE_MAX_RANKS) return -EINVAL;
  for (int i = 0; i < n; ++i) {
    if (!ctxs[i] || ctxs[i]->comm || ctxs[i]->loopback || ctxs[i]->S != ctxs[0]->S ||
        ctxs[i]->device != ctxs[0]->device)
      return -EINVAL;
    for (int j = 0; j < i; ++j)
      if (ctxs[j] == ctxs[i]) return -EINVAL;
  }
  for (int i = 0; i < n; ++i) {
    std::lock_guard<std::mutex> g(ctxs[i]->mu);
    ctxs[i]->loopback = true;
    ctxs[i]->nranks = n;
    ctxs[i]->rank = i;
  }
  return 0;
}

int l5dh_comm_destroy(l5dh_ctx* c) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->comm) {
    hipSetDevice(c->device);
    int r = sync_stream(c);
    if (r) return r;
    ncclCommDestroy(c->comm);
  }
  c->loopback = false;
  c->comm = nullptr;
  c->nranks = 1;
  c->rank = 0;
  return 0;
}

int l5dh_merge(l5dh_ctx* c, int mode, l5dh_summary* out, int32_t* counts_out, int64_t* totals_out, uint32_t* first,
               uint32_t* count) {
  if (!c || (mode != L5DH_MERGE_REDUCE_SCATTER && mode != L5DH_MERGE_ALL_REDUCE)) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  if (c->loopback) return fail(c, -EINVAL, "a loopback group merges through l5dh_merge_all");
  int r;
  if ((r = merge_export(c, mode))) return r;
  if ((r = merge_collectives(&c, 1, mode))) return r;
  return merge_finish(c, mode, out, counts_out, totals_out, first, count);
}

int l5dh_merge_all(l5dh_ctx** ctxs, int n, int mode, l5dh_summary** outs, int32_t** counts_outs, int64_t** totals_outs,
                   uint32_t* firsts, uint32_t* counts) {
  if (!ctxs || n < 1 || (mode != L5DH_MERGE_REDUCE_SCATTER && mode != L5DH_MERGE_ALL_REDUCE)) return -EINVAL;
  for (int i = 0; i < n; ++i)
    if (!ctxs[i] || !(ctxs[i]->comm || ctxs[i]->loopback) || ctxs[i]->loopback != ctxs[0]->loopback ||
        ctxs[i]->nranks != n || ctxs[i]->rank != i)
      return -EINVAL;
  std::vector<std::unique_lock<std::mutex>> locks;
  for (int i = 0; i < n; ++i) locks.emplace_back(ctxs[i]->mu);  // in rank order
  int r;
  for (int i = 0; i < n; ++i) {
    hipSetDevice(ctxs[i]->device);
    if ((r = merge_export(ctxs[i], mode))) return r;
  }
  if ((r = merge_collectives(ctxs, n, mode))) return r;
  for (int i = 0; i < n; ++i) {
    hipSetDevice(ctxs[i]->device);
    if ((r = merge_finish(ctxs[i], mode, outs ? outs[i] : nullptr, counts_outs ? counts_outs[i] : nullptr,
                          totals_outs ? totals_outs[i] : nullptr, firsts ? firsts + i : nullptr,
                          counts ? counts + i : nullptr)))
      return r;
  }
  return 0;
}

int l5dh_tile_totals(l5dh_ctx* c, uint64_t* out, size_t n) {
  if (!c || !out) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (n < c->F) return fail(c, -EINVAL, "tile totals: the output holds fewer than ceil(max_series / 32) entries");
  hipSetDevice(c->device);
  int r;
  if ((r = flush_ring(c))) return r;
  if (c->F == 1) {  // folded at ingest: the batch's samples (invalid ids included)
    out[0] = c->fold_last;
    return sync_stream(c);
  }
  std::vector<uint32_t> k(2 * (size_t)c->F);
  HIPCHK(c, hipMemcpyAsync(k.data(), c->d_kprev, k.size() * 4, hipMemcpyDeviceToHost, c->stream));
  if ((r = sync_stream(c))) return r;
  for (uint32_t t = 0; t < c->F; ++t) out[t] = (uint64_t)k[2 * t] + k[2 * t + 1];
  return 0;
}

int l5dh_partition_redos(l5dh_ctx* c, uint64_t* level1, uint64_t* level2, uint64_t* level2_counted) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  hipSetDevice(c->device);
  int r;
  if ((r = flush_ring(c))) return r;
  const MetaLayout L = meta_layout(c->F);
  static_assert(H_NOVR2 == H_NOVR1 + 1 && H_NCNT2 == H_NOVR1 + 3, "header words read together");
  uint32_t h[MAX_SEG][4] = {};
  if (c->F > 1)
    for (int j = 0; j < MAX_SEG; ++j)
      HIPCHK(c, hipMemcpyAsync(h[j], c->segs[j].meta + L.hdr() + H_NOVR1, 16, hipMemcpyDeviceToHost, c->stream));
  if ((r = sync_stream(c))) return r;
  uint64_t a = 0, b = 0, k = 0;
  for (int j = 0; j < MAX_SEG; ++j) {
    a += h[j][0];
    b += h[j][1];
    k += h[j][3];
  }
  if (level1) *level1 = a;
  if (level2) *level2 = b;
  if (level2_counted) *level2_counted = k;
  return 0;
}

int l5dh_merge_bytes(l5dh_ctx* c, uint64_t* dense, uint64_t* encoded, uint64_t* sent) {
  if (!c) return -EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  if (dense) *dense = c->m_dense_bytes;
  if (encoded) *encoded = c->m_encoded_bytes;
  if (sent) *sent = c->m_sent_bytes;
  return 0;
}

}  // extern "C"
