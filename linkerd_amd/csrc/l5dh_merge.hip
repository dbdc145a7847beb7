// l5dh_merge.hip -- the fleet merge's sparse exchange (l5dh_merge, config C4).
//
// A rank's exported dense rows [Sp][1798] (int32 counts) are mostly zeros (C4: a
// rank holds ~125 samples per series), so the reduce-scatter does not move them
// dense.  Each row is encoded as its non-empty buckets in bucket order, one u32
// per bucket: bucket << 21 | count (count < 2^21 - 1), or bucket << 21 | 0x1FFFFF
// followed by the count's full 32 bits.  A rank sends each other rank the encoding
// of that rank's row slice plus the words per row; the receiver adds the sources'
// entries into LDS rows (one wave per series; a source holds each bucket once, the
// sources are added in rank order -- integer sums, bit-exact), writes the summed
// dense row and summarizes it in the same pass.
//
//   k_mcount   words per row
//   k_menc     the rows' entries at their exclusive word offsets
//   k_mdecode  summed rows of this rank's slice from every source + HistogramSummary
//   k_scan_*   u32 word counts -> u64 exclusive offsets (tile sums, one-workgroup
//              scan of the tile sums, tile scans)
#include <algorithm>

#include "l5dh_device.hpp"
#include "l5dh_merge.hpp"

namespace l5dh {
namespace {

constexpr uint32_t CMAX = MERGE_CMAX;  // count field; CMAX marks an escaped count

__global__ __launch_bounds__(256) void k_mcount(const int32_t* __restrict__ rows, uint32_t nrows,
                                                uint32_t* __restrict__ words) {
  const uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const int lane = lane_id();
  const int32_t* row = rows + (size_t)r * NB;
  uint32_t w = 0;
  for (int b = lane; b < NB; b += 64) {
    const uint32_t c = (uint32_t)row[b];
    w += (c != 0u) + (c >= CMAX);
  }
  w = (uint32_t)wave_sum((uint64_t)w);
  if (lane == 0) words[r] = w;
}

__global__ __launch_bounds__(256) void k_menc(const int32_t* __restrict__ rows, uint32_t nrows,
                                              const uint64_t* __restrict__ offs, uint32_t* __restrict__ enc) {
  const uint32_t r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrows) return;
  const int lane = lane_id();
  const int32_t* row = rows + (size_t)r * NB;
  uint64_t at = offs[r];
  for (int b0 = 0; b0 < NB; b0 += 64) {  // 64 buckets per step, compacted by ballots
    const int b = b0 + lane;
    const uint32_t c = b < NB ? (uint32_t)row[b] : 0u;
    const bool nz = c != 0u, esc = c >= CMAX;
    const unsigned long long mn = __ballot(nz), me = __ballot(esc);
    const uint32_t pos = mask_below(mn) + mask_below(me);
    if (nz) {
      enc[at + pos] = ((uint32_t)b << 21) | (esc ? CMAX : c);
      if (esc) enc[at + pos + 1] = c;
    }
    at += (uint64_t)(__popcll(mn) + __popcll(me));
  }
}

// The sparse export's rows (encoded at their tiles' places by the accumulate kernels)
// packed in row order.  The 16 rows of a half-tile are contiguous in the unpacked
// encoding (each accumulate path writes a half's rows back to back from the half's
// first word) and in the packed one, so a wave copies one half-tile as ONE range:
// roff of its first row, offs of its first and past-last rows (loads unrolled 4 deep).
__global__ __launch_bounds__(256) void k_mpack(const uint32_t* __restrict__ src, const uint32_t* __restrict__ roff,
                                               const uint64_t* __restrict__ offs, uint32_t nrows,
                                               uint32_t* __restrict__ enc) {
  const uint32_t r = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 16u;
  if (r >= nrows) return;  // (wave-uniform)
  const uint32_t e = min(r + 16u, nrows);
  const uint64_t o0 = offs[r];
  const uint32_t n = (uint32_t)(offs[e] - o0);
  if (n == 0) return;
  const uint32_t* __restrict__ a = src + roff[r];
  uint32_t* __restrict__ o = enc + o0;
  const uint32_t lane = (uint32_t)lane_id();
  for (uint32_t i0 = 0; i0 < n; i0 += 256) {
    uint32_t x[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t i = i0 + 64u * q + lane;
      x[q] = i < n ? a[i] : 0u;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t i = i0 + 64u * q + lane;
      if (i < n) o[i] = x[q];
    }
  }
}

// A wave per series of the slice at a time: the LDS row accumulates every source's
// entries (a source's words are parsed 64 at a time; escape headers are rare, resolved
// by a loop over their ballot), then the dense row, the total and the summary.  The
// sources' word counts and offsets of a row come with one load per lane (the next
// row's while this one is decoded), the first chunks of MDEC_BATCH sources with loads
// in flight together.
constexpr int MDEC_WAVES = 4, MDEC_BATCH = 8, MDEC_GRID = 1280;  // (5 workgroups per CU: 28.8 KB of LDS each)
constexpr int MDEC_AHEAD = 4;
__global__ __launch_bounds__(64 * MDEC_WAVES) void k_mdecode(MergeRecv src, uint32_t nrows,
                                                             const int64_t* __restrict__ totals, Tables tb,
                                                             int32_t* __restrict__ out_rows,
                                                             Summary88* __restrict__ out_summ) {
  __shared__ __attribute__((aligned(16))) uint32_t lrow[MDEC_WAVES][ROW];
  const int w = threadIdx.x >> 6;
  const int lane = lane_id();
  // persistent waves: rows r, r + GW, ...; the next row's word counts and offsets are
  // loaded while this row is decoded (no barriers: a wave owns its LDS row)
  const uint32_t GW = gridDim.x * MDEC_WAVES;
  uint32_t r = blockIdx.x * MDEC_WAVES + w;
  uint32_t* row = lrow[w];
  for (int b = lane; b < ROW / 4; b += 64) reinterpret_cast<uint4*>(row)[b] = make_uint4(0u, 0u, 0u, 0u);
  const uint32_t* __restrict__ enc = src.enc;
  auto meta = [&](uint32_t rr, uint32_t& n, uint64_t& o) {  // lane s: source s's row rr
    const bool ok = rr < nrows && lane < src.n;
    const size_t ix = (size_t)lane * src.per + (rr < nrows ? rr : 0u);
    n = ok ? src.words[ix] : 0u;
    o = ok ? src.offs[ix] : 0ull;
  };
  // (a long row -- the head series hold up to 1798 words per source -- has its chunks
  // after the first loaded MDEC_AHEAD at a time: one load latency per group of chunks,
  // not per chunk; round 5 waited for each, which made the slice holding the head the
  // slowest rank)
  auto parse = [&](uint32_t x0, uint32_t nw, uint64_t off) {
    bool carry = false;  // the chunk's first word is the count of the previous chunk's last header
    static_assert(MDEC_AHEAD == 4, "four chunk registers");
    uint32_t xa0 = 0, xa1 = 0, xa2 = 0, xa3 = 0;  // chunks 4 g + 1 .. 4 g + 4 (no dynamic register index)
    for (uint32_t base = 0; base < nw; base += 64) {
      const uint32_t i = base + (uint32_t)lane;
      const bool valid = i < nw;
      const uint32_t c = base >> 6;
      if (c % 4u == 1u) {  // chunks c .. c + 3 in flight together
        xa0 = i < nw ? enc[off + i] : 0u;
        xa1 = i + 64u < nw ? enc[off + i + 64u] : 0u;
        xa2 = i + 128u < nw ? enc[off + i + 128u] : 0u;
        xa3 = i + 192u < nw ? enc[off + i + 192u] : 0u;
      }
      const uint32_t k4 = (c + 3u) % 4u;  // chunk c's register (c >= 1)
      const uint32_t x = c == 0 ? x0 : k4 == 0 ? xa0 : k4 == 1 ? xa1 : k4 == 2 ? xa2 : xa3;
      unsigned long long hm = __ballot(valid && (x & CMAX) == CMAX);  // escape headers, or counts that look like one
      unsigned long long pay = 0ull;
      if (carry) {
        pay |= 1ull;
        hm &= ~1ull;
      }
      bool next_carry = false;
      while (hm) {  // headers in order: the word after a header is its count, never a header
        const int h = __ffsll((long long)hm) - 1;
        hm &= ~(1ull << h);
        if (h == 63) {
          next_carry = true;
        } else {
          pay |= 1ull << (h + 1);
          hm &= ~(1ull << (h + 1));
        }
      }
      const uint32_t nxt = __shfl_down(x, 1, 64);
      if (valid && !((pay >> lane) & 1ull)) {
        const uint32_t b = x >> 21;
        uint32_t c = x & CMAX;
        if (c == CMAX) c = lane == 63 ? enc[off + i + 1] : nxt;
        atomicAdd(&row[b], c);  // (an LDS add: no read-modify-write latency; a source holds each bucket once)
      }
      carry = next_carry;
    }
  };
  uint32_t nwl;
  uint64_t offl;
  meta(r, nwl, offl);
  for (; r < nrows; r += GW) {
    const uint32_t cnw = nwl;
    const uint64_t coff = offl;
    meta(r + GW, nwl, offl);
    for (int s0 = 0; s0 < src.n; s0 += MDEC_BATCH) {  // (s0 <= 56: every lane index below is < 64)
      uint32_t xs[MDEC_BATCH], nws[MDEC_BATCH];
      uint64_t offs[MDEC_BATCH];
#pragma unroll
      for (int k = 0; k < MDEC_BATCH; ++k) {
        nws[k] = s0 + k < src.n ? (uint32_t)__builtin_amdgcn_readlane((int)cnw, s0 + k) : 0u;
        offs[k] = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)coff, s0 + k) |
                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(coff >> 32), s0 + k) << 32);
        xs[k] = (uint32_t)lane < nws[k] ? enc[offs[k] + lane] : 0u;
      }
#pragma unroll
      for (int k = 0; k < MDEC_BATCH; ++k) parse(xs[k], nws[k], offs[k]);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    const SrcLds32 lds{row};
    if (out_rows) {
      int32_t* orow = out_rows + (size_t)r * NB;
      for (int q = lane; q < NB4; q += 64) store4_1798(orow, 4 * q, lds.get4(4 * q));
    }
    uint32_t g[9];
    const int ng = lane_groups(lane);
#pragma unroll
    for (int q = 0; q < 9; ++q) g[q] = q < ng ? sum4(lds.get4(28 * lane + 4 * q)) : 0u;
    wave_summary(g, lds, totals ? totals[r] : 0, tb.mid, out_summ ? out_summ + r : nullptr);
    // cleared for the next row (this wave's LDS operations stay in order: the reads come first)
    for (int b = lane; b < ROW / 4; b += 64) reinterpret_cast<uint4*>(row)[b] = make_uint4(0u, 0u, 0u, 0u);
  }
}

// Exclusive u64 prefix of n u32 counts in tiles of SCAN_TILE: k_scan_sums writes
// each tile's sum, k_scan_top (one workgroup) scans the tile sums in place, and
// k_scan_tiles scans each tile from its offset.  tmp = the tile sums.
constexpr int SCAN_NT = 256, SCAN_PT = 16, SCAN_TILE = SCAN_NT * SCAN_PT;

__device__ __forceinline__ uint64_t block_scan256(uint64_t v, uint64_t* red /*[5]*/, uint64_t* total) {
  const int lane = lane_id(), w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan(v);
  if (lane == 63) red[w] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t acc = 0;
    for (int k = 0; k < SCAN_NT / 64; ++k) {
      const uint64_t q = red[k];
      red[k] = acc;
      acc += q;
    }
    red[SCAN_NT / 64] = acc;
  }
  __syncthreads();
  const uint64_t r = red[w] + incl - v;
  *total = red[SCAN_NT / 64];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(SCAN_NT) void k_scan_sums(const uint32_t* __restrict__ x, uint32_t n,
                                                       uint64_t* __restrict__ sums) {
  __shared__ uint64_t red[SCAN_NT / 64 + 1];
  const uint32_t base = blockIdx.x * (uint32_t)SCAN_TILE + threadIdx.x * SCAN_PT;
  uint64_t v = 0;
  for (int k = 0; k < SCAN_PT; ++k) v += base + k < n ? x[base + k] : 0u;
  uint64_t t;
  block_scan256(v, red, &t);
  if (threadIdx.x == 0) sums[blockIdx.x] = t;
}

__global__ __launch_bounds__(SCAN_NT) void k_scan_top(uint64_t* __restrict__ sums, uint32_t nt) {
  __shared__ uint64_t red[SCAN_NT / 64 + 1];
  uint64_t carry = 0;
  for (uint32_t c = 0; c < nt; c += SCAN_NT) {
    const uint32_t i = c + threadIdx.x;
    const uint64_t v = i < nt ? sums[i] : 0ull;
    uint64_t t;
    const uint64_t e = block_scan256(v, red, &t);
    if (i < nt) sums[i] = carry + e;
    carry += t;
  }
}

__global__ __launch_bounds__(SCAN_NT) void k_scan_tiles(const uint32_t* __restrict__ x, uint32_t n,
                                                        const uint64_t* __restrict__ sums, uint64_t* __restrict__ out) {
  __shared__ uint64_t red[SCAN_NT / 64 + 1];
  const uint32_t base = blockIdx.x * (uint32_t)SCAN_TILE + threadIdx.x * SCAN_PT;
  uint32_t v[SCAN_PT];
  uint64_t s = 0;
  for (int k = 0; k < SCAN_PT; ++k) {
    v[k] = base + k < n ? x[base + k] : 0u;
    s += v[k];
  }
  uint64_t t;
  uint64_t e = sums[blockIdx.x] + block_scan256(s, red, &t);
  for (int k = 0; k < SCAN_PT; ++k) {
    if (base + k < n) out[base + k] = e;
    e += v[k];
  }
}

hipError_t exclusive_scan_u32_u64(const uint32_t* x, uint32_t n, uint64_t* out, void* tmp, hipStream_t st) {
  if (n == 0) return hipSuccess;
  const uint32_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  uint64_t* sums = static_cast<uint64_t*>(tmp);
  hipLaunchKernelGGL(k_scan_sums, dim3(nt), dim3(SCAN_NT), 0, st, x, n, sums);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_NT), 0, st, sums, nt);
  hipLaunchKernelGGL(k_scan_tiles, dim3(nt), dim3(SCAN_NT), 0, st, x, n, (const uint64_t*)sums, out);
  return hipGetLastError();
}

size_t scan_tmp_bytes(uint32_t n) { return ((size_t)n / SCAN_TILE + 2) * 8; }

// The loopback transport's reductions: element-wise sums over the group's buffers.
template <class T>
struct SrcList {
  const T* p[MERGE_MAX_RANKS];
  int n;
};
template <class T>
__global__ __launch_bounds__(256) void k_loop_sum(SrcList<T> src, T* __restrict__ dst, size_t count) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
    T acc = 0;
    for (int k = 0; k < src.n; ++k) acc += src.p[k][i];
    dst[i] = acc;
  }
}
template <class T>
hipError_t loop_sum(const T* const* srcs, int n, T* dst, size_t count, hipStream_t st) {
  if (count == 0) return hipSuccess;
  if (n < 1 || n > MERGE_MAX_RANKS) return hipErrorInvalidValue;
  SrcList<T> l{};
  for (int k = 0; k < n; ++k) l.p[k] = srcs[k];
  l.n = n;
  const size_t blocks = std::min<size_t>((count + 255) / 256, 4096);
  hipLaunchKernelGGL(k_loop_sum<T>, dim3((unsigned)blocks), dim3(256), 0, st, l, dst, count);
  return hipGetLastError();
}

// The loopback transport's copies, one launch for many: entry blockIdx.y of the list,
// its words strided over blockIdx.x.
__global__ __launch_bounds__(256) void k_loop_copy(LoopCopies l) {
  const int e = blockIdx.y;
  if (e >= l.n) return;
  const uint32_t* __restrict__ src = l.src[e];
  uint32_t* __restrict__ dst = l.dst[e];
  const uint64_t n = l.words[e];
  for (uint64_t i0 = (uint64_t)blockIdx.x * 2048u; i0 < n; i0 += (uint64_t)gridDim.x * 2048u) {
    uint32_t x[8];  // 8 loads in flight per thread
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint64_t i = i0 + 256u * q + threadIdx.x;
      x[q] = i < n ? src[i] : 0u;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const uint64_t i = i0 + 256u * q + threadIdx.x;
      if (i < n) dst[i] = x[q];
    }
  }
}

// One rank's row of the W x W size matrix: words of each destination's slice.
__global__ void k_msizes(const uint64_t* __restrict__ offs, uint32_t per, int W, uint64_t* __restrict__ row) {
  const int q = threadIdx.x;
  if (q < W) row[q] = offs[(size_t)(q + 1) * per] - offs[(size_t)q * per];
}

}  // namespace

hipError_t merge_sizes_row(const uint64_t* offs, uint32_t per, int W, uint64_t* row, hipStream_t st) {
  if (W < 1 || W > MERGE_MAX_RANKS) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_msizes, dim3(1), dim3(64), 0, st, offs, per, W, row);
  return hipGetLastError();
}

hipError_t merge_loop_copy(const LoopCopies& l, hipStream_t st) {
  if (l.n == 0) return hipSuccess;
  if (l.n < 0 || l.n > LOOP_COPIES_MAX) return hipErrorInvalidValue;
  uint64_t most = 0;
  for (int e = 0; e < l.n; ++e) most = std::max<uint64_t>(most, l.words[e]);
  const uint32_t gx = (uint32_t)std::min<uint64_t>((most + 2047) / 2048, 256);
  hipLaunchKernelGGL(k_loop_copy, dim3(std::max(gx, 1u), (unsigned)l.n), dim3(256), 0, st, l);
  return hipGetLastError();
}

hipError_t merge_loop_sum_i32(const int32_t* const* srcs, int n, int32_t* dst, size_t count, hipStream_t st) {
  return loop_sum(srcs, n, dst, count, st);
}
hipError_t merge_loop_sum_i64(const int64_t* const* srcs, int n, int64_t* dst, size_t count, hipStream_t st) {
  return loop_sum(srcs, n, dst, count, st);
}

hipError_t merge_count(const int32_t* rows, uint32_t nrows, uint32_t* words, uint64_t* offs, void* tmp,
                       size_t* tmp_bytes, hipStream_t st) {
  if (!tmp) {  // size query of the scan's temporary storage
    *tmp_bytes = scan_tmp_bytes(nrows + 1);
    return hipSuccess;
  }
  // rows == nullptr: words[0..nrows) were written by the export (Outputs::words)
  if (rows && nrows) hipLaunchKernelGGL(k_mcount, dim3((nrows + 3) / 4), dim3(256), 0, st, rows, nrows, words);
  hipError_t e = hipMemsetAsync(words + nrows, 0, 4, st);  // offs[nrows] = the total
  if (e != hipSuccess) return e;
  return exclusive_scan_u32_u64(words, nrows + 1, offs, tmp, st);
}

hipError_t merge_encode(const int32_t* rows, uint32_t nrows, const uint64_t* offs, uint32_t* enc, hipStream_t st) {
  if (nrows == 0) return hipSuccess;
  hipLaunchKernelGGL(k_menc, dim3((nrows + 3) / 4), dim3(256), 0, st, rows, nrows, offs, enc);
  return hipGetLastError();
}

hipError_t merge_pack(const uint32_t* src, const uint32_t* roff, const uint64_t* offs, uint32_t nrows, uint32_t* enc,
                      hipStream_t st) {
  if (nrows == 0) return hipSuccess;
  const uint32_t halves = (nrows + 15) / 16;
  hipLaunchKernelGGL(k_mpack, dim3((halves + 3) / 4), dim3(256), 0, st, src, roff, offs, nrows, enc);
  return hipGetLastError();
}

hipError_t merge_offsets(const uint32_t* words, uint32_t nrows, uint64_t* offs, void* tmp, size_t tmp_bytes,
                         hipStream_t st) {
  if (tmp_bytes < scan_tmp_bytes(nrows)) return hipErrorInvalidValue;
  return exclusive_scan_u32_u64(words, nrows, offs, tmp, st);
}

hipError_t merge_decode(const MergeRecv& src, uint32_t nrows, const int64_t* totals, Tables tb, int32_t* out_rows,
                        Summary88* out_summ, hipStream_t st) {
  if (nrows == 0) return hipSuccess;
  if (src.n < 1 || src.n > MERGE_MAX_RANKS || nrows > src.per) return hipErrorInvalidValue;
  const uint32_t grid = std::min<uint32_t>((nrows + MDEC_WAVES - 1) / MDEC_WAVES, (uint32_t)MDEC_GRID);
  hipLaunchKernelGGL(k_mdecode, dim3(grid), dim3(64 * MDEC_WAVES), 0, st, src, nrows,
                     totals, tb, out_rows, out_summ);
  return hipGetLastError();
}

}  // namespace l5dh
