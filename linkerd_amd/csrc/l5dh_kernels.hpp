// l5dh_kernels.hpp -- device-side layout constants and host launchers for the
// MI355X histogram engine.  See DESIGN.md for the data layout in HBM.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

namespace l5dh {

constexpr int NL = 1797;            // BucketedHistogram.scala:42
constexpr int NB = 1798;            // counts = limits + overflow bucket
constexpr int INT_MAXV = 2147483647;
constexpr int LIM_PAD = 2048;       // limits padded with Int.MaxValue for an 11-step search
constexpr int TILE = 32;            // series per tile (unit of LDS privatization)
constexpr int TILE_SHIFT = 5;
constexpr int ROW = 1800;           // state row stride in u32 (16-B aligned rows)
constexpr int CROW = 900;           // u16-packed cold row in LDS, in u32 words
constexpr int HROW = 1800;          // u32 hot row in LDS
// Binned record (u32), the same at both partition levels and in the final layout:
//   [31:26] tile in super-tile | [25:21] series in tile | [20:0] payload,
//   payload = v = (long)sample when 0 <= v < V_ESC, else V_ESC + bucket (the
//   sample's exact contribution to `total` went to sumfix[series]).
// The accumulate kernels bucketize v (LUT) and sum the payloads below V_ESC.
constexpr uint32_t V_ESC = (1u << 21) - 2048u;
constexpr int MAX_SEG = 8;
constexpr int WG = 1024;            // threads per workgroup of the heavy kernels
constexpr uint32_t COLD_LIMIT_MAX = 65535u;  // u16 LDS bins cannot overflow below this

// LDS bytes of the accumulate kernels: 32 u16-packed rows (cold, big tiles) or 16 u32
// rows (split half-tiles), lane-private value sums, the bucket LUT
constexpr size_t ACC_LDS = (size_t)TILE * CROW * 4 + TILE * 64 * 4 + 1024 * 8 + TILE * 8 + 16;
// cold item of nser series (a tile, or half of one): u16-packed rows, lane-private sums, the LUT, sumfix
constexpr size_t acc_cold_lds(int nser) { return (size_t)nser * CROW * 4 + nser * 64 * 4 + 1024 * 8 + nser * 8 + 16; }
constexpr size_t acc_cold_p_lds(int nser) { return acc_cold_lds(nser) + ROW * 4; }  // + bucket midpoints
// split half-tile: 16 u32 rows, 16 x 64 lane-private u64 value sums, the bucket LUT
constexpr size_t ACC_SPLIT_LDS = (size_t)16 * HROW * 4 + 16 * 64 * 8 + 1024 * 8;
constexpr size_t ACC_HOT_LDS = (size_t)TILE * CROW * 4 + TILE * 64 * 8 + 1024 * 8;  // u16 bins of 32 series, u64 sums

constexpr int LUT_N = 1664;         // bucket bracket LUT: 64 direct + 25 octaves x 64
constexpr int LUT2_N = 1024;        // exact bucket + offset LUT for keys < 2^21 (64 direct + 15 octaves x 64)

struct Tables {            // constant tables in HBM (a few KB each, L2 resident)
  const int32_t* lim_pad;  // [2048] limits padded with Int.MaxValue
  const int32_t* mid;      // [1798] value reported for bucket b
  const int32_t* base;     // [1800] lower limit of bucket b (0 for b == 0), zero padded
  const uint32_t* lut;     // [LUT_N] bucket bracket + in-interval limit offsets (bucket_lut)
  const uint2* lut2;       // [LUT2_N] {o1 | o2 << 16, b0 | p << 16} (bucket_lut2)
};

// Split tiles: the big tiles of the previous batch (<= SPLIT_MAX) are counted,
// binned and laid out per half-tile (series 0-15 | 16-31): a split tile's region
// holds its half-0 records first, then its half-1 records, so the big-tile
// accumulation reads each half as one contiguous range.
constexpr int SPLIT_MAX = 2040;
constexpr int COLS = 2 * SPLIT_MAX;   // count-table columns past F: the half counters of split tiles
// Split-set slot (SPLIT_SLOT u32): [0] NS | [1 + s] tile id (ascending) | bitmap | word prefixes
constexpr int SPLIT_LIST = 1, SPLIT_BITS = 2048, SPLIT_PRE = 3072, SPLIT_SLOT = 4096;
// Per-segment split info (SINFO_WORDS(F) u32): [0] NS | [1 + s] tile | [2048 + s] half-0 records
// | u16 map tile -> s (0xFFFF: not split) from word 4096
constexpr int SINFO_H0 = 2048, SINFO_MAP = 4096;
constexpr size_t sinfo_words(uint32_t F) { return SINFO_MAP + (F + 1) / 2 + 1; }
constexpr uint16_t NO_SPLIT = 0xFFFF;

struct Segs {              // binned ingest batches awaiting aggregation
  const uint32_t* recs[MAX_SEG];
  const uint32_t* tbase[MAX_SEG];  // [F+1] record offset of each tile
  const uint32_t* sinfo[MAX_SEG];  // split info of the segment
  int n;
};

struct Summary88 {
  int64_t count, min, max, sum, p50, p90, p95, p99, p9990, p9999;
  double avg;
};
static_assert(sizeof(Summary88) == 88, "HistogramSummary layout");

struct State {
  uint32_t* counts;        // [S][ROW]
  int64_t* total;          // [S]
  int64_t* sumfix;         // [S] exact sum corrections from escaped records
  uint8_t* dirty;          // [F] tile holds live counts in `counts`
  uint32_t S, F;
};

constexpr uint8_t TF_SPLIT = 2;    // big tile accumulated per half (split in every pending segment)
constexpr uint8_t TF_DIRTY = 4;    // the tile held live counts when k_plan ran

struct Plan {
  uint32_t* tile_tot;      // [F]
  uint32_t* cold_tile;     // [F] cold item -> tile
  uint32_t* hot_item;      // [hot items] big-tile chunk item -> tile | chunk << 15 (mixed halves)
  uint2* split_item;       // [split items] {tile | half << 15, chunk} of split tiles
  uint32_t* hot_list;      // [F] big tiles
  uint8_t* tile_flags;     // [F] TF_*
  uint32_t* header;        // [4] cold items, big tiles, mixed-half items, split items
  uint32_t* header_host;   // [4] the same, written by the plan kernel into pinned host memory
};

struct Outputs {
  Summary88* summ;         // nullable, index = series - first
  int32_t* counts;         // nullable, [count][1798]
  uint32_t first, count;
  int64_t* totals;         // nullable, [count] exact sums (the fleet-merge export)
};

// ---- launchers (all enqueue on `st`) ----
// hint: 2 hot tile ids (or ~0u) used only to merge LDS atomics
// Count table: [G][F + COLS] (tile columns, then the half columns of split tiles).
hipError_t launch_count(const uint32_t* series, size_t n, size_t per, int G, uint32_t S, uint32_t F,
                        uint32_t* table, uint32_t* err, const uint32_t* hint, const uint32_t* split, bool vec,
                        hipStream_t st);
// Column prefixes over slabs (in place) and column totals coltot[F + COLS].
hipError_t launch_colscan(uint32_t* table, int G, uint32_t F, uint32_t* coltot, hipStream_t st);
// Tile totals (split tiles: sum of their halves, written to coltot[t]) and tile_base[F+1].
hipError_t launch_tilescan(uint32_t* coltot, uint32_t F, const uint32_t* split, uint32_t* tile_base, hipStream_t st);
// Both of the above and the segment's split info in one workgroup (F <= 32768).
hipError_t launch_tilescan_seg(uint32_t* coltot, uint32_t F, const uint32_t* split, uint32_t* tile_base,
                               uint32_t* sinfo, hipStream_t st);
// Segment split info from the batch's split set and half-0 totals.
hipError_t launch_seginfo(const uint32_t* split, const uint32_t* coltot, uint32_t F, uint32_t* sinfo, hipStream_t st);
// One-tile series spaces (F == 1): the records are the samples in input order
// (invalid ids: 0xFFFFFFFF), tile_base = {0, n}; no counting pass or partition.
// ... or folded into the tile's state rows at ingest (k_fold1_init + k_fold1, chunks of
// `chunk` samples, a multiple of 4), with no records or segment.  S <= 16: u32 LDS
// bins (wide: the 32-series u16 kernel anyway, A/B).
hipError_t launch_fold1(const uint32_t* series, const float* values, size_t n, uint32_t chunk, State state, Tables tb,
                       uint32_t* err, bool vec, bool wide, hipStream_t st);
hipError_t launch_encode1(const uint32_t* series, const float* values, size_t n, uint32_t S, Tables tb,
                          uint32_t* records, int64_t* sumfix, uint32_t* tile_base, uint32_t* err, bool vec, int num_cu,
                          hipStream_t st);
// Single-level scatter (batches counted without split tiles).
hipError_t launch_bin(const uint32_t* series, const float* values, size_t n, size_t per, int G, uint32_t S,
                      uint32_t F, const uint32_t* table, const uint32_t* tile_base, Tables tb, uint32_t* records,
                      int64_t* sumfix, bool vec, hipStream_t st);
// Two-level partition: k_bin1 (slab -> super-tiles, LDS-sorted runs) + k_bin2
// (super-tile -> tiles).  scratch1 holds n level-1 records.
// Direct tiles (the biggest tiles of THIS batch, <= DIRECT_MAX, from k_count's exact
// totals): two k_bin1 bins each (the halves of a split tile; for an unsplit tile
// both share the tile's range) bypass level 2 -- k_bin1 writes their records
// straight into the final layout.
constexpr int DIRECT_MAX = 255;
constexpr int BIN1_BINS = 1024;     // super-tiles (<= 512) + 2 x direct tiles + the trash bin
// k_bin1 LDS for a sub-chunk of ch slots: stage, cnt, oc, direct words + prefixes, hot slots, hot counters
constexpr size_t bin1_lds(int ch) { return (size_t)ch * 8 + BIN1_BINS * 12 + 1024 * 8 + BIN1_BINS + 9 * 64 * 4 + 32; }
constexpr size_t BIN1_SCRATCH_PAD = 16384 + 16;  // scratch1 entries past n (k_bin1 trash bin, any sub-chunk size)
// Ingest plan (device scratch of PLAN_WORDS u32), written by k_stplan:
constexpr int PLAN_HINT = 2040;     // [4] hot count-table columns: hints for the next batch's k_count
constexpr int PLAN_DBITS = 2048;    // [1024] direct-tile bitmap of this batch (bit t of word t/32)
constexpr int PLAN_DPRE = 3072;     // [1024] direct tiles before word w
constexpr int PLAN_DLIST = 4096;    // [256] direct tile ids, ascending
constexpr int PLAN_DSI = 4352;      // [256] their split index
constexpr int PLAN_ND = 4608;       // number of direct tiles
constexpr int PLAN_HS = 4609;       // 1: one k_bin1 bin holds >= half the batch (lane-private hot slots pay)
constexpr int PLAN_SPLIT = 8192;    // two split-set slots (this batch's, the next batch's)
constexpr int PLAN_ITEMS = PLAN_SPLIT + 2 * SPLIT_SLOT;  // u16 [level-2 item] -> its super-tile
constexpr int PLAN_ITEMS_MAX = (1 << 30) / 16384 + 1024;  // batch / smallest B2_ITEM + FS + 1
constexpr int PLAN_WORDS = PLAN_ITEMS + PLAN_ITEMS_MAX / 2;
// Super-tile plan (level-2 items, direct bins, hot keys) for this batch's split
// set `cur`: its direct tiles are the split tiles with records >= max(thr_min,
// 2^k), k the smallest power keeping <= dmax tiles.  The next batch's split set
// `nxt`: the tiles with records >= max(split_min, 2^k) (<= SPLIT_MAX tiles).
hipError_t launch_stplan(uint32_t F, int G, const uint32_t* coltot, uint32_t* stplan, const uint32_t* cur,
                         uint32_t* nxt, uint32_t thr_min, uint32_t dmax, uint32_t split_min, int hot_bins,
                         const uint32_t* err, uint32_t* err_host, hipStream_t st);
hipError_t launch_bin1(const uint32_t* series, const float* values, size_t n, size_t per, int G, uint32_t S,
                       uint32_t F, const uint32_t* pre, const uint32_t* tile_base, Tables tb, const uint32_t* stplan,
                       const uint32_t* coltot, const uint32_t* split, uint32_t* scratch1, uint32_t* records,
                       int64_t* sumfix, bool vec, int dbg, hipStream_t st);
hipError_t launch_bin2(const uint32_t* scratch1, size_t n, int G, uint32_t F, const uint32_t* pre,
                       const uint32_t* tile_base, const uint32_t* coltot, const uint32_t* split, Tables tb,
                       const uint32_t* stplan, uint32_t* records, int dbg, hipStream_t st);
hipError_t launch_plan(Segs segs, uint32_t F, int final_mode, uint32_t cold_limit, uint32_t hot_chunk,
                       const uint8_t* dirty, Plan plan, hipStream_t st);
// The accumulate launches take UPPER BOUNDS of their item counts (no host round
// trip for the plan header): the kernels are persistent and read the exact counts
// from plan.header on the device.  DEV_COUNT as a count: read it on the device.
constexpr uint32_t DEV_COUNT = 0xFFFFFFFFu;
// direct_out (a resetting snapshot of the whole series space into dense device rows):
// the big tiles that were clean at k_plan count straight into their output rows
// instead of their state rows, and k_hot_finish summarizes them in place.
hipError_t launch_hot_init(Plan plan, uint32_t max_hot, State state, Outputs out, int direct_out, uint32_t hot_chunk,
                           hipStream_t st);
hipError_t launch_accum(Segs segs, Plan plan, uint32_t cold_items, uint32_t max_hot_items, State state, Tables tb,
                        Outputs out, uint32_t cold_limit, uint32_t hot_chunk, int final_mode, int reset,
                        int direct_out, hipStream_t st);
hipError_t launch_accum_split(Segs segs, Plan plan, uint32_t max_split_items, State state, Tables tb,
                              Outputs out, int direct_out, uint32_t hot_chunk, hipStream_t st);
hipError_t launch_hot_finish(Plan plan, uint32_t max_hot, State state, Tables tb, Outputs out, int final_mode,
                             int reset, int direct_out, uint32_t hot_chunk, hipStream_t st);
// Summaries of state rows [first, first+count) (ext == nullptr) or of external
// dense rows ext[count][1798] + ext_total[count].
hipError_t launch_rows(State state, const int32_t* ext, const int64_t* ext_total, Tables tb, Outputs out,
                       int reset, int64_t* totals_out, hipStream_t st);
// Copy n (series, value) pairs from device-visible pinned host memory (zero-copy).
hipError_t launch_fetch_host(const uint32_t* hs, const uint32_t* hv, uint32_t* ds, uint32_t* dv, size_t n,
                             hipStream_t st);
// ---- paged ingest (L5DH_PARAM_BIN_MODE 3, l5dh_paged.hip) ----
// k_bin1's LDS counting sort into CU-private pools of PAGE-record pages (no counting
// pass); direct half-tiles folded into state rows at ingest; level 2 of the other
// tiles counted and placed from a page directory.  Items = KP pages.
constexpr int PG_BINS = BIN1_BINS;
constexpr uint32_t PAGE = 1024;  // records per page (4 KB): a cold bin's slab run fills most of one
constexpr uint32_t KP = 32;     // pages per level-2 item (32K records)
constexpr uint32_t KPD = 256;   // pages per direct-fold item (2^18 records)
constexpr int PD_WORDS = 5136;  // per-bin page / record counts, bases, item bases, header
constexpr size_t PFOLD_LDS = (size_t)16 * HROW * 4 + 16 * 64 * 8 + LUT2_N * 8 + (2 * DIRECT_MAX + 2) * 4;
constexpr size_t P2PLACE_LDS = (size_t)8192 * 8 + 3 * 64 * 4 + 513 * 4;
struct PagedArgs {
  const uint32_t* series;
  const float* values;
  size_t n, per;
  int G, num_cu;
  uint32_t S, F;
  uint32_t* plan;        // the ingest plan: this batch's direct tiles in, the next batch's out
  Tables tb;
  State state;
  uint32_t* err;
  uint32_t pool_pages;   // pages per slab
  uint32_t* pool;        // [G * pool_pages * PAGE] records
  uint2* plog;           // [G * pool_pages] allocation log
  uint32_t* nlog;        // [G]
  uint2* tailpg;         // [G * PG_BINS] last page and its fill
  uint32_t* pd;          // [PD_WORDS]
  uint2* dir;            // [G * pool_pages] page directory
  uint32_t* cnt2;        // [level-2 items * 64]
  uint32_t* tot;         // [F] tile totals of the final layout
  uint32_t* pcount;      // [F] sampled ids per tile (zero between batches)
  uint32_t* err_host;    // mapped pinned word: the invalid-id count, written after level 1
  uint32_t* tile_base;   // [F + 1] the segment's tile offsets
  uint32_t* records;     // the segment's final layout
  uint32_t thr_min, dmax;
  bool vec;
};
size_t paged_pool_pages(size_t per);
hipError_t set_paged_attributes();
// phase 0: direct set (sampled) + level 1, 1: page directory, 2: direct fold, 3: level 2
hipError_t launch_paged_ingest(const PagedArgs& a, int phase, hipStream_t st);

hipError_t set_ingest_attributes();
hipError_t set_snapshot_attributes();
hipError_t set_snapshot_debug(int dbg);
// LUT for bucket_lut: builds lut[LUT_N] from the limits; returns the largest
// number of limits inside one LUT interval (the device search assumes <= 2).
int build_bucket_lut(const int32_t* limits, uint32_t* lut);
// LUT for bucket_lut2 (keys < 2^21), verified exhaustively; 0 on success.
int build_bucket_lut2(const int32_t* limits, uint32_t* lut2);

}  // namespace l5dh
