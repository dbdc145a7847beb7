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
constexpr int ST_TILES = 64;        // tiles per super-tile (the level-1 partition unit)
constexpr int ST_SHIFT = 11;        // 64 tiles x 32 series
constexpr int ROW = 1800;           // state row stride in u32 (16-B aligned rows)
constexpr int CROW = 900;           // u16-packed cold row in LDS, in u32 words
constexpr int HROW = 1800;          // u32 hot row in LDS
// Level-1 record of a super-tile bin (u32, rec32):
//   [31:26] tile in super-tile | [25:21] series in tile | [20:0] payload,
//   payload = v = (long)sample when 0 <= v < V_ESC, else V_ESC + bucket (the
//   sample's exact contribution to `total` went to sumfix[series]).
// Final record (u16, rec16): [15:11] series in tile | [10:0] bucket.  Level 1 writes
//   them for the direct tiles (bucketized there, value sums folded in LDS into
//   sumfix), level 2 for the other tiles (value sums folded per super-tile).
constexpr uint32_t V_ESC = (1u << 21) - 2048u;
constexpr int MAX_SEG = 8;
constexpr int WG = 1024;            // threads per workgroup of the heavy kernels
constexpr uint32_t COLD_LIMIT_MAX = 65535u;  // u16 LDS bins cannot overflow below this

// LDS bytes of the accumulate kernels: 16 u16-packed rows + the half-tile's sumfix + the
// bucket midpoints (cold half-tiles), 16 u32 rows (big half-tiles)
constexpr size_t ACC_COLDH_LDS = (size_t)16 * CROW * 4 + 16 * 8 + ROW * 4;  // half-tile cold items
constexpr int ENC_LIST = 256;  // (sparse export) first-touched buckets listed per row of a half-tile item
constexpr size_t ACC_COLDHE_LDS = ACC_COLDH_LDS + 2 * 16 * 4 + (size_t)16 * ENC_LIST * 2;
constexpr size_t ACC_SPLIT_LDS = (size_t)16 * HROW * 4;
// k_fold1 (samples, not records): u32 rows of 16 series or u16-packed rows of 32, lane-private
// u64 value sums, the bucket LUT
constexpr size_t FOLD16_LDS = (size_t)16 * HROW * 4 + 16 * 64 * 8 + 1024 * 8;
constexpr size_t FOLD32_LDS = (size_t)TILE * CROW * 4 + TILE * 64 * 8 + 1024 * 8;

constexpr int LUT_N = 1664;         // bucket bracket LUT: 64 direct + 25 octaves x 64
constexpr int LUT2_N = 1024;        // exact bucket + offset LUT for keys < 2^21 (64 direct + 15 octaves x 64)

struct Tables {            // constant tables in HBM (a few KB each, L2 resident)
  const int32_t* lim_pad;  // [2048] limits padded with Int.MaxValue
  const int32_t* mid;      // [1798] value reported for bucket b
  const int32_t* base;     // [1800] lower limit of bucket b (0 for b == 0), zero padded
  const uint32_t* lut;     // [LUT_N] bucket bracket + in-interval limit offsets (bucket_lut)
  const uint2* lut2;       // [LUT2_N] {o1 | o2 << 16, b0 | p << 16} (bucket_lut2)
  const uint2* lut3;       // [LUT2_N] {b0 | lim1 << 11, lim2}: level 1's decode (build_bucket_lut3)
};

// ---- binned segments (one ingest batch each) -------------------------------
// Every (tile, half) "key" k = 2 t + h of a segment is ONE contiguous range of u16
// records: [kbase[k], kbase[k] + kcnt[k]) of rec16 -- written by level 1 when tile
// t is a direct tile of the batch (regions [0, H_D16)), by level 2 otherwise.
// Segment metadata (u32 words, `meta`), K = 2 F keys:
constexpr int DIRECT_MAX = 255;     // direct tiles per batch
constexpr int BIN1_BINS = 1024;     // level-1 bins: super-tiles (<= 512) + 2 x direct tiles + the trash bin
constexpr uint32_t ITEM2 = 6144;    // level-1 records per level-2 item (two level-2 workgroups per CU)
struct MetaLayout {
  uint32_t K;
  __host__ __device__ constexpr uint32_t kbase() const { return 0; }
  __host__ __device__ constexpr uint32_t kcnt() const { return K; }
  __host__ __device__ constexpr uint32_t kcap() const { return 2 * K; }
  __host__ __device__ constexpr uint32_t dbits() const { return 3 * K; }             // [1024] direct tiles bitmap
  __host__ __device__ constexpr uint32_t dpre() const { return 3 * K + 1024; }       // [1024] direct tiles before word w
  __host__ __device__ constexpr uint32_t dlist() const { return 3 * K + 2048; }      // [256] direct tile ids, ascending
  __host__ __device__ constexpr uint32_t bbase() const { return 3 * K + 2304; }      // [1024] level-1 bin region base
  __host__ __device__ constexpr uint32_t bcnt() const { return 3 * K + 3328; }       // [1024] bin cursor (= records)
  __host__ __device__ constexpr uint32_t bcap() const { return 3 * K + 4352; }       // [1024] bin region capacity
  __host__ __device__ constexpr uint32_t btot() const { return 3 * K + 5376; }       // [1024] exact bin totals
  __host__ __device__ constexpr uint32_t hdr() const { return 3 * K + 6400; }        // [64] header (H_*)
  __host__ __device__ constexpr uint32_t istart() const { return 3 * K + 6464; }     // [513] level-2 items per super-tile
  __host__ __device__ constexpr uint32_t wsum() const { return 3 * K + 6980; }       // u64 [64] per-workgroup key sums
  __host__ __device__ constexpr uint32_t words() const { return 3 * K + 7108; }
};
__host__ __device__ constexpr MetaLayout meta_layout(uint32_t F) { return MetaLayout{2 * F}; }
// header words
enum : uint32_t {
  H_ND = 0,       // direct tiles
  H_OV1 = 1,      // a level-1 run did not fit its region
  H_REDO1 = 2,    // level 1 runs again with exact regions
  H_OV2 = 3,      // a level-2 run did not fit its region
  H_REDO2 = 4,    // level 2 runs again with exact regions
  H_ITEMS = 5,    // level-2 items
  H_COUNT2 = 6,   // level 2's regions are known not to fit: its first pass only counts
  // (7-8: unused)
  H_EXACT = 9,    // 1: every sample of the batch was counted by k_rsample
  H_NOVR1 = 10,   // level-1 redos (diagnostics, monotonic per segment slot)
  H_NOVR2 = 11,   // level-2 redos after an overflow
  H_D16 = 12,     // rec16 records reserved for the direct keys' regions (level-2 regions follow)
  H_NCNT2 = 13    // level-2 counting first passes (H_COUNT2; monotonic)
};
constexpr uint32_t NOKEY = 0xFFFFFFFFu;

struct Segs {              // binned ingest batches awaiting aggregation
  const uint16_t* rec16[MAX_SEG];
  const uint32_t* meta[MAX_SEG];
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
  int64_t* sumfix;         // [S] exact sum contributions not carried by the records (escapes, level-2 sums)
  uint8_t* dirty;          // [F] tile holds live counts in `counts`
  uint32_t S, F;
};

constexpr uint32_t CI_DIRTY = 1u << 30;  // cold item: the tile held live counts
constexpr uint8_t TF_SPLIT = 2;    // big tile, accumulated per half
constexpr uint8_t TF_DIRTY = 4;    // the tile held live counts when k_plan ran
constexpr uint8_t TF_SOLO = 8;     // big tile of a direct_out snapshot, clean, each half ONE item:
                                   // k_accum_split writes its output rows and summaries itself

struct Plan {
  uint32_t* tile_tot;      // [F]
  uint32_t* enc_base;      // [F] (sparse export) the tile's first word in the unpacked encoding
  uint32_t* enc_h0;        // [F] (sparse export) words reserved for half 0 of a big or dirty tile (half 1 follows)
  uint32_t* enc_dw;        // [2F] (sparse export) words of each half of a dirty tile's state rows (k_enc_dirty)
  uint4* cold_item;        // [F] cold item -> {tile | CI_DIRTY, a0, a1, n0 | n1 << 16}: segment 0's
                           // key ranges (rec16) of the tile's halves
  uint2* split_item;       // [split items] {tile | half << 15, chunk} of big tiles
  uint32_t* hot_list;      // [F] big tiles
  uint8_t* tile_flags;     // [F] TF_*
  uint32_t* header;        // [4] cold items, big tiles, cold-item counter, split items; [4 + k B + b] per-workgroup
                           // sums of quantity k (B = ceil(F / 1024) plan workgroups); [4 + 4 B] split-item
                           // counter; [5 + 4 B] the unpacked encoding's words (sparse export)
  uint32_t* big_hint;      // pinned, host-mapped word: this plan's big tiles (the host reads the last value
                           // it sees only to pick the accumulate's launch order)
};
__host__ __device__ constexpr uint32_t plan_header_words(uint32_t F) { return 6 + 4 * ((F + 1023) / 1024); }
// Sparse export (the fleet merge's reduce-scatter): words a tile's rows may take in the
// unpacked encoding (a row: one word per non-empty bucket, a second one per count >=
// MERGE_CMAX) -- a clean cold tile at most its records (<= 65535 per tile: no escaped
// counts); a half of a clean big tile min(its records, 16 NB) + records / MERGE_CMAX;
// a half of a dirty tile its state rows' words (counted by k_enc_dirty) + 2 per record
// (a record adds at most one non-empty bucket and one escape); never more than
// ENC_HALF_CAP.  So the unpacked encoding of F <= 2^15 tiles stays below 2^32 words,
// and near the records (not 2x the dense rows) unless the state rows are dense.
constexpr uint32_t ENC_HALF_CAP = 16u * 2u * NB + 16u;
static_assert((uint64_t)((1u << 20) / TILE) * 2u * ENC_HALF_CAP < (1ull << 32),
              "the unpacked encoding's u32 word offsets (L5DH_MAX_SERIES = 2^20 series)");

struct Outputs {
  Summary88* summ;         // nullable, index = series - first
  int32_t* counts;         // nullable, [count][1798]
  uint32_t first, count;
  int64_t* totals;         // nullable, [count] exact sums (the fleet-merge export)
  uint32_t* words;         // nullable, [count] the fleet merge's encoding words per row: non-empty
                           // buckets + counts >= MERGE_CMAX (which take a second word)
  uint32_t* enc;           // nullable: sparse export -- the rows' encodings (unpacked: at Plan::enc_base of
                           // their tile) instead of dense rows (counts must be null, summ null)
  uint32_t* roff;          // [count] with enc: each row's first word in enc
};
constexpr uint32_t MERGE_CMAX = 0x1FFFFFu;  // count field of a merge entry; CMAX marks an escaped count

// ---- ingest launchers (l5dh_ingest.hip; all enqueue on `st`) ----
struct IngestArgs {
  const uint32_t* series;
  const float* values;
  size_t n, per;           // samples; samples per slab (multiple of 4)
  int G;                   // slabs (k_rbin1 workgroups)
  int num_cu;
  uint32_t S, F;
  Tables tb;
  int64_t* sumfix;
  uint32_t* err;           // invalid-id counter (monotonic)
  uint32_t* err_host;      // mapped pinned word: the counter, copied after level 1
  uint32_t* kest;          // [K] sampled ids per key (zero between batches)
  uint32_t* kprev;         // [K] exact records per key of the previous batch
  uint32_t* meta;          // the segment's metadata
  uint32_t* rec32;         // [cap32]
  uint16_t* rec16;         // [cap16]
  size_t cap32, cap16;
  size_t dlim16;           // rec16 records the direct keys' regions may take ([0, dlim16); level 2 gets the rest)
  uint32_t thr_min, dmax;  // direct tiles: >= thr_min estimated records, at most dmax of them
  uint32_t pct;            // region capacity scale, percent (100: as predicted)
  bool vec;                // 16-B aligned inputs
};
// Stages: 0 = sample + plans (level-1 bins and direct tiles, level-2 regions), 1 = level 1
// (+ its fix-up: exact totals, level-2 items; + redo), 3 = level 2 (+ fix-up, redo).
hipError_t launch_ingest(const IngestArgs& a, int stage, hipStream_t st);
hipError_t set_ingest_attributes();

// One-tile series spaces (F == 1): folded into the tile's state rows at ingest
// (k_fold1_init + k_fold1, chunks of `chunk` samples, a multiple of 4), with no
// records or segment.  S <= 16: u32 LDS bins (wide: the 32-series u16 kernel anyway).
hipError_t launch_fold1(const uint32_t* series, const float* values, size_t n, uint32_t chunk, State state, Tables tb,
                        uint32_t* err, bool vec, bool wide, hipStream_t st);

// ---- snapshot launchers (l5dh_snapshot.hip) ----
hipError_t launch_enc_dirty(State st, Plan plan, hipStream_t st_);
hipError_t launch_plan(Segs segs, uint32_t F, int final_mode, uint32_t cold_limit, uint32_t hot_chunk,
                       const uint8_t* dirty, int direct_out, int encode, Plan plan, hipStream_t st);
// The accumulate launches take UPPER BOUNDS of their item counts (no host round
// trip for the plan header): the kernels are persistent and read the exact counts
// from plan.header on the device.  DEV_COUNT as a count: read it on the device.
constexpr uint32_t DEV_COUNT = 0xFFFFFFFFu;
// direct_out (a resetting snapshot of the whole series space into dense device rows):
// the big tiles that were clean at k_plan count straight into their output rows
// instead of their state rows, and k_hot_finish summarizes them in place.
hipError_t launch_hot_init(Plan plan, uint32_t max_hot, State state, Outputs out, int direct_out, hipStream_t st);
hipError_t launch_accum_cold(Segs segs, Plan plan, uint32_t cold_items, State state, Tables tb, Outputs out,
                             int final_mode, int reset, hipStream_t st);
hipError_t launch_accum_split(Segs segs, Plan plan, uint32_t max_split_items, State state, Tables tb,
                              Outputs out, int direct_out, uint32_t hot_chunk, hipStream_t st);
hipError_t launch_hot_finish(Plan plan, uint32_t max_hot, State state, Tables tb, Outputs out, int final_mode,
                             int reset, int direct_out, hipStream_t st);
// Summaries of state rows [first, first+count) (ext == nullptr) or of external
// dense rows ext[count][1798] + ext_total[count].
hipError_t launch_rows(State state, const int32_t* ext, const int64_t* ext_total, Tables tb, Outputs out,
                       int reset, int64_t* totals_out, hipStream_t st);
// Copy n (series, value) pairs from device-visible pinned host memory (zero-copy).
hipError_t launch_fetch_host(const uint32_t* hs, const uint32_t* hv, uint32_t* ds, uint32_t* dv, size_t n,
                             hipStream_t st);
hipError_t set_snapshot_attributes();

// LUT for bucket_lut: builds lut[LUT_N] from the limits; returns the largest
// number of limits inside one LUT interval (the device search assumes <= 2).
int build_bucket_lut(const int32_t* limits, uint32_t* lut);
// LUT for bucket_lut2 (keys < 2^21), verified exhaustively; 0 on success.
int build_bucket_lut2(const int32_t* limits, uint32_t* lut2);
int build_bucket_lut3(const int32_t* limits, uint32_t* lut3);

}  // namespace l5dh
