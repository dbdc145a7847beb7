// l5dh_merge.hpp -- the fleet merge's sparse row exchange (l5dh_merge.hip).
#pragma once

#include "l5dh_kernels.hpp"

namespace l5dh {

constexpr int MERGE_MAX_RANKS = 64;

struct MergeRecv {  // the encodings of this rank's row slice from every source rank, source by source
  const uint32_t* enc;    // entries: source 0's rows, then source 1's, ...
  const uint32_t* words;  // [n][per] words per row
  const uint64_t* offs;   // [n][per] exclusive offsets of the rows' words in enc (one scan of words)
  uint32_t per;           // rows per source slice
  int n;                  // sources (<= MERGE_MAX_RANKS)
};

// words[r] = entry words of row r (words needs nrows + 1 slots; rows == nullptr: already
// there, from the export), offs[0..nrows] their exclusive prefix (offs[nrows] = the
// total).  tmp == nullptr: *tmp_bytes receives the scan's temporary storage size.
hipError_t merge_count(const int32_t* rows, uint32_t nrows, uint32_t* words, uint64_t* offs, void* tmp,
                       size_t* tmp_bytes, hipStream_t st);
hipError_t merge_encode(const int32_t* rows, uint32_t nrows, const uint64_t* offs, uint32_t* enc, hipStream_t st);
// the sparse export's row encodings (row r at src + roff[r]; the 16 rows of a half-tile back
// to back) packed at offs[r] (offs[nrows] = the total)
hipError_t merge_pack(const uint32_t* src, const uint32_t* roff, const uint64_t* offs, uint32_t nrows, uint32_t* enc,
                      hipStream_t st);
// row[q] = offs[(q + 1) per] - offs[q per] for q < W (a rank's row of the slice-size matrix)
hipError_t merge_sizes_row(const uint64_t* offs, uint32_t per, int W, uint64_t* row, hipStream_t st);
// offs[0..nrows) = exclusive prefix of words (a received slice); tmp from merge_count's query
hipError_t merge_offsets(const uint32_t* words, uint32_t nrows, uint64_t* offs, void* tmp, size_t tmp_bytes,
                         hipStream_t st);
// The loopback transport's copies (device to device, same device), one launch.
constexpr int LOOP_COPIES_MAX = 128;
struct LoopCopies {
  const uint32_t* src[LOOP_COPIES_MAX];
  uint32_t* dst[LOOP_COPIES_MAX];
  uint64_t words[LOOP_COPIES_MAX];
  int n;
};
hipError_t merge_loop_copy(const LoopCopies& l, hipStream_t st);
// dst[i] = sum over k < n of srcs[k][i] (the loopback transport's reductions; dst may be srcs[0])
hipError_t merge_loop_sum_i32(const int32_t* const* srcs, int n, int32_t* dst, size_t count, hipStream_t st);
hipError_t merge_loop_sum_i64(const int64_t* const* srcs, int n, int64_t* dst, size_t count, hipStream_t st);
// summed rows of the slice (nrows <= src.per; out_rows nullable: [nrows][1798]) and their summaries
hipError_t merge_decode(const MergeRecv& src, uint32_t nrows, const int64_t* totals, Tables tb, int32_t* out_rows,
                        Summary88* out_summ, hipStream_t st);

}  // namespace l5dh
