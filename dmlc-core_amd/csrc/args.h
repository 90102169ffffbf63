// args.h -- argument blocks of the tile kernels (plain C++, shared by the
// HIP launchers and the test-only CPU emulator).
#pragma once
#include <stdint.h>

#include "hd.h"

namespace dmlc_amd {

// ParseBlock units and InputSplit chunks.  `cs` lists the ParseBlock units
// (text_parser.h:116-155 FillData: each chunk cut into nthread ranges); the
// number decoders read on to the end of the InputSplit CHUNK holding a unit,
// as the reference's strtof / atoll / ParseTriple do over the chunk buffer
// (lcs = chunk starts, ldiv = units per chunk).
struct UnitLim {
  const uint64_t *lcs;
  int ldiv;
  DA_HD uint64_t lim(int unit) const { return lcs[(ldiv == 1 ? unit : unit / ldiv) + 1]; }
};

struct LibsvmArgs {
  const uint8_t *text;
  uint64_t n;
  const uint64_t *cs;  // ParseBlock unit starts, nchunk + 1 entries, cs[nchunk] == n
  int nchunk;          // units
  uint64_t tile_bytes;
  uint32_t ntiles;
  int wide;            // IndexType is uint64_t
  int indexing_mode;
  uint64_t *tile_cnt;         // [ntiles][C_N], count pass output
  const uint64_t *tile_base;  // [ntiles][C_N], exclusive scan of tile_cnt
  uint64_t *offset;
  float *label;
  float *weight;
  uint64_t *qid;
  void *index;
  float *value;
  uint64_t cap[8];
  uint64_t *chunk_tab;  // [nchunk][C_N] exclusive counts at each chunk start (may be a sink)
  uint64_t *chunk_min;  // [nchunk] min index per chunk (indexing_mode < 0)
  unsigned long long *err;
  const uint32_t *gate;  // when set, the tile kernels run only if *gate != 0
  UnitLim ul;            // decoder limit per unit
  DA_HD uint64_t lim(int unit) const { return ul.lim(unit); }
  // libsvm / libfm: what the count pass learnt per window for the write pass
  // (NULL: the write pass works it out again): rec [ntiles][rec_win][4][kThreads]
  // words -- index / value / dangling-value role masks and packed head
  // counts per thread (libfm: pair / value / dangling masks, head counts and
  // the sign-error position) -- and rec_meta [ntiles][rec_win][2]: the R1
  // carried past the window and the role state after it (libfm: bit 8 set =
  // the window has no record)
  uint32_t *rec;
  uint64_t *rec_meta;
  uint32_t rec_win;  // windows per tile with a record (the rest: worked out again)
  // count pass after the single-pass kernel (libsvm.hip libsvm_tile): its qid
  // shards and result block, to hand a qid / no-qid mix over (NULL: no check)
  const uint64_t *qsum;
  const uint64_t *qres;
};
// windows per exact tile with a count-pass record, and the record bytes
// (libsvm_core.h); the records are kept only while they stay within 5/8 of
// the text's size + 1 MiB (at the default 256 KiB exact tiles they are 0.55
// of it; smaller tiles need more per byte and lose them on large inputs)
DA_HD uint32_t exact_rec_win(uint64_t tile_bytes, uint64_t win_bytes) {
  return (uint32_t)(tile_bytes / win_bytes + 3);
}
DA_HD uint64_t exact_rec_bytes(uint64_t ntiles, uint32_t rec_win, int threads) {
  return ntiles * rec_win * ((uint64_t)threads * 16 + 16);
}
DA_HD bool exact_rec_on(uint64_t nbytes, uint64_t rec_bytes) { return rec_bytes <= nbytes / 8 * 5 + (1ull << 20); }

// libfm exact tile kernels (libfm_core.h): the libsvm block plus field ids.
struct LibfmArgs : LibsvmArgs {
  void *field;  // IndexType, one per index
};

// Single-pass uniform-grammar libsvm kernel (svm_fast.h).
struct FastSvmArgs {
  const uint8_t *text;
  uint64_t n;
  const uint64_t *cs;
  int nchunk;
  uint32_t ntiles;
  int wide;
  int indexing_mode;
  int skip_if_gated;  // fill phase: do nothing when the count phase fell back
  uint64_t *offset;
  float *label;
  float *weight;
  uint64_t *qid;        // libsvm "qid:" ids, one per row (svm_fast.h qid_decide)
  void *index;
  void *field;          // libfm: one field id per index (IndexType); null for libsvm
  float *value;
  uint64_t cap[8];
  uint64_t *chunk_tab;  // may be null
  uint64_t *lb;         // look-back records [5 ntiles] (status words zeroed per launch)
  uint64_t *qsum;       // libsvm: qid runs, sharded by tile [kLabShards][8] (zeroed per launch);
                        // word 1 of shard 0: some tile held a qid run
  uint64_t *umin;       // indexing_mode < 0: minimum stored index (libfm: and field) per ParseBlock
                        // unit [nchunk], ~0 = none; filled by the write pass (svm_fast.h umin_fix)
  uint32_t *gate;       // != 0: input left the grammar -> exact path
  unsigned long long *err;  // first error of this path
  uint64_t *res;        // dmlc_amd_result counts (written by the last tile)
  uint32_t *ticket;     // persistent launch: tiles handed out past the first gridDim.x (zeroed per launch)
  // the lean kernel (svm_lean.h) ahead of this one: its look-back words [5 ntiles]
  // and ~(its first poisoned tile) (0: none), zeroed per launch.  The full
  // kernel resumes at that tile, its look-back seeded by the lean inclusive
  // prefix before it (null: no lean launch, the full kernel takes every tile).
  uint64_t *lean_lb;
  uint64_t *lean_poison;
};

// look-back words per single-pass tile (fast_common.h: status + 4 prefix words);
// the persistent launch's ticket word follows them
constexpr uint64_t kFastLbWords = 5;
// the CSV single pass (csv_fast.h csv_look_back): status + 3 prefix words in
// one 64-byte record per tile
constexpr uint64_t kCsvLbWords = 8;

// Threads of a single-pass tile (fast_common.h): four waves, 16 KiB tiles.
// One wave per tile (4 KiB tiles, no barriers between waves, -DFAST_THREADS=64)
// and two (128) stay buildable for A/B timing; on MI355X they measured
// 3.90 / 2.25 ms against 1.78 ms on config 2 (profiles/r4_ab/ab_r4f.txt, PMC in gpurun_out/ab: per wave
// VALU 2725 / 1961 / 1709 -- the tile-level work of the look-back, the unit
// search and the run-list rounds does not shrink with the tile).
#ifndef FAST_THREADS
#define FAST_THREADS 256
#endif
constexpr int kFastThreads = FAST_THREADS;
constexpr uint64_t kFastTileBytes = (uint64_t)kFastThreads * 64;  // 64 text bytes per thread
constexpr int kFastMaxCs = kFastThreads == 64 ? 16 : 32;           // unit starts per tile (fast_common.h kMaxCs)

// Single-pass uniform-grammar CSV kernel (csv_fast.h).
constexpr int kLabShards = 64;  // FastCsvArgs::labsum shards, one 64-byte line each
struct FastCsvArgs {
  const uint8_t *text;
  uint64_t n;
  const uint64_t *cs;
  int nchunk;
  uint32_t ntiles;
  int wide;
  uint32_t delim;
  int skip_if_gated;
  int label_col;        // CSVParserParam::label_column, -1 = none
  int weight_col;       // CSVParserParam::weight_column, -1 = none (csv_fast_columns_ok)
  uint64_t *offset;
  float *label;         // one per row when label_col >= 0
  float *weight;        // one per row when weight_col >= 0
  uint64_t *labsum;     // [kLabShards][8], zeroed per launch: words 0/1/2 = sum(labels - rows),
                        // sum(first delimiters - rows), sum(weights - rows), sharded by tile (csv_fast.h)
  void *index;
  void *value;          // DType: float, or int32 / int64 (vtype)
  int vtype;            // 0 f32, 1 i32, 2 i64 (integer values: csv_fast_tile_int)
  uint64_t cap[8];
  uint64_t *chunk_tab;  // may be null
  uint64_t *lb;
  uint32_t *gate;
  unsigned long long *err;
  uint64_t *res;
};

// Label / weight columns the single-pass CSV kernel takes: every row holds a
// non-empty field at each (checked on the device), and then a row always keeps
// a non-special field -- unless the special columns are {0} or {0, 1}, where a
// row of only those fields is the reference's fatal "Delimiter not found"
// (csv_parser.h:128-132): label column 0 alone is checked on the device, the
// weight forms go to the exact kernels.
DA_HD bool csv_fast_columns_ok(int label_col, int weight_col) {
  if (weight_col < 0) return true;
  if (weight_col == label_col || weight_col == 0) return false;
  return label_col < 0 || (label_col > weight_col ? label_col : weight_col) >= 2;
}

// The single-pass integer-DType kernel: no label column; the weight column
// is an ordinary column for integer DTypes (csv_parser.h:111-114).
DA_HD bool csv_fast_int_ok(int label_col) { return label_col < 0; }

struct CsvArgs {
  const uint8_t *text;
  uint64_t n;
  const uint64_t *cs;
  int nchunk;
  uint64_t tile_bytes;
  uint32_t ntiles;
  int wide;
  int vtype;  // 0 f32, 1 i32, 2 i64
  int label_column, weight_column;
  uint32_t delim;
  int fast_delim;  // delimiter cannot be consumed by the field decoder
  uint64_t *tile_cnt;
  const uint64_t *tile_base;
  uint64_t *offset;
  void *label;  // DType
  float *weight;
  void *index;
  void *value;  // DType
  uint64_t cap[8];
  uint64_t *chunk_tab;
  unsigned long long *err;
  const uint32_t *gate;  // when set, the tile kernels run only if *gate != 0
  UnitLim ul;            // decoder limit per unit
  DA_HD uint64_t lim(int unit) const { return ul.lim(unit); }
  // the count pass's per-thread window counts for the write pass (NULL: it
  // counts again): [ntiles][rec_win][4][kThreads] words -- rows, values
  // (= indices), labels, weights
  uint32_t *rec;
  uint32_t rec_win;
};

}  // namespace dmlc_amd
