/*
 * dmlc_amd.h -- C ABI of the MI355X text -> CSR parse path.
 *
 * This is the drop-in boundary below dmlc-core's parser plugin API.  The host
 * side (dmlc::Parser<I,D>::Create, src/data.cc:152-186, and the text parsers
 * registered at src/data.cc:202-221) hands InputSplit chunks to these entry
 * points; each replaces the CPU ParseBlock of one parser:
 *
 *   format DMLC_AMD_LIBSVM -> LibSVMParser<I>::ParseBlock  (src/data/libsvm_parser.h:85-172)
 *   format DMLC_AMD_CSV    -> CSVParser<I,D>::ParseBlock   (src/data/csv_parser.h:71-149)
 *   format DMLC_AMD_LIBFM  -> LibFMParser<I>::ParseBlock   (src/data/libfm_parser.h:67-144)
 *
 * Semantics: the text buffer holds `nchunks` consecutive InputSplit chunks
 * (chunk c = [chunk_starts[c], chunk_starts[c+1]), chunk_starts[nchunks] ==
 * nbytes).  Each chunk goes through TextParserBase::FillData
 * (text_parser.h:116-155): it is cut into T = max(params.nthread, 1) ranges
 * (BackFindEndLine, text_parser.h:70-77) and each range is parsed as ONE
 * ParseBlock -- a "unit"; unit u = c * T + t.  The per-unit
 * RowBlockContainers are returned concatenated, exactly as
 * RowBlockContainer::Push(RowBlock) (src/data/row_block.h:126-168) would
 * concatenate them: offsets are global.  Per-unit boundaries are reported in
 * chunk_table so the caller can rebuild the per-unit RowBlock views (the
 * reference's blocks, parser.h:32-48) and run GetBlock's consistency CHECKs
 * (row_block.h:171-189) per unit.  T changes the result only through
 * indexing_mode < 0, whose 1-based detection is per unit
 * (libsvm_parser.h:165-171, libfm_parser.h likewise).
 *
 * All pointers named d_* and every pointer inside dmlc_amd_csr are DEVICE
 * pointers.  Calls are asynchronous on `stream` (a hipStream_t, NULL = default
 * stream); results land in *d_result.  No host synchronisation, allocation or
 * device-wide barrier happens inside a call, so calls can be captured into a
 * hipGraph.  Only plain pointers and sizes cross this boundary.
 */
#ifndef DMLC_AMD_H_
#define DMLC_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DMLC_AMD_ABI_VERSION 2

enum { DMLC_AMD_LIBSVM = 0, DMLC_AMD_CSV = 1, DMLC_AMD_LIBFM = 2 };
enum { DMLC_AMD_F32 = 0, DMLC_AMD_I32 = 1, DMLC_AMD_I64 = 2 };

/* counter slots of dmlc_amd_result.count / chunk_table rows / csr.cap */
enum {
  DMLC_AMD_ROWS = 0,   /* rows (RowBlock::size); offset has rows + 1 entries */
  DMLC_AMD_INDEX = 1,  /* feature indices (RowBlock::index) */
  DMLC_AMD_VALUE = 2,  /* values (RowBlock::value); 0 when the input has none */
  DMLC_AMD_WEIGHT = 3, /* instance weights (RowBlock::weight) */
  DMLC_AMD_QID = 4,    /* query ids (RowBlock::qid) */
  DMLC_AMD_LABEL = 5,  /* csv only: labels (rows carry labels only with label_column) */
  DMLC_AMD_FIELD = 6,  /* libfm only: field ids (RowBlock::field) */
  DMLC_AMD_NSLOT = 7
};

/* error codes in dmlc_amd_result.error & 0xFFFF (the first error by position) */
enum {
  DMLC_AMD_OK = 0,
  DMLC_AMD_ERR_NEG_INDEX = 1,   /* strtonum.h:416  CHECK_EQ(sign, true) */
  DMLC_AMD_ERR_NAN_LITERAL = 2, /* strtonum.h:163  "Invalid NAN literal" */
  DMLC_AMD_ERR_CSV_DELIM = 3,   /* csv_parser.h:128-132 delimiter not found */
  DMLC_AMD_ERR_CAPACITY = 16,   /* an output array was too small; counts are exact */
  DMLC_AMD_ERR_ARG = 32,        /* invalid argument (returned by the call itself) */
  DMLC_AMD_ERR_HIP = 33         /* HIP runtime error (returned by the call itself) */
};

typedef struct dmlc_amd_params {
  int32_t format;        /* DMLC_AMD_LIBSVM | CSV | LIBFM */
  int32_t index_bits;    /* 32 or 64: IndexType of dmlc::Parser<IndexType, DType> */
  int32_t value_type;    /* DMLC_AMD_F32 | I32 | I64: DType (csv only may be integral) */
  int32_t indexing_mode; /* libsvm/libfm: LibSVMParserParam::indexing_mode (libsvm_parser.h:32) */
  int32_t label_column;  /* csv: CSVParserParam::label_column, -1 = none (csv_parser.h:34) */
  int32_t weight_column; /* csv: CSVParserParam::weight_column, -1 = none (csv_parser.h:38) */
  int32_t delimiter;     /* csv: CSVParserParam::delimiter[0] (csv_parser.h:37) */
  uint32_t tile_bytes;   /* 0 = default tile size */
  uint32_t flags;        /* DMLC_AMD_FLAG_* */
  int32_t nthread;       /* FillData ranges per chunk (TextParserBase::nthread_, text_parser.h:32-35);
                            0 or 1 = one ParseBlock per chunk */
  uint32_t reserved[2];
} dmlc_amd_params;

#define DMLC_AMD_FLAG_COUNT_ONLY 1u /* run the counting passes only (size query) */
/* Run the write pass only, reusing the per-tile counts that a COUNT_ONLY call
 * on the same text, chunk starts, params and workspace left behind (earlier on
 * the same stream).  COUNT_ONLY then FILL_ONLY does exactly the work of one
 * full call, with a host-side allocation in between. */
#define DMLC_AMD_FLAG_FILL_ONLY 2u
/* Skip the single-pass uniform-grammar kernel and run the exact tile kernels
 * only (results are identical either way; this exists for testing/profiling). */
#define DMLC_AMD_FLAG_EXACT 4u
/* After the write pass, reduce the written index (and libfm field) arrays to
 * their maxima in dmlc_amd_result.max_index / max_field (the NumCol of the
 * reference's BasicRowIter, basic_row_iter.h:46-48). */
#define DMLC_AMD_FLAG_MAX_INDEX 8u

typedef struct dmlc_amd_csr {
  uint64_t *offset; /* rows + 1 (global, rebased across chunks) */
  void *label;      /* rows x DType (float for libsvm/libfm) */
  float *weight;
  uint64_t *qid;
  void *field;      /* IndexType */
  void *index;      /* IndexType */
  void *value;      /* DType */
  uint64_t cap[8];  /* capacity in elements per slot (cap[ROWS] counts labels; offset needs +1) */
} dmlc_amd_csr;

typedef struct dmlc_amd_result {
  uint64_t count[8];  /* exact totals per slot, even when a capacity was exceeded */
  uint64_t error;     /* 0, or (byte position << 16) | error code of the first error */
  uint64_t path;      /* 0 = single-pass uniform-grammar kernel, else exact tile kernels
                         (bit 1: the single-pass kernel handed over mid-launch) */
  uint64_t max_index; /* with DMLC_AMD_FLAG_MAX_INDEX: largest index written (0 if none) --
                         RowBlockContainer::max_index, row_block.h:126-168 */
  uint64_t max_field; /* likewise for libfm field ids (max_field) */
  uint64_t reserved[4];
} dmlc_amd_result;

/* Bytes of device workspace dmlc_amd_parse needs for this input. */
size_t dmlc_amd_workspace_bytes(uint64_t nbytes, int nchunks, const dmlc_amd_params *prm);

/* Parse.  d_chunk_table (optional, may be NULL) receives (nchunks * T) x 8
 * uint64, T = max(nthread, 1): the exclusive counts (slots above) at each
 * unit start.  Returns DMLC_AMD_OK
 * or DMLC_AMD_ERR_ARG / DMLC_AMD_ERR_HIP; parse errors are reported through
 * d_result->error once the stream reaches the end of the pipeline. */
int dmlc_amd_parse(const void *d_text, uint64_t nbytes, const uint64_t *d_chunk_starts, int nchunks,
                   const dmlc_amd_params *prm, const dmlc_amd_csr *out, uint64_t *d_chunk_table,
                   void *d_workspace, size_t workspace_bytes, dmlc_amd_result *d_result,
                   void *stream);

/* Batch dmlc::strtof (ParseFloat<float>, strtonum.h:95-264, :279-281): string i
 * is d_text[d_offsets[i] .. d_offsets[i+1]) read as NUL-terminated at its end.
 * Writes the value, the bytes consumed (endptr - nptr) and the "Invalid NAN
 * literal" flag (strtonum.h:163); d_consumed / d_nan_error may be NULL. */
int dmlc_amd_strtof_batch(const void *d_text, const uint64_t *d_offsets, uint64_t n, float *d_out,
                          uint32_t *d_consumed, uint32_t *d_nan_error, void *stream);

/* Stream copy of `bytes` between page-locked host memory (hipHostMalloc) and
 * device memory, or device to device, by a kernel instead of the DMA engine
 * (the host side of a parse pipeline: text batches in, CSR arrays out).  Both
 * pointers must be device-accessible; unaligned pointers fall back to
 * hipMemcpyAsync.  Asynchronous on `stream`. */
int dmlc_amd_copy(void *dst, const void *src, uint64_t bytes, void *stream);

/* n <= DMLC_AMD_COPY_MAX such copies (dst[i] <- src[i], bytes[i]) in one
 * kernel launch: the CSR arrays of a parsed batch in one D2H step.  Zero-byte
 * entries are skipped; a pair not 16-byte aligned is copied on its own. */
#define DMLC_AMD_COPY_MAX 16
int dmlc_amd_copy_n(void *const *dst, const void *const *src, const uint64_t *bytes, int n, void *stream);

/* The same with sizes known only on the device (a parse's result counts, so
 * the copy-out needs no host round trip after the parse): copy i moves
 * min(max_bytes[i], d_counts[slot[i]] * scale[i] + add[i]) bytes, or add[i]
 * when slot[i] < 0.  d_counts is read on the device when the copy runs: it
 * holds DMLC_AMD_COPY_SLOTS words (dmlc_amd_result.count), so slot[i] >=
 * DMLC_AMD_COPY_SLOTS is rejected (DMLC_AMD_ERR_ARG); slot / scale / add /
 * max_bytes are host arrays of n entries.  All pairs must be 16-byte
 * aligned. */
#define DMLC_AMD_COPY_SLOTS 8
int dmlc_amd_copy_n_dev(void *const *dst, const void *const *src, const uint64_t *d_counts, const int *slot,
                        const uint64_t *scale, const uint64_t *add, const uint64_t *max_bytes, int n,
                        void *stream);

/* Kernel timing for benchmarks: between profile_begin and profile_end, every
 * dmlc_amd_parse on this thread brackets its dominant kernel (the single-pass
 * kernel, or the exact write kernel) with HIP events on its stream.
 * profile_end synchronises, returns the summed kernel time, the number of
 * bracketed launches and the kernel's name. */
int dmlc_amd_profile_begin(void);
int dmlc_amd_profile_end(double *total_ms, int *launches, const char **kernel);

/* Human-readable message for an error code (matches the reference's CHECK text). */
const char *dmlc_amd_error_string(int code);

/* hipGetErrorString of the HIP error behind this thread's last DMLC_AMD_ERR_HIP. */
const char *dmlc_amd_last_hip_error(void);

/* Number of visible HIP devices (0 when no GPU / no driver). */
int dmlc_amd_device_count(void);

/* ABI version this library was built with. */
int dmlc_amd_abi_version(void);

/* Build id: SHA-256 (first 16 hex digits) of the kernel and C-ABI sources
 * this library was compiled from (dmlc-core_amd/Makefile).  bench.py stamps
 * its line with it and with the build id of the PMC run its HBM traffic
 * figure came from (profiles/traffic.json).  Not a reference interface. */
const char *dmlc_amd_build_id(void);

/* Geometry of the single-pass kernels this library was built with: text
 * bytes per tile and the most ParseBlock unit starts one tile takes before
 * the call goes to the exact kernels (diagnostics and tests; either pointer
 * may be NULL). */
int dmlc_amd_fast_geometry(uint32_t *tile_bytes, uint32_t *max_unit_starts);

#ifdef __cplusplus
}
#endif
#endif /* DMLC_AMD_H_ */
