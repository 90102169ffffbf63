/*
 * dmlc_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of dmlc-core's text -> RowBlock parse path, used as the
 * parity checker for the HIP path.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path never
 * links it.
 *
 * Pinned against golden vectors produced by the genuine reference (built from
 * /root/reference sources by oracle/Makefile.ref into oracle/_ref/) and against
 * the known answers of test/unittest_parser.cc; see tests/golden/ and
 * tests/test_oracle.py.
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef DMLC_ORACLE_H_
#define DMLC_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum { DMO_FMT_LIBSVM = 0, DMO_FMT_CSV = 1, DMO_FMT_LIBFM = 2 };
enum { DMO_VAL_F32 = 0, DMO_VAL_I32 = 1, DMO_VAL_I64 = 2 };

typedef struct {
  int32_t format;         /* DMO_FMT_* */
  int32_t index_bits;     /* 32 or 64: IndexType of Parser<IndexType, DType> */
  int32_t value_kind;     /* DMO_VAL_*: DType (label and value share it) */
  int32_t indexing_mode;  /* libsvm/libfm: libsvm_parser.h:32-39 */
  int32_t label_column;   /* csv: csv_parser.h:34-36 */
  int32_t weight_column;  /* csv: csv_parser.h:38-40 */
  int32_t delimiter;      /* csv: first char of `delimiter` param, csv_parser.h:37 */
  int32_t nthread;        /* ParseBlock ranges per chunk (text_parser.h:130-147) */
} dmo_params;

/* Concatenation of every block's arrays, exactly what BasicRowIter::Init sees
 * through RowBlockContainer::Push(RowBlock) (row_block.h:126-168). */
typedef struct {
  uint64_t n_rows, n_index, n_value, n_weight, n_qid, n_field, n_label;
  uint64_t *offset;  /* n_rows + 1, rebased across blocks */
  void *label;       /* n_label elements of DType (csv without label_column: 0) */
  float *weight;     /* n_weight */
  uint64_t *qid;     /* n_qid */
  uint64_t *field;   /* n_field (libfm) */
  uint64_t *index;   /* n_index, already wrapped to IndexType */
  void *value;       /* n_value elements of DType */
  /* per-block sizes, in block order (only non-empty blocks, like Next()) */
  uint64_t n_blocks;
  uint64_t *block_rows, *block_index, *block_value, *block_weight, *block_qid;
  int32_t status;    /* 0 ok, else an error in the reference's sense */
  char msg[256];
} dmo_csr;

/* strtonum.h:95-264 ParseFloat<float,false>; bytes at or past `lim` read as NUL */
float dmo_parse_float(const char *p, const char *lim, const char **endptr);
/* strtonum.h:392-428 ParseUnsignedInt<T>(p, NULL, 10); *err=1 on leading '-' */
uint64_t dmo_parse_uint(const char *p, const char *lim, int bits, int *err);
/* glibc atoll (used at libsvm_parser.h:127) */
int64_t dmo_atoll(const char *p, const char *lim);
/* glibc strtoll(p, &e, 0) (used at csv_parser.h:102,105) */
int64_t dmo_strtoll0(const char *p, const char *lim, const char **endptr);

/* Parse one InputSplit chunk the way TextParserBase::FillData does
 * (text_parser.h:116-155): split into nthread ranges snapped back to a line
 * end, ParseBlock each range, then append every non-empty block to `out`. */
int dmo_parse_chunk(const char *chunk, size_t size, const dmo_params *prm, dmo_csr *out);
/* Same, one ParseBlock over [begin, begin+size) (the unittest_parser.cc seam). */
int dmo_parse_block(const char *begin, size_t size, const dmo_params *prm, dmo_csr *out);

void dmo_csr_init(dmo_csr *out, int value_kind);
void dmo_csr_free(dmo_csr *out);

/* Text InputSplit restatement (input_split_base.cc:29-291, line_split.cc:11-45):
 * given in-memory files, produce the chunk sequence of part `rank` of `nsplit`.
 * Returns the number of chunks; chunk i is out_buf[out_off[i] .. out_off[i+1]). */
typedef struct {
  uint64_t n_chunks;
  uint64_t *off;  /* n_chunks + 1 */
  char *buf;
} dmo_chunks;
int dmo_split_text(const char *const *files, const uint64_t *sizes, int nfiles,
                   unsigned rank, unsigned nsplit, uint64_t buffer_bytes, dmo_chunks *out);
void dmo_chunks_free(dmo_chunks *c);

/* Timing helper for bench.py's cpu_baseline leg: parse chunk i = buf[off[i] ..
 * off[i+1]) for every i on the calling thread (fresh output per chunk, as the
 * reference reuses one container per chunk); returns seconds, *nnz = total
 * index count. */
double dmo_bench_chunks(const char *buf, const uint64_t *off, int nchunks, const dmo_params *prm,
                        uint64_t *nnz);

#ifdef __cplusplus
}
#endif
#endif  /* DMLC_ORACLE_H_ */
