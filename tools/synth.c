/*
 * synth.c -- canonical synthetic libsvm / CSV generator (bench + test input).
 *
 * Deterministic per row: row r draws from splitmix64 seeded with
 * mix(seed, r), so any row range can be produced independently (sharded
 * generation for multi-GPU runs, parallel generation with OpenMP).
 *
 *  libsvm row: "<label>( <id>:<value>)*\n", label = 1 random bit, exactly K
 *    features, ids strictly increasing (first = gap-1, then += gap, gap
 *    uniform in [1,16]), value = fp32 uniform [0,1) from a 24-bit mantissa,
 *    printed "%.9g" (round-trips exactly).
 *  CSV row: C values uniform [-1,1) (24-bit mantissa), "%.9g", ',' separated.
 *  libfm row: "<label>( <field>:<id>:<value>)*\n", the libsvm row's ids and
 *    values with a field in [0,32) per feature (libfm_parser.h:67-144).
 *  libsvm+qid row (fmt 3): "<label> qid:<q>( <id>:<value>)*\n", the libsvm
 *    row with q = row / 16 (ranking data, libsvm_parser.h:119-132).
 *  libsvm+comment row (fmt 4): the libsvm row with a trailing comment
 *    " # row <r>" (libsvm_parser.h:67-83), and a '#' header line first.
 *  CSV+blank row (fmt 5): the CSV row with ", " between values (ParseFloat
 *    skips the blank before each value, strtonum.h:95-264).
 *  libsvm 1-based row (fmt 6): the libsvm row with every id one higher (no 0
 *    id: indexing_mode=-1 shifts them back, libsvm_parser.h:165-171).
 *  libsvm directory (fmt 8): the libsvm rows as files of 16384 rows, each
 *    starting with the header line "# synth libsvm shard", read the way the
 *    text InputSplit reads a directory -- a '\n' between files
 *    (input_split_base.cc:204-210), so every header after the first sits
 *    mid-chunk after an empty line, where the reference parses it as a line
 *    (libsvm_parser.h:91-104; no digitchar in it: an empty line).
 *  libsvm with dirty rows (fmt 9): the libsvm row, and on every eighth row
 *    (r % 8 == 3) mid-row either a missing-value word " NA" / " n/a" or an
 *    infinite value "<id>:-inf" -- bytes outside the uniform grammar that
 *    ParsePair skips (strtonum.h:667-703) and ParseFloat's inf
 *    (strtonum.h:133-175).
 *  CSV with NaN(chars) fields (fmt 10): the CSV row, and on every 64th row
 *    (r % 64 == 17) the middle field "NaN(x)" -- ParseFloat's NAN(chars)
 *    form (strtonum.h:157-165), a quiet NaN.
 *  CSV with missing values (fmt 7): the CSV row with 0.1 % of its fields
 *    "nan" (numpy.savetxt's missing value; ParseFloat's NAN branch,
 *    strtonum.h:133-175), and a UTF-8 BOM at the head of the file
 *    (IgnoreUTF8BOM, csv_parser.h:83).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static inline uint64_t sm64(uint64_t *x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ULL);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
  return z ^ (z >> 31);
}
static inline uint64_t row_state(uint64_t seed, uint64_t r) {
  uint64_t s = seed * 0xD1B54A32D192ED03ULL ^ (r + 1) * 0x9E3779B97F4A7C15ULL;
  sm64(&s);
  return s;
}

static size_t fmt_libsvm_row(char *o, uint64_t seed, uint64_t r, int K, int qid, int cmt, int one_based, int dirty) {
  uint64_t s = row_state(seed, r);
  char *p = o;
  *p++ = (char)('0' + (sm64(&s) & 1));
  if (qid) p += sprintf(p, " qid:%llu", (unsigned long long)(r >> 4));
  uint64_t id = 0;
  for (int j = 0; j < K; ++j) {
    uint64_t x = sm64(&s);
    uint64_t gap = 1 + (x & 15);
    id = j == 0 ? gap - 1 + (uint64_t)one_based : id + gap;
    float v = (float)(x >> 40) * (1.0f / 16777216.0f);
    /* fmt 9: every eighth row carries a word or an infinite value mid-row */
    if (dirty && (r & 7) == 3 && j == K / 2) {
      const int kind = (int)((r >> 3) % 3);
      if (kind == 1) {
        p += sprintf(p, " %llu:-inf", (unsigned long long)id);
        continue;
      }
      p += sprintf(p, kind == 0 ? " NA" : " n/a");
    }
    p += sprintf(p, " %llu:%.9g", (unsigned long long)id, (double)v);
  }
  if (cmt) p += sprintf(p, " # row %llu", (unsigned long long)r);
  *p++ = '\n';
  return (size_t)(p - o);
}

static size_t fmt_libfm_row(char *o, uint64_t seed, uint64_t r, int K) {
  uint64_t s = row_state(seed, r);
  char *p = o;
  *p++ = (char)('0' + (sm64(&s) & 1));
  uint64_t id = 0;
  for (int j = 0; j < K; ++j) {
    uint64_t x = sm64(&s);
    uint64_t gap = 1 + (x & 15);
    id = j == 0 ? gap - 1 : id + gap;
    float v = (float)(x >> 40) * (1.0f / 16777216.0f);
    p += sprintf(p, " %u:%llu:%.9g", (unsigned)((x >> 4) & 31), (unsigned long long)id, (double)v);
  }
  *p++ = '\n';
  return (size_t)(p - o);
}

static size_t fmt_csv_row(char *o, uint64_t seed, uint64_t r, int C, int blank, int nan, int nanp) {
  uint64_t s = row_state(seed, r);
  char *p = o;
  for (int j = 0; j < C; ++j) {
    uint64_t x = sm64(&s);
    float v = (float)(x >> 40) * (1.0f / 8388608.0f) - 1.0f;
    if (nan && ((x >> 8) & 0xFFFF) % 1000 == 0) p += sprintf(p, j ? ",nan" : "nan");
    else if (nanp && (r & 63) == 17 && j == C / 2) p += sprintf(p, j ? ",NaN(x)" : "NaN(x)");
    else p += sprintf(p, j ? (blank ? ", %.9g" : ",%.9g") : "%.9g", (double)v);
  }
  *p++ = '\n';
  return (size_t)(p - o);
}

/* upper bound on the bytes of `nrows` rows */
size_t synth_bound(int fmt, uint64_t nrows, int width) {
  return fmt == 0 || fmt == 3 || fmt == 4 || fmt == 6 || fmt == 8 || fmt == 9 ? nrows * (size_t)(2 + 28 + width * 26) + 32
                  : fmt == 2 ? nrows * (size_t)(2 + width * 30) : nrows * (size_t)(width * 19 + 2) + 3;
}

/* Format rows [row0, row0+nrows) into out (capacity cap); returns bytes, or 0
 * if cap is too small.  If line_off != NULL it receives nrows+1 line offsets. */
size_t synth_rows(int fmt, uint64_t row0, uint64_t nrows, int width, uint64_t seed, char *out,
                  size_t cap, uint64_t *line_off) {
  const int nblk = 256;
  uint64_t per = (nrows + nblk - 1) / nblk;
  size_t *bsz = (size_t *)calloc(nblk, sizeof(size_t));
  char **bbuf = (char **)calloc(nblk, sizeof(char *));
  int overflow = 0;
#pragma omp parallel for schedule(dynamic, 1)
  for (int b = 0; b < nblk; ++b) {
    uint64_t r0 = (uint64_t)b * per, r1 = r0 + per < nrows ? r0 + per : nrows;
    if (r0 >= r1) continue;
    size_t cap_b = synth_bound(fmt, r1 - r0, width);
    char *buf = (char *)malloc(cap_b + 64);
    size_t n = 0;
    for (uint64_t r = r0; r < r1; ++r) {
      if (line_off) line_off[r] = n; /* block-relative; fixed below */
      if (fmt == 4 && row0 + r == 0) n += (size_t)sprintf(buf + n, "# label id:value ... # row r\n");
      if (fmt == 7 && row0 + r == 0) n += (size_t)sprintf(buf + n, "\xEF\xBB\xBF");
      if (fmt == 8 && (row0 + r) % 16384 == 0)
        n += (size_t)sprintf(buf + n, row0 + r ? "\n# synth libsvm shard\n" : "# synth libsvm shard\n");
      n += fmt == 0 || fmt == 3 || fmt == 4 || fmt == 6 || fmt == 8 || fmt == 9
               ? fmt_libsvm_row(buf + n, seed, row0 + r, width, fmt == 3, fmt == 4, fmt == 6, fmt == 9)
                    : fmt == 2 ? fmt_libfm_row(buf + n, seed, row0 + r, width)
                               : fmt_csv_row(buf + n, seed, row0 + r, width, fmt == 5, fmt == 7, fmt == 10);
    }
    bbuf[b] = buf;
    bsz[b] = n;
  }
  size_t total = 0;
  for (int b = 0; b < nblk; ++b) total += bsz[b];
  if (total > cap) overflow = 1;
  if (!overflow) {
    size_t *base = (size_t *)calloc(nblk, sizeof(size_t));
    for (int b = 1; b < nblk; ++b) base[b] = base[b - 1] + bsz[b - 1];
#pragma omp parallel for schedule(dynamic, 1)
    for (int b = 0; b < nblk; ++b) {
      if (!bsz[b]) continue;
      memcpy(out + base[b], bbuf[b], bsz[b]);
      if (line_off) {
        uint64_t r0 = (uint64_t)b * per, r1 = r0 + per < nrows ? r0 + per : nrows;
        for (uint64_t r = r0; r < r1; ++r) line_off[r] += base[b];
      }
    }
    if (line_off) line_off[nrows] = total;
    free(base);
  }
  for (int b = 0; b < nblk; ++b) free(bbuf[b]);
  free(bbuf);
  free(bsz);
  return overflow ? 0 : total;
}
