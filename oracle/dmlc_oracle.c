#define _POSIX_C_SOURCE 199309L
/*
 * dmlc_oracle.c -- TEST INFRASTRUCTURE ONLY (see dmlc_oracle.h).
 *
 * A plain-C restatement of dmlc-core's text parse path.  It is the parity
 * checker for the HIP kernels and is never linked into the product.
 *
 * Memory model: the reference dereferences bytes past the end of a ParseBlock
 * range (the decoders are unbounded).  Here every read goes through B(p, lim):
 * bytes at or beyond `lim` (the end of the chunk / test string) read as NUL,
 * which is exactly what the reference sees for the std::string inputs of
 * test/unittest_parser.cc.
 */
#include "dmlc_oracle.h"

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ---------------------------------------------------------------- bytes -- */

static inline unsigned B(const char *p, const char *lim) {
  return p < lim ? (unsigned char)*p : 0u;
}
/* strtonum.h:27-29 */
static inline int is_space(unsigned c) {
  return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f';
}
/* strtonum.h:37-39 */
static inline int is_blank(unsigned c) { return c == ' ' || c == '\t'; }
/* strtonum.h:47-49 */
static inline int is_digit(unsigned c) { return c >= '0' && c <= '9'; }
/* strtonum.h:57-61 */
static inline int is_alpha(unsigned c) {
  return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z');
}
/* strtonum.h:70-72 */
static inline int is_digitchar(unsigned c) {
  return is_digit(c) || c == '+' || c == '-' || c == '.' || c == 'e' || c == 'E';
}
static inline int is_nl(unsigned c) { return c == '\n' || c == '\r'; }
/* glibc isspace in the C locale (strtoll / atoll) */
static inline int is_cspace(unsigned c) { return c == ' ' || (c >= '\t' && c <= '\r'); }

/* -------------------------------------------------------------- decoders -- */

static int g_nan_error; /* set when ParseFloat hits "NAN(" without ')' */

/* strtonum.h:95-264, ParseFloat<float, CheckRange=false>. */
float dmo_parse_float(const char *nptr, const char *lim, const char **endptr) {
  const char *p = nptr;
  while (is_space(B(p, lim))) ++p;                                    /* :119-121 */
  int sign = 1;                                                       /* :124-130 */
  if (B(p, lim) == '-') {
    sign = 0;
    ++p;
  } else if (B(p, lim) == '+') {
    ++p;
  }
  {
    static const char kInf[] = "infinity", kNan[] = "nan";
    int i = 0;                                                        /* :134-148 */
    while (i < 8 && ((B(p, lim) | 32u) & 0xFFu) == (unsigned)kInf[i]) {
      ++i;
      ++p;
    }
    if (i == 3 || i == 8) {
      if (endptr) *endptr = p;
      return sign ? INFINITY : -INFINITY;
    }
    p -= i;
    i = 0;                                                            /* :151-174 */
    while (i < 3 && ((B(p, lim) | 32u) & 0xFFu) == (unsigned)kNan[i]) {
      ++i;
      ++p;
    }
    if (i == 3) {
      if (B(p, lim) == '(') {
        ++p;
        while (is_digit(B(p, lim)) || is_alpha(B(p, lim)) || B(p, lim) == '_') ++p;
        if (B(p, lim) != ')') g_nan_error = 1;                        /* :163 CHECK_EQ */
        ++p;
      }
      if (endptr) *endptr = p;
      uint32_t qnan = 0x7FC00000u;
      float f;
      memcpy(&f, &qnan, 4);
      return f;
    }
    p -= i;
  }
  uint64_t predec = 0;                                                /* :178-182 */
  for (; is_digit(B(p, lim)); ++p) predec = predec * 10ULL + (uint64_t)(B(p, lim) - '0');
  float value = (float)predec;
  if (B(p, lim) == '.') {                                             /* :185-199 */
    uint64_t pow10 = 1, val2 = 0;
    int digit_cnt = 0;
    ++p;
    while (is_digit(B(p, lim))) {
      if (digit_cnt < 19) {                                           /* kStrtofMaxDigits :78 */
        val2 = val2 * 10ULL + (uint64_t)(B(p, lim) - '0');
        pow10 *= 10ULL;
      }
      ++p;
      ++digit_cnt;
    }
    value += (float)((double)val2 / (double)pow10);
  }
  if (B(p, lim) == 'e' || B(p, lim) == 'E') {                         /* :202-254 */
    ++p;
    int frac = 0;
    float scale = 1.0f;
    unsigned expon;
    if (B(p, lim) == '-') {
      frac = 1;
      ++p;
    } else if (B(p, lim) == '+') {
      ++p;
    }
    for (expon = 0; is_digit(B(p, lim)); ++p) expon = expon * 10U + (unsigned)(B(p, lim) - '0');
    if (expon > 38U) expon = 38U;                                     /* clip, :218-228 */
    const float kMaxSig = (float)3.402823466, kMaxSigNeg = (float)1.175494351;
    if (expon == 38U && ((!frac && value > kMaxSig) || (frac && value < kMaxSigNeg)))
      value = frac ? kMaxSigNeg : kMaxSig;                            /* :230-242 */
    while (expon >= 8U) {
      scale *= 1E8f;
      expon -= 8U;
    }
    while (expon > 0U) {
      scale *= 10.0f;
      expon -= 1U;
    }
    value = frac ? (value / scale) : (value * scale);
  }
  if (B(p, lim) == 'f' || B(p, lim) == 'F') ++p;                       /* :256-258 */
  if (endptr) *endptr = p;
  return sign ? value : -value;
}

/* strtonum.h:392-428, ParseUnsignedInt<uint32_t|uint64_t>(p, NULL, 10). */
uint64_t dmo_parse_uint(const char *p, const char *lim, int bits, int *err) {
  while (is_space(B(p, lim))) ++p;
  if (B(p, lim) == '-') { /* :416 CHECK_EQ(sign, true) */
    if (err) *err = 1;
    return 0;
  } else if (B(p, lim) == '+') {
    ++p;
  }
  uint64_t v = 0;
  for (; is_digit(B(p, lim)); ++p) v = v * 10ULL + (uint64_t)(B(p, lim) - '0');
  if (bits == 32) v &= 0xFFFFFFFFULL;
  return v;
}

/* glibc strtoll core: base 10 or 0, saturating, C locale. */
static int64_t strtoll_impl(const char *nptr, const char *lim, int base, const char **endptr) {
  const char *p = nptr;
  while (is_cspace(B(p, lim))) ++p;
  int neg = 0;
  if (B(p, lim) == '-') {
    neg = 1;
    ++p;
  } else if (B(p, lim) == '+') {
    ++p;
  }
  if (base == 0) {
    if (B(p, lim) == '0') {
      unsigned x = B(p + 1, lim);
      unsigned h = B(p + 2, lim);
      int hexd = is_digit(h) || (h >= 'a' && h <= 'f') || (h >= 'A' && h <= 'F');
      if ((x == 'x' || x == 'X') && hexd) {
        base = 16;
        p += 2;
      } else {
        base = 8;
      }
    } else {
      base = 10;
    }
  }
  const uint64_t cutoff = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  uint64_t acc = 0;
  int any = 0, overflow = 0;
  for (;; ++p) {
    unsigned c = B(p, lim);
    int d;
    if (is_digit(c)) d = (int)(c - '0');
    else if (c >= 'a' && c <= 'z') d = (int)(c - 'a') + 10;
    else if (c >= 'A' && c <= 'Z') d = (int)(c - 'A') + 10;
    else break;
    if (d >= base) break;
    any = 1;
    if (overflow) continue;
    if (acc > (cutoff - (uint64_t)d) / (uint64_t)base) {
      overflow = 1;
      continue;
    }
    acc = acc * (uint64_t)base + (uint64_t)d;
  }
  if (endptr) *endptr = any ? p : nptr;
  if (overflow) return neg ? INT64_MIN : INT64_MAX;
  if (!any) return 0;
  return neg ? (int64_t)(0 - acc) : (int64_t)acc;
}

int64_t dmo_atoll(const char *p, const char *lim) { return strtoll_impl(p, lim, 10, NULL); }
int64_t dmo_strtoll0(const char *p, const char *lim, const char **endptr) {
  return strtoll_impl(p, lim, 0, endptr);
}

/* ----------------------------------------------------------- containers -- */

typedef struct {
  void *p;
  size_t n, cap, elem;
} vec;

static void vec_push(vec *v, const void *x) {
  if (v->n == v->cap) {
    v->cap = v->cap ? v->cap * 2 : 64;
    v->p = realloc(v->p, v->cap * v->elem);
  }
  memcpy((char *)v->p + v->n * v->elem, x, v->elem);
  v->n++;
}
static void vec_init(vec *v, size_t elem) {
  v->p = NULL;
  v->n = v->cap = 0;
  v->elem = elem;
}
static void vec_free(vec *v) {
  free(v->p);
  vec_init(v, v->elem);
}

/* One RowBlockContainer (row_block.h:27-76). */
typedef struct {
  vec offset, label, weight, qid, field, index, value;
} block;

static size_t val_size(int kind) { return kind == DMO_VAL_I64 ? 8 : 4; }

static void block_init(block *b, int kind) {
  vec_init(&b->offset, 8);
  vec_init(&b->label, val_size(kind));
  vec_init(&b->weight, 4);
  vec_init(&b->qid, 8);
  vec_init(&b->field, 8);
  vec_init(&b->index, 8);
  vec_init(&b->value, val_size(kind));
  uint64_t zero = 0;
  vec_push(&b->offset, &zero); /* Clear(): offset = {0}, row_block.h:65-68 */
}
static void block_free(block *b) {
  vec_free(&b->offset);
  vec_free(&b->label);
  vec_free(&b->weight);
  vec_free(&b->qid);
  vec_free(&b->field);
  vec_free(&b->index);
  vec_free(&b->value);
}
static void push_u64(vec *v, uint64_t x) { vec_push(v, &x); }
static void push_f32(vec *v, float x) { vec_push(v, &x); }

static void set_err(dmo_csr *o, int code, const char *msg) {
  if (o->status == 0) {
    o->status = code;
    snprintf(o->msg, sizeof(o->msg), "%s", msg);
  }
}

/* ---------------------------------------------------------------- libsvm -- */

/* libsvm_parser.h:67-83 IgnoreCommentAndBlank<'#'> */
static ptrdiff_t ignore_comment_and_blank(const char *beg, const char *line_end, const char *lim) {
  const char *p = beg;
  ptrdiff_t length = line_end - beg;
  while (p != line_end) {
    if (B(p, lim) == '#') return length;
    if (!is_blank(B(p, lim))) return p - beg;
    p++;
  }
  return length;
}

/* strtonum.h:667-703 ParsePair with T1 in {float, uint}, T2 = float. */
typedef struct {
  int err_neg;   /* ParseUnsignedInt CHECK */
} pp_status;

static int parse_pair(const char *begin, const char *end, const char *lim, const char **endptr,
                      int t1_is_uint, int bits, uint64_t *u1, float *f1, float *f2, pp_status *st) {
  const char *p = begin;
  while (p != end && !is_digitchar(B(p, lim))) ++p;
  if (p == end) {
    *endptr = end;
    return 0;
  }
  const char *q = p;
  while (q != end && is_digitchar(B(q, lim))) ++q;
  if (t1_is_uint) {
    int e = 0;
    *u1 = dmo_parse_uint(p, lim, bits, &e);
    if (e) st->err_neg = 1;
  } else {
    *f1 = dmo_parse_float(p, lim, NULL);
  }
  p = q;
  while (p != end && is_blank(B(p, lim))) ++p;
  if (p == end || B(p, lim) != ':') {
    *endptr = p;
    return 1;
  }
  p++;
  while (p != end && !is_digitchar(B(p, lim))) ++p;
  q = p;
  while (q != end && is_digitchar(B(q, lim))) ++q;
  *endptr = q;
  *f2 = dmo_parse_float(p, lim, NULL);
  return 2;
}

/* libsvm_parser.h:85-172 LibSVMParser::ParseBlock */
static void parse_block_libsvm(const char *begin, const char *end, const char *lim,
                               const dmo_params *prm, block *out, dmo_csr *err) {
  const char *lbegin = begin, *lend;
  uint64_t min_feat = prm->index_bits == 32 ? 0xFFFFFFFFULL : ~0ULL;
  while (lbegin != end) {
    lend = lbegin + 1;
    while (lend != end && !is_nl(B(lend, lim))) ++lend;
    const char *p = lbegin, *q = NULL;
    float label = 0, weight = 0;
    p += ignore_comment_and_blank(p, lend, lim);
    pp_status st = {0};
    uint64_t dummy;
    int r = parse_pair(p, lend, lim, &q, 0, 32, &dummy, &label, &weight, &st);
    if (r < 1) {
      lbegin = lend;
      continue;
    }
    if (r == 2) push_f32(&out->weight, weight);
    if (out->label.n != 0) push_u64(&out->offset, out->index.n);
    push_f32(&out->label, label);
    p = q;
    while (p != end && B(p, lim) == ' ') ++p;                       /* :122-124 */
    if (p != lend && B(p, lim) == 'q' && B(p + 1, lim) == 'i' && B(p + 2, lim) == 'd' &&
        B(p + 3, lim) == ':') {                                     /* :125 strncmp */
      p += 4;
      uint64_t qid = (uint64_t)dmo_atoll(p, lim);
      while (p != lend && is_digitchar(B(p, lim))) ++p;
      push_u64(&out->qid, qid);
    }
    while (p != lend) {                                             /* :134-153 */
      p += ignore_comment_and_blank(p, lend, lim);
      uint64_t fid = 0;
      float val = 0;
      int r2 = parse_pair(p, lend, lim, &q, 1, prm->index_bits, &fid, NULL, &val, &st);
      if (st.err_neg) {
        set_err(err, 2, "Check failed: sign == true");
        return;
      }
      if (r2 < 1) {
        p = q;
        continue;
      }
      push_u64(&out->index, fid);
      if (fid < min_feat) min_feat = fid;
      if (r2 == 2) push_f32(&out->value, val);
      p = q;
    }
    lbegin = lend;
  }
  if (out->label.n != 0) push_u64(&out->offset, out->index.n);
  /* :165-171 indexing mode */
  if (prm->indexing_mode > 0 || (prm->indexing_mode < 0 && out->index.n != 0 && min_feat > 0)) {
    uint64_t *ix = (uint64_t *)out->index.p;
    uint64_t mask = prm->index_bits == 32 ? 0xFFFFFFFFULL : ~0ULL;
    for (size_t i = 0; i < out->index.n; ++i) ix[i] = (ix[i] - 1) & mask;
  }
}

/* ----------------------------------------------------------------- libfm -- */

/* strtonum.h:718-772 ParseTriple<IndexType, IndexType, real_t> */
static int parse_triple(const char *begin, const char *end, const char *lim, const char **endptr,
                        int bits, uint64_t *v1, uint64_t *v2, float *v3, pp_status *st) {
  const char *p = begin;
  int e = 0;
  while (p != end && !is_digitchar(B(p, lim))) ++p;
  if (p == end) {
    *endptr = end;
    return 0;
  }
  const char *q = p;
  while (q != end && is_digitchar(B(q, lim))) ++q;
  *v1 = dmo_parse_uint(p, lim, bits, &e);
  if (e) st->err_neg = 1;
  p = q;
  while (p != end && is_blank(B(p, lim))) ++p;
  if (p == end || B(p, lim) != ':') {
    *endptr = p;
    return 1;
  }
  p++;
  while (p != end && !is_digitchar(B(p, lim))) ++p;
  q = p;
  while (q != end && is_digitchar(B(q, lim))) ++q;
  *v2 = dmo_parse_uint(p, lim, bits, &e);
  if (e) st->err_neg = 1;
  p = q;
  while (p != end && is_blank(B(p, lim))) ++p;
  if (p == end || B(p, lim) != ':') {
    *endptr = p;
    return 2;
  }
  p++;
  while (p != end && !is_digitchar(B(p, lim))) ++p;
  q = p;
  while (q != end && is_digitchar(B(q, lim))) ++q;
  *endptr = q;
  *v3 = dmo_parse_float(p, lim, NULL);
  return 3;
}

/* libfm_parser.h:67-144 LibFMParser::ParseBlock */
static void parse_block_libfm(const char *begin, const char *end, const char *lim,
                              const dmo_params *prm, block *out, dmo_csr *err) {
  const char *lbegin = begin, *lend;
  uint64_t mx = prm->index_bits == 32 ? 0xFFFFFFFFULL : ~0ULL;
  uint64_t min_field = mx, min_feat = mx;
  while (lbegin != end) {
    lend = lbegin + 1;
    while (lend != end && !is_nl(B(lend, lim))) ++lend;
    const char *p = lbegin, *q = NULL;
    float label = 0, weight = 0;
    pp_status st = {0};
    uint64_t dummy;
    int r = parse_pair(p, lend, lim, &q, 0, 32, &dummy, &label, &weight, &st);
    if (r < 1) {
      lbegin = lend;
      continue;
    }
    if (r == 2) push_f32(&out->weight, weight);
    if (out->label.n != 0) push_u64(&out->offset, out->index.n);
    push_f32(&out->label, label);
    p = q;
    while (p != lend) {
      uint64_t fld = 0, fid = 0;
      float val = 0;
      int r3 = parse_triple(p, lend, lim, &q, prm->index_bits, &fld, &fid, &val, &st);
      if (st.err_neg) {
        set_err(err, 2, "Check failed: sign == true");
        return;
      }
      if (r3 <= 1) {
        p = q;
        continue;
      }
      push_u64(&out->field, fld);
      push_u64(&out->index, fid);
      if (fld < min_field) min_field = fld;
      if (fid < min_feat) min_feat = fid;
      if (r3 == 3) push_f32(&out->value, val);
      p = q;
    }
    lbegin = lend;
  }
  if (out->label.n != 0) push_u64(&out->offset, out->index.n);
  if (prm->indexing_mode > 0 ||
      (prm->indexing_mode < 0 && out->index.n != 0 && min_feat > 0 && out->field.n != 0 &&
       min_field > 0)) {
    uint64_t *ix = (uint64_t *)out->index.p, *fx = (uint64_t *)out->field.p;
    for (size_t i = 0; i < out->index.n; ++i) ix[i] = (ix[i] - 1) & mx;
    for (size_t i = 0; i < out->field.n; ++i) fx[i] = (fx[i] - 1) & mx;
  }
}

/* ------------------------------------------------------------------- csv -- */

/* text_parser.h:83-102 IgnoreUTF8BOM */
static void ignore_utf8_bom(const char **begin, const char *end, const char *lim) {
  int count;
  for (count = 0; *begin != end && count < 3; count++, ++*begin) {
    unsigned c = B(*begin, lim);
    if (c != 0xEF && count == 0) break;
    if (c != 0xBB && count == 1) break;
    if (c != 0xBF && count == 2) break;
  }
  if (count < 3) *begin -= count;
}

/* csv_parser.h:71-149 CSVParser::ParseBlock */
static void parse_block_csv(const char *begin, const char *end, const char *lim,
                            const dmo_params *prm, block *out, dmo_csr *err) {
  const char *lbegin = begin, *lend;
  const unsigned delim = (unsigned)(prm->delimiter & 0xFF);
  while (lbegin != end && is_nl(B(lbegin, lim))) ++lbegin;
  while (lbegin != end) {
    ignore_utf8_bom(&lbegin, end, lim);
    if (lbegin == end) break; /* the reference reads past `end` here (UB); stop instead */
    lend = lbegin + 1;
    while (lend != end && !is_nl(B(lend, lim))) ++lend;
    const char *p = lbegin;
    int column_index = 0;
    uint64_t idx = 0;
    float weight = NAN;
    while (p != lend) {
      const char *endptr;
      float vf = 0;
      int64_t vi = 0;
      if (prm->value_kind == DMO_VAL_F32) {
        vf = dmo_parse_float(p, lim, &endptr);
      } else {
        vi = dmo_strtoll0(p, lim, &endptr);
        if (prm->value_kind == DMO_VAL_I32) vi = (int64_t)(int32_t)vi;
      }
      int32_t vi32 = (int32_t)vi;
      const void *vptr = prm->value_kind == DMO_VAL_F32   ? (const void *)&vf
                         : prm->value_kind == DMO_VAL_I32 ? (const void *)&vi32
                                                          : (const void *)&vi;
      if (column_index == prm->label_column) {
        vec_push(&out->label, vptr);
      } else if (prm->value_kind == DMO_VAL_F32 && column_index == prm->weight_column) {
        weight = vf;
      } else {
        if (endptr != p) {
          vec_push(&out->value, vptr);
          push_u64(&out->index, idx++ & (prm->index_bits == 32 ? 0xFFFFFFFFULL : ~0ULL));
        } else {
          idx++;
        }
      }
      p = (endptr >= lend) ? lend : endptr;
      ++column_index;
      while (B(p, lim) != delim && p != lend) ++p;
      if (p == lend && idx == 0) {
        char m[200];
        snprintf(m, sizeof(m), "Delimiter '%c' is not found in the line. Expected '%c' as the "
                 "delimiter to separate fields.", (char)delim, (char)delim);
        set_err(err, 3, m);
        return;
      }
      if (p != lend) ++p;
    }
    while (is_nl(B(lend, lim)) && lend != end) ++lend;
    lbegin = lend;
    if (!isnan(weight)) push_f32(&out->weight, weight);
    push_u64(&out->offset, out->index.n);
  }
  if (!(out->label.n == 0 || out->label.n + 1 == out->offset.n)) {
    set_err(err, 4, "Check failed: out->label.size() == 0 || out->label.size() + 1 == "
                    "out->offset.size()");
    return;
  }
  if (!(out->weight.n == 0 || out->weight.n + 1 == out->offset.n)) {
    set_err(err, 4, "Check failed: out->weight.size() == 0 || out->weight.size() + 1 == "
                    "out->offset.size()");
  }
}

/* ------------------------------------------------------------- plumbing -- */

static void vec_append(void **dst, uint64_t *n, size_t elem, const vec *src) {
  if (src->n == 0) return;
  *dst = realloc(*dst, (*n + src->n) * elem);
  memcpy((char *)*dst + *n * elem, src->p, src->n * elem);
  *n += src->n;
}

void dmo_csr_init(dmo_csr *o, int value_kind) {
  memset(o, 0, sizeof(*o));
  o->offset = (uint64_t *)malloc(8);
  o->offset[0] = 0;
  (void)value_kind;
}

void dmo_csr_free(dmo_csr *o) {
  free(o->offset);
  free(o->label);
  free(o->weight);
  free(o->qid);
  free(o->field);
  free(o->index);
  free(o->value);
  free(o->block_rows);
  free(o->block_index);
  free(o->block_value);
  free(o->block_weight);
  free(o->block_qid);
  memset(o, 0, sizeof(*o));
}

/* RowBlockContainer::GetBlock checks (row_block.h:171-189), then
 * RowBlockContainer::Push(RowBlock) onto the running concatenation
 * (row_block.h:126-168).  Empty blocks are skipped as ParserImpl::Next does
 * (parser.h:34-39). */
static void append_block(dmo_csr *o, const block *b, const dmo_params *prm) {
  size_t rows = b->offset.n - 1;
  if (rows == 0) return;
  const uint64_t *off = (const uint64_t *)b->offset.p;
  if (b->label.n && b->label.n + 1 != b->offset.n) {
    set_err(o, 5, "Check failed: label.size() + 1 == offset.size()");
    return;
  }
  if (off[rows] != b->index.n) {
    set_err(o, 5, "Check failed: offset.back() == index.size()");
    return;
  }
  if (!(b->value.n == 0 || b->value.n == off[rows])) {
    set_err(o, 5, "Check failed: offset.back() == value.size() || value.size() == 0");
    return;
  }
  size_t vs = val_size(prm->value_kind);
  uint64_t shift = o->offset[o->n_rows];
  o->offset = (uint64_t *)realloc(o->offset, (o->n_rows + rows + 1) * 8);
  for (size_t i = 0; i < rows; ++i) o->offset[o->n_rows + 1 + i] = shift + off[i + 1] - off[0];
  vec_append(&o->label, &o->n_label, vs, &b->label);
  o->n_rows += rows;
  vec_append((void **)&o->weight, &o->n_weight, 4, &b->weight);
  vec_append((void **)&o->qid, &o->n_qid, 8, &b->qid);
  vec_append((void **)&o->field, &o->n_field, 8, &b->field);
  vec_append((void **)&o->index, &o->n_index, 8, &b->index);
  vec_append(&o->value, &o->n_value, vs, &b->value);
  size_t nb = o->n_blocks + 1;
  o->block_rows = (uint64_t *)realloc(o->block_rows, nb * 8);
  o->block_index = (uint64_t *)realloc(o->block_index, nb * 8);
  o->block_value = (uint64_t *)realloc(o->block_value, nb * 8);
  o->block_weight = (uint64_t *)realloc(o->block_weight, nb * 8);
  o->block_qid = (uint64_t *)realloc(o->block_qid, nb * 8);
  o->block_rows[o->n_blocks] = rows;
  o->block_index[o->n_blocks] = b->index.n;
  o->block_value[o->n_blocks] = b->value.n;
  o->block_weight[o->n_blocks] = b->weight.n;
  o->block_qid[o->n_blocks] = b->qid.n;
  o->n_blocks = nb;
}

static void parse_range(const char *begin, const char *end, const char *lim, const dmo_params *prm,
                        dmo_csr *out) {
  block b;
  block_init(&b, prm->value_kind);
  g_nan_error = 0;
  if (prm->format == DMO_FMT_LIBSVM) parse_block_libsvm(begin, end, lim, prm, &b, out);
  else if (prm->format == DMO_FMT_CSV) parse_block_csv(begin, end, lim, prm, &b, out);
  else parse_block_libfm(begin, end, lim, prm, &b, out);
  if (g_nan_error) set_err(out, 6, "Check failed: *p == ')' Invalid NAN literal");
  if (out->status == 0) append_block(out, &b, prm);
  block_free(&b);
}

int dmo_parse_block(const char *begin, size_t size, const dmo_params *prm, dmo_csr *out) {
  parse_range(begin, begin + size, begin + size, prm, out);
  return out->status;
}

/* text_parser.h:70-77 BackFindEndLine */
static const char *back_find_end_line(const char *bptr, const char *begin, const char *lim) {
  for (; bptr != begin; --bptr)
    if (is_nl(B(bptr, lim))) return bptr;
  return begin;
}

/* text_parser.h:116-155 FillData: ranges per thread, parsed in tid order. */
int dmo_parse_chunk(const char *head, size_t size, const dmo_params *prm, dmo_csr *out) {
  const int nthread = prm->nthread > 0 ? prm->nthread : 1;
  const char *lim = head + size;
  size_t nstep = (size + nthread - 1) / nthread;
  for (int tid = 0; tid < nthread && out->status == 0; ++tid) {
    size_t sbegin = (size_t)tid * nstep < size ? (size_t)tid * nstep : size;
    size_t send = (size_t)(tid + 1) * nstep < size ? (size_t)(tid + 1) * nstep : size;
    const char *pbegin = back_find_end_line(head + sbegin, head, lim);
    const char *pend = (tid + 1 == nthread) ? head + send : back_find_end_line(head + send, head, lim);
    parse_range(pbegin, pend, lim, prm, out);
  }
  return out->status;
}

/* ------------------------------------------------------------ InputSplit -- */

typedef struct {
  const char *const *files;
  const uint64_t *sizes;
  int nfiles;
  uint64_t *file_offset; /* nfiles + 1 */
  uint64_t offset_begin, offset_end, offset_curr;
  int file_ptr;
  uint64_t fpos; /* read position inside files[file_ptr] */
  char *overflow;
  size_t olen;
} split_state;

/* line_split.cc:11-36 SeekRecordBegin on one file stream starting at `pos`. */
static uint64_t seek_record_begin(const char *f, uint64_t fsize, uint64_t pos) {
  uint64_t nstep = 0;
  for (;;) {
    if (pos >= fsize) return nstep;
    char c = f[pos++];
    nstep += 1;
    if (c == '\n' || c == '\r') break;
  }
  for (;;) {
    if (pos >= fsize) return nstep;
    char c = f[pos++];
    if (c != '\n' && c != '\r') break;
    nstep += 1;
  }
  return nstep;
}

static int file_of(const split_state *s, uint64_t off) { /* upper_bound - 1 */
  int i = 0;
  while (i + 1 <= s->nfiles && s->file_offset[i + 1] <= off) ++i;
  return i;
}

/* input_split_base.cc:178-229 Read (text: '\n' inserted at each file end) */
static size_t split_read(split_state *s, char *buf, size_t size) {
  if (s->offset_begin >= s->offset_end) return 0;
  if (s->offset_curr + size > s->offset_end) size = s->offset_end - s->offset_curr;
  if (size == 0) return 0;
  size_t nleft = size;
  for (;;) {
    uint64_t avail = s->sizes[s->file_ptr] - s->fpos;
    size_t n = nleft < avail ? nleft : (size_t)avail;
    memcpy(buf, s->files[s->file_ptr] + s->fpos, n);
    s->fpos += n;
    nleft -= n;
    buf += n;
    s->offset_curr += n;
    if (nleft == 0) break;
    if (n == 0) {
      buf[0] = '\n';
      ++buf;
      --nleft;
      if (s->file_ptr + 1 >= s->nfiles) break;
      s->file_ptr += 1;
      s->fpos = 0;
    }
  }
  return size - nleft;
}

/* line_split.cc:37-45 FindLastRecordBegin */
static const char *find_last_record_begin(const char *begin, const char *end) {
  for (const char *p = end - 1; p != begin; --p)
    if (*p == '\n' || *p == '\r') return p + 1;
  return begin;
}

/* input_split_base.cc:231-270 ReadChunk; returns 0 at end, else 1 with *size set */
static int split_read_chunk(split_state *s, char *buf, size_t *size) {
  size_t max_size = *size;
  if (max_size <= s->olen) {
    *size = 0;
    return 1;
  }
  if (s->olen) memcpy(buf, s->overflow, s->olen);
  size_t olen = s->olen;
  s->olen = 0;
  size_t nread = split_read(s, buf + olen, max_size - olen) + olen;
  if (nread == 0) return 0;
  if (nread == olen) buf[nread++] = '\n';
  const char *bend = find_last_record_begin(buf, buf + nread);
  *size = (size_t)(bend - buf);
  s->olen = nread - *size;
  s->overflow = (char *)realloc(s->overflow, s->olen ? s->olen : 1);
  if (s->olen) memcpy(s->overflow, bend, s->olen);
  return 1;
}

int dmo_split_text(const char *const *files, const uint64_t *sizes, int nfiles, unsigned rank,
                   unsigned nsplit, uint64_t buffer_bytes, dmo_chunks *out) {
  memset(out, 0, sizeof(*out));
  out->off = (uint64_t *)calloc(1, 8);
  split_state s;
  memset(&s, 0, sizeof(s));
  /* InitInputFileInfo keeps only non-empty files (input_split_base.cc:139-161) */
  const char **fs = (const char **)malloc(sizeof(char *) * (nfiles + 1));
  uint64_t *sz = (uint64_t *)malloc(8 * (nfiles + 1));
  int nf = 0;
  for (int i = 0; i < nfiles; ++i)
    if (sizes[i]) {
      fs[nf] = files[i];
      sz[nf++] = sizes[i];
    }
  s.files = fs;
  s.sizes = sz;
  s.nfiles = nf;
  s.file_offset = (uint64_t *)calloc(nf + 1, 8);
  for (int i = 0; i < nf; ++i) s.file_offset[i + 1] = s.file_offset[i] + sz[i];
  /* ResetPartition, input_split_base.cc:29-63 (align_bytes = 1 for text) */
  uint64_t ntotal = s.file_offset[nf];
  uint64_t nstep = (ntotal + nsplit - 1) / nsplit;
  s.offset_begin = nstep * rank < ntotal ? nstep * rank : ntotal;
  s.offset_end = nstep * (rank + 1) < ntotal ? nstep * (rank + 1) : ntotal;
  if (s.offset_begin < s.offset_end) {
    int fpe = file_of(&s, s.offset_end);
    if (s.offset_end != s.file_offset[fpe])
      s.offset_end += seek_record_begin(fs[fpe], sz[fpe], s.offset_end - s.file_offset[fpe]);
    int fp = file_of(&s, s.offset_begin);
    if (s.offset_begin != s.file_offset[fp])
      s.offset_begin += seek_record_begin(fs[fp], sz[fp], s.offset_begin - s.file_offset[fp]);
    /* BeforeFirst, input_split_base.cc:65-82 */
    s.file_ptr = file_of(&s, s.offset_begin);
    s.fpos = s.offset_begin - s.file_offset[s.file_ptr];
    s.offset_curr = s.offset_begin;
    /* Chunk::Load loop, input_split_base.cc:272-291 */
    size_t words = buffer_bytes / 4;
    for (;;) {
      size_t cap_words = words + 1;
      char *buf = NULL;
      size_t got = 0;
      int ok;
      for (;;) {
        size_t size = (cap_words - 1) * 4;
        buf = (char *)realloc(buf, cap_words * 4);
        memset(buf + (cap_words - 1) * 4, 0, 4);
        ok = split_read_chunk(&s, buf, &size);
        if (!ok) break;
        if (size == 0) {
          cap_words *= 2;
        } else {
          got = size;
          break;
        }
      }
      if (!ok) {
        free(buf);
        break;
      }
      uint64_t base = out->off[out->n_chunks];
      out->buf = (char *)realloc(out->buf, base + got);
      memcpy(out->buf + base, buf, got);
      free(buf);
      out->n_chunks++;
      out->off = (uint64_t *)realloc(out->off, (out->n_chunks + 1) * 8);
      out->off[out->n_chunks] = base + got;
    }
  }
  free(s.overflow);
  free(s.file_offset);
  free(fs);
  free(sz);
  return (int)out->n_chunks;
}

void dmo_chunks_free(dmo_chunks *c) {
  free(c->off);
  free(c->buf);
  memset(c, 0, sizeof(*c));
}

/* ---------------------------------------------------------------- bench -- */

double dmo_bench_chunks(const char *buf, const uint64_t *off, int nchunks, const dmo_params *prm,
                        uint64_t *nnz) {
  struct timespec t0, t1;
  uint64_t total = 0;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (int i = 0; i < nchunks; ++i) {
    dmo_csr c;
    dmo_csr_init(&c, prm->value_kind);
    dmo_parse_chunk(buf + off[i], (size_t)(off[i + 1] - off[i]), prm, &c);
    total += c.n_index;
    dmo_csr_free(&c);
  }
  clock_gettime(CLOCK_MONOTONIC, &t1);
  if (nnz) *nnz = total;
  return (double)(t1.tv_sec - t0.tv_sec) + 1e-9 * (double)(t1.tv_nsec - t0.tv_nsec);
}
