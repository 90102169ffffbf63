// TEST INFRASTRUCTURE ONLY: the 32-bit window decoders of fast_common.h
// (wfloat32 / wuint32) against the exact byte decoders of decode.h on
// generated number strings; every string the window form accepts must decode
// bit-identically.  usage: dec_check <count> <seed>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "fast_common.h"
#include "csv_core.h"
#include "libsvm_core.h"

using namespace dmlc_amd;
using namespace dmlc_amd::fast;

struct Blk {
  int t;
  int tid() const { return t; }
};

static uint64_t st = 88172645463325252ull;
static uint64_t rnd() {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}

static std::string gen() {
  std::string s;
  const int kind = (int)(rnd() % 10);
  if (rnd() % 8 == 0) s += "+-"[rnd() % 2];
  if (kind < 6) {  // %.9g-like canonical values
    char buf[64];
    const double x = (double)(rnd() % 16777216) / 16777216.0 * (rnd() % 4 == 0 ? 100.0 : 1.0);
    snprintf(buf, sizeof buf, "%.*g", (int)(1 + rnd() % 12), x);
    s += buf;
  } else {  // random digitchar soup
    const char *al = "0123456789012345678901234567890123456789..eE+-";
    const int n = 1 + (int)(rnd() % 18);
    for (int i = 0; i < n; ++i) s += al[rnd() % strlen(al)];
  }
  return s;
}

int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  st ^= argc > 2 ? (uint64_t)atoll(argv[2]) * 0x9E3779B97F4A7C15ull : 0;
  DecTables tb;
  for (int t = 0; t < 256; ++t) {
    Blk b{t};
    init_dec_tables(tb, b);
  }
  long fast_f = 0, fast_i = 0, bad = 0;
  {  // exact kernels' segment masks (exact_dec.h seg_masks) against the byte classes
    uint8_t win[64 + 40];
    for (int it = 0; it < 20000; ++it) {
      for (auto &c : win) c = (uint8_t)(rnd() % 4 ? "0123456789+-.eE \n\r:#xq"[rnd() % 22] : rnd() % 256);
      const uint32_t off = (uint32_t)(rnd() % 40);
      const int len = 1 + (int)(rnd() % 32);
      uint32_t dm, nl, rd = 0, rn = 0;
      seg_masks(win, off, len, &dm, &nl);
      for (int i = 0; i < len; ++i) {
        rd |= (uint32_t)is_digitchar(win[off + i]) << i;
        rn |= (uint32_t)is_nl(win[off + i]) << i;
      }
      if (dm != rd || nl != rn) {
        if (bad++ < 10) printf("seg_masks mismatch off %u len %d\n", off, len);
      }
      {
        uint32_t d5, n5, c5, b5, h5, rc = 0, rb = 0, rh = 0;
        seg_masks5(win, off, len, &d5, &n5, &c5, &b5, &h5);
        for (int i = 0; i < len; ++i) {
          rc |= (uint32_t)(win[off + i] == ':') << i;
          rb |= (uint32_t)is_blank(win[off + i]) << i;
          rh |= (uint32_t)(win[off + i] == '#') << i;
        }
        if (d5 != rd || n5 != rn || c5 != rc || b5 != rb || h5 != rh) {
          if (bad++ < 10) printf("seg_masks5 mismatch off %u len %d\n", off, len);
        }
      }
      const uint32_t delim = "\n,;| \t:\xff"[rnd() % 8] & 0xFFu;
      uint32_t cn, cd, rd2 = 0;
      seg_masks_csv(win, off, len, delim, &cn, &cd);
      for (int i = 0; i < len; ++i) rd2 |= (uint32_t)(win[off + i] == delim) << i;
      if (cn != rn || cd != rd2) {
        if (bad++ < 10) printf("seg_masks_csv mismatch off %u len %d delim %u\n", off, len, delim);
      }
    }
  }
  for (long it = 0; it < n; ++it) {
    std::string s = gen();
    s += " :\n"[rnd() % 3];
    while (s.size() < 40) s += ' ';
    const uint8_t *p = reinterpret_cast<const uint8_t *>(s.data());
    uint32_t w[4];
    memcpy(w, p, 16);
    auto at = [&](uint64_t i) -> uint32_t { return i < s.size() ? p[i] : 0u; };
    bool ok = false;
    const float v = wfloat32(w, tb, &ok);
    if (ok) {
      ++fast_f;
      uint64_t e;
      bool ne = false;
      const float r = parse_float(at, 0, &e, &ne);
      if (memcmp(&v, &r, 4)) {
        if (bad++ < 10) printf("float mismatch '%.20s' fast=%.9g ref=%.9g\n", s.c_str(), v, r);
      }
    }
    uint64_t iv = 0;
    bool iok = false;
    const bool pos = wuint32(w, tb, &iv, &iok);
    if (iok) {
      ++fast_i;
      uint64_t r = 0;
      const bool rpos = parse_uint(at, 0, false, &r);
      if (pos != rpos || (pos && (uint32_t)iv != (uint32_t)r)) {
        if (bad++ < 10) printf("uint mismatch '%.20s' fast=%llu ref=%llu\n", s.c_str(),
                               (unsigned long long)iv, (unsigned long long)r);
      }
    }
  }
  // the exact kernels' use (libsvm_core.h value_at / index_at): a run that
  // starts with a digitchar, followed by any bytes (letters, inf / nan,
  // bytes >= 0x80); the window result must equal the byte decoder's
  long ex_f = 0, ex_c = 0;
  for (long it = 0; it < n; ++it) {
    std::string s;
    const char *head = (it & 1) ? "0123456789+-.eE" : "0123456789+-.eE a,\n\tiInNfF\v\f\rx";
    s += head[rnd() % strlen(head)];
    const char *al = "0123456789012345678901234567890123456789..eE+-infaINFANx :#\t";
    const int m = (int)(rnd() % 24);
    for (int i = 0; i < m; ++i) {
      const uint64_t r = rnd() % 64;
      if (r == 0) s += (char)(0x80 + rnd() % 128);
      else if (r == 1) s += "inf";
      else if (r == 2) s += "nan";
      else s += al[rnd() % strlen(al)];
    }
    while (s.size() < 48) s += (char)(rnd() % 2 ? ' ' : '\n');
    const uint8_t *p = reinterpret_cast<const uint8_t *>(s.data());
    const uint64_t lim = 16 + rnd() % 24;  // the chunk end: bytes at or past it read as NUL
    Src src;
    src.g = p;
    src.lim = lim;
    src.lds = p;
    src.wbase = 0;
    src.wend = s.size();
    GSrc at{p, lim};
    bool ne1 = false, ne2 = false;
    uint64_t e;
    const float v = value_at(src, 0, &tb, &ne1);
    const float r = parse_float(at, 0, &e, &ne2);
    const bool run = true;  // value_at / index_at take any start
    ex_f += run;
    if (run && (memcmp(&v, &r, 4) || ne1 != ne2)) {
      if (bad++ < 10) printf("exact float mismatch '%.24s' win=%.9g byte=%.9g\n", s.c_str(), v, r);
    }
    {  // CSV fields (csv_core.h decode_field): value and endptr
      float cv;
      uint64_t ce = 0;
      if (csv_value_at(src, 0, &tb, &cv, &ce)) {
        ++ex_c;
        if (memcmp(&cv, &r, 4) || ce != e) {
          if (bad++ < 10) printf("csv mismatch '%.24s' win=%.9g end %llu byte=%.9g end %llu\n", s.c_str(), cv,
                                 (unsigned long long)ce, r, (unsigned long long)e);
        }
      }
    }
    for (int vt = 0; vt < 3; ++vt) {  // CSV count pass: field_consumed == (decode_field's end != p)
      const csv::Field f = csv::decode_field(src, vt, 0);
      if (csv::field_consumed(src, vt, 0) != (f.end != 0)) {
        if (bad++ < 10) printf("consumed mismatch vt %d '%.24s'\n", vt, s.c_str());
      }
    }
    for (int wide = 0; wide < 2; ++wide) {
      uint64_t a = 0, b = 0;
      const bool pa = index_at(src, 0, wide, &tb, &a);
      const bool pb = parse_uint(at, 0, wide, &b);
      if (run && (pa != pb || (pa && a != b))) {
        if (bad++ < 10) printf("exact uint mismatch '%.24s' win=%llu byte=%llu\n", s.c_str(),
                               (unsigned long long)a, (unsigned long long)b);
      }
    }
  }
  printf("strings %ld, float fast %ld, uint fast %ld, exact-form %ld, csv window %ld, mismatches %ld\n", n,
         fast_f, fast_i, ex_f, ex_c, bad);
  return bad != 0;
}
