// ranges.hip -- TextParserBase::FillData's per-chunk thread ranges
// (src/data/text_parser.h:116-155, BackFindEndLine :70-77) as ParseBlock
// unit starts for the tile kernels.
//
// Chunk c of size S is cut into T = nthread ranges: range t starts at
// BackFindEndLine(head + min(t * ceil(S/T), S), head) -- the last '\n' / '\r'
// at or before that byte and after the chunk's first byte, else the chunk
// start -- and ends where range t + 1 starts (the last range at the chunk
// end).  Unit u = c * T + t; units[nchunk * T] = n.  Bytes at or past the
// chunk end read as NUL (never a newline), as the oracle restates the byte the
// reference reads one past a chunk.
//
// One wave per cut scans back 1 KiB per step (16 coalesced byte loads per
// lane, one ballot each), so a 35 KB line costs ~35 steps, not 35k loads.
#include "common.h"
#include "dmlc_amd_kernels.h"

namespace dmlc_amd {
namespace {

__global__ void __launch_bounds__(256) range_kernel(const uint8_t *text, const uint64_t *cs, int nchunk,
                                                    int nthread, uint64_t n, uint64_t *units) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t u = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);  // one wave per unit
  const uint64_t nunits = (uint64_t)nchunk * nthread;
  if (u > nunits) return;
  if (u == nunits) {
    if (lane == 0) units[u] = n;
    return;
  }
  const uint64_t c = u / (uint64_t)nthread, t = u % (uint64_t)nthread;
  const uint64_t head = cs[c], size = cs[c + 1] - head;
  const uint64_t nstep = (size + nthread - 1) / (uint64_t)nthread;
  const uint64_t sbegin = t * nstep < size ? t * nstep : size;
  uint64_t res = head;
  // BackFindEndLine(head + sbegin, head): positions head+sbegin down to head+1
  for (uint64_t top = head + sbegin; top > head;) {
    uint64_t found = 0;
    bool hit = false;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint64_t off = (uint64_t)i * 64 + lane;  // distance below top
      bool nl = false;
      if (off < top - head) {
        const uint64_t p = top - off;
        nl = p < head + size && is_nl(text[p]);
      }
      const uint64_t m = __ballot(nl);
      if (!hit && m) {
        hit = true;
        found = top - ((uint64_t)i * 64 + (uint64_t)__builtin_ctzll(m));
      }
    }
    if (hit) {
      res = found;
      break;
    }
    top = top - head > 1024 ? top - 1024 : head;
  }
  if (lane == 0) units[u] = t == 0 ? head : res;
}

}  // namespace

hipError_t launch_ranges(const uint8_t *text, const uint64_t *cs, int nchunk, int nthread, uint64_t n,
                         uint64_t *units, hipStream_t s) {
  const uint64_t waves = (uint64_t)nchunk * nthread + 1;
  range_kernel<<<(unsigned)((waves + 3) / 4), 256, 0, s>>>(text, cs, nchunk, nthread, n, units);
  return hipGetLastError();
}

}  // namespace dmlc_amd
