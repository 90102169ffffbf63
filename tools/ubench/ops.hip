// Instruction-rate probe: each kernel runs 8 independent chains of one op per
// lane; time per wave-instruction across the whole chip.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define N_IT 4096
template <int OP>
__global__ void __launch_bounds__(256) k(uint32_t *out, uint32_t seed) {
  uint32_t a[8];
  double d[8];
  for (int i = 0; i < 8; ++i) { a[i] = seed * (threadIdx.x + i * 77 + 1); d[i] = (double)a[i]; }
  const uint32_t c = seed | 0x01010101u;
  const double dc = 1.0000001;
#pragma unroll 1
  for (int it = 0; it < N_IT; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (OP == 0) a[i] = a[i] + c;                                   // v_add_u32
      if (OP == 1) a[i] = a[i] * c;                                   // v_mul_lo_u32
      if (OP == 2) a[i] = __umul24(a[i], c) + i;                      // v_mad_u32_u24
      if (OP == 3) a[i] = __builtin_amdgcn_udot4(a[i], c, a[i], false);  // v_dot4_u32_u8
      if (OP == 4) a[i] = __builtin_amdgcn_perm(a[i], c, 0x05040100u + i);  // v_perm_b32
      if (OP == 5) d[i] = __builtin_fma(d[i], dc, 1.0);               // v_fma_f64
      if (OP == 6) a[i] = __umulhi(a[i], c);                          // v_mul_hi_u32
      if (OP == 7) { uint64_t x = ((uint64_t)a[i] << 32 | c) * 0x0102040810204080ull; a[i] = (uint32_t)(x >> 40); }
      if (OP == 8) a[i] = __builtin_amdgcn_alignbit(a[i], c, a[i] & 31);
      if (OP == 9) d[i] = d[i] / 3.0;                                 // f64 divide sequence
      if (OP == 10) a[i] = __builtin_amdgcn_sad_u8(a[i], c, a[i]);
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < 8; ++i) s += a[i] + (uint32_t)d[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}
template <int OP>
void run(const char *name, uint32_t *buf, int blocks) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  k<OP><<<blocks, 256>>>(buf, 3);
  hipEventRecord(e0);
  k<OP><<<blocks, 256>>>(buf, 3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  double winst = (double)blocks * 4 * N_IT * 8;  // wave-instructions of the op
  // cycles per wave-instruction per CU at 2.4 GHz on 256 CUs
  printf("%-14s %8.3f ms  %.3f CU-cycles per wave-op (0.5 = full rate SIMD32)\n", name, ms,
         ms * 1e-3 * 2.4e9 * 256 / winst);
}
int main() {
  uint32_t *buf; int blocks = 256 * 8 * 4;
  hipMalloc(&buf, blocks * 256 * 4);
  run<0>("add_u32", buf, blocks); run<1>("mul_lo_u32", buf, blocks); run<2>("mad_u24", buf, blocks);
  run<3>("dot4_u32_u8", buf, blocks); run<4>("perm_b32", buf, blocks); run<5>("fma_f64", buf, blocks);
  run<6>("mul_hi_u32", buf, blocks); run<7>("mul_u64", buf, blocks); run<8>("alignbit", buf, blocks);
  run<9>("div_f64", buf, blocks); run<10>("sad_u8", buf, blocks);
  return 0;
}
