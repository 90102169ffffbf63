// FETCH_SIZE / WRITE_SIZE calibration by access width (MI355X_MICROARCH.md:
// on gfx950 FETCH_SIZE counts half the bytes of 16-byte-per-lane streaming
// reads; "other access widths are uncalibrated: calibrate on a known byte
// count in your own access pattern").  One launch per kernel below, each
// moving exactly kBytes (1 GiB, far past the 256 MiB Infinity Cache) in
// coalesced lanes of 1 / 4 / 8 / 16 bytes; run under
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -- ./pmc_calib   (then WRITE_SIZE)
// and divide each kernel's counter (KiB) by kBytes / 1024.
// The exact tile kernels read their count-pass records and store the CSR by
// 4-byte lanes and stage the text by 16-byte lanes; the single-pass kernels
// stage by 16-byte lanes and store by 4- / 8-byte lanes.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint64_t kBytes = 1ull << 30;

template <class T>
__global__ void __launch_bounds__(256) read_w(const T *__restrict__ src, uint64_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const T v = src[i];
    const uint32_t *w = reinterpret_cast<const uint32_t *>(&v);
    if (sizeof(T) >= 4)
      for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc ^= w[k];
    else
      acc ^= (uint32_t) * reinterpret_cast<const uint8_t *>(&v);
  }
  if (acc == 0x9E3779B9u) sink[threadIdx.x] = acc;  // (keeps the loads; practically never stores)
}

template <class T>
__global__ void __launch_bounds__(256) write_w(T *__restrict__ dst, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    T v;
    uint8_t *b = reinterpret_cast<uint8_t *>(&v);
    for (int k = 0; k < (int)sizeof(T); ++k) b[k] = (uint8_t)(i + k);
    dst[i] = v;
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      return 1;                                                                \
    }                                                                          \
  } while (0)

int main() {
  void *buf = nullptr;
  uint32_t *sink = nullptr;
  CK(hipMalloc(&buf, kBytes));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(buf, 1, kBytes));
  const unsigned grid = 256 * 32;
  read_w<uint8_t><<<grid, 256>>>(static_cast<const uint8_t *>(buf), kBytes, sink);
  read_w<uint32_t><<<grid, 256>>>(static_cast<const uint32_t *>(buf), kBytes / 4, sink);
  read_w<uint2><<<grid, 256>>>(static_cast<const uint2 *>(buf), kBytes / 8, sink);
  read_w<uint4><<<grid, 256>>>(static_cast<const uint4 *>(buf), kBytes / 16, sink);
  write_w<uint8_t><<<grid, 256>>>(static_cast<uint8_t *>(buf), kBytes);
  write_w<uint32_t><<<grid, 256>>>(static_cast<uint32_t *>(buf), kBytes / 4);
  write_w<uint2><<<grid, 256>>>(static_cast<uint2 *>(buf), kBytes / 8);
  write_w<uint4><<<grid, 256>>>(static_cast<uint4 *>(buf), kBytes / 16);
  CK(hipDeviceSynchronize());
  std::printf("{\"case\": \"pmc_calib\", \"bytes_per_kernel\": %llu, \"kib_per_kernel\": %llu}\n",
              (unsigned long long)kBytes, (unsigned long long)(kBytes >> 10));
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}
