// Read ceilings for k_crc's access pattern, round 6 (measurement only, not
// product code): does the order in which a CU's waves walk their chunks decide
// the HBM read rate? k_crc's shape (one wave per 32 KiB chunk, rows of 1 KiB,
// 4 register buffers of 4 rows, W waves per workgroup, one workgroup per CU)
// with the fold replaced by an XOR, and the wave's 8 stages of 4 KiB visited
// from stage ROT(wave) on (rotated, wrapping) instead of from stage 0: with
// every wave at the same stage, the chip reads 3,072 addresses 32 KiB apart at
// once; rotated, their low address bits differ. 16 GiB swept per launch.
// Build: hipcc -O3 --offload-arch=gfx950 tools/membench3.hip -o /tmp/mb3
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);     \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kRows = 4, kBufs = 4, kStages = 32 / kRows;

__device__ __forceinline__ void load_stage(u32x4 (&u)[kRows], const uint8_t *ck, int q, int l) {
  const u32x4 *row = reinterpret_cast<const u32x4 *>(ck) + 64 * kRows * (q & (kStages - 1)) + l;
#pragma unroll
  for (int r = 0; r < kRows; r++) u[r] = __builtin_nontemporal_load(row + 64 * r);
}

// MODE 0: stages 0..7 in order; 1: from stage (wave in CU) mod 8; 2: from stage
// (chunk index) mod 8; 3: from stage (CU index) mod 8
template <int W, int MODE>
__global__ void __launch_bounds__(64 * W) shape(const uint8_t *__restrict__ span, size_t nchunks, uint32_t *sink) {
  const int l = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t nwaves = (size_t)gridDim.x * W;
  size_t c = (size_t)blockIdx.x * W + wv;
  if (c >= nchunks) return;
  auto rot = [&](size_t ch) -> int {
    return MODE == 0 ? 0 : MODE == 1 ? (wv & 7) : MODE == 2 ? (int)(ch & 7) : (int)(blockIdx.x & 7);
  };
  u32x4 buf[kBufs][kRows];
  uint32_t s = 0;
  int r0 = rot(c);
#pragma unroll
  for (int q = 0; q < kBufs - 1; q++) load_stage(buf[q], span + c * 32768, q + r0, l);
  for (;;) {
    const uint8_t *ck = span + c * 32768;
    const size_t cn = c + nwaves;
    const bool more = cn < nchunks;
    const int r1 = more ? rot(cn) : 0;
#pragma unroll
    for (int q = 0; q < kStages; q++) {
      const int nq = q + kBufs - 1;
      if (nq < kStages) load_stage(buf[nq % kBufs], ck, nq + r0, l);
      else if (more) load_stage(buf[nq % kBufs], span + cn * 32768, nq - kStages + r1, l);
#pragma unroll
      for (int r = 0; r < kRows; r++)
        s ^= buf[q % kBufs][r].x ^ buf[q % kBufs][r].y ^ buf[q % kBufs][r].z ^ buf[q % kBufs][r].w;
    }
    if (!more) break;
    c = cn;
    r0 = r1;
  }
  if (s == 0x12345678u) sink[0] = s;
}

template <class F>
float timeit(F f, int reps = 5) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; i++) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const size_t bytes = 16ull << 30;
  uint8_t *in;
  uint32_t *sink;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(in, 1, bytes));
  int ncu = 0;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const size_t nch = bytes / 32768;
#define RUN(W, M)                                                                                                  \
  {                                                                                                                \
    float ms = timeit([&] { hipLaunchKernelGGL((shape<W, M>), dim3(ncu), dim3(64 * W), 0, 0, in, nch, sink); }); \
    printf("{\"k\":\"crc_shape\",\"waves\":%d,\"mode\":%d,\"ms\":%.3f,\"TBs\":%.3f}\n", W, M, ms, bytes / ms / 1e9); \
  }
  for (int rep = 0; rep < 2; rep++) {
    RUN(8, 0) RUN(8, 1) RUN(8, 2) RUN(8, 3)
    RUN(12, 0) RUN(12, 1) RUN(12, 2) RUN(12, 3)
    RUN(16, 0) RUN(16, 1) RUN(16, 2)
  }
  return 0;
}
