// Read ceilings for k_crc's access pattern (measurement only, not product code):
// a plain grid-stride 16 B/lane read (default and nontemporal), and k_crc's
// shape -- one wave per 32 KiB chunk, rows of 1 KiB, 4 register buffers of 4
// rows (3 stages in flight), W waves per workgroup, one workgroup per CU --
// with the fold replaced by an XOR. 16 GiB swept per launch.
// Build: hipcc -O3 --offload-arch=gfx950 tools/membench2.hip -o /tmp/mb2
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

template <bool NT>
__global__ void read_flat(const u32x4 *__restrict__ in, size_t n, uint32_t *sink) {
  uint32_t s = 0;
#pragma unroll 4
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 v = NT ? __builtin_nontemporal_load(in + i) : in[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) sink[0] = s;
}

constexpr int kRows = 4, kBufs = 4, kStages = 32 / kRows;

template <bool NT>
__device__ __forceinline__ void load_stage(u32x4 (&u)[kRows], const uint8_t *ck, int q, int l) {
  const u32x4 *row = reinterpret_cast<const u32x4 *>(ck) + 64 * kRows * q + l;
#pragma unroll
  for (int r = 0; r < kRows; r++) u[r] = NT ? __builtin_nontemporal_load(row + 64 * r) : row[64 * r];
}

template <int W, bool NT>
__global__ void __launch_bounds__(64 * W) chunk_crc_shape(const uint8_t *__restrict__ span, size_t nchunks,
                                                          uint32_t *sink) {
  const int l = threadIdx.x & 63;
  const size_t nwaves = (size_t)gridDim.x * W;
  size_t c = (size_t)blockIdx.x * W + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (c >= nchunks) return;
  u32x4 buf[kBufs][kRows];
  uint32_t s = 0;
#pragma unroll
  for (int q = 0; q < kBufs - 1; q++) load_stage<NT>(buf[q], span + c * 32768, q, l);
  for (;;) {
    const uint8_t *ck = span + c * 32768;
    const size_t cn = c + nwaves;
    const bool more = cn < nchunks;
#pragma unroll
    for (int q = 0; q < kStages; q++) {
      const int nq = q + kBufs - 1;
      if (nq < kStages) load_stage<NT>(buf[nq % kBufs], ck, nq, l);
      else if (more) load_stage<NT>(buf[nq % kBufs], span + cn * 32768, nq - kStages, l);
#pragma unroll
      for (int r = 0; r < kRows; r++) s ^= buf[q % kBufs][r].x ^ buf[q % kBufs][r].y ^ buf[q % kBufs][r].z ^ buf[q % kBufs][r].w;
    }
    if (!more) break;
    c = cn;
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
  const size_t n16 = bytes / 16, nch = bytes / 32768;
  for (int g : {2048, 4096, 8192}) {
    float ms = timeit([&] { hipLaunchKernelGGL(read_flat<false>, dim3(g), dim3(256), 0, 0, (const u32x4 *)in, n16, sink); });
    printf("{\"k\":\"read_flat\",\"grid\":%d,\"ms\":%.3f,\"TBs\":%.3f}\n", g, ms, bytes / ms / 1e9);
    ms = timeit([&] { hipLaunchKernelGGL(read_flat<true>, dim3(g), dim3(256), 0, 0, (const u32x4 *)in, n16, sink); });
    printf("{\"k\":\"read_flat_nt\",\"grid\":%d,\"ms\":%.3f,\"TBs\":%.3f}\n", g, ms, bytes / ms / 1e9);
  }
#define RUN(W, NT, G)                                                                                          \
  {                                                                                                            \
    float ms = timeit([&] { hipLaunchKernelGGL((chunk_crc_shape<W, NT>), dim3(G), dim3(64 * W), 0, 0, in, nch, sink); }); \
    printf("{\"k\":\"crc_shape\",\"waves\":%d,\"nt\":%d,\"grid\":%d,\"ms\":%.3f,\"TBs\":%.3f}\n", W, NT, G, ms,   \
           bytes / ms / 1e9);                                                                                  \
  }
  RUN(12, true, ncu) RUN(12, false, ncu) RUN(16, true, ncu) RUN(8, true, ncu) RUN(12, true, 2 * ncu)
  RUN(4, true, 4 * ncu) RUN(4, true, 8 * ncu)
  return 0;
}
