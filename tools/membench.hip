// HBM ceiling microbenchmarks on MI355X (measurement only, not product code).
// Build+run on the GPU box: hipcc -O3 --offload-arch=gfx950 tools/membench.hip -o /tmp/mb && /tmp/mb
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);           \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void copy_f4(const uint4 *__restrict__ in, uint4 *__restrict__ out, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
#pragma unroll 4
  for (; i < n; i += stride) out[i] = in[i];
}

__global__ void read_f4(const uint4 *__restrict__ in, size_t n, uint32_t *sink) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t s = 0;
#pragma unroll 4
  for (; i < n; i += stride) {
    uint4 v = in[i];
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) sink[0] = s;
}

// wave per 32 KiB chunk, 32 rows of 1 KiB, U rows in flight
template <int U, bool COPY>
__global__ void chunk_pat(const uint8_t *__restrict__ in, uint8_t *__restrict__ out, size_t nchunks,
                          uint32_t *sink) {
  const int l = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t s = 0;
  for (size_t c = wave; c < nchunks; c += nw) {
    const uint8_t *ck = in + c * 32768;
#pragma unroll U
    for (int i = 0; i < 32; i++) {
      const int o = 1024 * i + 16 * l;
      uint4 v = *reinterpret_cast<const uint4 *>(ck + o);
      if (COPY) *reinterpret_cast<uint4 *>(out + c * 32768 + o) = v;
      else s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (s == 0x12345678u) sink[0] = s;
}

// same, but all 32 loads of the chunk issued before use (32 x 16 B per lane)
__global__ void chunk_all(const uint8_t *__restrict__ in, size_t nchunks, uint32_t *sink) {
  const int l = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t s = 0;
  for (size_t c = wave; c < nchunks; c += nw) {
    const uint8_t *ck = in + c * 32768;
    uint4 v[16];
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = *reinterpret_cast<const uint4 *>(ck + 1024 * i + 16 * l);
#pragma unroll
    for (int i = 0; i < 16; i++) s ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = *reinterpret_cast<const uint4 *>(ck + 16384 + 1024 * i + 16 * l);
#pragma unroll
    for (int i = 0; i < 16; i++) s ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
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
  uint8_t *in, *out;
  uint32_t *sink;
  CK(hipMalloc(&in, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(in, 1, bytes));
  CK(hipMemset(out, 0, bytes));
  const size_t n4 = bytes / 16, nch = bytes / 32768;
  int grids[] = {1024, 2048, 4096, 8192};
  for (int g : grids) {
    float ms = timeit([&] { hipLaunchKernelGGL(copy_f4, dim3(g), dim3(256), 0, 0, (const uint4 *)in, (uint4 *)out, n4); });
    printf("{\"k\":\"copy_f4\",\"grid\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", g, ms, 2.0 * bytes / ms / 1e6);
    ms = timeit([&] { hipLaunchKernelGGL(read_f4, dim3(g), dim3(256), 0, 0, (const uint4 *)in, n4, sink); });
    printf("{\"k\":\"read_f4\",\"grid\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", g, ms, 1.0 * bytes / ms / 1e6);
  }
  for (int g : {1024, 2048, 4096}) {
#define RUN(U, C)                                                                                              \
  {                                                                                                            \
    float ms = timeit([&] { hipLaunchKernelGGL((chunk_pat<U, C>), dim3(g), dim3(256), 0, 0, in, out, nch, sink); }); \
    printf("{\"k\":\"chunk_%s_u%d\",\"grid\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", C ? "copy" : "read", U, g, ms,     \
           (C ? 2.0 : 1.0) * bytes / ms / 1e6);                                                                 \
  }
    RUN(1, false) RUN(4, false) RUN(8, false) RUN(32, false) RUN(4, true) RUN(8, true)
    float ms = timeit([&] { hipLaunchKernelGGL(chunk_all, dim3(g), dim3(256), 0, 0, in, nch, sink); });
    printf("{\"k\":\"chunk_all16\",\"grid\":%d,\"ms\":%.3f,\"GBs\":%.1f}\n", g, ms, 1.0 * bytes / ms / 1e6);
  }
  float ms = timeit([&] { CK(hipMemcpyAsync(out, in, bytes, hipMemcpyDeviceToDevice, 0)); });
  printf("{\"k\":\"hipMemcpyD2D\",\"ms\":%.3f,\"GBs\":%.1f}\n", ms, 2.0 * bytes / ms / 1e6);
  return 0;
}
