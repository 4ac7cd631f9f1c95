// Device -> pinned-host copies on an SDMA engine through the HSA API
// (hsa_amd_memory_async_copy_on_engine, force_copy_on_sdma) against
// hipMemcpyAsync (which this runtime runs as a blit kernel), alone and beside
// a streaming kernel on the compute queue: the copy rate and the kernel's
// slowdown in each case. Measurement only (end-to-end).
// Build: hipcc -O3 --offload-arch=gfx950 tools/sdma_probe.cpp -lhsa-runtime64 -o /tmp/sdma_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <chrono>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                 \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)
#define HK(x)                                                                         \
  do {                                                                                \
    hsa_status_t e = (x);                                                             \
    if (e != HSA_STATUS_SUCCESS) {                                                    \
      const char *m = nullptr;                                                        \
      hsa_status_string(e, &m);                                                       \
      printf("HSA error %d (%s) at %d\n", (int)e, m ? m : "?", __LINE__);             \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

__global__ void stream_read(const uint4 *__restrict__ in, size_t n, uint32_t *sink, int reps) {
  uint32_t s = 0;
  for (int r = 0; r < reps; r++)
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(in) + i);
      s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
  if (s == 0x12345678u) sink[0] = s;
}

static hsa_agent_t g_gpu{}, g_cpu{};
static hsa_status_t find_agents(hsa_agent_t a, void *) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !g_gpu.handle) g_gpu = a;
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  return HSA_STATUS_SUCCESS;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  CK(hipSetDevice(0));
  CK(hipFree(0));
  HK(hsa_init());
  HK(hsa_iterate_agents(find_agents, nullptr));
  uint32_t mask = 0;
  HK(hsa_amd_memory_copy_engine_status(g_cpu, g_gpu, &mask));
  printf("{\"sdma_engines_free_mask\": %u}\n", mask);
  const size_t N = 512ull << 20, S = 8ull << 30;
  void *d, *h, *big;
  uint32_t *sink;
  CK(hipMalloc(&d, N));
  CK(hipMalloc(&big, S));
  CK(hipMalloc(&sink, 64));
  CK(hipHostMalloc(&h, N, hipHostMallocDefault));
  CK(hipMemset(d, 1, N));
  CK(hipMemset(big, 2, S));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hsa_signal_t sig;
  HK(hsa_signal_create(1, 0, nullptr, &sig));
  CK(hipDeviceSynchronize());
  auto sdma = [&](int engine) {
    hsa_signal_store_relaxed(sig, 1);
    HK(hsa_amd_memory_async_copy_on_engine(h, g_cpu, d, g_gpu, N, 0, nullptr, sig,
                                           (hsa_amd_sdma_engine_id_t)(1u << engine), true));
  };
  auto sdma_wait = [&]() { hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED); };
  auto kern = [&](int reps) {
    hipLaunchKernelGGL(stream_read, dim3(2048), dim3(256), 0, st, (const uint4 *)big, S / 16, sink, reps);
  };
  int engine = 0;
  for (int e = 0; e < 16; e++)
    if (mask & (1u << e)) {
      engine = e;
      break;
    }
  hipEvent_t k0, k1;
  CK(hipEventCreate(&k0));
  CK(hipEventCreate(&k1));
  auto kern_timed = [&](int reps) {
    CK(hipEventRecord(k0, st));
    kern(reps);
    CK(hipEventRecord(k1, st));
  };
  auto kern_ms = [&]() {
    CK(hipEventSynchronize(k1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, k0, k1));
    return (double)ms;
  };
  const int R = 8;  // ~11 ms of streaming, about one copy's time
  for (int it = 0; it < 3; it++) {
    double t0 = now_ms();
    CK(hipMemcpyAsync(h, d, N, hipMemcpyDeviceToHost, st));
    CK(hipStreamSynchronize(st));
    double t1 = now_ms();
    sdma(engine);
    sdma_wait();
    double t2 = now_ms();
    kern_timed(R);
    const double ka = kern_ms();
    // beside the kernel: a blit copy on another stream, then the SDMA copy
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    kern_timed(R);
    double t3 = now_ms();
    CK(hipMemcpyAsync(h, d, N, hipMemcpyDeviceToHost, s2));
    CK(hipStreamSynchronize(s2));
    double t4 = now_ms();
    const double kb = kern_ms();
    kern_timed(R);
    double t5 = now_ms();
    sdma(engine);
    sdma_wait();
    double t6 = now_ms();
    const double ks = kern_ms();
    CK(hipStreamDestroy(s2));
    printf("{\"it\":%d,\"blit_alone_GBs\":%.1f,\"sdma_alone_GBs\":%.1f,\"kernel_alone_ms\":%.3f,"
           "\"blit_beside_GBs\":%.1f,\"kernel_beside_blit_ms\":%.3f,\"sdma_beside_GBs\":%.1f,\"kernel_beside_sdma_ms\":%.3f}\n",
           it, N / (t1 - t0) / 1e6, N / (t2 - t1) / 1e6, ka, N / (t4 - t3) / 1e6, kb, N / (t6 - t5) / 1e6, ks);
  }
  // each engine alone, both directions, and the runtime's preferred engines
  uint32_t pref_out = 0, pref_in = 0, st_in = 0;
  hsa_amd_memory_get_preferred_copy_engine(g_cpu, g_gpu, &pref_out);
  hsa_amd_memory_get_preferred_copy_engine(g_gpu, g_cpu, &pref_in);
  hsa_amd_memory_copy_engine_status(g_gpu, g_cpu, &st_in);
  printf("{\"preferred_out\": %u, \"preferred_in\": %u, \"status_in\": %u}\n", pref_out, pref_in, st_in);
  for (int e = 0; e < 16; e++) {
    if (!(mask & (1u << e))) continue;
    double best_out = 0, best_in = 0;
    for (int it = 0; it < 3; it++) {
      double t0 = now_ms();
      sdma(e);
      sdma_wait();
      double t1 = now_ms();
      hsa_signal_store_relaxed(sig, 1);
      HK(hsa_amd_memory_async_copy_on_engine(d, g_gpu, h, g_cpu, N, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)(1u << e),
                                             true));
      sdma_wait();
      double t2 = now_ms();
      best_out = std::max(best_out, N / (t1 - t0) / 1e6);
      best_in = std::max(best_in, N / (t2 - t1) / 1e6);
    }
    printf("{\"engine\": %d, \"out_GBs\": %.1f, \"in_GBs\": %.1f}\n", e, best_out, best_in);
  }
  // check the bytes
  CK(hipMemset(d, 7, N));
  CK(hipDeviceSynchronize());
  sdma(engine);
  sdma_wait();
  size_t bad = 0;
  for (size_t i = 0; i < N; i += 4093) bad += ((uint8_t *)h)[i] != 7;
  printf("{\"sdma_bytes_ok\": %s}\n", bad ? "false" : "true");
  return 0;
}
