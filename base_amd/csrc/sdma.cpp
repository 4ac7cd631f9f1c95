// Host <-> device copies of host spans and host results on SDMA engines, through
// the HSA API (hsa_amd_memory_async_copy_on_engine with force_copy_on_sdma).
//
// Why not hipMemcpyAsync: this runtime runs large copies between device memory
// and pinned host memory as blit kernels (__amd_rocclr_copyBuffer) on a compute
// queue. A blit copy reaches ~30 GB/s and takes CUs from the decode kernels
// (on the kernels' stream it also sits between them); an SDMA engine copies at
// ~57 GB/s device -> host and leaves the CUs alone (tools/sdma_probe.cpp: a
// streaming kernel beside it 10.04 -> 10.10 ms, the copy 52 GB/s). DESIGN.md §5
// (end-to-end).
//
// Each context has an engine per direction and, per direction, completion
// signals for the copies in flight (one per copy). The callers order copies against the
// kernels on the host: a copy is issued only once the kernels it depends on
// have completed, and the kernels that depend on a copy are enqueued only after
// sdma_wait. Memory the HSA runtime does not know (pageable host memory) is not
// SDMA-copyable: sdma_copy declines it and the caller copies with hipMemcpyAsync.
#include "sdma.h"

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>

#include <atomic>
#include <chrono>

namespace rio {

// a completion signal per copy in flight (one shared signal counting several
// copies is valid HSA, but tools that wrap completion signals -- rocprofv3's
// memory-copy trace -- expect a signal per copy, value 1)
constexpr int kSdmaSlots = 16;
struct Sdma {
  hsa_agent_t gpu{}, cpu{};
  hsa_signal_t sig[2][kSdmaSlots]{};
  int used[2]{};  // signals of copies issued and not yet waited for
  hsa_amd_sdma_engine_id_t eng[2]{};
  bool hsa_up = false;
};

static hsa_status_t first_cpu(hsa_agent_t a, void *out) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t *>(out) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// the k-th set bit of m (k taken mod the bit count), as an engine id; 0 when m is 0
static uint32_t kth_bit(uint32_t m, uint32_t k) {
  const uint32_t n = (uint32_t)__builtin_popcount(m);
  if (n == 0) return 0;
  k %= n;
  for (uint32_t b = 0; b < 32; b++)
    if (m & (1u << b)) {
      if (k == 0) return 1u << b;
      k--;
    }
  return 0;
}

static std::atomic<uint32_t> g_next{0};

Sdma *sdma_open(const void *dev_ptr) {
  Sdma *s = new Sdma();
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    delete s;
    return nullptr;
  }
  s->hsa_up = true;
  hsa_amd_pointer_info_t pi{};
  pi.size = sizeof(pi);
  bool ok = hsa_amd_pointer_info(dev_ptr, &pi, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
            pi.type == HSA_EXT_POINTER_TYPE_HSA;
  if (ok) {
    s->gpu = pi.agentOwner;
    s->cpu.handle = 0;
    hsa_iterate_agents(first_cpu, &s->cpu);
    ok = s->cpu.handle != 0;
  }
  uint32_t m_out = 0, m_in = 0;
  if (ok)
    ok = hsa_amd_memory_copy_engine_status(s->cpu, s->gpu, &m_out) == HSA_STATUS_SUCCESS &&
         hsa_amd_memory_copy_engine_status(s->gpu, s->cpu, &m_in) == HSA_STATUS_SUCCESS && m_out && m_in;
  if (ok) {
    // The engines are not alike: on the MI355X box device -> host copies run at
    // 57 GB/s on engines 0-3 and at 7-13 GB/s on 4-15, host -> device at 57 GB/s
    // on all (tools/sdma_probe.cpp). The runtime's preferred engines for each
    // direction (engines 1-2 out, 0 in there) are taken, contexts taking them in
    // turn; without a preference, the free engines among 0-3.
    uint32_t p_out = 0, p_in = 0;
    if (hsa_amd_memory_get_preferred_copy_engine(s->cpu, s->gpu, &p_out) != HSA_STATUS_SUCCESS) p_out = 0;
    if (hsa_amd_memory_get_preferred_copy_engine(s->gpu, s->cpu, &p_in) != HSA_STATUS_SUCCESS) p_in = 0;
    p_out &= m_out;
    p_in &= m_in;
    if (!p_out) p_out = m_out & 0xfu;
    if (!p_in) p_in = m_in & 0xfu;
    ok = p_out && p_in;
    const uint32_t k = g_next.fetch_add(1);
    s->eng[kSdmaOut] = (hsa_amd_sdma_engine_id_t)kth_bit(p_out, k);
    s->eng[kSdmaIn] = (hsa_amd_sdma_engine_id_t)kth_bit(p_in, k);
  }
  if (ok) {
    for (int d = 0; d < 2 && ok; d++)
      for (int i = 0; i < kSdmaSlots && ok; i++)
        ok = hsa_signal_create(0, 0, nullptr, &s->sig[d][i]) == HSA_STATUS_SUCCESS;
  }
  if (!ok) {
    sdma_close(s);
    return nullptr;
  }
  return s;
}

void sdma_close(Sdma *s) {
  if (!s) return;
  for (int d = 0; d < 2; d++) {
    sdma_wait(s, d);
    for (int i = 0; i < kSdmaSlots; i++)
      if (s->sig[d][i].handle) hsa_signal_destroy(s->sig[d][i]);
  }
  if (s->hsa_up) hsa_shut_down();
  delete s;
}

bool sdma_known(const void *p) {
  hsa_amd_pointer_info_t pi{};
  pi.size = sizeof(pi);
  return hsa_amd_pointer_info(p, &pi, nullptr, nullptr, nullptr) == HSA_STATUS_SUCCESS &&
         pi.type != HSA_EXT_POINTER_TYPE_UNKNOWN;
}

int sdma_copy(Sdma *s, void *dst, const void *src, uint64_t n, int dir) {
  if (!s) return -1;
  if (n == 0) return 0;
  if (!sdma_known(dir == kSdmaOut ? dst : src)) return -1;  // pageable host memory
  if (s->used[dir] == kSdmaSlots && sdma_wait(s, dir) != 0) return -1;  // (all slots in flight: drain)
  const hsa_agent_t da = dir == kSdmaOut ? s->cpu : s->gpu, sa = dir == kSdmaOut ? s->gpu : s->cpu;
  const hsa_signal_t sg = s->sig[dir][s->used[dir]];
  hsa_signal_store_relaxed(sg, 1);
  if (hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, n, 0, nullptr, sg, s->eng[dir], true) !=
      HSA_STATUS_SUCCESS) {
    hsa_signal_store_relaxed(sg, 0);
    return -1;
  }
  s->used[dir]++;
  return 0;
}

// (a copy that never completes -- an engine fault -- ends the wait after 60 s
// with an error rather than hanging the caller)
int sdma_wait(Sdma *s, int dir) {
  if (!s) return 0;
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < s->used[dir]; i++)
    while (hsa_signal_wait_scacquire(s->sig[dir][i], HSA_SIGNAL_CONDITION_EQ, 0, 1000000000ull,
                                     HSA_WAIT_STATE_BLOCKED) != 0)
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return -1;
  s->used[dir] = 0;
  return 0;
}

}  // namespace rio
