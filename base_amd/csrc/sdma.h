// SDMA copies of host spans and host results (sdma.cpp).
#pragma once
#include <stdint.h>

namespace rio {

struct Sdma;
enum { kSdmaOut = 0, kSdmaIn = 1 };  // device -> host, host -> device

// engines and completion signals for one context (dev_ptr: any allocation on
// its device); nullptr when the HSA runtime offers no SDMA engine
Sdma *sdma_open(const void *dev_ptr);
void sdma_close(Sdma *s);
// n bytes on the direction's engine: 0 issued, -1 not (pageable host memory,
// no engine): the caller then copies another way
int sdma_copy(Sdma *s, void *dst, const void *src, uint64_t n, int dir);
// every copy of the direction issued so far has completed (0), or -1
int sdma_wait(Sdma *s, int dir);
// the HSA runtime knows the allocation (device, or pinned host memory)
bool sdma_known(const void *p);

}  // namespace rio
