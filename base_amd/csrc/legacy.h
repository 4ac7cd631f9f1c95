// v1 (legacy) record decode shared by the host driver (pipeline.cpp) and the
// packed-record kernel (legacy.hip). See legacy.hip for the algorithm.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rio {

// one packed record to unpack (Unpacker.Unpack, deprecated/packer.go:214-272)
struct V1Job {
  unsigned long long off;        // its payload's offset in the device staging
  unsigned long long size;       // payload length
  unsigned long long nbufs;      // item count (the first varint, checked on the host)
  unsigned long long item_base;  // its first item slot in the batch
  unsigned long long hbytes;     // payload bytes staged: the header's bound, or all of it
  unsigned long long span_off;   // the payload's offset in the caller's span (item views)
};

// host-side record table of a v1 span (pipeline.cpp)
struct V1Rec {
  uint64_t off, first;  // span offset of the record, its first item slot
};
struct V1Unp {
  uint64_t slot, off, len;  // an unpacked record's item
};

enum V1Status : uint32_t {
  kV1Ok = 0,
  kV1ItemSize = 1,  // "failed to read size of packed item %v: %v"     a = item, b = n
  kV1Crc = 2,       // "crc check failed - corrupt packed record header" a = computed, b = stored
  kV1Offset = 3,    // "offset greater than buf size (%v > %v)"          a = end, b = max
  kV1Range = 4,     // item sizes the reference would panic slicing
  kV1More = 5,      // the header runs past the staged bytes: restage the whole record
};

struct V1Res {
  uint32_t status;
  uint32_t pad;
  unsigned long long a, b;
  unsigned long long pad2;
};

void launch_v1_unpack(const uint8_t *dstage, const V1Job *jobs, uint64_t njobs,
                      unsigned long long *item_off, unsigned long long *item_len, V1Res *res, hipStream_t st);

}  // namespace rio
