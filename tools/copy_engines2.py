"""Which engine the runtime picks for a 512 MiB device -> pinned-host copy that
follows a kernel: on the kernel's own stream (the pipeline's collect before round
5), on a copy-only stream that waits for the kernel's event, and with the
hipMemcpyDeviceToDeviceNoCU kind. Run one case per process under
`rocprofv3 --kernel-trace --memory-copy-trace --stats`: SDMA copies show as memory
copies, blit copies as __amd_rocclr_copyBuffer kernels. Prints the case's rate.
Usage: copy_engines2.py <same|copystream|nocu|copystream_nocu>"""
import ctypes
import json
import sys
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
N = 512 << 20
D2H, NOCU = 2, 1024


def ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


def main():
    case = sys.argv[1]
    torch.cuda.init()
    st, cst = ctypes.c_void_p(), ctypes.c_void_p()
    ok(hip.hipStreamCreateWithFlags(ctypes.byref(st), 1), "stream")
    ok(hip.hipStreamCreateWithFlags(ctypes.byref(cst), 1), "copy stream")
    ev = ctypes.c_void_p()
    ok(hip.hipEventCreateWithFlags(ctypes.byref(ev), 2), "event")  # hipEventDisableTiming
    d, h = ctypes.c_void_p(), ctypes.c_void_p()
    ok(hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(N)), "malloc")
    ok(hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(N), 0), "hostmalloc")
    x = torch.empty(N // 4, dtype=torch.float32, device="cuda:0")
    tstream = torch.cuda.ExternalStream(st.value)
    rates = []
    for it in range(6):
        ok(hip.hipDeviceSynchronize(), "sync")
        t0 = time.perf_counter()
        with torch.cuda.stream(tstream):
            x.add_(1.0)  # a kernel ahead of the copy on the pipeline's stream
        if case == "same":
            ok(hip.hipMemcpyAsync(h, d, ctypes.c_size_t(N), D2H, st), "copy")
        elif case == "nocu":
            ok(hip.hipMemcpyAsync(h, d, ctypes.c_size_t(N), NOCU, st), "copy")
        else:
            ok(hip.hipEventRecord(ev, st), "record")
            ok(hip.hipStreamWaitEvent(cst, ev, 0), "wait")
            ok(hip.hipMemcpyAsync(h, d, ctypes.c_size_t(N), NOCU if case == "copystream_nocu" else D2H, cst), "copy")
        ok(hip.hipDeviceSynchronize(), "sync")
        rates.append(N / (time.perf_counter() - t0) / 1e9)
    print(json.dumps({"case": case, "GBs": [round(r, 1) for r in rates]}), flush=True)


if __name__ == "__main__":
    main()
