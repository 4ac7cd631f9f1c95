"""Which engine runs a host<->device copy (SDMA, or a blit kernel on the
stream's queue) when copies of several streams are in flight at once, as in the
scanner's spans ahead: run under `rocprofv3 --kernel-trace --memory-copy-trace`
(SDMA copies show as memory copies, blit copies as __amd_rocclr_copyBuffer
kernels). Prints each case's wall rate as one JSON line."""
import ctypes
import json
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
N = 512 << 20
H2D, D2H = 1, 2


def ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


def main():
    torch.cuda.init()
    streams = []
    for _ in range(3):
        s = ctypes.c_void_p()
        ok(hip.hipStreamCreateWithFlags(ctypes.byref(s), 1), "stream")
        streams.append(s)
    dev, host = [], []
    for _ in range(3):
        d, h = ctypes.c_void_p(), ctypes.c_void_p()
        ok(hip.hipMalloc(ctypes.byref(d), ctypes.c_size_t(N)), "malloc")
        ok(hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(N), 0), "hostmalloc")
        ctypes.memset(h, 1, N)
        dev.append(d)
        host.append(h)

    def copy(i, kind):
        src, dst = (host[i], dev[i]) if kind == H2D else (dev[i], host[i])
        ok(hip.hipMemcpyAsync(dst, src, ctypes.c_size_t(N), kind, streams[i]), "copy")

    def sync():
        for s in streams:
            ok(hip.hipStreamSynchronize(s), "sync")

    cases = {
        "d2h_alone": [(0, D2H)],
        "d2h_then_h2d_other_stream": [(0, D2H), (1, H2D)],
        "d2h_then_two_h2d": [(0, D2H), (1, H2D), (2, H2D)],
        "two_d2h": [(0, D2H), (1, D2H)],
        "fill_then_d2h_then_h2d_other": [("fill", 0), (0, D2H), (1, H2D)],
    }
    res = {}
    for name, ops in cases.items():
        sync()
        time.sleep(0.05)
        t0 = time.perf_counter()
        nbytes = 0
        for a, b in ops:
            if a == "fill":  # a kernel pending on stream b ahead of its copy
                for _ in range(20):
                    ok(hip.hipMemsetAsync(dev[b], 0, ctypes.c_size_t(N), streams[b]), "fill")
                continue
            copy(a, b)
            nbytes += N
        sync()
        res[name] = round(nbytes / (time.perf_counter() - t0) / 1e9, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
