"""Host<->device copy rates by pinned-allocation flavour: hipHostMalloc with each
flag the scan path could use, torch's pin_memory, and the GPU's NUMA node, so the
e2e scan's copy rate (pipeline.cpp collect / scan_span) can be compared with what
the link gives. Prints one JSON line."""
import ctypes
import glob
import json
import os

import torch

hip = ctypes.CDLL("libamdhip64.so")
N = 1 << 30
REPS = 4
H2D, D2H = 1, 2


def ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: hip error {rc}")


def numa():
    out = {"nodes": len(glob.glob("/sys/devices/system/node/node[0-9]*"))}
    for p in glob.glob("/sys/class/drm/card*/device/numa_node"):
        try:
            out[p.split("/")[4]] = int(open(p).read())
        except OSError:
            pass
    return out


def rate(host, dev, kind, st, fill=0, cst=None, n=N):
    e0, e1 = ctypes.c_void_p(), ctypes.c_void_p()
    ok(hip.hipEventCreate(ctypes.byref(e0)), "event")
    ok(hip.hipEventCreate(ctypes.byref(e1)), "event")
    ev = ctypes.c_void_p()
    ok(hip.hipEventCreateWithFlags(ctypes.byref(ev), 2), "event")
    src, dst = (host, dev) if kind == H2D else (dev, host)
    ok(hip.hipMemcpyAsync(dst, src, ctypes.c_size_t(n), kind, st), "copy")
    ok(hip.hipEventRecord(e0, st), "rec")
    for _ in range(REPS):
        for _ in range(fill):  # kernels just before the copy, as the scan has
            ok(hip.hipMemsetAsync(dev, 0, ctypes.c_size_t(N), st), "fill")
        if cst is not None:  # the copy on its own stream, ordered by an event
            ok(hip.hipEventRecord(ev, st), "rec")
            ok(hip.hipStreamWaitEvent(cst, ev, 0), "wait")
            ok(hip.hipMemcpyAsync(dst, src, ctypes.c_size_t(n), kind, cst), "copy")
            ok(hip.hipEventRecord(ev, cst), "rec")
            ok(hip.hipStreamWaitEvent(st, ev, 0), "wait")
            continue
        ok(hip.hipMemcpyAsync(dst, src, ctypes.c_size_t(n), kind, st), "copy")
    ok(hip.hipEventRecord(e1, st), "rec")
    ok(hip.hipEventSynchronize(e1), "sync")
    ms = ctypes.c_float()
    ok(hip.hipEventElapsedTime(ctypes.byref(ms), e0, e1), "elapsed")
    return round(n * REPS / (ms.value / 1e3) / 1e9, 1)


def main():
    torch.cuda.init()
    dev = ctypes.c_void_p()
    ok(hip.hipMalloc(ctypes.byref(dev), ctypes.c_size_t(N)), "malloc")
    st = ctypes.c_void_p()
    ok(hip.hipStreamCreateWithFlags(ctypes.byref(st), 1), "stream")
    res = {"numa": numa()}
    flags = {"default": 0, "portable": 1, "coherent": 0x40000000, "noncoherent": 0x80000000,
             "numa_user": 0x20000000}
    for name, f in flags.items():
        h = ctypes.c_void_p()
        if hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(N), ctypes.c_uint(f)) != 0:
            res[name] = "alloc failed"
            continue
        ctypes.memset(h, 1, N)
        res[name] = {"h2d": rate(h, dev, H2D, st), "d2h": rate(h, dev, D2H, st)}
        ok(hip.hipHostFree(h), "free")
    t = torch.empty(N, dtype=torch.uint8).pin_memory()
    p = ctypes.c_void_p(t.data_ptr())
    res["torch_pin"] = {"h2d": rate(p, dev, H2D, st), "d2h": rate(p, dev, D2H, st)}
    res["after_kernel"] = {"h2d": rate(p, dev, H2D, st, 1), "d2h": rate(p, dev, D2H, st, 1)}
    res["after_40_kernels"] = {"h2d": rate(p, dev, H2D, st, 40), "d2h": rate(p, dev, D2H, st, 40)}
    # after the host heap has churned (the e2e bench builds GBs of files first):
    # pinned buffers whose pages are scattered rather than contiguous
    import numpy as np
    keep, junk = [], []
    for i in range(48):
        (keep if i % 2 else junk).append(np.ones(128 << 20, np.uint8))
    del junk
    for name, size in (("churned_1g", N), ("churned_360m", 360 << 20)):
        h = ctypes.c_void_p()
        ok(hip.hipHostMalloc(ctypes.byref(h), ctypes.c_size_t(N), ctypes.c_uint(0)), "alloc")
        ctypes.memset(h, 1, N)
        res[name] = {"h2d": rate(h, dev, H2D, st, n=size), "d2h": rate(h, dev, D2H, st, n=size)}
        ok(hip.hipHostFree(h), "free")
    del keep
    # while 16 host threads copy memory (the scanner's range readers do)
    import threading
    stop = threading.Event()
    bufs = [(np.ones(64 << 20, np.uint8), np.empty(64 << 20, np.uint8)) for _ in range(16)]
    done = [0]

    def churn(a, b):
        while not stop.is_set():
            np.copyto(b, a)
            done[0] += 1
    ths = [threading.Thread(target=churn, args=ab) for ab in bufs]
    for t_ in ths:
        t_.start()
    import time
    t1 = time.perf_counter()
    res["under_host_copies"] = {"h2d": rate(p, dev, H2D, st), "d2h": rate(p, dev, D2H, st)}
    dt = time.perf_counter() - t1
    stop.set()
    for t_ in ths:
        t_.join()
    res["under_host_copies"]["host_GBs"] = round(done[0] * (64 << 20) / dt / 1e9, 1)
    cst = ctypes.c_void_p()
    ok(hip.hipStreamCreateWithFlags(ctypes.byref(cst), 1), "stream")
    res["copy_stream_after_40"] = {"h2d": rate(p, dev, H2D, st, 40, cst), "d2h": rate(p, dev, D2H, st, 40, cst)}
    res["env"] = {k: v for k, v in os.environ.items() if k.startswith(("GPU_", "HSA_", "ROC_", "DEBUG_CLR"))}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
