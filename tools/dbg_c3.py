"""Development aid: C3 flate file through the device path, item-by-item
against the generator (first mismatching block / item / byte)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

import c3_data  # noqa: E402
from base_amd.recordio import gpu  # noqa: E402


def main():
    mib = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    per = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    data, nrec, _ = c3_data.make_file(mib << 20, per, workers=8)
    CH = 32768
    body = data[CH:]
    dev = torch.frombuffer(bytearray(body), dtype=torch.uint8).cuda()
    ctx = gpu.Context(0, max_span_bytes=len(body) + CH)
    b = ctx.scan_device(dev.data_ptr(), len(body), file_off=CH, is_file_end=True, codec=gpu.RIO_CODEC_FLATE)
    print("stop", b.stop, "err", b.err.code, b.err.msg, "n_items", b.n_items, "nrec", nrec, flush=True)
    items = gpu.device_batch_items(b, body)
    want = []
    for first in range(0, nrec, per):
        want.extend(c3_data.records(first, min(per, nrec - first)))
    bad = [i for i in range(min(len(items), len(want))) if items[i] != want[i]]
    print("mismatching items", len(bad), "of", len(want), flush=True)
    blocks = sorted(set(i // per for i in bad))
    print("bad blocks", blocks[:40], len(blocks))
    for i in bad[:5]:
        a, w = items[i], want[i]
        j = next((k for k in range(min(len(a), len(w))) if a[k] != w[k]), None)
        print(" item", i, "block", i // per, "lens", len(a), len(w), "first diff byte", j,
              "got", a[max(0, (j or 0) - 4):(j or 0) + 8], "want", w[max(0, (j or 0) - 4):(j or 0) + 8])


if __name__ == "__main__":
    main()
