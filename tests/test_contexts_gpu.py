"""Contexts in flight together on one GPU (a scanner's consecutive spans, or two
scanners): each context's results must be exactly what it gives alone.

Regression: k_parse_slow once ranked a group's slow-header blocks by a ballot
of their statuses, which the team's other workgroups rewrite as they finish
them; alone on the GPU a team's four workgroups start together, but with a
second context's kernels resident they are dispatched apart, the late ones
ranked a shrunken set and ~25 % of the blocks kept k_parse's status with no
items written (tools/ctx_check.py, DESIGN.md "Contexts in flight"). The C3
shape (1,024 records per block, headers past the 1 KiB fast window) sends
every block to k_parse_slow.
"""
import os
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "tools"))

CH = 32768


@pytest.mark.parametrize("nctx", [2, 3])
def test_contexts_in_flight_match_alone(nctx):
    import torch
    import c3_data
    import devcheck
    from base_amd.recordio import gpu

    data, nrec, _ = c3_data.make_file(32 << 20, 1024, workers=8)
    want = []
    for first in range(0, nrec, 1024):
        want.extend(c3_data.records(first, min(1024, nrec - first)))
    body = data[CH:]
    R = 48  # ~4,900 blocks per context: a k_parse_slow grid of many teams
    dev = torch.empty(CH + R * len(body), dtype=torch.uint8, device="cuda:0")
    dev[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    for r in range(1, R):
        dev[CH + r * len(body):CH + (r + 1) * len(body)].copy_(dev[CH:len(data)])
    torch.cuda.synchronize()
    cuts = [R * k // nctx for k in range(nctx + 1)]
    parts = [(CH + a * len(body), (z - a) * len(body), z - a) for a, z in zip(cuts[:-1], cuts[1:])]
    ctxs = [gpu.Context(0, max_span_bytes=m + CH, max_items=nrec * r + 1024, item_end=True) for _, m, r in parts]
    w, wl = devcheck.records_tensors(want, dev.device)
    base = dev.data_ptr()
    try:
        for step in range(3):
            for c, (o, m, _) in zip(ctxs, parts):
                c.scan_device_async(base + o, m, o, gpu.RIO_CODEC_FLATE)
            for k, (c, (o, m, r)) in enumerate(zip(ctxs, parts)):
                b = c.sync()
                assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
                chk = devcheck.check_replicated(b, dev[o:o + m], w, wl, r)
                assert chk["ok"], (step, k, chk)
    finally:
        for c in ctxs:
            c.close()
