"""Two contexts in flight over one device-resident C3 span (tools/bench_flate.py
--contexts): every step's output checked, and the first bad item described.

  python tools/ctx_check.py [--per-block 1024] [--replicas 83] [--steps 4] [--contexts 2]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))


def describe(bb, span, w, wl, nrec, a, per_block, span_items=900000):
    """The bad items among the span_items from item a: each one's index, block,
    and how its bytes differ from the expected record."""
    import torch
    import devcheck
    off, ln, in_rec, rec = devcheck.batch_tensors(bb, span.device)
    z = min(a + span_items, int(ln.numel()), (a // nrec + 1) * nrec)
    got = devcheck.gather_items(span, rec, off[a:z], ln[a:z], in_rec[a:z])
    i1 = a % nrec
    wstart = torch.cumsum(wl, 0) - wl
    w0 = int(wstart[i1])
    exp = w[w0:w0 + got.numel()]
    ne = (got != exp).nonzero().flatten()
    if ne.numel() == 0:
        return {"ndiff": 0}
    starts = torch.cumsum(ln[a:z], 0) - ln[a:z]
    items = torch.searchsorted(starts, ne, right=True) - 1
    bad_items = torch.unique(items).tolist()
    first = ne[0].item()
    it = bad_items[0]
    s0 = int(starts[it])
    gb = got.cpu().numpy().tobytes()
    eb = exp.cpu().numpy().tobytes()
    st = starts.cpu().tolist()

    def rid(buf, k):
        x = buf[st[k]:st[k] + 12]
        return x[:x.find(b"\n")].decode(errors="replace") if b"\n" in x else x.hex()
    ids = {k: (rid(gb, k), rid(eb, k)) for k in (0, 1, it - 1, it, it + 1, len(st) - 1) if 0 <= k < len(st)}
    return {"ids_got_exp": ids, "ndiff": int(ne.numel()), "nbad_items": len(bad_items), "first_bad": a + it,
            "record_in_file": (a + it) % nrec, "block_in_file": ((a + it) % nrec) // per_block,
            "bad_items_rel": bad_items[:16], "first_byte_in_item": first - s0, "item_len": int(ln[a + it]),
            "in_records": bool(in_rec[a + it]), "off": int(off[a + it]),
            "got": got[first:first + 32].cpu().numpy().tobytes().hex(),
            "exp": exp[first:first + 32].cpu().numpy().tobytes().hex()}


def block_report(bb, nrec, per_block, device):
    """Per block of an item-end batch: the record id its decoded bytes start with
    (region + header end) against the expected one; the first mismatching blocks."""
    import torch
    import devcheck
    nb = int(bb.n_blocks)
    data = devcheck.dev_copy(devcheck._ptr(bb.block_data), 8 * nb, device, torch.int64)
    foff = devcheck.dev_copy(devcheck._ptr(bb.block_first_off), 8 * nb, device, torch.int64)
    first = devcheck.dev_copy(devcheck._ptr(bb.block_first_item), 8 * (nb + 1), device, torch.int64)
    rec = devcheck.dev_copy(bb.records, int(bb.records_len), device)
    D = data & ((1 << 63) - 1)
    pos = (D + foff)[:, None] + torch.arange(12, device=device)[None, :]
    heads = rec[pos.clamp(max=rec.numel() - 1)].cpu().numpy()
    per_rep = -(-nrec // per_block)
    bad = []
    for b in range(nb):
        h = heads[b].tobytes()
        got = h[2:h.find(b"\n")] if b"\n" in h else h
        want = str((b % per_rep) * per_block).encode()
        if got != want:
            bad.append((b, got.decode(errors="replace"), want.decode(), int(D[b]), int(foff[b]), int(first[b])))
    return {"nbad_blocks": len(bad), "first_bad_blocks": bad[:8],
            "dec_off_sorted": bool((D[1:] >= D[:-1]).all().item())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-block", type=int, default=1024)
    ap.add_argument("--replicas", type=int, default=83)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--contexts", type=int, default=2)
    ap.add_argument("--serial", action="store_true", help="collect each part before launching the next")
    ap.add_argument("--reverse", action="store_true", help="launch the parts last first")
    args = ap.parse_args()
    import torch
    import c3_data
    import devcheck
    from base_amd.recordio import gpu

    data, nrec, _ = c3_data.make_file(128 << 20, args.per_block, workers=16)
    want = []
    for first in range(0, nrec, args.per_block):
        want.extend(c3_data.records(first, min(args.per_block, nrec - first)))
    CH = 32768
    body = data[CH:]
    R = args.replicas
    dev = torch.empty(CH + R * len(body), dtype=torch.uint8, device="cuda:0")
    dev[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    for r in range(1, R):
        dev[CH + r * len(body):CH + (r + 1) * len(body)].copy_(dev[CH:len(data)])
    torch.cuda.synchronize()
    n = max(1, min(args.contexts, R))
    cuts = [R * k // n for k in range(n + 1)]
    parts = [(CH + a * len(body), (z - a) * len(body), z - a) for a, z in zip(cuts[:-1], cuts[1:])]
    ctxs = [gpu.Context(0, max_span_bytes=m + CH, max_items=nrec * r + 1024, item_end=True) for _, m, r in parts]
    w, wl = devcheck.records_tensors(want, dev.device)
    w_host = w.cpu()
    base = dev.data_ptr()
    bad = 0
    for s in range(args.steps):
        if args.serial:
            bbs = []
            for c, (o, m, _) in zip(ctxs, parts):
                c.scan_device_async(base + o, m, o, gpu.RIO_CODEC_FLATE)
                bbs.append(c.sync())
        else:
            order = list(range(len(ctxs)))[::-1] if args.reverse else list(range(len(ctxs)))
            for k in order:
                o, m, _ = parts[k]
                ctxs[k].scan_device_async(base + o, m, o, gpu.RIO_CODEC_FLATE)
            bbs = [None] * len(ctxs)
            for k in order:
                bbs[k] = ctxs[k].sync()
        torch.cuda.synchronize()
        wc = w.cpu()
        ch = (wc != w_host).nonzero().flatten()
        if ch.numel():  # the expected records' own device copy changed under the step
            print(json.dumps({"step": s, "expected_tensor_changed_bytes": int(ch.numel()), "first": int(ch[0]),
                              "last": int(ch[-1]), "w_ptr": w.data_ptr(),
                              "ctx_dec": [c.debug_ptrs() if hasattr(c, "debug_ptrs") else None for c in ctxs]}),
                  flush=True)
            w.copy_(w_host.to(w.device))
        for k, (bb, (o, m, r)) in enumerate(zip(bbs, parts)):
            rep = {"step": s, "part": k, "stop": int(bb.stop), "err": int(bb.err.code), "n_items": int(bb.n_items),
                   "want_items": nrec * r, "n_blocks": int(bb.n_blocks)}
            chk = devcheck.check_replicated(bb, dev[o:o + m], w, wl, r)
            rep["blocks"] = block_report(bb, nrec, args.per_block, dev.device)
            rep.update(chk)
            if not chk["ok"]:
                bad += 1
                fb = chk["first_bad_item"]
                if fb is not None and fb >= 0:  # the first bad item's block and bytes
                    rep["bad_detail"] = describe(bb, dev[o:o + m], w, wl, nrec, fb, args.per_block)
            print(json.dumps(rep), flush=True)
    print(json.dumps({"bad_parts": bad}), flush=True)


if __name__ == "__main__":
    main()
