"""Device-side parity checks of a device batch (rio_scan_device / _async +
rio_sync results) against expected records, for bench.py and the -m gpu tests.

Every record of the batch is gathered on the GPU (torch index ops over copies
of the batch's item views and records buffer) and compared byte for byte with
the expected records, which are uploaded once: a replicated span of R copies
is checked replica by replica against the same expected set. Test and bench
tooling only -- the product path is the C ABI.
"""
from __future__ import annotations

import ctypes

import torch

ITEM_IN_RECORDS = 1 << 63


def dev_copy(ptr: int, nbytes: int, device, dtype=torch.uint8) -> torch.Tensor:
    """A new tensor holding a copy of nbytes of device memory at ptr."""
    from base_amd.recordio import gpu
    el = torch.empty((), dtype=dtype).element_size()
    t = torch.empty(max(nbytes // el, 1), dtype=dtype, device=device)
    if nbytes:
        torch.cuda.synchronize(device)
        rc = gpu._hip().hipMemcpy(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes),
                                  3)  # hipMemcpyDeviceToDevice
        if rc != 0:
            raise RuntimeError(f"hipMemcpy D2D failed: {rc}")
    return t[:nbytes // el]


def _ptr(p):
    return ctypes.cast(p, ctypes.c_void_p).value


def item_end_tensors(b, device):
    """(off, length, in_records) of an item-end batch (RIO_CFG_ITEM_END), by the
    consumer rule of include/rio_gpu.h, computed on the device."""
    n, nb = int(b.n_items), int(b.n_blocks)
    end = dev_copy(_ptr(b.item_end), 8 * n, device, torch.int64)
    first = dev_copy(_ptr(b.block_first_item), 8 * (nb + 1), device, torch.int64)
    data = dev_copy(_ptr(b.block_data), 8 * nb, device, torch.int64)
    foff = dev_copy(_ptr(b.block_first_off), 8 * nb, device, torch.int64)
    counts = first[1:] - first[:-1]
    blk = torch.repeat_interleave(torch.arange(nb, device=device), counts, output_size=n)
    prev = torch.zeros_like(end)
    prev[1:] = end[:-1]
    prev[first[:-1][counts > 0]] = 0  # each block's first item starts at the header's end
    s = foff[blk] + prev
    e = foff[blk] + end
    rec_blk = data[blk] < 0  # bit 63
    D = data[blk] & ((1 << 63) - 1)
    k = torch.div(s, 32740, rounding_mode="floor")
    chunked = D + k * 32768 + 28 + (s - k * 32740)
    cross = (~rec_blk) & (e > s) & (torch.div(e - 1, 32740, rounding_mode="floor") != k)
    off = torch.where(rec_blk, D + s, chunked)
    return off, e - s, rec_blk | cross


def batch_tensors(b, device):
    """(off int64, length int64, in_records bool, records uint8) of a device batch."""
    n = int(b.n_items)
    if b.item_end:
        off, ln, in_rec = item_end_tensors(b, device)
    else:
        raw = dev_copy(_ptr(b.item_off), 8 * n, device, torch.int64)
        ln = dev_copy(_ptr(b.item_len), 8 * n, device, torch.int64)
        in_rec = raw < 0  # bit 63
        off = raw & ((1 << 63) - 1)
    rec = dev_copy(b.records, int(b.records_len), device) if b.records_len else torch.zeros(1, dtype=torch.uint8,
                                                                                             device=device)
    return off, ln, in_rec, rec


def gather_items(span: torch.Tensor, rec: torch.Tensor, off, ln, in_rec) -> torch.Tensor:
    """The concatenated bytes of items (off, ln, in_rec) -- views into span or,
    flagged, into the records buffer."""
    total = int(ln.sum().item())
    if total == 0:
        return torch.zeros(0, dtype=torch.uint8, device=span.device)
    starts = torch.cumsum(ln, 0) - ln
    item = torch.repeat_interleave(torch.arange(ln.numel(), device=span.device), ln, output_size=total)
    pos = torch.arange(total, device=span.device, dtype=torch.int64) - starts[item] + off[item]
    r = in_rec[item]
    out = torch.empty(total, dtype=torch.uint8, device=span.device)
    if bool((~r).any()):
        out[~r] = span[pos[~r]]
    if bool(r.any()):
        out[r] = rec[pos[r]]
    return out


def check_replicated(b, span: torch.Tensor, want: torch.Tensor, want_len: torch.Tensor, replicas: int,
                     max_bytes: int = 256 << 20) -> dict:
    """Every item of a batch over `replicas` copies of one file body against the
    expected records: `want` = their bytes back to back (uint8, on the device),
    `want_len` = their lengths (int64, on the device). Returns a summary dict
    with "ok" (bool), items and bytes checked, and the first bad item."""
    n1 = int(want_len.numel())
    res = {"ok": False, "items_checked": 0, "bytes_checked": 0, "first_bad_item": None}
    if int(b.n_items) != n1 * replicas:
        res["first_bad_item"] = -1
        return res
    off, ln, in_rec, rec = batch_tensors(b, span.device)
    if not torch.equal(ln.view(replicas, n1), want_len.expand(replicas, n1)):
        bad = (ln.view(replicas, n1) != want_len).flatten().nonzero()
        res["first_bad_item"] = int(bad[0].item())
        return res
    wstart = torch.cumsum(want_len, 0) - want_len
    # item ranges of at most max_bytes each within one replica
    cuts = [0]
    cum = torch.cumsum(want_len, 0).cpu()
    while cuts[-1] < n1:
        base = int(cum[cuts[-1] - 1]) if cuts[-1] else 0
        k = int(torch.searchsorted(cum, base + max_bytes, right=True))
        cuts.append(max(k, cuts[-1] + 1) if k < n1 else n1)
    for r in range(replicas):
        for lo, hi in zip(cuts[:-1], cuts[1:]):
            a, z = r * n1 + lo, r * n1 + hi
            got = gather_items(span, rec, off[a:z], ln[a:z], in_rec[a:z])
            w0 = int(wstart[lo])
            exp = want[w0:w0 + got.numel()]
            if not torch.equal(got, exp):
                res["first_bad_item"] = a
                return res
            res["items_checked"] += hi - lo
            res["bytes_checked"] += got.numel()
    res["ok"] = True
    return res


def records_tensors(records, device):
    """Expected records (a list of bytes, or an (n, L) uint8 numpy array) as
    (bytes back to back, lengths) tensors on the device."""
    import numpy as np
    if isinstance(records, np.ndarray):
        n, L = records.shape
        return (torch.from_numpy(np.ascontiguousarray(records).reshape(-1)).to(device),
                torch.full((n,), L, dtype=torch.int64, device=device))
    blob = b"".join(records)
    w = torch.frombuffer(bytearray(blob), dtype=torch.uint8) if blob else torch.zeros(0, dtype=torch.uint8)
    return w.to(device), torch.tensor([len(x) for x in records], dtype=torch.int64, device=device)
