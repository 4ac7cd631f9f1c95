"""The exact device-resident paths the bench times, checked record by record
(pytest -m gpu).

- C2 (configs[1], the headline): rio_scan_device_async + rio_sync -- the call
  pair bench.py's timed step makes -- over the 1x C2 file body and over a
  4-replica span; every record of every replica gathered on the GPU and
  compared byte for byte with the generator's records (tools/devcheck.py); the
  generator's records are in turn the oracle's scan of the same file.
- C3 (configs[2]): the flate workload's 128 MiB base file (tools/c3_data.py,
  1,024 records per block, level-6 Go-framed raw DEFLATE) through the same
  async pair, over the 1x body and 2 replicas: every record against the
  generator; three blocks (first, middle, last) against the oracle's
  Go-semantics inflater (oracle/inflate.c via oracle.scan).
"""
import ctypes
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu
sys.path.insert(0, os.path.join(ROOT, "tools"))
CH = 32768


def _replicated(data, replicas, device="cuda:0"):
    """Header chunk + `replicas` copies of the body on the device (as bench.py lays it out)."""
    import torch
    body = data[CH:]
    dev = torch.empty(CH + replicas * len(body), dtype=torch.uint8, device=device)
    dev[:len(data)].copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    for r in range(1, replicas):
        dev[CH + r * len(body):CH + (r + 1) * len(body)].copy_(dev[CH:len(data)])
    torch.cuda.synchronize()
    return dev


def _async_scan(ctx, dev, codec):
    ctx.scan_device_async(dev.data_ptr() + CH, dev.numel() - CH, CH, codec)
    return ctx.sync()


@pytest.fixture(scope="module")
def c2():
    import bench
    data, nrec = bench.make_c2_file()
    return data, nrec, bench.c2_records()


def test_c2_generator_is_oracle(c2, oracle):
    """The generator's records are what the oracle's scan of the C2 file returns."""
    data, nrec, recs = c2
    assert len(data) == 259096576
    ref = oracle.scan(data)
    assert ref.err == "" and len(ref.items) == nrec
    assert b"".join(ref.items) == recs.tobytes()


@pytest.mark.parametrize("item_end", [True, False])
@pytest.mark.parametrize("replicas", [1, 4])
def test_c2_device_async_every_record(c2, replicas, item_end):
    """bench.py's timed call pair, in both output shapes: item_end (cumSize,
    RIO_CFG_ITEM_END, what the bench times) and item_off / item_len."""
    import devcheck
    import torch
    from base_amd.recordio import gpu
    data, nrec, recs = c2
    dev = _replicated(data, replicas)
    ctx = gpu.Context(0, max_span_bytes=dev.numel(), max_items=nrec * replicas + 1024, item_end=item_end)
    for _ in range(2):  # a second run over the same ctx (the bench's steps reuse it)
        b = _async_scan(ctx, dev, gpu.RIO_CODEC_NONE)
        assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
        assert b.n_items == nrec * replicas and b.n_blocks == 3953 * replicas
        assert bool(b.item_end) == item_end and bool(b.item_off) != item_end
        first = np.frombuffer(gpu.dev_to_host(ctypes.cast(b.block_first_item, ctypes.c_void_p).value,
                                              8 * (int(b.n_blocks) + 1)), dtype=np.uint64)
        per = np.diff(first.astype(np.int64)).reshape(replicas, 3953)  # 3,952 blocks of 253, one of 144
        assert first[0] == 0 and np.all(per[:, :-1] == 253) and np.all(per[:, -1] == 1000000 - 3952 * 253)
        want, want_len = devcheck.records_tensors(recs, dev.device)
        res = devcheck.check_replicated(b, dev[CH:], want, want_len, replicas)
        assert res["ok"], res
        assert res["items_checked"] == nrec * replicas and res["bytes_checked"] == nrec * replicas * 256
    ctx.close()
    del dev
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def c3():
    import c3_data
    data, nrec, rec_bytes = c3_data.make_file(128 << 20, 1024, workers=16)
    recs = []
    for first in range(0, nrec, 1024):
        recs.extend(c3_data.records(first, min(1024, nrec - first)))
    return data, nrec, rec_bytes, recs


@pytest.mark.parametrize("replicas,item_end", [(1, False), (2, True)])
def test_c3_base_file_device_async(c3, replicas, item_end):
    import devcheck
    import torch
    from base_amd.recordio import gpu
    data, nrec, rec_bytes, recs = c3
    assert len(recs) == nrec and sum(map(len, recs)) == rec_bytes
    dev = _replicated(data, replicas)
    ctx = gpu.Context(0, max_span_bytes=dev.numel(), max_items=nrec * replicas + 1024, item_end=item_end)
    b = _async_scan(ctx, dev, gpu.RIO_CODEC_FLATE)
    assert b.stop == gpu.RIO_STOP_EOF and b.err.code == 0, b.err.msg
    want, want_len = devcheck.records_tensors(recs, dev.device)
    res = devcheck.check_replicated(b, dev[CH:], want, want_len, replicas)
    assert res["ok"], res
    assert res["bytes_checked"] == rec_bytes * replicas
    ctx.close()
    del dev
    torch.cuda.empty_cache()


def test_c3_blocks_against_oracle(c3, oracle):
    """Blocks of the C3 base file: the GPU scanner and the oracle's inflater agree
    (and equal the generator's records)."""
    from base_amd.recordio import gpu
    data, nrec, rec_bytes, recs = c3
    hdr = data[:CH]
    pos, blocks = CH, []
    while pos < len(data):
        total = int.from_bytes(data[pos + 20:pos + 24], "little")
        blocks.append(data[pos:pos + total * CH])
        pos += total * CH
    assert len(blocks) == -(-nrec // 1024)
    for k in (0, len(blocks) // 2, len(blocks) - 1):
        ref = oracle.scan(hdr + blocks[k])
        assert ref.err == "" and ref.items == recs[k * 1024:(k + 1) * 1024]
        sc = gpu.NewScanner(hdr + blocks[k])
        got = []
        while sc.Scan():
            got.append(sc.Get())
        assert sc.Finish() is None and got == ref.items
