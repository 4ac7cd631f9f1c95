"""Gather by ItemLocation (batch decode of an index-selected
set of blocks). rio_scanner_gather must return, for every location, what Seek +
Scan + Get returns (scannerv2.go:348-361, 390-403): the oracle's scan gives
every item's location; an invalid location fails with the error the oracle's
Seek sets (orc_seek_get, the reference's Seek restated)."""
import random

import pytest

from conftest import oracle_has_zstd

CODECS = [[], ["flate"], ["zstd"]]


def _file(transformers, seed, n=700, max_items=37, trailer=None):
    from base_amd.recordio.writer import WriterOpts, write_file
    rng = random.Random(seed)
    recs = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 300))) * rng.choice([1, 1, 40])
            for _ in range(n)]
    return recs, write_file(recs, WriterOpts(Transformers=list(transformers), MaxItems=max_items), trailer=trailer)


def _skip(transformers, oracle):
    if transformers == ["zstd"] and not oracle_has_zstd(oracle):
        pytest.skip("zstd oracle unavailable")


@pytest.mark.gpu
@pytest.mark.parametrize("transformers", CODECS)
def test_gather_random_locations(gpu_ctx, oracle, transformers):
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import ItemLocation
    _skip(transformers, oracle)
    recs, data = _file(transformers, 11 + len(transformers), trailer=b"tail")
    ref = oracle.scan(data)
    assert ref.err == "" and ref.items == recs
    rng = random.Random(5)
    pick = [rng.randrange(len(recs)) for _ in range(300)]  # unsorted, with repeats
    locs = [ItemLocation(*ref.locations[i]) for i in pick]
    sc = gpu.NewScanner(data, ctx=gpu_ctx)
    got = sc.Gather(locs)
    assert got == [recs[i] for i in pick]
    # the scan position is untouched: a full scan after the gather is the file
    items = []
    while sc.Scan():
        items.append(sc.Get())
    assert sc.Finish() is None and items == recs


@pytest.mark.gpu
@pytest.mark.parametrize("transformers", CODECS)
def test_gather_invalid_location(gpu_ctx, oracle, transformers):
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import ItemLocation
    _skip(transformers, oracle)
    recs, data = _file(transformers, 21, n=200)
    ref = oracle.scan(data)
    b0, _ = ref.locations[50]
    bad = [ItemLocation(ref.locations[3][0], ref.locations[3][1]), ItemLocation(b0, 9999), ItemLocation(*ref.locations[60])]
    sc = gpu.NewScanner(data, ctx=gpu_ctx)
    with pytest.raises(gpu.RecordioError) as ei:
        sc.Gather(bad)
    assert ei.value.index == 1 and ei.value.items == [recs[3]]
    assert str(ei.value) == oracle.seek_get(data, b0, 9999).err
    # a location that is not a block start: the error the reference's Seek + Scan sets
    with pytest.raises(gpu.RecordioError) as ei:
        sc.Gather([ItemLocation(b0 + 100, 0)])
    want = oracle.seek_get(data, b0 + 100, 0)
    assert want.err and str(ei.value) == want.err
    sc.Finish()


@pytest.mark.gpu
def test_gather_many_batches(oracle):
    """More blocks than one span holds: the gather runs in several batches."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import ItemLocation
    recs, data = _file(["flate"], 31, n=3000, max_items=11)
    ref = oracle.scan(data)
    ctx = gpu.Context(max_span_bytes=8 * 32768)
    sc = gpu.NewScanner(data, ctx=ctx)
    idx = list(range(0, len(recs), 3))[::-1]
    assert sc.Gather([ItemLocation(*ref.locations[i]) for i in idx]) == [recs[i] for i in idx]
    sc.Finish()
    ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("transformers", CODECS)
def test_memory_reader_and_readahead(oracle, transformers):
    """rio_memory_reader (no Python on the read path) with spans much smaller
    than the file, so every span after the first comes from the read-ahead
    thread (previous span's tail + prefetched bytes); scanners in 4 threads,
    each with its own ctx. Items equal the oracle's."""
    import threading
    from base_amd.recordio import gpu
    _skip(transformers, oracle)
    recs, data = _file(transformers, 41 + len(transformers), n=2500, max_items=23)
    ref = oracle.scan(data)
    out = [None] * 4

    def work(w):
        ctx = gpu.Context(max_span_bytes=(5 + w) * 32768)
        sc = gpu.NewScanner(gpu.MemorySource(data), ctx=ctx)
        items = []
        while sc.Scan():
            items.append(sc.Get())
        out[w] = (items, sc.Finish())
        ctx.close()
    th = [threading.Thread(target=work, args=(w,)) for w in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for items, err in out:
        assert err is None and items == ref.items


@pytest.mark.gpu
@pytest.mark.parametrize("transformers", CODECS)
def test_gather_respects_shard_limit(gpu_ctx, oracle, transformers):
    """Gather on a NewShardScanner: a location in a block at or past the shard's
    limit is what Seek + Scan gives there -- ChunkScanner.Scan stops at the limit
    (chunk.go:259-262), so there is no item -- on the fast path as on the exact
    one; locations inside the shard return their items."""
    from base_amd.recordio import gpu
    from base_amd.recordio.writer import ItemLocation
    _skip(transformers, oracle)
    recs, data = _file(transformers, 51, n=900, max_items=29)
    ref = oracle.scan(data)
    sc = gpu.NewShardScanner(data, gpu.ScannerOpts(), 0, 1, 2, ctx=gpu_ctx)
    mine = []
    while sc.Scan():
        mine.append(sc.Get())
    assert sc.Err() is None and 0 < len(mine) < len(recs)
    inside = [ItemLocation(*ref.locations[i]) for i in range(0, len(mine), 7)]
    assert sc.Gather(inside) == [recs[i] for i in range(0, len(mine), 7)]
    outside = ItemLocation(*ref.locations[len(mine) + 5])
    # the exact path: Seek + Scan on a scanner of the same shard finds no item
    ex = gpu.NewShardScanner(data, gpu.ScannerOpts(), 0, 1, 2, ctx=gpu_ctx)
    ex.Seek(outside)
    assert ex.Err() is None and not ex.Scan()
    ex.Finish()
    with pytest.raises(gpu.RecordioError) as ei:
        sc.Gather(inside[:2] + [outside])
    assert ei.value.index == 2 and ei.value.items == [recs[0], recs[7]]
    assert ei.value.code == gpu.RIO_ERR_LOCATION
    sc.Finish()
