"""GPU flate decoder stress parity (pytest -m gpu): the two-pass decoder
(k_flate_tok / k_flate_lz) on inputs chosen for its edge paths,
bit-exact against the records the writer compressed and, for corrupt streams,
against the CPU oracle's error text (recordioflate.go:54-65 semantics)."""
import os
import random

import pytest

from conftest import golden_bytes  # noqa: F401  (conftest puts the repo on sys.path)

pytestmark = pytest.mark.gpu


def make_ctx(env=None, span=64 << 20):
    """A ctx with the flate decoder's test parameters (rio_config.flate_tok_limit,
    flate_grid, RIO_CFG_FLATE_ONE_WAVE) from `env` = {"tok_limit": n, "grid": n,
    "one_wave": bool}."""
    from base_amd.recordio import gpu
    env = env or {}
    return gpu.Context(0, max_span_bytes=span, flate_tok_limit=env.get("tok_limit", 0),
                       flate_grid=env.get("grid", 0), flate_one_wave=env.get("one_wave", False))


def scan_all(data, ctx):
    from base_amd.recordio import gpu
    sc = gpu.NewScanner(data, ctx=ctx)
    items = []
    while sc.Scan():
        items.append(sc.Get())
    err = sc.Err()
    sc.Finish()
    return items, ("" if err is None else str(err))


def write(recs, level=-1, style="go", max_items=0):
    from base_amd.recordio.writer import write_file, WriterOpts
    spec = "flate" if level < 0 else "flate %d" % level
    return write_file(recs, WriterOpts(Transformers=[spec], MaxItems=max_items, FlateStyle=style))


def mixed_records(seed, n):
    rng = random.Random(seed)
    words = [bytes(rng.choice(b"ACGTN@+\n") for _ in range(rng.randrange(1, 12))) for _ in range(200)]
    out = []
    for i in range(n):
        k = rng.random()
        if k < 0.3:
            out.append(bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 400))))
        elif k < 0.9:
            out.append(b"".join(rng.choice(words) for _ in range(rng.randrange(0, 80))))
        else:
            out.append(bytes([rng.randrange(256)]) * rng.randrange(0, 3000))
    return out


@pytest.fixture(scope="module", params=[False, True], ids=["default", "one_wave"])
def ctx(gpu_lib, request):
    """Both Huffman-pass variants: the tests' small spans take the 4-wave
    k_flate_sync by default; one_wave forces the one-wave kernel that large
    spans (the C3 bench's) run."""
    c = make_ctx({"one_wave": request.param})
    yield c
    c.close()


@pytest.mark.parametrize("level", [0, 1, 6, 9])
@pytest.mark.parametrize("style", ["go", "zlib"])
def test_levels_and_styles(ctx, level, style):
    recs = mixed_records(level * 7 + len(style), 600)
    items, err = scan_all(write(recs, level, style, max_items=97), ctx)
    assert err == "" and items == recs


def test_long_runs_split_batches(ctx):
    # 258-byte matches at distance 1 and 2: 64-token batches span > 16 KiB
    recs = [b"\0" * 300000, b"ab" * 150000, b"x" + b"yz" * 70000, b"q" * 5]
    items, err = scan_all(write(recs), ctx)
    assert err == "" and items == recs


def test_distance_32k(ctx):
    rng = random.Random(5)
    a = bytes(rng.getrandbits(8) for _ in range(32760))
    b = bytes(rng.getrandbits(8) for _ in range(32768))
    recs = [a + a + a[:1000], b + b[:4000], a[:100] + b + a[:100]]
    items, err = scan_all(write(recs, 9), ctx)
    assert err == "" and items == recs


def test_stored_blocks(ctx):
    rng = random.Random(6)
    recs = [bytes(rng.getrandbits(8) for _ in range(n)) for n in (0, 1, 65535, 65536, 200000, 3)]
    items, err = scan_all(write(recs, 0), ctx)
    assert err == "" and items == recs


def test_many_blocks_per_stream(gpu_lib):
    # 2 Huffman-pass waves = 16 streams for ~700 blocks: every stream decodes
    # dozens of blocks (state carried from block to block must be reset)
    recs = mixed_records(11, 700)
    data = write(recs, 6, "go", max_items=1)
    c = make_ctx({"grid": 2})
    try:
        items, err = scan_all(data, c)
    finally:
        c.close()
    assert err == "" and items == recs


@pytest.mark.parametrize("cap", [128, 300, 2000])
def test_token_region_yield_and_resume(gpu_lib, cap):
    # a small token region per round: blocks yield and resume across rounds;
    # at 128 tokens a block needs more than the 6 launched rounds and the host
    # retries with more
    recs = mixed_records(cap, 300)
    data = write(recs, 6, "go", max_items=49)  # 50 records per block
    c = make_ctx({"tok_limit": cap})
    try:
        items, err = scan_all(data, c)
    finally:
        c.close()
    assert err == "" and items == recs


def test_c3_like_fastq(ctx):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import c3_data
    data, nrec, _ = c3_data.make_file(3 << 20, 1024, workers=4)
    items, err = scan_all(data, ctx)
    want = []
    for first in range(0, nrec, 1024):
        want.extend(c3_data.records(first, min(1024, nrec - first)))
    assert err == "" and items == want


def test_rounds_exhausted_is_a_capacity_error(gpu_lib):
    # more rounds than the host will ever launch (64): a capacity error, never
    # a decode error or garbled records
    rng = random.Random(3)
    recs = [bytes(rng.getrandbits(8) for _ in range(30000))]  # stored: ~10k tokens
    data = write(recs, 6, "go")
    c = make_ctx({"tok_limit": 64})
    try:
        items, err = scan_all(data, c)
    finally:
        c.close()
    assert items == [] and "capacity" in err


def test_corrupt_streams_match_oracle(ctx, oracle):
    # corrupt compressed bytes (the chunk CRC is computed over them, so only
    # the inflater can notice): error text and items before it as the oracle
    from base_amd.recordio import format as F
    from base_amd.recordio.codecs import flate_compress
    rng = random.Random(9)
    checked = 0
    for trial in range(40):
        recs = mixed_records(100 + trial, 40)
        payload = F.packed_block_payload(recs)
        comp = bytearray(flate_compress(payload, rng.choice([1, 6, 9]), rng.choice(["go", "zlib"])))
        for _ in range(rng.randrange(1, 4)):
            i = rng.randrange(len(comp))
            comp[i] ^= 1 << rng.randrange(8)
        if rng.random() < 0.3:
            del comp[rng.randrange(len(comp)):]
        hdr = F.chunk_block(F.MAGIC_HEADER, F.packed_block_payload([F.marshal_header([("transformer", "flate")])]))
        good = F.chunk_block(F.MAGIC_PACKED, flate_compress(F.packed_block_payload(recs[:5]), 6, "go"))
        data = hdr + good + F.chunk_block(F.MAGIC_PACKED, bytes(comp))
        items, err = scan_all(data, ctx)
        ref = oracle.scan(data)
        assert err == ref.err, (trial, err, ref.err)
        assert items == ref.items
        checked += err != ""
    assert checked > 10
