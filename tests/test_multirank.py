"""The N>1 path on CPU: two ranks over gloo (world_size 2), each decoding its own
shard of one file, the ordered-output prefix exchanged by all_gather. The
per-rank decode here is the oracle (the checker, standing in for the GPU scanner
that the same code calls on an MI355X); what is under test is the shard plan,
the collective and the file-order reassembly."""
import os
import random
import socket

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, data, k, q, on_gpu=False):
    import sys
    sys.path.insert(0, ROOT)
    if on_gpu:
        import torch  # noqa: F401  (one HIP runtime for torch and librio_gpu.so)
    import torch.distributed as dist
    from base_amd.recordio import shard
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        if on_gpu:  # the default path: gpu.NewShardScanner on this rank's device (both on 0 here)
            recs, off, total = shard.scan_rank(data, rank, world, k, device=0)
        else:
            from oracle import oracle as O

            def scan(d, s, l, n):
                r = O.scan(d, s, l, n)
                assert r.err == "", r.err
                return r.items
            recs, off, total = shard.scan_rank(data, rank, world, k, scan=scan)
        q.put((rank, off, total, recs))
    finally:
        dist.destroy_process_group()


def _run_two_ranks(k, codec="", on_gpu=False):
    import torch.multiprocessing as mp
    from base_amd.recordio.writer import write_file, WriterOpts
    rng = random.Random(5 + k)
    recs = [bytes(rng.getrandbits(8) for _ in range(rng.randrange(0, 400))) for _ in range(3000)]
    data = write_file(recs, WriterOpts(MaxItems=29, Transformers=[codec] if codec else []))
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, k, q, on_gpu)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    got.sort()
    out = [None] * len(recs)
    for rank, off, total, part in got:
        assert total == len(recs)
        out[off:off + len(part)] = part
    assert out == recs
    # the ranks' shards are disjoint and non-empty at this size
    assert all(len(g[3]) > 0 for g in got)


@pytest.mark.parametrize("k", [1, 3])
def test_two_ranks_reassemble_file_order(oracle, k):
    _run_two_ranks(k)


@pytest.mark.gpu
@pytest.mark.parametrize("k,codec", [(1, ""), (3, "flate")])
def test_two_ranks_gpu_scanner(gpu_lib, k, codec):
    """shard.scan_rank's default path -- the GPU scanner -- on two gloo ranks
    sharing device 0 (the 8-GPU bench gives each rank its own)."""
    _run_two_ranks(k, codec, on_gpu=True)


def test_rank_shard_and_file_assignment():
    from base_amd.recordio import shard
    assert shard.rank_shard(0, 2) == (0, 1, 2)
    assert shard.rank_shard(3, 8, 4) == (12, 16, 32)
    with pytest.raises(ValueError):
        shard.rank_shard(2, 2)
    sizes = [64, 10, 10, 30, 30, 5, 1]
    a = shard.assign_files(sizes, 3)
    assert sorted(i for r in a for i in r) == list(range(len(sizes)))
    loads = [sum(sizes[i] for i in r) for r in a]
    assert sorted(loads, reverse=True) == [64, 45, 41]  # largest first onto the least-loaded rank


def _split_worker(rank, world, port, data, q, on_gpu=False, backend="gloo"):
    """scan_file_split on one rank: trailer index broadcast from rank 0, this
    rank's block range decoded (GPU batch, or the oracle on CPU). backend "nccl"
    (RCCL) needs on_gpu: the collectives' tensors live on cuda:0."""
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    if on_gpu:
        import torch  # noqa: F401
    import torch.distributed as dist
    import c5_data
    from base_amd.recordio import shard
    if backend == "nccl":
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                                device_id=torch.device("cuda", 0))
        assert dist.get_backend() == "nccl"
    else:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        hdr_end = int.from_bytes(data[20:24], "little") * 32768
        if on_gpu:
            from base_amd.recordio import gpu
            ctx = gpu.Context(0, max_span_bytes=len(data))

            def scan_range(lo, hi):
                b = ctx.scan_span(data[lo:hi], file_off=lo, is_file_end=True, codec=gpu.RIO_CODEC_FLATE)
                assert b.err.code == 0, b.err.msg
                return gpu.batch_items(b)
            read_trailer = None
        else:
            from oracle import oracle as O

            def scan_range(lo, hi):
                r = O.scan(data[:hdr_end] + data[lo:hi], read_trailer=False)
                assert r.err == "", r.err
                return r.items

            def read_trailer(d):
                return O.scan(d).trailer
        recs, off, total = shard.scan_file_split(data, rank, world, c5_data.parse_index, scan_range,
                                                 read_trailer=read_trailer)
        if backend == "nccl":  # the other two collectives on their own (RCCL on this rank's GPU)
            blob = bytes(range(256)) * 3 + b"index"
            assert shard.broadcast_bytes(blob if rank == 0 else None, 0) == blob
            assert shard.broadcast_bytes(b"" if rank == 0 else None, 0) == b""
            assert shard.ordered_prefix(7, 1000) == (7 * rank, 1000 * rank, 7 * world, 1000 * world)
        q.put((rank, off, total, recs))
    finally:
        dist.destroy_process_group()


def _run_split(world, on_gpu=False, backend="gloo"):
    import sys
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import c5_data
    data, nrec, _, offsets = c5_data.make_base(0, record_bytes=4 << 20, workers=4)
    want = c5_data.base_records(0, record_bytes=4 << 20)
    assert len(want) == nrec and len(offsets) == (nrec + 1023) // 1024
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, data, q, on_gpu, backend)) for r in range(world)]
    for p in procs:
        p.start()
    got = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    out = [None] * nrec
    for rank, off, total, part in got:
        assert total == nrec and len(part) > 0
        out[off:off + len(part)] = part
    assert out == want


def test_index_split_two_ranks(oracle):
    """configs[4]'s single-file case: a trailer-indexed flate file split by its
    block index over two gloo ranks (index broadcast, ordered prefix)."""
    _run_split(2)


def test_split_blocks_ranges():
    from base_amd.recordio import shard
    offs = [32768 * k for k in (1, 2, 5, 6, 7, 20)]
    end = 32768 * 25
    for world in (1, 2, 3, 7):
        rs = [shard.split_blocks(offs, end, r, world) for r in range(world)]
        assert rs[0][0] == offs[0] and rs[-1][1] == end
        for (a, b), (c, d) in zip(rs, rs[1:]):
            assert b == c  # contiguous, on block boundaries
        assert all(lo in offs + [end] for lo, _ in rs)
    assert shard.split_blocks([], end, 0, 2) == (end, end)


@pytest.mark.gpu
def test_index_split_two_ranks_gpu(gpu_lib):
    _run_split(2, on_gpu=True)


@pytest.mark.gpu
def test_index_split_rccl_world1(gpu_lib):
    """The RCCL ("nccl") branches of shard.broadcast_bytes / ordered_prefix /
    scan_file_split on the GPU box: a world-size-1 process group on cuda:0 in a
    fresh spawned process (no GPU call before its init), a C5-shaped file split by
    its trailer index and decoded on the GPU (the 8-rank run is the driver's)."""
    _run_split(1, on_gpu=True, backend="nccl")
