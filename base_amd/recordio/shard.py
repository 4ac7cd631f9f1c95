"""Multi-GPU scan: one process per GPU, independent shards.

Recordio blocks are independent (per-chunk CRC, no cross-block state), so a file
is split with the reference's own shard math -- NewShardScanner(start, limit,
nshard) -> ChunkScanner.LimitShard (recordio/scannerv2.go:211-235,
recordio/internal/chunk.go:198-236) -- with nshard = world * k and rank r taking
shards [r*k, (r+1)*k). Every rank decodes its shard on its own GPU; no record
bytes move between GPUs. The one exchange step is the ordered-output prefix: an
all_gather of (n_items, n_bytes) per rank, so each rank knows where its records
land in the file-order result. Many files (config C5) are assigned to ranks by
size-balanced greedy assignment instead.
"""
from __future__ import annotations

import heapq
from typing import Callable, List, Sequence, Tuple


def rank_shard(rank: int, world: int, k: int = 1) -> Tuple[int, int, int]:
    """(start, limit, nshard) of rank `rank` for NewShardScanner."""
    if not 0 <= rank < world or k < 1:
        raise ValueError(f"invalid rank {rank} of {world} (k={k})")
    return rank * k, (rank + 1) * k, world * k


def assign_files(sizes: Sequence[int], world: int) -> List[List[int]]:
    """Greedy size-balanced assignment of files to ranks (largest first)."""
    heap = [(0, r) for r in range(world)]
    out: List[List[int]] = [[] for _ in range(world)]
    for i in sorted(range(len(sizes)), key=lambda i: (-sizes[i], i)):
        load, r = heapq.heappop(heap)
        out[r].append(i)
        heapq.heappush(heap, (load + sizes[i], r))
    for files in out:
        files.sort()
    return out


def split_blocks(offsets: Sequence[int], body_end: int, rank: int, world: int) -> Tuple[int, int]:
    """The single-file split by a block index (the "trailer-indexed" case,
    SURVEY.md §8(e)): block file offsets `offsets` (ascending), body ending at
    `body_end` (the trailer block's offset or the file size). Rank r takes the
    blocks whose offsets fall in the r-th byte share, so every rank starts on a
    block boundary without reading chunk headers (no LimitShard peek). Returns
    the rank's byte range [lo, hi) (empty when it has no block)."""
    if not 0 <= rank < world:
        raise ValueError(f"invalid rank {rank} of {world}")
    if not offsets:
        return body_end, body_end
    base, span = offsets[0], body_end - offsets[0]

    def first_block_at(cut):  # first block whose offset >= cut
        lo, hi = 0, len(offsets)
        while lo < hi:
            mid = (lo + hi) // 2
            if offsets[mid] < cut:
                lo = mid + 1
            else:
                hi = mid
        return lo
    a = first_block_at(base + span * rank // world)
    b = first_block_at(base + span * (rank + 1) // world) if rank + 1 < world else len(offsets)
    lo = offsets[a] if a < len(offsets) else body_end
    hi = offsets[b] if b < len(offsets) else body_end
    return lo, hi


def broadcast_bytes(data, src: int = 0, group=None) -> bytes:
    """Broadcast a byte string (the trailer index) from rank `src`: its length,
    then its bytes, as uint8 tensors -- RCCL over xGMI for "nccl", gloo on CPU."""
    import torch
    import torch.distributed as dist
    dev = "cpu"
    if dist.get_backend(group) == "nccl":
        dev = f"cuda:{torch.cuda.current_device()}"
    n = torch.tensor([len(data) if data is not None else 0], dtype=torch.int64, device=dev)
    dist.broadcast(n, src, group=group)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=dev)
    if dist.get_rank(group) == src and len(buf):
        buf.copy_(torch.frombuffer(bytearray(data), dtype=torch.uint8))
    if len(buf):
        dist.broadcast(buf, src, group=group)
    return bytes(buf.cpu().numpy().tobytes())


def ordered_prefix(n_items: int, n_bytes: int, group=None):
    """All-gather (n_items, n_bytes) of every rank; returns this rank's exclusive
    (item_offset, byte_offset) and the totals. The backend's collective (RCCL over
    xGMI for "nccl", gloo on CPU) moves 16 B per rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = "cpu"
    if dist.get_backend(group) == "nccl":
        dev = f"cuda:{torch.cuda.current_device()}"
    mine = torch.tensor([n_items, n_bytes], dtype=torch.int64, device=dev)
    allv = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(allv, mine, group=group)
    vals = [tuple(int(x) for x in t.cpu().tolist()) for t in allv]
    item_off = sum(v[0] for v in vals[:rank])
    byte_off = sum(v[1] for v in vals[:rank])
    return item_off, byte_off, sum(v[0] for v in vals), sum(v[1] for v in vals)


def scan_rank(data, rank: int, world: int, k: int = 1,
              scan: Callable = None, group=None, device: int = None):
    """Decode this rank's shard of one file and place it in file order.

    scan(data, start, limit, nshard) -> list of record bytes; by default the GPU
    scanner (gpu.NewShardScanner) on `device` -- this rank's LOCAL_RANK unless
    given (several ranks may share one device, e.g. tests). Returns (records,
    item_offset, total_items)."""
    start, limit, nshard = rank_shard(rank, world, k)
    if scan is None:
        import os
        from base_amd.recordio import gpu
        dev = int(os.environ.get("LOCAL_RANK", "0")) if device is None else device
        ctx = gpu.default_context(dev)

        def scan(d, s, l, n):
            sc = gpu.NewShardScanner(d, gpu.ScannerOpts(), s, l, n, ctx=ctx)
            out = []
            while sc.Scan():
                out.append(sc.Get())
            err = sc.Finish()
            if err is not None:
                raise err
            return out
    recs = scan(data, start, limit, nshard)
    off, _, total, _ = ordered_prefix(len(recs), sum(len(r) for r in recs), group)
    return recs, off, total


def scan_file_split(data, rank: int, world: int, read_index: Callable, scan_range: Callable,
                    read_trailer: Callable = None, group=None):
    """One trailer-indexed file split over the ranks:

    1. rank 0 reads the trailer (Scanner.Trailer, scannerv2.go:316-342; by
       default through the GPU scanner) and broadcasts it (RCCL over xGMI);
    2. every rank turns it into block offsets (`read_index`), takes its byte
       share on block boundaries (split_blocks) and decodes it with
       `scan_range(lo, hi) -> records` -- one batch over those bytes;
    3. all_gather of (n_items, n_bytes) gives each rank its place in file order.

    Returns (records, item_offset, total_items)."""
    trailer = None
    if rank == 0:
        trailer = (read_trailer or read_index_trailer)(data)
    idx = broadcast_bytes(trailer, 0, group)
    offsets = read_index(idx)
    lo, hi = split_blocks(offsets, trailer_offset(data), rank, world)
    recs = scan_range(lo, hi) if hi > lo else []
    off, _, total, _ = ordered_prefix(len(recs), sum(len(r) for r in recs), group)
    return recs, off, total


def trailer_offset(data) -> int:
    """File offset of the trailer block: ReadLastBlock's arithmetic
    (recordio/internal/chunk.go:380-407) on the last chunk's index."""
    import struct
    n = len(data)
    index = struct.unpack_from("<I", data, n - 32768 + 24)[0]
    return n - (index + 1) * 32768


def read_index_trailer(data) -> bytes:
    """The trailer item of an in-memory file through the GPU scanner."""
    from base_amd.recordio import gpu
    sc = gpu.NewScanner(data)
    t = sc.Trailer()
    err = sc.Finish()
    if err is not None or t is None:
        raise RuntimeError(f"no trailer index: {err}")
    return t
