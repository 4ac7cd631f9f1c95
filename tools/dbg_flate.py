"""Debug aid: rerun test_encode_flate_decodes' write loop and dump the first
file whose blocks zlib cannot inflate to gpurun_out/flate_fail.rio."""
import os
import random
import sys
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from base_amd.recordio.gpu import Context  # noqa: E402
from base_amd.recordio.writer import WriterOpts  # noqa: E402
from test_encode_gpu import gpu_write, records, fastq_records  # noqa: E402

ctx = Context(0)
rng = random.Random(5)
sets = [fastq_records(rng, 3000), records(rng, 300), [b""] * 50, [b"x" * 100000] * 3,
        [bytes([i % 7]) * rng.randrange(0, 600) for i in range(2000)]]
sets.append([bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40000))) for _ in range(20)])
sets.append([b"ACGT"[rng.randrange(4):][:1] * rng.randrange(1, 70000) for _ in range(12)])
os.makedirs("gpurun_out", exist_ok=True)
for level in ("flate", "flate 0", "flate 1", "flate 5"):
    for i, recs in enumerate(sets):
        mi = rng.choice([1, 50, 1000])
        data = gpu_write(recs, WriterOpts(Transformers=[level], MaxItems=mi), trailer=b"trail" * 3, ctx=ctx,
                         batch_bytes=1 << 18)
        off, nbad = 32768, 0
        while off < len(data):
            total = int.from_bytes(data[off + 20:off + 24], "little")
            pay = b"".join(data[off + c * 32768 + 28: off + c * 32768 + 28 +
                                int.from_bytes(data[off + c * 32768 + 16:off + c * 32768 + 20], "little")]
                           for c in range(total))
            try:
                zlib.decompress(pay, -15)
            except zlib.error as e:
                if nbad == 0:
                    open("gpurun_out/flate_fail_block.bin", "wb").write(pay)
                    print("bad block", level, i, mi, off, len(pay), e, flush=True)
                nbad += 1
            off += total * 32768
        print(level, i, mi, "bad blocks", nbad, flush=True)
        if nbad:
            open("gpurun_out/flate_fail.rio", "wb").write(data)
            sys.exit(0)
