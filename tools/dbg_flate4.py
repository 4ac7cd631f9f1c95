"""Development aid: small flate cases through the GPU scanner vs the writer's records."""
import os, sys, random
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from base_amd.recordio import gpu
from base_amd.recordio.writer import write_file, WriterOpts

cases = {
    "fixed_small": [b"hello hello hello hello"],
    "dyn_text": [(b"the quick brown fox jumps over the lazy dog %d " % i) * 3 for i in range(200)],
    "dyn_rand_bytes": [bytes(random.Random(i).getrandbits(8) for _ in range(300)) for i in range(50)],
    "runs": [b"a" * 1000 + b"b" * 1000],
}
ctx = gpu.Context(0, max_span_bytes=8 << 20)
for name, recs in cases.items():
    data = write_file(recs, WriterOpts(Transformers=["flate"]))
    sc = gpu.NewScanner(data, ctx=ctx)
    got = []
    while sc.Scan():
        got.append(sc.Get())
    err = sc.Err()
    print(name, "ok" if (err is None and got == recs) else "FAIL", err, len(got), len(recs), flush=True)
    if err is not None or got != recs:
        os.environ["RIO_DEBUG"] = "1"
        sc = gpu.NewScanner(data, ctx=ctx)
        while sc.Scan():
            pass
        os.environ.pop("RIO_DEBUG")
