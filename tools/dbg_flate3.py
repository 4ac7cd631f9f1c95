import os, sys, random, io
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import torch
from base_amd.recordio import gpu
from base_amd.recordio.writer import Writer, WriterOpts
from oracle import oracle as O

def rnd_file(rng, nrec, maxlen):
    buf = io.BytesIO()
    w = Writer(buf, WriterOpts(Transformers=['flate'], KeyTrailer=True, MaxItems=rng.choice([1, 3, 17, 253, 1000, 16384])))
    recs = []
    for i in range(nrec):
        n = rng.choice([0, 1, 2, rng.randrange(maxlen + 1), rng.randrange(128, 300)])
        x = os.urandom(n)
        recs.append(x); w.Append(x)
        if rng.random() < 0.02: w.Flush()
    w.SetTrailer(b'Trailer'); w.Finish()
    return buf.getvalue(), recs

def main(seed):
    ctx = gpu.Context(0, max_span_bytes=64 << 20)
    rng = random.Random(seed)
    for trial in range(12):
        data, recs = rnd_file(rng, rng.randrange(0, 3000), rng.choice([10, 300, 5000, 70000]))
        sc = gpu.NewScanner(data, ctx=ctx)
        tr = sc.Trailer()
        items = []
        while sc.Scan(): items.append(sc.Get())
        err = sc.Err()
        ok = err is None and items == recs and tr == b'Trailer'
        print('trial', trial, 'len', len(data), 'nrec', len(recs), 'ok', ok, 'err', err, flush=True)
        if not ok:
            k = next((i for i in range(min(len(items), len(recs))) if items[i] != recs[i]), None)
            print(' first diff item', k, 'ngot', len(items))
            if k is not None:
                a, b = items[k], recs[k]
                j = next((i for i in range(min(len(a), len(b))) if a[i] != b[i]), None)
                print(' lens', len(a), len(b), 'first byte diff', j)
            os.environ['RIO_DEBUG'] = '1'
            sc = gpu.NewScanner(data, ctx=ctx)
            while sc.Scan(): pass
            break


if __name__ == '__main__':
    for sd in range(int(sys.argv[1]), int(sys.argv[2])):
        print('seed', sd, flush=True)
        main(sd)
