import os, sys
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tools')
import torch
os.environ['RIO_DEBUG'] = '1'
import c3_data
from base_amd.recordio import gpu
data, nrec, rb = c3_data.make_file(int(sys.argv[1]) << 20 if len(sys.argv) > 1 else 2 << 20, 1024, workers=8)
body = data[32768:]
ctx = gpu.Context(0, max_span_bytes=len(body) + 32768)
b = ctx.scan_span(body, file_off=32768, is_file_end=True, codec=gpu.RIO_CODEC_FLATE)
print('stop', b.stop, b.err.msg, b.n_items, nrec)
