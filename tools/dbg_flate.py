import sys, os, json
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import torch
os.environ['RIO_DEBUG'] = '1'
from base_amd.recordio import gpu
from conftest import golden_bytes
m = json.load(open('/root/repo/tests/golden/manifest.json'))['cases']
case = [c for c in m if c['name'] == 'transformer_flate'][0]
data = golden_bytes(case)
ctx = gpu.Context(0, max_span_bytes=8 << 20)
sc = gpu.NewScanner(data, ctx=ctx)
n = 0
while sc.Scan():
    n += 1
print('items', n, 'err', sc.Err())
