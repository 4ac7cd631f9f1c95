import torch, time, json
n = 1 << 30
h1 = torch.empty(n, dtype=torch.uint8).pin_memory()
h2 = torch.empty(n, dtype=torch.uint8).pin_memory()
d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
def t(f, reps=5):
    f(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps
h2d = t(lambda: d1.copy_(h1, non_blocking=True))
d2h = t(lambda: h2.copy_(d2, non_blocking=True))
def both():
    with torch.cuda.stream(s1): d1.copy_(h1, non_blocking=True)
    with torch.cuda.stream(s2): h2.copy_(d2, non_blocking=True)
bo = t(both)
print(json.dumps({"h2d_GBs": n / h2d / 1e9, "d2h_GBs": n / d2h / 1e9, "duplex_total_GBs": 2 * n / bo / 1e9}))
