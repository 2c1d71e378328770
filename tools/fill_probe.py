"""Store ceilings of the box with torch fills of a 16 GiB buffer: zero_
(hipMemsetAsync), fill_ with a non-zero constant, fill_ from a changing
scalar, and a kernel writing varied (sin-like) data via torch ops."""
import json
import torch

dev = torch.device("cuda", 0)
n = 4 * 2 ** 30  # floats = 16 GiB
buf = torch.empty(n, dtype=torch.float32, device=dev)
res = {}


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1))
    return 4 * n / best / 1e6  # GB/s


res["zero_"] = timed(buf.zero_)
res["fill_1.0"] = timed(lambda: buf.fill_(1.0))
res["fill_0.3717"] = timed(lambda: buf.fill_(0.3717))
idx = torch.arange(2 ** 20, dtype=torch.float32, device=dev) * 1e-3
src = torch.sin(idx)
view = buf.view(-1, 2 ** 20)
res["copy_varied_rows (write-dominated, 4 MiB src in cache)"] = timed(lambda: view.copy_(src.expand_as(view)))
print(json.dumps(res, indent=1))
