"""Host-side bandwidth probe for the FITS stream: device -> pinned copy and
pinned -> file writes (single write, concurrent pwrite) on the GPU box."""
import os
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

import torch

N = 1 << 30
dev = torch.device("cuda", 0)
d = torch.empty(N, dtype=torch.uint8, device=dev).fill_(7)
h = torch.empty(N, dtype=torch.uint8, pin_memory=True)
for k in range(3):
    torch.cuda.synchronize()
    t = time.perf_counter()
    h.copy_(d, non_blocking=True)
    torch.cuda.synchronize()
    print(f"D2H pinned 1 GiB: {N / (time.perf_counter() - t) / 1e9:.1f} GB/s", flush=True)
mv = memoryview(h.numpy())
with tempfile.TemporaryDirectory() as td:
    for k in range(3):
        p = os.path.join(td, f"a{k}")
        t = time.perf_counter()
        with open(p, "wb") as f:
            f.write(mv)
        print(f"file write 1 GiB (one write): {N / (time.perf_counter() - t) / 1e9:.1f} GB/s", flush=True)
    for nt in (4, 8, 16):
        p = os.path.join(td, f"b{nt}")
        fd = os.open(p, os.O_WRONLY | os.O_CREAT)
        piece = N // (nt * 4)
        t = time.perf_counter()
        with ThreadPoolExecutor(nt) as ex:
            list(ex.map(lambda a: os.pwrite(fd, mv[a:a + piece], a), range(0, N, piece)))
        os.close(fd)
        print(f"file write 1 GiB ({nt} threads pwrite): {N / (time.perf_counter() - t) / 1e9:.1f} GB/s", flush=True)
        os.unlink(p)
    t = time.perf_counter()
    x = bytearray(N)
    x[:] = mv
    print(f"host memcpy 1 GiB: {N / (time.perf_counter() - t) / 1e9:.1f} GB/s")
