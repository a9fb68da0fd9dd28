"""Can a read-only file mapping be page-locked (hipHostRegister, ReadOnly flag) and DMA'd to the
device directly?  Times: staging-ring copy vs registered zero-copy H2D of a ~1 GB file."""
import mmap
import os
import sys
import time
import warnings

import numpy as np
import torch

path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "hostreg_probe.bin")
nbytes = int(float(os.environ.get("BYTES", "1e9")))
if not os.path.exists(path) or os.path.getsize(path) != nbytes:
    with open(path, "wb") as f:
        blk = np.random.default_rng(0).integers(0, 255, 1 << 26, dtype=np.uint8).tobytes()
        left = nbytes
        while left > 0:
            f.write(blk[:min(left, len(blk))])
            left -= len(blk)
with open(path, "rb") as f:
    mm = mmap.mmap(f.fileno(), 0, flags=mmap.MAP_SHARED | mmap.MAP_POPULATE, prot=mmap.PROT_READ)
ptr = np.frombuffer(mm, dtype=np.uint8).ctypes.data
cudart = torch.cuda.cudart()
dev = torch.device("cuda")
dst = torch.empty(nbytes, dtype=torch.uint8, device=dev)
with warnings.catch_warnings():
    warnings.simplefilter("ignore")
    host = torch.frombuffer(mm, dtype=torch.uint8)
for flags in (8, 0):
    t0 = time.perf_counter()
    r = cudart.cudaHostRegister(ptr, nbytes, flags)
    t1 = time.perf_counter()
    print(f"hipHostRegister(flags={flags}) -> {r} in {1e3 * (t1 - t0):.1f} ms; is_pinned={host.is_pinned()}", flush=True)
    if int(r) == 0:
        break
for rep in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dst.copy_(host, non_blocking=True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"H2D {nbytes / 1e9:.2f} GB: enqueue {1e3 * (t1 - t0):.1f} ms, done {1e3 * (t2 - t0):.1f} ms "
          f"({nbytes / (t2 - t0) / 1e9:.1f} GB/s)", flush=True)
ok = bool((dst[:4096].cpu().numpy() == np.frombuffer(mm, dtype=np.uint8, count=4096)).all())
print("content ok", ok)
print("unregister", cudart.cudaHostUnregister(ptr))
del host
mm.close()
