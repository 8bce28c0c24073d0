"""Host-side cost probe for Moeva2.generate's result hand-off (development aid, GPU box):
pinned vs pageable device->host copies of the final populations / history sizes, the cost of
fresh host memory (page faults), and whether host-buffer preparation overlaps device work.

    python tools/host_copy_probe.py
"""
import ctypes
import threading
import time

import numpy as np
import torch

MB = 1 << 20


def t(f, n=1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        r = f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n, r


def main():
    dev = torch.device("cuda", 0)
    for size_mb in (271, 930):
        n = size_mb * MB // 8
        src = torch.empty(n, dtype=torch.float64, device=dev).fill_(1.0)
        # fresh pageable numpy + torch copy
        dt, _ = t(lambda: src.cpu())
        print(f"{size_mb} MB  .cpu() (fresh pageable)         {dt * 1e3:7.1f} ms  "
              f"{size_mb / 1024 / dt:6.1f} GB/s", flush=True)
        dt, _ = t(lambda: src.cpu())
        print(f"{size_mb} MB  .cpu() again                     {dt * 1e3:7.1f} ms", flush=True)
        h = np.empty(n)
        h.fill(0.0)
        ht = torch.from_numpy(h)
        dt, _ = t(lambda: ht.copy_(src))
        print(f"{size_mb} MB  copy_ into touched pageable     {dt * 1e3:7.1f} ms  "
              f"{size_mb / 1024 / dt:6.1f} GB/s", flush=True)
        dt, pin = t(lambda: torch.empty(n, dtype=torch.float64, pin_memory=True))
        print(f"{size_mb} MB  torch pinned alloc (fresh)       {dt * 1e3:7.1f} ms", flush=True)
        dt, _ = t(lambda: pin.copy_(src, non_blocking=True))
        print(f"{size_mb} MB  copy_ into pinned                {dt * 1e3:7.1f} ms  "
              f"{size_mb / 1024 / dt:6.1f} GB/s", flush=True)
        dt, _ = t(lambda: pin.copy_(src, non_blocking=True), 3)
        print(f"{size_mb} MB  copy_ into pinned (x3 avg)       {dt * 1e3:7.1f} ms  "
              f"{size_mb / 1024 / dt:6.1f} GB/s", flush=True)
        del pin
        # numpy fresh + touch + register
        cudart = torch.cuda.cudart()

        def reg():
            a = np.empty(n)
            t0 = time.perf_counter()
            a.fill(0.0)
            t1 = time.perf_counter()
            rc = cudart.cudaHostRegister(a.ctypes.data, a.nbytes, 0)
            t2 = time.perf_counter()
            return a, rc, t1 - t0, t2 - t1

        dt, (a, rc, tf, tr) = t(reg)
        print(f"{size_mb} MB  np touch {tf * 1e3:.1f} ms + hostRegister {tr * 1e3:.1f} ms "
              f"(rc {rc})", flush=True)
        at = torch.from_numpy(a)
        dt, _ = t(lambda: at.copy_(src, non_blocking=True), 3)
        print(f"{size_mb} MB  copy_ into registered            {dt * 1e3:7.1f} ms  "
              f"{size_mb / 1024 / dt:6.1f} GB/s", flush=True)
        cudart.cudaHostUnregister(a.ctypes.data)
        del src, a, at, h, ht
        torch.cuda.empty_cache()

    # does pinned allocation run while the GPU is busy (no implicit device sync)?
    x = torch.randn(8192, 8192, device=dev)
    torch.cuda.synchronize()
    dt_busy, _ = t(lambda: [x @ x for _ in range(40)])
    print(f"busy loop alone {dt_busy * 1e3:.1f} ms", flush=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(40):
        y = x @ x
    t_enq = time.perf_counter() - t0
    p = torch.empty(930 * MB // 8, dtype=torch.float64, pin_memory=True)
    t_alloc = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"busy loop + pinned 930 MB alloc: enqueue {t_enq * 1e3:.1f} ms, alloc done at "
          f"{t_alloc * 1e3:.1f} ms, all done {t_all * 1e3:.1f} ms", flush=True)
    del p

    # threaded preparation (touch in 8 threads) during device work
    def prep(out, n):
        a = np.empty(n)
        chunks = np.array_split(a, 8)
        ths = [threading.Thread(target=c.fill, args=(0.0,)) for c in chunks]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        out.append(a)

    t0 = time.perf_counter()
    box = []
    prep(box, 930 * MB // 8)
    print(f"8-thread touch of 930 MB alone: {(time.perf_counter() - t0) * 1e3:.1f} ms",
          flush=True)
    _ = y, ctypes


if __name__ == "__main__":
    main()
