#!/usr/bin/env python3
"""HBM streaming calibration: per-call time of a device-to-device copy (torch's copy
kernel) of S bytes, amortized over a replayed CUDA graph of back-to-back copies --
the regime bench.py's per-op times are measured in. Tells what "HBM-bound" costs for
an op that reads S and writes S bytes at these (MALL-sized) footprints.

  python tools/bwprobe.py
"""
import torch


def main():
    torch.cuda.init()
    for mb in (1, 4, 12, 16, 22, 32, 64, 128):
        n = mb * (1 << 20) // 4
        a = torch.randn(n, device="cuda")
        b = torch.empty_like(a)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            for _ in range(3):
                b.copy_(a)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        reps = 50
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                b.copy_(a)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        best = 1e9
        for _ in range(5):
            e0.record(s)
            with torch.cuda.stream(s):
                g.replay()
            e1.record(s)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1) / reps)
        us = best * 1e3
        print("copy %4d MiB: %8.2f us/call  %7.0f GB/s (read+write)" % (mb, us, 2 * mb * (1 << 20) / (us * 1e-6) / 1e9),
              flush=True)


if __name__ == "__main__":
    main()
