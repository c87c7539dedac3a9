#!/usr/bin/env python3
"""Dereddening + normalisation alone (GPU box): engine.deredden_normalise on a
cfg2-shaped batch (16 x 2^23 samples, 4 s running-median width at 256 us),
5 timed runs after one warm-up; ms per run.  Run under rocprofv3
--kernel-trace --stats for the per-kernel split.

usage: python tools/prep_bench.py [batch] [runs]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from riptide_amd import engine
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    runs = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    n, tsamp = 1 << 23, 256e-6
    x = torch.randn((B, n), device="cuda", dtype=torch.float32) + 3.0
    out = torch.empty_like(x)
    w = int(round(4.0 / tsamp))
    engine.deredden_normalise(x, w, 101, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(runs):
        engine.deredden_normalise(x, w, 101, out=out)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / runs * 1e3
    print(json.dumps({"batch": B, "ms_per_run": round(ms, 4), "env": {k: v for k, v in os.environ.items()
                                                                     if k.startswith("RIPTIDE_AMD_")}}))


if __name__ == "__main__":
    main()
