#!/usr/bin/env python3
"""Per-phase cycle breakdown of the cone kernel (diagnostic build).

Run on the GPU box after `make -C riptide_amd/csrc stamps`:
    RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so python tools/diag_stamps.py
Phases (thread 0 of every workgroup, s_memtime deltas summed over units):
  6 setup (unit descriptor, range tree, source rows), 0 LDS-DMA issue,
  2 descriptor table, 1 DMA wait, 3 merge levels, 4 HBM store, 5 fused S/N
  epilogue; slot 7 counts units.
"""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from riptide_amd import _lib, engine
    L = _lib.load()
    n = 1 << 23
    plan = engine.PeriodogramPlan.for_search(n, 256e-6, 0.1, 10.0, 240, 260, ducy_max=0.05)
    buf = (ctypes.c_uint64 * 8)()
    _lib.check(L.rt_diag_stamps(buf, 1))     # allocates the device counters first
    B = 4
    x = torch.randn((B, n), device="cuda", dtype=torch.float32)
    out = plan.run(x)
    torch.cuda.synchronize()
    _lib.check(L.rt_diag_stamps(buf, 1))
    out = plan.run(x, out=out)
    torch.cuda.synchronize()
    _lib.check(L.rt_diag_stamps(buf, 1))
    names = ["dma_issue", "fill_wait", "desc_table", "merge", "store", "snr", "setup", "items"]
    tot = sum(buf[i] for i in range(7))
    res = {names[i]: buf[i] for i in range(8)}
    res["fractions"] = {names[i]: round(buf[i] / tot, 4) for i in range(7)}
    res["cycles_per_item"] = tot / max(1, buf[7])
    print(json.dumps(res))


if __name__ == "__main__":
    main()
