#!/usr/bin/env python3
"""Periodogram ms per trial of each cfg5 search range (tests/golden/inputs.py
CFG5, 2^23 samples @ 64 us) on the GPU box, 8 device-resident trials, with
each range's kernel variant (merge slots of its bins) -- where cfg5's device
time goes.

usage: python tools/bench_ranges.py
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def main():
    import torch
    import inputs
    from riptide_amd import engine
    c = inputs.CFG5
    n, ts, B = 1 << 23, 64e-6, 8
    x = torch.randn((B, n), device="cuda", dtype=torch.float32)
    for r in c["ranges"]:
        fs = r["ffa_search"]
        plan = engine.PeriodogramPlan.for_search(n, ts, fs["period_min"], fs["period_max"], fs["bins_min"],
                                                 fs["bins_max"], wtsp=fs.get("wtsp", 1.5))
        out = torch.empty((B, plan.length, plan.num_widths), device="cuda", dtype=torch.float32)
        ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
        plan.run(x, out=out, workspace=ws)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            plan.run(x, out=out, workspace=ws)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / (3 * B)
        print(json.dumps({"range": r["name"], "L": plan.length, "W": plan.num_widths, "ms_per_trial": dt * 1e3}),
              flush=True)


if __name__ == "__main__":
    main()
