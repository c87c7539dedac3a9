#!/usr/bin/env python3
"""Schedule sweep on the GPU box: per-trial scratch budget of a transform
group (RIPTIDE_AMD_SCRATCH_MFLOATS) x batch size -> cone ms per trial.

A small budget keeps each group's ping/pong working set inside the 256 MiB
Infinity Cache, so the intermediate FFA passes re-read on-die instead of HBM.
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
    n = 1 << 23
    budgets = [float(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "33.5,8,4,2,1").split(",")]
    batches = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,4,8").split(",")]
    x = torch.randn((max(batches), n), device="cuda", dtype=torch.float32)
    for bud in budgets:
        os.environ["RIPTIDE_AMD_SCRATCH_MFLOATS"] = str(bud)
        plan = engine.PeriodogramPlan.for_search(n, 256e-6, 0.1, 10.0, 240, 260, ducy_max=0.05)
        st = plan.stats()
        for B in batches:
            xb = x[:B]
            out = torch.empty((B, plan.length, plan.num_widths), device="cuda", dtype=torch.float32)
            ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
            plan.run(xb, out=out, workspace=ws)
            torch.cuda.synchronize()
            reps = max(1, 16 // B)
            t0 = time.perf_counter()
            for _ in range(reps):
                plan.run(xb, out=out, workspace=ws)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / (reps * B)
            print(json.dumps({"budget_mfloats": bud, "batch": B, "ms_per_trial": dt * 1e3,
                              "launches": st["launches"], "ws_gb": ws.numel() / 1e9}), flush=True)
            del out, ws
        del plan


if __name__ == "__main__":
    main()
