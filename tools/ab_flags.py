#!/usr/bin/env python3
"""A/B of cone-kernel feature bits (RIPTIDE_AMD_CONE_FLAGS, read per launch
batch) on the cfg2 workload: ms per trial of the periodogram for each value.

usage (GPU box): python tools/ab_flags.py 3,2,1,0 [cfg1|cfg2|cfg3|cfg4]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    import torch
    from riptide_amd import engine
    from bench_configs import CONFIGS
    flags = sys.argv[1].split(",") if len(sys.argv) > 1 else ["3", "0"]
    c = {k["name"]: k for k in CONFIGS}[sys.argv[2] if len(sys.argv) > 2 else "cfg2"]
    n = c["n"]
    B = int(os.environ.get("AB_BATCH", "8"))     # tools/gpu_run.sh pmc: 16, the configs table's batch
    plan = engine.PeriodogramPlan.for_search(n, c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"])
    x = torch.randn((B, n), device="cuda", dtype=torch.float32)
    out = torch.empty((B, plan.length, plan.num_widths), device="cuda", dtype=torch.float32)
    ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
    ref = None
    for rnd in range(2):
        for f in flags:
            os.environ["RIPTIDE_AMD_CONE_FLAGS"] = f
            plan.run(x, out=out, workspace=ws)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                plan.run(x, out=out, workspace=ws)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / (3 * B)
            same = None
            if ref is None:
                ref = out.clone()
            else:
                same = bool(torch.equal(ref, out))
            print(json.dumps({"round": rnd, "flags": f, "ms_per_trial": dt * 1e3, "identical_to_first": same}),
                  flush=True)


if __name__ == "__main__":
    main()
