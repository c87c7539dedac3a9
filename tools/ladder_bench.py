#!/usr/bin/env python3
"""Downsampling ladder alone (GPU box): ms per trial of plan.ladder (the fused
one-read ladder, downsample_fused_kernel) on device-resident white noise, its
algorithmic bytes (series read once + every rung's output written once) over
the HIP-event time against the 8 TB/s HBM peak.  Per library given in
RIPTIDE_AMD_LIB, for same-box A/B of ladder kernels.

usage: python tools/ladder_bench.py [cfg2] [batch] [reps]
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
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    c = {k["name"]: k for k in CONFIGS}[name]
    plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"])
    x = torch.randn((B, c["n"]), device="cuda", dtype=torch.float32)
    ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
    engine.profile_enable(True)
    for rnd in range(2):
        plan.ladder(x, ws)
        torch.cuda.synchronize()
        engine.profile_reset()
        t0 = time.perf_counter()
        for _ in range(reps):
            plan.ladder(x, ws)
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / (reps * B) * 1e3
        p = engine.profile_read(1)
        ev = p["ms"] / (reps * B)
        gbs = p["alg_bytes"] / (p["ms"] * 1e-3) / 1e9 if p["ms"] else 0.0
        print(json.dumps({"round": rnd, "config": name, "batch": B, "lib": os.environ.get("RIPTIDE_AMD_LIB", ""),
                          "ms_per_trial_wall": round(wall, 5), "ms_per_trial_events": round(ev, 5),
                          "alg_mb_per_trial": round(p["alg_bytes"] / (reps * B) / 1e6, 3),
                          "GB_s": round(gbs, 1), "frac": round(gbs / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
