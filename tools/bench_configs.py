#!/usr/bin/env python3
"""Periodogram throughput of every BASELINE.json search configuration on one
GPU: ms per trial of plan.run (downsampling
ladder + cone passes + fused S/N) on device-resident white-noise trials, and
the cone kernels' algorithmic bytes / HIP-event time against the 8 TB/s HBM
peak.  The headline (cfg2 with dereddening) is bench.py's; this is the
per-config table of DESIGN.md §5.

usage (GPU box): python tools/bench_configs.py [batch] [cfg5]
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

CONFIGS = [
    dict(name="cfg1", n=2343750, tsamp=256e-6, pmin=0.5, pmax=2.0, bmin=240, bmax=260, ducy_max=0.2),
    dict(name="cfg2", n=1 << 23, tsamp=256e-6, pmin=0.1, pmax=10.0, bmin=240, bmax=260, ducy_max=0.05),
    dict(name="cfg3", n=1 << 22, tsamp=256e-6, pmin=0.2, pmax=5.0, bmin=240, bmax=260, ducy_max=0.2),
    dict(name="cfg4", n=1 << 22, tsamp=64e-6, pmin=0.002, pmax=0.5, bmin=16, bmax=32, ducy_max=0.2),
]
# cfg5's three search ranges (riptide's example.yaml, tests/golden/inputs.py
# CFG5) as periodograms alone: `python tools/bench_configs.py 16 cfg5`
CONFIGS_CFG5 = [
    dict(name="cfg5-short", n=1 << 23, tsamp=64e-6, pmin=0.2, pmax=0.5, bmin=240, bmax=260, ducy_max=0.2),
    dict(name="cfg5-medium", n=1 << 23, tsamp=64e-6, pmin=0.5, pmax=2.0, bmin=480, bmax=520, ducy_max=0.2),
    dict(name="cfg5-long", n=1 << 23, tsamp=64e-6, pmin=2.0, pmax=120.0, bmin=960, bmax=1040, ducy_max=0.2),
]


def main():
    import torch
    from riptide_amd import engine
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    configs = CONFIGS_CFG5 if len(sys.argv) > 2 and sys.argv[2] == "cfg5" else CONFIGS
    for c in configs:
        plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                                 ducy_max=c["ducy_max"])
        x = torch.randn((B, c["n"]), device="cuda", dtype=torch.float32)
        out = torch.empty((B, plan.length, plan.num_widths), device="cuda", dtype=torch.float32)
        ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
        plan.run(x, out=out, workspace=ws)
        torch.cuda.synchronize()
        steps = 3
        engine.profile_reset()
        engine.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            plan.run(x, out=out, workspace=ws)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        engine.profile_enable(False)
        cone = engine.profile_read(0)
        st = plan.stats()
        gbs = cone["alg_bytes"] / (cone["ms"] * 1e-3) / 1e9
        print(json.dumps({"config": c["name"], "batch": B, "L": plan.length, "W": plan.num_widths,
                          "transforms": st["transforms"], "ms_per_trial": dt / (steps * B) * 1e3,
                          "trials_per_s": steps * B / dt, "cone_ms_per_trial": cone["ms"] / (steps * B),
                          "cone_alg_gb_per_trial": st["alg_bytes"] / 1e9, "cone_gbs": gbs,
                          "cone_frac_of_8tbs": gbs / 8000.0}), flush=True)
        del x, out, ws, plan
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
