#!/usr/bin/env python3
"""A/B of one environment knob of the engine (read per launch, or by the
planner: one plan per value) on one BASELINE config: ms per trial of the
periodogram for each value, two rounds, and whether the S/N equals the first
value's.

usage (GPU box): python tools/ab_env.py VAR v1,v2,... [cfg1|cfg2|cfg3|cfg4] [batch]
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
    var = sys.argv[1]
    vals = sys.argv[2].split(",")
    c = {k["name"]: k for k in CONFIGS}[sys.argv[3] if len(sys.argv) > 3 else "cfg2"]
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 16
    n = c["n"]
    # one plan per value, built with the knob set (planner knobs are read
    # when a plan is built, kernel knobs per launch)
    plans = {}
    for v in vals:
        os.environ[var] = v
        plans[v] = engine.PeriodogramPlan.for_search(n, c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                                     ducy_max=c["ducy_max"])
    plan = plans[vals[0]]
    x = torch.randn((B, n), device="cuda", dtype=torch.float32)
    out = torch.empty((B, plan.length, plan.num_widths), device="cuda", dtype=torch.float32)
    ws = torch.empty(max(p.workspace_bytes(B) for p in plans.values()), dtype=torch.uint8, device="cuda")
    ref = None
    for rnd in range(2):
        for v in vals:
            os.environ[var] = v
            plan = plans[v]
            plan.run(x, out=out, workspace=ws)
            torch.cuda.synchronize()
            engine.profile_reset()
            engine.profile_enable(True)
            t0 = time.perf_counter()
            for _ in range(3):
                plan.run(x, out=out, workspace=ws)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / (3 * B)
            engine.profile_enable(False)
            cone = engine.profile_read(0)
            plan.check()
            same = None
            if ref is None:
                ref = out.clone()
            else:
                same = bool(torch.equal(ref, out))
            print(json.dumps({"round": rnd, var: v, "config": c["name"], "ms_per_trial": dt * 1e3,
                              "cone_ms_per_trial": cone["ms"] / (3 * B),
                              "cone_frac": cone["alg_bytes"] / (cone["ms"] * 1e-3) / 8e12,
                              "identical_to_first": same}), flush=True)


if __name__ == "__main__":
    main()
