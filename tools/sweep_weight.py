#!/usr/bin/env python3
"""Tile-pass cost-model sweep on the GPU box: RIPTIDE_AMD_PASS_WEIGHT (read
when a plan is built) -> periodogram ms per trial, per configuration.

usage: python tools/sweep_weight.py 25,100,400 cfg4,cfg2
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
    weights = sys.argv[1].split(",") if len(sys.argv) > 1 else ["25", "100", "400"]
    names = sys.argv[2].split(",") if len(sys.argv) > 2 else ["cfg4"]
    B = 8
    for name in names:
        c = {k["name"]: k for k in CONFIGS}[name]
        x = torch.randn((B, c["n"]), device="cuda", dtype=torch.float32)
        for rnd in range(2):
            for w in weights:
                os.environ["RIPTIDE_AMD_PASS_WEIGHT"] = w
                plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"],
                                                         c["bmax"], ducy_max=c["ducy_max"])
                out = torch.empty((B, plan.length, plan.num_widths), device="cuda", dtype=torch.float32)
                ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
                plan.run(x, out=out, workspace=ws)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(3):
                    plan.run(x, out=out, workspace=ws)
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / (3 * B)
                print(json.dumps({"config": name, "round": rnd, "pass_weight": float(w), "ms_per_trial": dt * 1e3}),
                      flush=True)
                del plan, out, ws


if __name__ == "__main__":
    main()
