#!/usr/bin/env python3
"""Schedule A/B on one BASELINE config (default cfg2): transform-group scratch budget
(RIPTIDE_AMD_SCRATCH_MFLOATS, read at plan creation) x number of HIP streams
the batch is split over (each stream runs its share of the trials with its
own workspace, so one stream's launch tails overlap the other's work).
Prints ms per trial and whether the S/N equals the first configuration's.

usage (GPU box): python tools/ab_sched.py 96:1,96:2,384:1 [batch] [cfg1|cfg2|cfg3|cfg4]
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
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from bench_configs import CONFIGS
    c = {k["name"]: k for k in CONFIGS}[sys.argv[3] if len(sys.argv) > 3 else "cfg2"]
    n = c["n"]
    cfgs = [tuple(int(v) for v in c.split(":")) for c in (sys.argv[1] if len(sys.argv) > 1 else "96:1,96:2").split(",")]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    x = torch.randn((B, n), device="cuda", dtype=torch.float32)
    ref = None
    for scratch, ns in cfgs:
        os.environ["RIPTIDE_AMD_SCRATCH_MFLOATS"] = str(scratch)
        plan = engine.PeriodogramPlan.for_search(n, c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                                 ducy_max=c["ducy_max"])
        out = torch.empty((B, plan.length, plan.num_widths), device="cuda", dtype=torch.float32)
        parts = [(k * B // ns, (k + 1) * B // ns) for k in range(ns)]
        streams = [torch.cuda.Stream() for _ in range(ns)]
        wss = [torch.empty(plan.workspace_bytes(b1 - b0), dtype=torch.uint8, device="cuda") for b0, b1 in parts]

        def step():
            cur = torch.cuda.current_stream()
            for s in streams:
                s.wait_stream(cur)
            for (b0, b1), s, ws in zip(parts, streams, wss):
                with torch.cuda.stream(s):
                    plan.run(x[b0:b1], out=out[b0:b1], workspace=ws, stream=s)
            for s in streams:
                cur.wait_stream(s)

        step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / (3 * B)
        same = None
        if ref is None:
            ref = out.clone()
        else:
            same = bool(torch.equal(ref, out))
        print(json.dumps({"config": c["name"], "scratch_mfloats": scratch,
                          "workspace_gb": sum(w.numel() for w in wss) / 1e9, "streams": ns, "batch": B, "launches": plan.stats()["launches"],
                          "ms_per_trial": dt * 1e3, "identical_to_first": same}), flush=True)
        del out, wss, plan
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
