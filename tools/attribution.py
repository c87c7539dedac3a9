#!/usr/bin/env python3
"""Phase attribution of the cone kernel on one config (GPU box): ms per trial
of the periodogram with the diagnostic flags (common.hpp kConeDiag*) that
leave one phase running at a time -- fill only, merge only, S/N only -- and
none (skeleton: launches, unit setup, barriers), against the full kernel.
Each phase's isolated cost = its run - skeleton; sum_over_full = (skeleton +
the three isolated costs) / full: 1.0 when the phases add up, > 1 when they
overlap.  Two alternated rounds, the second reported; stamped with the
csrc_sha of the sources (bench.source_digest).

usage: python tools/attribution.py [cfg2] [out.json]     (RIPTIDE_AMD_SCRATCH_MFLOATS as for bench.py)
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

FEAT = 15                        # kConeDefaultFeatures
NO_SNR, NO_MERGE, NO_FILL = 1 << 30, 1 << 29, 1 << 23
RUNS = {"full": FEAT, "fill_only": FEAT | NO_SNR | NO_MERGE, "merge_only": FEAT | NO_SNR | NO_FILL,
        "snr_only": FEAT | NO_MERGE | NO_FILL, "skeleton": FEAT | NO_SNR | NO_MERGE | NO_FILL}


def main():
    import torch
    from riptide_amd import engine
    from bench import source_digest
    from bench_configs import CONFIGS
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg2"
    c = {k["name"]: k for k in CONFIGS}[name]
    B = 16
    plan = engine.PeriodogramPlan.for_search(c["n"], c["tsamp"], c["pmin"], c["pmax"], c["bmin"], c["bmax"],
                                             ducy_max=c["ducy_max"])
    x = torch.randn((B, c["n"]), device="cuda", dtype=torch.float32)
    out = torch.empty((B, plan.length, plan.num_widths), device="cuda", dtype=torch.float32)
    ws = torch.empty(plan.workspace_bytes(B), dtype=torch.uint8, device="cuda")
    ms = {}
    for rnd in range(2):
        for k, f in RUNS.items():
            os.environ["RIPTIDE_AMD_CONE_FLAGS"] = str(f)
            plan.run(x, out=out, workspace=ws)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                plan.run(x, out=out, workspace=ws)
            torch.cuda.synchronize()
            ms[k] = (time.perf_counter() - t0) / (3 * B) * 1e3
            print(json.dumps({"round": rnd, "run": k, "flags": f, "ms_per_trial": ms[k]}), flush=True)
    os.environ.pop("RIPTIDE_AMD_CONE_FLAGS")
    sk = ms["skeleton"]
    iso = {"fill": ms["fill_only"] - sk, "merge": ms["merge_only"] - sk, "snr": ms["snr_only"] - sk}
    res = {"config": name, "batch": B, "csrc_sha": source_digest(),
           "scratch_mfloats": os.environ.get("RIPTIDE_AMD_SCRATCH_MFLOATS"),
           "ms_per_trial": {k: round(v, 4) for k, v in ms.items()},
           "isolated_ms_per_trial": {k: round(v, 4) for k, v in iso.items()},
           "sum_over_full": round((sk + sum(iso.values())) / ms["full"], 4),
           "note": "ms per trial of plan.run (ladder included, in every run); isolated = run - skeleton"}
    print(json.dumps(res))
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
