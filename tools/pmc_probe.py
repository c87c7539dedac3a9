#!/usr/bin/env python3
"""Small cfg2 workload for PMC A/B runs (rocprofv3 --pmc ... -- python3
tools/pmc_probe.py): one warm plan.run and one profiled plan.run of B trials;
the cone feature flags come from RIPTIDE_AMD_CONE_FLAGS."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    from riptide_amd import engine
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    n = 1 << 23
    plan = engine.PeriodogramPlan.for_search(n, 256e-6, 0.1, 10.0, 240, 260, ducy_max=0.05)
    x = torch.randn((B, n), device="cuda", dtype=torch.float32)
    out = plan.run(x)
    out = plan.run(x, out=out)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
