#!/usr/bin/env python3
"""Device vs host find_peaks on cfg2 periodograms (GPU box):
ms per trial of PeakFinder (HIP order statistics + threshold selection, host
polyfit/cluster) and of the reference-restated numpy find_peaks."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np
    import torch
    from riptide_amd import engine
    from riptide_amd.metadata import Metadata
    from riptide_amd.peak_detection import find_peaks
    from riptide_amd.peaks import PeakFinder
    from riptide_amd.periodogram import Periodogram
    n, tsamp, B = 1 << 23, 256e-6, 8
    plan = engine.PeriodogramPlan.for_search(n, tsamp, 0.1, 10.0, 240, 260, ducy_max=0.05)
    x = torch.randn((B, n), device="cuda", dtype=torch.float32)
    snr = plan.run(x)
    finder = PeakFinder(plan, n * tsamp)
    finder(snr, dms=[0.0] * B)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        res = finder(snr, dms=[0.0] * B)
    torch.cuda.synchronize()
    dev_ms = (time.perf_counter() - t0) / (3 * B) * 1e3
    periods, foldbins = plan.grid()
    s0 = snr[0].cpu().numpy()
    t0 = time.perf_counter()
    pg = Periodogram(plan.widths, periods, foldbins, s0, metadata=Metadata({"tobs": n * tsamp, "dm": 0.0}))
    ref, _ = find_peaks(pg)
    host_ms = (time.perf_counter() - t0) * 1e3
    print(json.dumps({"device_ms_per_trial": dev_ms, "host_ms_per_trial": host_ms, "peaks_trial0": len(res[0][0]),
                      "identical_trial0": res[0][0] == ref, "nseg": finder.nseg, "per_seg": finder.per_seg}))


if __name__ == "__main__":
    main()
