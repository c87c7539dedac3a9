#!/usr/bin/env python3
"""Aggregate rocprofv3 --pmc per-dispatch CSVs (tools/gpu_run.sh TAG pmc) per kernel.

usage: tools/pmc_summary.py gpurun_out/<tag> [kernel-substring]
Prints, per counter, the sum over the matching kernel's dispatches and the
per-dispatch mean.  FETCH_SIZE/WRITE_SIZE are in KB (rocprofv3 derived
metrics); on gfx950 FETCH_SIZE reports half the bytes of wide streaming reads
(MI355X_MICROARCH.md, HBM section) -- the corrected value is printed too.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else "cone_kernel"
    sums = defaultdict(float)
    disp = defaultdict(set)
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if pat not in r.get("Kernel_Name", ""):
                    continue
                name = r["Counter_Name"]
                sums[name] += float(r["Counter_Value"])
                disp[name].add((f, r.get("Dispatch_Id")))
    for k in sorted(sums):
        n = len(disp[k])
        print(f"{k:28s} total {sums[k]:.6g}  dispatches {n}  mean {sums[k] / max(n, 1):.6g}")
    if "FETCH_SIZE" in sums:
        print(f"FETCH_SIZE corrected (x2, GB total): {2 * sums['FETCH_SIZE'] * 1024 / 1e9:.4f}")
    if "WRITE_SIZE" in sums:
        print(f"WRITE_SIZE (GB total): {sums['WRITE_SIZE'] * 1024 / 1e9:.4f}")


if __name__ == "__main__":
    main()
