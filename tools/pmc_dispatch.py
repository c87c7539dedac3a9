#!/usr/bin/env python3
"""Per-launch counters of the cone kernel from tools/gpu_run.sh pmc passes
(rocprofv3 --pmc, one counter group per pass directory p1..pN): the cone
dispatches of each pass in dispatch order, cut into steps of N launches, the
counters of each launch position summed over the chosen steps.  Prints one
line per launch position with the ratios that matter here: wave-parked
(SQ_WAIT_ANY) and VALU-active fractions of wave cycles, LDS bank-conflict
fraction of LDS-active cycles, VALU / LDS / SALU instructions.

usage: tools/pmc_dispatch.py <pmc dir> N_LAUNCHES_PER_STEP [SKIP_STEPS [STEPS]]
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    root, n = sys.argv[1], int(sys.argv[2])
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    want = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 30
    acc = defaultdict(lambda: defaultdict(float))
    names = {}
    for pdir in sorted(glob.glob(os.path.join(root, "p*"))):
        disp = defaultdict(dict)
        for f in glob.glob(pdir + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                if "cone_kernel" not in r.get("Kernel_Name", ""):
                    continue
                d = int(r["Dispatch_Id"])
                disp[d][r["Counter_Name"]] = disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
                disp[d]["_name"] = r["Kernel_Name"]
        ids = sorted(disp)[skip * n:]
        ids = ids[:min(want, len(ids) // n) * n]
        for k, d in enumerate(ids):
            pos = k % n
            names[pos] = disp[d]["_name"].split("(")[0].replace("void rt::", "")
            for c, v in disp[d].items():
                if c != "_name":
                    acc[pos][c] += v
    for pos in sorted(acc):
        a = acc[pos]
        wc = a.get("SQ_WAVE_CYCLES", 0.0)
        out = [f"{pos:3d} {names[pos]:32s}"]
        if wc:
            out.append(f"wait {a.get('SQ_WAIT_ANY', 0) / wc:5.3f} valu {a.get('SQ_ACTIVE_INST_VALU', 0) / wc:5.3f}"
                       f" lds {a.get('SQ_ACTIVE_INST_LDS', 0) / wc:5.3f}")
        if a.get("SQ_LDS_IDX_ACTIVE"):
            out.append(f"conflict {a['SQ_LDS_BANK_CONFLICT'] / a['SQ_LDS_IDX_ACTIVE']:5.3f}")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_LDS_IDX_ACTIVE"):
            if c in a:
                out.append(f"{c[8:] if c.startswith('SQ_INSTS') else c[3:]} {a[c] / 1e6:8.1f}M")
        if "FETCH_SIZE" in a:
            out.append(f"fetchx2 {2 * a['FETCH_SIZE'] * 1024 / 1e9:6.2f}GB")
        if "WRITE_SIZE" in a:
            out.append(f"write {a['WRITE_SIZE'] * 1024 / 1e9:6.2f}GB")
        print(" ".join(out))


if __name__ == "__main__":
    main()
