#!/usr/bin/env python3
"""Turn a tools/gpu_run.sh pmc run into profiles/<name>.json: per-trial HBM bytes of
the cone kernel from FETCH_SIZE / WRITE_SIZE (rocprofv3, KB units), with the
gfx950 correction of MI355X_MICROARCH.md (FETCH_SIZE reports half the bytes of
wide streaming reads: x2), plus the SQ counters as ratios.

usage: tools/pmc_to_json.py gpurun_out/<pmc dir> profiles/<name>.json TRIALS [--config CFG] [--kernel NAME]
(TRIALS = trials the profiled run processed: tools/gpu_run.sh pmc cfg2 runs
bench.py warmup 1 + steps 1 at batch 2 -> 4; pmc CFG runs tools/ab_flags.py,
2 rounds x 4 runs x 8 trials -> 64)
"""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict


def main():
    root, out, trials = sys.argv[1], sys.argv[2], int(sys.argv[3])
    config = sys.argv[sys.argv.index("--config") + 1] if "--config" in sys.argv else "cfg2"
    kernel = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "cone_kernel"
    sums = defaultdict(float)
    disp = defaultdict(set)
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel not in r.get("Kernel_Name", ""):
                    continue
                sums[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add((f, r.get("Dispatch_Id")))
    fetch = 2.0 * sums["FETCH_SIZE"] * 1024.0
    write = sums["WRITE_SIZE"] * 1024.0
    launches = len(disp["FETCH_SIZE"])
    commit = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True, text=True).stdout.strip()
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import source_digest
    res = {
        "kernel": kernel,
        "config": config,
        "source": root,
        "commit": commit,
        "csrc_sha": source_digest(),      # bench.py uses the summary only for these exact kernel sources
        "trials": trials,
        "launches": launches,
        "fetch_bytes_per_trial": fetch / trials,
        "write_bytes_per_trial": write / trials,
        "hbm_bytes_per_trial": (fetch + write) / trials,
        "note": "FETCH_SIZE x2 (gfx950 wide-read correction), WRITE_SIZE as reported; Infinity-Cache hits "
                "are counted by these memory-side counters",
        "sq": {k: sums[k] for k in sorted(sums) if k.startswith("SQ_")},
    }
    if sums.get("SQ_LDS_IDX_ACTIVE"):
        res["lds_bank_conflict_frac"] = sums["SQ_LDS_BANK_CONFLICT"] / sums["SQ_LDS_IDX_ACTIVE"]
    if sums.get("SQ_WAVE_CYCLES"):
        res["wait_any_frac"] = sums["SQ_WAIT_ANY"] / sums["SQ_WAVE_CYCLES"]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "sq"}))


if __name__ == "__main__":
    main()
