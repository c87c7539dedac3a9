#!/bin/bash
# Phase attribution at HEAD (cfg2): VALU / SALU / LDS instructions of the cone
# kernel with the S/N, the merge, both or neither skipped (diagnostic flags).
set -o pipefail
O=gpurun_out/r03s
mkdir -p $O
bash tools/pmc_flags.sh r03s/pmc 7 1073741831 536870919 1610612743 > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 - > $O/summary.txt <<'PY'
import csv, glob, collections
for f in ("7", "1073741831", "536870919", "1610612743"):
    s = collections.defaultdict(float)
    for fn in glob.glob(f"gpurun_out/r03s/pmc/f{f}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(fn)):
            if "cone_kernel" in r.get("Kernel_Name", ""):
                s[r["Counter_Name"]] += float(r["Counter_Value"])
    print(f, {k: "%.4g" % (v / 64) for k, v in sorted(s.items())})
PY
cat $O/summary.txt
