#!/bin/bash
# LDS bank-conflict attribution: one rocprofv3 --pmc pass per cone flag value
# over a short bench run (2 trials x 2 steps).
# Usage (GPU box, repo root): bash tools/pmc_conflicts.sh TAG FLAG [FLAG ...]
set -o pipefail
TAG=$1; shift
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for f in "$@"; do
  RIPTIDE_AMD_CONE_FLAGS=$f timeout -s KILL 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU --kernel-trace -f csv -d "$O/f$f" -o run -- python3 "$R/bench.py" --steps 1 --warmup 1 --batch 2 --no-cpu-baseline > "$O/f$f.log" 2>&1 || { echo "pmc flag $f failed"; tail -20 "$O/f$f.log"; exit 1; }
  python3 - "$O/f$f" "$f" <<'PY'
import csv, glob, sys
from collections import defaultdict
S = defaultdict(float)
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if "cone_kernel" in r.get("Kernel_Name", ""):
            S[r["Counter_Name"]] += float(r["Counter_Value"])
print("flags", sys.argv[2], {k: "%.3g" % (v / 4) for k, v in sorted(S.items())})
PY
done
