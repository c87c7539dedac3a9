#!/bin/bash
# Instruction counters of the cone kernel per diagnostic flag value (phase
# attribution of VALU / SALU / LDS work): one rocprofv3 --pmc pass per flag
# over tools/ab_flags.py (2 rounds x 4 runs x 8 trials = 64 cfg2 trials).
# Usage (GPU box, repo root): bash tools/pmc_flags.sh TAG FLAG [FLAG ...]
set -o pipefail
TAG=$1; shift
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for f in "$@"; do
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE --kernel-trace -f csv -d "$O/f$f" -o run -- python3 "$R/tools/ab_flags.py" "$f" cfg2 > "$O/f$f.log" 2>&1 || { echo "pmc flag $f failed"; tail -20 "$O/f$f.log"; exit 1; }
  echo "flag $f ok"
done
