#!/bin/bash
# LDS / VALU counters of the cone kernel on one config for several feature /
# diagnostic flag values (phase attribution of bank conflicts), one rocprofv3
# run per flag value.  Usage (GPU box): bash tools/gpu_pmc_flags_cfg.sh CFG TAG flags...
set -o pipefail
CFG=$1; TAG=$2; shift 2
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for f in "$@"; do
  timeout -s KILL 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -f csv -d "$O/f$f" -o run -- python3 "$R/tools/ab_flags.py" $f $CFG > "$O/f$f.log" 2>&1 || { echo "pmc flags $f failed"; tail -20 "$O/f$f.log"; exit 1; }
  echo "== flags $f"; python3 "$R/tools/pmc_summary.py" "$O/f$f" | grep -E "SQ_"
done
