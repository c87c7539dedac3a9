#!/bin/bash
# PMC passes of the cone kernel on one BASELINE config (tools/ab_flags.py with
# the default feature bits: 2 rounds x 4 runs x 8 trials = 64 trials), one
# counter group per rocprofv3 run, each under its own time limit.
# Usage (GPU box, repo root): bash tools/gpu_pmc_cfg.sh CFG TAG
set -o pipefail
CFG=${1:-cfg4}
TAG=${2:-pmc_$CFG}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
  "FETCH_SIZE" \
  "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$O/p$i" -o run -- python3 "$R/tools/ab_flags.py" 7 $CFG > "$O/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$O/p$i.log"; exit 1; }
  echo "pass $i ok"
done
