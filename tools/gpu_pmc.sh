#!/bin/bash
# PMC passes over a short bench run (one counter group per rocprofv3 run, each
# under its own time limit; the first failure ends the script).
# Usage (GPU box, repo root): bash tools/gpu_pmc.sh TAG
set -o pipefail
TAG=${1:-pmc}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
BENCH="$R/bench.py --steps 1 --warmup 1 --batch 2 --no-cpu-baseline"
timeout -k 10 60 rocprofv3 -L > "$O/counters_list.txt" 2>&1 || true
i=0
for grp in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU" \
  "FETCH_SIZE" \
  "WRITE_SIZE" ; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$O/p$i" -o run -- python3 $BENCH > "$O/p$i.log" 2>&1 || { echo "pmc pass $i failed"; tail -20 "$O/p$i.log"; exit 1; }
  echo "pass $i ok"
done
