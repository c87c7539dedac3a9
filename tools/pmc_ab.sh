#!/bin/bash
# PMC A/B of cone-kernel feature flags (GPU box): for each flag value and
# counter group one rocprofv3 --pmc pass over tools/pmc_probe.py, summarised
# per kernel.  Usage: bash tools/pmc_ab.sh TAG FLAGS...
set -o pipefail
TAG=$1; shift
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for f in "$@"; do
  i=0
  for grp in \
    "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
    "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA" ; do
    i=$((i+1))
    RIPTIDE_AMD_CONE_FLAGS=$f timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$O/f$f/p$i" -o run -- python3 $R/tools/pmc_probe.py 2 > "$O/f${f}_p$i.log" 2>&1 || { echo "pmc flags $f pass $i failed"; tail -20 "$O/f${f}_p$i.log"; exit 1; }
  done
  echo "== flags $f"
  python3 $R/tools/pmc_summary.py "$O/f$f" cone_kernel
done
