#!/bin/bash
# S/N-store cache policy and the nt merge stores re-checked on every config:
# same-box cone ms per trial.  Usage: bash tools/gpu_r03zh.sh TAG
set -o pipefail
TAG=${1:-r03zh}
O=gpurun_out/$TAG; mkdir -p $O
L=riptide_amd/libriptide_amd
for c in cfg2 cfg3 cfg4 cfg1; do
  bash tools/ab_libs.sh $c $L.so ${L}_s0.so ${L}_snrnt.so 2>&1 | tee $O/ab_$c.log || exit 1
done
