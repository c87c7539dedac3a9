#!/bin/bash
# Phase priorities (RT_PRIO_START: unit start at setprio 2; RT_PRIO_TAIL: the
# S/N at setprio 1): same-box cone A/B on cfg2 and cfg3.
# Usage: bash tools/gpu_r03zl.sh TAG
set -o pipefail
TAG=${1:-r03zl}
O=gpurun_out/$TAG; mkdir -p $O
L=riptide_amd/libriptide_amd
for c in cfg2 cfg3; do
  bash tools/ab_libs.sh $c $L.so ${L}_ps.so ${L}_pt.so 2>&1 | tee $O/ab_$c.log || exit 1
done
