#!/bin/bash
# Cache-policy A/B (RT_FILL_CPOL / RT_STORE_CPOL = nt): same-box cone ms per
# trial on cfg2 and cfg3.  Usage: bash tools/gpu_r03zg.sh TAG
set -o pipefail
TAG=${1:-r03zg}
O=gpurun_out/$TAG; mkdir -p $O
L=riptide_amd/libriptide_amd
for c in cfg2 cfg3; do
  bash tools/ab_libs.sh $c $L.so ${L}_fnt.so ${L}_snt.so ${L}_bnt.so 2>&1 | tee $O/ab_$c.log || exit 1
done
