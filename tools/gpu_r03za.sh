#!/bin/bash
# S/N prefix from running sums (RT_SNR_RUNSUM 1 vs 0): GPU tests, then
# on cfg2, cfg3, cfg4.
set -o pipefail
O=gpurun_out/r03za
mkdir -p $O
L=riptide_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "^FAILED|Error" $O/gpu_tests.log | head -20; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in cfg2 cfg3 cfg4; do
  bash tools/ab_libs.sh $c $L/libriptide_amd_old.so $L/libriptide_amd.so > $O/ab_$c.log 2>&1 || { cat $O/ab_$c.log; exit 1; }
  cut -c1-190 $O/ab_$c.log
done
