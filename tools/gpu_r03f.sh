#!/bin/bash
set -o pipefail
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
L=riptide_amd
bash tools/ab_libs.sh cfg2 $L/libriptide_amd_base.so $L/libriptide_amd.so $L/libriptide_amd_nopack.so $L/libriptide_amd_nostd6.so > $O/ab_cfg2.log 2>&1 || { cat $O/ab_cfg2.log; exit 1; }
cut -c1-170 $O/ab_cfg2.log
bash tools/ab_libs.sh cfg3 $L/libriptide_amd_base.so $L/libriptide_amd.so > $O/ab_cfg3.log 2>&1 || { cat $O/ab_cfg3.log; exit 1; }
cut -c1-170 $O/ab_cfg3.log
bash tools/ab_libs.sh cfg4 $L/libriptide_amd_base.so $L/libriptide_amd.so > $O/ab_cfg4.log 2>&1 || { cat $O/ab_cfg4.log; exit 1; }
cut -c1-170 $O/ab_cfg4.log
