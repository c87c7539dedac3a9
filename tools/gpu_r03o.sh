#!/bin/bash
set -o pipefail
O=gpurun_out/r03o
mkdir -p $O
L=riptide_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "main: $(tail -1 $O/gpu_tests.log)"
grep -E "^FAILED|Error" $O/gpu_tests.log | head -10
bash tools/ab_libs.sh cfg4 $L/libriptide_amd_old.so $L/libriptide_amd.so > $O/ab_cfg4.log 2>&1 || { cat $O/ab_cfg4.log; exit 1; }
cut -c1-150 $O/ab_cfg4.log
