#!/bin/bash
set -o pipefail
O=gpurun_out/r03g
mkdir -p $O
L=riptide_amd
RIPTIDE_AMD_LIB=$L/libriptide_amd_nohalf.so timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests_nohalf.log 2>&1; echo "nohalf: $(tail -1 $O/gpu_tests_nohalf.log)"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "main: $(tail -1 $O/gpu_tests.log)"
grep -E "^FAILED" $O/gpu_tests.log | head -10
bash tools/ab_libs.sh cfg2 $L/libriptide_amd_nozpad.so $L/libriptide_amd_nohalf.so $L/libriptide_amd.so > $O/ab_cfg2.log 2>&1 || { cat $O/ab_cfg2.log; exit 1; }
cut -c1-170 $O/ab_cfg2.log
