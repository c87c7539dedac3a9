#!/bin/bash
set -o pipefail
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -20; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
bash tools/ab_libs.sh cfg2 riptide_amd/libriptide_amd_base.so riptide_amd/libriptide_amd.so > $O/ab.log 2>&1 || { cat $O/ab.log; exit 1; }
cat $O/ab.log | cut -c1-200
bash tools/pmc_conflicts.sh r03e_conf 536870919 > $O/conf.log 2>&1 || { tail -20 $O/conf.log; exit 1; }
grep flags $O/conf.log
