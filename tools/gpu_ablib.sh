#!/bin/bash
# Parity tests on the default library, then bench A/B over alternative builds.
# Usage: bash tools/gpu_ablib.sh TAG lib1.so lib2.so ...   (default lib first)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -2 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
for lib in "$@"; do
  n=$(basename $lib .so)
  if [ -n "$PARITY_ALL" ]; then
    RIPTIDE_AMD_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/parity_$n.log 2>&1 || { echo "$n parity FAILED"; grep -E "FAIL|Error|assert" $O/parity_$n.log | head -20; exit 1; }
    echo "$n parity: $(tail -1 $O/parity_$n.log)"
  fi
  RIPTIDE_AMD_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$n.log 2>&1 || { tail -20 $O/bench_$n.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$n.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', round(d['value'],2), 'trials/s', round(r['kernel_ms_per_step']/16,3), 'ms/trial cone', round(r['frac'],4), 'alg GB/trial', round(r['alg_bytes_per_trial']/1e9,2))"
done
