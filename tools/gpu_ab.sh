#!/bin/bash
# Parity tests + bench A/B of cone feature flags (GPU box, repo root).
# Usage: bash tools/gpu_ab.sh TAG FLAGS_A FLAGS_B ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -3 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/gpu_tests.log | head -30; exit 1; }
fi
for f in "$@"; do
  RIPTIDE_AMD_CONE_FLAGS=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$f.log 2>&1 || { tail -20 $O/bench_$f.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_$f.log').read().strip().splitlines()[-1]); r=d['roofline']; print('flags=$f', round(d['value'],2), 'trials/s', round(r['kernel_ms_per_step']/16,3), 'ms/trial cone', round(r['frac'],4))"
done
