#!/bin/bash
# Unrolled ladder window sums + prep/passes overlap: GPU tests, then the cfg2
# bench with one stream and with the prep of step k+1 overlapping step k.
set -o pipefail
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "^FAILED|Error" $O/gpu_tests.log | head -20; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for ov in 0 1 0 1; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --overlap $ov > $O/bench_ov$ov.log 2>&1 || { tail -5 $O/bench_ov$ov.log; exit 1; }
  python3 -c "
import json,sys; d=json.loads(open('$O/bench_ov$ov.log').read().strip().splitlines()[-1]); r=d['roofline']
print('overlap $ov', round(d['value'],2), 'ms/step', round(d['ms_per_step'],2), 'cone', round(r['kernel_ms_per_step'],2), 'ladder', round(r['ladder_ms_per_step'],3), 'frac', round(r['frac'],4))"
done
