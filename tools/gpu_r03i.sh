#!/bin/bash
set -o pipefail
O=gpurun_out/r03k
mkdir -p $O
L=riptide_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "main: $(tail -1 $O/gpu_tests.log)"
grep -E "^FAILED" $O/gpu_tests.log | head -10
for c in cfg3 cfg1; do
timeout -k 10 300 python -u tools/ab_env.py RIPTIDE_AMD_SNR_WIDE 1,0 $c > $O/env_$c.jsonl 2>&1 || { tail -5 $O/env_$c.jsonl; exit 1; }
grep round $O/env_$c.jsonl | cut -c1-200
done
for c in cfg3 cfg2 cfg1; do
bash tools/ab_libs.sh $c $L/libriptide_amd_old.so $L/libriptide_amd_nowide.so $L/libriptide_amd.so > $O/ab_$c.log 2>&1 || { cat $O/ab_$c.log; exit 1; }
cut -c1-150 $O/ab_$c.log
done
