#!/bin/bash
# trials-per-workgroup cone kernel: parity, then the A/B of the knob.
set -o pipefail
O=gpurun_out/r03c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u tools/ab_env.py RIPTIDE_AMD_TRIALS_PER_WG 1,2,4,8,16 cfg2 > $O/tpw_cfg2.jsonl 2>&1 || { tail -5 $O/tpw_cfg2.jsonl; exit 1; }
cat $O/tpw_cfg2.jsonl | grep round
timeout -k 10 300 python -u tools/ab_env.py RIPTIDE_AMD_TRIALS_PER_WG 1,4,8,16 cfg4 > $O/tpw_cfg4.jsonl 2>&1 || { tail -5 $O/tpw_cfg4.jsonl; exit 1; }
cat $O/tpw_cfg4.jsonl | grep round
timeout -k 10 300 python -u tools/ab_env.py RIPTIDE_AMD_TRIALS_PER_WG 1,4,8 cfg3 > $O/tpw_cfg3.jsonl 2>&1 || { tail -5 $O/tpw_cfg3.jsonl; exit 1; }
cat $O/tpw_cfg3.jsonl | grep round
