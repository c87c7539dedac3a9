#!/bin/bash
# Round 3, second box: the new host paths (multi-rank file path, cfg3 / cfg5
# bench legs with CPU baselines), cfg4 PMC, phase attribution and stamps.
set -o pipefail
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py -x -v --timeout 240 --timeout-method thread -k "search_files or mixed_shapes or error_flag or cfg5" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python -u bench.py --workload cfg3 --steps 2 --warmup 1 > $O/bench_cfg3.log 2>&1 || { tail -20 $O/bench_cfg3.log; exit 1; }
tail -1 $O/bench_cfg3.log | cut -c1-1500
timeout -k 10 500 python -u bench.py --workload cfg5 --files 64 --batch 16 > $O/bench_cfg5.log 2>&1 || { tail -20 $O/bench_cfg5.log; exit 1; }
tail -1 $O/bench_cfg5.log | cut -c1-1500
bash tools/gpu_pmc_cfg.sh cfg4 r03b_pmc_cfg4 > $O/pmc_cfg4.log 2>&1 || { tail -20 $O/pmc_cfg4.log; exit 1; }
timeout -k 10 200 python -u tools/ab_flags.py 7,1073741831,536870919,1610612743 cfg4 > $O/flags_cfg4.jsonl 2>&1 || { tail -5 $O/flags_cfg4.jsonl; exit 1; }
timeout -k 10 300 python -u tools/ab_flags.py 7,1073741831,536870919,1610612743 cfg2 > $O/flags_cfg2.jsonl 2>&1 || { tail -5 $O/flags_cfg2.jsonl; exit 1; }
cat $O/flags_cfg4.jsonl $O/flags_cfg2.jsonl | grep round
bash tools/gpu_stamps4.sh r03b cfg2 > /dev/null && bash tools/gpu_stamps4.sh r03b cfg4 > /dev/null && echo stamps ok
