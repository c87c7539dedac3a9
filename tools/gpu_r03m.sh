#!/bin/bash
set -o pipefail
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u tools/ab_flags.py 7,1073741831,536870919,1610612743 cfg4 > $O/flags_cfg4.jsonl 2>&1 || { tail -5 $O/flags_cfg4.jsonl; exit 1; }
grep round $O/flags_cfg4.jsonl | cut -c1-120
bash tools/gpu_pmc_cfg.sh cfg4 r03m/pmc_cfg4 || exit 1
python3 tools/pmc_summary.py gpurun_out/r03m/pmc_cfg4 > $O/pmc_cfg4_summary.txt 2>&1; tail -30 $O/pmc_cfg4_summary.txt
