#!/bin/bash
# Round 3, first box: schedule locality A/B (Infinity-Cache-sized transform
# groups, batch, streams) and per-config batch sizes.
set -o pipefail
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 300 python -u tools/ab_sched.py 384:1,24:1,6:1,6:2,2:2 16 > $O/ab_sched16.jsonl 2>&1 || { tail -5 $O/ab_sched16.jsonl; exit 1; }
cat $O/ab_sched16.jsonl
timeout -k 10 300 python -u tools/ab_sched.py 384:1,6:1,6:2,2:1,2:4 4 > $O/ab_sched4.jsonl 2>&1 || { tail -5 $O/ab_sched4.jsonl; exit 1; }
cat $O/ab_sched4.jsonl
timeout -k 10 400 python -u tools/bench_configs.py 32 > $O/configs32.jsonl 2>&1 || { tail -5 $O/configs32.jsonl; exit 1; }
cut -c1-220 $O/configs32.jsonl
