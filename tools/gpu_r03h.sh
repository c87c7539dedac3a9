#!/bin/bash
set -o pipefail
O=gpurun_out/r03h
mkdir -p $O
L=riptide_amd
timeout -k 10 300 python -u tools/ab_flags.py 7,1073741831,536870919,1610612743 cfg3 > $O/flags_cfg3.jsonl 2>&1 || { tail -5 $O/flags_cfg3.jsonl; exit 1; }
grep round $O/flags_cfg3.jsonl
bash tools/ab_libs.sh cfg2 $L/libriptide_amd_nohalf.so $L/libriptide_amd.so > $O/ab_cfg2.log 2>&1 || { cat $O/ab_cfg2.log; exit 1; }
cut -c1-170 $O/ab_cfg2.log
timeout -k 10 300 python -u tools/ab_sched.py 384:1,384:2,96:2 16 > $O/ab_sched.jsonl 2>&1 || { tail -5 $O/ab_sched.jsonl; exit 1; }
cat $O/ab_sched.jsonl | grep scratch
