#!/bin/bash
# Transform-group scratch budget sweep (cfg2 at 16 trials, cfg3 at 32, cfg1 /
# cfg4 at 16) and the per-launch tails on the device-wide clock.
set -o pipefail
O=gpurun_out/r03zd
mkdir -p $O
L=riptide_amd
for cb in cfg2:16 cfg3:32 cfg1:16 cfg4:16; do
  c=${cb%:*}; b=${cb#*:}
  timeout -k 10 400 python -u tools/ab_sched.py 384:1,1536:1,3072:1,6144:1,384:1 $b $c > $O/sched_$c.jsonl 2>$O/sched_$c.err || { tail -5 $O/sched_$c.err; exit 1; }
  cut -c1-230 $O/sched_$c.jsonl
done
for cb in cfg2:16 cfg3:32 cfg4:16; do
  c=${cb%:*}; b=${cb#*:}
  for s in 384 3072; do
    RIPTIDE_AMD_SCRATCH_MFLOATS=$s RIPTIDE_AMD_LIB=$L/libriptide_amd_stamps.so timeout -k 10 300 python -u tools/diag_stamps.py $b $c > $O/stamps_${c}_s$s.json 2>$O/stamps_${c}_s$s.err || { tail -5 $O/stamps_${c}_s$s.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['launch_tails'])" $O/stamps_${c}_s$s.json
  done
done
