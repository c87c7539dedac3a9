#!/bin/bash
# Round-3 verdict item 1(a) at HEAD: the double-buffered persistent cone
# (RT_CONE_BUFFERS=2: one 16-wave workgroup per CU, unit u + grid streams
# into the second buffer while unit u merges) vs the default; parity of the
# variant on the full-config tests first.  Then the transform-group budget.
set -o pipefail
O=gpurun_out/r03zc
mkdir -p $O
L=riptide_amd
RIPTIDE_AMD_LIB=$L/libriptide_amd_buf2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -x --timeout 240 --timeout-method thread -k "full_config or ffa2" > $O/buf2_tests.log 2>&1 || { grep -E "^FAILED|Error" $O/buf2_tests.log | head -20; tail -3 $O/buf2_tests.log; exit 1; }
tail -1 $O/buf2_tests.log
for c in cfg2 cfg4; do
  bash tools/ab_libs.sh $c $L/libriptide_amd.so $L/libriptide_amd_buf2.so > $O/ab_$c.log 2>&1 || { cat $O/ab_$c.log; exit 1; }
  cut -c1-190 $O/ab_$c.log
done
timeout -k 10 300 python -u tools/ab_env.py RIPTIDE_AMD_SCRATCH_MFLOATS 384,1536 cfg2 > $O/ab_scratch.log 2>&1 || { tail $O/ab_scratch.log; exit 1; }
cut -c1-190 $O/ab_scratch.log
# verdict item 6: trials per launch per config, and the per-launch tail from
# the stamps build (last workgroup exit - median exit, per XCD)
for b in 16 32 64; do
  timeout -k 10 400 python -u tools/bench_configs.py $b > $O/configs_b$b.jsonl 2>$O/configs_b$b.err || { tail -5 $O/configs_b$b.err; exit 1; }
  cut -c1-220 $O/configs_b$b.jsonl
done
for cb in cfg1:16 cfg1:32 cfg2:16 cfg3:16 cfg3:32 cfg4:16 cfg4:32; do
  c=${cb%:*}; b=${cb#*:}
  RIPTIDE_AMD_LIB=$L/libriptide_amd_stamps.so timeout -k 10 300 python -u tools/diag_stamps.py $b $c > $O/stamps_${c}_b$b.json 2>$O/stamps_${c}_b$b.err || { tail -5 $O/stamps_${c}_b$b.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['launch_tails'])" $O/stamps_${c}_b$b.json
done
