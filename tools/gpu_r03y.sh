#!/bin/bash
# 32-bit ladder kernel: GPU tests, then the cfg2 bench (ladder / cone ms per
# step) with the old and the new library, alternated.
set -o pipefail
O=gpurun_out/r03y
mkdir -p $O
L=riptide_amd
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1 || { grep -E "^FAILED|Error" $O/gpu_tests.log | head -20; tail -3 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for lib in libriptide_amd_old.so libriptide_amd.so libriptide_amd_old.so libriptide_amd.so; do
  RIPTIDE_AMD_LIB=$L/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline > $O/bench_$lib.log 2>&1 || { tail -5 $O/bench_$lib.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/bench_$lib.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$lib', round(d['value'],2), 'ms/step', round(d['ms_per_step'],2), 'cone', round(r['kernel_ms_per_step'],2), 'ladder', round(r['ladder_ms_per_step'],3))"
done
# multi-rank bench legs on the one-GPU box (gloo, all ranks on cuda:0)
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline --one-gpu-rehearsal > $O/rehearsal_cfg2.log 2>&1 || { tail -20 $O/rehearsal_cfg2.log; exit 1; }
grep '"metric"' $O/rehearsal_cfg2.log | cut -c1-300
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 2 --workload cfg3 --trials 128 --steps 1 --warmup 1 --no-cpu-baseline --one-gpu-rehearsal > $O/rehearsal_cfg3.log 2>&1 || { tail -20 $O/rehearsal_cfg3.log; exit 1; }
grep '"metric"' $O/rehearsal_cfg3.log | cut -c1-300
