#!/bin/bash
# Per-config throughput (tools/bench_configs.py) for each library given.
# Usage: bash tools/gpu_cfgs.sh TAG lib1.so [lib2.so ...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for lib in "$@"; do
  n=$(basename $lib .so)
  RIPTIDE_AMD_LIB=$lib timeout -k 10 400 python -u tools/bench_configs.py > $O/configs_$n.jsonl 2>$O/configs_$n.err || { tail -20 $O/configs_$n.err; exit 1; }
  echo "== $n"; python3 -c "
import json
for l in open('$O/configs_$n.jsonl'):
    d=json.loads(l); print(d['config'], round(d['trials_per_s'],1), 'trials/s', round(d['cone_ms_per_trial'],3), 'ms cone', round(d['cone_frac_of_8tbs'],3), 'frac', round(d['cone_alg_gb_per_trial'],2), 'GB')"
done
