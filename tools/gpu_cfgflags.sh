#!/bin/bash
# Per-config throughput under cone feature / diagnostic flags.
# Usage: bash tools/gpu_cfgflags.sh TAG flags1 [flags2 ...]
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
for f in "$@"; do
  RIPTIDE_AMD_CONE_FLAGS=$f timeout -k 10 400 python -u tools/bench_configs.py > $O/configs_$f.jsonl 2>$O/configs_$f.err || { tail -20 $O/configs_$f.err; exit 1; }
  echo "== flags $f"; python3 -c "
import json
for l in open('$O/configs_$f.jsonl'):
    d=json.loads(l); print(d['config'], round(d['cone_ms_per_trial'],3), 'ms cone')"
done
