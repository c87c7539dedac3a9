#!/bin/bash
# Same-box A/B of the fused ladder's RIPTIDE_AMD_DS_VARIANT values (and of
# extra libraries) on cfg2: tools/ladder_bench.py, alternated twice.
# usage: bash tools/ladder_variants.sh TAG "0 1 2" [LIB...]
set -o pipefail
TAG=$1; VARS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p "$O"
for rep in 1 2; do
  for v in $VARS; do
    RIPTIDE_AMD_DS_VARIANT=$v timeout -k 10 200 python -u tools/ladder_bench.py cfg2 16 10 2>&1 | grep '"round": 1' \
      | sed "s/^/variant=$v /" | tee -a "$O/ladder_variants.log" || { echo "variant $v failed"; exit 1; }
  done
  for lib in "$@"; do
    RIPTIDE_AMD_LIB=$lib timeout -k 10 200 python -u tools/ladder_bench.py cfg2 16 10 2>&1 | grep '"round": 1' \
      | tee -a "$O/ladder_variants.log" || { echo "$lib failed"; exit 1; }
  done
done
