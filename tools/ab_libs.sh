#!/bin/bash
# Same-box A/B of engine builds (GPU box): ms per cfg2 trial for each library,
# alternating twice.  Usage: bash tools/ab_libs.sh libA.so libB.so ...
set -o pipefail
for rep in 1 2; do
  for lib in "$@"; do
    r=$(RIPTIDE_AMD_LIB=$lib timeout -k 10 120 python -u tools/ab_flags.py 1 2>&1 | tail -1) || { echo "$lib failed"; exit 1; }
    echo "$lib $r"
  done
done
