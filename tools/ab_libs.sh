#!/bin/bash
# Same-box A/B of engine builds (GPU box): cone ms per trial for each library
# on one config (tools/ab_env.py, default feature bits), libraries alternated
# twice.  Usage: bash tools/ab_libs.sh CFG libA.so libB.so ...
set -o pipefail
CFG=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    r=$(RIPTIDE_AMD_LIB=$lib timeout -k 10 200 python -u tools/ab_env.py RIPTIDE_AMD_CONE_FLAGS 7 $CFG 2>&1 | grep '"round": 1') || { echo "$lib failed"; exit 1; }
    echo "$(basename $lib) $r"
  done
done
