#!/bin/bash
# Same-box A/B of engine builds over configurations (GPU box, repo root):
# parity tests per library, then ms per trial (default cone flags) for each
# library and config, alternating twice.
# Usage: CFGS="cfg2 cfg4" bash tools/ab_cfgs.sh TAG libA.so libB.so ...
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
CFGS=${CFGS:-"cfg2 cfg4"}
for lib in "$@"; do
  n=$(basename $lib .so)
  if [ -z "$NO_PARITY" ]; then
    RIPTIDE_AMD_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/parity_$n.log 2>&1 || { echo "$n parity FAILED"; grep -E "FAIL|Error|assert" $O/parity_$n.log | head -20; exit 1; }
    echo "$n parity: $(tail -1 $O/parity_$n.log)"
  fi
done
for rep in 1 2; do
  for lib in "$@"; do
    n=$(basename $lib .so)
    for c in $CFGS; do
      RIPTIDE_AMD_LIB=$lib timeout -k 10 200 python -u tools/ab_flags.py 3 $c > $O/ab_${n}_${c}_$rep.log 2>&1 || { tail -5 $O/ab_${n}_${c}_$rep.log; exit 1; }
      python3 -c "import json; r=[json.loads(l) for l in open('$O/ab_${n}_${c}_$rep.log') if l.startswith('{')]; print('$n $c', ' '.join('%.3f' % d['ms_per_trial'] for d in r))"
    done
  done
done
