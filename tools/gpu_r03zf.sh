#!/bin/bash
# Short-row S/N lane groups (RT_SNR_SHORT_G = 4 / 2 vs 8): parity of each
# alternative build, then the same-box cone A/B on cfg4.
# Usage: bash tools/gpu_r03zf.sh TAG
set -o pipefail
TAG=${1:-r03zf}
O=gpurun_out/$TAG; mkdir -p $O
for n in g4 g2; do
  RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_$n.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/parity_$n.log 2>&1 || { echo "$n parity FAILED"; grep -E "FAIL|Error|assert" $O/parity_$n.log | head -20; exit 1; }
  echo "$n parity: $(tail -1 $O/parity_$n.log)"
done
bash tools/ab_libs.sh cfg4 riptide_amd/libriptide_amd.so riptide_amd/libriptide_amd_g4.so riptide_amd/libriptide_amd_g2.so 2>&1 | tee $O/ab_cfg4.log
