#!/bin/bash
# Short-row task stores as 16-byte buffer stores (RT_PACK_STORE16): parity of
# the build, then the same-box cone A/B on cfg4.  Usage: bash tools/gpu_r03zi.sh TAG
set -o pipefail
TAG=${1:-r03zi}
O=gpurun_out/$TAG; mkdir -p $O
L=riptide_amd/libriptide_amd
RIPTIDE_AMD_LIB=${L}_ps16.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > $O/parity_ps16.log 2>&1 || { echo "ps16 parity FAILED"; grep -E "FAIL|Error|assert" $O/parity_ps16.log | head -20; exit 1; }
echo "ps16 parity: $(tail -1 $O/parity_ps16.log)"
bash tools/ab_libs.sh cfg4 $L.so ${L}_ps16.so 2>&1 | tee $O/ab_cfg4.log
