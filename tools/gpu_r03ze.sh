#!/bin/bash
# HEAD measurement pass (tools/gpu_r03x.sh) + the cfg2 / cfg3 per-launch
# tails from the stamps build.  Usage: bash tools/gpu_r03ze.sh TAG
set -o pipefail
TAG=${1:-r03ze}
bash tools/gpu_r03x.sh $TAG || exit 1
O=gpurun_out/$TAG
for cb in cfg2:16:1536 cfg2:16:384 cfg3:32:384; do
  IFS=: read c b s <<< "$cb"
  RIPTIDE_AMD_SCRATCH_MFLOATS=$s RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so timeout -k 10 300 python -u tools/diag_stamps.py $b $c > $O/stamps_${c}_s$s.json 2>$O/stamps_${c}_s$s.err || { tail -5 $O/stamps_${c}_s$s.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['launch_tails'])" $O/stamps_${c}_s$s.json | cut -c1-300
done
