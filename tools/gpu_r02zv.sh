set -o pipefail
bash tools/gpu_ab.sh r02zv 3 || exit 1
bash tools/gpu_pmc.sh r02zv_pmc > gpurun_out/r02zv/pmc.log 2>&1 || { tail -5 gpurun_out/r02zv/pmc.log; exit 1; }
python3 tools/pmc_to_json.py gpurun_out/r02zv_pmc gpurun_out/r02zv/pmc.json 4 | cut -c1-200
python3 -c "
import json; sq=json.load(open('gpurun_out/r02zv/pmc.json'))['sq']
print({k: '%.3g' % (v/4) for k, v in sq.items()})"
