#!/bin/bash
# Round-end measurement pass on one GPU box (repo root):
#   PMC passes -> profiles/<TAG>_pmc_cone.json (so bench.py's traffic is current),
#   parity tests, smoke, bench (cfg2 with cpu_baseline, cfg5), rocprofv3
#   kernel-trace summary, per-config table.  Everything lands in gpurun_out/<TAG>.
# Usage: bash tools/gpu_final.sh TAG
set -o pipefail
TAG=${1:-r02f}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
bash tools/gpu_pmc.sh ${TAG}_pmc > "$O/pmc.log" 2>&1 || { tail -20 "$O/pmc.log"; exit 1; }
python3 tools/pmc_to_json.py gpurun_out/${TAG}_pmc profiles/${TAG}_pmc_cone.json 4 > "$O/pmc_json.log" 2>&1 || { cat "$O/pmc_json.log"; exit 1; }
cp profiles/${TAG}_pmc_cone.json "$O/"
echo "pmc ok: $(cat $O/pmc_json.log | head -c 300)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { grep -E "FAIL|Error" "$O/gpu_tests.log" | head -20; exit 1; }
tail -1 "$O/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 500 python -u bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | head -c 600; echo
timeout -k 10 400 python -u bench.py --workload cfg5 --files 32 --batch 16 --no-cpu-baseline > "$O/bench_cfg5.log" 2>&1 || { tail -20 "$O/bench_cfg5.log"; exit 1; }
tail -1 "$O/bench_cfg5.log" | head -c 300; echo
timeout -k 10 400 python -u tools/bench_configs.py > "$O/configs.jsonl" 2> "$O/configs.err" || { tail -20 "$O/configs.err"; exit 1; }
cat "$O/configs.jsonl" | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -f csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
tail -1 "$O/bench_prof.log" | head -c 300; echo
find "$O/prof" -name '*stats*'
