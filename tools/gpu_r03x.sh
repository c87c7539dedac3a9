#!/bin/bash
# Round-3 measurement pass at HEAD (GPU box, repo root): PMC passes -> the
# traffic summary bench.py reads, GPU tests, smoke, the cfg2 headline bench
# (CPU baselines), the cfg3 job leg (BASELINE configs[2]), the cfg5 files leg
# (cold / warm, CPU baseline), the per-config table, a rocprofv3 kernel-trace
# summary of the headline bench.  Usage: bash tools/gpu_r03x.sh TAG
set -o pipefail
TAG=${1:-r03x}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
bash tools/gpu_pmc.sh ${TAG}_pmc > "$O/pmc.log" 2>&1 || { tail -20 "$O/pmc.log"; exit 1; }
python3 tools/pmc_to_json.py gpurun_out/${TAG}_pmc profiles/${TAG}_pmc_cone.json 4 > "$O/pmc_json.log" 2>&1 || { cat "$O/pmc_json.log"; exit 1; }
cp profiles/${TAG}_pmc_cone.json "$O/"
echo "pmc ok"
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { grep -E "FAIL|Error" "$O/gpu_tests.log" | head -20; exit 1; }
tail -1 "$O/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 600 python -u bench.py > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log" | cut -c1-400
timeout -k 10 900 python -u bench.py --workload cfg3 > "$O/bench_cfg3.log" 2>&1 || { tail -20 "$O/bench_cfg3.log"; exit 1; }
tail -1 "$O/bench_cfg3.log" | cut -c1-300
timeout -k 10 900 python -u bench.py --workload cfg5 > "$O/bench_cfg5.log" 2>&1 || { tail -20 "$O/bench_cfg5.log"; exit 1; }
tail -1 "$O/bench_cfg5.log" | cut -c1-300
timeout -k 10 400 python -u tools/bench_configs.py > "$O/configs.jsonl" 2> "$O/configs.err" || { tail -20 "$O/configs.err"; exit 1; }
cut -c1-200 "$O/configs.jsonl"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -f csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/bench_prof.log" 2>&1 || { tail -20 "$O/bench_prof.log"; exit 1; }
tail -1 "$O/bench_prof.log" | cut -c1-300
find "$O/prof" -name '*stats*'
