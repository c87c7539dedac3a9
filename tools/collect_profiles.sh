#!/bin/bash
# Copies one tools/gpu_final.sh pass (gpurun_out/TAG, merged back from the GPU
# box) into the tracked profiles/ directory under the same TAG.
# Usage (this container, repo root): bash tools/collect_profiles.sh TAG
set -eo pipefail
TAG=$1
O=gpurun_out/$TAG
[ -d "$O" ] || { echo "no $O"; exit 1; }
tail -1 "$O/bench.log" > profiles/${TAG}_bench.json
tail -1 "$O/bench_cfg5.log" > profiles/${TAG}_bench_cfg5.json
tail -1 "$O/bench_prof.log" > profiles/${TAG}_bench_prof.json
cp "$O/configs.jsonl" profiles/${TAG}_configs.jsonl
cp "$O/gpu_tests.log" profiles/${TAG}_gpu_tests.log
cp "$O/${TAG}_pmc_cone.json" profiles/${TAG}_pmc_cone.json
python3 tools/prof_summary.py "$O/prof/run_kernel_stats.csv" profiles/${TAG}_bench_kernel_stats.csv > /dev/null
python3 - "$TAG" <<'EOF'
import json, sys
t = sys.argv[1]
b = json.load(open(f"profiles/{t}_bench.json"))
r = b["roofline"]
print(f"{t}: {b['value']:.2f} trials/s, cone {r['kernel_ms_per_step'] / b['config']['trials_per_step_per_gpu']:.3f} ms/trial, "
      f"frac {r['frac']:.4f}, traffic {r['traffic_status']}, cpu {b['cpu_baseline']['value']:.2f} trials/s")
EOF
