#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# Usage (from the repo root, on the GPU box via gpurun): bash tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-r01}
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/gpu_tests.log" 2>&1 || { echo "gpu tests failed"; tail -30 "$O/gpu_tests.log"; exit 1; }
tail -3 "$O/gpu_tests.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -30 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 400 python -u bench.py > "$O/bench.log" 2>&1 || { echo "bench failed"; tail -30 "$O/bench.log"; exit 1; }
tail -1 "$O/bench.log"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -f csv -- python3 "$R/bench.py" --no-cpu-baseline > "$O/bench_prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$O/bench_prof.log"; exit 1; }
tail -1 "$O/bench_prof.log"
find "$O/prof" -name '*stats*' | head
