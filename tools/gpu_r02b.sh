set -o pipefail
O=gpurun_out/r02b; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_tests.log 2>&1; rc=$?
tail -5 $O/gpu_tests.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|error" $O/gpu_tests.log | head -30; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 400 python -u bench.py --workload cfg5 --files 32 --batch 16 > $O/bench_cfg5.log 2>&1 || { tail -30 $O/bench_cfg5.log; exit 1; }
tail -1 $O/bench_cfg5.log
