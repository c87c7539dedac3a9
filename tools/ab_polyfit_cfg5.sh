set -o pipefail
mkdir -p gpurun_out/r06zr
timeout -k 10 120 python -u tools/import_order_check.py > gpurun_out/r06zr/import_order.log 2>&1 || exit 1
timeout -k 10 500 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread -k "peak or cfg5 or e2e or find or search or pipeline" > gpurun_out/r06zr/tests.log 2>&1 || exit 1
for v in loop batched loop batched; do
  if [ $v = loop ]; then
    timeout -k 10 300 python -u -c "import sys, runpy, torch, numpy as np; import riptide_amd.peaks as P; P.polyfit_columns = lambda x, Y, d: np.array([np.polyfit(x, y, d) for y in Y]); sys.argv = ['bench.py', '--workload', 'cfg5', '--no-cpu-baseline']; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/r06zr/b_$v.log 2>&1 || exit 1
  else
    timeout -k 10 300 python -u bench.py --workload cfg5 --no-cpu-baseline > gpurun_out/r06zr/b_$v.log 2>&1 || exit 1
  fi
  grep "^{" gpurun_out/r06zr/b_$v.log | tail -1 | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],2), round(d['warm']['value'],2), d['config']['peaks_found'], d['config']['clusters_found'])" >> gpurun_out/r06zr/ab_cfg5.log
done
cat gpurun_out/r06zr/ab_cfg5.log
