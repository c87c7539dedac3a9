set -o pipefail
bash tools/gpu_ab.sh r02j 3 || exit 1
RIPTIDE_AMD_CONE_PERSIST=0 timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/r02j/bench_np.log 2>&1 || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/r02j/bench_np.log').read().strip().splitlines()[-1]); r=d['roofline']; print('nonpersist', round(d['value'],2), round(r['kernel_ms_per_step']/16,3))"
RIPTIDE_AMD_SCRATCH_MFLOATS=384 RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so timeout -k 10 200 python -u tools/diag_stamps.py 4 > gpurun_out/r02j/stamps.json 2>gpurun_out/r02j/stamps.err; cat gpurun_out/r02j/stamps.json
