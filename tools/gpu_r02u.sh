set -o pipefail
bash tools/gpu_ab.sh r02u 3 || exit 1
RIPTIDE_AMD_SCRATCH_MFLOATS=384 RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so timeout -k 10 200 python -u tools/diag_stamps.py 4 > gpurun_out/r02u/stamps.json 2>gpurun_out/r02u/stamps.err || { tail -5 gpurun_out/r02u/stamps.err; exit 1; }
cat gpurun_out/r02u/stamps.json
