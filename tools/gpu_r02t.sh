set -o pipefail
mkdir -p gpurun_out/r02t
RIPTIDE_AMD_SCRATCH_MFLOATS=384 RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so timeout -k 10 200 python -u tools/diag_stamps.py 4 > gpurun_out/r02t/stamps.json 2>gpurun_out/r02t/stamps.err || { tail -5 gpurun_out/r02t/stamps.err; exit 1; }
cat gpurun_out/r02t/stamps.json
