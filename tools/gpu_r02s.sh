set -o pipefail
bash tools/gpu_ab.sh r02s 3 16777219 || exit 1
for f in 3 16777219; do
RIPTIDE_AMD_CONE_FLAGS=$f RIPTIDE_AMD_SCRATCH_MFLOATS=384 RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so timeout -k 10 200 python -u tools/diag_stamps.py 4 > gpurun_out/r02s/stamps_$f.json 2>gpurun_out/r02s/stamps_$f.err || { tail -5 gpurun_out/r02s/stamps_$f.err; exit 1; }
cat gpurun_out/r02s/stamps_$f.json
done
