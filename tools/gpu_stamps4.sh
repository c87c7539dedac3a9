set -o pipefail
T=${1:-r02zg}
mkdir -p gpurun_out/$T
for lib in riptide_amd/libriptide_amd_stamps.so riptide_amd/libriptide_amd_stamps_pack.so; do
n=$(basename $lib .so)
RIPTIDE_AMD_LIB=$lib timeout -k 10 200 python -u tools/diag_stamps.py 4 cfg4 > gpurun_out/$T/stamps_$n.json 2>gpurun_out/$T/stamps_$n.err || { tail -5 gpurun_out/$T/stamps_$n.err; exit 1; }
echo "== $n"; cat gpurun_out/$T/stamps_$n.json
done
