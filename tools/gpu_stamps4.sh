set -o pipefail
T=${1:-r02zk}
CFG=${2:-cfg4}
mkdir -p gpurun_out/$T
RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so timeout -k 10 200 python -u tools/diag_stamps.py 4 $CFG > gpurun_out/$T/stamps_$CFG.json 2>gpurun_out/$T/stamps_$CFG.err || { tail -5 gpurun_out/$T/stamps_$CFG.err; exit 1; }
cat gpurun_out/$T/stamps_$CFG.json
