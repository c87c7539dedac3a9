#!/bin/bash
set -o pipefail
O=gpurun_out/r03d
mkdir -p $O
bash tools/ab_libs.sh cfg2 riptide_amd/libriptide_amd.so riptide_amd/libriptide_amd_prio.so > $O/ab_prio.log 2>&1 || { cat $O/ab_prio.log; exit 1; }
cat $O/ab_prio.log
bash tools/pmc_conflicts.sh r03d_conf 7 1073741831 536870919 > $O/conf.log 2>&1 || { tail -20 $O/conf.log; exit 1; }
grep flags $O/conf.log
