#!/bin/bash
# One parameterised GPU-box runner (repo root, via gpurun) for every
# measurement this repo makes.  Each step runs under its own time limit and
# the first failure ends the script (no retries).  Output: gpurun_out/TAG/.
#
#   bash tools/gpu_run.sh TAG tests                 GPU parity tests + smoke
#   bash tools/gpu_run.sh TAG bench [ARGS...]        bench.py (cfg2 headline unless --workload)
#   bash tools/gpu_run.sh TAG prof                   rocprofv3 kernel-trace summary of the cfg2 bench
#   bash tools/gpu_run.sh TAG pmc [CFG]              PMC passes (4 counter groups) -> profiles/TAG_pmc_cone[_CFG].json
#   bash tools/gpu_run.sh TAG configs [LIB...]       per-config table (tools/bench_configs.py) per library
#   bash tools/gpu_run.sh TAG ab CFG LIB...          same-box A/B of builds: cone ms per trial, alternated twice
#                                                    (AB_FLAGS=v1,v2: values of AB_VAR, default RIPTIDE_AMD_CONE_FLAGS)
#   bash tools/gpu_run.sh TAG flags CFG FLAGS...     same-box A/B of RIPTIDE_AMD_CONE_FLAGS values
#   bash tools/gpu_run.sh TAG stamps CFG             per-phase stamps (libriptide_amd_stamps.so)
#   bash tools/gpu_run.sh TAG trace LIB...           per-launch cone durations of the cfg2 bench per library
#   bash tools/gpu_run.sh TAG parity LIB...          GPU parity tests (test_gpu_parity.py) per library
#   bash tools/gpu_run.sh TAG pmclib CFG LIB...      SQ counter groups of the cone kernel per library
#   bash tools/gpu_run.sh TAG pmcflags CFG FLAGS...  instruction counters per RIPTIDE_AMD_CONE_FLAGS value
#                                                    (diagnostic bits: phase attribution of VALU / SALU / LDS)
#   bash tools/gpu_run.sh TAG attrib [CFG]           phase attribution (fill / merge / S/N / skeleton alone)
#   bash tools/gpu_run.sh TAG ladder LIB...          ladder alone (tools/ladder_bench.py, cfg2) per library, alternated twice,
#                                                    then the two SQ counter groups of the ladder kernel (first library)
#   bash tools/gpu_run.sh TAG prep [ENV=V...]       dereddening + normalisation alone (tools/prep_bench.py) under
#                                                    rocprofv3 --kernel-trace --stats, once per environment setting
#   bash tools/gpu_run.sh TAG readrate [FILES]       cold-read rate of the box's storage, 1/2/4/8 readers (CPU only)
#   bash tools/gpu_run.sh TAG round                  round-end pass: attribution (cfg2), pmc (cfg2, cfg3, cfg4),
#                                                    tests, smoke, bench cfg2 / cfg3 / cfg5, configs, prof
set -o pipefail
TAG=$1; CMD=$2; shift 2
R=$(pwd)
O=$R/gpurun_out/$TAG
mkdir -p "$O"
LIB=riptide_amd/libriptide_amd.so
PMC_GROUPS=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU"
  "FETCH_SIZE"
  "WRITE_SIZE")

fail() { echo "$1 failed"; tail -25 "$2"; exit 1; }

do_tests() {
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > "$O/gpu_tests.log" 2>&1 \
    || { grep -E "FAIL|Error|assert" "$O/gpu_tests.log" | head -30; exit 1; }
  tail -1 "$O/gpu_tests.log"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || fail smoke "$O/smoke.log"
  tail -1 "$O/smoke.log"
}

do_bench() {   # $1: log name, rest: bench.py arguments
  local name=$1; shift
  timeout -k 10 900 python -u bench.py "$@" > "$O/$name.log" 2>&1 || fail "bench $*" "$O/$name.log"
  tail -1 "$O/$name.log" | cut -c1-700
}

do_prof() {
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run -f csv \
     -- python3 "$R/bench.py" --no-cpu-baseline --no-self-check > "$O/bench_prof.log" 2>&1) || fail rocprof "$O/bench_prof.log"
  tail -1 "$O/bench_prof.log" | cut -c1-300
  find "$O/prof" -name '*stats*'
  python3 tools/prof_json.py "$O/prof/run_kernel_stats.csv" "$O/bench_prof.log" "profiles/${TAG}_kernel_trace.json" \
    > "$O/prof_json.log" 2>&1 || fail prof_json "$O/prof_json.log"
  cp "profiles/${TAG}_kernel_trace.json" "$O/"
  cut -c1-400 "$O/prof_json.log"
}

do_pmc() {     # $1: cfg2 (bench.py at its batch of 16) or a config name (tools/ab_flags.py, 128 trials)
  local cfg=${1:-cfg2} d="$O/pmc_$1" i=0
  mkdir -p "$d"
  for grp in "${PMC_GROUPS[@]}"; do
    i=$((i+1))
    if [ "$cfg" = cfg2 ]; then
      (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$d/p$i" -o run \
         -- python3 "$R/bench.py" --steps 1 --warmup 1 --batch 16 --no-cpu-baseline --no-self-check > "$d/p$i.log" 2>&1) \
        || fail "pmc pass $i" "$d/p$i.log"
    else
      (cd /tmp && export TMPDIR=/tmp && export AB_BATCH=16 && timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -f csv -d "$d/p$i" -o run \
         -- python3 "$R/tools/ab_flags.py" 15 "$cfg" > "$d/p$i.log" 2>&1) || fail "pmc pass $i" "$d/p$i.log"
    fi
  done
  local out=profiles/${TAG}_pmc_cone.json
  [ "$cfg" = cfg2 ] || out=profiles/${TAG}_pmc_cone_$cfg.json
  # trials per PMC pass: bench.py at the benchmarked batch (1 warmup + 1 step x 16 trials);
  # ab_flags.py: 2 rounds x 4 runs x AB_BATCH 16 trials
  local per=32; [ "$cfg" = cfg2 ] || per=128
  python3 tools/pmc_to_json.py "$d" "$out" $per --config "$cfg" > "$d/json.log" 2>&1 || fail pmc_to_json "$d/json.log"
  cp "$out" "$O/"
  echo "pmc $cfg ok: $(head -c 300 "$d/json.log")"
}

do_configs() {
  local libs=("$@"); [ ${#libs[@]} -gt 0 ] || libs=($LIB)
  for lib in "${libs[@]}"; do
    local n=$(basename "$lib" .so)
    RIPTIDE_AMD_LIB=$lib timeout -k 10 500 python -u tools/bench_configs.py > "$O/configs_$n.jsonl" 2> "$O/configs_$n.err" \
      || fail "configs $n" "$O/configs_$n.err"
    echo "== $n"; cut -c1-220 "$O/configs_$n.jsonl"
  done
}

do_ab() {      # CFG LIB...
  local cfg=$1; shift
  for rep in 1 2; do
    for lib in "$@"; do
      local r
      r=$(RIPTIDE_AMD_LIB=$lib timeout -k 10 300 python -u tools/ab_env.py "${AB_VAR:-RIPTIDE_AMD_CONE_FLAGS}" "${AB_FLAGS:-15}" "$cfg" 2>&1 | grep '"round": 1') \
        || { echo "$lib failed"; exit 1; }
      echo "$r" | sed "s|^|$(basename "$lib") |" | tee -a "$O/ab_$cfg.log"
    done
  done
}

do_flags() {   # CFG FLAGS...
  local cfg=$1; shift
  for rep in 1 2; do
    for f in "$@"; do
      local r
      r=$(timeout -k 10 200 python -u tools/ab_flags.py "$f" "$cfg" 2>&1 | tail -1) || { echo "flags $f failed"; exit 1; }
      echo "flags=$f $r" | tee -a "$O/flags_$cfg.log"
    done
  done
}

do_stamps() {
  local cfg=${1:-cfg2}
  RIPTIDE_AMD_LIB=riptide_amd/libriptide_amd_stamps.so timeout -k 10 300 python -u tools/diag_stamps.py "${STAMPS_B:-4}" "$cfg" \
    > "$O/stamps_$cfg.json" 2> "$O/stamps_$cfg.err" || fail "stamps $cfg" "$O/stamps_$cfg.err"
  cut -c1-1500 "$O/stamps_$cfg.json"
}

do_trace() {
  for lib in "$@"; do
    local n=$(basename "$lib" .so)
    (cd /tmp && export TMPDIR=/tmp && RIPTIDE_AMD_LIB=$R/$lib timeout -k 10 400 rocprofv3 --kernel-trace -d "$O/trace_$n" \
       -o run -f csv -- python3 "$R/bench.py" --no-cpu-baseline --steps 4 > "$O/trace_$n.log" 2>&1) \
      || fail "trace $n" "$O/trace_$n.log"
    grep '^{"metric"' "$O/trace_$n.log" > "$O/trace_$n.json" || fail "trace $n (no bench line)" "$O/trace_$n.log"
    echo "== $n: $(python3 -c 'import json,sys; d=json.load(open(sys.argv[1])); print(round(d["value"],2), "trials/s", d["config"]["cone_launches_per_step"], "launches", "checked", d.get("checked"))' "$O/trace_$n.json")"
    python3 tools/prof_dispatch.py "$O/trace_$n" \
      "$(python3 -c 'import json,sys; print(json.load(open(sys.argv[1]))["config"]["cone_launches_per_step"])' "$O/trace_$n.json")" 1 4 \
      | tee "$O/trace_$n.txt"
  done
}

do_parity() {
  for lib in "$@"; do
    local n=$(basename "$lib" .so)
    RIPTIDE_AMD_LIB=$R/$lib timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 \
      --timeout-method thread > "$O/parity_$n.log" 2>&1 || { echo "$n parity FAILED"; grep -E "FAIL|Error|assert" "$O/parity_$n.log" | head -20; exit 1; }
    echo "$n parity: $(tail -1 "$O/parity_$n.log")"
  done
}

do_pmcflags() {   # CFG FLAGS...
  local cfg=$1; shift
  for f in "$@"; do
    local d="$O/pmcflags_${cfg}_$f"
    (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
       SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT \
       --kernel-trace -f csv -d "$d" -o run -- python3 "$R/tools/ab_flags.py" "$f" "$cfg" > "$d.log" 2>&1) \
      || fail "pmcflags $f" "$d.log"
    python3 - "$d" "$f" <<'PY'
import csv, glob, sys
from collections import defaultdict
S = defaultdict(float); t = 0.0
for fn in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if "cone_kernel" in r.get("Kernel_Name", ""):
            S[r["Counter_Name"]] += float(r["Counter_Value"])
for fn in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if "cone_kernel" in r["Kernel_Name"]:
            t += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
tr = 64.0
print("flags", sys.argv[2], "per trial:", {k: "%.4g" % (v / tr) for k, v in sorted(S.items())},
      "cone_ms_per_trial %.4f" % (t / tr * 1e3), "clock_GHz %.3f" % (S["GRBM_GUI_ACTIVE"] / 8 / t / 1e9 if t else 0))
PY
  done
}

do_attrib() {   # CFG: phase attribution (tools/attribution.py) -> profiles/TAG_attribution_CFG.json
  local cfg=${1:-cfg2}
  timeout -k 10 400 python -u tools/attribution.py "$cfg" "profiles/${TAG}_attribution_$cfg.json" \
    > "$O/attrib_$cfg.log" 2>&1 || fail "attrib $cfg" "$O/attrib_$cfg.log"
  cp "profiles/${TAG}_attribution_$cfg.json" "$O/"
  tail -1 "$O/attrib_$cfg.log" | cut -c1-600
}

do_pmclib() {   # CFG LIB...: the SQ counter groups of the cone kernel per library (tools/ab_flags.py, default flags 15)
  local cfg=$1; shift
  for lib in "$@"; do
    local n=$(basename "$lib" .so) i=0
    for grp in "${PMC_GROUPS[@]:0:2}"; do
      i=$((i+1))
      local d="$O/pmclib_${cfg}_${n}_p$i"
      (cd /tmp && export TMPDIR=/tmp && RIPTIDE_AMD_LIB=$R/$lib timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -f csv \
         -d "$d" -o run -- python3 "$R/tools/ab_flags.py" 15 "$cfg" > "$d.log" 2>&1) || fail "pmclib $n $i" "$d.log"
    done
    python3 - "$O" "pmclib_${cfg}_${n}" <<'PY'
import csv, glob, sys
from collections import defaultdict
S = defaultdict(float); t = 0.0
for fn in glob.glob(sys.argv[1] + "/" + sys.argv[2] + "_p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(fn)):
        if "cone_kernel" in r.get("Kernel_Name", ""):
            S[r["Counter_Name"]] += float(r["Counter_Value"])
tr = 64.0
print(sys.argv[2], "per trial:", {k: "%.4g" % (v / tr) for k, v in sorted(S.items())})
PY
  done
}

do_ladder() {  # LIB...
  for rep in 1 2; do
    for lib in "$@"; do
      RIPTIDE_AMD_LIB=$lib timeout -k 10 200 python -u tools/ladder_bench.py cfg2 16 10 2>&1 | grep '"round": 1' \
        | tee -a "$O/ladder.log" || { echo "ladder $lib failed"; exit 1; }
    done
  done
  local i=0
  for grp in "${PMC_GROUPS[@]:0:2}"; do
    i=$((i+1))
    (cd /tmp && export TMPDIR=/tmp && export RIPTIDE_AMD_LIB=$R/$1 && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -f csv \
       -d "$O/pmc_ladder/p$i" -o run -- python3 "$R/tools/ladder_bench.py" cfg2 16 2 > "$O/pmc_ladder_p$i.log" 2>&1) \
      || fail "ladder pmc $i" "$O/pmc_ladder_p$i.log"
  done
  python3 tools/pmc_to_json.py "$O/pmc_ladder" "$O/pmc_ladder.json" 96 --config cfg2 --kernel downsample_fused \
    > "$O/pmc_ladder_json.log" 2>&1 || fail pmc_ladder_json "$O/pmc_ladder_json.log"
  head -c 600 "$O/pmc_ladder_json.log"
}

do_prep() {    # ENV=V... ("-" = none)
  local settings=("$@"); [ ${#settings[@]} -gt 0 ] || settings=(-)
  local i=0
  for e in "${settings[@]}"; do
    i=$((i+1))
    local envs=(); [ "$e" = - ] || envs=("$e")
    (cd /tmp && export TMPDIR=/tmp && { [ ${#envs[@]} -eq 0 ] || export "${envs[@]}"; } && timeout -k 10 200 rocprofv3 --kernel-trace --stats \
       -d "$O/prep$i" -o run -f csv -- python3 "$R/tools/prep_bench.py" > "$O/prep$i.log" 2>&1) || fail "prep $e" "$O/prep$i.log"
    echo "== $e $(grep ms_per_run "$O/prep$i.log")"
    python3 - "$O/prep$i" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        print("  %-48s calls %5s avg_us %10.2f" % (r["Name"][:48], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  done
}

do_readrate() {   # [FILES]: cold-read rate with 1 / 2 / 4 / 8 reader processes -> profiles/TAG_read_rate.jsonl
  # /tmp (bench.py cfg5's files without TMPDIR) and the repo's own file system
  mkdir -p "$O/rr"
  timeout -k 10 600 python -u tools/read_rate.py "${1:-128}" "profiles/${TAG}_read_rate.jsonl" /tmp "$O/rr" \
    > "$O/read_rate.log" 2>&1 || fail readrate "$O/read_rate.log"
  rm -rf "$O/rr"
  cp "profiles/${TAG}_read_rate.jsonl" "$O/"
  grep 'readers' "$O/read_rate.log"
}

case "$CMD" in
  tests) do_tests ;;
  bench) do_bench bench "$@" ;;
  bench3) do_bench bench_cfg3 --workload cfg3 "$@" ;;
  bench5) do_bench bench_cfg5 --workload cfg5 "$@" ;;
  prof) do_prof ;;
  pmc) do_pmc "${1:-cfg2}" ;;
  configs) do_configs "$@" ;;
  ab) do_ab "$@" ;;
  flags) do_flags "$@" ;;
  stamps) do_stamps "$@" ;;
  trace) do_trace "$@" ;;
  parity) do_parity "$@" ;;
  pmcflags) do_pmcflags "$@" ;;
  pmclib) do_pmclib "$@" ;;
  attrib) do_attrib "$@" ;;
  ladder) do_ladder "$@" ;;
  prep) do_prep "$@" ;;
  readrate) do_readrate "$@" ;;
  round)
    RIPTIDE_AMD_SCRATCH_MFLOATS=1024 RIPTIDE_AMD_COSCHED=1 do_attrib cfg2
    do_pmc cfg2
    do_pmc cfg3
    do_pmc cfg4
    do_tests
    do_bench bench
    do_bench bench_cfg3 --workload cfg3
    do_bench bench_cfg5 --workload cfg5
    do_readrate
    do_configs
    do_prof ;;
  *) echo "unknown command $CMD"; exit 2 ;;
esac
