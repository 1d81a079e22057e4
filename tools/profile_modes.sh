#!/bin/bash
# rocprofv3 passes of the bench workload for several delta-f modes (run on the GPU box from the repo root).
#   trace : --kernel-trace --stats (per-kernel durations)
#   pmcA  : SQ instruction / cycle counters + GRBM_GUI_ACTIVE (effective clock)
#   pmcE  : FP64 VALU instruction mix (ADD / MUL / FMA / TRANS), INT32 / INT64 / CVT, FP64 flops
#   pmcD  : wave-cycle breakdown and LDS (bank conflicts, LDS waits)
#   pmcB/C: FETCH_SIZE / WRITE_SIZE in separate passes (TCC slot limits, MI355X_MICROARCH.md)
#   pmcK  : scalar-cache requests / misses (the F_TS launches read their per-(cell, phi) operands by scalar loads)
# Every pass is its own process under its own time limit; the script stops at the first failure.
# usage: tools/profile_modes.sh <tag> <config> "<modes>" [bench args...]
# output: gpurun_out/prof_<tag>_<config>[_op0]_m<mode>/ (operation 0 runs get their own directory: the same tag and
# mode for both operations used to overwrite operation 1's raw CSVs)
set -e
TAG=$1; CFG=$2; MODES=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
PY=$(command -v python3)
OPN=""
case " $* " in *" --operation 0 "*) OPN="_op0" ;; esac
for M in $MODES; do
  OUT=$R/gpurun_out/prof_${TAG}_${CFG}${OPN}_m$M
  mkdir -p "$OUT"
  B="$R/bench.py --no-cpu-baseline --no-per-species --north-star-steps 0 --config $CFG --df-mode $M --steps 2 --warmup 1 $*"
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$PY" $B > "$OUT/trace.log" 2>&1
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmcA" -o run -- "$PY" $B > "$OUT/pmcA.log" 2>&1
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FLOPS_FP64 -d "$OUT/pmcE" -o run -- "$PY" $B > "$OUT/pmcE.log" 2>&1
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS -d "$OUT/pmcD" -o run -- "$PY" $B > "$OUT/pmcD.log" 2>&1
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$OUT/pmcB" -o run -- "$PY" $B > "$OUT/pmcB.log" 2>&1
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$OUT/pmcC" -o run -- "$PY" $B > "$OUT/pmcC.log" 2>&1
  timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ -d "$OUT/pmcK" -o run -- "$PY" $B > "$OUT/pmcK.log" 2>&1
  echo "mode $M profiled"
done
