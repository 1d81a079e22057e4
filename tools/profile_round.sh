#!/bin/bash
# rocprofv3 recipe for the bench workload (run on the GPU box from the repo root).
#   trace : --kernel-trace --stats (per-kernel durations)
#   pmcA  : SQ instruction / cycle counters + GRBM_GUI_ACTIVE (effective clock)
#   pmcD  : wave-cycle breakdown (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES) and LDS
#   pmcB/C: FETCH_SIZE / WRITE_SIZE in separate passes (TCC slot limits, MI355X_MICROARCH.md)
# usage: tools/profile_round.sh <tag> [bench args...]
set -e
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
PY=$(command -v python3)
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- "$PY" "$R/bench.py" --no-cpu-baseline --no-per-species --north-star-steps 0 "$@"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/pmcA" -o run -- "$PY" "$R/bench.py" --no-cpu-baseline --no-per-species --north-star-steps 0 "$@"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS -d "$OUT/pmcD" -o run -- "$PY" "$R/bench.py" --no-cpu-baseline --no-per-species --north-star-steps 0 "$@"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d "$OUT/pmcB" -o run -- "$PY" "$R/bench.py" --no-cpu-baseline --no-per-species --north-star-steps 0 "$@"
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d "$OUT/pmcC" -o run -- "$PY" "$R/bench.py" --no-cpu-baseline --no-per-species --north-star-steps 0 "$@"
