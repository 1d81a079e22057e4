#!/bin/bash
# Counter A/B of engine builds on one workload: tools/pmc_ab.sh <config> <mode> <lib.so|default> ...
# Per build: one --pmc pass of the VALU / LDS / wait counters (each pass its own process and time limit);
# prints k_spectra's per-launch averages.
CFG=$1; M=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
PY=$(command -v python3)
for LIB in "$@"; do
  if [ "$LIB" = default ]; then L=""; else L="$R/$LIB"; fi
  N=$(basename "$LIB" .so)
  OUT=$R/gpurun_out/pmcab_${CFG}_m${M}_$N
  B="$R/bench.py --no-cpu-baseline --north-star-steps 0 --config $CFG --df-mode $M --steps 1 --warmup 0"
  IS3D_LIB=$L timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d "$OUT/a" -o run -- "$PY" $B > "$OUT.a.log" 2>&1 || exit $?
  IS3D_LIB=$L timeout -s KILL 180 rocprofv3 --kernel-trace --output-format csv --pmc SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FLOPS_FP64 -d "$OUT/e" -o run -- "$PY" $B > "$OUT.e.log" 2>&1 || exit $?
  "$PY" - "$OUT" "$N" <<'PY'
import csv, glob, sys
from collections import defaultdict
out, n = sys.argv[1], sys.argv[2]
acc = defaultdict(float); dur = []
for f in glob.glob(out + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "k_spectra" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(n, " ".join("%s=%.4g" % (k, v) for k, v in sorted(acc.items())), flush=True)
PY
done
