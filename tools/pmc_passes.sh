#!/bin/bash
# Counter passes of one engine build on one workload, one rocprofv3 process per pass (each its own time limit):
#   tools/pmc_passes.sh <config> <mode> <lib.so|default> "<counters>" ["<counters>" ...]
# prints the k_spectra totals per pass (summed over the launches of one bench step).
CFG=$1; M=$2; LIB=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
PY=$(command -v python3)
if [ "$LIB" = default ]; then L=""; else L="$R/$LIB"; fi
N=$(basename "$LIB" .so)
B="$R/bench.py --no-cpu-baseline --no-per-species --north-star-steps 0 --config $CFG --df-mode $M --steps 1 --warmup 0"
i=0
for C in "$@"; do
  i=$((i + 1))
  OUT=$R/gpurun_out/pmcp_${CFG}_m${M}_${N}_$i
  IS3D_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $C -d "$OUT" -o run -- "$PY" $B > "$OUT.log" 2>&1 || exit $?
  "$PY" - "$OUT" "$N" <<'PY'
import csv, glob, sys
from collections import defaultdict
out, n = sys.argv[1], sys.argv[2]
acc = defaultdict(float)
for f in glob.glob(out + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_spectra" in r["Kernel_Name"]:
            acc[r["Counter_Name"]] += float(r["Counter_Value"])
print(n, " ".join("%s=%.4g" % (k, v) for k, v in sorted(acc.items())), flush=True)
PY
done
