#!/bin/bash
# A/B of is3d_set_tuning knobs on one workload: tools/ab_tune.sh <config> <mode> "<knobs>" ["<knobs>" ...]
# each argument is one run's space-separated KEY=VALUE list ("" = defaults); prints value, k_spectra / pass times and splits
CFG=$1; M=$2; shift 2
for T in "$@"; do
  A=""; for kv in $T; do A="$A --tune $kv"; done
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-per-species --north-star-steps 0 --steps ${AB_STEPS:-2} --warmup 1 \
    --config "$CFG" --df-mode "$M" $A > /tmp/ab_tune.json || exit $?
  python - "$T" <<'PY'
import json, sys
r = json.loads(open("/tmp/ab_tune.json").read().strip().splitlines()[-1])
print("[%s] value %.4e  k_spectra %.1f ms  pass %.1f ms  splits %s" % (sys.argv[1] or "defaults", r["value"],
      r["roofline"]["kernel_ms"], r["roofline"]["pass_ms"], r["config"].get("cell_splits")), flush=True)
PY
done
