#!/bin/bash
# A/B of engine builds: tools/ab.sh <config> "<modes>" <lib.so|default> [<lib.so|default> ...]
# Prints one compact line per (mode, build): value and the k_spectra / pass times (HIP events).
CFG=$1; MODES=$2; shift 2
EXTRA=${AB_EXTRA:-}
for m in $MODES; do
  for LIB in "$@"; do
    if [ "$LIB" = default ]; then L=""; else L="$LIB"; fi
    IS3D_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-per-species --north-star-steps 0 --steps 3 --warmup 1 \
      --config "$CFG" --df-mode "$m" $EXTRA > /tmp/ab_out.json || exit $?
    python - "$m" "${LIB##*/}" <<'PY'
import json, sys
r = json.loads(open("/tmp/ab_out.json").read().strip().splitlines()[-1])
print("mode %s %-14s value %.4e  k_spectra %.1f ms  pass %.1f ms" % (sys.argv[1], sys.argv[2], r["value"],
      r["roofline"]["kernel_ms"], r["roofline"]["pass_ms"]), flush=True)
PY
  done
done
