#!/bin/bash
# A/B of engine builds across df modes on config2: tools/ab_modes.sh <lib.so|default> [modes...]
LIB=$1; shift
MODES=${@:-1 2 3 4 5}
for m in $MODES; do
  if [ "$LIB" = default ]; then
    python bench.py --no-cpu-baseline --steps 2 --warmup 1 --df-mode $m || exit $?
  else
    IS3D_LIB=$LIB python bench.py --no-cpu-baseline --steps 2 --warmup 1 --df-mode $m || exit $?
  fi
done
