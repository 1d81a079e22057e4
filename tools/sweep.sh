#!/bin/bash
# Mode sweep on the GPU box: config3 (shear + bulk + baryon; PTB without baryon) for every
# delta-f mode, then the config5 stress case on a cell prefix.  usage: tools/sweep.sh [config5 cells]
C5=${1:-1000000}
for m in 1 2 3 4 5; do
  python bench.py --no-cpu-baseline --steps 2 --warmup 1 --config config3 --df-mode $m || exit $?
done
python bench.py --no-cpu-baseline --steps 1 --warmup 1 --config config5 --cells $C5 || exit $?
