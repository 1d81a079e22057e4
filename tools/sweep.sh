#!/bin/bash
# Workload sweep on the GPU box (one JSON line per run into gpurun_out/<tag>_sweep.jsonl):
#   config2 modes 2-5 (config2 mode 1 is the default bench line), config3 modes 1-5 (shear + bulk + baryon;
#   PTB without baryon), config5 (5e6 UrQMD cells, PTMA + baryon, 64-pt GL) and operation 0 on config2.
# Every run is its own process under its own time limit; the script stops at the first failure.
# usage: tools/sweep.sh <tag> [config5 cells]
TAG=${1:-sweep}; C5=${2:-5000000}
OUT=gpurun_out/${TAG}_sweep.jsonl
mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --no-cpu-baseline --north-star-steps 0 "$@" >> "$OUT" || exit $?; }
for m in 2 3 4 5; do run --steps 3 --warmup 1 --config config2 --df-mode $m; done
for m in 1 2 3 4 5; do run --steps 2 --warmup 1 --config config3 --df-mode $m --no-per-species; done
for m in 1 3; do run --steps 2 --warmup 1 --config config2 --operation 0 --df-mode $m --no-per-species; done
run --steps 1 --warmup 1 --config config5 --cells $C5 --no-per-species
# config 1's shape (pikp 2+1D, 24 pT x 24 phi x 24 eta, 1e5 cells) in every mode
for m in 1 2 3 4 5; do run --steps 3 --warmup 1 --config config1 --cells 100000 --df-mode $m --no-per-species; done
