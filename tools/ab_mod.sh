set -o pipefail
for m in 3 4 5; do
  python bench.py --no-cpu-baseline --steps 2 --warmup 1 --config config3 --df-mode $m || exit $?
  IS3D_LIB=is3d2_amd/variants/mod_w3.so python bench.py --no-cpu-baseline --steps 2 --warmup 1 --config config3 --df-mode $m || exit $?
done
