set -o pipefail
# round 6 r6y: the default bench line and the config-5 line on the final build e0d2a2c88be8 with its committed counter profiles (r6x)
timeout -k 10 300 python -u bench.py > gpurun_out/r6y_bench_default.json 2> gpurun_out/r6y_bench_default.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config config5 --no-cpu-baseline --north-star-steps 0 --no-per-species --steps 2 --warmup 1 > gpurun_out/r6y_bench_config5.json 2> gpurun_out/r6y_bench_config5.err; rc=$?; echo "bench config5 rc=$rc"; exit $rc
