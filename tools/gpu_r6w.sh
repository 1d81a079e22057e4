set -o pipefail
# round 6 r6w: the whole GPU tier on the final build e0d2a2c88be8 (slowest tests listed), then the default bench line and the config-5 line
timeout -k 10 880 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=30 > gpurun_out/r6w_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r6w_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py > gpurun_out/r6w_bench_default.json 2> gpurun_out/r6w_bench_default.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config config5 --no-cpu-baseline --north-star-steps 0 --no-per-species --steps 2 --warmup 1 > gpurun_out/r6w_bench_config5.json 2> gpurun_out/r6w_bench_config5.err; rc=$?; echo "bench config5 rc=$rc"; exit $rc
