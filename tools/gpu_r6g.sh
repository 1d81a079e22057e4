set -o pipefail
timeout -k 10 880 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6g_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r6g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u bench.py > gpurun_out/r6g_bench.json 2> gpurun_out/r6g_bench.err; rc=$?; echo "bench rc=$rc"; tail -c 3000 gpurun_out/r6g_bench.json; exit $rc
