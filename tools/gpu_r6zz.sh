set -o pipefail
# round 6 r6zz: the whole GPU tier on the final tree (build e0d2a2c88be8, clean build(); + the config-3 full-size cases)
timeout -k 10 880 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > gpurun_out/r6zz_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; grep -E "passed|failed" gpurun_out/r6zz_tests.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6zz_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r6zz_smoke.log; exit $rc
