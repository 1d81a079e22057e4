set -o pipefail
V=is3d2_amd/variants
# round 6 r6r: k_dndx's Grad / RTA-CE launches with 4-cell record tiles (dtg4) against 8 (default); the default build has
# the modified launch at 4 (r6q); oracle suites of operation 0 on the default build and on dtg4
timeout -k 10 400 python -u -m pytest tests/test_gpu_dndx.py tests/test_gpu_yield.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6r_tests.log 2>&1; rc=$?; echo "default tests rc=$rc"; tail -1 gpurun_out/r6r_tests.log; [ $rc -eq 0 ] || exit $rc
IS3D_LIB=$V/dtg4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dndx.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6r_tests2.log 2>&1; rc=$?; echo "dtg4 tests rc=$rc"; tail -1 gpurun_out/r6r_tests2.log; [ $rc -eq 0 ] || exit $rc
AB_EXTRA="--operation 0" timeout -k 10 500 tools/ab.sh config2 "1 2" default $V/dtg4.so default $V/dtg4.so && \
AB_EXTRA="--operation 0" timeout -k 10 300 tools/ab.sh config2 "3 4" default $V/r5final.so
