set -o pipefail
V=is3d2_amd/variants
# round 6 r6k: HEAD (separable launches on the round-5 index arithmetic again) against r5final; GPU oracle suites of the touched code
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_north_star.py tests/test_gpu_dndx.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6k_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r6k_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/ab.sh config4 "2" default $V/r5final.so default $V/r5final.so && \
timeout -k 10 300 tools/ab.sh config2 "1 2 5" default $V/r5final.so default $V/r5final.so
