set -o pipefail
V=is3d2_amd/variants
# round 6 r6q: k_dndx's modified launch with 4-cell record tiles (dt4: ~28 KB of LDS, 128 VGPRs -> 4 workgroups per CU)
# against 8-cell tiles (default: 53 KB, 3 per CU); oracle suites of operation 0 on dt4
IS3D_LIB=$V/dt4.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dndx.py tests/test_gpu_yield.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6q_tests.log 2>&1; rc=$?; echo "dt4 tests rc=$rc"; tail -2 gpurun_out/r6q_tests.log; [ $rc -eq 0 ] || exit $rc
AB_EXTRA="--operation 0" timeout -k 10 500 tools/ab.sh config2 "3 4" default $V/dt4.so default $V/dt4.so
