set -o pipefail
V=is3d2_amd/variants
# round 6 r6i: tab11 = IS3D_MOD_TAB_BITS=11 (modified lanes' own 2^(j/2048) table, degree-2 polynomial); default = HEAD
# (modified launches without the unused {b', Phi} rows); r5final = the round-5 final build d6c93a5
IS3D_LIB=$V/tab11.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6i_tests.log 2>&1; echo "tab11 tests rc=$?"; tail -3 gpurun_out/r6i_tests.log
timeout -k 10 400 tools/ab.sh config2 "5 3" default $V/tab11.so $V/r5final.so default $V/tab11.so && \
timeout -k 10 300 tools/ab.sh config4 "2" default $V/r5final.so default $V/r5final.so && \
timeout -k 10 200 tools/ab.sh config2 "1" default $V/r5final.so default $V/r5final.so
