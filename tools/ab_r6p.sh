set -o pipefail
V=is3d2_amd/variants
# round 6 r6p: k_dndx's PTM renorm factors per (cell, species) instead of per lane and no {b', Phi} rows in the modified
# launch (PTM: 69 -> 53 KB of LDS, 2 -> 3 workgroups per CU); default = this build, r5final = the round-5 final build
timeout -k 10 400 python -u -m pytest tests/test_gpu_dndx.py tests/test_gpu_yield.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6p_tests.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r6p_tests.log; [ $rc -eq 0 ] || exit $rc
AB_EXTRA="--operation 0" timeout -k 10 500 tools/ab.sh config2 "3 4 1" default $V/r5final.so default $V/r5final.so
