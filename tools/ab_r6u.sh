set -o pipefail
V=is3d2_amd/variants
# round 6 r6u: k_dndx's modified launch with per-(cell, phi) {PDm, Qv} rows (pdm = IS3D_DNDX_PDM=1: p.dsigma in one op)
# against the final build 36fe6b8ec066 (default); operation-0 oracle suites on pdm
IS3D_LIB=$V/pdm.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dndx.py tests/test_gpu_yield.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6u_tests.log 2>&1; rc=$?; echo "pdm tests rc=$rc"; tail -1 gpurun_out/r6u_tests.log; [ $rc -eq 0 ] || exit $rc
AB_EXTRA="--operation 0" timeout -k 10 500 tools/ab.sh config2 "3 4" default $V/pdm.so default $V/pdm.so
