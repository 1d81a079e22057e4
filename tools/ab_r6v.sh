set -o pipefail
V=is3d2_amd/variants
# round 6 r6v: k_dndx's Grad / RTA-CE launches with per-(cell, phi) PD rows (pd = IS3D_DNDX_PD=1: sep_quad_pd_t /
# sep_quad_pd_tail_t fours) against default (the modified launch's {PDm, Qv} rows on, IS3D_DNDX_PDM=1); oracle suites on both
timeout -k 10 400 python -u -m pytest tests/test_gpu_dndx.py tests/test_gpu_yield.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6v_tests.log 2>&1; rc=$?; echo "default tests rc=$rc"; tail -1 gpurun_out/r6v_tests.log; [ $rc -eq 0 ] || exit $rc
IS3D_LIB=$V/pd.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dndx.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6v_tests2.log 2>&1; rc=$?; echo "pd tests rc=$rc"; tail -1 gpurun_out/r6v_tests2.log; [ $rc -eq 0 ] || exit $rc
AB_EXTRA="--operation 0" timeout -k 10 500 tools/ab.sh config2 "1 2" default $V/pd.so default $V/pd.so
