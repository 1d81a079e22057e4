set -o pipefail
V=is3d2_amd/variants
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dndx.py tests/test_gpu_north_star.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6e_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r6e_tests.log
timeout -k 10 300 tools/ab.sh config2 "1 2" default $V/inva0.so default $V/inva0.so && \
timeout -k 10 200 tools/ab.sh config3 "1 2" default $V/inva0.so && \
AB_EXTRA="--operation 0" timeout -k 10 300 tools/ab.sh config2 "1 3" default $V/base0.so $V/inva0.so
