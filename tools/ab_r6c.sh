set -o pipefail
V=is3d2_amd/variants
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r6d_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r6d_tests.log
timeout -k 10 400 tools/ab.sh config2 "1 2 3 5" default $V/base0.so $V/fdiv0.so && \
timeout -k 10 200 tools/ab.sh config2 "3 5" $V/eskip3.so default $V/base0.so
