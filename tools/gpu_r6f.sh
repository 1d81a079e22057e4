set -o pipefail
timeout -k 10 700 python -u -m pytest tests/test_gpu_dndx.py tests/test_gpu_parity.py tests/test_gpu_configs.py tests/test_gpu_classes.py tests/test_gpu_north_star.py tests/test_gpu_chains.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6f_tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r6f_tests.log
timeout -k 10 300 tools/ab.sh config2 "1 2 3 5" default
