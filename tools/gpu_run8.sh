set -e
cd $GRAFT_REPO_ROOT
tools/gpu_session.sh \
  "fbtests|600|python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_dndx.py tests/test_gpu_classes.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread" \
  "abtile|300|tools/ab.sh config2 \"3 5\" default is3d2_amd/variants/ktile9.so default is3d2_amd/variants/ktile9.so" \
  "trace5|300|cd /tmp && export TMPDIR=/tmp && timeout -s KILL 250 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r5e_config5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-per-species --north-star-steps 0 --config config5 --steps 1 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_r5e_config5.json"
