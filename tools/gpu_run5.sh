set -e
cd $GRAFT_REPO_ROOT
tools/gpu_session.sh "gputests|800|python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread" \
  "abptm|200|tools/ab.sh config2 3 default is3d2_amd/variants/gclass1.so default is3d2_amd/variants/gclass1.so" \
  "trace_c1|300|cd /tmp && export TMPDIR=/tmp && for m in 1 5; do timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r5c_config1_m\$m -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-per-species --north-star-steps 0 --config config1 --cells 100000 --df-mode \$m --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/prof_r5c_config1_m\$m.json; done" \
  "op0|400|tools/profile_modes.sh r5c config2 3 --operation 0"
