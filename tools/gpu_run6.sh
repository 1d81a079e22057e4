set -e
cd $GRAFT_REPO_ROOT
tools/gpu_session.sh "abaniso|300|tools/ab.sh config1 5 default is3d2_amd/variants/afast0.so is3d2_amd/variants/afast2.so default is3d2_amd/variants/afast0.so is3d2_amd/variants/afast2.so" \
  "abaniso2|300|AB_EXTRA='--cells 100000' tools/ab.sh config1 5 default is3d2_amd/variants/afast0.so default is3d2_amd/variants/afast0.so" \
  "abaniso5|200|tools/ab.sh config2 5 default is3d2_amd/variants/afast0.so" \
  "slots|300|for sl in 16384 2048 1536 1024 512; do echo slots \$sl; IS3D_CHAIN_SLOTS=\$sl AB_EXTRA='--cells 100000' tools/ab.sh config1 5 default; done" \
  "chains|600|python -u -m pytest tests/test_gpu_chains.py tests/test_gpu_group.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread"
