#!/bin/bash
# Run GPU steps on the gpurun box, each under its own time limit.  Exit code 0 (pass) or 1
# (test/assert failure, no crash) continues; anything else (abort 134, segv 139, timeout
# 124/137, ...) stops the session so nothing else touches the GPU after a fault.
# usage: tools/gpu_session.sh "name|seconds|command" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for step in "$@"; do
  name="${step%%|*}"; rest="${step#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "=== stopping: $name ended with rc=$rc"
    exit $rc
  fi
done
