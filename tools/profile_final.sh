#!/bin/bash
# Counter + trace passes of the BASELINE workloads on the current build (run on the GPU box from the repo root),
# one tools/profile_modes.sh call per configuration; stops at the first failure.
# usage: tools/profile_final.sh <tag> a|b   (two halves: one gpurun call holds at most 20 minutes)
set -e
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
if [ "$2" = a ]; then
  timeout -k 10 700 tools/profile_modes.sh "$TAG" config2 "1 2 3 4 5"
  timeout -k 10 400 tools/profile_modes.sh "$TAG" config4 "2"
else
  timeout -k 10 600 tools/profile_modes.sh "$TAG" config5 "5" --steps 1 --warmup 0
  timeout -k 10 300 tools/profile_modes.sh "$TAG" config3 "1 2"
  timeout -k 10 200 tools/profile_modes.sh "$TAG" config1 "1 5" --cells 100000
  timeout -k 10 300 tools/profile_modes.sh "$TAG" config2 "1 3" --operation 0
fi
