set -o pipefail
V=is3d2_amd/variants
# round 6 r6aa: the whole engine compiled with -mllvm -amdgpu-sched-strategy=max-ilp (ilp) against the final build (default)
timeout -k 10 400 tools/ab.sh config2 "1 2 5" default $V/ilp.so default $V/ilp.so && \
timeout -k 10 300 tools/ab.sh config4 "2" default $V/ilp.so
