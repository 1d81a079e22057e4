set -o pipefail
V=is3d2_amd/variants
# round 6 r6h: HEAD (default) against the round-5 final build (r5final = d6c93a5), same box
timeout -k 10 300 tools/ab.sh config4 "2" default $V/r5final.so default $V/r5final.so && \
timeout -k 10 300 tools/ab.sh config2 "1 2" default $V/r5final.so default $V/r5final.so
