set -o pipefail
V=is3d2_amd/variants
timeout -k 10 500 tools/ab.sh config2 "3 5" default $V/abl1.so $V/abl2.so $V/abl3.so $V/iexp.so $V/eskip3.so && \
timeout -k 10 300 tools/ab.sh config2 "1 2" default $V/abl1.so $V/abl2.so && \
timeout -k 10 200 tools/ab.sh config2 "3 5" default $V/iexp.so
