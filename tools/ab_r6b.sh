set -o pipefail
V=is3d2_amd/variants
timeout -k 10 300 tools/ab.sh config2 "1 3" default $V/abl2.so $V/abl4.so $V/abl5.so && \
C="SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS" && \
timeout -k 10 200 tools/pmc_passes.sh config2 1 default "$C" && \
timeout -k 10 200 tools/pmc_passes.sh config2 1 $V/abl2.so "$C" && \
timeout -k 10 200 tools/pmc_passes.sh config2 1 $V/abl4.so "$C" && \
timeout -k 10 200 tools/pmc_passes.sh config2 3 default "$C" && \
timeout -k 10 200 tools/pmc_passes.sh config2 3 $V/abl1.so "$C"
