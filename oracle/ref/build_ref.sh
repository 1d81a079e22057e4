#!/bin/bash
# Build oracle/_ref/ref_harness from the GSL-free reference sources, compiled where they
# lie under /root/reference (never copied), plus our own driver oracle/ref/ref_harness.cpp.
# Build container only; the GPU box uses the prebuilt binary (oracle/_ref is git-ignored,
# not gpurun-ignored).  Sources that need GSL (MomentumSpectra, DeltafData, AnisoVariables,
# EmissionFunction) are unbuildable here and are not attempted.
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
REF=/root/reference/src/cpp
OUT="$HERE/../_ref"
[ -d "$REF" ] || { echo "no /root/reference: skipping oracle/_ref"; exit 0; }
mkdir -p "$OUT"
SRCS="$REF/readindata.cpp $REF/GaussThermal.cpp $REF/LocalRestFrame.cpp $REF/Table.cpp $REF/ParameterReader.cpp $REF/Arsenal.cpp"
if [ ! -x "$OUT/ref_harness" ] || [ "$HERE/ref_harness.cpp" -nt "$OUT/ref_harness" ]; then
  g++ -std=c++11 -O2 -w -I"$REF" -o "$OUT/ref_harness" "$HERE/ref_harness.cpp" $SRCS
fi
