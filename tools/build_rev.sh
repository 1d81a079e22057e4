#!/bin/bash
# Build libis3d_amd.so from a git revision into is3d2_amd/variants/<name>.so (A/B against the working tree).
# usage: tools/build_rev.sh <rev> <name>
set -e
REV=$1; NAME=$2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/is3d_rev_XXXX)
git -C "$R" archive "$REV" is3d2_amd/csrc include | tar -x -C "$T"
make -s -j8 -C "$T/is3d2_amd/csrc" > /dev/null
mkdir -p "$R/is3d2_amd/variants"
cp "$T/is3d2_amd/libis3d_amd.so" "$R/is3d2_amd/variants/$NAME.so"
rm -rf "$T"
echo "built $REV -> is3d2_amd/variants/$NAME.so"
