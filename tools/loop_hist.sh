#!/bin/bash
# Static VALU count of the k_spectra<MODE,0,KJ> phi loops: for each basic block holding reciprocals /
# rsq (the unrolled per-lane phi loops) print the instruction histogram.  usage: [KJ=32] tools/loop_hist.sh MODE
M=${1:-1}
cd "$(dirname "$0")/../is3d2_amd/csrc" || exit 1
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only $EXTRA -DIS3D_TU=$([ "$M" -le 2 ] && echo 12 || echo $M) -S -o /tmp/engine.s spectra_tu.hip 2>/dev/null || exit 1
awk -v pat="^_Z.*k_spectraILi${M}ELi0ELi${KJ:-32}EEEvNS[0-9_]*8SpecArgsE:" '$0 ~ pat {p=1} p && /^.Lfunc_end/ {exit} p' /tmp/engine.s > /tmp/kern.s
awk '/^.LBB/{name=$1} /v_rcp_f64|v_rsq_f64/{c[name]++} END{for(n in c) if (c[n] >= 8) print n}' /tmp/kern.s | while read b; do
  awk -v b="$b" '$1==b {p=1; next} p && /^.LBB/ {exit} p' /tmp/kern.s | grep -v "^\s*;" | awk '{print $1}' | sort | uniq -c | sort -rn |
    awk -v b="$b" 'BEGIN{printf "%s:", b} /v_|ds_/{printf " %s=%d", $2, $1; if ($2 ~ /^v_/) v+=$1} END{printf "  VALU=%d\n", v}'
done
