"""Per-pT census of the separable lanes of a Grad F_TB launch (skipped / Boltzmann-tail / other), from the
host build of the device math (tests/native/cf_emulator.cpp) on a cell sample of BASELINE config 2.
usage: python tools/lane_census.py [cells] | --waves (per-wavefront mix, wave_census)"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from helpers import emu_spectra, emulator  # noqa: E402
from is3d2_amd import make_spec, synth  # noqa: E402

def lane_census(n):
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=1, dimension=3, pT="pT48", phi="phi32", y="y21")
    s = synth.as_read(synth.surface(n, seed=7, dimension=3))
    npT = len(spec["pT"])
    cnt = np.zeros(npT * 3, dtype=np.int64)
    emulator().emu_set_census(cnt.ctypes.data_as(C.POINTER(C.c_long)))
    emu_spectra(spec, s, variant=3)
    cnt = cnt.reshape(npT, 3)
    tot = cnt.sum(axis=1)
    print("pT      skip   tail  other")
    for i in range(npT):
        print("%6.3f %6.3f %6.3f %6.3f" % (spec["pT"][i], cnt[i, 0] / tot[i], cnt[i, 1] / tot[i], cnt[i, 2] / tot[i]))
    a = cnt.sum(axis=0) / cnt.sum()
    print("all    %6.3f %6.3f %6.3f" % tuple(a))


def wave_census(n=60, pTs=(0, 8, 16, 24, 32, 40, 47)):
    """Per-wavefront census of the Grad F_TB launch with integrand classes: for each (pT, cell, 64-lane wave of
    class lanes, task = class + nclass q) the mix of lane kinds among its live lanes.  A wave holding both
    Boltzmann-tail and other fast lanes runs both phi loops back to back."""
    sp = make_spec(hrg_eos=2, chosen="smash", df_mode=1, dimension=3, pT="pT48", phi="phi32", y="y21")
    s = synth.as_read(synth.surface(n, seed=7, dimension=3))
    npT, ns, nq = len(sp["pT"]), len(sp["species"]["mass"]), len(sp["y"])
    buf = np.zeros(npT * n * ns * nq, dtype=np.int8)
    emulator().emu_set_census_lanes(buf.ctypes.data_as(C.c_void_p))
    emu_spectra(sp, s, variant=3)
    emulator().emu_set_census_lanes(None)
    buf = buf.reshape(npT, n, ns, nq)
    key = list(zip(sp["species"]["mass"], sp["species"]["sign"], sp["species"]["baryon"]))
    rep, seen = [], set()
    for i, k in enumerate(key):
        if k not in seen:
            seen.add(k); rep.append(i)
    nc = len(rep)
    ntask = nc * nq
    nw = (ntask + 63) // 64
    tot = {"skip": 0, "tail": 0, "near": 0, "fast": 0, "mixed": 0}
    lanes_in_mixed = 0
    for i in pTs:
        cat = buf[i][:, rep, :]                      # [cell][class][q]
        task = np.transpose(cat, (0, 2, 1)).reshape(n, ntask)   # task = class + nc q
        task = np.concatenate([task, np.zeros((n, nw * 64 - ntask), np.int8)], axis=1).reshape(n, nw, 64)
        # lane codes 1 + (skip 0 / tail 1 / other 2 / near-tail 3, cf_emulator.cpp); the device votes per wave:
        # tail if every live lane is, else near if every live lane is near or tail, else the normal fours
        has_t = (task == 2).any(axis=2); has_f = (task == 3).any(axis=2); has_n = (task == 4).any(axis=2)
        tot["mixed"] += int((has_t & has_f).sum()); tot["tail"] += int((has_t & ~has_f & ~has_n).sum())
        tot["near"] += int((has_n & ~has_f).sum())
        tot["fast"] += int((~has_t & has_f).sum()); tot["skip"] += int((~has_t & ~has_f & ~has_n).sum())
    allw = sum(tot.values())
    print("waves: " + "  ".join("%s %.3f" % (k, v / allw) for k, v in tot.items()))


if __name__ == "__main__":
    if "--waves" in sys.argv:
        wave_census()
    else:
        lane_census(int(sys.argv[1]) if len(sys.argv) > 1 else 200)
