"""Per-pT census of the separable lanes of a Grad F_TB launch (skipped / Boltzmann-tail / other), from the
host build of the device math (tests/native/cf_emulator.cpp) on a cell sample of BASELINE config 2.
usage: python tools/lane_census.py [cells]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from helpers import emu_spectra, emulator  # noqa: E402
from is3d2_amd import make_spec, synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
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
