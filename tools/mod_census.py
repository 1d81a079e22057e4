"""Per-wavefront census of the modified (PTM / PTB / PTMA) table lanes of k_spectra on a cell sample of BASELINE
config 2, from the host build of the device math (tests/native/cf_emulator.cpp, variant 4 | 16).

For every live lane the emulator records its margin k - chem log2(e): the binades between the smallest
E = e^x 2^-k of its phi points and |s| = e^chem 2^-k, so u = s / E <= 2^-margin at every point.  The device votes
per wavefront (64 consecutive class + nclass * q tasks of one cell and pT): the Boltzmann-tail fours when every live
lane has margin > 55, else the normal fours.  This prints the share of wavefronts (and of live lane-points)
whose smallest live margin clears a threshold t -- the candidates for a near-tail form that replaces the shared
reciprocal by 1 / (1 + u) = 1 - u + ... (t = 27: first order, t = 18: second order).
usage: python tools/mod_census.py [mode=3] [cells=40]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from helpers import emu_spectra, emulator  # noqa: E402
from is3d2_amd import make_spec, synth  # noqa: E402


def census(mode=3, n=40, thresholds=(55, 40, 30, 27, 24, 20, 18, 14, 10)):
    sp = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=3, pT="pT48", phi="phi32", y="y21")
    s = synth.as_read(synth.surface(n, seed=7, dimension=3, full3d=True))
    npT, ns, nq = len(sp["pT"]), len(sp["species"]["mass"]), len(sp["y"])
    lanes = np.zeros(npT * n * ns * nq, dtype=np.int8)
    marg = np.full(npT * n * ns * nq, 255, dtype=np.uint8)
    cnt = np.zeros(4, dtype=np.int64)
    lib = emulator()
    lib.emu_set_census_mod(cnt.ctypes.data_as(C.POINTER(C.c_long)))
    lib.emu_set_census_lanes(lanes.ctypes.data_as(C.c_void_p))
    lib.emu_set_census_margin(marg.ctypes.data_as(C.c_void_p))
    emu_spectra(sp, s, variant=4 | 16)
    lib.emu_set_census_lanes(None)
    lib.emu_set_census_margin(None)
    lib.emu_set_census_mod(None)
    marg = marg.reshape(npT, n, ns, nq)
    lanes = lanes.reshape(npT, n, ns, nq)
    spc = sp["species"]
    key = list(zip(spc["mass"], spc["sign"], spc["baryon"], np.asarray(spc["degen"]) == 0))
    rep, seen = [], set()
    for i, k in enumerate(key):
        if k not in seen:
            seen.add(k)
            rep.append(i)
    nc = len(rep)
    ntask = nc * nq
    nw = (ntask + 63) // 64
    waves = {"skip": 0, "clamped": 0}
    live_pts = {}
    tot_waves, tot_live = 0, 0
    for i in range(npT):
        m = marg[i][:, rep, :].transpose(0, 2, 1).reshape(n, ntask)          # task = class + nc q
        c = lanes[i][:, rep, :].transpose(0, 2, 1).reshape(n, ntask)
        pad = nw * 64 - ntask
        m = np.concatenate([m, np.full((n, pad), 255, np.uint8)], axis=1).reshape(n, nw, 64).astype(np.int32)
        c = np.concatenate([c, np.full((n, pad), 11, np.int8)], axis=1).reshape(n, nw, 64)
        live = (c == 13) | (c == 14)
        clamp = (c == 12).any(axis=2)
        nlive = live.sum(axis=2)
        mmin = np.where(live, m, 1000).min(axis=2)
        tot_waves += n * nw
        waves["skip"] += int(((nlive == 0) & ~clamp).sum())
        waves["clamped"] += int(clamp.sum())
        ok = (nlive > 0) & ~clamp
        tot_live += int(nlive[ok].sum())
        for t in thresholds:
            sel = ok & (mmin > t)
            waves[t] = waves.get(t, 0) + int(sel.sum())
            live_pts[t] = live_pts.get(t, 0) + int(nlive[sel].sum())
    print("mode %d, %d cells, %d classes, %d waves per (cell, pT); lane census skip/clamp/tail/other %s"
          % (mode, n, nc, nw, list(cnt)))
    print("waves: skipped %.3f  clamped %.4f" % (waves["skip"] / tot_waves, waves["clamped"] / tot_waves))
    print("threshold  waves(min live margin > t)  live lanes in them")
    for t in thresholds:
        print("  %3d      %.3f                      %.3f" % (t, waves[t] / tot_waves, live_pts[t] / max(1, tot_live)))


if __name__ == "__main__":
    census(int(sys.argv[1]) if len(sys.argv) > 1 else 3, int(sys.argv[2]) if len(sys.argv) > 2 else 40)
