#!/usr/bin/env python3
"""Per-cell cost of the separable-fallback cells of the modified delta-f modes (PTM, PTB), relative to a
modified cell: the cost model of the device group's / torch.distributed shard windows.

Times the config-2 shape (SMASH 444 species, 48 x 32 x 21, 3+1D) on a normal surface and on the same surface
with bulkPi scaled so that a fraction f of the cells breaks down (MomentumSpectra.cpp:877-929); with t_a the
k_spectra time of the normal surface (no breakdowns) and t_b that of the scaled one,
    c_fb / c_mod = (t_b / t_a - (1 - f)) / f.
usage: python tools/fb_cost_probe.py [cells] [scale ...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from is3d2_amd import build_engine, make_spec, synth  # noqa: E402


def timed(spec, s, reps=3):
    e = build_engine(spec, s)
    e.calculate_spectra()
    ms = []
    for _ in range(reps):
        e.calculate_spectra()
        ms.append(e.stats()["ms_spectra"])
    st = e.stats()
    e.close()
    return float(np.median(ms)), st


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    scales = [float(x) for x in sys.argv[2:]] or [4.0, 10.0, 30.0]
    base = synth.as_read(synth.surface(n, seed=7, dimension=3, full3d=True))
    for mode in (3, 4):
        spec = make_spec(hrg_eos=2, chosen="smash", pT="pT48", phi="phi32", y="y21", dimension=3, df_mode=mode)
        ta, sa = timed(spec, base)
        for sc in scales:
            s = dict(base)
            s["bulkPi"] = base["bulkPi"] * sc
            tb, sb = timed(spec, s)
            f = sb["breakdown"] / float(sb["cells"])
            ratio = (tb / ta - (1.0 - f)) / f if f > 0 else None
            print(json.dumps(dict(mode=mode, cells=n, scale=sc, t_normal_ms=ta, breakdown_normal=sa["breakdown"],
                                  t_scaled_ms=tb, breakdown_frac=f, fb_over_mod=ratio)), flush=True)


if __name__ == "__main__":
    main()
