#!/usr/bin/env python3
"""PTMA warm-start chain cost on the GPU: prepass / k_spectra / total ms of one pass for famod_chains = 0
(every cell solved cold, one wavefront per cell) and C = 1, 8, 64 (the reference's per-thread warm-start
chains, MomentumSpectra.cpp:1308-1364; C = 1 is the reference as shipped, serial).
usage: python tools/ptma_chain_probe.py [cells] [chains...]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from is3d2_amd import build_engine, make_spec, synth
    cells = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
    chains = [int(c) for c in sys.argv[2:]] or [0, 1, 8, 64]
    s = synth.as_read(synth.surface(cells, seed=7, dimension=3, baryon=True, full3d=True))
    for C in chains:
        spec = make_spec(hrg_eos=1, chosen="urqmd", df_mode=5, dimension=3, pT="pT48", phi="phi32", y="y21",
                         gla_points=64, include_baryon=1, include_baryondiff_deltaf=1, famod_chains=C)
        e = build_engine(spec, s)
        e.calculate_spectra()                      # warm-up (tables, allocations)
        t = time.perf_counter()
        e.calculate_spectra()
        wall = time.perf_counter() - t
        st = e.stats()
        e.close()
        print(json.dumps(dict(cells=cells, chains=C, wall_s=wall, ms_prepass=st["ms_prepass"],
                              ms_spectra=st["ms_spectra"], ms_total=st["ms_total"], iterations=st["iterations"],
                              us_per_cell_prepass=1e3 * st["ms_prepass"] / cells)), flush=True)


if __name__ == "__main__":
    main()
