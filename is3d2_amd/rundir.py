"""Materialise a reference-layout iS3D run directory from the packed input tables
(is3d2_amd/data/*.npz), so the drop-in workflow (iS3D_amd / is3d_host_run_particlization)
can be exercised anywhere, including on the GPU box where /root/reference is absent.

Layout (iS3D.cpp:96-257): iS3D_parameters.dat, input/surface.dat, PDG/<pdg file>,
PDG/chosen_particles.dat, deltaf_coefficients/vh/<hrg>/*.dat, tables/momentum/{pT,phi,y}_table.dat,
tables/spacetime_rapidity/eta_table.dat, tables/gauss/gla_roots_weights.txt,
tables/thermodynamic/, results/continuous/.
"""
import os

import numpy as np

from . import data, synth

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
DF_NAMES = ["c0", "c1", "c2", "c3", "c4", "F", "G", "betabulk", "betaV", "betapi"]
PARAM_KEYS = ["operation", "mode", "hrg_eos", "dimension", "df_mode", "include_baryon", "include_bulk_deltaf",
              "include_shear_deltaf", "include_baryondiff_deltaf", "regulate_deltaf", "outflow", "deta_min",
              "mass_pion0", "group_particles", "famod_chains"]


def _table(path, v, w):
    with open(path, "w") as f:
        for a, b in zip(v, w):
            f.write("%.17g\t%.17g\n" % (a, b))


def write_pdg(d, hrg_eos):
    p = np.load(os.path.join(_DATA, "pdg.npz"))
    os.makedirs(os.path.join(d, "PDG"), exist_ok=True)
    if hrg_eos in (1, 2):
        key = "urqmd" if hrg_eos == 1 else "smash"
        fn = "pdg-urqmd_v3.3+.dat" if hrg_eos == 1 else "pdg_smash.dat"
        with open(os.path.join(d, "PDG", fn), "w") as f:
            for m, mass, w, g, b in zip(p[key + "_mcid"], p[key + "_mass"], p[key + "_width"], p[key + "_gspin"],
                                        p[key + "_baryon"]):
                # decay channels are not needed on the continuous-spectra path: written as 0 channels
                f.write("%d h%d %.17g %.17g %d %d 0 0 0 1 0 0\n" % (m, abs(m), mass, w, g, b))
    else:
        with open(os.path.join(d, "PDG", "pdg_box.dat"), "w") as f:
            f.write("# NAME MASS[GEV] WIDTH[GEV] PARITY PDG\n")
            for mass, w, ids in zip(p["box_mass"], p["box_width"], p["box_mcids"]):
                f.write("h %.17g %.17g + %s\n" % (mass, w, " ".join(str(int(i)) for i in ids if i != 0)))


def write_run_dir(d, surf, params, hrg_eos=2, chosen="pikp", pT="pT24", phi="phi24", y="y21", eta="eta24",
                  surface_format=1):
    """Write a complete run directory.  `params` maps iS3D_parameters.dat keys to values."""
    for sub in ("input", "PDG", "tables/momentum", "tables/spacetime_rapidity", "tables/gauss",
                "tables/thermodynamic", "results/continuous"):
        os.makedirs(os.path.join(d, sub), exist_ok=True)
    p = dict(operation=1, mode=surface_format, hrg_eos=hrg_eos)
    p.update(params)
    with open(os.path.join(d, "iS3D_parameters.dat"), "w") as f:
        for k, v in p.items():
            f.write("%s = %s\t\t# %s\n" % (k, repr(v), k))
    baryon = bool(p.get("include_baryon", 0))
    if surface_format == 6:
        synth.write_music(os.path.join(d, "input", "surface.dat"), surf, include_baryon=baryon)
    elif surface_format == 7:
        synth.write_hic(os.path.join(d, "input", "surface.dat"), surf)
    else:       # 1, or 5 = 1 + thermal-vorticity columns
        synth.write_mode1(os.path.join(d, "input", "surface.dat"), surf, include_baryon=baryon,
                          vorticity_seed=(5 if surface_format == 5 else None))
    write_pdg(d, hrg_eos)
    pp = np.load(os.path.join(_DATA, "pdg.npz"))
    mc = pp["chosen_" + chosen] if isinstance(chosen, str) else np.asarray(chosen)
    with open(os.path.join(d, "PDG", "chosen_particles.dat"), "w") as f:
        for m in mc:
            f.write("%d\n" % m)
    T, muB, tab = data.df_tables(hrg_eos)
    hdir = os.path.join(d, "deltaf_coefficients", "vh", data.DF_HRG[hrg_eos])
    os.makedirs(hdir, exist_ok=True)
    for k, name in enumerate(DF_NAMES):
        with open(os.path.join(hdir, name + ".dat"), "w") as f:
            f.write("%d\n%d\nT [GeV]\t\tmuB [GeV]\t\t%s\n" % (len(T), len(muB), name))
            for iB in range(len(muB)):
                for iT in range(len(T)):
                    f.write("%.17g\t\t%.17g\t\t%.17g\n" % (T[iT], muB[iB], tab[k, iB, iT]))
    _table(os.path.join(d, "tables/momentum/pT_table.dat"), *data.grid(pT))
    _table(os.path.join(d, "tables/momentum/phi_table.dat"), *data.grid(phi))
    _table(os.path.join(d, "tables/momentum/y_table.dat"), *data.grid(y))
    _table(os.path.join(d, "tables/spacetime_rapidity/eta_table.dat"), *data.grid(eta))
    r, w = data.gauss_laguerre(32)
    with open(os.path.join(d, "tables/gauss/gla_roots_weights.txt"), "w") as f:
        f.write("%d\t%d\n" % r.shape)
        for a in range(r.shape[0]):
            for j in range(r.shape[1]):
                f.write("%d\t%.17g\t%.17g\n" % (a, r[a, j], w[a, j]))
    return d
