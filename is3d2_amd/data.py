"""Reference input tables (packed by tools/pack_reference_data.py)."""
import os

import numpy as np

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
DF_HRG = {1: "urqmd", 2: "smash", 3: "smash_box"}   # DeltafData.cpp:30-45


def grid(name):
    """(values, weights) of a 2-column quadrature table, e.g. 'pT48', 'phi32', 'y21', 'eta24', or an
    explicit table given as rows [[value, weight], ...] / a (values, weights) pair."""
    if not isinstance(name, str):
        g = np.asarray(name, dtype=np.float64)
        if g.ndim == 2 and g.shape[0] == 2 and g.shape[1] != 2:
            g = g.T
        return np.ascontiguousarray(g[:, 0]), np.ascontiguousarray(g[:, 1])
    g = np.load(os.path.join(_DATA, "grids.npz"))[name]
    return g[:, 0].copy(), g[:, 1].copy()


def gauss_laguerre(points=32):
    """(roots, weights) arrays [alpha][points] of tables/gauss/gla_roots_weights.txt (32 pt)
    or tables/gla_roots_weights_64_points.txt (64 pt)."""
    g = np.load(os.path.join(_DATA, "grids.npz"))
    return g["gla%d_root" % points].copy(), g["gla%d_weight" % points].copy()


def df_tables(hrg_eos):
    """(T[nT], muB[nmuB], tab[10][nmuB][nT]) for deltaf_coefficients/vh/<hrg>/."""
    d = np.load(os.path.join(_DATA, "deltaf.npz"))
    k = DF_HRG[hrg_eos]
    return d[k + "_T"].copy(), d[k + "_muB"].copy(), np.ascontiguousarray(d[k + "_tab"])
