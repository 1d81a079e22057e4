#!/usr/bin/env python3
"""Pack the reference's physics INPUT tables (not code) into is3d2_amd/data/*.npz.

The GPU box has no /root/reference, but the parity tests and bench need the same
inputs the reference workflow reads: PDG hadron lists, chosen-species lists,
delta-f coefficient tables, momentum / rapidity quadrature tables and the
Gauss-Laguerre tables.  This script (run once, in the build container) parses
those whitespace tables and stores the numbers as float64/int64 arrays.

Sources (all under /root/reference):
  PDG/pdg_smash.dat, PDG/pdg-urqmd_v3.3+.dat       conventional format (readindata.cpp:973-1095)
  PDG/pdg_box.dat                                  smash-box format    (readindata.cpp:1098-1215)
  PDG/chosen_particles*.dat                         one MCID per row
  deltaf_coefficients/vh/<hrg>/*.dat               header nT, nmuB, label; rows "T muB value" (DeltafData.cpp:120-197)
  tables/all_tables/{pT,phi}/*gauss_table_*.dat, tables/momentum/*.dat, tables/spacetime_rapidity/eta_table.dat
  tables/gauss/gla_roots_weights.txt, tables/gla_roots_weights_64_points.txt
"""
import os
import sys

import numpy as np

REF = "/root/reference"
DF_NAMES = ["c0", "c1", "c2", "c3", "c4", "F", "G", "betabulk", "betaV", "betapi"]


def read_pdg_conventional(path):
    toks = open(path, encoding="utf-8").read().split()
    rows = []
    i = 0
    while i < len(toks):
        mcid = int(toks[i]); mass = float(toks[i + 2]); width = float(toks[i + 3])
        gspin = int(toks[i + 4]); baryon = int(toks[i + 5]); strange = int(toks[i + 6])
        charge = int(toks[i + 10]); ndec = int(toks[i + 11])
        rows.append((mcid, mass, width, gspin, baryon, strange, charge))
        i += 12 + 8 * ndec
    a = np.array(rows, dtype=object)
    return dict(mcid=a[:, 0].astype(np.int64), mass=a[:, 1].astype(np.float64), width=a[:, 2].astype(np.float64),
                gspin=a[:, 3].astype(np.int64), baryon=a[:, 4].astype(np.int64))


def read_pdg_box(path):
    rows = []
    for line in open(path, encoding="utf-8"):
        if not line.strip() or line.startswith("#"):
            continue
        t = line.split()
        mcids = []
        for v in t[4:8]:          # istringstream >> long stops at the first non-integer ('#')
            try:
                mcids.append(int(v))
            except ValueError:
                break
        mcids += [0] * (4 - len(mcids))
        rows.append([float(t[1]), float(t[2])] + mcids)
    a = np.array(rows)
    return dict(mass=a[:, 0], width=a[:, 1], mcids=a[:, 2:6].astype(np.int64))


def read_table(path):
    """Reference Table semantics (Arsenal.cpp:86-121): rows end with a newline; a final
    unterminated line is not read."""
    txt = open(path).read()
    lines = txt.split("\n")[:-1]
    rows = [[float(v) for v in ln.split()] for ln in lines if ln.split()]
    return np.array(rows, dtype=np.float64)


def read_df(hrg):
    d = os.path.join(REF, "deltaf_coefficients/vh", hrg)
    tabs = []
    T = muB = None
    for name in DF_NAMES:
        lines = open(os.path.join(d, name + ".dat")).read().split("\n")
        nT, nmuB = int(lines[0]), int(lines[1])
        vals = np.array([[float(v) for v in ln.split()] for ln in lines[3:3 + nT * nmuB]])
        vals = vals.reshape(nmuB, nT, 3)
        T = vals[0, :, 0]
        muB = vals[:, 0, 1]
        tabs.append(vals[:, :, 2])
    return dict(T=T, muB=muB, tab=np.stack(tabs))


def read_gla(path):
    toks = open(path).read().split()
    alpha, pts = int(toks[0]), int(toks[1])
    v = np.array([float(x) for x in toks[2:2 + 3 * alpha * pts]]).reshape(alpha, pts, 3)
    return v[:, :, 1].copy(), v[:, :, 2].copy()


def main(out_dir):
    os.makedirs(out_dir, exist_ok=True)
    pdg = {}
    for key, fn in (("smash", "pdg_smash.dat"), ("urqmd", "pdg-urqmd_v3.3+.dat")):
        for k, v in read_pdg_conventional(os.path.join(REF, "PDG", fn)).items():
            pdg["%s_%s" % (key, k)] = v
    for k, v in read_pdg_box(os.path.join(REF, "PDG", "pdg_box.dat")).items():
        pdg["box_%s" % k] = v
    for key, fn in (("pikp", "chosen_particles_pikp.dat"), ("smash", "chosen_particles_smash.dat"),
                    ("urqmd", "chosen_particles_urqmd_v3.3+.dat"), ("box", "chosen_particles_box.dat"),
                    ("default", "chosen_particles.dat")):
        pdg["chosen_%s" % key] = read_table(os.path.join(REF, "PDG", fn))[:, 0].astype(np.int64)
    np.savez_compressed(os.path.join(out_dir, "pdg.npz"), **pdg)

    df = {}
    for hrg in ("smash", "urqmd", "smash_box"):
        for k, v in read_df(hrg).items():
            df["%s_%s" % (hrg, k)] = v
    np.savez_compressed(os.path.join(out_dir, "deltaf.npz"), **df)

    grids = {}
    for key, rel in (("pT24", "tables/all_tables/pT/pT_gauss_table_24pt.dat"),
                     ("pT48", "tables/all_tables/pT/pT_gauss_table_48pt.dat"),
                     ("phi24", "tables/all_tables/phi/phi_gauss_table_24pt.dat"),
                     ("phi32", "tables/all_tables/phi/phi_gauss_table_32pt.dat"),
                     ("pT_default", "tables/momentum/pT_table.dat"),
                     ("phi_default", "tables/momentum/phi_table.dat"),
                     ("phi48", "tables/momentum/phi_table_48pt.dat"),
                     ("y21", "tables/momentum/y_table.dat"),
                     ("eta24", "tables/spacetime_rapidity/eta_table.dat")):
        grids[key] = read_table(os.path.join(REF, rel))
    r, w = read_gla(os.path.join(REF, "tables/gauss/gla_roots_weights.txt"))
    grids["gla32_root"], grids["gla32_weight"] = r, w
    r, w = read_gla(os.path.join(REF, "tables/gla_roots_weights_64_points.txt"))
    grids["gla64_root"], grids["gla64_weight"] = r, w
    np.savez_compressed(os.path.join(out_dir, "grids.npz"), **grids)
    print("wrote", sorted(os.listdir(out_dir)))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "is3d2_amd/data")
