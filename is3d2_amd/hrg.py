"""Hadron-resonance-gas species lists.

Mirrors the reference's PDG readers so the species arrays fed to the engine are
the ones iS3D builds from the same files:

* conventional format (hrg_eos = 1 UrQMD, 2 SMASH): readindata.cpp:973-1095 --
  every baryon row is followed by its antibaryon (-mcid, -baryon), and the
  quantum-statistics sign is -1 for even baryon number, +1 otherwise;
* smash-box format (hrg_eos = 3): readindata.cpp:1098-1215 with the
  mcid-digit decoding of read_mcid (readindata.cpp:736-969);
* chosen particles: first PDG entry with a matching mcid
  (EmissionFunction.cpp:356-372).

The numeric content of the PDG files is packed in is3d2_amd/data/pdg.npz by
tools/pack_reference_data.py.
"""
import os

import numpy as np

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
HRG_NAMES = {1: "urqmd", 2: "smash", 3: "box"}


def _load():
    return np.load(os.path.join(_DATA, "pdg.npz"))


def read_mcid(mcid):
    """Spin degeneracy, baryon number, statistics sign, has-antiparticle from a PDG code."""
    x = abs(int(mcid))
    d = [(x // 10 ** i) % 10 for i in range(10)]
    nJ, nq3, nq2, nq1 = d[0], d[1], d[2], d[3]
    n8 = d[7]
    nJ = (nJ + n8) & 0xF                    # 4-bit bitfield in the reference
    is_deuteron = (mcid == 1000010020)
    is_hadron = (not is_deuteron) and nq3 != 0 and nq2 != 0
    is_meson = is_hadron and nq1 == 0
    is_baryon = is_hadron and nq1 != 0
    if is_hadron:
        spin = 0 if nJ == 0 else nJ - 1
    elif is_deuteron:
        spin = 2
    else:
        spin = nq3
    if is_hadron and nJ > 0:
        gspin = nJ
    elif is_deuteron:
        gspin = 3
    else:
        gspin = spin + 1
    if is_deuteron:
        baryon = 2
    elif is_hadron:
        baryon = 0 if is_meson else (1 if is_baryon else 0)
    else:
        baryon = 0
    if is_deuteron:
        sign = -1
    elif is_hadron:
        sign = -1 if is_meson else 1
    else:
        sign = spin % 2
    if is_hadron:
        has_anti = (baryon != 0) or (nq2 != nq3)
    elif is_deuteron:
        has_anti = True
    else:
        has_anti = (nq3 == 1)
    return gspin, baryon, sign, has_anti


def _c_mod2(b):
    return int(np.fmod(b, 2))


def pdg_particles(hrg):
    """Full particle list in reference order: dict of mcid, mass, gspin, baryon, sign arrays."""
    name = HRG_NAMES.get(hrg, hrg)
    d = _load()
    rows = []
    if name in ("smash", "urqmd"):
        for mcid, mass, gs, b in zip(d[name + "_mcid"], d[name + "_mass"], d[name + "_gspin"], d[name + "_baryon"]):
            rows.append((int(mcid), float(mass), int(gs), int(b)))
            if b > 0:
                rows.append((-int(mcid), float(mass), int(gs), -int(b)))
        sign = [(-1 if _c_mod2(b) == 0 else 1) for (_, _, _, b) in rows]
    elif name == "box":
        sign = []
        for mass, mcids in zip(d["box_mass"], d["box_mcids"]):
            for m in mcids:
                if m == 0:
                    continue
                gs, b, sg, anti = read_mcid(int(m))
                rows.append((int(m), float(mass), gs, b)); sign.append(sg)
                if anti:
                    rows.append((-int(m), float(mass), gs, -b)); sign.append(sg)
    else:
        raise ValueError("hrg_eos must be 1, 2 or 3")
    a = np.array(rows, dtype=object)
    return dict(mcid=a[:, 0].astype(np.int64), mass=a[:, 1].astype(np.float64),
                gspin=a[:, 2].astype(np.float64), baryon=a[:, 3].astype(np.float64),
                sign=np.array(sign, dtype=np.float64))


def chosen_mcids(name):
    return _load()["chosen_" + name].copy()


def chosen_species(particles, mcids):
    """Species arrays (mass, sign, degeneracy, baryon, mcid) for the chosen MCIDs."""
    idx = []
    for m in mcids:
        hit = np.nonzero(particles["mcid"] == m)[0]
        if len(hit) == 0:
            raise ValueError("chosen particle %d not in PDG list" % m)
        idx.append(hit[0])
    idx = np.array(idx)
    return dict(mass=particles["mass"][idx].copy(), sign=particles["sign"][idx].copy(),
                degen=particles["gspin"][idx].copy(), baryon=particles["baryon"][idx].copy(),
                mcid=particles["mcid"][idx].copy())
