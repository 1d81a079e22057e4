"""Synthetic freeze-out surfaces (the reference ships only a 1-cell, mis-formatted
input/surface.dat), generated exactly as SURVEY.md section
8(d) prescribes, plus the unit round trip of the mode-1 reader.

All values are returned in the engine's (= reader-converted) units: GeV, fm.
``as_read`` applies the text-file round trip of readindata.cpp:233-290: the file
stores E, T, P, pi, Pi divided by hbarc and the reader multiplies back.
"""
import numpy as np

HBARC = 0.197327053
FIELDS = ["tau", "x", "y", "eta", "dat", "dax", "day", "dan", "ux", "uy", "un", "E", "T", "P",
          "pixx", "pixy", "pixn", "piyy", "piyn", "bulkPi", "muB", "nB", "Vx", "Vy", "Vn"]
_HBARC_FIELDS = ("E", "T", "P", "pixx", "pixy", "pixn", "piyy", "piyn", "bulkPi", "muB")


def _roundtrip(v):
    # '%.17g' round-trips a double exactly, so the file -> reader path is fl(fl(v/hbarc)*hbarc)
    return (np.asarray(v, dtype=np.float64) / HBARC) * HBARC


def as_read(surf):
    out = dict(surf)
    for k in _HBARC_FIELDS:
        if k in out and out[k] is not None:
            out[k] = _roundtrip(out[k])
    return out


def surface(n, seed=7, dimension=2, baryon=False, full3d=False):
    """SURVEY.md 8(d) config-1 distributions, drawn with default_rng(seed) in the order
    tau, x, y, dsigma_tau, dsigma_x, dsigma_y, u^x, u^y, T, pi^xx, pi^xy, pi^yy, Pi;
    dimension=3 then draws eta ~ U(-4, 4); baryon=True draws muB ~ U(0, 0.3) GeV,
    nB ~ U(0, 0.1) fm^-3, V^x, V^y ~ N(0, 0.01) fm^-3; full3d=True adds nonzero
    u^eta, dsigma_eta, pi^{x eta}, pi^{y eta}, V^eta (all small)."""
    rng = np.random.default_rng(seed)
    s = {}
    tau = rng.uniform(0.5, 10.0, n)
    s["tau"] = tau
    s["x"] = rng.uniform(-10.0, 10.0, n)
    s["y"] = rng.uniform(-10.0, 10.0, n)
    s["dat"] = rng.uniform(0.1, 5.0, n) * tau
    s["dax"] = rng.normal(0.0, 0.5, n) * tau
    s["day"] = rng.normal(0.0, 0.5, n) * tau
    s["ux"] = rng.normal(0.0, 0.6, n)
    s["uy"] = rng.normal(0.0, 0.6, n)
    T = rng.uniform(0.145, 0.155, n)
    s["T"] = T
    s["pixx"] = rng.normal(0.0, 0.01, n)
    s["pixy"] = rng.normal(0.0, 0.005, n)
    s["piyy"] = rng.normal(0.0, 0.01, n)
    s["bulkPi"] = -np.abs(rng.normal(0.0, 0.005, n))
    s["E"] = 0.28 * (T / 0.15) ** 4
    s["P"] = 0.045 * (T / 0.15) ** 4
    zeros = np.zeros(n)
    s["eta"] = rng.uniform(-4.0, 4.0, n) if dimension == 3 else zeros.copy()
    s["dan"] = zeros.copy(); s["un"] = zeros.copy(); s["pixn"] = zeros.copy(); s["piyn"] = zeros.copy()
    if baryon:
        s["muB"] = rng.uniform(0.0, 0.3, n)
        s["nB"] = rng.uniform(0.0, 0.1, n)
        s["Vx"] = rng.normal(0.0, 0.01, n)
        s["Vy"] = rng.normal(0.0, 0.01, n)
        s["Vn"] = zeros.copy()
    else:
        for k in ("muB", "nB", "Vx", "Vy", "Vn"):
            s[k] = zeros.copy()
    if full3d:
        s["un"] = rng.normal(0.0, 0.1, n) / tau
        s["dan"] = rng.normal(0.0, 0.3, n) * tau
        s["pixn"] = rng.normal(0.0, 0.002, n) / tau
        s["piyn"] = rng.normal(0.0, 0.002, n) / tau
        if baryon:
            s["Vn"] = rng.normal(0.0, 0.003, n) / tau
    return {k: np.ascontiguousarray(s[k], dtype=np.float64) for k in FIELDS}


def write_mode1(path, surf, include_baryon=False, vorticity_seed=None):
    """input/surface.dat in the CPU-VH format (readindata.cpp:179-202): E, T, P, pi, Pi and muB
    stored in fm units (divided by hbarc), %.17g.  vorticity_seed: mode 5 -- six thermal-vorticity
    columns wbar^{tx ty tn xy xn yn} after the rest (readindata.cpp:298-306; read, not used by the spectra)."""
    cols = ["tau", "x", "y", "eta", "dat", "dax", "day", "dan", "ux", "uy", "un", "E", "T", "P",
            "pixx", "pixy", "pixn", "piyy", "piyn", "bulkPi"]
    if include_baryon:
        cols += ["muB", "nB", "Vx", "Vy", "Vn"]
    arr = []
    for k in cols:
        v = np.asarray(surf[k], dtype=np.float64)
        arr.append(v / HBARC if k in _HBARC_FIELDS else v)
    if vorticity_seed is not None:
        w = np.random.default_rng(vorticity_seed).normal(0.0, 0.05, (6, len(surf["tau"])))
        arr.extend(list(w))
    a = np.stack(arr, axis=1)
    with open(path, "w") as f:
        for row in a:
            f.write(" ".join("%.17g" % v for v in row) + "\n")


def write_music(path, surf, include_baryon=False):
    """MUSIC (public) surface format (readindata.cpp:383-390, mode 6): dsigma_mu/tau, u^tau, tau u^eta,
    E, T, muB [fm^-n], muS, muC, (E+P)/T, pi^{mu nu} with tau factors, Pi, [nB, V^mu]."""
    n = len(surf["tau"])
    tau = surf["tau"]
    ut = np.sqrt(1.0 + surf["ux"] ** 2 + surf["uy"] ** 2 + tau * tau * surf["un"] ** 2)
    cols = [tau, surf["x"], surf["y"], surf["eta"],
            surf["dat"] / tau, surf["dax"] / tau, surf["day"] / tau, surf["dan"] / tau,
            ut, surf["ux"], surf["uy"], tau * surf["un"],
            surf["E"] / HBARC, surf["T"] / HBARC, surf["muB"] / HBARC, np.zeros(n), np.zeros(n),
            (surf["E"] + surf["P"]) / surf["T"],
            np.zeros(n), np.zeros(n), np.zeros(n), np.zeros(n),
            surf["pixx"] / HBARC, surf["pixy"] / HBARC, tau * surf["pixn"] / HBARC,
            surf["piyy"] / HBARC, tau * surf["piyn"] / HBARC, np.zeros(n), surf["bulkPi"] / HBARC]
    if include_baryon:
        cols += [surf["nB"], np.zeros(n), surf["Vx"], surf["Vy"], tau * surf["Vn"]]
    a = np.stack(cols, axis=1)
    with open(path, "w") as f:
        for row in a:
            f.write(" ".join("%.17g" % v for v in row) + "\n")


def write_hic(path, surf):
    """HIC-EventGen surface format (readindata.cpp:570-731, mode 7), GeV units, v = u/u^tau."""
    n = len(surf["tau"])
    tau = surf["tau"]
    ut = np.sqrt(1.0 + surf["ux"] ** 2 + surf["uy"] ** 2)
    z = np.zeros(n)
    cols = [tau, surf["x"], surf["y"], z, surf["dat"] / tau, surf["dax"] / tau, surf["day"] / tau, z,
            surf["ux"] / ut, surf["uy"] / ut, z, z, z, z, z, surf["pixx"], surf["pixy"], z, surf["piyy"], z, z,
            surf["bulkPi"], surf["T"], surf["E"], surf["P"], surf["muB"]]
    a = np.stack(cols, axis=1)
    with open(path, "w") as f:
        for row in a:
            f.write(" ".join("%.17g" % v for v in row) + "\n")
