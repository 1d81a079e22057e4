"""ctypes binding of the oracle (oracle/libis3d_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, never by the product package.
"""
import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "libis3d_oracle.so")
SURFACE_FIELDS = ["tau", "x", "y", "eta", "dat", "dax", "day", "dan", "ux", "uy", "un", "E", "T", "P",
                  "pixx", "pixy", "pixn", "piyy", "piyn", "bulkPi", "muB", "nB", "Vx", "Vy", "Vn"]
PD = C.POINTER(C.c_double)


class OrcParams(C.Structure):
    _fields_ = [("dimension", C.c_int), ("df_mode", C.c_int), ("include_baryon", C.c_int),
                ("include_bulk_deltaf", C.c_int), ("include_shear_deltaf", C.c_int),
                ("include_baryondiff_deltaf", C.c_int), ("regulate_deltaf", C.c_int), ("outflow", C.c_int),
                ("threads", C.c_int), ("omp_threads", C.c_int), ("deta_min", C.c_double), ("mass_pion0", C.c_double)]


class OrcSetup(C.Structure):
    _fields_ = [("npart", C.c_int), ("mass", PD), ("sign", PD), ("degen", PD), ("baryon", PD),
                ("npdg", C.c_int), ("pdg_mass", PD), ("pdg_sign", PD), ("pdg_degen", PD), ("pdg_baryon", PD),
                ("npT", C.c_int), ("nphi", C.c_int), ("ny", C.c_int), ("neta", C.c_int),
                ("pT", PD), ("phi", PD), ("y", PD), ("eta", PD), ("eta_w", PD),
                ("gla_alpha", C.c_int), ("gla_points", C.c_int), ("gla_root", PD), ("gla_weight", PD),
                ("nT", C.c_int), ("nmuB", C.c_int), ("Tarr", PD), ("muBarr", PD), ("dftab", PD),
                ("T_avg", C.c_double), ("pT_w", PD), ("phi_w", PD)]


class OrcBins(C.Structure):
    _fields_ = [("tau_min", C.c_double), ("tau_max", C.c_double), ("tau_bins", C.c_int),
                ("r_min", C.c_double), ("r_max", C.c_double), ("r_bins", C.c_int), ("phip_bins", C.c_int),
                ("carry", C.c_int)]


class OrcSurface(C.Structure):
    _fields_ = [("n", C.c_long)] + [(k, PD) for k in SURFACE_FIELDS]


_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def load():
    """The oracle library: oracle/libis3d_oracle.so, or IS3D_ORACLE_LIB (bench.py's cpu_baseline leg points it at
    a -march=native build made on the GPU box's host)."""
    global _lib
    if _lib is None:
        path = os.environ.get("IS3D_ORACLE_LIB") or LIB
        if path == LIB and not os.path.exists(LIB):
            build()
        lib = C.CDLL(path)
        lib.orc_spectra.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcSetup), C.POINTER(OrcSurface), PD,
                                    C.POINTER(C.c_long), C.c_char_p, C.c_int]
        lib.orc_dndx.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcSetup), C.POINTER(OrcSurface),
                                 C.POINTER(OrcBins), PD, PD, PD, PD, C.POINTER(C.c_long), C.c_char_p, C.c_int]
        lib.orc_gauss_thermal.restype = C.c_double
        lib.orc_gauss_thermal.argtypes = [C.c_int, PD, PD, C.c_int, C.c_double, C.c_double, C.c_double, C.c_double]
        lib.orc_gauss1d_mod.restype = C.c_double
        lib.orc_gauss1d_mod.argtypes = [C.c_int, PD, PD, C.c_int, C.c_double, C.c_double, C.c_double]
        lib.orc_milne_lrf.argtypes = [PD, PD]
        lib.orc_dsigma_lrf.argtypes = [PD, PD]
        lib.orc_lu3_solve.argtypes = [PD, PD, PD, C.POINTER(C.c_int)]
        lib.orc_df_coefficients.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcSetup), C.c_double, C.c_double,
                                            C.c_double, C.c_double, C.c_double, PD, C.c_char_p, C.c_int]
        lib.orc_jonah_table.argtypes = [C.POINTER(OrcSetup), PD, PD, PD, PD]
        lib.orc_surface_averages.argtypes = [C.POINTER(OrcSurface), PD]
        lib.orc_total_yield.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcSetup), C.POINTER(OrcSurface), PD,
                                        C.c_double, PD, PD, C.c_char_p, C.c_int]
        lib.orc_aniso_solve.argtypes = [C.POINTER(OrcSetup), C.c_double, C.c_double, C.c_double, C.c_double,
                                        C.c_double, C.c_double, PD]
        lib.orc_famod_chain.restype = C.c_long
        lib.orc_famod_chain.argtypes = [C.POINTER(OrcParams), C.POINTER(OrcSetup), C.POINTER(OrcSurface),
                                        C.POINTER(C.c_long), C.c_long, PD, PD, C.POINTER(C.c_int)]
        _lib = lib
    return _lib


def _a(x):
    return np.ascontiguousarray(x, dtype=np.float64)


def _p(a):
    return a.ctypes.data_as(PD)


class _Inputs:
    """Keeps the numpy buffers alive while the C structs point into them."""

    def __init__(self, spec, surf=None, T_avg=None, threads=1, omp_threads=0):
        p = spec["params"]
        self.params = OrcParams(p["dimension"], p["df_mode"], p["include_baryon"], p["include_bulk_deltaf"],
                                p["include_shear_deltaf"], p["include_baryondiff_deltaf"], p["regulate_deltaf"],
                                p["outflow"], int(threads), int(omp_threads), p["deta_min"], p["mass_pion0"])
        sp, pdg = spec["species"], spec["pdg"]
        self.keep = [_a(sp["mass"]), _a(sp["sign"]), _a(sp["degen"]), _a(sp["baryon"]),
                     _a(pdg["mass"]), _a(pdg["sign"]), _a(pdg["gspin"]), _a(pdg["baryon"]),
                     _a(spec["pT"]), _a(spec["phi"]), _a(spec["y"]), _a(spec["eta"]), _a(spec["eta_w"]),
                     _a(spec["gla"][0]), _a(spec["gla"][1]), _a(spec["df"][0]), _a(spec["df"][1]), _a(spec["df"][2]),
                     _a(spec.get("pT_w", np.zeros(len(spec["pT"])))), _a(spec.get("phi_w", np.zeros(len(spec["phi"]))))]
        k = self.keep
        self.surf = None
        if surf is not None:
            cols = [(_a(surf[f]) if surf.get(f) is not None else None) for f in SURFACE_FIELDS]
            self.keep_s = cols
            n = len(cols[0])
            self.surf = OrcSurface(n, *[(_p(c) if c is not None else PD()) for c in cols])
            if T_avg is None:
                T_avg = averages(surf, p["include_baryon"])[0]
        self.setup = OrcSetup(len(k[0]), _p(k[0]), _p(k[1]), _p(k[2]), _p(k[3]),
                              len(k[4]), _p(k[4]), _p(k[5]), _p(k[6]), _p(k[7]),
                              len(k[8]), len(k[9]), len(k[10]), len(k[11]),
                              _p(k[8]), _p(k[9]), _p(k[10]), _p(k[11]), _p(k[12]),
                              k[13].shape[0], k[13].shape[1], _p(k[13]), _p(k[14]),
                              len(k[15]), len(k[16]), _p(k[15]), _p(k[16]), _p(k[17]),
                              float(T_avg) if T_avg is not None else 0.0, _p(k[18]), _p(k[19]))


def averages(surf, include_baryon=0):
    lib = load()
    cols = [(_a(surf[f]) if surf.get(f) is not None else None) for f in SURFACE_FIELDS]
    if not include_baryon:
        cols[SURFACE_FIELDS.index("muB")] = None
        cols[SURFACE_FIELDS.index("nB")] = None
    s = OrcSurface(len(cols[0]), *[(_p(c) if c is not None else PD()) for c in cols])
    out = np.zeros(5)
    lib.orc_surface_averages(C.byref(s), _p(out))
    return out


def spectra(spec, surf, T_avg=None, threads=1, omp_threads=0, return_stats=False):
    """Reference-semantics dN/(pT dpT dphi dy), flat [species][pT][phi][y]."""
    lib = load()
    inp = _Inputs(spec, surf, T_avg, threads, omp_threads)
    p = spec["params"]
    ny = len(spec["y"]) if p["dimension"] == 3 else 1
    out = np.zeros(len(spec["species"]["mass"]) * len(spec["pT"]) * len(spec["phi"]) * ny)
    stats = (C.c_long * 8)()
    err = C.create_string_buffer(256)
    rc = lib.orc_spectra(C.byref(inp.params), C.byref(inp.setup), C.byref(inp.surf), _p(out), stats, err, 256)
    if rc:
        raise RuntimeError("oracle: " + err.value.decode())
    if return_stats:
        return out, list(stats)
    return out


class FamodChain:
    """The PTMA warm-start chain step of the oracle (orc_famod_chain, MomentumSpectra.cpp:1288-1368) over explicit
    cell lists of one surface: walk(cells, state) solves the cells in order from state = (prev_ok, lambda, aT, aL)
    and returns (states after each cell [n][4], Newton iterations per cell (-1: not in the chain), end state)."""

    def __init__(self, spec, surf, T_avg=None):
        self.lib = load()
        self.inp = _Inputs(spec, surf, T_avg, 1)

    def walk(self, cells, state):
        cells = np.ascontiguousarray(cells, dtype=np.int64)
        st = np.array(state, dtype=np.float64)
        states = np.zeros((len(cells), 4))
        iters = np.zeros(len(cells), dtype=np.int32)
        self.lib.orc_famod_chain(C.byref(self.inp.params), C.byref(self.inp.setup), C.byref(self.inp.surf),
                                 cells.ctypes.data_as(C.POINTER(C.c_long)), len(cells), _p(st), _p(states),
                                 iters.ctypes.data_as(C.POINTER(C.c_int)))
        return states, iters, st


def df_coefficients(spec, T, muB, E, P, bulkPi, T_avg=0.0):
    lib = load()
    inp = _Inputs(spec, None, T_avg)
    out = np.zeros(15)
    err = C.create_string_buffer(256)
    rc = lib.orc_df_coefficients(C.byref(inp.params), C.byref(inp.setup), T, muB, E, P, bulkPi, _p(out), err, 256)
    return rc, out


def lu3_solve(A, b):
    """The restated GSL 3x3 LU solve (gsl_linalg_LU_decomp / _solve): x and the row permutation."""
    lib = load()
    A, b, x = _a(np.asarray(A).ravel()), _a(b), np.zeros(3)
    perm = (C.c_int * 3)()
    lib.orc_lu3_solve(_p(A), _p(b), _p(x), perm)
    return x, list(perm)


def jonah_table(spec, T_avg):
    lib = load()
    inp = _Inputs(spec, None, T_avg)
    l2, z, bp, mx = np.zeros(301), np.zeros(301), np.zeros(301), np.zeros(1)
    rc = lib.orc_jonah_table(C.byref(inp.setup), _p(l2), _p(z), _p(bp), _p(mx))
    return rc, l2, z, bp, mx[0]


def dndx(spec, surf, T_avg=None, threads=1, omp_threads=0, carry=None, return_cells=False):
    """operation = 0 (SpacetimeDistribution.cpp): (dN_taudtaudy, dN_2pirdrdy, dN_dphidy), each
    [species][bins] as written to results/continuous/, and optionally dN_dy_cell [species][cell].
    `threads` = the reference's CORES; carry (default: threads > 1... see orc_bins) = reproduce the
    byte-count memset carry between species."""
    lib = load()
    inp = _Inputs(spec, surf, T_avg, threads, omp_threads)
    b = spec["bins"]
    if carry is None:
        carry = 1
    bins = OrcBins(b["tau_min"], b["tau_max"], b["tau_bins"], b["r_min"], b["r_max"], b["r_bins"],
                   b["phip_bins"], int(carry))
    npart = len(spec["species"]["mass"])
    n = len(surf["tau"])
    t = np.zeros(npart * b["tau_bins"]); r = np.zeros(npart * b["r_bins"]); ph = np.zeros(npart * b["phip_bins"])
    cy = np.zeros(max(1, npart * n))
    stats = (C.c_long * 8)()
    err = C.create_string_buffer(256)
    rc = lib.orc_dndx(C.byref(inp.params), C.byref(inp.setup), C.byref(inp.surf), C.byref(bins), _p(cy),
                      _p(t), _p(r), _p(ph), stats, err, 256)
    if rc:
        raise RuntimeError("oracle: " + err.value.decode())
    out = (t.reshape(npart, -1), r.reshape(npart, -1), ph.reshape(npart, -1))
    if return_cells:
        return out + (cy[:npart * n].reshape(npart, n),)
    return out


def total_yield(spec, surf, plasma=None, y_cut=0.5):
    """operation = 2 oversampling estimate (ParticleSampler.cpp:447-636): (Ntotal, densities[3][npart]).
    plasma = (T, E, P, muB, nB) averages (default: this surface's)."""
    lib = load()
    p = spec["params"]
    if plasma is None:
        plasma = averages(surf, p["include_baryon"])
    inp = _Inputs(spec, surf, plasma[0], 1)
    pl = _a(plasma)
    npart = len(spec["species"]["mass"])
    dens = np.zeros(3 * npart)
    nt = np.zeros(1)
    err = C.create_string_buffer(256)
    rc = lib.orc_total_yield(C.byref(inp.params), C.byref(inp.setup), C.byref(inp.surf), _p(pl), float(y_cut),
                             _p(nt), _p(dens), err, 256)
    if rc:
        raise RuntimeError("oracle: " + err.value.decode())
    return float(nt[0]), dens.reshape(3, npart)
