"""Python host binding of the MI355X engine, shaped like the reference's plug-in
surface for operation = 1:

  EmissionFunctionArray(params, chosen species, pT/phi/y/eta tables, PDG, FO surface, Deltaf_Data)
      -> calculate_spectra()  ->  dN/(pT dpT dphi dy)[species][pT][phi][y]

(EmissionFunction.h:135-140, EmissionFunction.cpp:114-391, 981-1231).  Every call goes
through libis3d_amd.so; there is no CPU fallback.
"""
import ctypes as C

import numpy as np

from . import _lib
from . import data as _data
from . import hrg as _hrg

# famod_chains = 1: PTMA's Newton solves warm-start along one chain over every cell, as the reference does as
# shipped (serial: CORES = 1, EmissionFunction.cpp:131-135; MomentumSpectra.cpp:1308-1364); C > 1 reproduces
# a reference run with OMP_NUM_THREADS = C, 0 solves every cell from (T, 1, 1) -- differently converged
# solutions, measured 3.6e-6 from the one-chain spectra (tests/test_gpu_chains.py)
_DEFAULTS = dict(operation=1, dimension=2, df_mode=1, include_baryon=0, include_bulk_deltaf=1,
                 include_shear_deltaf=1, include_baryondiff_deltaf=0, regulate_deltaf=0, outflow=0,
                 famod_chains=1, deta_min=1.e-5, mass_pion0=0.138)


# operation = 0 binning (iS3D_parameters.dat defaults; EmissionFunction.cpp:232-247).  `threads` is the
# reference's CORES: 0 bins every species from zero; C >= 1 reproduces a reference run with
# OMP_NUM_THREADS = C, including its per-species byte-count memset carry (SpacetimeDistribution.cpp:165-167)
SPACETIME_BINS = dict(tau_min=0.0, tau_max=12.0, tau_bins=120, r_min=0.0, r_max=12.0, r_bins=60, phip_bins=100,
                      threads=0)


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _arr(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class IS3DError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("is3d error %d: %s" % (code, msg))
        self.code = code


class Engine:
    """One engine per GPU (device index in the current process's visible devices), or -- devices = [d0, d1,
    ...] -- one engine over several GPUs of this process (is3d_create_devices: cells sharded by estimated cost,
    spectra summed with one RCCL all-reduce inside the compute call)."""

    def __init__(self, device=0, devices=None):
        self.lib = _lib.load()
        if devices is not None:
            dv = (C.c_int * len(devices))(*[int(d) for d in devices])
            self._e = self.lib.is3d_create_devices(len(devices), dv)
            if not self._e:
                raise IS3DError(_lib.IS3D_ERR_DEVICE, "is3d_create_devices(%s) failed" % list(devices))
        else:
            self._e = self.lib.is3d_create(int(device))
        if not self._e:
            raise IS3DError(_lib.IS3D_ERR_DEVICE, "is3d_create(%d) failed (no HIP device?)" % device)
        self._keep = []

    def close(self):
        if getattr(self, "_e", None):
            self.lib.is3d_destroy(self._e)
            self._e = None

    def __del__(self):
        self.close()

    def _chk(self, rc):
        if rc != 0:
            raise IS3DError(rc, self.lib.is3d_last_error(self._e).decode())
        return rc

    # --- setup, mirroring the reference services --------------------------------------
    def set_params(self, **kw):
        p = dict(_DEFAULTS)
        p.update({k: v for k, v in kw.items() if k in _DEFAULTS})
        self.params = p
        self._chk(self.lib.is3d_set_params(self._e, C.byref(_lib.Params(**p))))

    def set_tuning(self, key, value):
        """Engine knob (is3d_set_tuning): "phitab_one_bytes" / "phitab_chunk_bytes" (F_TS table chunking),
        "max_splits" / "slab_bytes" / "split_bytes" (k_spectra's cell splits); a negative value restores the default."""
        self._chk(self.lib.is3d_set_tuning(self._e, key.encode(), int(value)))

    def get_tuning(self, key):
        """is3d_get_tuning: the knobs above, "phitab_chunks" (F_TS chunks of the last launch) or "splits" (cell splits
        of the last launch); -1 = unknown."""
        return self.lib.is3d_get_tuning(self._e, key.encode())

    def set_species(self, mass, sign, degen, baryon):
        a = [_arr(x) for x in (mass, sign, degen, baryon)]
        self._chk(self.lib.is3d_set_species(self._e, len(a[0]), *[_dp(x) for x in a]))
        self.npart = len(a[0])

    def set_species_classes(self, on=True):
        """Integrate species with identical (mass, sign, baryon [, degeneracy for PTM]) once (default on);
        the spectra equal the per-species integration (bit for bit at the BASELINE sizes, include/is3d_amd.h)."""
        self._chk(self.lib.is3d_set_species_classes(self._e, int(bool(on))))

    def species_integrated(self):
        n = self.lib.is3d_species_integrated(self._e)
        if n < 0:
            self._chk(-n)     # an error comes back as minus its IS3D_ERR_* code
        return n

    def set_pdg(self, mass, sign, degen, baryon):
        a = [_arr(x) for x in (mass, sign, degen, baryon)]
        self._chk(self.lib.is3d_set_pdg(self._e, len(a[0]), *[_dp(x) for x in a]))

    def set_momentum_grid(self, pT, phi, y, eta, eta_w):
        a = [_arr(x) for x in (pT, phi, y, eta, eta_w)]
        self._chk(self.lib.is3d_set_momentum_grid(self._e, len(a[0]), _dp(a[0]), len(a[1]), _dp(a[1]),
                                                  len(a[2]), _dp(a[2]), len(a[3]), _dp(a[3]), _dp(a[4])))

    def set_momentum_weights(self, pT_w, phi_w):
        a, b = _arr(pT_w), _arr(phi_w)
        self._chk(self.lib.is3d_set_momentum_weights(self._e, _dp(a), _dp(b)))

    def set_spacetime_bins(self, **kw):
        b = dict(SPACETIME_BINS)
        b.update({k: v for k, v in kw.items() if k in SPACETIME_BINS})
        self.bins = b
        self._chk(self.lib.is3d_set_spacetime_bins(self._e, C.byref(_lib.SpacetimeBins(**b))))

    def set_gauss_laguerre(self, roots, weights):
        r, w = _arr(roots), _arr(weights)
        self._chk(self.lib.is3d_set_gauss_laguerre(self._e, r.shape[0], r.shape[1], _dp(r), _dp(w)))

    def set_df_tables(self, T, muB, tab, T_avg):
        T, muB, tab = _arr(T), _arr(muB), _arr(tab)
        self._chk(self.lib.is3d_set_df_tables(self._e, len(T), len(muB), _dp(T), _dp(muB), _dp(tab), float(T_avg)))

    def set_surface(self, surf):
        cols = [_arr(surf[k]) if surf.get(k) is not None else None for k in _lib.SURFACE_FIELDS]
        n = len(cols[0])
        self._keep = cols
        s = _lib.Surface(*[(_dp(c) if c is not None else C.POINTER(C.c_double)()) for c in cols])
        self._chk(self.lib.is3d_set_surface(self._e, n, C.byref(s)))
        self.ncell = n

    def set_surface_device(self, ptr, n):
        self._chk(self.lib.is3d_set_surface_device(self._e, int(n), C.c_void_p(ptr)))
        self.ncell = n

    def set_cell_window(self, lo, hi):
        """Integrate only cells [lo, hi) of the surface (-1, -1: all); PTMA chains still walk every cell."""
        self._chk(self.lib.is3d_set_cell_window(self._e, int(lo), int(hi)))

    # --- compute -----------------------------------------------------------------------
    def cell_costs(self):
        """Per-cell shard cost estimate of the surface set last (is3d_cell_costs: 0.02 skipped, PTM / PTB
        separable-fallback cells 1.4 / 1.8, else 1)."""
        n = self.ncell
        out = np.zeros(max(n, 1))
        self._chk(self.lib.is3d_cell_costs(self._e, _dp(out)))
        return out[:n]

    def output_size(self):
        return self.lib.is3d_output_size(self._e)

    def calculate_spectra(self):
        out = np.zeros(self.output_size(), dtype=np.float64)
        self._chk(self.lib.is3d_calculate_spectra(self._e, _dp(out)))
        return out

    def calculate_dN_dX(self):
        """operation = 0: (dN_taudtaudy, dN_2pirdrdy, dN_dphidy), each [species][bins]."""
        b = self.bins
        t = np.zeros((self.npart, b["tau_bins"])); r = np.zeros((self.npart, b["r_bins"]))
        ph = np.zeros((self.npart, b["phip_bins"]))
        self._chk(self.lib.is3d_calculate_dN_dX(self._e, _dp(t), _dp(r), _dp(ph)))
        return t, r, ph

    def cell_yields(self):
        """dN_dy_cell [species][cell] of the last calculate_dN_dX."""
        out = np.zeros((self.npart, self.ncell))
        self._chk(self.lib.is3d_get_cell_yields(self._e, _dp(out)))
        return out

    def launch(self, dev_out_ptr, stream_ptr=None):
        self._chk(self.lib.is3d_launch(self._e, C.c_void_p(dev_out_ptr), C.c_void_p(stream_ptr or 0)))

    def finish(self):
        self._chk(self.lib.is3d_finish(self._e))

    # --- staged launch: PTMA warm-start chains split over processes (include/is3d_amd.h, dist.launch_chained) ---
    def set_chain_range(self, q0, q1):
        """Solve chain positions [q0, q1) of every PTMA warm-start chain and integrate cells [q0 C, q1 C)
        (-1, -1: off).  Needs the staged launch (dist.launch_chained)."""
        self._chk(self.lib.is3d_set_chain_range(self._e, int(q0), int(q1)))

    def launch_begin(self, dev_out_ptr, stream_ptr=None):
        self._chk(self.lib.is3d_launch_begin(self._e, C.c_void_p(dev_out_ptr), C.c_void_p(stream_ptr or 0)))

    def chain_passes(self):
        return self.lib.is3d_chain_passes(self._e)

    def chain_pass(self, j):
        self._chk(self.lib.is3d_chain_pass(self._e, int(j)))

    def chain_end(self):
        self._chk(self.lib.is3d_chain_end(self._e))

    def launch_end(self):
        self._chk(self.lib.is3d_launch_end(self._e))

    def chain_boundary_size(self):
        return self.lib.is3d_chain_boundary_size(self._e)

    def chain_boundary_get(self, slot, buf):
        """Copy this range's boundary slot (0, 1: pass parity, 2: final) into the device tensor buf (launch stream)."""
        self._chk(self.lib.is3d_chain_boundary_get(self._e, int(slot), C.c_void_p(buf.data_ptr())))

    def chain_boundary_put(self, slot, buf):
        """Copy the device tensor buf (the previous range's end states) into this range's incoming slot."""
        self._chk(self.lib.is3d_chain_boundary_put(self._e, int(slot), C.c_void_p(buf.data_ptr())))

    def stats(self):
        s = _lib.Stats()
        self._chk(self.lib.is3d_get_stats(self._e, C.byref(s)))
        return {k: getattr(s, k) for k, _ in s._fields_}

    def evaluate_df_coefficients(self, T, muB, E, P, bulkPi):
        out = np.zeros(15)
        self._chk(self.lib.is3d_evaluate_df_coefficients(self._e, T, muB, E, P, bulkPi, _dp(out)))
        return out

    def total_yield(self, plasma, y_cut=0.5):
        """operation = 2 oversampling estimate (ParticleSampler.cpp:447-636): (Ntotal, densities[3][npart]).
        plasma = (T, E, P, muB, nB) averages; the engine's Gauss-Laguerre table must be the 32-point one."""
        pl = _arr(plasma)
        nt = np.zeros(1)
        dens = np.zeros(3 * self.npart)
        self._chk(self.lib.is3d_total_yield(self._e, _dp(pl), float(y_cut), _dp(nt), _dp(dens)))
        return float(nt[0]), dens.reshape(3, self.npart)

    def jonah_table(self):
        l2, z, bp, mx = np.zeros(301), np.zeros(301), np.zeros(301), np.zeros(1)
        self._chk(self.lib.is3d_get_jonah_table(self._e, _dp(l2), _dp(z), _dp(bp), _dp(mx)))
        return l2, z, bp, mx[0]


def surface_averages(surf, include_baryon=0):
    """Plasma averages (T, E, P, muB, nB) after the reference's setprecision(15) file round trip."""
    lib = _lib.load()
    cols = [_arr(surf[k]) if surf.get(k) is not None else None for k in _lib.SURFACE_FIELDS]
    s = _lib.Surface(*[(_dp(c) if c is not None else C.POINTER(C.c_double)()) for c in cols])
    out = np.zeros(5)
    rc = lib.is3d_surface_averages(len(cols[0]), C.byref(s), int(include_baryon), _dp(out))
    if rc:
        raise IS3DError(rc, "surface averages")
    return out


# ------------------------------------------------------------------------------------------
# run specifications (inputs shared by the engine, the oracle and the bench)
# ------------------------------------------------------------------------------------------
def make_spec(hrg_eos=2, chosen="pikp", pT="pT24", phi="phi24", y="y21", eta="eta24", dimension=2, df_mode=1,
              gla_points=32, **flags):
    """Everything calculate_spectra needs except the surface: parameters, species, grids,
    Gauss-Laguerre table, delta-f tables.  `chosen` is a key of PDG/chosen_particles_*.dat
    ('pikp', 'smash', 'urqmd', 'box', 'default') or an explicit MCID list."""
    parts = _hrg.pdg_particles(hrg_eos)
    mcids = _hrg.chosen_mcids(chosen) if isinstance(chosen, str) else np.asarray(chosen, dtype=np.int64)
    sp = _hrg.chosen_species(parts, mcids)
    pTv, pTw = _data.grid(pT)
    phiv, phiw = _data.grid(phi)
    yv, _ = _data.grid(y)
    etav, etaw = _data.grid(eta)
    roots, weights = _data.gauss_laguerre(gla_points)
    T, muB, tab = _data.df_tables(hrg_eos)
    params = dict(_DEFAULTS)
    params.update(dimension=dimension, df_mode=df_mode)
    params.update({k: v for k, v in flags.items() if k in _DEFAULTS})
    bins = dict(SPACETIME_BINS)
    bins.update({k: v for k, v in flags.items() if k in SPACETIME_BINS})
    return dict(params=params, species=sp, pdg=parts, pT=pTv, phi=phiv, y=yv, eta=etav, eta_w=etaw,
                pT_w=pTw, phi_w=phiw, bins=bins, gla=(roots, weights), df=(T, muB, tab), hrg_eos=hrg_eos)


def build_engine(spec, surf, T_avg=None, device=0, devices=None, species_classes=True):
    e = Engine(device, devices)
    p = spec["params"]
    e.set_params(**p)
    sp = spec["species"]
    e.set_species(sp["mass"], sp["sign"], sp["degen"], sp["baryon"])
    if not species_classes:
        e.set_species_classes(False)
    pdg = spec["pdg"]
    e.set_pdg(pdg["mass"], pdg["sign"], pdg["gspin"], pdg["baryon"])
    e.set_momentum_grid(spec["pT"], spec["phi"], spec["y"], spec["eta"], spec["eta_w"])
    if "pT_w" in spec:
        e.set_momentum_weights(spec["pT_w"], spec["phi_w"])
    e.set_spacetime_bins(**spec.get("bins", {}))
    e.set_gauss_laguerre(*spec["gla"])
    if T_avg is None:
        T_avg = surface_averages(surf, p["include_baryon"])[0]
    e.set_df_tables(*spec["df"], T_avg)
    if surf is not None:
        e.set_surface(surf)
    return e


def output_shape(spec):
    ny = len(spec["y"]) if spec["params"]["dimension"] == 3 else 1
    return (len(spec["species"]["mass"]), len(spec["pT"]), len(spec["phi"]), ny)
