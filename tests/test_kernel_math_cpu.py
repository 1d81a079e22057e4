"""CPU tier: the engine's device math (cf_math.h / aniso_math.h), run serially on the
host by the test-only emulator, against the oracle.  The GPU tier repeats this through
libis3d_amd.so on the MI355X."""
import numpy as np
import pytest

import ctypes as C

from helpers import emu_spectra, emulator, parity, rel_quantile
from is3d2_amd import make_spec, synth
from oracle import oracle as O

CASES = [(d, m) for d in (2, 3) for m in (1, 2, 3, 4, 5)]


@pytest.mark.parametrize("dim,mode", CASES)
def test_factorised_math_matches_oracle(dim, mode):
    s = synth.as_read(synth.surface(150, seed=11, dimension=dim, full3d=(dim == 3)))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode, dimension=dim, pT="pT24", phi="phi24")
    ref = O.spectra(spec, s, threads=1)
    # variant 0: per-lane linear forms (k_dndx's form); 4: k_spectra's table form of the modified path
    for variant in ((0, 4) if mode >= 3 else (0,)):
        got, _ = emu_spectra(spec, s, chains=1, variant=variant)
        rel, zr, zg = parity(got, ref)
        assert rel < 1e-9, (variant, rel)
        assert zr == zg


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_baryon_bilinear_tables(mode):
    s = synth.as_read(synth.surface(80, seed=5, dimension=3, baryon=True, full3d=True))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode, dimension=3, include_baryon=1,
                     include_baryondiff_deltaf=1)
    ref = O.spectra(spec, s, threads=1)
    got, _ = emu_spectra(spec, s)
    assert parity(got, ref)[0] < 1e-9


def test_flags_outflow_regulate():
    s = synth.as_read(synth.surface(80, seed=9))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1, regulate_deltaf=1, outflow=1)
    ref = O.spectra(spec, s)
    got, _ = emu_spectra(spec, s)
    assert parity(got, ref)[0] < 1e-9


def test_ptma_chains_match_reference_thread_count():
    s = synth.as_read(synth.surface(90, seed=4))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5)
    for C in (1, 3):
        ref, st = O.spectra(spec, s, threads=C, return_stats=True)
        got, st2 = emu_spectra(spec, s, chains=C)
        assert parity(got, ref)[0] < 1e-9
        assert st[3] == st2[3]        # identical Newton iteration counts


@pytest.mark.parametrize("hrg_eos,dim", [(2, 2), (2, 3), (1, 3)])
def test_ptma_merged_hadron_sums(hrg_eos, dim):
    """The engine sums the PTMA Newton integrands over hadrons merged by identical (mass, sign) (SMASH 320 ->
    92, UrQMD 320 -> 83, engine.hip finalize_tables); the reference sums per hadron in PDG order
    (AnisoVariables.cpp:30-117).  On the breakdown-heavy chain (bulk x10, one warm-start chain, the surface
    of test_gpu_configs.py::test_modified_fallback_launch) both orders must take the same Newton steps and
    agree with the oracle to rounding."""
    s = synth.as_read(synth.surface(200, seed=31, dimension=dim, full3d=(dim == 3)))
    s["bulkPi"] = s["bulkPi"].copy()
    s["bulkPi"][::2] *= 10.0
    chosen = "pikp" if hrg_eos == 2 else [211, 321, 2212]
    spec = make_spec(hrg_eos=hrg_eos, chosen=chosen, df_mode=5, dimension=dim, famod_chains=1)
    ref, rst = O.spectra(spec, s, threads=1, return_stats=True)
    per, pst = emu_spectra(spec, s, chains=1, variant=4)
    mrg, mst = emu_spectra(spec, s, chains=1, variant=4 | 8)
    assert rst[3] == pst[3] == mst[3], (rst[3], pst[3], mst[3])
    assert parity(np.nan_to_num(per), np.nan_to_num(ref))[0] < 1e-9
    assert parity(np.nan_to_num(mrg), np.nan_to_num(ref))[0] < 1e-9
    assert parity(np.nan_to_num(mrg), np.nan_to_num(per))[0] < 1e-9


def test_kernel_exp_accuracy():
    """exp_dom690/exp_clamped (cf_math.h) against libm exp: <= 2 ulp over the fast-path domain,
    saturation to +inf past the overflow point, exact zero far below underflow."""
    import ctypes as C
    from helpers import emulator
    lib = emulator()
    rng = np.random.default_rng(3)
    x = np.concatenate([rng.uniform(-690, 690, 200000), rng.uniform(-2, 2, 100000),
                        np.array([0.0, 1e-300, -1e-300, 690.0, -690.0, 709.78, 709.79, 800.0, -746.0, -1e6, 1e6])])
    out = np.empty_like(x)
    lib.emu_exp(x.ctypes.data_as(C.POINTER(C.c_double)), C.c_long(len(x)), out.ctypes.data_as(C.POINTER(C.c_double)))
    ref = np.exp(x)
    fin = np.isfinite(ref) & (np.abs(x) <= 700)
    ulp = np.abs(out[fin] - ref[fin]) / np.spacing(ref[fin])
    assert ulp.max() <= 2.0, ulp.max()
    assert np.isinf(out[x >= 709.79]).all()
    assert (out[x <= -746.0] == 0.0).all()


def test_kernel_exp_tab_accuracy():
    """exp_tab (cf_math.h, per-point exp of the modified-momentum path) against libm exp: the table /
    polynomial part within 2 ulp (256-entry table, degree 4; 4 ulp for the 1024-entry table's degree 3,
    truncation 5.5e-16), plus the rounding of the scaled argument x N/ln2 (|x| 2.5e-16)."""
    import ctypes as C
    from helpers import emulator
    lib = emulator()
    rng = np.random.default_rng(4)
    x = np.concatenate([rng.uniform(-700, 700, 200000), rng.uniform(-2, 2, 100000), rng.uniform(-1e6, -746, 1000),
                        np.array([0.0, 1e-300, -1e-300, 690.0, -690.0, 700.0, -745.0])])
    out = np.empty_like(x)
    P = C.POINTER(C.c_double)
    lib.emu_exp_tab(x.ctypes.data_as(P), C.c_long(len(x)), out.ctypes.data_as(P))
    ref = np.exp(x)
    norm = (ref > 1e-300) & np.isfinite(ref)
    rel = np.abs(out[norm] - ref[norm]) / ref[norm]
    ulps = 4.0 if lib.emu_exp_tab_n() == 1024 else 2.0
    bound = ulps * 2.0 ** -52 + np.abs(x[norm]) * 2.5e-16
    assert (rel <= bound).all(), (rel / bound).max()
    small = np.abs(x) <= 2
    # 1024 entries: up to 6 spacings measured for |x| <= 2 (4.3e-16 truncation + the x N/ln2 rounding)
    assert (np.abs(out[small] - ref[small]) <= (8 if ulps > 2 else 2) * np.spacing(ref[small])).all()
    assert (out[x < -746.0] == 0.0).all()


def test_kernel_sinh_cosh_accuracy():
    """sinh_cosh (cf_math.h, y-terms) against libm over |y - eta| <= 12: <= 4 ulp, odd / even symmetry."""
    import ctypes as C
    from helpers import emulator
    rng = np.random.default_rng(6)
    x = np.concatenate([rng.uniform(-12, 12, 100000), rng.uniform(-0.6, 0.6, 100000),
                        np.array([0.0, 1e-300, -1e-300, 0.5, -0.5, np.nextafter(0.5, 0), 12.0])])
    sh, ch = np.empty_like(x), np.empty_like(x)
    P = C.POINTER(C.c_double)
    emulator().emu_sinh_cosh(x.ctypes.data_as(P), C.c_long(len(x)), sh.ctypes.data_as(P), ch.ctypes.data_as(P))
    nz = x != 0
    assert (np.abs(sh[nz] - np.sinh(x[nz])) <= 4 * np.spacing(np.abs(np.sinh(x[nz])))).all()
    assert (np.abs(ch - np.cosh(x)) <= 4 * np.spacing(np.cosh(x))).all()
    assert sh[x == 0].tolist() == [0.0] and ch[x == 0].tolist() == [1.0]


@pytest.mark.parametrize("dim,mode,reg_out", [(3, 1, (0, 0)), (3, 1, (1, 1)), (3, 1, (1, 0)), (3, 1, (0, 1)),
                                               (3, 2, (0, 0)), (3, 2, (1, 1)), (2, 1, (0, 0)), (2, 2, (1, 0))])
def test_table_and_tail_algebra(dim, mode, reg_out):
    """k_spectra's F_TB algebra (variant 1, sep_quad_tb_t: linear delta-f part from the {PD, T1} / {TE, T2}
    tables) and its Boltzmann-tail lanes (variant 3, sep_quad_tb_tail_t: den == a, no reciprocal) on the
    host, against the oracle: every regulate / outflow variant, 2+1D lanes with w_eta != 1 (escw), and the
    3+1D grid's 2^-k-scaled lanes (x - zb > 150).  Same bar as the GPU tier: entries that sum
    mixed-sign contributions keep ~1e-10 relative (measured 1e-10..3e-9 for every variant alike)."""
    s = synth.as_read(synth.surface(6, seed=19, dimension=dim, full3d=(dim == 3)))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=dim, pT="pT24", phi="phi24",
                     regulate_deltaf=reg_out[0], outflow=reg_out[1])
    ref = O.spectra(spec, s, threads=1)
    base, _ = emu_spectra(spec, s)
    for variant in (1, 3):
        got, _ = emu_spectra(spec, s, variant=variant)
        rel, zr, zg = parity(got, ref, floor=1e-290)
        assert rel < 1e-8, (variant, rel)
        assert zr == zg
        assert not np.array_equal(got, base)       # the variant's arithmetic really ran


@pytest.mark.parametrize("dim,outflow", [(3, 0), (3, 1), (2, 0)])
def test_near_tail_lanes(dim, outflow):
    """Near-tail Grad lanes of the F_TS launch (sep_quad_tb_near_t, smallest exponent in (kNearX, kTailX]:
    1 / (1 + u) = 1 - u with u <= e^-18, no reciprocal) on the host against the oracle: the lanes occur, the
    max relative error keeps the 1e-8 bar and the 99th percentile the 1e-11 drift guard of the GPU tier."""
    s = synth.as_read(synth.surface(8, seed=41, dimension=dim, full3d=(dim == 3)))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=1, dimension=dim, pT="pT24", phi="phi24", outflow=outflow)
    ref = O.spectra(spec, s, threads=1)
    # [pT][cell][species][q] lane kinds (1 + skip 0 / tail 1 / other 2 / near 3), sized for any q layout
    kinds = np.zeros(len(spec["pT"]) * 8 * len(spec["species"]["mass"]) * len(spec["y"]) * len(spec["eta"]), np.int8)
    emulator().emu_set_census_lanes(kinds.ctypes.data_as(C.c_void_p))
    try:
        got, _ = emu_spectra(spec, s, variant=3)
    finally:
        emulator().emu_set_census_lanes(None)
    assert (kinds == 4).sum() > 0.05 * (kinds > 1).sum()      # near-tail lanes really ran
    rel, zr, zg = parity(got, ref, floor=1e-290)
    assert rel < 1e-8, rel
    assert zr == zg
    assert rel_quantile(got, ref, floor=1e-290) < 1e-11


PHI30 = (2 * np.pi * np.arange(30) / 30, np.full(30, 2 * np.pi / 30))


@pytest.mark.parametrize("dim,mode,baryon,reg_out,phi", [
    (3, 1, 1, (0, 0), "phi32"), (3, 2, 1, (0, 0), "phi32"), (3, 2, 0, (1, 1), "phi24"), (3, 1, 1, (1, 0), PHI30),
    (3, 2, 1, (0, 1), PHI30), (2, 1, 0, (0, 0), "phi24"), (2, 2, 1, (1, 0), "phi24")])
def test_pd_tail_lanes(dim, mode, baryon, reg_out, phi):
    """Boltzmann-tail lanes of k_spectra's per-lane Grad / RTA-CE launches (variant 2, sep_quad_pd_tail_t: the
    PD-table fours with 1/a folded into p.dsigma, 1 - sign f_eq = 1, one 1/E per four points for RTA-CE) on the
    host, against the oracle: baryon on (the launches that carry it), regulate / outflow, a 30-point phi
    row padded to the 32-point block, 2+1D eta-weighted lanes."""
    s = synth.as_read(synth.surface(6, seed=23, dimension=dim, baryon=bool(baryon), full3d=(dim == 3)))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=dim, pT="pT24", phi=phi,
                     include_baryon=baryon, include_baryondiff_deltaf=baryon,
                     regulate_deltaf=reg_out[0], outflow=reg_out[1])
    ref = O.spectra(spec, s, threads=1)
    base, _ = emu_spectra(spec, s)
    got, _ = emu_spectra(spec, s, variant=2)
    rel, zr, zg = parity(got, ref, floor=1e-290)
    assert rel < 1e-8, rel
    assert zr == zg
    assert not np.array_equal(got, base)       # the tail arithmetic really ran


@pytest.mark.parametrize("dim,baryon,reg_out,phi", [(3, 1, (0, 0), "phi32"), (3, 0, (1, 1), "phi32"),
                                                      (3, 1, (1, 0), PHI30), (3, 1, (0, 1), "phi24"),
                                                      (2, 0, (0, 0), "phi24")])
def test_ce_te_table_lanes(dim, baryon, reg_out, phi):
    """RTA-CE lanes of k_spectra's per-lane launch with the per-(cell, phi) {TE, T2} table (variant 64,
    sep_quad_pde_t: E = E0 + TE, linear delta-f part fma(a, T2, L0)), normal and Boltzmann-tail (2), against the
    oracle: baryon on, regulate / outflow, a 30-point phi row padded to the 32-point block, 2+1D."""
    s = synth.as_read(synth.surface(6, seed=31, dimension=dim, baryon=bool(baryon), full3d=(dim == 3)))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=2, dimension=dim, pT="pT24", phi=phi,
                     include_baryon=baryon, include_baryondiff_deltaf=baryon,
                     regulate_deltaf=reg_out[0], outflow=reg_out[1])
    ref = O.spectra(spec, s, threads=1)
    base, _ = emu_spectra(spec, s)
    for variant in (64, 64 | 2):
        got, _ = emu_spectra(spec, s, variant=variant)
        rel, zr, zg = parity(got, ref, floor=1e-290)
        assert rel < 1e-8, (variant, rel)
        assert zr == zg
        assert not np.array_equal(got, base)


@pytest.mark.parametrize("mode,baryon", [(3, 0), (4, 0), (5, 0), (3, 1), (5, 1)])
def test_modified_table_lanes(mode, baryon):
    """k_spectra's modified-path table lanes (variant 4: mod_quad_tab_t in exp-table units -- e^(-E_mod/T_mod)
    with e^chem folded into the lane's sign and p.dsigma coefficients, four points per reciprocal
    accumulated by FMA) against the oracle on the config-2 grid, with baryon chemistry (chem != 0) on."""
    s = synth.as_read(synth.surface(6, seed=23, dimension=3, full3d=True, baryon=bool(baryon)))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=3, pT="pT24", phi="phi32", famod_chains=1,
                     include_baryon=baryon)
    ref = O.spectra(spec, s, threads=1)
    got, _ = emu_spectra(spec, s, chains=1, variant=4)
    rel, zr, zg = parity(got, ref, floor=1e-290)
    assert rel < 1e-8, rel
    assert zr == zg
    # the Boltzmann-tail table lanes (variant 16, mod_quad_tab_tail_t: |sign e^chem 2^-k| < 2^-55, no denominators)
    tail, _ = emu_spectra(spec, s, chains=1, variant=4 | 16)
    rel, zr, zg = parity(tail, ref, floor=1e-290)
    assert rel < 1e-8, rel
    assert zr == zg
    assert not np.array_equal(tail, got)


def test_modified_wide_lanes_exact_range():
    """Modified lanes whose momentum bounds |mT U| -+ pT |V|max span more than 250 binades (high pT, strong
    modification): mod_setup<KJ> takes the exact range of the lane's points (IS3D_MOD_EXACT), so they run the
    table / Boltzmann-tail fours instead of the clamped en form.  On the config-2 grid the clamped share falls from
    ~5% of the lanes to ~0.1% (tools: /tmp census of round 5); the spectra still meet the oracle."""
    s = synth.as_read(synth.surface(6, seed=31, dimension=3, full3d=True))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=3, dimension=3, pT="pT48", phi="phi32")
    cnt = np.zeros(4, dtype=np.int64)
    lib = emulator()
    lib.emu_set_census_mod(cnt.ctypes.data_as(C.POINTER(C.c_long)))
    try:
        got, _ = emu_spectra(spec, s, variant=4 | 16)
    finally:
        lib.emu_set_census_mod(None)
    skip, clamp, tail, other = (int(v) for v in cnt)
    live = clamp + tail + other
    assert tail > 0 and other > 0
    assert clamp < 0.01 * live, cnt
    ref = O.spectra(spec, s, threads=4)
    rel, zr, zg = parity(got, ref, floor=1e-290)
    assert rel < 1e-8, rel
    assert zr == zg
    assert rel_quantile(got, ref) < 1e-11


@pytest.mark.parametrize("mode", [1, 2])
def test_slow_cell_bound_sweep(mode):
    """sep_slow_cell (k_prep's per-cell bound that sends a surface to the kernels with the slow per-point loop instead
    of F_TS, engine.hip launch_end): swept across its threshold -- mu_B / T from 250 to 340 in 1-unit steps, flow
    u_perp up to ~3 -- every separable lane whose smallest exponent x - zb falls below kExpFast = -300 must sit in a
    flagged cell, and the bound flags nothing below mu_B / T = 290 (its margin of 10)."""
    n = 91
    s = synth.as_read(synth.surface(n, seed=37, dimension=3, baryon=True, full3d=True))
    chem = 250.0 + np.arange(n)
    s["T"] = np.full(n, 0.12)
    s["muB"] = chem * 0.12
    flow = 1.0 + 2.0 * (np.arange(n) % 7) / 6.0
    s["ux"] = s["ux"] * flow
    s["uy"] = s["uy"] * flow
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode, dimension=3, pT="pT24", phi="phi32", y="y21",
                     include_baryon=1, include_baryondiff_deltaf=1)
    T, muB, tab = spec["df"]
    spec["df"] = (T, np.asarray(muB) * 100.0, tab)     # stretched mu_B axis: the tables reach mu_B / T = 375
    out = np.zeros(5, dtype=np.int64)
    lib = emulator()
    lib.emu_set_slow_check(out.ctypes.data_as(C.POINTER(C.c_long)))
    try:
        emu_spectra(spec, s, variant=1 | 2)
    finally:
        lib.emu_set_slow_check(None)
    off_fast, violations, flagged, live = (int(v) for v in out[:4])
    min_ok = float(out[4:5].view(np.float64)[0])
    assert live > 0.9 * n                  # (u.dsigma <= 0 cells are skipped)
    assert off_fast > 0                    # the sweep reaches lanes off the fast path ...
    assert violations == 0, out            # ... and every one of them is in a flagged cell
    assert 0 < flagged < n                 # the threshold falls inside the sweep
    assert min_ok > -300.0, min_ok         # unflagged cells keep every lane on the fast path
    assert flagged <= int(np.sum(chem >= 289.0)), (flagged, out)   # nothing flagged well below mu_B / T = 290
