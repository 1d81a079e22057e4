"""CPU tier: pin the oracle (CPU restatement) before trusting it.

Pins available for this path:
  * the SURVEY's known-answer test, measured on the reference binary: Grad (c0, c2, shear14)
    = (-136.921523, -17.198566, 0.014627) for the config-1 synthetic surface (1000 cells,
    seed 7) with SMASH tables at the surface-average T and Pi = -0.1 P
    (Deltaf_Data::test_df_coefficients, DeltafData.cpp:522-553, called iS3D.cpp:249);
  * the reference's hard-coded 16-point Gauss-Laguerre literals (bit-identical regeneration);
  * the GSL-free reference sources compiled into oracle/_ref (tests/test_ref_pins.py).
"""
import re

import numpy as np
import pytest

from is3d2_amd import make_spec, synth
from oracle import oracle as O


def test_survey_kat_grad_coefficients():
    s = synth.as_read(synth.surface(1000, seed=7))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1)
    T, E, P, muB, nB = O.averages(s)
    rc, out = O.df_coefficients(spec, T, muB, E, P, -0.1 * P)
    assert rc == 0
    got = "(%lf, %lf, %lf)" % (out[0], out[2], out[5])
    assert got == "(-136.921523, -17.198566, 0.014627)"


def test_gl16_header_is_the_reference_quadrature():
    # values checked bit-for-bit against AnisoVariables.h when generated (tools/gen_gl16.py);
    # here: they are the 16-point generalized Gauss-Laguerre rules for alpha = 1, 2, 3
    from scipy.special import roots_genlaguerre
    hdr = open("include/is3d_gl16.h").read()
    for a in (1, 2, 3):
        r = np.array([float(v) for v in re.search(r"ROOT_A%d \{([^}]*)\}" % a, hdr).group(1).split(",")])
        w = np.array([float(v) for v in re.search(r"WEIGHT_A%d \{([^}]*)\}" % a, hdr).group(1).split(",")])
        x, wt = roots_genlaguerre(16, a)
        assert np.max(np.abs(r - x) / x) < 1e-14
        assert np.max(np.abs(w - wt) / wt) < 1e-12


@pytest.mark.parametrize("mode", [1, 2, 3, 4])
def test_oracle_thread_count_invariance(mode):
    # Grad/CE/PTM/PTB: results depend on the OpenMP thread count only through summation order
    s = synth.as_read(synth.surface(120, seed=3))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode, pT="pT24", phi="phi24")
    a = O.spectra(spec, s, threads=1)
    b = O.spectra(spec, s, threads=7)
    assert np.max(np.abs(a - b) / np.abs(a)) < 1e-11


def test_oracle_ptma_warm_start_depends_on_threads():
    # PTMA warm-starts from the previous cell of the same thread (tol 1e-4)
    s = synth.as_read(synth.surface(120, seed=3))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5, pT="pT24", phi="phi24")
    a, sa = O.spectra(spec, s, threads=1, return_stats=True)
    b = O.spectra(spec, s, threads=4)
    d = np.max(np.abs(a - b) / np.abs(a))
    assert 0 < d < 1e-5
    assert 2.0 < sa[3] / 120 < 6.0   # mean Newton iterations (SURVEY: 3.8)


def test_oracle_out_of_range_temperature_is_an_error():
    s = synth.as_read(synth.surface(10, seed=3))
    s["T"] = s["T"].copy(); s["T"][4] = 0.25      # outside T in [0.1, 0.2] GeV: GSL aborts in the reference
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=2)
    with pytest.raises(RuntimeError, match="interpolation"):
        O.spectra(spec, s, T_avg=0.15)


def test_analytic_ideal_single_cell():
    # physics KAT independent of the reference: one static 3+1D cell, no viscous terms,
    # dN/(pT dpT dphi dy) = g/(2 pi hbarc)^3 * mT cosh(y-eta) dat / (exp(mT cosh(y-eta)/T) + sign)
    n = 1
    s = {k: np.zeros(n) for k in synth.FIELDS}
    s.update(tau=np.ones(n), dat=np.full(n, 2.0), T=np.full(n, 0.15), E=np.full(n, 0.3), P=np.full(n, 0.1),
             eta=np.full(n, 0.3))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=2, dimension=3, include_bulk_deltaf=0, include_shear_deltaf=0)
    out = O.spectra(spec, s).reshape(3, 24, 24, 21)
    sp = spec["species"]
    pT = spec["pT"][:, None]; y = spec["y"][None, :]
    for i in range(3):
        mT = np.sqrt(sp["mass"][i] ** 2 + pT ** 2)
        ch = np.cosh(y - 0.3)
        want = sp["degen"][i] * (2 * np.pi * 0.197327053) ** -3 * mT * ch * 2.0 / (np.exp(mT * ch / 0.15) + sp["sign"][i])
        np.testing.assert_allclose(out[i, :, 0, :], want, rtol=1e-12)
