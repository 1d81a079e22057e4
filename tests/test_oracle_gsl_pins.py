"""CPU tier: the oracle's restatement of GSL's natural cubic spline against an independent implementation.

The reference interpolates its delta-f coefficient tables and PTB's Jonah table with GSL's gsl_interp_cspline
(DeltafData.cpp:298-402, GSL 2.x cspline.c + linalg/tridiag.c: the natural cubic spline, second derivatives
zero at both ends).  GSL is not in this image, so oracle/is3d_oracle.c restates it (cspline_init /
cspline_eval).  scipy.interpolate.CubicSpline(bc_type="natural") is an independent implementation of the same
published algorithm; on the reference's own tables the two agree to rounding (~5e-16), which pins the restated
GSL step of the oracle to a third-party implementation (the spectra loops and the Newton solve remain pinned to
the reference-compiled sources and fixtures only: DESIGN.md section 4).
"""
import numpy as np
import pytest
from scipy.interpolate import CubicSpline

from is3d2_amd import make_spec
from oracle import oracle as O

# oracle df_coefficients output slots (orc_df_coefficients) and the table column / T power they come from
# (DeltafData.cpp:324-366: c0, c2 / T^4 for Grad, F T, betabulk T^4, betapi T^4 for the other modes)
SLOTS = {1: [(0, 0, -4), (2, 2, -4)], 2: [(6, 5, 1), (8, 7, 4), (10, 9, 4)], 3: [(6, 5, 1), (8, 7, 4), (10, 9, 4)]}


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_df_table_splines_match_natural_cubic_spline(mode):
    sp = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode)
    T, muB, tab = (np.asarray(a) for a in sp["df"])
    tab = tab.reshape(-1, len(muB), len(T))
    # table nodes, midpoints and a dense sweep of the whole T range (the range check is GSL's: test_oracle_pins)
    ts = np.unique(np.concatenate([T, 0.5 * (T[1:] + T[:-1]), np.linspace(T[0], T[-1], 257)]))
    worst = 0.0
    for t in ts:
        rc, out = O.df_coefficients(sp, t, 0.0, 0.5, 0.15, -0.01)
        assert rc == 0
        for slot, col, pw in SLOTS[mode]:
            ref = CubicSpline(T, tab[col, 0], bc_type="natural")(t) * t ** pw
            worst = max(worst, abs(out[slot] - ref) / abs(ref))
    assert worst < 1e-14, worst


def test_jonah_table_splines_match_natural_cubic_spline():
    # PTB: lambda(bulkPi / P) and z(bulkPi / P) from the 301-point Jonah table (DeltafData.cpp:369-380)
    sp = make_spec(hrg_eos=2, chosen="smash", df_mode=4)
    T_avg = 0.15
    rc, l2, z, bp, bpmax = O.jonah_table(sp, T_avg)
    assert rc == 0 and np.all(np.diff(bp) > 0)
    s_l2 = CubicSpline(bp, l2, bc_type="natural")
    s_z = CubicSpline(bp, z, bc_type="natural")
    P = 0.1
    worst = 0.0
    for x in np.linspace(bp[0], bp[-1], 41)[1:-1]:
        rc, out = O.df_coefficients(sp, T_avg, 0.0, 0.3, P, x * P, T_avg=T_avg)
        assert rc == 0
        lam = np.sqrt(s_l2(x)) * np.sign(x)
        worst = max(worst, abs(out[11] - lam) / max(abs(lam), 1e-3), abs(out[12] - s_z(x)) / abs(s_z(x)))
    assert worst < 1e-12, worst


def test_lu3_matches_lapack_partial_pivoting():
    # gsl_linalg_LU_decomp / _solve (AnisoVariables.cpp:470-480 Newton steps, MomentumSpectra.cpp:1132-1135 A^-1):
    # partial pivoting on the first largest |a_ij| of the column, as LAPACK's dgetrf (scipy.linalg.lu_factor)
    from scipy.linalg import lu_factor, lu_solve
    rng = np.random.default_rng(11)
    mats = [rng.normal(size=(3, 3)) for _ in range(200)]
    # modified-momentum transforms A = 1 + shear + bulk (close to the identity) and Newton Jacobians (wide scales)
    mats += [np.eye(3) + 0.3 * rng.normal(size=(3, 3)) for _ in range(100)]
    mats += [rng.normal(size=(3, 3)) * np.array([1e3, 1.0, 1e-3])[:, None] for _ in range(100)]
    worst = 0.0
    for A in mats:
        b = rng.normal(size=3)
        x, perm = O.lu3_solve(A, b)
        lu, piv = lu_factor(A)
        ref = lu_solve((lu, piv), b)
        # LAPACK's row swaps (piv: row i swapped with piv[i]) applied to the identity order give GSL's permutation
        order = list(range(3))
        for i, p in enumerate(piv):
            order[i], order[p] = order[p], order[i]
        assert order == perm
        # forward error in units of eps x cond(A): rounding of two different operation orders only
        worst = max(worst, np.max(np.abs(x - ref)) / np.max(np.abs(ref)) / (np.finfo(float).eps * np.linalg.cond(A)))
    assert worst < 4.0, worst
