"""GPU tier for the operation = 2 oversampling estimate: is3d_total_yield (k_densities + k_yield)
against the oracle's restatement of ParticleSampler.cpp:447-636 / DeltafData.cpp:555-690 on the
same seeded surfaces, every df_mode, 2+1D / 3+1D, baryon diffusion on / off, plus exact
properties at the BASELINE config-2 surface size."""
import numpy as np
import pytest

from is3d2_amd import IS3DError, build_engine, make_spec, surface_averages, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-12   # sums of ~1e3..1e5 positive-dominated cell terms; only the summation order differs


@pytest.mark.parametrize("mode,dim,baryon", [(1, 2, 0), (2, 2, 0), (3, 3, 0), (4, 2, 0), (5, 3, 0),
                                             (1, 3, 1), (2, 3, 1), (3, 2, 1), (5, 2, 1), (4, 3, 0)])
def test_total_yield_parity(mode, dim, baryon):
    flags = dict(include_baryon=baryon, include_baryondiff_deltaf=baryon)
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=dim, **flags)
    s = synth.as_read(synth.surface(3000, seed=21, dimension=dim, baryon=bool(baryon), full3d=(dim == 3)))
    plasma = O.averages(s, baryon)
    n_ref, d_ref = O.total_yield(spec, s, plasma, y_cut=0.5)
    e = build_engine(spec, s, T_avg=plasma[0])
    n, d = e.total_yield(plasma, y_cut=0.5)
    e.close()
    assert abs(n - n_ref) <= TOL * abs(n_ref), (n, n_ref)
    np.testing.assert_allclose(d, d_ref, rtol=1e-13, atol=1e-300)


def test_total_yield_empty_surface_and_plasma_from_engine():
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=2, dimension=2)
    s = synth.as_read(synth.surface(500, seed=3))
    plasma = surface_averages(s, 0)
    np.testing.assert_array_equal(plasma, O.averages(s, 0))
    e = build_engine(spec, s)
    n, _ = e.total_yield(plasma)
    e.set_surface({k: v[:0] for k, v in s.items()})
    n0, d0 = e.total_yield(plasma)
    e.close()
    assert n > 0 and n0 == 0.0 and np.all(np.isfinite(d0))


def test_total_yield_out_of_table_is_an_error():
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1, dimension=2)
    s = synth.as_read(synth.surface(100, seed=3))
    s["T"] = s["T"].copy()
    s["T"][17] = 0.5                      # outside the 0.1..0.2 GeV coefficient spline
    e = build_engine(spec, s, T_avg=0.15)
    with pytest.raises(IS3DError):
        e.total_yield(O.averages(s, 0))
    e.close()


@pytest.mark.parametrize("mode", [1, 4])
def test_total_yield_full_size_properties(mode):
    """config-2 surface (10^5 3+1D cells, SMASH): exact linearity in dsigma (every cell term doubles
    exactly and the fixed-order sum with it), additivity over a cell split, and the oracle on a prefix."""
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=3)
    s = synth.as_read(synth.surface(100000, seed=7, dimension=3, full3d=True))
    plasma = O.averages(s, 0)
    e = build_engine(spec, s, T_avg=plasma[0])
    n, _ = e.total_yield(plasma)
    s2 = dict(s)
    for k in ("dat", "dax", "day", "dan"):
        s2[k] = 2.0 * s[k]
    e.set_surface(s2)
    n2, _ = e.total_yield(plasma)
    h = 40000
    e.set_surface({k: np.ascontiguousarray(v[:h]) for k, v in s.items()})
    a, _ = e.total_yield(plasma)
    e.set_surface({k: np.ascontiguousarray(v[h:]) for k, v in s.items()})
    b, _ = e.total_yield(plasma)
    e.close()
    assert n2 == 2.0 * n
    assert abs((a + b) - n) <= TOL * abs(n)
    ref_a, _ = O.total_yield(spec, {k: v[:h] for k, v in s.items()}, plasma, y_cut=0.5)
    assert abs(a - ref_a) <= TOL * abs(ref_a)
