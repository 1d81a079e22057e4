"""GPU tier for operation = 0 (spacetime distributions, SpacetimeDistribution.cpp:31-1250):
libis3d_amd.so (k_prep op 0 + k_dndx + k_stkeys/k_stbin) against the oracle on the same
seeded inputs.  Per-cell yields dN_dy_cell and the binned, normalised distributions the
reference writes (dN_taudtaudy, dN_2pirdrdy, dN_dphidy)."""
import numpy as np
import pytest

from helpers import parity
from is3d2_amd import IS3DError, build_engine, make_spec, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-9   # FP64 sums over the momentum grid in a different order than the reference


def run_gpu(spec, surf):
    e = build_engine(spec, surf)
    t, r, ph = e.calculate_dN_dX()
    cy = e.cell_yields()
    e.close()
    return t, r, ph, cy


def check(got, ref):
    for g, f in zip(got, ref):
        rel, zr, zg = parity(g.ravel(), f.ravel())
        assert rel < TOL, rel
        assert zr == zg


@pytest.mark.parametrize("dim", [2, 3])
@pytest.mark.parametrize("mode", [1, 2, 3, 4])
def test_dndx_parity(dim, mode):
    s = synth.as_read(synth.surface(200, seed=31, dimension=dim, full3d=(dim == 3)))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode, dimension=dim)
    ref = O.dndx(spec, s, threads=1, carry=0, return_cells=True)
    got = run_gpu(spec, s)
    check(got, ref)


@pytest.mark.parametrize("C", [1, 4])
def test_dndx_reference_thread_carry(C):
    s = synth.as_read(synth.surface(300, seed=32))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1, dimension=2, threads=C)
    ref = O.dndx(spec, s, threads=C, carry=1)
    got = run_gpu(spec, s)[:3]
    check(got, ref)


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_dndx_baryon_flags(mode):
    s = synth.as_read(synth.surface(120, seed=33, dimension=3, baryon=True, full3d=True))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode, dimension=3, include_baryon=1,
                     include_baryondiff_deltaf=1, regulate_deltaf=1, outflow=1)
    check(run_gpu(spec, s), O.dndx(spec, s, carry=0, return_cells=True))


@pytest.mark.parametrize("mode", [2, 3, 4])
def test_dndx_smash_many_lane_groups(mode):
    # 444 species: 7 species groups of 64 mass-sorted species, 21 y tasks over 4 slots; 70 cells end in a ragged record
    # tile of the 8-cell separable launches and of the modified launch's 4-cell tiles (its per-(cell, species) PTM
    # renorm rows and {PDm, Qv} rows, round 6)
    s = synth.as_read(synth.surface(70, seed=34, dimension=3))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=3, pT="pT48", phi="phi32")
    check(run_gpu(spec, s), O.dndx(spec, s, threads=8, carry=0, omp_threads=8, return_cells=True))


def test_dndx_many_tasks_and_phi_blocks():
    # 70 y x 4 phi blocks (100-point phi grid, padded to 128) = 280 tasks per species over 4 x 21 slots
    s = synth.as_read(synth.surface(20, seed=35, dimension=3))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1, dimension=3)
    spec["y"] = np.linspace(-5.0, 5.0, 70)
    spec["phi"] = 2 * np.pi * (np.arange(100) + 0.5) / 100
    spec["phi_w"] = np.full(100, 2 * np.pi / 100)
    check(run_gpu(spec, s), O.dndx(spec, s, carry=0, return_cells=True))


def test_dndx_ptma_rejected_and_empty_surface():
    s = synth.as_read(synth.surface(10, seed=36))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5)
    e = build_engine(spec, s)
    with pytest.raises(IS3DError, match="no spacetime distribution routine for famod"):
        e.calculate_dN_dX()
    e.close()
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1)
    e = build_engine(spec, s)
    e.set_surface({k: (v[:0] if v is not None else None) for k, v in s.items()})
    t, r, ph = e.calculate_dN_dX()
    e.close()
    assert not t.any() and not r.any() and not ph.any()
