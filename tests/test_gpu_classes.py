"""GPU tier: integrand classes (is3d_set_species_classes, include/is3d_amd.h).

The momentum integrals see a chosen species only through its (mass, sign, baryon) -- plus, in PTM, whether its
degeneracy is zero: the n_linear / n_mod renormalisation (MomentumSpectra.cpp:800-808) is a ratio of two sums that
both carry g, except for g = 0 (0 / 0: the species is skipped) -- and the degeneracy
multiplies the result (MomentumSpectra.cpp:365).  The engine therefore integrates one lane species per class
(SMASH 444 -> 193, UrQMD 305 -> 124) and its reduction writes every member.  These tests check that the
spectra, dN/dX and per-cell yields are bit-identical to the per-species integration (classes off) wherever
both launches take the same plan (phi block, cell splits: the BASELINE sizes) and the same lane forms, and
equal to rounding where the class count changes the plan or the wavefront-wide tail decision of the Grad
F_TB launch; every oracle comparison elsewhere in the GPU tier runs with classes on (the default)."""
import numpy as np
import pytest

from helpers import parity
from is3d2_amd import build_engine, make_spec, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def spectra(spec, s, classes):
    e = build_engine(spec, s, species_classes=classes)
    n = e.species_integrated()
    out = e.calculate_spectra()
    st = e.stats()
    e.close()
    return out, n, st


@pytest.mark.parametrize("mode", [1, 2, 3, 4, 5])
def test_classes_config3_grid(mode):
    """Config 3's shape (SMASH 444 x 48 x 32 x 21, 3+1D, shear + bulk (+ baryon + diffusion; PTB without,
    DeltafData.cpp:480-483)): classes on and off give the same spectra to rounding (every mode's Boltzmann-tail
    form is decided per wavefront, and the two launches group different lanes into wavefronts; before the
    wavefront-wide decisions they agreed bit for bit), the same breakdown count, and the class count is the key's."""
    baryon = mode != 4
    s = synth.as_read(synth.surface(10, seed=41, dimension=3, baryon=baryon, full3d=True))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=3, pT="pT48", phi="phi32", y="y21",
                     include_baryon=int(baryon), include_baryondiff_deltaf=int(baryon), famod_chains=1)
    on, n_on, st_on = spectra(spec, s, True)
    off, n_off, st_off = spectra(spec, s, False)
    sp = spec["species"]
    # PTM keys on whether the degeneracy is zero (its renormalisation ratio is g-independent otherwise, engine.hip
    # ptm_gkey): SMASH has no g = 0 species, so every mode integrates 193 classes
    key = zip(sp["mass"], sp["sign"], sp["baryon"], [g == 0 for g in sp["degen"]] if mode == 3 else [0] * len(sp["mass"]))
    assert n_off == len(sp["mass"]) == 444
    assert n_on == len(set(key)) == 193
    # Boltzmann-tail forms decided per wavefront (sep_setup allow_tail = 2, mod_setup allow_tail): equal to rounding
    assert parity(on, off, floor=1e-290)[0] < 1e-9
    assert np.array_equal(np.isfinite(on), np.isfinite(off))
    assert st_on["breakdown"] == st_off["breakdown"]


def test_classes_grad_config2_full_size():
    """Config 2 at full size (10^5 cells, Grad without baryon: the headline's F_TB table launch): the class and
    per-species launches pick the same phi block and cell splits here.  The F_TB launch decides the
    Boltzmann-tail form once per wavefront (sep_setup allow_tail = 2) and the two launches group different
    lanes into their wavefronts, so a lane may take the tail form in one and the normal fours in the other:
    the same f_eq (1 + delta-f) to rounding (the tail form drops a sign e^-x < 2^-54 term), not bit for bit."""
    s = synth.as_read(synth.surface(100000, seed=7, dimension=3))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=1, dimension=3, pT="pT48", phi="phi32", y="y21")
    on, n_on, _ = spectra(spec, s, True)
    off, _, _ = spectra(spec, s, False)
    assert n_on == 193
    rel, _, _ = parity(on, off, floor=1e-290)
    print("classes on vs off: max rel %.3g" % rel)
    assert rel < 1e-9, rel
    assert np.array_equal(np.isfinite(on), np.isfinite(off))


def test_classes_small_surface_split_plan():
    """On a small surface the cell-split count follows the launch's workgroup count (engine.hip: >= 8k
    workgroups), which the class count changes (16 vs 8 splits at 2000 cells): the slabs group the cells
    differently, so the sums agree to rounding, not bit for bit (4.3e-11 measured, on entries where the
    delta-f terms nearly cancel; the oracle bar elsewhere is 1e-8)."""
    s = synth.as_read(synth.surface(2000, seed=7, dimension=3))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=1, dimension=3, pT="pT48", phi="phi32", y="y21")
    on, _, _ = spectra(spec, s, True)
    off, _, _ = spectra(spec, s, False)
    assert parity(on, off, floor=1e-290)[0] < 1e-9


@pytest.mark.parametrize("mode", [1, 3, 5])
def test_classes_urqmd_2d(mode):
    """UrQMD (305 -> 124 classes) in 2+1D with 24 eta nodes: a different class count can change the phi-block
    plan, so the check is the oracle's tolerance plus agreement with the per-species run to rounding."""
    s = synth.as_read(synth.surface(30, seed=5, dimension=2, baryon=mode == 5))
    spec = make_spec(hrg_eos=1, chosen="urqmd", df_mode=mode, dimension=2, include_baryon=int(mode == 5),
                     famod_chains=1)
    on, n_on, _ = spectra(spec, s, True)
    off, n_off, _ = spectra(spec, s, False)
    assert n_off == 305 and n_on < n_off
    assert parity(on, off, floor=1e-290)[0] < 1e-12
    ref = O.spectra(spec, s, threads=1)
    assert parity(on, ref, floor=1e-290)[0] < 1e-8


@pytest.mark.parametrize("mode", [1, 3])
def test_classes_dndx_and_cell_yields(mode):
    """operation = 0 (k_dndx integrates the classes, k_stbin scales each member): bit-identical bins and
    per-cell yields."""
    s = synth.as_read(synth.surface(200, seed=3, dimension=2))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=2)
    res = []
    for classes in (True, False):
        e = build_engine(spec, s, species_classes=classes)
        t, r, ph = e.calculate_dN_dX()
        res.append((t, r, ph, e.cell_yields()))
        e.close()
    for a, b in zip(*res):
        assert np.array_equal(a, b)


def test_classes_device_group():
    """A device list that repeats GPU 0 (the group engine forwards the setting to every shard): against the
    oracle at the parity bar (the shards sum the cells in another grouping, and with classes on RTA-CE takes
    the per-lane launch where 444 species take the table launch, so the class and per-species runs agree to
    rounding only: 1.4e-9 measured on near-cancelling entries)."""
    s = synth.as_read(synth.surface(60, seed=9, dimension=3))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=2, dimension=3, pT="pT48", phi="phi32", y="y21")
    e = build_engine(spec, s, devices=[0, 0])
    assert e.species_integrated() == 193
    got = e.calculate_spectra()
    e.close()
    off, _, _ = spectra(spec, s, False)
    ref = O.spectra(spec, s, threads=8)
    assert parity(got, ref, floor=1e-290)[0] < 1e-8
    assert parity(off, ref, floor=1e-290)[0] < 1e-8


def test_ptm_classes_ignore_the_degeneracy_except_zero():
    """PTM's classes key on g == 0 only (engine.hip ptm_gkey): SMASH species that differ only in g share a class,
    and a species given g = 0 keeps its own (its renormalisation is 0 / 0 = NaN, so the reference skips it and its
    spectrum stays 0) -- against the oracle, which evaluates every species with its own g."""
    s = synth.as_read(synth.surface(12, seed=61, dimension=3, full3d=True))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=3, dimension=3, pT="pT24", phi="phi32", y="y21")
    sp = dict(spec["species"])
    g = np.array(sp["degen"], dtype=float)
    z = int(np.argmax(np.array(sp["mass"]) > 1.0))      # the first species above 1 GeV
    g[z] = 0.0
    sp["degen"] = g
    spec = dict(spec, species=sp)
    out, n_on, _ = spectra(spec, s, True)
    key = set(zip(sp["mass"], sp["sign"], sp["baryon"], [v == 0 for v in g]))
    assert n_on == len(key)
    ref = O.spectra(spec, s, threads=8)
    rel, zr, zg = parity(out, ref)
    assert rel < 1e-8, (rel, zr, zg)
    assert zr == zg
    nph = out.size // len(g)
    assert not np.any(out.reshape(len(g), nph)[z])      # the g = 0 species: skipped, all zero
