"""CPU tier: the engine's device math (cf_math.h / aniso_math.h), run serially on the
host by the test-only emulator, against the oracle.  The GPU tier repeats this through
libis3d_amd.so on the MI355X."""
import numpy as np
import pytest

from helpers import emu_spectra, parity
from is3d_amd import make_spec, synth
from oracle import oracle as O

CASES = [(d, m) for d in (2, 3) for m in (1, 2, 3, 4, 5)]


@pytest.mark.parametrize("dim,mode", CASES)
def test_factorised_math_matches_oracle(dim, mode):
    s = synth.as_read(synth.surface(150, seed=11, dimension=dim, full3d=(dim == 3)))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode, dimension=dim, pT="pT24", phi="phi24")
    ref = O.spectra(spec, s, threads=1)
    got, _ = emu_spectra(spec, s, chains=1)
    rel, zr, zg = parity(got, ref)
    assert rel < 1e-9, rel
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
