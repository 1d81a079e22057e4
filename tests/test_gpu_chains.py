"""GPU tier: PTMA warm-start chains (MomentumSpectra.cpp:1308-1364) on the segmented chain solver
(engine.hip k_chain_pass / k_chain_finish) against the oracle's serial chains.

The reference warm-starts every Newton solve from the state the previous cell of its OpenMP thread left; as
shipped it is serial (one chain).  The engine cuts each chain into segments solved in parallel and
re-synchronises them pass by pass until no segment's end state changes -- which must reproduce the serial
chain bit for bit: the same Newton iteration count as the oracle and spectra at rounding level.  The
surfaces hold thousands of cells so every chain spans many 32-cell segments."""
import numpy as np
import pytest

from helpers import parity
from is3d2_amd import build_engine, make_spec, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu
TOL = 1e-8


def run_gpu(spec, surf):
    e = build_engine(spec, surf)
    out = e.calculate_spectra()
    st = e.stats()
    e.close()
    return out, st


@pytest.mark.parametrize("chains", [1, 3, 16])
def test_segmented_chains_match_serial_chains(chains):
    s = synth.as_read(synth.surface(3000, seed=57, dimension=2))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5, dimension=2, famod_chains=chains)
    ref, rst = O.spectra(spec, s, threads=chains, return_stats=True)
    got, st = run_gpu(spec, s)
    assert st["iterations"] == rst[3], (st["iterations"], rst[3])
    assert st["breakdown"] == rst[0]
    assert parity(got, ref)[0] < TOL


def test_segmented_chain_breakdown_heavy():
    """bulk x10 on every other cell: failed solves reset the chain state (cold retry, AnisoVariables.cpp), the
    state passes through p_L < 0 cells -- every kind of chain transition crosses segment boundaries."""
    s = synth.as_read(synth.surface(2500, seed=31, dimension=3, full3d=True))
    s["bulkPi"] = s["bulkPi"].copy()
    s["bulkPi"][::2] *= 10.0
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5, dimension=3, famod_chains=1)
    ref, rst = O.spectra(spec, s, threads=1, return_stats=True)
    got, st = run_gpu(spec, s)
    assert rst[0] > 0 and st["breakdown"] == rst[0]
    assert st["iterations"] == rst[3], (st["iterations"], rst[3])
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    assert parity(np.nan_to_num(got), np.nan_to_num(ref))[0] < TOL


def test_skipped_cells_inside_chains():
    """u.dsigma <= 0 cells are not part of the chain (MomentumSpectra.cpp:1146): runs of them inside and across
    segments leave the state untouched."""
    s = synth.as_read(synth.surface(2000, seed=61, dimension=2))
    s["dat"] = s["dat"].copy()
    s["dat"][100:400] *= -20.0
    s["dat"][1000::7] *= -20.0
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5, dimension=2, famod_chains=1)
    ref, rst = O.spectra(spec, s, threads=1, return_stats=True)
    got, st = run_gpu(spec, s)
    assert st["iterations"] == rst[3]
    assert parity(got, ref)[0] < TOL


def test_ptma_default_is_the_reference_chain():
    """UrQMD, PTMA + baryon, 3+1D, 600 cells.  The drop-in default (one chain) equals the
    oracle's one chain; every-cell-cold (famod_chains = 0) converges the Newton solves elsewhere and misses the
    north_star bar (1e-6) -- measured 3.6e-6 on the CPU build of the same math -- so it is an opt-in only."""
    s = synth.as_read(synth.surface(600, seed=43, dimension=3, baryon=True, full3d=True))
    kw = dict(hrg_eos=1, chosen=[211, 321, 2212, 3122], df_mode=5, dimension=3, pT="pT24", phi="phi24", y="y21",
              gla_points=64, include_baryon=1, include_baryondiff_deltaf=1)
    spec = make_spec(**kw)
    assert spec["params"]["famod_chains"] == 1
    ref, rst = O.spectra(spec, s, threads=1, return_stats=True)
    got, st = run_gpu(spec, s)
    assert st["iterations"] == rst[3]
    assert parity(got, ref)[0] < TOL
    cold, _ = run_gpu(make_spec(famod_chains=0, **kw), s)
    gap = parity(cold, ref)[0]
    print("PTMA cold-start vs one-chain gap: %.3e" % gap)
    assert gap > 1e-7
