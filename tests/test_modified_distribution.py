"""The reference's own test configurations: tests/modified_distribution/ of iS3D2,
packed as data by tests/golden/make_modified_distribution.py -- 64 iS3D_parameters.dat variants over
{central, noncentral} x {small, large}_bulk x {grad, ce, ptm, ptb} x {none, shear, bulk, shear_bulk},
with the reference's test tables (51-point pT grid starting at pT = 0, a 1-point (central) or
24-point (noncentral) phi grid, 24 eta nodes, 21 y) and its chosen list {111, 321, 2212}.

The reference ships neither the surfaces nor any outputs for these runs, so the surfaces here are
synthetic (SURVEY.md 8d generator; 'large_bulk' multiplies the bulk pressure by 8, which drives PTM /
PTB into breakdown and the PTB bulk clamp) and the expected values come from the oracle:
  CPU tier: the fixture, and the kernels' math (host emulator) against the oracle for all 64;
  GPU tier: the drop-in workflow -- run directory -> libis3d_host.so (C++ IS3D over the HIP engine)
            -> results/continuous files -- against the oracle for all 64.
"""
import json
import os

import numpy as np
import pytest

from helpers import emu_spectra, parity
from is3d2_amd import make_spec, synth
from oracle import oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "modified_distribution.json")))
CASES = sorted(FIX["cases"])
FLAGS = ("include_baryon", "include_bulk_deltaf", "include_shear_deltaf", "include_baryondiff_deltaf",
         "regulate_deltaf", "outflow", "deta_min", "mass_pion0")
TOL = 1e-8


def check(got, ref, tol):
    """parity on the finite entries; NaN exactly where the reference has NaN.  (PTB with |Pi| > P in
    2+1D: the clamp leaves lambda ~ -1, eta_scale = detA / (1 + lambda)^2 ~ 1e4 and cosh / sinh of
    y - eta_scale eta overflow, so p.dsigma = inf dsigma_tau - inf 0 = NaN, MomentumSpectra.cpp:932-936:
    the reference's own output for those runs is NaN, and so is the oracle's and the engine's.)"""
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan)
    rel, zr, zg = parity(got[~nan], ref[~nan])
    assert rel < tol, (rel, zr, zg)
    assert zr == zg


def case_spec(name):
    p = FIX["cases"][name]
    t = FIX["tables"][name.split("/")[0]]
    flags = {k: (p[k] if k in ("deta_min", "mass_pion0") else int(p[k])) for k in FLAGS if k in p}
    spec = make_spec(hrg_eos=int(p["hrg_eos"]), chosen=FIX["chosen"], pT=t["pT"], phi=t["phi"], y=t["y"],
                     eta=t["eta"], dimension=int(p["dimension"]), df_mode=int(p["df_mode"]), **flags)
    return p, t, spec


def raw_surface(name, n, seed):
    s = synth.surface(n, seed=seed)
    if "/large_bulk/" in name:
        s = dict(s)
        s["bulkPi"] = 8.0 * s["bulkPi"]
    return s


def test_fixture_matches_the_reference_test_matrix():
    assert len(CASES) == 64 and FIX["chosen"] == [111, 321, 2212]
    modes = {"grad": 1, "ce": 2, "ptm": 3, "ptb": 4}
    for name in CASES:
        geom, bulk, df, visc = name.split("/")
        p = FIX["cases"][name]
        assert (p["operation"], p["mode"], p["dimension"], p["hrg_eos"]) == (1, 1, 2, 2)
        assert p["df_mode"] == modes[df]
        assert p["include_shear_deltaf"] == ("shear" in visc) and p["include_bulk_deltaf"] == ("bulk" in visc)
    assert [len(FIX["tables"][g]["phi"]) for g in ("central", "noncentral")] == [1, 24]
    assert len(FIX["tables"]["central"]["pT"]) == 51 and FIX["tables"]["central"]["pT"][0][0] == 0.0


@pytest.mark.parametrize("name", CASES)
def test_kernel_math_on_reference_test_configuration(name):
    _, _, spec = case_spec(name)
    s = synth.as_read(raw_surface(name, 40, 23))
    ref = O.spectra(spec, s, threads=1)
    got, _ = emu_spectra(spec, s)
    check(got, ref, 1e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("name", CASES)
def test_dropin_on_reference_test_configuration(tmp_path, name):
    from is3d2_amd import host, rundir
    p, t, spec = case_spec(name)
    raw = raw_surface(name, 150, 17)
    d = rundir.write_run_dir(str(tmp_path), raw, dict(p), hrg_eos=int(p["hrg_eos"]), chosen=FIX["chosen"],
                             pT=t["pT"], phi=t["phi"], y=t["y"], eta=t["eta"], surface_format=int(p["mode"]))
    fields, avg = host.read_surface(d, int(p["mode"]), int(p["dimension"]), int(p["include_baryon"]))
    surf = {k: fields[i] for i, k in enumerate(synth.FIELDS)}
    ref = O.spectra(spec, surf, T_avg=avg[0], threads=1)
    got = host.run_particlization(d, len(ref))
    check(got, ref, TOL)
    npT, nphi = len(t["pT"]), len(t["phi"])
    for mc in FIX["chosen"]:
        rows = [ln for ln in open(os.path.join(d, "results/continuous/dN_pTdpTdphidy_%d.dat" % mc)).read().split("\n")[1:]
                if ln]
        assert len(rows) == npT * nphi
