"""C++ host layer (libis3d_host.so): reference file formats on both sides of the hot path.

CPU tier: readers pinned bit-for-bit against the reference's own readindata.cpp /
ParameterReader.cpp (oracle/_ref harness, where built); GPU tier: the whole drop-in
workflow (run directory in, results/continuous/*.dat out) against the oracle."""
import os
import subprocess

import numpy as np
import pytest

from helpers import parity
from is3d2_amd import host, make_spec, rundir, synth
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
REF = "/root/reference"
need_ref = pytest.mark.skipif(not (os.path.exists(HARNESS) and os.path.isdir(REF)), reason="oracle/_ref absent")


def harness(args, cwd):
    out = subprocess.run([HARNESS] + args, cwd=cwd, capture_output=True, text=True, check=True).stdout
    return out.split("@@BEGIN\n", 1)[1] if "@@BEGIN\n" in out else out


@need_ref
@pytest.mark.parametrize("fmt,dim,baryon", [(1, 2, 0), (1, 3, 1), (5, 2, 0), (5, 3, 1), (6, 3, 0), (6, 3, 1), (7, 2, 0)])
def test_surface_readers_match_reference(tmp_path, fmt, dim, baryon):
    s = synth.surface(200, seed=21, dimension=dim, baryon=bool(baryon), full3d=(dim == 3 and fmt != 7))
    d = rundir.write_run_dir(str(tmp_path), s, dict(dimension=dim, df_mode=1, include_baryon=baryon,
                                                    include_bulk_deltaf=1, include_shear_deltaf=1,
                                                    include_baryondiff_deltaf=baryon), surface_format=fmt)
    out = harness(["surface"], d).strip().split("\n")
    n = int(out[0])
    ref = np.array([[float(v) for v in ln.split()] for ln in out[1:1 + n]])
    ref_avg = np.array([float(v) for v in out[1 + n].split()])
    fields, avg = host.read_surface(d, fmt, dim, baryon)
    for k, name in enumerate(synth.FIELDS):
        if not baryon and name in ("nB", "Vx", "Vy", "Vn") or (fmt in (1, 5) and not baryon and name == "muB"):
            continue
        np.testing.assert_array_equal(fields[k], ref[:, k], err_msg=name)
    np.testing.assert_array_equal(avg, ref_avg)


@need_ref
@pytest.mark.parametrize("hrg_eos", [1, 2, 3])
def test_pdg_reader_matches_reference_on_reference_files(tmp_path, hrg_eos):
    os.symlink(os.path.join(REF, "PDG"), tmp_path / "PDG")
    (tmp_path / "iS3D_parameters.dat").write_text("hrg_eos = %d\n" % hrg_eos)
    out = harness(["pdg"], str(tmp_path)).split("\n")
    n = int(out[0])
    ref = np.array([[float(v) for v in ln.split()] for ln in out[1:1 + n]])
    mine = host.read_pdg(str(tmp_path), hrg_eos)
    assert len(mine["mcid"]) == n
    for k, name in enumerate(["mcid", "mass", "gspin", "baryon", "sign"]):
        np.testing.assert_array_equal(mine[name], ref[:, k], err_msg=name)


@need_ref
def test_parameter_reader_matches_reference():
    path = os.path.join(REF, "iS3D_parameters.dat")
    keys = ["operation", "mode", "hrg_eos", "dimension", "df_mode", "include_baryon", "deta_min", "mass_pion0",
            "threads_per_block", "min_num_hadrons", "y_cut", "pT_bins", "lightest_particle"]
    out = harness(["params", path] + keys, ROOT).split()
    for k, v in zip(keys, out):
        assert host.param(path, k) == float(v), k


def test_table_reader_drops_unterminated_last_line(tmp_path):
    # Arsenal.cpp readBlockData: rows are '\n'-terminated lines
    (tmp_path / "iS3D_parameters.dat").write_text("a = 1\nb=2 # c\n  C  =  3.5e-2\n")
    assert host.param(str(tmp_path / "iS3D_parameters.dat"), "c") == 0.035
    assert host.param(str(tmp_path / "iS3D_parameters.dat"), "B") == 2.0


def _spec_for(params, hrg, chosen, pT, phi):
    return make_spec(hrg_eos=hrg, chosen=chosen, pT=pT, phi=phi, **params)


@pytest.mark.gpu
@pytest.mark.parametrize("fmt,dim,mode", [(1, 2, 1), (1, 3, 2), (6, 3, 2), (7, 2, 3), (1, 2, 4)])
def test_dropin_workflow_matches_oracle(tmp_path, fmt, dim, mode):
    s = synth.surface(150, seed=31, dimension=dim, full3d=(dim == 3 and fmt != 7))
    params = dict(dimension=dim, df_mode=mode, include_baryon=0, include_bulk_deltaf=1, include_shear_deltaf=1,
                  include_baryondiff_deltaf=0, regulate_deltaf=0, outflow=0, deta_min=1e-5, mass_pion0=0.138)
    d = rundir.write_run_dir(str(tmp_path), s, params, hrg_eos=2, chosen="pikp", surface_format=fmt)
    spec = _spec_for(params, 2, "pikp", "pT24", "phi24")
    fields, avg = host.read_surface(d, fmt, dim, 0)
    surf = {k: fields[i] for i, k in enumerate(synth.FIELDS)}
    ref = O.spectra(spec, surf, T_avg=avg[0])
    got = host.run_particlization(d, len(ref))
    assert parity(got, ref)[0] < 1e-8
    # the five reference output files per species, reference layout
    npT, nphi, ny = 24, 24, (21 if dim == 3 else 1)
    for mc in spec["species"]["mcid"]:
        lines = open(os.path.join(d, "results/continuous/dN_pTdpTdphidy_%d.dat" % mc)).read().split("\n")
        assert lines[0] == "y\tphip\tpT\tdN_pTdpTdphidy"
        assert len([ln for ln in lines[1:] if ln]) == npT * nphi * ny
        for name in ("vn", "dN_2pipTdpTdy", "dN_dphidy", "dN_dy"):
            assert os.path.exists(os.path.join(d, "results/continuous/%s_%d.dat" % (name, mc)))
    vals = np.array([float(ln.split("\t")[3]) for ln in lines[1:] if ln])
    last = ref.reshape(3, npT, nphi, ny)[2]          # file order: y, phi, pT
    np.testing.assert_allclose(vals, np.transpose(last, (2, 1, 0)).ravel(), rtol=5e-9)


@pytest.mark.gpu
@pytest.mark.parametrize("dim,mode,threads", [(2, 1, 0), (3, 3, 0), (2, 4, 4)])
def test_dropin_spacetime_workflow_matches_oracle(tmp_path, dim, mode, threads):
    # operation = 0: results/continuous/dN_taudtaudy_, dN_2pirdrdy_, dN_dphidy_<MCID>.dat (appended)
    s = synth.surface(150, seed=41, dimension=dim, full3d=(dim == 3))
    params = dict(operation=0, dimension=dim, df_mode=mode, include_baryon=0, include_bulk_deltaf=1,
                  include_shear_deltaf=1, include_baryondiff_deltaf=0, regulate_deltaf=0, outflow=0, deta_min=1e-5,
                  mass_pion0=0.138, tau_min=0.0, tau_max=12.0, tau_bins=60, r_min=0.0, r_max=15.0, r_bins=30,
                  phip_bins=50, spacetime_threads=threads)
    d = rundir.write_run_dir(str(tmp_path), s, params, hrg_eos=2, chosen="pikp", surface_format=1)
    spec = make_spec(hrg_eos=2, chosen="pikp", pT="pT24", phi="phi24",
                     **{k: v for k, v in params.items() if k != "operation"})
    fields, avg = host.read_surface(d, 1, dim, 0)
    surf = {k: fields[i] for i, k in enumerate(synth.FIELDS)}
    t, r, ph = O.dndx(spec, surf, T_avg=avg[0], threads=max(threads, 1), carry=int(threads > 0))
    ref = np.concatenate([t, r, ph], axis=1).ravel()
    got = host.run_particlization(d, len(ref))
    assert parity(got, ref)[0] < 1e-9
    for k, mc in enumerate(spec["species"]["mcid"]):
        rows = np.loadtxt(os.path.join(d, "results/continuous/dN_2pirdrdy_%d.dat" % mc))
        assert rows.shape == (30, 2)
        np.testing.assert_allclose(rows[:, 0], 0.25 + 0.5 * np.arange(30), rtol=1e-6)
        np.testing.assert_allclose(rows[:, 1], r[k], rtol=1e-6, atol=1e-300)
    host.run_particlization(d, len(ref))            # the reference opens the files in append mode
    assert np.loadtxt(os.path.join(d, "results/continuous/dN_taudtaudy_%d.dat" % mc)).shape == (120, 2)


@pytest.mark.gpu
@pytest.mark.parametrize("dim,mode,oversample", [(2, 2, 1), (3, 1, 1), (2, 4, 1), (2, 2, 0)])
def test_dropin_oversampling_estimate_matches_oracle(tmp_path, dim, mode, oversample):
    # operation = 2: Ntotal (ParticleSampler.cpp:447-636) and Nevents (EmissionFunction.cpp:1237-1249)
    s = synth.surface(400, seed=43, dimension=dim, full3d=(dim == 3))
    params = dict(operation=2, dimension=dim, df_mode=mode, include_baryon=0, include_bulk_deltaf=1,
                  include_shear_deltaf=1, include_baryondiff_deltaf=0, regulate_deltaf=0, outflow=0, deta_min=1e-5,
                  mass_pion0=0.138, oversample=oversample, min_num_hadrons=1.0e7, max_num_samples=1.0e4, y_cut=0.75)
    d = rundir.write_run_dir(str(tmp_path), s, params, hrg_eos=2, chosen="smash", surface_format=1)
    spec = make_spec(hrg_eos=2, chosen="smash", **{k: v for k, v in params.items() if k != "operation"})
    fields, avg = host.read_surface(d, 1, dim, 0)
    surf = {k: fields[i] for i, k in enumerate(synth.FIELDS)}
    ntot, nev = host.total_yield(d)
    if not oversample:
        assert (ntot, nev) == (0.0, 1)
        return
    ref, _ = O.total_yield(spec, surf, avg, y_cut=0.75)
    assert abs(ntot - ref) <= 1e-12 * abs(ref)
    assert nev == int(min(np.ceil(1.0e7 / ref), 1.0e4))


GOLDEN = os.path.join(ROOT, "tests", "golden")


def _shipped_surface_run_dir(tmp_path):
    """A run directory around the reference's only shipped input, input/surface.dat (one 26-column
    cell in the retired GPU-VH layout, kept as data in tests/golden/reference_input_surface.dat), read
    as BASELINE config 1 reads it: mode 1, 2+1D, pikp, Grad."""
    s = synth.surface(4, seed=1, dimension=2)
    params = dict(dimension=2, df_mode=1, include_baryon=0, include_bulk_deltaf=1, include_shear_deltaf=1,
                  include_baryondiff_deltaf=0, regulate_deltaf=0, outflow=0, deta_min=1e-5, mass_pion0=0.138)
    d = rundir.write_run_dir(str(tmp_path), s, params, hrg_eos=2, chosen="pikp", surface_format=1)
    with open(os.path.join(GOLDEN, "reference_input_surface.dat")) as f, \
            open(os.path.join(d, "input", "surface.dat"), "w") as g:
        g.write(f.read())
    return d


@need_ref
def test_shipped_surface_reader_matches_reference(tmp_path):
    # the mis-parse pinned bit for bit: column 13 (1.40186 fm^-1) is read as T, so T = 0.2766 GeV
    d = _shipped_surface_run_dir(tmp_path)
    out = harness(["surface"], d).strip().split("\n")
    assert int(out[0]) == 1
    ref = np.array([float(v) for v in out[1].split()])
    ref_avg = np.array([float(v) for v in out[2].split()])
    fields, avg = host.read_surface(d, 1, 2, 0)
    for k, name in enumerate(synth.FIELDS):
        if name in ("muB", "nB", "Vx", "Vy", "Vn"):
            continue
        assert fields[k][0] == ref[k], name
    np.testing.assert_array_equal(avg, ref_avg)
    assert abs(fields[synth.FIELDS.index("T")][0] - 1.40186 * 0.197327053) < 1e-15


def test_shipped_surface_is_outside_the_df_tables_in_the_oracle(tmp_path):
    # the reference aborts in gsl_spline_eval ("interpolation error"): T = 0.2766 GeV > 0.2 GeV table edge
    d = _shipped_surface_run_dir(tmp_path)
    fields, avg = host.read_surface(d, 1, 2, 0)
    surf = {k: fields[i] for i, k in enumerate(synth.FIELDS)}
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1, dimension=2)
    with pytest.raises(RuntimeError, match="interpolation"):
        O.spectra(spec, surf, T_avg=avg[0])


@pytest.mark.gpu
def test_shipped_surface_dropin_returns_df_range_error(tmp_path):
    # the drop-in workflow on the reference's own input: IS3D_ERR_DF_RANGE with the GSL message
    # instead of the reference's abort
    from is3d2_amd import _lib
    d = _shipped_surface_run_dir(tmp_path)
    with pytest.raises(host.HostError, match="interpolation") as ei:
        host.run_particlization(d, 3 * 24 * 24)
    assert ei.value.code == _lib.IS3D_ERR_DF_RANGE
