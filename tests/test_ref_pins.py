"""CPU tier: pin the oracle and the host-side data handling against the reference's own
GSL-free sources (readindata / GaussThermal / LocalRestFrame / Table / ParameterReader),
compiled in place into oracle/_ref/ref_harness by oracle/ref/build_ref.sh.

Skipped where the harness or /root/reference is absent (the GPU box)."""
import os
import subprocess

import numpy as np
import pytest

from is3d2_amd import data, hrg, synth
from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HARNESS = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
REF = "/root/reference"
pytestmark = pytest.mark.skipif(not (os.path.exists(HARNESS) and os.path.isdir(REF)),
                                reason="oracle/_ref not built or /root/reference absent")

PARAMS = """operation = 1
mode = {mode}
hrg_eos = {hrg}
dimension = {dim}
df_mode = 1
include_baryon = {baryon}
include_bulk_deltaf = 1
include_shear_deltaf = 1
include_baryondiff_deltaf = {baryon}
"""


def run(args, cwd, stdin=None):
    r = subprocess.run([HARNESS] + args, cwd=cwd, input=stdin, capture_output=True, text=True, check=True)
    out = r.stdout
    return out.split("@@BEGIN\n", 1)[1] if "@@BEGIN\n" in out else out


def rundir(tmp_path, mode=1, hrg_eos=2, dim=2, baryon=0):
    (tmp_path / "input").mkdir(exist_ok=True)
    (tmp_path / "tables" / "thermodynamic").mkdir(parents=True, exist_ok=True)
    if not (tmp_path / "PDG").exists():
        os.symlink(os.path.join(REF, "PDG"), tmp_path / "PDG")
    (tmp_path / "iS3D_parameters.dat").write_text(PARAMS.format(mode=mode, hrg=hrg_eos, dim=dim, baryon=baryon))
    return tmp_path


@pytest.mark.parametrize("hrg_eos", [1, 2, 3])
def test_pdg_lists_match_reference_reader(tmp_path, hrg_eos):
    out = run(["pdg"], rundir(tmp_path, hrg_eos=hrg_eos)).split("\n")
    n = int(out[0])
    rows = np.array([[float(v) for v in ln.split()] for ln in out[1:1 + n]])
    mine = hrg.pdg_particles(hrg_eos)
    assert len(mine["mcid"]) == n
    np.testing.assert_array_equal(mine["mcid"], rows[:, 0])
    np.testing.assert_array_equal(mine["mass"], rows[:, 1])
    np.testing.assert_array_equal(mine["gspin"], rows[:, 2])
    np.testing.assert_array_equal(mine["baryon"], rows[:, 3])
    np.testing.assert_array_equal(mine["sign"], rows[:, 4])


@pytest.mark.parametrize("dim,baryon", [(2, 0), (3, 0), (3, 1)])
def test_mode1_surface_reader_and_averages(tmp_path, dim, baryon):
    d = rundir(tmp_path, mode=1, dim=dim, baryon=baryon)
    s = synth.surface(300, seed=13, dimension=dim, baryon=bool(baryon), full3d=(dim == 3))
    synth.write_mode1(str(d / "input" / "surface.dat"), s, include_baryon=bool(baryon))
    out = run(["surface"], d).strip().split("\n")
    n = int(out[0])
    cells = np.array([[float(v) for v in ln.split()] for ln in out[1:1 + n]])
    avg = np.array([float(v) for v in out[1 + n].split()])
    r = synth.as_read(s)
    for i, k in enumerate(synth.FIELDS):
        if not baryon and k in ("muB", "nB", "Vx", "Vy", "Vn"):
            continue
        np.testing.assert_array_equal(cells[:, i], r[k], err_msg=k)
    rb = r if baryon else {k: v for k, v in r.items() if k not in ("muB", "nB")}
    mine = O.averages(rb, include_baryon=baryon)
    np.testing.assert_allclose(mine, avg, rtol=1e-14, atol=0)


def test_gauss_thermal_matches_reference():
    roots, weights = data.gauss_laguerre(32)
    rng = np.random.default_rng(0)
    lines, want = [], []
    for _ in range(200):
        kind = int(rng.integers(0, 6)); alpha = int(rng.integers(1, 4))
        mbar = float(rng.uniform(0.1, 20)); aB = float(rng.uniform(-1, 1)); b = float(rng.choice([-1, 0, 1]))
        sign = float(rng.choice([-1, 1]))
        lines.append("%d %d %.17g %.17g %.17g %.17g" % (kind, alpha, mbar, aB, b, sign))
        lib = O.load()
        want.append(lib.orc_gauss_thermal(kind, O._p(roots[alpha]), O._p(weights[alpha]), roots.shape[1],
                                          mbar, aB, b, sign))
    got = np.array([float(v) for v in run(["gauss", os.path.join(REF, "tables/gauss/gla_roots_weights.txt")],
                                          ROOT, "\n".join(lines) + "\n").split()])
    np.testing.assert_array_equal(np.array(want), got)


def test_gauss1d_mod_matches_reference():
    roots, weights = data.gauss_laguerre(32)
    rng = np.random.default_rng(1)
    lines, want = [], []
    lib = O.load()
    for _ in range(100):
        kind = int(rng.integers(0, 2)); mbar = float(rng.uniform(0.1, 20)); lam = float(rng.uniform(-0.9, 2))
        sign = float(rng.choice([-1, 1]))
        lines.append("%d 2 %.17g %.17g %.17g" % (kind, mbar, lam, sign))
        want.append(lib.orc_gauss1d_mod(kind, O._p(roots[2]), O._p(weights[2]), roots.shape[1], mbar, lam, sign))
    got = np.array([float(v) for v in run(["gaussmod", os.path.join(REF, "tables/gauss/gla_roots_weights.txt")],
                                          ROOT, "\n".join(lines) + "\n").split()])
    np.testing.assert_array_equal(np.array(want), got)


def test_lrf_boost_matches_reference():
    rng = np.random.default_rng(2)
    lib = O.load()
    rows, want = [], []
    for _ in range(100):
        tau = rng.uniform(0.5, 10); ux, uy = rng.normal(0, 0.8, 2); un = rng.normal(0, 0.1) / tau
        ut = np.sqrt(1 + ux * ux + uy * uy + tau * tau * un * un)
        pis = rng.normal(0, 0.01, 10); V = rng.normal(0, 0.01, 4)
        vals = [ut, ux, uy, un, tau] + list(pis) + list(V)
        rows.append(" ".join("%.17g" % v for v in vals))
        out = np.zeros(14)
        lib.orc_milne_lrf(O._p(np.array(vals[:15])), O._p(out))
        want.append(out)
    got = np.array([[float(v) for v in ln.split()] for ln in run(["lrf"], ROOT, "\n".join(rows) + "\n").strip().split("\n")])
    np.testing.assert_array_equal(np.array(want), got[:, :14])


@pytest.mark.parametrize("name,rel", [("pT48", "tables/all_tables/pT/pT_gauss_table_48pt.dat"),
                                      ("phi32", "tables/all_tables/phi/phi_gauss_table_32pt.dat"),
                                      ("y21", "tables/momentum/y_table.dat"),
                                      ("eta24", "tables/spacetime_rapidity/eta_table.dat")])
def test_packed_grids_match_reference_table_reader(name, rel):
    out = run(["table", os.path.join(REF, rel)], ROOT).strip().split("\n")
    ncol, nrow = map(int, out[0].split())
    tab = np.array([[float(v) for v in ln.split()] for ln in out[1:1 + nrow]])
    v, w = data.grid(name)
    np.testing.assert_array_equal(tab[:, 0], v)
    np.testing.assert_array_equal(tab[:, 1], w)
