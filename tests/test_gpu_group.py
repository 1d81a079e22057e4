"""GPU tier: the multi-device engine (is3d_create_devices, group.hip) -- SURVEY.md 8(b)/(e): the fan-out over
GPUs happens inside the compute call, cells are split into cost-balanced contiguous windows, and the
per-device spectra are summed on the devices (one RCCL ncclAllReduce over distinct GPUs; peer copy +
fixed-order add when the list repeats a GPU).

A one-GPU box can only list GPU 0 repeatedly, which exercises the sharding, the windows, the concurrent
launches and the copy reduction; IS3D_REDUCE=rccl on a one-device list runs the RCCL path itself (a
one-rank communicator: ncclCommInitAll, grouped ncclAllReduce on the launch stream).  Results are compared
with one single-device engine (summation order only: <= 1e-12) and with the oracle."""
import os

import numpy as np
import pytest

from helpers import parity
from is3d2_amd import Engine, build_engine, make_spec, synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def spectra(spec, surf, devices=None, T_avg=None):
    e = build_engine(spec, surf, T_avg=T_avg, devices=devices)
    out = e.calculate_spectra()
    st = e.stats()
    e.close()
    return out, st


@pytest.mark.parametrize("mode,dim", [(1, 3), (2, 2), (3, 3), (4, 2)])
@pytest.mark.parametrize("ndev", [2, 3, 8])
def test_group_equals_single_engine(mode, dim, ndev):
    s = synth.as_read(synth.surface(300, seed=71, dimension=dim, full3d=(dim == 3)))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=mode, dimension=dim)
    one, st1 = spectra(spec, s)
    grp, stg = spectra(spec, s, devices=[0] * ndev)
    assert parity(grp, one)[0] < 1e-12
    assert stg["cells"] == st1["cells"] == 300
    assert stg["breakdown"] == st1["breakdown"]
    ref = O.spectra(spec, s, threads=8)
    assert parity(grp, ref)[0] < 1e-8


def test_group_smash_grid_grad_table_launch():
    s = synth.as_read(synth.surface(64, seed=2, dimension=3))
    spec = make_spec(hrg_eos=2, chosen="smash", df_mode=1, dimension=3, pT="pT48", phi="phi32", y="y21")
    one, _ = spectra(spec, s)
    grp, _ = spectra(spec, s, devices=[0, 0, 0, 0])
    # 444 species: the sum over shards reorders near-cancelling delta-f contributions (measured 6.5e-12)
    assert parity(grp, one)[0] < 1e-10


@pytest.mark.parametrize("dist", ["1", "0"])
def test_group_ptma_chain_walks_whole_surface(monkeypatch, dist):
    """PTMA with the reference's warm-start chain: every shard holds the whole surface; with the chains split
    (default) each shard solves only its window's chain positions from its predecessor's boundary states, with
    IS3D_CHAIN_DIST=0 each walks the whole chain -- either way the same Newton solves (iteration count) as one
    device."""
    monkeypatch.setenv("IS3D_CHAIN_DIST", dist)
    s = synth.as_read(synth.surface(900, seed=73, dimension=2))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5, dimension=2, famod_chains=1)
    one, st1 = spectra(spec, s)
    grp, stg = spectra(spec, s, devices=[0, 0])
    assert stg["iterations"] == st1["iterations"]
    assert stg["breakdown"] == st1["breakdown"]
    assert parity(grp, one)[0] < 1e-12


@pytest.mark.parametrize("chains,ndev,passes", [(1, 3, None), (3, 2, None), (1, 5, None), (16, 3, None),
                                                 (1, 4, "1"), (3, 3, "2"), (32, 3, None), (48, 2, None)])
def test_group_ptma_distributed_chains(monkeypatch, chains, ndev, passes):
    """Chains split over the shards on a breakdown-heavy surface (failed solves reset the state, p_L < 0 cells pass
    it through) with u.dsigma <= 0 runs: the iteration / failure counts equal one device's, which equal the
    oracle's serial chains.  IS3D_CHAIN_PASSES = 1 or 2 leaves most of the ripple to the finishers, which hand the
    final boundary states from shard to shard.  (32, 3) and (48, 2) give every shard 25 positions per chain, one
    segment each: the first shard is exact after pass 0 and its later passes return at once (both
    parity slots of its boundary must still hold its end states)."""
    if passes:
        monkeypatch.setenv("IS3D_CHAIN_PASSES", passes)
    s = synth.as_read(synth.surface(2400, seed=109, dimension=3, full3d=True))
    s["bulkPi"] = s["bulkPi"].copy()
    s["bulkPi"][::2] *= 10.0
    s["dat"] = s["dat"].copy()
    s["dat"][700:900] *= -20.0
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5, dimension=3, famod_chains=chains)
    one, st1 = spectra(spec, s)
    grp, stg = spectra(spec, s, devices=[0] * ndev)
    for k in ("iterations", "breakdown", "pl_negative", "recon_fail", "cells"):
        assert stg[k] == st1[k], (k, stg[k], st1[k])
    assert np.array_equal(np.isnan(grp), np.isnan(one))
    assert parity(np.nan_to_num(grp), np.nan_to_num(one))[0] < 1e-12
    _, rst = O.spectra(spec, s, threads=chains, return_stats=True)
    assert stg["iterations"] == rst[3]


def test_group_rccl_one_rank(monkeypatch):
    monkeypatch.setenv("IS3D_REDUCE", "rccl")
    s = synth.as_read(synth.surface(200, seed=79, dimension=2))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=2, dimension=2)
    one, _ = spectra(spec, s)
    grp, _ = spectra(spec, s, devices=[0])
    assert np.array_equal(grp, one)       # a one-rank all-reduce is the identity


def test_group_balances_skipped_cells():
    """The first two thirds of the surface are u.dsigma <= 0 (free): cost-balanced windows put them all on the
    first shard, so the result still matches and every shard carries live cells."""
    s = synth.as_read(synth.surface(600, seed=83, dimension=2))
    s["dat"] = s["dat"].copy()
    s["dat"][:400] *= -20.0
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1, dimension=2)
    one, _ = spectra(spec, s)
    grp, _ = spectra(spec, s, devices=[0, 0, 0])
    assert parity(grp, one)[0] < 1e-12


def test_group_launch_on_caller_stream():
    torch = pytest.importorskip("torch")
    s = synth.as_read(synth.surface(300, seed=89, dimension=3, full3d=True))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=2, dimension=3)
    one, _ = spectra(spec, s)
    e = build_engine(spec, s, devices=[0, 0])
    out = torch.zeros(e.output_size(), dtype=torch.float64, device="cuda:0")
    stream = torch.cuda.current_stream(0).cuda_stream
    for _ in range(2):
        e.launch(out.data_ptr(), stream)
        e.finish()
    got = out.cpu().numpy()
    e.close()
    assert parity(got, one)[0] < 1e-12


def test_group_dndx_and_yield():
    s = synth.as_read(synth.surface(400, seed=97, dimension=2))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=1, dimension=2)
    outs = []
    for dv in (None, [0, 0, 0]):
        e = build_engine(spec, s, devices=dv)
        t, r, ph = e.calculate_dN_dX()
        cy = e.cell_yields()
        from is3d2_amd.engine import surface_averages
        nt, dens = e.total_yield(surface_averages(s))
        e.close()
        outs.append((t, r, ph, cy, nt, dens))
    for a, b in zip(outs[0][:4], outs[1][:4]):
        assert parity(b, a, floor=1e-300)[0] < 1e-12
    assert abs(outs[1][4] - outs[0][4]) <= 1e-12 * abs(outs[0][4])
    assert np.array_equal(outs[1][5], outs[0][5])


def test_group_surface_from_device():
    torch = pytest.importorskip("torch")
    s = synth.as_read(synth.surface(300, seed=101, dimension=2))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=2, dimension=2)
    one, _ = spectra(spec, s)
    from is3d2_amd import _lib
    dev = torch.from_numpy(np.stack([np.asarray(s[k], dtype=np.float64) if s.get(k) is not None
                                     else np.zeros(300) for k in _lib.SURFACE_FIELDS])).to("cuda:0").contiguous()
    e = build_engine(spec, s, devices=[0, 0])
    e.set_surface_device(dev.data_ptr(), 300)
    got = e.calculate_spectra()
    e.close()
    assert parity(got, one)[0] < 1e-12


def test_group_bad_device_list():
    with pytest.raises(Exception):
        Engine(devices=[0, 97])


def test_group_stale_split_after_params_change():
    """Surface split for PTMA warm-start chains (every shard holds the whole surface), then params without
    chains: the launch refuses until the surface is set again (it would double-count cells otherwise), and
    then matches one engine."""
    s = synth.as_read(synth.surface(300, seed=103, dimension=2))
    spec5 = make_spec(hrg_eos=2, chosen="pikp", df_mode=5, dimension=2, famod_chains=1)
    spec1 = make_spec(hrg_eos=2, chosen="pikp", df_mode=1, dimension=2)
    one, _ = spectra(spec1, s)
    e = build_engine(spec5, s, devices=[0, 0])
    e.set_params(**spec1["params"])
    with pytest.raises(Exception, match="set the surface again"):
        e.calculate_spectra()
    e.set_surface(s)
    got = e.calculate_spectra()
    e.close()
    assert parity(got, one)[0] < 1e-12


def test_group_window_error_message():
    e = Engine(devices=[0, 0])
    with pytest.raises(Exception, match="places its own windows"):
        e.set_cell_window(0, 1)
    e.close()


@pytest.mark.skipif(not __import__("torch").cuda.is_available() or __import__("torch").cuda.device_count() < 2,
                    reason="needs two GPUs: the distinct-device RCCL all-reduce and peer-copy reduction")
@pytest.mark.parametrize("reduce", ["rccl", "copy"])
def test_group_distinct_devices(monkeypatch, reduce):
    """devices = [0, 1]: ncclCommInitAll over distinct GPUs + grouped in-place ncclAllReduce (IS3D_REDUCE unset
    or rccl), or hipMemcpyPeerAsync + fixed-order add (copy).  Skipped on a one-GPU box."""
    monkeypatch.setenv("IS3D_REDUCE", reduce)
    s = synth.as_read(synth.surface(400, seed=107, dimension=3, full3d=True))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=2, dimension=3)
    one, _ = spectra(spec, s)
    grp, _ = spectra(spec, s, devices=[0, 1])
    assert parity(grp, one)[0] < 1e-12


def test_group_balances_breakdown_cluster():
    """PTB with the separable-fallback cells (breakdown, 1.8x a modified cell) clustered in the first half of the
    surface: is3d_cell_costs sees them, the cost-balanced split moves below n / 2, and the device group (which
    balances with the same costs) still equals one engine."""
    from is3d2_amd import dist as D
    n = 1200
    s = synth.as_read(synth.surface(n, seed=113, dimension=2))
    s["bulkPi"] = s["bulkPi"].copy()
    s["bulkPi"][: n // 2] *= 30.0
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=4, dimension=2)
    costs = D.device_cell_costs(spec, s)
    assert costs.shape == (n,)
    fb = costs > 1.0
    assert fb[: n // 2].sum() > 0.3 * (n // 2) and fb[n // 2:].sum() < 0.05 * (n // 2)
    assert set(np.unique(costs)) <= {0.02, 1.0, 1.8}
    lo, hi = D.shard_bounds(s, 0, 2, costs=costs)
    assert lo == 0 and hi < n // 2
    one, st1 = spectra(spec, s)
    grp, stg = spectra(spec, s, devices=[0, 0])
    assert stg["breakdown"] == st1["breakdown"] > 0
    assert parity(grp, one)[0] < 1e-12
