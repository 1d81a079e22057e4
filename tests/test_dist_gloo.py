"""N > 1 decomposition on CPU: world_size-2 and -4 gloo processes shard the cells, integrate their
shard (oracle as the per-rank worker; on the GPU the engine does this) and all-reduce the
spectra -- the result equals the single-process integral over the whole surface."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from is3d2_amd import dist as D, make_spec, synth
    from oracle import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s = synth.as_read(synth.surface(101, seed=5))
    s["dat"] = s["dat"].copy()
    s["dat"][:40] *= -20.0                   # a free (u.dsigma <= 0) prefix: the shards are cost-balanced
    lo, hi = D.shard_bounds(s, rank, world)
    shard = {k: v[lo:hi] for k, v in s.items()}
    avg = D.global_averages(D.average_sums(shard), D.torch_all_reduce(dist))
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=4)        # PTB: needs the global T_avg
    part = torch.from_numpy(O.spectra(spec, shard, T_avg=avg[0]))
    dist.all_reduce(part)
    if rank == 0:
        q.put((avg, part.numpy()))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gloo_shard_and_allreduce(world):
    import torch.multiprocessing as mp
    from is3d2_amd import make_spec, synth
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    port += 7 * world
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    avg, got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = synth.as_read(synth.surface(101, seed=5))
    s["dat"] = s["dat"].copy()
    s["dat"][:40] *= -20.0
    full_avg = O.averages(s)
    assert abs(avg[0] - full_avg[0]) <= 1e-14 * full_avg[0]
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=4)
    ref = O.spectra(spec, s, T_avg=full_avg[0])
    np.testing.assert_allclose(got, ref, rtol=1e-11)


def test_cost_balanced_ranges():
    """contiguous ranges of ~equal estimated cost -- u.dsigma <= 0 cells cost SKIP_COST."""
    from is3d2_amd import dist as D, synth
    s = synth.as_read(synth.surface(1000, seed=3))
    s["dat"] = s["dat"].copy()
    s["dat"][:600] *= -20.0                  # 600 free cells, then 400 live ones
    c = D.cell_costs(s)
    assert (c[:600] == D.SKIP_COST).all() and (c[600:] == 1.0).mean() > 0.9
    for world in (2, 4, 8):
        r = D.balanced_ranges(c, world)
        assert r[0][0] == 0 and r[-1][1] == 1000
        assert all(r[k][1] == r[k + 1][0] for k in range(world - 1))
        cost = [c[lo:hi].sum() for lo, hi in r]
        assert max(cost) - min(cost) <= 1.0 + D.SKIP_COST * 2, cost
        # equal counts would have given rank 0 only free cells
        assert cost[0] > 0.5 * c.sum() / world
    assert D.balanced_ranges(np.ones(3), 8)[-1] == (3, 3)     # more ranks than cells: empty tail ranges


def test_cost_balanced_ranges_with_fallback_costs():
    """Given per-cell costs (is3d_cell_costs: PTB separable-fallback cells 1.8, modified 1, free 0.02) the ranges
    balance those instead of counting cells: a fallback-heavy first half gets fewer cells."""
    from is3d2_amd import dist as D, synth
    s = synth.as_read(synth.surface(1000, seed=5))
    costs = np.r_[np.full(500, 1.8), np.full(500, 1.0)]
    costs[::97] = D.SKIP_COST
    for world in (2, 4):
        r = [D.shard_bounds(s, k, world, costs=costs) for k in range(world)]
        cost = [costs[lo:hi].sum() for lo, hi in r]
        assert max(cost) - min(cost) <= 2 * 1.8 + 1e-9, cost     # each boundary within one cell
    assert D.shard_bounds(s, 0, 2, costs=costs)[1] < 450


def _chain_worker(rank, world, port, npass, chains, q):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch.distributed as dist
    from chain_emu import EmuChainEngine
    from is3d2_amd import dist as D
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    spec, s = _chain_case(chains)
    q0, q1 = D.chain_bounds(s, rank, world, chains)
    eng = EmuChainEngine(spec, s, q0, q1, npass=npass)
    D.launch_chained(eng, None, None, rank, world, dist)
    q.put((rank, q0, q1, eng.iterations(), eng.final_states()))
    dist.destroy_process_group()


def _chain_case(chains):
    """Breakdown-heavy 3+1D surface with a u.dsigma <= 0 run (failed solves reset the chain state, p_L < 0 cells
    pass it through), UrQMD-free pikp PTMA -- the shape of tests/test_gpu_group.py's distributed-chain test."""
    from is3d2_amd import make_spec, synth
    s = synth.as_read(synth.surface(360, seed=109, dimension=3, full3d=True))
    s["bulkPi"] = s["bulkPi"].copy()
    s["bulkPi"][::2] *= 10.0
    s["dat"] = s["dat"].copy()
    s["dat"][100:130] *= -20.0
    spec = make_spec(hrg_eos=2, chosen="pikp", df_mode=5, dimension=3, famod_chains=chains)
    return spec, s


@pytest.mark.parametrize("world,npass,chains", [(2, 24, 1), (4, 24, 1), (4, 1, 1), (3, 2, 3), (4, 24, 5)])
def test_gloo_ptma_chains_split_over_ranks(world, npass, chains):
    """The PTMA warm-start chains split over gloo ranks through dist.launch_chained (the protocol bench.py runs over
    RCCL; a CPU stand-in engine with the oracle's chain step, tests/chain_emu.py): each rank solves only its chain
    positions, yet the per-rank Newton iteration counts add up to the oracle's one-process count for C chains and
    every cell's chain state is the serial chain's bit for bit.  npass = 1 / 2 leave the ripple to the finishers."""
    import torch.multiprocessing as mp
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 31500 + os.getpid() % 1000 + 11 * world + npass + chains
    procs = [ctx.Process(target=_chain_worker, args=(r, world, port, npass, chains, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    spec, s = _chain_case(chains)
    n = len(s["tau"])
    assert res[0][1] == 0 and all(res[k][2] == res[k + 1][1] for k in range(world - 1))
    assert all(r[2] > r[1] for r in res)                        # every rank holds positions
    _, st = O.spectra(spec, s, threads=chains, return_stats=True)
    assert sum(r[3] for r in res) == st[3]
    walker = O.FamodChain(spec, s)
    for c in range(chains):
        states, _, _ = walker.walk(np.arange(c, n, chains), np.zeros(4))
        for cell, ref in zip(range(c, n, chains), states):
            got = next(r[4][cell] for r in res if cell in r[4])
            assert got.tobytes() == ref.tobytes(), cell


def test_chain_bounds_whole_positions():
    from is3d2_amd import dist as D, synth
    s = synth.as_read(synth.surface(1003, seed=3))
    for C in (1, 3, 16):
        P = (1003 + C - 1) // C
        for world in (1, 2, 4, 8):
            b = [D.chain_bounds(s, k, world, C) for k in range(world)]
            assert b[0][0] == 0 and b[-1][1] == P
            assert all(b[k][1] == b[k + 1][0] for k in range(world - 1))
            # cost-balanced cell boundaries (the synthetic surface has a few u.dsigma <= 0 cells) rounded to positions
            sizes = [hi - lo for lo, hi in b]
            assert max(sizes) - min(sizes) <= 0.02 * P + 2, sizes
