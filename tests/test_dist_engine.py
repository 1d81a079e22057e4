"""Engine in the loop under torch.distributed: world_size-2 gloo processes, both on GPU 0 (the GPU box
has one), each drive libis3d_amd.so on their contiguous cell shard -- the Plasma sums behind the PTB
table and the spectra are all-reduced exactly as bench.py does with RCCL on a node -- and the result
must equal one engine on the whole surface.  Also the C++ facade's multi-device path
(EmissionFunctionArray::run_sharded: one engine per shard, host sum) with both shards on device 0."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


def _surface():
    from is3d2_amd import synth
    return synth.as_read(synth.surface(301, seed=45, dimension=2))


def _spec(mode):
    from is3d2_amd import make_spec
    return make_spec(hrg_eos=2, chosen="smash", df_mode=mode, dimension=2, pT="pT24", phi="phi32")


def _worker(rank, world, port, mode, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from is3d2_amd import build_engine, dist as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = _surface()
        lo, hi = D.shard_range(len(s["tau"]), rank, world)
        shard = {k: np.ascontiguousarray(v[lo:hi]) for k, v in s.items()}
        avg = D.global_averages(D.average_sums(shard), D.torch_all_reduce(dist))
        e = build_engine(_spec(mode), shard, T_avg=avg[0], device=0)
        part = torch.from_numpy(e.calculate_spectra())
        e.close()
        dist.all_reduce(part)
        if rank == 0:
            q.put((avg, part.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", [4, 2])
def test_two_rank_engine_shards_equal_whole_surface(mode):
    import torch.multiprocessing as mp
    from is3d2_amd import build_engine, surface_averages
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + (os.getpid() + mode) % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    avg, got = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = _surface()
    full_avg = surface_averages(s)
    assert abs(avg[0] - full_avg[0]) <= 1e-14 * full_avg[0]
    e = build_engine(_spec(mode), s, T_avg=full_avg[0], device=0)
    ref = e.calculate_spectra()
    e.close()
    m = np.abs(ref) > 1e-290
    # only the summation order over cells differs (two shard sums + their sum vs one pass): 1e-16 per
    # entry except entries that sum mixed-sign contributions (measured 2.7e-12 for RTA-CE; the reference
    # itself moves by 2.2e-11 between OpenMP thread counts)
    assert np.max(np.abs(got[m] - ref[m]) / np.abs(ref[m])) < 1e-10
    assert np.array_equal(got[~m] == 0.0, ref[~m] == 0.0)


@pytest.mark.parametrize("mode", [1, 4])
def test_facade_multi_device_path_on_one_gpu(tmp_path, mode):
    from helpers import parity
    from is3d2_amd import host, rundir, synth
    s = synth.surface(203, seed=47, dimension=2)
    params = dict(dimension=2, df_mode=mode, include_baryon=0, include_bulk_deltaf=1, include_shear_deltaf=1,
                  include_baryondiff_deltaf=0, regulate_deltaf=0, outflow=0, deta_min=1e-5, mass_pion0=0.138)
    d = rundir.write_run_dir(str(tmp_path), s, params, hrg_eos=2, chosen="pikp", surface_format=1)
    n_out = 3 * 24 * 24
    one = host.run_particlization(d, n_out, device=0, num_devices=1)
    two = host.run_particlization_devices(d, n_out, [0, 0])
    three = host.run_particlization_devices(d, n_out, [0, 0, 0])
    assert parity(two, one)[0] < 1e-12
    assert parity(three, one)[0] < 1e-12


def _chain_surface():
    from is3d2_amd import synth
    s = synth.as_read(synth.surface(1200, seed=109, dimension=3, full3d=True))
    s["bulkPi"] = s["bulkPi"].copy()
    s["bulkPi"][::2] *= 10.0
    s["dat"] = s["dat"].copy()
    s["dat"][300:380] *= -20.0
    return s


def _chain_spec(chains):
    from is3d2_amd import make_spec
    return make_spec(hrg_eos=2, chosen="pikp", df_mode=5, dimension=3, famod_chains=chains)


def _chain_worker(rank, world, port, chains, npass, q):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    if npass:
        os.environ["IS3D_CHAIN_PASSES"] = str(npass)
    import torch
    import torch.distributed as dist
    from is3d2_amd import build_engine, dist as D
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        s = _chain_surface()
        q0, q1 = D.chain_bounds(s, rank, world, chains)
        e = build_engine(_chain_spec(chains), s, device=0)
        e.set_chain_range(q0, q1)
        out = torch.zeros(e.output_size(), dtype=torch.float64, device="cuda:0")
        stream = torch.cuda.current_stream(0)
        for _ in range(2):        # a second pass: the engine's chain buffers are reused
            D.launch_chained(e, out.data_ptr(), stream.cuda_stream, rank, world, dist, sync=stream.synchronize)
            e.finish()
        st = e.stats()
        e.close()
        part = out.cpu()
        dist.all_reduce(part)
        q.put((rank, st["iterations"], st["cells"], part.numpy() if rank == 0 else None))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,chains,npass", [(2, 1, 0), (3, 3, 0), (2, 16, 1), (4, 1, 2)])
def test_ptma_chains_split_over_processes(world, chains, npass):
    """PTMA warm-start chains split over processes: every rank holds the whole surface, solves
    its chain positions (Engine.set_chain_range) through the staged launch and hands its boundary states to the
    next rank after every pass (dist.launch_chained, here over gloo with host staging; bench.py runs it over RCCL).
    The per-rank Newton iteration counts add up to the oracle's serial-chain count, every cell is integrated once,
    and the all-reduced spectra equal one engine's (summation order only)."""
    import torch.multiprocessing as mp
    from helpers import parity
    from is3d2_amd import build_engine
    from oracle import oracle as O
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29700 + (os.getpid() + 13 * world + chains + 7 * npass) % 1000
    procs = [ctx.Process(target=_chain_worker, args=(r, world, port, chains, npass, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = _chain_surface()
    spec = _chain_spec(chains)
    _, rst = O.spectra(spec, s, threads=chains, return_stats=True)
    assert sum(r[1] for r in res) == rst[3]
    assert sum(r[2] for r in res) == len(s["tau"])
    e = build_engine(spec, s, device=0)
    one = e.calculate_spectra()
    e.close()
    got = res[0][3]
    assert np.array_equal(np.isnan(got), np.isnan(one))
    assert parity(np.nan_to_num(got), np.nan_to_num(one))[0] < 1e-12
