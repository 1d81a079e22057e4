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
