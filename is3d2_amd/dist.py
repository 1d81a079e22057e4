"""Multi-GPU decomposition of the continuous-spectra path (one process per GPU).

Freeze-out cells are independent and dN/(pT dpT dphi dy) is a plain sum over cells
(MomentumSpectra.cpp:365, 383-411), so the path shards by cells with no exchange until
the end: each rank integrates its contiguous cell range and one all-reduce (sum, FP64)
over torch.distributed ('nccl' = RCCL over xGMI on MI355X, 'gloo' in CPU tests) combines
the [species][pT][phi][y] accumulators.  The only other collective is the tiny
ds_max-weighted Plasma average (5 sums) the PTB table needs (readindata.cpp:316-366).
Shards are contiguous cell ranges balanced by estimated cost: a cell with
u.dsigma <= 0 is skipped by every kernel (MomentumSpectra.cpp:132) and costs only its record prep.
PTMA with the reference's warm-start chains (famod_chains > 0) is a serial recurrence over the whole
surface (MomentumSpectra.cpp:1132-1135, 1308-1364): every rank then holds the whole surface and solves only its
range of chain positions (Engine.set_chain_range), starting each chain from the end state the previous rank
sends after every pass of the segmented solve (launch_chained: point-to-point send / recv of 4 C + 1 doubles per
pass, RCCL on the GPU), so each rank's solutions are the serial chain's and its prepass shrinks with the rank count.
"""
import numpy as np

SKIP_COST = 0.02     # a u.dsigma <= 0 cell relative to a live one (record prep only); group.hip kSkipCost


def shard_range(n, rank, world):
    """Contiguous cell range [lo, hi) of `rank` (equal counts, to within one cell)."""
    return n * rank // world, n * (rank + 1) // world


def cell_costs(surf):
    """Estimated integration cost per cell: 1 for a live cell, SKIP_COST for u.dsigma <= 0."""
    tau = surf["tau"]
    ut = np.sqrt(1. + surf["ux"] ** 2 + surf["uy"] ** 2 + tau * tau * surf["un"] ** 2)
    uds = ut * surf["dat"] + surf["ux"] * surf["dax"] + surf["uy"] * surf["day"] + surf["un"] * surf["dan"]
    return np.where(uds > 0.0, 1.0, SKIP_COST)


def balanced_ranges(costs, world):
    """Contiguous [lo, hi) per rank with ~equal summed cost (the rule group.hip applies in-library)."""
    n = len(costs)
    pre = np.concatenate([[0.0], np.cumsum(costs)])
    bounds = [0]
    for k in range(1, world):
        c = int(np.searchsorted(pre, pre[-1] * k / world, side="left"))
        bounds.append(min(max(c, bounds[-1]), n))
    bounds.append(n)
    return [(bounds[k], bounds[k + 1]) for k in range(world)]


def device_cell_costs(spec, surf, T_avg=None, device=0):
    """Per-cell costs from the engine's prepass (is3d_cell_costs: PTM / PTB separable-fallback cells cost
    1.4 / 1.8 of a modified one, u.dsigma <= 0 cells 0.02) -- the model is3d_create_devices balances with."""
    from .engine import build_engine
    e = build_engine(spec, surf, T_avg=T_avg, device=device)
    try:
        return e.cell_costs()
    finally:
        e.close()


def shard_bounds(surf, rank, world, costs=None):
    """This rank's cost-balanced contiguous cell range of `surf` (costs: e.g. device_cell_costs; default the
    u.dsigma model of cell_costs)."""
    return balanced_ranges(cell_costs(surf) if costs is None else np.asarray(costs), world)[rank]


def average_sums(surf, include_baryon=0):
    """The six ds_max-weighted sums behind the Plasma averages (vol, T, E, P, muB, nB)."""
    tau = surf["tau"]; tau2 = tau * tau
    ut = np.sqrt(1. + surf["ux"] ** 2 + surf["uy"] ** 2 + tau2 * surf["un"] ** 2)
    uds = ut * surf["dat"] + surf["ux"] * surf["dax"] + surf["uy"] * surf["day"] + surf["un"] * surf["dan"]
    ds_ds = surf["dat"] ** 2 - surf["dax"] ** 2 - surf["day"] ** 2 - surf["dan"] ** 2 / tau2
    w = np.abs(uds) + np.sqrt(np.abs(uds * uds - ds_ds))
    z = np.zeros_like(w)
    muB = surf["muB"] if include_baryon else z
    nB = surf["nB"] if include_baryon else z
    return np.array([w.sum(), (surf["T"] * w).sum(), (surf["E"] * w).sum(), (surf["P"] * w).sum(),
                     (muB * w).sum(), (nB * w).sum()])


def global_averages(local_sums, all_reduce):
    """Plasma averages of the whole (sharded) surface, 15-digit rounded like the reference file.
    all_reduce(np.ndarray) -> np.ndarray sums over ranks."""
    s = all_reduce(np.asarray(local_sums, dtype=np.float64))
    return np.array([float("%.15g" % (s[k] / s[0])) for k in range(1, 6)])


def torch_all_reduce(dist, device=None):
    """np.ndarray sum over ranks via torch.distributed (on `device` for nccl, CPU for gloo)."""
    import torch

    def f(a):
        t = torch.as_tensor(a, dtype=torch.float64)
        if device is not None:
            t = t.to(device)
        dist.all_reduce(t)
        return t.cpu().numpy()
    return f


def chain_bounds(surf, rank, world, chains, costs=None):
    """Chain positions [q0, q1) of `rank` when the PTMA warm-start chains (C = chains) are split over the ranks: the
    cost-balanced cell boundaries rounded to whole positions (C cells each), as group.hip chain_windows does."""
    n = len(surf["tau"])
    C = max(1, min(int(chains), n))
    P = (n + C - 1) // C
    r = balanced_ranges(cell_costs(surf) if costs is None else np.asarray(costs), world)
    q = [0]
    for k in range(world - 1):
        q.append(max(q[-1], min(P, (r[k][1] + C // 2) // C)))
    q.append(P)
    if P >= world:
        # every rank holds at least one position (launch_chained needs a live range on each rank): clamp the inner
        # boundaries into [k, P - (world - k)] -- a no-op unless the cost balance collapsed a range
        for k in range(1, world):
            q[k] = min(max(q[k], q[k - 1] + 1), P - (world - k))
    return q[rank], q[rank + 1]


def launch_chained(eng, out_ptr, stream_ptr, rank, world, dist, device=None, sync=None):
    """One pass of the PTMA hot path with the warm-start chains split over the ranks (include/is3d_amd.h staged
    launch): rank k solves its chain positions; after every chain pass j but the last it sends its range's end states
    (slot j & 1) to rank k + 1, which puts them into its incoming slot before its pass j + 1; then the finishers run in
    rank order, each handing its final states (slot 2) on.  With the 'nccl' backend every copy, send and receive
    is ordered on the GPU streams (torch's current stream = the launch stream) and the host never waits; with
    'gloo' the boundary buffers live on the host (device=None) and sync() -- e.g. the launch stream's synchronize --
    runs after each copy out of the engine, before the send reads the buffer.  Every rank's range must hold at
    least one position (chain_bounds gives one whenever there are >= world positions); a rank whose range is empty
    or whose launch_begin fails makes every rank raise -- the check is one collective before the first send, so no
    successor is left waiting in recv.  The caller then all-reduces the spectra and calls eng.finish()."""
    import torch
    err = None
    try:
        eng.launch_begin(out_ptr, stream_ptr)
        npass, nb = eng.chain_passes(), eng.chain_boundary_size()
        if npass <= 0 or nb <= 0:
            err = "rank %d has no PTMA chain positions (empty chain range)" % rank
    except Exception as exc:       # noqa: BLE001 -- re-raised below on this rank, after the collective
        err, npass, nb = exc, 0, 0
    ok = torch.tensor([0.0 if err is not None else 1.0], dtype=torch.float64, device=device)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if err is not None:
        raise err if isinstance(err, Exception) else RuntimeError("launch_chained: " + err)
    if ok.item() < 1.0:
        raise RuntimeError("launch_chained: another rank could not start its chain range (see its error)")
    pred = rank - 1 if rank > 0 else None
    succ = rank + 1 if rank + 1 < world else None
    rbuf = [torch.zeros(nb, dtype=torch.float64, device=device) for _ in range(3)]
    sbuf = [torch.zeros(nb, dtype=torch.float64, device=device) for _ in range(3)]
    sends = [None, None, None]

    def send(slot):
        if sends[slot] is not None:
            sends[slot].wait()          # the buffer's previous send (two passes back) is out before it is rewritten
        eng.chain_boundary_get(slot, sbuf[slot])
        if sync is not None:
            sync()
        sends[slot] = dist.isend(sbuf[slot], dst=succ)

    for j in range(npass):
        if pred is not None and j > 0:
            dist.recv(rbuf[(j - 1) & 1], src=pred)
            eng.chain_boundary_put((j - 1) & 1, rbuf[(j - 1) & 1])
        eng.chain_pass(j)
        if succ is not None and j + 1 < npass:      # the successor reads pass j's states in its pass j + 1
            send(j & 1)
    if pred is not None:
        dist.recv(rbuf[2], src=pred)
        eng.chain_boundary_put(2, rbuf[2])
    eng.chain_end()
    if succ is not None:
        send(2)
    eng.launch_end()
    for w in sends:
        if w is not None:
            w.wait()
