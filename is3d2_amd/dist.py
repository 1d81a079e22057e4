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
surface: every rank then holds the whole surface, walks the chains itself and integrates its range
only (Engine.set_cell_window), so each rank sees the serial chain's solutions.
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
