"""Multi-GPU decomposition of the continuous-spectra path (one process per GPU).

Freeze-out cells are independent and dN/(pT dpT dphi dy) is a plain sum over cells
(MomentumSpectra.cpp:365, 383-411), so the path shards by cells with no exchange until
the end: each rank integrates its contiguous cell range and one all-reduce (sum, FP64)
over torch.distributed ('nccl' = RCCL over xGMI on MI355X, 'gloo' in CPU tests) combines
the [species][pT][phi][y] accumulators.  The only other collective is the tiny
ds_max-weighted Plasma average (5 sums) the PTB table needs (readindata.cpp:316-366).
PTMA with reference warm-start chains (famod_chains > 0) does not shard (it is a serial
recurrence per chain) and runs on one rank.
"""
import numpy as np


def shard_range(n, rank, world):
    """Contiguous cell range [lo, hi) of `rank` (balanced to within one cell)."""
    return n * rank // world, n * (rank + 1) // world


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
