#!/usr/bin/env python3
"""Benchmark of the Cooper-Frye continuous-spectra hot path on MI355X.

Metric (BASELINE.json): freezeout-cell x species x momentum-point evaluations per
second, i.e. N_cells x N_species x N_pT x N_phi x N_y / wall time of one full pass
(prepass + integral + reduction, plus the RCCL all-reduce of the spectra for N > 1),
surface already resident in HBM.

Default workload = BASELINE config 2 (the configuration the metric is quoted on):
10^5 synthetic 3+1D cells per GPU, SMASH HRG (444 chosen species), Grad-14 delta-f
with shear + bulk, 48-pt pT x 32-pt phi x 21 y.  N > 1 GPUs: weak scaling, each rank
owns its own 10^5-cell shard of an N x 10^5-cell surface; the per-rank spectra are
summed with one RCCL all-reduce (torch.distributed 'nccl' = RCCL over xGMI).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config config2] [--df-mode 1..5]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FLOPS_PER_NODE = {1: 65, 2: 67, 3: 140, 4: 140, 5: 140}   # SURVEY.md 8(d), frozen algorithmic counts
FP64_PEAK_TFLOPS = 78.6                                     # MI355X FP64 vector (= FP64 matrix) dense peak
HBM_PEAK_BPS = 8.0e12                                       # MI355X HBM3E
MODE_NAMES = {1: "grad14", 2: "rta-ce", 3: "ptm", 4: "ptb", 5: "ptma"}

CONFIGS = {
    # name: cells per GPU, hrg, chosen, grid, dimension, default df_mode, flags, scaling
    "config1": dict(cells=1000, hrg=2, chosen="pikp", pT="pT24", phi="phi24", dim=2, mode=1, flags={}, scaling="weak"),
    "config2": dict(cells=100000, hrg=2, chosen="smash", pT="pT48", phi="phi32", dim=3, mode=1, flags={}, scaling="weak"),
    "config3": dict(cells=100000, hrg=2, chosen="smash", pT="pT48", phi="phi32", dim=3, mode=2,
                    flags=dict(include_baryon=1, include_baryondiff_deltaf=1), scaling="weak"),
    "config4": dict(cells=1000000, hrg=2, chosen="smash", pT="pT48", phi="phi32", dim=3, mode=2, flags={}, scaling="strong"),
    # HBM stress case: UrQMD HRG, PTMA + baryon, 64-pt Gauss-Laguerre tables for the thermal integrals
    "config5": dict(cells=5000000, hrg=1, chosen="urqmd", pT="pT48", phi="phi32", dim=3, mode=5, gla=64,
                    flags=dict(include_baryon=1, include_baryondiff_deltaf=1), scaling="strong"),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def make_surface(cfg, rank, world, dim, baryon):
    from is3d2_amd import synth
    if cfg["scaling"] == "strong":
        total = cfg["cells"]
        lo = rank * total // world
        hi = (rank + 1) * total // world
        s = synth.as_read(synth.surface(total, seed=7, dimension=dim, baryon=baryon, full3d=(dim == 3)))
        return {k: np.ascontiguousarray(v[lo:hi]) for k, v in s.items()}
    return synth.as_read(synth.surface(cfg["cells"], seed=7 + rank, dimension=dim, baryon=baryon, full3d=(dim == 3)))


def cpu_baseline(spec, surf, units_per_cell, target_s=15.0, operation=1):
    """Oracle ('port' of the reference loop) on the host cores, on a cell prefix of the same workload."""
    from oracle import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS") or min(16, os.cpu_count() or 1))
    T_avg = O.averages(surf)[0]

    def run(sample):
        if operation == 0:
            O.dndx(spec, sample, T_avg=T_avg, threads=threads, omp_threads=threads, carry=0)
        else:
            O.spectra(spec, sample, T_avg=T_avg, threads=threads, omp_threads=threads)

    n_probe = min(len(surf["tau"]), max(2 * threads, 32))
    probe = {k: v[:n_probe] for k, v in surf.items()}
    t = time.perf_counter()
    run(probe)
    dt = time.perf_counter() - t
    n = int(min(len(surf["tau"]), max(n_probe, n_probe * target_s / max(dt, 1e-3))))
    n = max(threads, (n // threads) * threads)
    sample = {k: v[:n] for k, v in surf.items()}
    t = time.perf_counter()
    run(sample)
    dt = time.perf_counter() - t
    return dict(value=n * units_per_cell / dt, unit="cell-species-mom-points/s", cores=threads, kind="port",
                sample="first %d cells of rank 0's shard, same species/grid/df mode; %.1f s with %d OpenMP threads"
                       % (n, dt, threads))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="config2", choices=sorted(CONFIGS))
    ap.add_argument("--df-mode", type=int, default=0)
    ap.add_argument("--cells", type=int, default=0, help="override cells per GPU (weak) / total (strong)")
    ap.add_argument("--chosen", default="", help="override the chosen-species list (pikp, smash, urqmd)")
    ap.add_argument("--operation", type=int, default=1, choices=[0, 1],
                    help="1 continuous spectra (default, the BASELINE metric); 0 spacetime distributions dN/dX")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=25.0)
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))

    import torch
    import torch.distributed as dist
    # rehearsal knobs for a 1-GPU box (never set by the driver): every rank on one device, gloo
    backend = os.environ.get("IS3D_BENCH_BACKEND", "nccl")
    local_rank = int(os.environ.get("IS3D_BENCH_DEVICE", local_rank))
    if world > 1:
        dist.init_process_group(backend, init_method="env://")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from is3d2_amd import build_engine, make_spec

    cfg = dict(CONFIGS[args.config])
    if args.cells:
        cfg["cells"] = args.cells
    if args.chosen:
        cfg["chosen"] = args.chosen
    mode = args.df_mode or cfg["mode"]
    flags = dict(cfg["flags"])
    if mode == 4:
        flags.pop("include_baryon", None); flags.pop("include_baryondiff_deltaf", None)
    spec = make_spec(hrg_eos=cfg["hrg"], chosen=cfg["chosen"], pT=cfg["pT"], phi=cfg["phi"], y="y21", eta="eta24",
                     dimension=cfg["dim"], df_mode=mode, gla_points=cfg.get("gla", 32), **flags)
    surf = make_surface(cfg, rank, world, cfg["dim"], bool(flags.get("include_baryon", 0)))
    n_local = len(surf["tau"])
    from is3d2_amd import dist as D
    reduce = D.torch_all_reduce(dist, dev) if world > 1 else (lambda a: a)
    T_avg = D.global_averages(D.average_sums(surf, flags.get("include_baryon", 0)), reduce)[0]

    eng = build_engine(spec, surf, T_avg=T_avg, device=local_rank)
    outsize = eng.output_size()
    out = torch.zeros(outsize, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    nsp, npT, nphi = len(spec["species"]["mass"]), len(spec["pT"]), len(spec["phi"])
    ny = len(spec["y"]) if cfg["dim"] == 3 else 1
    neta = 1 if cfg["dim"] == 3 else len(spec["eta"])
    units_per_cell = nsp * npT * nphi * ny
    units_local = n_local * units_per_cell

    def step():
        if args.operation == 0:
            t, r, ph = eng.calculate_dN_dX()      # synchronous: device passes + small host binning epilogue
            if world > 1:
                binned = torch.from_numpy(np.concatenate([t.ravel(), r.ravel(), ph.ravel()])).to(dev)
                dist.all_reduce(binned)
            return eng.stats()
        eng.launch(out.data_ptr(), stream)
        if world > 1:
            dist.all_reduce(out)
        eng.finish()
        return eng.stats()

    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kstats = [step() for _ in range(args.steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    units_all = torch.tensor([float(units_local)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(units_all)
    elapsed = tmax.item()
    total_units = units_all.item() * args.steps

    if args.operation == 0 and world > 1 and spec["bins"].get("threads", 0):
        raise SystemExit("operation 0 with reference thread emulation runs on one rank")
    ms_spectra = float(np.mean([s["ms_spectra"] for s in kstats]))
    ms_total = float(np.mean([s["ms_total"] for s in kstats]))
    flops = FLOPS_PER_NODE[mode] * neta * units_local
    achieved = flops / (ms_spectra * 1e-3) / 1e12
    traffic, executed = None, None
    key = "%s_mode%d" % (args.config, mode) if args.operation == 1 else "%s_op0_mode%d" % (args.config, mode)
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc):
        traffic = json.load(open(pmc)).get(key)
    pv = os.path.join(ROOT, "profiles", "pmc_valu.json")
    if os.path.exists(pv):
        executed = json.load(open(pv)).get(key)
    if executed is not None:
        executed = dict(executed, note="PMC pass (tag) of this workload: share of SIMD cycles issuing VALU; "
                                       "achieved/frac above use the reference's frozen flop counts")

    if rank == 0:
        res = {
            "metric": "freezeout-cell-species-mom-points/sec",
            "value": total_units / elapsed,
            "unit": "cell-species-mom-points/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": cfg["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md 8d surface generator, seed 7+rank)",
            "config": {
                "workload": "%s%s: %s %s synthetic freeze-out cells%s x %s HRG (%d species) x %s delta-f, %d pT x %d phi x %d y%s"
                            % (args.config, " operation 0 (dN/dX)" if args.operation == 0 else "", cfg["cells"],
                               "3+1D" if cfg["dim"] == 3 else "2+1D", " per GPU" if cfg["scaling"] == "weak" else " total",
                               "SMASH" if cfg["hrg"] == 2 else "UrQMD", nsp, MODE_NAMES[mode], npT, nphi, ny,
                               "" if neta == 1 else " x %d eta" % neta),
                "operation": args.operation,
                "cells_per_gpu": n_local, "species": nsp, "grid": [npT, nphi, ny, neta], "df_mode": mode,
                "parallelism": "dp%d (cell shards + RCCL all-reduce of spectra)" % world if world > 1 else "1 GPU",
            },
            "roofline": {
                "bound": "mfma", "pipe": "fp64 (vector ALU; MI355X FP64 vector peak = FP64 matrix peak)",
                "kernel": "k_spectra" if args.operation == 1 else "k_dndx", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                "algorithmic_flops_per_launch": flops, "flops_per_point": FLOPS_PER_NODE[mode] * neta,
                "kernel_ms": ms_spectra, "pass_ms": ms_total, "executed": executed,
                # HBM view (north_star): PMC bytes per launch over the live kernel time, vs 8 TB/s
                "hbm_gbs": None if traffic is None else traffic / (ms_spectra * 1e-3) / 1e9,
                "hbm_frac": None if traffic is None else traffic / (ms_spectra * 1e-3) / HBM_PEAK_BPS,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(spec, surf, units_per_cell, args.cpu_seconds, args.operation)
        print(json.dumps(res), flush=True)
    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
