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

Ranks: under a launcher (torch.distributed.run sets WORLD_SIZE / RANK / LOCAL_RANK) the world comes from the
environment and --gpus must agree with it; a plain `python bench.py --gpus N` with N > 1 starts the N rank
processes itself (spawn_ranks: fresh interpreters with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, started
before anything touches the GPU) and exits with the first failing rank's status.
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
FP64_LANE_OPS_PEAK = 256 * 4 * 16 * 2.4e9                  # FP64 VALU lane-ops/s: 16 lanes/clk per SIMD
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


def spawn_ranks(n, argv):
    """`bench.py --gpus N` without a launcher: run N rank processes of this script (rank r on GPU r, rendezvous on
    127.0.0.1) and return the exit status -- 0, or the first failing rank's (the other ranks are then terminated,
    so a rank stuck in a collective cannot hang the run).  Called before torch is imported: the parent never
    touches the GPU and never replaces itself (no exec)."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), IS3D_BENCH_LAUNCHER="bench.py --gpus")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    rc = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.send_signal(signal.SIGTERM)
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    if rc == 0:
        rc = next((p.returncode for p in procs if p.returncode != 0), 0)
    if rc:
        log("bench.py: a rank exited with status %s" % rc)
    return 1 if rc < 0 else rc


def resolve_world(gpus, environ):
    """(world, spawn) from --gpus and the launcher's environment.  Under a launcher WORLD_SIZE decides and a
    different --gpus is an error (a SCALE run must never time fewer ranks than it names); without one, --gpus N
    (default 1) ranks, spawned by this script when N > 1."""
    if environ.get("WORLD_SIZE"):
        world = int(environ["WORLD_SIZE"])
        if gpus is not None and gpus != world:
            raise SystemExit("bench.py: --gpus %d but the launcher started WORLD_SIZE=%d ranks" % (gpus, world))
        return world, False
    n = 1 if gpus is None else gpus
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    return n, n > 1


def make_surface(cfg, rank, world, dim, baryon, whole=False):
    """This rank's cells: weak scaling -- its own surface (seed 7 + rank); strong scaling -- its cost-balanced
    contiguous range of the one surface (dist.shard_bounds), or the whole surface (whole=True, PTMA warm-start
    chains: every rank then solves and integrates its own chain positions, dist.chain_bounds)."""
    from is3d2_amd import dist as D, synth
    if cfg["scaling"] == "strong":
        s = synth.as_read(synth.surface(cfg["cells"], seed=7, dimension=dim, baryon=baryon, full3d=(dim == 3)))
        lo, hi = D.shard_bounds(s, rank, world)
        if whole:
            return s, (lo, hi)
        return {k: np.ascontiguousarray(v[lo:hi]) for k, v in s.items()}, None
    return synth.as_read(synth.surface(cfg["cells"], seed=7 + rank, dimension=dim, baryon=baryon, full3d=(dim == 3))), None


def _host_cpu():
    """CPU model, logical CPUs of the host (nproc), CPUs this process may run on, and the cgroup CPU quota."""
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return model, os.cpu_count() or 1, len(os.sched_getaffinity(0)), quota


_NATIVE_ORACLE = {}     # the -march=native oracle built on this host by the first CPU leg (compiler line)


def cpu_baseline(spec, surf, units_per_cell, n_full, target_s=25.0, operation=1):
    """Oracle (a C/OpenMP 'port' of the reference loop, oracle/Makefile flags) on the host cores, on a
    cell prefix of the same workload sized to >= target_s, extrapolated linearly to the full shard
    (the cost is linear in the cell count).  Threads: OMP_NUM_THREADS when set (the GPU
    pool sets it to the box's CPU share, 16 per GPU; nproc there counts the whole host), else every
    CPU in this process's affinity mask."""
    import subprocess
    import tempfile
    # -O3 -fopenmp -march=native, built here on the box's own host (a -march=native binary cannot
    # ship from the build container); the portable in-tree build if no compiler is at hand
    compiler = _NATIVE_ORACLE.get("compiler")
    if not os.environ.get("IS3D_ORACLE_LIB"):
        out = os.path.join(tempfile.gettempdir(), "is3d_oracle_native_%d.so" % os.getpid())
        try:
            r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "native", "NATIVE_OUT=" + out],
                               capture_output=True, text=True, timeout=120)
            if r.returncode == 0 and os.path.exists(out):
                os.environ["IS3D_ORACLE_LIB"] = out
                compiler = r.stdout.strip().splitlines()[-1] + " (built on this host)"
                _NATIVE_ORACLE["compiler"] = compiler
        except (OSError, subprocess.SubprocessError):
            pass
    from oracle import oracle as O
    model, nproc, affinity, quota = _host_cpu()
    threads = int(os.environ.get("OMP_NUM_THREADS") or affinity)
    T_avg = O.averages(surf)[0]

    def run(sample):
        if operation == 0:
            O.dndx(spec, sample, T_avg=T_avg, threads=threads, omp_threads=threads, carry=0)
        else:
            O.spectra(spec, sample, T_avg=T_avg, threads=threads, omp_threads=threads)

    n_probe = min(len(surf["tau"]), max(8 * threads, 64))      # ~4 s: thread start-up stays negligible
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
    if compiler is None:
        try:
            mk = open(os.path.join(ROOT, "oracle", "Makefile")).read()
            compiler = "gcc " + [ln.split("=", 1)[1].strip() for ln in mk.splitlines() if ln.startswith("CFLAGS")][0]
            compiler += " (portable in-tree build: no compiler on this host)"
        except (OSError, IndexError):
            compiler = "unknown"
    return dict(value=n * units_per_cell / dt, unit="cell-species-mom-points/s", cores=threads, kind="port",
                sample="first %d cells of rank 0's shard (same species/grid/df mode): %.1f s with %d OpenMP threads"
                       % (n, dt, threads),
                sample_cells=n, sample_s=dt, extrapolated_s=dt * n_full / n, extrapolated_cells=n_full,
                nproc=nproc, affinity_cpus=affinity, cgroup_cpu_quota=quota, cpu_model=model,
                compiler=compiler,
                note="cores = OMP_NUM_THREADS when set: the GPU pool gives a one-GPU box a 16-CPU share "
                     "(cgroup_cpu_quota) of a host whose nproc counts every CPU")


def executed_roofline(args, mode, ms_spectra, ms_total, neta, units_local, n_local, outsize, kernel):
    """Roofline record of the dominant kernel (k_spectra).  The kernel is FP64-VALU bound (SURVEY.md 8d:
    ~1e-5 B per unit), so `achieved` is the FP64 work the kernel EXECUTES per launch -- the hardware
    counter SQ_INSTS_VALU_FLOPS_FP64 (FMA = 2) from the committed rocprofv3 pass of this workload
    (profiles/pmc_valu.json) -- over the launch's average duration measured live here with HIP events on
    the launch stream, against the 78.6 TFLOP/s FP64 vector peak.  fp64_pipe_frac counts issue slots
    instead (every FP64 add / mul / fma / transcendental wave-instruction takes the pipe for 4 cycles).
    The reference-loop operation count of SURVEY.md 8d (F flops per node) is reported separately as
    reference_equivalent_tflops: the factorised kernel executes ~1/4 of those operations, so that rate
    is not a fraction of any peak."""
    cfg = args.config + ("_cells%d" % args.cells if getattr(args, "cells", 0) else "")
    key = "%s_mode%d" % (cfg, mode) if args.operation == 1 else "%s_op0_mode%d" % (cfg, mode)
    pmc = {}
    for name in ("pmc_traffic", "pmc_valu"):
        path = os.path.join(ROOT, "profiles", name + ".json")
        pmc[name] = json.load(open(path)).get(key) if os.path.exists(path) else None
    from is3d2_amd import _lib
    bid = _lib.build_id()
    traffic, ex = pmc["pmc_traffic"], pmc["pmc_valu"]
    stale = []
    # counter summaries count only for the identical build (is3d_build_id: hash of the sources and flags):
    # a profile of an older kernel would price this run's time against another kernel's instruction counts
    if isinstance(traffic, dict):
        if traffic.get("build_id") != bid:
            stale.append("traffic: %s (build %s)" % (traffic.get("tag"), traffic.get("build_id")))
            traffic = None
        else:
            traffic = traffic.get("hbm_bytes_per_pass", traffic["hbm_bytes_per_launch"])
    elif traffic is not None:
        stale.append("traffic: untagged")
        traffic = None
    if ex is not None and ex.get("build_id") != bid:
        stale.append("executed: %s (build %s)" % (ex.get("tag"), ex.get("build_id")))
        ex = None
    t = ms_spectra * 1e-3
    ref_flops = FLOPS_PER_NODE[mode] * neta * units_local
    algo_bytes = 200.0 * n_local + 8.0 * outsize           # surface read once + spectra written once
    r = {"bound": "valu", "pipe": "fp64 vector ALU (k_spectra issues no MFMA)", "kernel": kernel,
         "achieved": None, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": None, "traffic": traffic,
         "kernel_ms": ms_spectra, "pass_ms": ms_total,
         "reference_equivalent_tflops": ref_flops / t / 1e12, "reference_flops_per_node": FLOPS_PER_NODE[mode] * neta,
         "algorithmic_bytes": algo_bytes,
         "traffic_over_algorithmic": None if traffic is None else traffic / algo_bytes,
         "hbm_gbs": None if traffic is None else traffic / t / 1e9,
         "hbm_frac": None if traffic is None else traffic / t / HBM_PEAK_BPS,
         "build_id": bid}
    if stale:
        r["stale_profiles"] = "counter summaries of another build, not used: " + "; ".join(stale)
    if ex is not None:
        if "fp64_flops_per_launch" in ex:
            # per pass: an F_TS launch over more than one table chunk runs k_spectra once per chunk
            flops = ex.get("fp64_flops_per_pass", ex["fp64_flops_per_launch"])
            r["achieved"] = flops / t / 1e12
            r["frac"] = r["achieved"] / FP64_PEAK_TFLOPS
            r["executed_flops_per_unit"] = flops / units_local
            r["launches_per_pass"] = ex.get("launches_per_pass", 1.0)
        if "fma_f64_insts_per_launch" in ex:
            ins = ex.get("launches_per_pass", 1.0) * sum(ex.get(c + "_insts_per_launch", 0.0)
                                                          for c in ("add_f64", "mul_f64", "fma_f64", "trans_f64"))
            r["fp64_pipe_frac"] = 64.0 * ins / (t * FP64_LANE_OPS_PEAK)
        r["executed"] = dict(ex, note="rocprofv3 PMC passes of this workload (tag); counts per k_spectra launch")
    return r


def run_workload(args, cfg_name, mode, steps, warmup, rank, world, local_rank, dev, dist, classes=True):
    """Build the engine for one workload on this rank's shard, run `warmup` untimed and `steps` timed
    passes (barrier + synchronize on both sides, max over ranks) and return the measurement.  classes: the
    engine's integrand classes (is3d_set_species_classes; the default) or one integral per species."""
    import torch
    from is3d2_amd import build_engine, make_spec
    from is3d2_amd import dist as D

    cfg = dict(CONFIGS[cfg_name])
    if args.cells and cfg_name == args.config:
        cfg["cells"] = args.cells
    if args.chosen and cfg_name == args.config:
        cfg["chosen"] = args.chosen
    mode = mode or cfg["mode"]
    flags = dict(cfg["flags"])
    if mode == 4:
        flags.pop("include_baryon", None); flags.pop("include_baryondiff_deltaf", None)
    spec = make_spec(hrg_eos=cfg["hrg"], chosen=cfg["chosen"], pT=cfg["pT"], phi=cfg["phi"], y="y21", eta="eta24",
                     dimension=cfg["dim"], df_mode=mode, gla_points=cfg.get("gla", 32), **flags)
    # one surface split over the ranks (strong scaling) with PTMA warm-start chains: a recurrence over the whole surface
    chained = mode == 5 and spec["params"]["famod_chains"] > 0 and world > 1 and cfg["scaling"] == "strong"
    surf, window = make_surface(cfg, rank, world, cfg["dim"], bool(flags.get("include_baryon", 0)), whole=chained)
    qrange = None
    if chained:
        # PTMA warm-start chains split over the ranks (dist.launch_chained): every rank holds the whole surface and
        # solves its own chain positions, the boundary states passed rank to rank after every pass
        C = spec["params"]["famod_chains"]
        qrange = D.chain_bounds(surf, rank, world, C)
        n_all = len(surf["tau"])
        window = (min(n_all, qrange[0] * C), min(n_all, qrange[1] * C))
    n_local = len(surf["tau"]) if window is None else window[1] - window[0]
    reduce = D.torch_all_reduce(dist, dev) if world > 1 else (lambda a: a)
    mine = surf if window is None else {k: v[window[0]:window[1]] for k, v in surf.items()}
    T_avg = D.global_averages(D.average_sums(mine, flags.get("include_baryon", 0)), reduce)[0]

    eng = build_engine(spec, surf, T_avg=T_avg, device=local_rank, species_classes=classes)
    for kv in args.tune or []:      # is3d_set_tuning knobs (A/B experiments; the driver's runs use the defaults)
        k, v = kv.split("=", 1)
        eng.set_tuning(k, int(float(v)))
    n_integrated = eng.species_integrated()
    if qrange is not None:
        eng.set_chain_range(*qrange)
    elif window is not None:
        eng.set_cell_window(*window)
    outsize = eng.output_size()
    out = torch.zeros(outsize, dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    nsp, npT, nphi = len(spec["species"]["mass"]), len(spec["pT"]), len(spec["phi"])
    ny = len(spec["y"]) if cfg["dim"] == 3 else 1
    neta = 1 if cfg["dim"] == 3 else len(spec["eta"])
    units_per_cell = nsp * npT * nphi * ny
    units_local = n_local * units_per_cell
    operation = args.operation if cfg_name == args.config else 1
    if operation == 0 and world > 1 and spec["bins"].get("threads", 0):
        raise SystemExit("operation 0 with reference thread emulation runs on one rank")

    def step():
        if operation == 0:
            t, r, ph = eng.calculate_dN_dX()      # synchronous: device passes + small host binning epilogue
            if world > 1:
                binned = torch.from_numpy(np.concatenate([t.ravel(), r.ravel(), ph.ravel()])).to(dev)
                dist.all_reduce(binned)
            return eng.stats()
        if qrange is not None:
            if args.backend == "nccl":
                # boundary states in HBM; copies, sends and receives ordered on the launch stream
                D.launch_chained(eng, out.data_ptr(), stream, rank, world, dist, device=dev)
            else:
                # gloo's transport is the host: host boundary buffers, and the launch stream synchronised after each
                # copy out of the engine so a send never reads a buffer before the copy has landed
                D.launch_chained(eng, out.data_ptr(), stream, rank, world, dist, device=None,
                                 sync=torch.cuda.current_stream(dev).synchronize)
        else:
            eng.launch(out.data_ptr(), stream)
        if world > 1:
            dist.all_reduce(out)
        eng.finish()
        return eng.stats()

    for _ in range(warmup):
        step()
    nsplit = eng.get_tuning("splits")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kstats = [step() for _ in range(steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    units_all = torch.tensor([float(units_local)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        dist.all_reduce(units_all)
    elapsed = tmax.item()
    total_units = units_all.item() * steps
    eng.close()
    del out

    ms_spectra = float(np.mean([s["ms_spectra"] for s in kstats]))
    ms_total = float(np.mean([s["ms_total"] for s in kstats]))
    kernel = "k_spectra" if operation == 1 else "k_dndx"
    sub = argparse.Namespace(config=cfg_name, operation=operation, cells=args.cells if cfg_name == args.config else 0)
    roofline = executed_roofline(sub, mode, ms_spectra, ms_total, neta, units_local, n_local, outsize, kernel)
    extras = []
    if flags.get("include_baryon"):
        extras.append("baryon on" + (" + baryon diffusion delta-f" if flags.get("include_baryondiff_deltaf") else ""))
    if cfg.get("gla", 32) != 32:
        extras.append("%d-pt Gauss-Laguerre" % cfg["gla"])
    if mode == 5 and spec["params"]["famod_chains"] > 0:
        extras.append("%d warm-start Newton chain%s" % (spec["params"]["famod_chains"],
                                                       "" if spec["params"]["famod_chains"] == 1 else "s"))
    backend_name = {"nccl": "RCCL"}.get(args.backend, args.backend)
    config = {
        "workload": "%s%s: %s %s synthetic freeze-out cells%s x %s HRG (%d species) x %s delta-f%s, %d pT x %d phi x %d y%s"
                    % (cfg_name, " operation 0 (dN/dX)" if operation == 0 else "", cfg["cells"],
                       "3+1D" if cfg["dim"] == 3 else "2+1D", " per GPU" if cfg["scaling"] == "weak" else " total",
                       "SMASH" if cfg["hrg"] == 2 else "UrQMD", nsp, MODE_NAMES[mode],
                       "".join(" (%s)" % e for e in extras[:1]) + "".join(", %s" % e for e in extras[1:]),
                       npT, nphi, ny, "" if neta == 1 else " x %d eta" % neta),
        "operation": operation,
        "cells_per_gpu": n_local, "species": nsp, "grid": [npT, nphi, ny, neta], "df_mode": mode,
        "species_integrated": n_integrated,
        "famod_chains": spec["params"]["famod_chains"] if mode == 5 else None,
        "cell_splits": nsplit if operation == 1 else None,
        "parallelism": ("dp%d (cell shards + %s all-reduce of spectra%s)"
                        % (world, backend_name,
                           "; PTMA chain positions split, boundary states sent rank to rank per pass" if chained else "")
                        if world > 1 else "1 GPU"),
    }
    if world > 1:
        config["backend"] = args.backend
        config["launcher"] = os.environ.get("IS3D_BENCH_LAUNCHER", "external (WORLD_SIZE from the environment)")
        if os.environ.get("IS3D_BENCH_DEVICE") is not None:
            config["rehearsal"] = "every rank on device %s (IS3D_BENCH_DEVICE)" % os.environ["IS3D_BENCH_DEVICE"]
    return dict(value=total_units / elapsed, elapsed=elapsed, steps=steps, warmup=warmup, cfg=cfg, config=config,
                roofline=roofline, spec=spec, surf=surf, units_per_cell=units_per_cell, n_local=n_local)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (one per GPU); default 1, or WORLD_SIZE under a launcher (which must then agree)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="config2", choices=sorted(CONFIGS))
    ap.add_argument("--df-mode", type=int, default=0)
    ap.add_argument("--cells", type=int, default=0, help="override cells per GPU (weak) / total (strong)")
    ap.add_argument("--chosen", default="", help="override the chosen-species list (pikp, smash, urqmd)")
    ap.add_argument("--operation", type=int, default=1, choices=[0, 1],
                    help="1 continuous spectra (default, the BASELINE metric); 0 spacetime distributions dN/dX")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-per-species", action="store_true",
                    help="skip the second timing of the main workload with one integral per species (classes off)")
    ap.add_argument("--cpu-seconds", type=float, default=25.0)
    ap.add_argument("--tune", action="append", metavar="KEY=VALUE",
                    help="engine tuning knob (is3d_set_tuning), e.g. max_splits=128; repeatable")
    ap.add_argument("--north-star-steps", type=int, default=3,
                    help="timed passes of the north_star workload (config4: 10^6 3+1D cells, SMASH, RTA-CE, "
                         "sharded over the ranks) reported beside the main line; 0 skips it")
    ap.add_argument("--north-star-cpu-seconds", type=float, default=20.0,
                    help="CPU-leg sample length of the north_star workload (rank 0, N = 1); 0 skips that leg")
    args = ap.parse_args()

    world, spawn = resolve_world(args.gpus, os.environ)
    if spawn:
        sys.exit(spawn_ranks(world, sys.argv[1:]))
    rank = int(os.environ.get("RANK", 0))
    local_rank = int(os.environ.get("LOCAL_RANK", 0))

    import torch
    import torch.distributed as dist
    # rehearsal knobs for a 1-GPU box (never set by the driver): every rank on one device, gloo
    args.backend = os.environ.get("IS3D_BENCH_BACKEND", "nccl") if world > 1 else "none"
    local_rank = int(os.environ.get("IS3D_BENCH_DEVICE", local_rank))
    ndev = torch.cuda.device_count()
    if local_rank >= ndev:
        raise SystemExit("bench.py: rank %d needs GPU %d but %d GPU(s) are visible" % (rank, local_rank, ndev))
    if world > 1:
        dist.init_process_group(args.backend, init_method="env://")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    from is3d2_amd import _lib
    log("build_id %s" % _lib.build_id())
    m = run_workload(args, args.config, args.df_mode, args.steps, args.warmup, rank, world, local_rank, dev, dist)
    per_species = None
    if not args.no_per_species and m["config"]["species_integrated"] < m["config"]["species"]:
        # the same workload with one integral per species (integrand classes off): the same spectra to rounding
        # (< 1e-9, tests/test_gpu_classes.py), the kernel's per-species rate
        o = run_workload(args, args.config, args.df_mode, args.steps, 1, rank, world, local_rank, dev, dist,
                         classes=False)
        per_species = {"value": o["value"], "ms_per_step": 1e3 * o["elapsed"] / o["steps"], "steps": o["steps"],
                       "species_integrated": o["config"]["species_integrated"],
                       "kernel_ms": o["roofline"]["kernel_ms"],
                       "note": "same workload and clock rules with integrand classes off (is3d_set_species_classes(e, 0)): "
                               "every species integrated separately; equal to rounding (< 1e-9), tests/test_gpu_classes.py"}
    ns = None
    if args.north_star_steps > 0 and args.config != "config4" and args.operation == 1:
        n = run_workload(args, "config4", 0, args.north_star_steps, 1, rank, world, local_rank, dev, dist)
        ns = {"metric": "freezeout-cell-species-mom-points/sec", "value": n["value"],
              "unit": "cell-species-mom-points/s", "steps": n["steps"], "warmup": n["warmup"],
              "ms_per_step": 1e3 * n["elapsed"] / n["steps"], "scaling": n["cfg"]["scaling"], "config": n["config"],
              "roofline": n["roofline"],
              "note": "north_star target workload (BASELINE config 4) timed in this same run, same clock rules"}
        if rank == 0 and world == 1 and not args.no_cpu_baseline and args.north_star_cpu_seconds > 0:
            # north_star: ">= 10x the reference OpenMP continuous-spectra path on a 10^6-cell synthetic surface", the
            # CPU timed on this box's host cores in the same run -- the oracle (MomentumSpectra.cpp:32-415, df_mode 2)
            # on a cell prefix of the same 10^6-cell surface, extrapolated to the whole surface
            cb = cpu_baseline(n["spec"], n["surf"], n["units_per_cell"], n["n_local"], args.north_star_cpu_seconds, 1)
            cb["speedup"] = n["value"] / cb["value"]
            cb["gpu_s_per_pass"] = n["elapsed"] / n["steps"]
            ns["cpu_baseline"] = cb
    if rank == 0:
        res = {
            "metric": "freezeout-cell-species-mom-points/sec",
            "value": m["value"],
            "unit": "cell-species-mom-points/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * m["elapsed"] / args.steps,
            "higher_is_better": True,
            "scaling": m["cfg"]["scaling"],
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md 8d surface generator, seed 7+rank)",
            "config": m["config"],
            "roofline": m["roofline"],
        }
        if per_species is not None:
            res["per_species_integration"] = per_species
        if ns is not None:
            res["north_star"] = ns
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(m["spec"], m["surf"], m["units_per_cell"], m["n_local"], args.cpu_seconds,
                                               args.operation)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
