#!/usr/bin/env python3
"""Benchmark: reactor integrations/s for the GRI-Mech 3.0 CH4 ensemble (BASELINE.json metric).

One step = integrating the ensemble from t=0 to tf=10 s with the CVODE-style BDF (rtol 1e-6,
atol 1e-10) on MI355X. Inputs are synthetic, generated per rank for its own
contiguous shard and resident in HBM before timing. Reactors are independent, so ranks share no
data during integration; at N > 1 the final states and counters are all-gathered over RCCL once per
step, inside the timed region. `value_incl_h2d_d2h` repeats one step with host-resident inputs and
the results copied back (the PCIe-inclusive rate of BASELINE.md's definition).

Scaling (BASELINE.json: "ensemble of 1e5 reactors, sharded over 1/2/4/8 GPUs"):
  --scaling strong (default): the config's total N (1e5 for GRI) is split into contiguous slices
                              over the ranks;
  --scaling weak:             every rank integrates N reactors (--n).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config gri|h2o2|surf|gas_surf]
                  [--scaling strong|weak] [--n N] [--no-cpu] [--no-phase] [--dry-run]

Launch: under torch.distributed.run (WORLD_SIZE set) every process is one rank. Without a launcher,
--gpus N > 1 makes this process spawn N rank processes (RANK / LOCAL_RANK / WORLD_SIZE, rendezvous on
127.0.0.1) before it touches any GPU, wait for them and exit with the first non-zero status; a rank
whose process group reports another world size than --gpus exits non-zero. --dry-run runs the same
launch and sharding over gloo on the CPU without touching a GPU (tests/test_shard.py).
"""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 dense (vector; the fp64 matrix rate is the same)
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_ACHIEVABLE_GBS = 6300.0   # achievable HBM read rate (MI355X_MICROARCH.md, HBM section)
# parity samples of the cpu_baseline leg, fixed per config so the bench's parity windows are
# deterministic: (analytic-Jacobian sample = the timed CPU sample, DQ-Jacobian sample); the first K
# reactors of the workload. scripts/parity_outliers.py derives tests/parity_bands.py's bounds from the
# oracle's own spread on exactly these reactors.
PARITY_SAMPLE = {"gri": (8000, 2000), "gas_surf": (3000, 1000), "h2o2": (50000, 2000), "surf": (50000, 2000)}
CONFIGS = {
    "gri": dict(gas="grimech.dat", surf=None, n=100000, tf=10.0,
                name="C3 test/batch_ch4 GRI-Mech 3.0 CH4/O2/N2 ensemble (53 species, 325 reactions)"),
    "h2o2": dict(gas="h2o2.dat", surf=None, n=1000000, tf=10.0, name="C2 H2/O2 ignition ensemble (9 species)"),
    "surf": dict(gas=None, surf="ch4ni.xml", n=100000, tf=10.0, name="C4 surface-only Ni/CH4 ensemble"),
    "gas_surf": dict(gas="grimech.dat", surf="ch4ni.xml", n=100000, tf=10.0,
                     name="C5 GRI-Mech 3.0 gas + Ni surface ensemble (66 components, 325+42 reactions)"),
}


def make_mech(pkg, config):
    cfg = CONFIGS[config]
    lib = os.path.join(ROOT, "tests", "golden", "lib")
    return pkg.Mechanism.from_files(lib, gas_mech=cfg["gas"], surface_mech=cfg["surf"],
                                    gasphase=None if cfg["gas"] else "CH4 H2O H2 CO CO2 O2 N2".split())


def ensemble_inputs(pkg, mech, config, count, start=0):
    """T, Asv, U0 of reactors [start, start + count) of the config's synthetic workload"""
    from batchreactor_amd import ensemble
    return ensemble.make_inputs(mech, config, start, count)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="gri", choices=sorted(CONFIGS))
    ap.add_argument("--scaling", default="strong", choices=("strong", "weak"))
    ap.add_argument("--n", type=int, default=0, help="total reactors (strong) or reactors per GPU (weak); "
                                                     "default: the config's N")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-phase", action="store_true", help="skip the rate+Jacobian phase split (diag build)")
    ap.add_argument("--no-pcie", action="store_true", help="skip the PCIe-inclusive extra step (counter runs: "
                                                          "one integrator dispatch per timed step only)")
    ap.add_argument("--dry-run", action="store_true", help="launch + sharding over gloo, no GPU (CPU test)")
    ap.add_argument("--phase-only", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.phase_only:
        return phase_split(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)   # (no torch import, no GPU call in this process)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        return dry_run(args, dist, world, rank)
    import _pkgload
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        if dist.get_world_size() != args.gpus:   # the line's n_gpus is the world RCCL reports
            print(f"bench.py: --gpus {args.gpus} but the process group has {dist.get_world_size()} ranks",
                  file=sys.stderr)
            dist.destroy_process_group()
            return 2
        world = dist.get_world_size()
    elif args.gpus != 1:
        print(f"bench.py: --gpus {args.gpus} with WORLD_SIZE=1", file=sys.stderr)
        return 2
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    pkg = _pkgload.load()
    from batchreactor_amd import ensemble, shard
    cfg = CONFIGS[args.config]
    mech = make_mech(pkg, args.config)
    eng = pkg.Engine(mech, device=local)
    if args.scaling == "strong":
        total = args.n or cfg["n"]
        start, stop = shard.shard_range(rank, world, total)
    else:
        per = args.n or cfg["n"]
        total = per * world
        start, stop = shard.shard_slice(rank, per)
    N = stop - start
    T, Asv, U0 = ensemble.make_inputs(mech, args.config, start, N)
    tf = np.full(N, cfg["tf"])
    dT = torch.from_numpy(T).to(dev)
    dA = torch.from_numpy(Asv).to(dev)
    dU0 = torch.from_numpy(U0).to(dev)
    dtf = torch.from_numpy(tf).to(dev)
    dU = torch.empty_like(dU0)
    dst = torch.zeros((N, pkg._lib.NSTAT), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)

    gathered = [None]

    def step():
        dU.copy_(dU0)
        eng.integrate_device(dT.data_ptr(), dA.data_ptr(), dU.data_ptr(), dtf.data_ptr(), dst.data_ptr(), N,
                             stream.cuda_stream)
        if world > 1:   # the single RCCL all-gather of final states + solver counters (north_star)
            gathered[0] = shard.gather_ensemble(dU, dst, dist, total if args.scaling == "strong" else None)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    kms = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        kms.append(eng.last_kernel_ms())   # HIP events on the launch stream; syncs that stream
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = shard.max_over_ranks(time.perf_counter() - t0, dist if world > 1 else None, dev)

    st = dst.cpu().numpy()
    stats = {k: st[:, i] for i, k in enumerate(pkg.STAT_FIELDS)}
    nbad = int(np.sum(stats["status"] != 0))
    nbad_all = nbad
    if world > 1:   # failures summed over ranks (outside the timed region)
        t_bad = torch.tensor([float(nbad)], dtype=torch.float64, device=dev)
        dist.all_reduce(t_bad)
        nbad_all = int(t_bad.item())
    flops = ensemble.algorithmic_flops(mech, stats)
    kernel_ms = float(np.mean(kms))
    achieved = flops / (kernel_ms * 1e-3) / 1e12
    # algorithmic HBM bytes per launch: inputs (T, Asv, tf, u0[n]) read, u[n] + stats written
    alg_bytes = N * 8.0 * ((3 + mech.n) + (mech.n + pkg._lib.NSTAT))

    # measured L2-fabric-side bytes per reactor of this kernel (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE
    # passes, scripts/pmc_traffic.py -> profiles/rNN_traffic_<config>.json); Infinity-Cache hits are
    # counted there, so it is not HBM traffic. The DRAM-destined view and the HBM bound come from
    # scripts/pmc_dram.sh -> profiles/rNN_dram_<config>.json.
    def newest(kind):
        for rnd in ("r06", "r05", "r04", "r03", "r02"):
            cand = os.path.join(ROOT, "profiles", f"{rnd}_{kind}_{args.config}.json")
            if os.path.exists(cand):
                with open(cand) as fh:
                    return json.load(fh), os.path.relpath(cand, ROOT)
        return None, None
    traffic = None
    tj, traffic_src = newest("traffic")
    if tj:
        traffic = tj["bytes_per_reactor"] * N
    dj, dram_src = newest("dram")

    gather_ms = None
    if world > 1:   # the gather alone (it is also inside every timed step above)
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        shard.gather_ensemble(dU, dst, dist, total if args.scaling == "strong" else None)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    # PCIe-inclusive rate (the integrate call including H2D/D2H): one more step with
    # the inputs in pinned host memory and the final states + counters copied back to it. Reported
    # beside `value` (which, per the bench contract, starts with the inputs resident in HBM).
    pcie_s = None
    if not args.no_pcie:
        pcie_s = pcie_step(torch, dist, world, dev, (T, Asv, U0, tf), (dT, dA, dU0, dtf), dU, dst, step, gathered, shard)

    cpu = parity = phases = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu, parity = cpu_baseline(mech, args.config, T, Asv, U0, tf, dU.cpu().numpy(), stats["status"],
                                   args.cpu_seconds, eng)
    if rank == 0 and world == 1 and not args.no_phase:
        phases = run_phase_split(args.config)

    if rank == 0:
        per_step = elapsed / args.steps
        kernel_s = kernel_ms * 1e-3
        roof = {"bound": "fp64 valu", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                "traffic_unit": "B per launch at the L2 memory side (PMC FETCH_SIZE x2 + WRITE_SIZE, per reactor x N; "
                                "Infinity-Cache hits included, not HBM bytes: see hbm.dram_*)",
                "traffic_source": traffic_src, "kernel": eng.kernel_name, "kernel_ms": kernel_ms,
                "launch": eng.launch_info,
                "algorithmic_flop_per_launch": flops,
                "hbm": {"algorithmic_bytes_per_launch": alg_bytes,
                        "algorithmic_GBs": alg_bytes / kernel_s / 1e9,
                        "peak_GBs": HBM_PEAK_GBS,
                        # everything the L2 sent to the fabric: Infinity-Cache (MALL) hits included
                        "l2_fabric_GBs": (traffic / kernel_s / 1e9) if traffic else None,
                        "l2_fabric_frac_of_hbm_peak": (traffic / kernel_s / 1e9 / HBM_PEAK_GBS) if traffic else None,
                        "l2_fabric_source": traffic_src}}
        if dj:
            dram_b = dj["dram_destined"]["bytes_per_reactor"] * N
            roof["hbm"].update({
                # requests addressed to DRAM, counted before the Infinity Cache serves them (no gfx950
                # counter separates MALL hits), so an upper bound of HBM bytes
                "dram_destined_GBs": dram_b / kernel_s / 1e9,
                "dram_destined_frac_of_hbm_peak": dram_b / kernel_s / 1e9 / HBM_PEAK_GBS,
                # HBM cannot have moved more than its achievable rate x this kernel's time: the rest of
                # the fabric-side bytes were Infinity-Cache hits
                "hbm_achievable_GBs": HBM_ACHIEVABLE_GBS,
                "min_infinity_cache_share": (max(0.0, 1.0 - HBM_ACHIEVABLE_GBS * 1e9 * kernel_s / traffic)
                                             if traffic else None),
                "dram_source": dram_src})
        if phases:
            # the north_star's rate+Jacobian figure: their FLOPs over the kernel time spent in them
            f = ensemble.flop_model(mech)
            rj_flops = float(np.sum(stats["nfe"]) * f["rhs"] + np.sum(stats["nje"]) * f["jac"])
            share = phases["rhs_share"] + phases["jac_share"]
            rj = rj_flops / (kernel_s * share) / 1e12 if share > 0 else None
            roof["rate_jacobian"] = {"achieved": rj, "frac": rj / FP64_PEAK_TFLOPS if rj else None,
                                     "unit": "TFLOP/s", "flop_per_launch": rj_flops, "kernel_time_share": share,
                                     "phase_shares": phases, "source": "diagnostic build (libbrhip_diag.so) "
                                     "per-phase shader clocks on a sample of the same workload"}
        ok_all = total - nbad_all
        line = {
            "metric": "reactor integrations/sec (CH4 GRI ensemble)" if args.config == "gri"
            else f"reactor integrations/sec ({args.config} ensemble)",
            # successful integrations only: a reactor that stops with a CVODE failure status is
            # not counted (the work it did still costs time)
            "value": ok_all / per_step,
            "unit": "reactors/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1e3,
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 seed 20250711, SURVEY.md 8(d))",
            "config": {"workload": cfg["name"], "total_reactors": total, "reactors_rank0": N,
                       "tf_s": cfg["tf"], "rtol": 1e-6, "atol": 1e-10, "parallelism": f"ensemble dp{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "solver": {"failed_all_ranks": nbad_all, "attempted": total, "failed": nbad, "status_counts": {str(int(k)): int(np.sum(stats["status"] == k))
                                                         for k in np.unique(stats["status"])},
                       "mean_steps": float(stats["nsteps"].mean()), "mean_nfe": float(stats["nfe"].mean()),
                       "mean_nje": float(stats["nje"].mean()), "mean_nsetups": float(stats["nsetups"].mean()),
                       "mean_t_ign": float(np.nanmean(stats["t_ign"])) if np.any(np.isfinite(stats["t_ign"])) else None},
            "parity_vs_oracle": parity,
            "gather_ms": gather_ms,
            "gather_in_timed_region": world > 1,
            "value_incl_h2d_d2h": (ok_all / pcie_s) if pcie_s else None,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def spawn_ranks(n):
    """One child process per rank (the driver's torch.distributed.run launch, done here): each gets
    RANK = LOCAL_RANK = r, WORLD_SIZE = n and a 127.0.0.1 rendezvous, runs this script with the same
    arguments, and rank 0 prints the line. Returns the first non-zero child status (0 if all pass)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def dry_run(args, dist, world, rank):
    """--dry-run: the rank layout and shard slices over gloo on the CPU (no GPU, no integration);
    rank 0 prints {"n_gpus": world size from the process group, "slices": [[start, stop], ...]}."""
    import importlib.util   # the package's pure-Python shard module alone (no library load)
    spec = importlib.util.spec_from_file_location("br_shard", os.path.join(ROOT, "batchreactor.jl_amd", "shard.py"))
    shard = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(shard)
    if world > 1:
        dist.init_process_group("gloo")
        world = dist.get_world_size()
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the process group has {world} ranks", file=sys.stderr)
            dist.destroy_process_group()
            return 2
    elif args.gpus != 1:
        print(f"bench.py: --gpus {args.gpus} with WORLD_SIZE=1", file=sys.stderr)
        return 2
    cfg = CONFIGS[args.config]
    if args.scaling == "strong":
        total = args.n or cfg["n"]
        mine = list(shard.shard_range(rank, world, total))
    else:
        total = (args.n or cfg["n"]) * world
        mine = list(shard.shard_slice(rank, args.n or cfg["n"]))
    slices = [None] * world
    if world > 1:
        dist.all_gather_object(slices, mine)
        dist.destroy_process_group()
    else:
        slices = [mine]
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": world, "scaling": args.scaling, "total_reactors": total,
                          "slices": slices}), flush=True)
    return 0


def pcie_step(torch, dist, world, dev, host_in, dev_in, dU, dst, step, gathered, shard):
    """One more step with the inputs in pinned host memory and the final states + counters copied
    back to it (PCIe-inclusive wall time, max over ranks)."""
    hT, hA, hU0, htf = (torch.from_numpy(a).pin_memory() for a in host_in)
    dT, dA, dU0, dtf = dev_in
    hU = torch.empty_like(hU0).pin_memory()
    hst = torch.empty(dst.shape, dtype=dst.dtype).pin_memory()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    p0 = time.perf_counter()
    dT.copy_(hT, non_blocking=True); dA.copy_(hA, non_blocking=True); dtf.copy_(htf, non_blocking=True)
    dU0.copy_(hU0, non_blocking=True)
    step()
    if world > 1:   # every rank receives the gathered ensemble
        for t in gathered[0]:
            t.cpu()
    else:
        hU.copy_(dU, non_blocking=True); hst.copy_(dst, non_blocking=True)
    torch.cuda.synchronize()
    return shard.max_over_ranks(time.perf_counter() - p0, dist if world > 1 else None, dev)


def run_phase_split(config):
    """Per-phase kernel-time shares from the diagnostic build, in a child process (its own
    library instance); a sample of the same workload."""
    env = dict(os.environ)
    env["BRHIP_LIB"] = os.path.join(ROOT, "batchreactor.jl_amd", "libbrhip_diag.so")
    if not os.path.exists(env["BRHIP_LIB"]):
        return None
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--phase-only", "--config", config],
                           env=env, capture_output=True, text=True, timeout=300)
        return json.loads(r.stdout.strip().splitlines()[-1])
    except Exception:
        return None


def phase_split(args):
    import _pkgload
    pkg = _pkgload.load()
    from batchreactor_amd import ensemble
    mech = make_mech(pkg, args.config)
    N = min(20000, CONFIGS[args.config]["n"])
    T, Asv, U0 = ensemble.make_inputs(mech, args.config, 0, N)
    U, st = pkg.Engine(mech).integrate(T, Asv, U0, CONFIGS[args.config]["tf"])
    clk = float(np.sum(st["cyc_clk"]))
    out = {f"{ph}_share": float(np.sum(st["cyc_" + ph]) / clk) for ph in ("rhs", "jac", "lu", "sol", "ctl")}
    out["reactors"] = N
    print(json.dumps(out))


def cpu_baseline(mech, config, T, Asv, U0, tf, U_gpu, gpu_status, seconds, eng):
    """The C CPU oracle (CVODE restatement, analytic Jacobian, OpenMP over reactors) on a bounded
    sample of the same workload, all threads and one thread; also checks the GPU results of that
    sample against it: per reactor at t = tf, and per ignition window at the 28 output times of
    tests/test_gpu_parity.py against that test's per-case bounds (tests/parity_bands.py; the GPU
    states there come from one more, untimed integration of the sample with dense output)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle
    import parity_bands as PB
    cfg = CONFIGS[config]
    lib = os.path.join(ROOT, "tests", "golden", "lib")
    om = oracle.Mech(os.path.join(lib, cfg["gas"]) if cfg["gas"] else None, os.path.join(lib, "therm.dat"),
                     os.path.join(lib, cfg["surf"]) if cfg["surf"] else None,
                     gas_species=None if cfg["gas"] else mech.gas_species)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    k = min(threads, len(T))
    t0 = time.perf_counter()
    om.integrate_batch(T[:k], Asv[:k], U0[:k], tf[:k], analytic_jac=True, nthreads=threads)
    dt = time.perf_counter() - t0
    per = dt / k * threads
    k = min(len(T), PARITY_SAMPLE[config][0])   # the fixed parity sample (deterministic windows)
    t0 = time.perf_counter()   # (dense output at the test's 28 times: the same step sequence)
    Uo, sto, bad, Yo = om.integrate_batch(T[:k], Asv[:k], U0[:k], tf[:k], analytic_jac=True, nthreads=threads,
                                          tout=PB.OUT_T)
    dt = time.perf_counter() - t0
    k1 = int(max(1, min(k, 0.25 * seconds / max(per, 1e-6))))      # single thread, a quarter of the budget
    t1 = time.perf_counter()
    om.integrate_batch(T[:k1], Asv[:k1], U0[:k1], tf[:k1], analytic_jac=True, nthreads=1)
    dt1 = time.perf_counter() - t1
    ok = np.array([s["status"] == 0 for s in sto]) & (gpu_status[:k] == 0)
    if ok.any():
        err = np.max(np.abs(U_gpu[:k][ok] - Uo[ok]) / (1e-4 * np.abs(Uo[ok]) + 1e-8), axis=1)
        rel = {"metric": "max_k |u_gpu-u_orc| / (1e-4 |u_orc| + 100 atol) per reactor at t = tf (post-ignition: "
                         "rounding-level differences grow through ignition, see tests/test_gpu_parity.py bands)",
               "reactors": int(ok.sum()), "failed_either": int((~ok).sum()), "median": float(np.median(err)),
               "p99": float(np.percentile(err, 99)), "max": float(err.max()),
               "frac_le_1": float(np.mean(err <= 1.0)), "frac_le_30": float(np.mean(err <= 30.0))}
        # per ignition window, the test's metric and bounds (the bench integrates with the analytic J)
        _, stg = eng.integrate(T[:k], Asv[:k], U0[:k], tf[:k], tout=PB.OUT_T)
        okw = ok & (stg["status"] == 0)
        W = np.array([PB.band_errors(stg["yout"][i], Yo[i], sto[i]["t_ign"]) for i in np.nonzero(okw)[0]])
        bnd = PB.BOUNDS[(config, False)]
        rel["windows"] = {
            "metric": "max over the 28 output times of tests/test_gpu_parity.py in each window of t/t_ign "
                      "(pre < 0.5, front 0.5..2, post >= 2) of max_k |Y_gpu-Y_orc| / (1e-4 |Y_orc| + 100 atol)",
            "reactors": int(okw.sum()), "bounds": list(bnd[:3]),
            "max": W.max(0).tolist(), "p99": np.percentile(W, 99, axis=0).tolist(),
            "median": np.median(W, axis=0).tolist(),
            "frac_within_bounds": float(np.mean(np.all(W <= np.array(bnd[:3]), axis=1)))}
        # the same windows with CVODE's DQ Jacobian on both sides (the reference's own setting: the
        # wavefront engine's dq_jacobian path against the oracle's cvLsDenseDQJac), bounded sample
        if (config, True) in PB.BOUNDS:
            kd = min(k, PARITY_SAMPLE[config][1])
            t2 = time.perf_counter()
            _, stq, _, Yq = om.integrate_batch(T[:kd], Asv[:kd], U0[:kd], tf[:kd], analytic_jac=False,
                                               nthreads=threads, tout=PB.OUT_T)
            dt2 = time.perf_counter() - t2
            _, sgq = eng.integrate(T[:kd], Asv[:kd], U0[:kd], tf[:kd], tout=PB.OUT_T, dq_jacobian=True)
            okq = np.array([s["status"] == 0 for s in stq]) & (sgq["status"] == 0)
            Wq = np.array([PB.band_errors(sgq["yout"][i], Yq[i], stq[i]["t_ign"]) for i in np.nonzero(okq)[0]])
            bq = PB.BOUNDS[(config, True)]
            rel["windows_dq"] = {
                "metric": rel["windows"]["metric"] + "; both sides with CVODE's difference-quotient Jacobian",
                "reactors": int(okq.sum()), "failed_either": int((~okq).sum()), "bounds": list(bq[:3]),
                "max": Wq.max(0).tolist(), "p99": np.percentile(Wq, 99, axis=0).tolist(),
                "median": np.median(Wq, axis=0).tolist(),
                "frac_within_bounds": float(np.mean(np.all(Wq <= np.array(bq[:3]), axis=1))),
                "oracle_s": dt2}
    else:
        rel = None
    return ({"value": k / dt, "unit": "reactors/s", "cores": threads, "kind": "port",
             "single_thread_value": k1 / dt1,
             "sample": f"first {k} reactors of the same synthetic workload ({k1} for the single-thread figure), "
                       f"C oracle (oracle/oracle.c, CVODE restatement, analytic Jacobian), OpenMP {threads} "
                       f"threads, {dt:.1f} s; 1 thread {dt1:.1f} s"}, rel)


if __name__ == "__main__":
    sys.exit(main() or 0)
