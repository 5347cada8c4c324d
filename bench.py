#!/usr/bin/env python3
"""Benchmark: reactor integrations/s for the GRI-Mech 3.0 CH4 ensemble (BASELINE.json metric).

One step = integrating one batch of N reactors (per GPU) from t=0 to tf=10 s with the
CVODE-style BDF (rtol 1e-6, atol 1e-10) on MI355X. Inputs are synthetic,
generated per rank for its own contiguous shard and resident in HBM before timing. Reactors are
independent, so ranks share no data during integration (weak scaling: N reactors per GPU); the
final states are all-gathered over RCCL once, after the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--n REACTORS_PER_GPU] [--config gri]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_PEAK_TFLOPS = 78.6   # MI355X fp64 dense (vector and matrix rate are equal for fp64)
CONFIGS = {
    "gri": dict(gas="grimech.dat", surf=None, n=100000, tf=10.0,
                name="C3 test/batch_ch4 GRI-Mech 3.0 CH4/O2/N2 ensemble (53 species, 325 reactions)"),
    "h2o2": dict(gas="h2o2.dat", surf=None, n=1000000, tf=10.0, name="C2 H2/O2 ignition ensemble (9 species)"),
    "surf": dict(gas=None, surf="ch4ni.xml", n=100000, tf=10.0, name="C4 surface-only Ni/CH4 ensemble"),
    "gas_surf": dict(gas="grimech.dat", surf="ch4ni.xml", n=100000, tf=10.0,
                     name="C5 GRI-Mech 3.0 gas + Ni surface ensemble (66 components, 325+42 reactions)"),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="gri", choices=sorted(CONFIGS))
    ap.add_argument("--n", type=int, default=0, help="reactors per GPU (default: the config's N)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic_gri.json"),
                    help="PMC summary (scripts/pmc_traffic.py) giving HBM bytes per reactor for roofline.traffic")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import _pkgload

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    pkg = _pkgload.load()
    from batchreactor_amd import ensemble, shard
    cfg = CONFIGS[args.config]
    lib = os.path.join(ROOT, "tests", "golden", "lib")
    mech = pkg.Mechanism.from_files(lib, gas_mech=cfg["gas"], surface_mech=cfg["surf"],
                                    gasphase=None if cfg["gas"] else "CH4 H2O H2 CO CO2 O2 N2".split())
    eng = pkg.Engine(mech, device=local)
    N = args.n or cfg["n"]
    start, _ = shard.shard_slice(rank, N)
    T, Asv, U0 = ensemble.make_inputs(mech, args.config, start, N)
    tf = np.full(N, cfg["tf"])
    dT = torch.from_numpy(T).to(dev)
    dA = torch.from_numpy(Asv).to(dev)
    dU0 = torch.from_numpy(U0).to(dev)
    dtf = torch.from_numpy(tf).to(dev)
    dU = torch.empty_like(dU0)
    dst = torch.zeros((N, pkg._lib.NSTAT), dtype=torch.float64, device=dev)
    stream = torch.cuda.current_stream(dev)

    def step():
        dU.copy_(dU0)
        eng.integrate_device(dT.data_ptr(), dA.data_ptr(), dU.data_ptr(), dtf.data_ptr(), dst.data_ptr(), N,
                             stream.cuda_stream)

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
    flops = ensemble.algorithmic_flops(mech, stats)
    kernel_ms = float(np.mean(kms))
    achieved = flops / (kernel_ms * 1e-3) / 1e12

    # HBM bytes per launch from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this
    # kernel on this workload (bytes per reactor x reactors in this launch); None if absent
    traffic = None
    if args.config == "gri" and os.path.exists(args.traffic):
        with open(args.traffic) as fh:
            traffic = json.load(fh)["bytes_per_reactor"] * N

    gather_ms = None
    if world > 1:   # the single result gather over RCCL/xGMI (outside the timed region)
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        shard.gather_ensemble(dU, dst, dist)
        torch.cuda.synchronize()
        gather_ms = (time.perf_counter() - g0) * 1e3

    cpu = None
    parity = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu, parity = cpu_baseline(mech, T, Asv, U0, tf, dU.cpu().numpy(), stats["status"], args.cpu_seconds)

    if rank == 0:
        total = N * world
        per_step = elapsed / args.steps
        line = {
            "metric": "reactor integrations/sec (CH4 GRI ensemble)" if args.config == "gri"
            else f"reactor integrations/sec ({args.config} ensemble)",
            "value": total / per_step,
            "unit": "reactors/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": per_step * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (splitmix64 seed 20250711, SURVEY.md 8(d))",
            "config": {"workload": cfg["name"], "reactors_per_gpu": N, "total_reactors": total,
                       "tf_s": cfg["tf"], "rtol": 1e-6, "atol": 1e-10, "parallelism": f"ensemble dp{world}"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / FP64_PEAK_TFLOPS, "traffic": traffic,
                         "traffic_unit": "B per launch (PMC, profiles/traffic_gri.json)",
                         "kernel": eng.kernel_name, "kernel_ms": kernel_ms,
                         "algorithmic_flop_per_launch": flops},
            "cpu_baseline": cpu,
            "solver": {"failed": nbad, "status_counts": {str(int(k)): int(np.sum(stats["status"] == k))
                                                         for k in np.unique(stats["status"])}, "mean_steps": float(stats["nsteps"].mean()),
                       "mean_nfe": float(stats["nfe"].mean()), "mean_nje": float(stats["nje"].mean()),
                       "mean_nsetups": float(stats["nsetups"].mean())},
            "parity_vs_oracle_err": parity,
            "gather_ms": gather_ms,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(mech, T, Asv, U0, tf, U_gpu, gpu_status, seconds):
    """The C CPU oracle (CVODE restatement, analytic Jacobian, OpenMP over reactors) on a bounded
    sample of the same workload; also checks the GPU results of that sample against it."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    lib = os.path.join(ROOT, "tests", "golden", "lib")
    om = oracle.Mech(os.path.join(lib, "grimech.dat") if mech.nrg and mech.ng > 9 else
                     (os.path.join(lib, "h2o2.dat") if mech.nrg else None),
                     os.path.join(lib, "therm.dat"),
                     os.path.join(lib, "ch4ni.xml") if mech.ns else None,
                     gas_species=None if mech.nrg else mech.gas_species)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, 64))
    k = min(threads, len(T))
    t0 = time.perf_counter()
    om.integrate_batch(T[:k], Asv[:k], U0[:k], tf[:k], analytic_jac=True, nthreads=threads)
    dt = time.perf_counter() - t0
    per = dt / k * threads
    k = int(max(k, min(len(T), seconds / max(per, 1e-6) * threads)))
    t0 = time.perf_counter()
    Uo, sto, bad = om.integrate_batch(T[:k], Asv[:k], U0[:k], tf[:k], analytic_jac=True, nthreads=threads)
    dt = time.perf_counter() - t0
    # parity metric of tests/test_gpu_parity.py: max |du| / (1e-4 |u| + 100 atol), pass <= 1,
    # over the reactors both sides integrated successfully
    ok = np.array([s["status"] == 0 for s in sto]) & (gpu_status[:k] == 0)
    if ok.any():
        err = np.max(np.abs(U_gpu[:k][ok] - Uo[ok]) / (1e-4 * np.abs(Uo[ok]) + 1e-8), axis=1)
        rel = {"metric": "max_k |u_gpu-u_orc| / (1e-4 |u_orc| + 100 atol) per reactor", "reactors": int(ok.sum()),
               "failed_either": int((~ok).sum()), "median": float(np.median(err)),
               "p99": float(np.percentile(err, 99)), "max": float(err.max()),
               "frac_le_1": float(np.mean(err <= 1.0)), "frac_le_10": float(np.mean(err <= 10.0))}
    else:
        rel = None
    return ({"value": k / dt, "unit": "reactors/s", "cores": threads, "kind": "port",
             "sample": f"first {k} reactors of the same synthetic workload, C oracle (oracle/oracle.c, "
                       f"CVODE restatement, analytic Jacobian), OpenMP {threads} threads, {dt:.1f} s"}, rel)


if __name__ == "__main__":
    main()
