"""Per-reactor cost dump for the strong-scaling tail model (scripts/tail_model.py): integrates the
bench workload of one config on cuda:0 once (warm-up run first) and saves each reactor's wall clock
cycles (br_stats.cyc_total: the wave's s_memrealtime span, 100 MHz), accepted steps and inputs.
Usage: python scripts/dump_costs.py gri 100000 gpurun_out/costs_gri.npz"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    config, N, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    import torch
    import _pkgload
    import bench
    pkg = _pkgload.load()
    from batchreactor_amd import ensemble
    mech = bench.make_mech(pkg, config)
    eng = pkg.Engine(mech)
    T, Asv, U0 = ensemble.make_inputs(mech, config, 0, N)
    tf = np.full(N, bench.CONFIGS[config]["tf"])
    for _ in range(2):
        U, st = eng.integrate(T, Asv, U0, tf)
    ms = eng.last_kernel_ms()
    np.savez(out, cyc_total=st["cyc_total"], nsteps=st["nsteps"], status=st["status"], T=T,
             kernel_ms=ms, kernel=eng.kernel_name, launch=str(eng.launch_info),
             ncu=torch.cuda.get_device_properties(0).multi_processor_count)
    print(config, N, eng.kernel_name, f"{ms:.1f} ms", eng.launch_info)


if __name__ == "__main__":
    main()
