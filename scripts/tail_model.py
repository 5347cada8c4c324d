"""Strong-scaling tail model: list scheduling of the measured per-reactor wall
times onto the persistent grid's slots, per GPU count, for the bench's contiguous shards.

Input: scripts/dump_costs.py output (per-reactor br_stats.cyc_total, 100 MHz wall clock, measured at
full occupancy on one MI355X). Each GPU runs its shard on S resident slots (waves); a slot takes the
next reactor index from the work counter when its reactor finishes (k_integrate's persistent grid).
Makespan per GPU = the last slot's finish time; efficiency(g) = T(1) / (g T(g)). Variants: reactor
order as issued (index order), longest-first with the measured costs (the bound any cost-aware
ordering could reach), and longest-first by a predictor fitted on the inputs.
Usage: python scripts/tail_model.py gpurun_out/costs_gri.npz [slots] > profiles/r04_tail_model_gri.json"""
import heapq
import json
import os
import sys

import numpy as np


def makespan(costs, slots, beta=0.0, per_simd=4):
    """List scheduling of `costs` (s at full occupancy) onto `slots` (per_simd waves per SIMD, slot i
    on SIMD i % (slots / per_simd)); once the work counter is empty each SIMD finishes its remaining
    reactors under processor sharing: with w waves left a wave runs (per_simd / w)^beta times its
    full-occupancy speed (beta = 0: no speed-up; 1: the SIMD's throughput stays constant)."""
    nsimd = max(1, slots // per_simd)
    h = [(0.0, i) for i in range(slots)]
    heapq.heapify(h)
    end = [0.0] * slots
    for c in costs:
        t, i = heapq.heappop(h)
        end[i] = t + c
        heapq.heappush(h, (t + c, i))
    # the counter runs dry at the last start: t_last; each slot then has end[i] - t_last left
    t_last = max(end[i] - 0.0 for i in range(slots)) if len(costs) <= slots else None
    starts = sorted(end)
    if len(costs) <= slots:
        t_last = 0.0
    else:
        # time of the last assignment = the (len(costs) - slots)-th earliest completion before it
        t_last = _last_start(costs, slots)
    rem = [[] for _ in range(nsimd)]
    for i in range(slots):
        r = end[i] - t_last
        if r > 0:
            rem[i % nsimd].append(r)
    fin = 0.0
    for rs in rem:
        rs.sort()
        t, done, w = 0.0, 0.0, len(rs)
        for k, r in enumerate(rs):   # processor sharing: the smallest remaining finishes first
            f = (per_simd / w) ** beta if w else 1.0
            t += (r - done) / f
            done = r
            w -= 1
        fin = max(fin, t)
    return t_last + fin


def _last_start(costs, slots):
    h = [0.0] * slots
    t = 0.0
    for c in costs:
        t = heapq.heappop(h)
        heapq.heappush(h, t + c)
    return t


def shards(total, world):
    base, extra = divmod(total, world)
    out, s = [], 0
    for r in range(world):
        n = base + (1 if r < extra else 0)
        out.append((s, s + n))
        s += n
    return out


def main():
    d = np.load(sys.argv[1])
    beta = float(os.environ.get("TAIL_BETA", "0"))
    cost = d["cyc_total"] * 10e-9            # s (100 MHz wall clock)
    N = len(cost)
    slots = int(sys.argv[2]) if len(sys.argv) > 2 else None
    if slots is None:
        launch = eval(str(d["launch"]))      # dict literal written by dump_costs.py
        slots = int(launch["waves_per_cu"]) * int(d["ncu"])
    T = d["T"]
    # predictor: mean cost per 20-K temperature bin (the ensemble's dominant cost variable)
    bins = np.clip(((T - T.min()) / 20.0).astype(int), 0, None)
    mean_bin = np.bincount(bins, weights=cost) / np.maximum(np.bincount(bins), 1)
    pred = mean_bin[bins]
    out = {"source": sys.argv[1], "kernel": str(d["kernel"]), "reactors": N, "slots_per_gpu": slots,
           "measured_kernel_ms_1gpu": float(d["kernel_ms"]),
           "cost_s": {"mean": float(cost.mean()), "p50": float(np.median(cost)), "p99": float(np.percentile(cost, 99)),
                      "max": float(cost.max()), "sum": float(cost.sum())},
           "processor_sharing_beta": beta,
           "lower_bound_ms_1gpu": float(max(cost.sum() / slots, cost.max()) * 1e3),
           "gpus": {}}
    t1 = None
    for g in (1, 2, 4, 8):
        row = {}
        for name, key in (("index_order", None), ("longest_first_measured", cost), ("longest_first_predicted", pred)):
            ms = []
            for a, b in shards(N, g):
                c = cost[a:b]
                if key is not None:
                    c = c[np.argsort(-key[a:b], kind="stable")]
                ms.append(makespan(c, slots, beta))
            row[name] = {"makespan_ms": max(ms) * 1e3, "per_gpu_ms": [m * 1e3 for m in ms]}
        if g == 1:
            t1 = {k: v["makespan_ms"] for k, v in row.items()}
        for k, v in row.items():
            v["efficiency_vs_1gpu_same_order"] = t1[k] / (g * v["makespan_ms"])
            v["efficiency_vs_1gpu_index_order"] = t1["index_order"] / (g * v["makespan_ms"])
            v["ideal_ms"] = cost.sum() / (g * slots) * 1e3
        out["gpus"][str(g)] = row
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
