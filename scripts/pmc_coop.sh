#!/bin/bash
# Memory-side traffic and SQ counters of the cooperative LU + solve experiment (scripts/exp_coop.py): FETCH_SIZE
# (x2, the gfx950 correction of MI355X_MICROARCH.md) and WRITE_SIZE per unit (one LU + NSOLVE
# solves) for every kernel launch, in launch order (base, coop panel capped / uncapped, coop step
# capped / uncapped; each launched twice, the second is the timed one).
#   bash scripts/pmc_coop.sh [N] [REPS] [NSOLVE]   -> gpurun_out/pmc_coop.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
N=${1:-65536}; R=${2:-8}; S=${3:-9}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pcoop_f -o run -- python3 scripts/exp_coop.py $N $R $S pmcf > gpurun_out/pcoop_f.log 2>&1 || { echo "fetch pass failed"; tail -5 gpurun_out/pcoop_f.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pcoop_w -o run -- python3 scripts/exp_coop.py $N $R $S pmcw > gpurun_out/pcoop_w.log 2>&1 || { echo "write pass failed"; tail -5 gpurun_out/pcoop_w.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/pcoop_s -o run -- python3 scripts/exp_coop.py $N $R $S pmcs > gpurun_out/pcoop_s.log 2>&1 || { echo "sq pass failed"; tail -5 gpurun_out/pcoop_s.log; exit 1; }
python3 - "$N" "$R" "$S" <<'PY'
import csv, glob, json, sys
N, R, S = map(int, sys.argv[1:4])
def per_dispatch(pattern, name):
    d = {}
    for f in glob.glob(pattern, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if ("k_base" in k or "k_coop" in k) and r["Counter_Name"] == name:
                key = int(r["Dispatch_Id"])
                d.setdefault(key, [k, 0.0])
                d[key][1] += float(r["Counter_Value"])
    return [d[k] for k in sorted(d)]
fe = per_dispatch("gpurun_out/pcoop_f/**/*counter_collection.csv", "FETCH_SIZE")
wr = per_dispatch("gpurun_out/pcoop_w/**/*counter_collection.csv", "WRITE_SIZE")
names = ["base_wavefront", "coop_panel_16w_per_cu", "coop_panel_uncapped", "coop_step_16w_per_cu", "coop_step_uncapped"]
units = N * R
out = {"units": units, "nsolve": S, "note": "bytes per unit (one LU + nsolve solves); FETCH_SIZE x2 (gfx950), KiB -> B; timed launch of each mode", "modes": {}}
for i, nm in enumerate(names):
    j = 2 * i + 1
    if j < len(fe) and j < len(wr):
        rd = 2.0 * fe[j][1] * 1024.0 / units
        wb = wr[j][1] * 1024.0 / units
        out["modes"][nm] = {"kernel": fe[j][0][:60], "read_bytes_per_unit": rd, "write_bytes_per_unit": wb, "bytes_per_unit": rd + wb}
for cn in ("SQ_INSTS_VALU", "SQ_WAIT_ANY", "SQ_WAVE_CYCLES", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
    sq = per_dispatch("gpurun_out/pcoop_s/**/*counter_collection.csv", cn)
    for i, nm in enumerate(names):
        j = 2 * i + 1
        if j < len(sq) and nm in out["modes"]:
            out["modes"][nm][cn + "_per_unit"] = sq[j][1] / units
json.dump(out, open("gpurun_out/pmc_coop.json", "w"), indent=1)
print(json.dumps(out, indent=1))
PY
