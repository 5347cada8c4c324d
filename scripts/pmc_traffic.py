"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes of k_integrate into HBM bytes per reactor.

  python scripts/pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> N out.json

FETCH_SIZE and WRITE_SIZE are in KiB (rocprofv3 derived counters from the L2's memory-side
requests, Infinity-Cache hits included). Per MI355X_MICROARCH.md (HBM section) FETCH_SIZE reads
half the bytes on gfx950 (128-B requests tallied as 64 B), so it is doubled; WRITE_SIZE is taken
as is. The integrator reads 8 B per lane (dwordx2), a width the guide lists as uncalibrated, so
the TCC_MISS x 128 B estimate (when a third file is given) is reported beside it.
"""
import csv
import json
import sys


def total(path, name):
    s = 0.0
    for r in csv.DictReader(open(path)):
        if any(k in r["Kernel_Name"] for k in ("k_integrate", "k_lane", "k_quad", "k_group")) and r["Counter_Name"] == name:
            s += float(r["Counter_Value"])
    return s


def main():
    fetch_csv, write_csv, n, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    fetch_kib = total(fetch_csv, "FETCH_SIZE")
    write_kib = total(write_csv, "WRITE_SIZE")
    rd = 2.0 * fetch_kib * 1024.0
    wr = write_kib * 1024.0
    res = {"reactors": n, "fetch_size_kib": fetch_kib, "write_size_kib": write_kib,
           "read_bytes_corrected": rd, "write_bytes": wr,
           "bytes_per_reactor": (rd + wr) / n,
           "note": "FETCH_SIZE x2 (gfx950 correction), KiB->B; integrator dispatches (k_integrate / k_lane / k_group) only"}
    if len(sys.argv) > 5:
        hit = total(sys.argv[5], "TCC_HIT_sum")
        miss = total(sys.argv[5], "TCC_MISS_sum")
        res["tcc_hit_rate"] = hit / max(hit + miss, 1.0)
        res["tcc_miss_bytes_per_reactor"] = miss * 128.0 / n
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
