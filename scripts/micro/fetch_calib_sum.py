"""FETCH_SIZE / WRITE_SIZE (kB per dispatch) against the bytes each dispatch streamed."""
import csv
import glob
import json

names = {0: "raw_buffer_load_b64 (8 B/lane)", 1: "raw_buffer_load_b128 (16 B/lane)", 2: "global_load_dwordx2 (8 B/lane)",
         3: "raw_buffer_store_b64 (8 B/lane)"}
out = []
for d in sorted(glob.glob("gpurun_out/fc_*_*")):
    if not __import__("os").path.isdir(d):
        continue
    _, m, s = d.rsplit("/", 1)[1].split("_")
    m, s = int(m), int(s)
    vals = []
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_stream" in r["Kernel_Name"]:
                vals.append(float(r["Counter_Value"]) * 1024)
    out.append({"mode": names[m], "bytes_per_dispatch": s, "counter_bytes_per_dispatch": vals,
                "ratio_counter_over_bytes": [v / s for v in vals]})
json.dump(out, open("gpurun_out/fetch_calib.json", "w"), indent=1)
print(json.dumps(out, indent=1))
