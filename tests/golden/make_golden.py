"""Builds the committed golden fixtures from the reference's own data (run in the build
container, where /root/reference exists). Data only: inputs and expected outputs.

  gas_and_surf_golden.csv / gas_and_surf_covg_golden.csv
      every 8th row (plus the first 48 accepted steps, every 2nd row of the ignition window
      3.7-3.95 ms and the last 3) of
      test/batch_gas_and_surf/gas_profile.csv and surface_covg.csv (CVODE_BDF, rtol 1e-6,
      atol 1e-10, GRI-Mech 3.0 + ch4ni.xml, T=1173 K, p0=1e5 Pa, tf=10 s)
  golden_meta.json
      scalars of the full golden: accepted steps, ignition time (max dX_OH/dt, midpoint of
      the steepest accepted-step difference)
  doc_surf_rows.csv
      the surface-only sample rows printed in docs/src/index.md:160-185 (4-5 digits)
  lib/ and batch_*/batch.xml
      the reference's test inputs (test/lib/*, test/batch_*/batch.xml), copied verbatim
"""
import csv
import json
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def subsample(src, dst):
    rows = list(csv.reader(open(src)))
    hdr, data = rows[0], rows[1:]
    t = [float(r[0]) for r in data]
    ign = {i for i in range(0, len(data), 2) if 3.7e-3 <= t[i] <= 3.95e-3}
    keep = sorted(set(range(48)) | set(range(0, len(data), 8)) | ign | {len(data) - 3, len(data) - 2, len(data) - 1})
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["row"] + hdr)
        for i in keep:
            w.writerow([i] + data[i])


def doc_rows(dst):
    txt = open(os.path.join(REF, "docs/src/index.md")).read()
    blocks = re.findall(r"```\n(\s+t\s+T.*?)```", txt, re.S)
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        for bi, b in enumerate(blocks):
            lines = [l for l in b.strip().splitlines() if l.strip() and not l.strip().startswith("...")]
            hdr = lines[0].split()
            w.writerow(["block", "kind"] + hdr)
            for l in lines[1:]:
                w.writerow([bi, "gas" if "rho" in hdr else "surf"] + l.split())


def meta(src, dst):
    rows = list(csv.reader(open(src)))
    hdr, data = rows[0], rows[1:]
    k = hdr.index("OH")
    t = [float(r[0]) for r in data]
    x = [float(r[k]) for r in data]
    d = [(x[i + 1] - x[i]) / (t[i + 1] - t[i]) for i in range(len(t) - 1)]
    j = max(range(len(d)), key=lambda i: d[i])
    json.dump({"source": "test/batch_gas_and_surf/gas_profile.csv", "accepted_steps": len(data) - 1,
               "t_ign_max_dXOH_dt": 0.5 * (t[j] + t[j + 1]), "t_final": t[-1]}, open(dst, "w"), indent=1)


if __name__ == "__main__":
    meta(os.path.join(REF, "test/batch_gas_and_surf/gas_profile.csv"), os.path.join(HERE, "golden_meta.json"))
    subsample(os.path.join(REF, "test/batch_gas_and_surf/gas_profile.csv"), os.path.join(HERE, "gas_and_surf_golden.csv"))
    subsample(os.path.join(REF, "test/batch_gas_and_surf/surface_covg.csv"), os.path.join(HERE, "gas_and_surf_covg_golden.csv"))
    doc_rows(os.path.join(HERE, "doc_surf_rows.csv"))
