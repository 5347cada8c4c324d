"""Builds the committed golden fixtures from the reference's own data (run in the build
container, where /root/reference exists). Data only: inputs and expected outputs.

  gas_and_surf_golden.csv / surf_and_gas_covg_golden.csv
      every 8th row (plus the first 12 and the last 3) of
      test/batch_gas_and_surf/gas_profile.csv and surface_covg.csv (CVODE_BDF, rtol 1e-6,
      atol 1e-10, GRI-Mech 3.0 + ch4ni.xml, T=1173 K, p0=1e5 Pa, tf=10 s)
  doc_surf_rows.csv
      the surface-only sample rows printed in docs/src/index.md:160-185 (4-5 digits)
  lib/ and batch_*/batch.xml
      the reference's test inputs (test/lib/*, test/batch_*/batch.xml), copied verbatim
"""
import csv
import os
import re

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


def subsample(src, dst):
    rows = list(csv.reader(open(src)))
    hdr, data = rows[0], rows[1:]
    keep = sorted(set(range(12)) | set(range(0, len(data), 8)) | {len(data) - 3, len(data) - 2, len(data) - 1})
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


if __name__ == "__main__":
    subsample(os.path.join(REF, "test/batch_gas_and_surf/gas_profile.csv"), os.path.join(HERE, "gas_and_surf_golden.csv"))
    subsample(os.path.join(REF, "test/batch_gas_and_surf/surface_covg.csv"), os.path.join(HERE, "gas_and_surf_covg_golden.csv"))
    doc_rows(os.path.join(HERE, "doc_surf_rows.csv"))
