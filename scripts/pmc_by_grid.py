#!/usr/bin/env python3
"""Per-launch HBM bytes from the two rocprofv3 PMC passes (FETCH_SIZE x2 +
WRITE_SIZE, as pmc_summary.py), split by kernel AND grid size, so launches of
one kernel at different sizes (the C2 line's 100-scan batches beside the
fleet's 5,120-scan calls) are not averaged together.
Usage: pmc_by_grid.py <run dir> [kernel substring]"""
import csv
import re
import sys
from collections import defaultdict
from pathlib import Path


def rows(path, counter):
    out = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = re.sub(r"<[^<>]*>", "", r["Kernel_Name"].split("(")[0]).replace("void ", "")
        if name.startswith("__amd"):
            continue
        grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        out[(name, grid)].append(float(r["Counter_Value"]))
    return out


def main():
    run = Path(sys.argv[1])
    want = sys.argv[2] if len(sys.argv) > 2 else ""
    f = rows(next(run.glob("pmc_fetch/**/*counter_collection.csv")), "FETCH_SIZE")
    w = rows(next(run.glob("pmc_write/**/*counter_collection.csv")), "WRITE_SIZE")
    for key in sorted(f, key=lambda k: -sum(f[k]) / len(f[k])):
        if want not in key[0]:
            continue
        rd = sum(f[key]) / len(f[key]) * 2 * 1024
        wr = (sum(w[key]) / len(w[key]) * 1024) if key in w else 0.0
        print(f"{key[0]:28s} grid {key[1]:>10s} x{len(f[key]):3d}: read {rd / 1e6:9.2f} MB  write {wr / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
