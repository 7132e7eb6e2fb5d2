#!/usr/bin/env python3
"""HBM bytes per launch from two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE;
scripts/gpu_profile.sh), with MI355X_MICROARCH.md's gfx950 correction:
FETCH_SIZE x2 (it reports half of wide coalesced reads), WRITE_SIZE as
reported, KiB -> bytes.  Usage: pmc_summary.py <run dir> <out.json> <source note> [commit]"""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path


def per_launch(path, counter):
    tot, n = defaultdict(float), defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = re.sub(r"<[^<>]*>", "", r["Kernel_Name"].split("(")[0]).replace("void ", "")  # k_odom<true> -> k_odom
        if name.startswith("__amd"):
            continue
        tot[name] += float(r["Counter_Value"])
        n[name] += 1
    return {k: tot[k] / n[k] for k in tot}


def main():
    run, out, note = Path(sys.argv[1]), Path(sys.argv[2]), sys.argv[3]
    f = per_launch(run / "pmc_fetch" / "run_counter_collection.csv", "FETCH_SIZE")
    w = per_launch(run / "pmc_write" / "run_counter_collection.csv", "WRITE_SIZE")
    res = {"source": note, "commit": sys.argv[4] if len(sys.argv) > 4 else None,
           "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads, MI355X_MICROARCH.md HBM "
                         "section); WRITE_SIZE as reported; KiB -> bytes",
           "per_launch": {}}
    for k in f:
        rd, wr = f[k] * 2 * 1024, w.get(k, 0.0) * 1024
        res["per_launch"][k] = {"FETCH_SIZE_KiB_raw": f[k], "read_bytes": rd, "WRITE_SIZE_KiB_raw": w.get(k, 0.0),
                                "write_bytes": wr, "hbm_bytes": rd + wr}
    res["k_odom_hbm_bytes_per_launch"] = res["per_launch"].get("lego::k_odom", {}).get("hbm_bytes")
    out.write_text(json.dumps(res, indent=1))
    print(json.dumps({k: round(v["hbm_bytes"] / 1e6, 2) for k, v in res["per_launch"].items()}))


if __name__ == "__main__":
    main()
