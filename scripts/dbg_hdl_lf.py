"""Debug: HDL-64E seed 2 scan 7 less-flat cloud, product (repeated) vs oracle."""
import os
import sys
from pathlib import Path
import numpy as np
sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tests"))
from conftest import _load_ffi
L = _load_ffi()
cfg = L.sensor_cfg("HDL-64E", L.hip_lib())
sc = L.synth_cfg("HDL-64E", 2)
o = L.Oracle(L.sensor_cfg("HDL-64E"))
scans = [L.synth_scan(sc, k) for k in range(8)]
for pts, st in scans:
    o.ip(pts, st)
    of = o.fa()
ref = of["less_flat"]
res = []
for rep in range(6):
    g = L.Lego(cfg, max_points=140000, max_batch=1)
    for pts, st in scans:
        g.ip(pts, st)
        gf = g.fa()
    a = gf["less_flat"]
    res.append((len(a), len(a) == len(ref) and np.array_equal(a.view(np.uint32), ref.view(np.uint32))))
    g.close()
print(os.environ.get("LEGO_XLDS_PAD"), "oracle", len(ref), "product runs", res, flush=True)
