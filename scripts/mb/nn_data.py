"""Real-shaped NN inputs for mb_nn: the oracle's C2 stream (VLP-16, seed 1);
for each scan k that follows a published scan, the previous scan's
surf_last / corner_last clouds (the LM's "last" clouds) and scan k's flat /
sharp features (the queries).  Writes build/nn_data.bin:
  int32 npairs; per pair: int32 nLS, nQS, nLC, nQC; float4 arrays in that order."""
import importlib.util
import struct
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[2]
spec = importlib.util.spec_from_file_location("legoffi", REPO / "lego-loam_amd" / "legoffi.py")
L = importlib.util.module_from_spec(spec)
sys.modules["legoffi"] = L
spec.loader.exec_module(L)

ora = L.Oracle(L.sensor_cfg("VLP-16"))
sc = L.synth_cfg("VLP-16", 1)
prev = None
pairs = []
for k in range(24):
    pts, stamp = L.synth_scan(sc, k)
    ora.ip(pts, stamp)
    f = ora.fa()
    if prev is not None:
        pairs.append((prev["surf_last"], f["flat"], prev["corner_last"], f["sharp"]))
    prev = f if len(f["surf_last"]) else prev


def f4(a):
    return np.stack([a["x"], a["y"], a["z"], a["intensity"]], axis=1).astype(np.float32)


out = REPO / "build" / "nn_data.bin"
out.parent.mkdir(exist_ok=True)
with open(out, "wb") as fh:
    fh.write(struct.pack("<i", len(pairs)))
    for ls, qs, lc, qc in pairs:
        fh.write(struct.pack("<4i", len(ls), len(qs), len(lc), len(qc)))
        for a in (ls, qs, lc, qc):
            fh.write(f4(a).tobytes())
print(len(pairs), "pairs", [(len(p[0]), len(p[1]), len(p[2]), len(p[3])) for p in pairs[:3]])
