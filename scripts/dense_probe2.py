"""Diagnostic: the C3 aux (dense_bench) with and without the context's stage
timer, to see why the aux rate sits below the main-line HDL-64E rate."""
import ctypes as C
import importlib.util
import json
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
spec = importlib.util.spec_from_file_location("bench", REPO / "bench.py")
b = importlib.util.module_from_spec(spec)
sys.modules["bench"] = b
spec.loader.exec_module(b)
L = b.load_ffi()
import torch  # noqa: E402

torch.cuda.init()
orig = L.Lego


class Timed(orig):
    def __init__(self, *a, **k):
        super().__init__(*a, **k)
        n = C.c_int32()
        on = (C.c_float * 1)()
        self.lib.lego_stage_times(self.h, None, on, 0, C.byref(n))


out = {"plain_1": b.dense_bench(L, 200, 20, 0)["scans_per_s"]}
L.Lego = Timed
out["stage_timer"] = b.dense_bench(L, 200, 20, 0)["scans_per_s"]
L.Lego = orig
out["plain_2"] = b.dense_bench(L, 200, 20, 0)["scans_per_s"]
print(json.dumps(out))
