"""Diagnostic: bench.py's C3 aux (dense_bench) alone, twice, and after the
fleet aux, to see what the aux line's rate depends on."""
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
out = {}
out["dense_1"] = b.dense_bench(L, 200, 20, 0)["scans_per_s"]
out["dense_2"] = b.dense_bench(L, 200, 20, 0)["scans_per_s"]
out["fleet"] = b.fleet_bench(L, 64, 20, 3, 0)["scans_per_s"]
out["dense_after_fleet"] = b.dense_bench(L, 200, 20, 0)["scans_per_s"]
print(json.dumps(out))
