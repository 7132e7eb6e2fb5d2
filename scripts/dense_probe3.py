"""Diagnostic: the C3 aux rate with another (idle) context alive on the
device, as in bench.py where the headline's context stays open."""
import importlib.util
import json
import sys
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
spec = importlib.util.spec_from_file_location("bench", REPO / "bench.py")
b = importlib.util.module_from_spec(spec)
sys.modules["bench"] = b
spec.loader.exec_module(b)
L = b.load_ffi()
import torch  # noqa: E402

torch.cuda.init()
out = {"alone": b.dense_bench(L, 200, 20, 0)["scans_per_s"]}
pts, off, stamps, maxn = b.make_stream(L, "VLP-16", 1, 100)
d_pts = torch.from_numpy(pts.view(np.uint8)).to(0)
d_off = torch.from_numpy(off.astype(np.int64)).to(0)
g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), device=0, max_points=maxn + 16, max_batch=100, opts=L.opts_from_env())
out["vlp_ctx_idle"] = b.dense_bench(L, 200, 20, 0)["scans_per_s"]
recs = (L.PoseRec * 100)()
g.submit_device(d_pts.data_ptr(), d_off.data_ptr(), stamps, 100)
g.wait(recs)
torch.cuda.synchronize()
out["vlp_ctx_after_batch"] = b.dense_bench(L, 200, 20, 0)["scans_per_s"]
g.close()
out["vlp_ctx_closed"] = b.dense_bench(L, 200, 20, 0)["scans_per_s"]
print(json.dumps(out))
