#!/usr/bin/env python3
"""k_ip_lds phase profile (GPU box, diagnostic build): run with
LEGO_HIP_LIB_AB=build/prof/liblego_hip.so (make OUT=../build/prof
EXTRA=-DIP_PROF=1).  Thread 0 of every workgroup sums the clock64 ticks
between its phase barriers; printed per workgroup for (a) one 100-scan C2
batch alone and (b) fleet calls (256 VLP-16 streams x 20 scans, two front-end
parts, the odometry beside).  Diagnostic."""
import ctypes as C
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
import bench  # noqa: E402

PH = ["init", "project", "pixels", "ground", "unions", "find+counts", "flags", "prefix", "outputs"]


def read(lib):
    out = (C.c_ulonglong * 12)()
    assert lib.lego_ip_profile(out) == 0
    n = max(out[11], 1)
    return {"workgroups": out[11], **{PH[i]: round(out[i] / n) for i in range(9)},
            "total": round(sum(out[i] for i in range(9)) / n)}


def main():
    import torch

    L = bench.load_ffi()
    lib = L.hip_lib()
    lib.lego_ip_profile.argtypes = [C.POINTER(C.c_ulonglong)]
    cfg = L.sensor_cfg("VLP-16", lib)
    # (a) C2: one stream, 100-scan batches
    sc = L.synth_cfg("VLP-16", 1)
    scans = [L.synth_scan(sc, k) for k in range(200)]
    g = L.Lego(cfg, max_points=max(len(p) for p, _ in scans) + 16, max_batch=100)
    for w in range(2):
        pts = np.concatenate([p for p, _ in scans[w * 100:(w + 1) * 100]])
        off = np.concatenate([[0], np.cumsum([len(p) for p, _ in scans[w * 100:(w + 1) * 100]])]).astype(np.int64)
        st = np.array([s for _, s in scans[w * 100:(w + 1) * 100]])
        if w == 1:
            read(lib)
        g.odom_batch(pts, off, st)
    print(json.dumps({"line": "C2 batch of 100", **read(lib)}), flush=True)
    g.close()
    # (b) the fleet
    S, K = 256, 20
    src = [[L.synth_scan(L.synth_cfg("VLP-16", 10 + s), j)[0] for j in range(3 * K)] for s in range(S)]
    maxn = max(len(p) for s in src for p in s)
    fl = L.Lego(cfg, device=0, max_points=maxn + 16, max_batch=K, streams=S)
    recs = (L.PoseRec * (S * K))()
    for w in range(3):
        scans_w = [src[s][w * K + j] for s in range(S) for j in range(K)]
        off = np.zeros(len(scans_w) + 1, np.int64)
        off[1:] = np.cumsum([len(p) for p in scans_w])
        dp = torch.from_numpy(np.concatenate(scans_w).view(np.uint8)).cuda()
        do = torch.from_numpy(off).cuda()
        st = np.concatenate([np.arange(w * K, (w + 1) * K) * 0.1] * S)
        if w == 1:
            read(lib)
        t0 = time.perf_counter()
        fl.odom_batch_device(dp.data_ptr(), do.data_ptr(), st, S * K, recs)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    print(json.dumps({"line": "fleet call (2 calls)", "last_call_ms": round(dt * 1e3, 2), **read(lib)}), flush=True)
    fl.close()


if __name__ == "__main__":
    main()
