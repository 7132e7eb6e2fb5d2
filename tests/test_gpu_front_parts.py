"""A fleet batch's front end in parts (submit_batch: projection + extraction of
whole streams per part, each part on its own HIP stream; lego_ctx_opts::front_parts)
is a scheduling change only: every stream's records equal, byte for
byte, the one-part order's, and the one-part records equal the oracle's (the
C4 test checks the default split against the oracle scan by scan).
Reference: featureAssociation.cpp:1817-1860 (runFeatureAssociation, per
stream), imageProjection.cpp:300-460."""
import ctypes as C
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "lego-loam_amd"))
import multistream as ms  # noqa: E402

STREAMS = 8
K = 8  # scans per stream: two calls of four


def _pack(scans):
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(len(scans) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    return pts, off, np.array([t for _, t in scans])


def _run(L, cfg, cap, scans, parts):
    h = K // 2
    fl = L.Lego(cfg, max_points=cap, max_batch=h, streams=STREAMS, opts={"front_parts": parts})
    got = []
    for part in (slice(0, h), slice(h, K)):
        recs = fl.odom_batch(*_pack([x for s in range(STREAMS) for x in scans[s][part]]))  # stream-major
        got.append([bytes(C.string_at(C.addressof(r), C.sizeof(r))) for r in recs])
    fl.close()
    return got


def test_front_parts_are_only_scheduling(L):
    scans = []
    for s in range(STREAMS):
        sc = L.synth_cfg("VLP-16", ms.stream_seed(s))
        scans.append([L.synth_scan(sc, k) for k in range(K)])
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    cap = max(len(p) for sc in scans for p, _ in sc) + 16
    one = _run(L, cfg, cap, scans, 1)
    for parts in (2, 4, 3):  # 3 does not divide 8 streams: two parts
        got = _run(L, cfg, cap, scans, parts)
        for c in range(2):
            for i, (a, b) in enumerate(zip(got[c], one[c])):
                assert a == b, (parts, c, i // (K // 2), i % (K // 2))
    # stream 0's one-part records against the oracle (poses bit-exact)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    recs = [L.PoseRec.from_buffer_copy(b) for c in range(2) for b in one[c][:K // 2]]
    for k, (p, t) in enumerate(scans[0]):
        ora.ip(p, t)
        f = ora.fa()
        ts = np.array(list(recs[k].transform_sum), np.float32)
        assert np.array_equal(ts.view(np.uint32), f["transform_sum"].astype(np.float32).view(np.uint32)), k
