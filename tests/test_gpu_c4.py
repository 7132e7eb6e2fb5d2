"""Config C4 with product records: the eight VLP-16 streams of seeds 10..17
(SURVEY.md §8d C4), each through the HIP pipeline, checked scan by scan
against the oracle (feature counts and the odometry flag exact, transformSum
within the north-star 1e-4, the bit-exact fraction printed).

* as eight single-stream contexts and as one 8-stream fleet context
  (lego_fleet_create): both give every stream the oracle's records;
* the stream-per-rank partition at world size 2: two processes on GPU 0, each
  running its streams (s mod 2 == rank) through the product, hand their 64-B
  pose records of every step to rank 0 through `multistream.gather_pose_records`
  (gloo here; the bench runs the same gather over RCCL), and rank 0 checks the
  gathered product records against the oracle.  8-GPU scaling itself is not
  measured by this test."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "lego-loam_amd"))
import multistream as ms  # noqa: E402

POSE_TOL = 1e-4  # BASELINE.json north_star: "within 1e-4 on the 6-DoF pose"
STREAMS = 8
K = 24           # scans per stream (two batches of 12)


def _scans(L, stream):
    sc = L.synth_cfg("VLP-16", ms.stream_seed(stream))
    return [L.synth_scan(sc, k) for k in range(K)]


def _pack(scans):
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(len(scans) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    return pts, off, np.array([t for _, t in scans])


def _oracle(L, scans):
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    out = []
    for p, s in scans:
        ora.ip(p, s)
        f = ora.fa()
        out.append((f["transform_sum"].astype(np.float64), len(f["sharp"]), len(f["less_sharp"]),
                    len(f["flat"]), len(f["less_flat"]), int(f["odom_valid"])))
    return out


def _check(recs, ref, label):
    """recs: sequence of lego_pose_rec; returns (worst |dpose|, bit-exact count)."""
    worst, exact = 0.0, 0
    assert len(recs) == len(ref), label
    for k, (r, o) in enumerate(zip(recs, ref)):
        ts = np.array(list(r.transform_sum), np.float64)
        assert (r.n_sharp, r.n_less_sharp, r.n_flat, r.n_less_flat, r.odom_valid) == o[1:], (label, k)
        d = float(np.max(np.abs(ts - o[0])))
        assert d <= POSE_TOL, (label, k, ts, o[0])
        worst = max(worst, d)
        exact += int(np.array_equal(ts.astype(np.float32), o[0].astype(np.float32)))
    assert exact == len(recs), f"{label}: only {exact}/{len(recs)} poses bit-exact"
    return worst, exact


@pytest.fixture(scope="module")
def c4(L):
    scans = [_scans(L, s) for s in range(STREAMS)]
    return scans, [_oracle(L, sc) for sc in scans]


def test_c4_contexts_and_fleet_match_oracle(L, c4):
    scans, ref = c4
    cfg = L.sensor_cfg("VLP-16", L.hip_lib())
    cap = max(len(p) for sc in scans for p, _ in sc) + 16
    h = K // 2
    tot = [0.0, 0, 0]
    for s in range(STREAMS):  # one context per stream, as one stream per GPU runs it
        g = L.Lego(cfg, max_points=cap, max_batch=h)
        recs = list(g.odom_batch(*_pack(scans[s][:h]))) + list(g.odom_batch(*_pack(scans[s][h:])))
        g.close()
        w, e = _check(recs, ref[s], f"context s{s}")
        tot = [max(tot[0], w), tot[1] + e, tot[2] + K]
    fl = L.Lego(cfg, max_points=cap, max_batch=h, streams=STREAMS)
    got = [[] for _ in range(STREAMS)]
    for part in (slice(0, h), slice(h, K)):
        recs = fl.odom_batch(*_pack([x for s in range(STREAMS) for x in scans[s][part]]))  # stream-major
        for s in range(STREAMS):
            got[s].extend(recs[s * h:(s + 1) * h])
    fl.close()
    for s in range(STREAMS):
        w, e = _check(got[s], ref[s], f"fleet s{s}")
        tot = [max(tot[0], w), tot[1] + e, tot[2] + K]
    print(f"C4 product records: {tot[2]} scans (8 contexts + 8-stream fleet), worst |dpose| {tot[0]:.3g}, "
          f"bit-exact {tot[1]}/{tot[2]}")


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    torch.cuda.init()  # torch's HIP runtime first (tests/conftest.py)
    sys.path.insert(0, str(REPO / "tests"))
    from conftest import _load_ffi

    L = _load_ffi()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = ms.streams_of_rank(STREAMS, world, rank)
        cfg = L.sensor_cfg("VLP-16", L.hip_lib())
        scans = {s: _scans(L, s) for s in mine}
        cap = max(len(p) for sc in scans.values() for p, _ in sc) + 16
        h = K // 2
        # this rank's streams as one fleet on its GPU (stream-major batches)
        fl = L.Lego(cfg, max_points=cap, max_batch=h, streams=len(mine))
        gathered = []
        for part in (slice(0, h), slice(h, K)):
            recs = fl.odom_batch(*_pack([x for s in mine for x in scans[s][part]]))
            gathered.append(ms.gather_pose_records(ms.recs_to_bytes(recs), dist))
        fl.close()
        if rank == 0:
            for r in range(world):
                theirs = ms.streams_of_rank(STREAMS, world, r)
                for i, s in enumerate(theirs):
                    recs = []
                    for step in gathered:
                        blk = ms.bytes_to_recs(step[r], L.PoseRec)
                        recs.extend(blk[i * h:(i + 1) * h])
                    _check(recs, _oracle(L, _scans(L, s)), f"rank {r} stream {s}")
            Path(out).write_text("ok")
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_c4_world2_gather_of_product_records(L, tmp_path):
    import torch.multiprocessing as mp

    out = tmp_path / "rank0.txt"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    assert out.read_text() == "ok"
