"""Stream-per-rank sharding and the pose-record gather, world_size 2 over gloo
on the CPU (the GPU bench runs the same code over RCCL).  Each rank runs its
own stream through the oracle (test infrastructure) and hands its 64-B records
to rank 0, which checks them against streams it recomputes itself."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO / "lego-loam_amd"))
import multistream as ms  # noqa: E402

K = 3


def stream_recs(L, stream):
    """The oracle's pose records for the first K scans of `stream`."""
    sc = L.synth_cfg("VLP-16", ms.stream_seed(stream))
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    recs = (L.PoseRec * K)()
    for k in range(K):
        pts, stamp = L.synth_scan(sc, k)
        ora.ip(pts, stamp)
        fa = ora.fa()
        r = recs[k]
        r.stamp = stamp
        for i in range(6):
            r.transform_sum[i] = float(fa["transform_sum"][i])
        r.n_sharp, r.n_less_sharp = len(fa["sharp"]), len(fa["less_sharp"])
        r.n_flat, r.n_less_flat = len(fa["flat"]), len(fa["less_flat"])
        r.odom_valid = int(fa["odom_valid"])
    return recs


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    sys.path.insert(0, str(REPO / "tests"))
    from conftest import _load_ffi, ensure_built

    ensure_built()
    L = _load_ffi()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = ms.streams_of_rank(world, world, rank)
        assert mine == [rank]
        got = ms.gather_pose_records(ms.recs_to_bytes(stream_recs(L, mine[0])), dist)
        if rank == 0:
            assert len(got) == world
            for r in range(world):
                exp = ms.recs_to_bytes(stream_recs(L, r))
                np.testing.assert_array_equal(got[r], exp)
                back = ms.bytes_to_recs(got[r], L.PoseRec)
                assert back[K - 1].odom_valid == 1 and back[0].odom_valid == 0
            Path(out).write_text("ok")
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_partition():
    assert ms.streams_of_rank(8, 2, 0) == [0, 2, 4, 6]
    assert ms.streams_of_rank(8, 2, 1) == [1, 3, 5, 7]
    assert sorted(sum((ms.streams_of_rank(5, 3, r) for r in range(3)), [])) == list(range(5))


def test_pose_record_layout(L):
    assert L.C.sizeof(L.PoseRec) == ms.POSE_REC_BYTES


def test_gather_world2_gloo(L, tmp_path):
    import torch.multiprocessing as mp

    out = tmp_path / "rank0.txt"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    assert out.read_text() == "ok"
