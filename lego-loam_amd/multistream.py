"""Stream-per-GPU sharding and the pose-record hand-off.

Each lidar stream is an independent unit: scans of one stream are serially
dependent through the odometry state, so a stream never spans GPUs.  Stream s
runs on rank s mod world.  The only exchange is the gather of the fixed 64-B
`lego_pose_rec`s of every step to rank 0, the serial consumer (the reference's
mapOptimization / transformFusion nodes).  On ROCm the "nccl" backend is RCCL
over xGMI; the CPU tests drive the same code over gloo.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

POSE_REC_BYTES = 64


def streams_of_rank(n_streams: int, world: int, rank: int) -> list[int]:
    """Streams owned by `rank` under the s mod world partition."""
    return [s for s in range(n_streams) if s % world == rank]


def stream_seed(stream: int) -> int:
    """C4's seeds: stream s is the synthetic VLP-16 stream with seed 10 + s."""
    return 10 + stream


def recs_to_bytes(recs) -> np.ndarray:
    """ctypes array of lego_pose_rec -> uint8[K*64] (no copy of semantics)."""
    raw = np.frombuffer(bytearray(bytes(recs)), dtype=np.uint8)
    assert raw.size == len(recs) * POSE_REC_BYTES
    return raw


def bytes_to_recs(raw: np.ndarray, rec_type):
    """uint8[K*64] -> ctypes array of rec_type."""
    k = raw.size // POSE_REC_BYTES
    out = (rec_type * k)()
    C.memmove(out, np.ascontiguousarray(raw).ctypes.data, raw.size)
    return out


def gather_pose_records(raw: np.ndarray, dist, device=None):
    """Gathers every rank's uint8[K*64] record block to rank 0.

    All ranks pass blocks of the same K (one step of the same batch size).
    Returns the list of per-rank uint8 arrays on rank 0, None elsewhere.  With
    a device the tensors live in HBM (RCCL); otherwise on the host (gloo)."""
    import torch

    t = torch.from_numpy(np.ascontiguousarray(raw))
    if device is not None:
        t = t.to(device)
    world = dist.get_world_size()
    rank = dist.get_rank()
    glist = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, glist, dst=0)
    if rank != 0:
        return None
    return [g.cpu().numpy() for g in glist]
