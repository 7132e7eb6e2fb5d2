"""featureAssociation's hand-off to the serial mapping consumer on rank 0
(publishCloudsLast, featureAssociation.cpp:1790-1815): the
product's batch packet (lego_handoff_pack), mapping on a packet
(lego_handoff_unpack -> lego_mo_process), the RCCL collective behind the
C-ABI (lego_comm_*) and the stream-per-rank gather at world size 2.

* the packet of a batch equals what lego_batch_fetch returns scan by scan;
* a mapping context that only sees packets maps the stream exactly as the
  oracle maps it from its own node-shaped pipeline (poses within 1e-4, the
  bit-exact count printed);
* lego_comm_gather_handoff over RCCL at world size 1 (RCCL needs one GPU per
  rank; this box has one): the gathered packet is the context's own;
* two processes on GPU 0 run streams 0 and 1 (seeds 10, 11) and gather their
  packets to rank 0 over gloo; rank 0 maps both streams from the packets and
  matches the oracle."""
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

POSE_TOL = 1e-4
K = 24


def _scans(L, seed, n=K):
    sc = L.synth_cfg("VLP-16", seed)
    return [L.synth_scan(sc, k) for k in range(n)]


def _pack(scans):
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(len(scans) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    return pts, off, np.array([t for _, t in scans])


def _oracle_mapping(L, scans):
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    out = []
    for p, s in scans:
        ora.ip(p, s)
        ora.fa()
        out.append(ora.mo())
    return out


def _map_packets(L, packets, ref, label):
    """Maps the scans of the packets in order on a fresh context; checks
    against the oracle's mapping outputs."""
    cap = 40000
    m = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=cap)
    k, steps, exact, worst = 0, 0, 0, 0.0
    for pkt in packets:
        for j in range(L.handoff_header(pkt).nscans):
            g, o = m.mo_handoff(pkt, j), ref[k]
            k += 1
            assert g["processed"] == o["processed"], (label, k)
            if not o["processed"]:
                continue
            steps += 1
            for key in ("optimized", "n_corner_map_ds", "n_surf_map_ds", "n_corner_scan_ds", "n_surf_scan_ds"):
                assert g[key] == o[key], (label, k, key)
            d = float(np.max(np.abs(g["transform_aft_mapped"].astype(np.float64) - o["transform_aft_mapped"])))
            assert d <= POSE_TOL, (label, k)
            worst = max(worst, d)
            exact += int(np.array_equal(g["transform_aft_mapped"].view(np.uint32),
                                        o["transform_aft_mapped"].view(np.uint32)))
    m.close()
    assert steps >= 4
    print(f"{label}: {steps} mapping steps from packets, worst |dpose| {worst:.3g}, bit-exact {exact}/{steps}")
    assert exact == steps, f"{label}: only {exact}/{steps} mapped poses bit-exact"


def test_packet_equals_batch_fetch(L):
    scans = _scans(L, 1)
    g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, max_batch=K)
    recs = g.odom_batch(*_pack(scans))
    pkt = g.handoff_packet()
    h = L.handoff_header(pkt)
    assert h.magic == L.HANDOFF_MAGIC and h.nscans == K and h.bytes == pkt.size
    npub = 0
    for k in range(K):
        rec, fa = L.handoff_unpack(pkt, k)
        assert bytes(rec)[:60] == bytes(recs[k])[:60], k
        _, ref = g.batch_fetch(k)
        npub += fa["publish_to_mapping"]
        for key in ("publish_to_mapping", "odom_valid"):
            assert fa[key] == ref[key], (k, key)
        for key in ("transform_sum", "transform_cur", "odom_quat", "odom_pos"):
            assert np.array_equal(fa[key], ref[key]), (k, key)
        for key in ("corner_last", "surf_last", "outlier_last"):
            assert np.array_equal(fa[key].view(np.uint8), ref[key].view(np.uint8)), (k, key)
    assert npub == h.npub and npub >= K // 2 - 1
    g.close()


def test_mapping_from_packets_matches_oracle(L):
    scans = _scans(L, 6, 40)
    ref = _oracle_mapping(L, scans)
    g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, max_batch=20)
    packets = []
    for part in (scans[:20], scans[20:]):
        g.odom_batch(*_pack(part))
        packets.append(g.handoff_packet())
    g.close()
    _map_packets(L, packets, ref, "seed 6")


def test_native_rccl_gather_world1(L):
    """lego_comm over RCCL with one rank: the gathered packet is the
    context's own, byte for byte, over two consecutive batches."""
    import ctypes as C

    lib = L.hip_lib()
    uid = (C.c_uint8 * 128)()
    L.check(lib.lego_comm_unique_id(uid), "lego_comm_unique_id", lib)
    comm = C.c_void_p()
    L.check(lib.lego_comm_create(uid, 1, 0, 0, C.byref(comm)), "lego_comm_create", lib)
    scans = _scans(L, 2)
    g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, max_batch=K // 2)
    for part in (scans[:K // 2], scans[K // 2:]):
        g.odom_batch(*_pack(part))
        got = ms.native_gather_handoff(L, comm, g, 0)
        assert len(got) == 1 and np.array_equal(got[0], g.handoff_packet())
    g.close()
    lib.lego_comm_destroy(comm)


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
        scans = _scans(L, ms.stream_seed(rank))
        g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, max_batch=K // 2)
        gathered = []
        for part in (scans[:K // 2], scans[K // 2:]):
            g.odom_batch(*_pack(part))
            gathered.append(ms.gather_packets(g.handoff_packet(), dist))
        g.close()
        if rank == 0:  # the serial consumer maps every stream from its packets
            for r in range(world):
                _map_packets(L, [step[r] for step in gathered], _oracle_mapping(L, _scans(L, ms.stream_seed(r))),
                             f"rank {r} stream")
            Path(out).write_text("ok")
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_world2_packets_mapped_on_rank0(L, tmp_path):
    import torch.multiprocessing as mp

    out = tmp_path / "rank0.txt"
    mp.spawn(_worker, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    assert out.read_text() == "ok"


def test_native_rccl_gather_device_result_world1(L):
    """LEGO_COMM_DEVICE_RESULT: the packet stays in HBM, the call does not wait
    for the transfer; after lego_comm_wait its bytes equal the host path's."""
    import ctypes as C

    lib = L.hip_lib()
    uid = (C.c_uint8 * 128)()
    L.check(lib.lego_comm_unique_id(uid), "lego_comm_unique_id", lib)
    comm = C.c_void_p()
    L.check(lib.lego_comm_create(uid, 1, 0, 0, C.byref(comm)), "lego_comm_create", lib)
    scans = _scans(L, 2)
    g = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=40000, max_batch=K // 2)
    for part in (scans[:K // 2], scans[K // 2:]):
        g.odom_batch(*_pack(part))
        got = ms.native_gather_handoff(L, comm, g, 0, device=True)
        assert len(got) == 1
        L.check(lib.lego_comm_wait(comm), "lego_comm_wait", lib)
        ptr, n = got[0]
        host = np.zeros(n, np.uint8)
        assert L.hip_memcpy_d2h(host.ctypes.data, ptr, n) == 0
        assert np.array_equal(host, g.handoff_packet())
        # the host result is only produced by the host-result call
        p, b = C.c_void_p(), C.c_uint64()
        assert lib.lego_comm_handoff(comm, 0, C.byref(p), C.byref(b)) == L.LEGO_E_STATE
    g.close()
    lib.lego_comm_destroy(comm)


def _native_worker(rank, world, port, out):
    """One process per GPU: the C-ABI collective (RCCL send/recv between the
    GPUs) gathers every rank's packets to rank 0, host and device results."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist

    torch.cuda.set_device(rank)
    sys.path.insert(0, str(REPO / "tests"))
    from conftest import _load_ffi

    L = _load_ffi()
    lib = L.hip_lib()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        comm = ms.native_comm(L, dist, rank)
        scans = _scans(L, ms.stream_seed(rank))
        g = L.Lego(L.sensor_cfg("VLP-16", lib), device=rank, max_points=40000, max_batch=K // 2)
        host_steps, dev_steps = [], []
        for part in (scans[:K // 2], scans[K // 2:]):
            g.odom_batch(*_pack(part))
            own = g.handoff_packet()
            host_steps.append(ms.native_gather_handoff(L, comm, g, 0))
            dev = ms.native_gather_handoff(L, comm, g, 0, device=True)
            L.check(lib.lego_comm_wait(comm), "lego_comm_wait", lib)
            if rank == 0:
                copies = []
                for ptr, n in dev:
                    h = np.zeros(n, np.uint8)
                    assert L.hip_memcpy_d2h(h.ctypes.data, ptr, n) == 0
                    copies.append(h)
                dev_steps.append(copies)
                assert np.array_equal(host_steps[-1][0], own)
        g.close()
        lib.lego_comm_destroy(comm)
        if rank == 0:
            for r in range(world):
                for hs, ds in zip(host_steps, dev_steps):
                    assert np.array_equal(hs[r], ds[r]), f"rank {r}: device result differs from host result"
                _map_packets(L, [step[r] for step in host_steps],
                             _oracle_mapping(L, _scans(L, ms.stream_seed(r))), f"rank {r} stream")
            Path(out).write_text("ok")
    finally:
        dist.destroy_process_group()


def test_native_rccl_gather_all_gpus(L, tmp_path):
    """lego_comm_gather_handoff(_ex) with one rank per visible GPU (world =
    torch.cuda.device_count(), up to 8): the ncclSend / ncclRecv branch.  Rank
    0 maps every stream from the gathered packets bit-exactly like the
    oracle.  Needs two GPUs or more (skipped on a one-GPU box)."""
    import torch
    import torch.multiprocessing as mp

    world = min(torch.cuda.device_count(), 8)
    if world < 2:
        pytest.skip("one GPU: RCCL needs a device per rank")
    out = tmp_path / "rank0.txt"
    mp.spawn(_native_worker, args=(world, _free_port(), str(out)), nprocs=world, join=True)
    assert out.read_text() == "ok"
