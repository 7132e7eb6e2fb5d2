"""Stream-per-GPU sharding and the hand-off to rank 0.

Each lidar stream is an independent unit: scans of one stream are serially
dependent through the odometry state, so a stream never spans GPUs.  Stream s
runs on rank s mod world.  The only exchange is the hand-off to rank 0, the
serial consumer (the reference's mapOptimization / transformFusion nodes):
the fixed 64-B `lego_pose_rec`s of every step (`gather_pose_records`, the
bench's per-step gather) and the batch's hand-off packet with the published
corner / surf / outlier clouds (`gather_packets` over torch.distributed, or
`native_gather_handoff`, the C-ABI's RCCL collective, lego_comm.hip — what
bench.py's N > 1 path times), which rank 0 maps with `Lego.mo_handoff`.  On ROCm the "nccl" backend is RCCL over
xGMI; the CPU tests drive the same code over gloo.
"""
from __future__ import annotations

import ctypes as C
import os
import sys
import threading
import time

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


def gather_packets(packet, dist, device=None, to_host: bool = True):
    """Gathers every rank's variable-size uint8 hand-off packet
    (lego_handoff_pack; a numpy array, or a torch tensor already in HBM from
    Lego.handoff_tensor) to rank 0 over torch.distributed: the sizes first,
    then the packets padded to the largest.  Returns the list of per-rank
    packets on rank 0 (numpy, or device tensors with to_host=False), None
    elsewhere.  The native RCCL path is `native_gather_handoff`."""
    import torch

    world, rank = dist.get_world_size(), dist.get_rank()
    t = packet if isinstance(packet, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(packet))
    if device is not None:
        t = t.to(device)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(s.item()) for s in sizes]
    if t.numel() < max(sizes):
        t = torch.cat([t, torch.zeros(max(sizes) - t.numel(), dtype=torch.uint8, device=t.device)])
    glist = [torch.empty_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, glist, dst=0)
    if rank != 0:
        return None
    out = [g[:sizes[r]] for r, g in enumerate(glist)]
    return [g.cpu().numpy().copy() for g in out] if to_host else out


def native_comm(L, dist, device: int):
    """A lego_comm (RCCL) over the ranks of `dist`: rank 0's unique id is
    broadcast with torch.distributed, then every rank joins on its device."""
    import ctypes as C

    lib = L.hip_lib()
    uid = (C.c_uint8 * 128)()
    if dist.get_rank() == 0:
        L.check(lib.lego_comm_unique_id(uid), "lego_comm_unique_id", lib)
    box = [bytes(uid)]
    dist.broadcast_object_list(box, src=0)
    C.memmove(uid, box[0], 128)
    comm = C.c_void_p()
    L.check(lib.lego_comm_create(uid, dist.get_world_size(), dist.get_rank(), device, C.byref(comm)),
            "lego_comm_create", lib)
    # the bound of the native gather's waits: the tooling's environment
    # (LEGO_COMM_TIMEOUT_MS), handed to the library explicitly
    if os.environ.get("LEGO_COMM_TIMEOUT_MS"):
        L.check(lib.lego_comm_set_timeout(comm, max(1, int(os.environ["LEGO_COMM_TIMEOUT_MS"]))),
                "lego_comm_set_timeout", lib)
    return comm


LEGO_COMM_DEVICE_RESULT = 1


def native_gather_handoff(L, comm, ctx, root: int = 0, device: bool = False):
    """lego_comm_gather_handoff(_ex): every rank's last batch packet to root
    over RCCL.  Returns on root the host packets (list per rank) or, with
    device=True (LEGO_COMM_DEVICE_RESULT: no D2H copy, no wait for the
    transfer), the (device pointer, bytes) of each rank's packet, complete once
    lego_comm_wait or a device synchronisation returns; None elsewhere."""
    import ctypes as C

    lib = L.hip_lib()
    if device:
        L.check(lib.lego_comm_gather_handoff_ex(comm, ctx.h, root, LEGO_COMM_DEVICE_RESULT),
                "lego_comm_gather_handoff_ex", lib)
        out = []
        for r in range(10 ** 6):
            ptr, n = C.c_void_p(), C.c_uint64()
            st = lib.lego_comm_handoff_device(comm, r, C.byref(ptr), C.byref(n))
            if st == L.LEGO_E_STATE:
                return None  # not root
            if st != L.LEGO_OK:
                break  # past the last rank
            out.append((ptr.value, n.value))
        return out
    L.check(lib.lego_comm_gather_handoff(comm, ctx.h, root), "lego_comm_gather_handoff", lib)
    out = []
    r = 0
    while True:
        ptr, n = C.c_void_p(), C.c_uint64()
        st = lib.lego_comm_handoff(comm, r, C.byref(ptr), C.byref(n))
        if st == L.LEGO_E_STATE:
            return None  # not root
        if st != L.LEGO_OK:
            break  # past the last rank
        pkt = np.zeros(n.value, np.uint8)
        C.memmove(pkt.ctypes.data, ptr.value, n.value)
        out.append(pkt)
        r += 1
    return out


class Watchdog:
    """Ends a rank that stops making progress, with a message that names the
    step and phase it stalled in, instead of leaving it (and the ranks waiting
    on it in a collective) to the launcher's time limit.

    `mark(step, phase)` records progress; a daemon thread checks every
    `poll_s` seconds and, once `bound_s` seconds pass without a mark while
    armed, writes one line to stderr and calls os._exit(exit_code) — the
    process ends where it stands (no re-exec, no interpreter teardown that
    could block on the device or a collective).  `disarm()` stops the checks.
    A rank whose peer died is itself stuck in that collective until its own
    bound: every rank exits non-zero within about bound_s."""

    def __init__(self, bound_s: float, rank: int = 0, exit_code: int = 3, poll_s: float = 0.25, out=None):
        self.bound_s, self.rank, self.exit_code, self.poll_s = float(bound_s), rank, exit_code, poll_s
        self.out = out if out is not None else sys.stderr
        self._lock = threading.Lock()
        self._t = time.monotonic()
        self._where = (None, "start")
        self._armed = True
        self._thread = threading.Thread(target=self._run, name="lego-watchdog", daemon=True)
        self._thread.start()

    def mark(self, step, phase: str) -> None:
        with self._lock:
            self._t = time.monotonic()
            self._where = (step, phase)

    def disarm(self) -> None:
        with self._lock:
            self._armed = False

    def _run(self) -> None:
        while True:
            time.sleep(self.poll_s)
            with self._lock:
                if not self._armed:
                    return
                idle = time.monotonic() - self._t
                step, phase = self._where
            if idle > self.bound_s:
                try:
                    self.out.write(f"lego watchdog: rank {self.rank} made no progress for {idle:.1f} s "
                                   f"(bound {self.bound_s:g} s) in step {step}, phase '{phase}'; exiting "
                                   f"with status {self.exit_code}\n")
                    self.out.flush()
                finally:
                    os._exit(self.exit_code)


def agree(dist, ok: bool, group=None) -> bool:
    """True on every rank iff `ok` is True on every rank (an all-reduce of a
    failure flag over `group`, the host control channel).  Raises if the
    ranks cannot agree (the process then exits non-zero, as every rank does)."""
    import torch

    t = torch.tensor([0 if ok else 1], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item()) == 0


class HandoffTransport:
    """The per-step hand-off of every rank's packet to rank 0, with ONE
    transport for all ranks at every step.

    `native()` runs the C-ABI collective (lego_comm_gather_handoff_ex) and
    returns rank 0's result; `fallback()` gathers the same step's packet over
    torch.distributed; `abort()` aborts the native communicator (lego_comm_abort:
    cancels a send still queued, so nothing blocks on it later).  After every
    native gather the ranks agree over `ctrl` (a gloo group: host only, never
    queued behind device work) whether it succeeded everywhere.  If any rank
    failed, EVERY rank aborts its communicator, gathers that step again over
    the fallback and stays on the fallback from then on: no rank ever waits in
    ncclGather / ncclRecv while another is in a torch collective."""

    def __init__(self, dist, ctrl, native_ok: bool, native_error: str | None = None):
        self.dist, self.ctrl = dist, ctrl
        self.native = agree(dist, native_ok, ctrl)
        self.errors = self._errors(native_error) if not self.native else []
        self.switched_at = 0 if self.errors else None  # the step from which the fallback runs (None: never switched)
        self.steps = 0
        # this rank's host seconds in the step's gather and in the agreement
        # after it, summed over steps (bench.py reports them per step)
        self.t_gather = 0.0
        self.t_agree = 0.0

    def _errors(self, mine):
        box = [None] * self.dist.get_world_size()
        self.dist.all_gather_object(box, mine, group=self.ctrl)
        return [f"rank {r}: {e}" for r, e in enumerate(box) if e]

    def step(self, native, fallback, abort):
        """One step's gather; returns (transport name, rank 0's result)."""
        out, err = None, None
        if self.native:
            t0 = time.perf_counter()
            try:
                out = native()
            except Exception as e:  # noqa: BLE001
                err = f"step {self.steps}: {e}"
            t1 = time.perf_counter()
            ok = agree(self.dist, err is None, self.ctrl)
            self.t_gather += t1 - t0
            self.t_agree += time.perf_counter() - t1
            if ok:
                self.steps += 1
                return "native", out
            self.native = False
            self.switched_at = self.steps
            self.errors = self._errors(err)
            abort()
        self.steps += 1
        t0 = time.perf_counter()
        out = fallback()
        self.t_gather += time.perf_counter() - t0
        return "fallback", out

    @property
    def name(self) -> str:
        return "native" if self.native else "fallback"
