"""The HBM-resident odometry's ring of hand-off slots (k_odom<true>,
OdomBufs::ring; featureAssociation.cpp:1759-1815 keeps one last cloud and
kd-tree per node) across launches whose scans do not rebuild the index.

A hand-off rebuilds the clouds' index only when laserCloudCornerLastNum > 10
and laserCloudSurfLastNum > 100 (featureAssociation.cpp:1785-1788); the
others keep the last snapshot.  Every hand-off still takes the next slot of
the ring, skipping the snapshot's, and k_ring_prep zeroes the control words of
exactly the slots the launch will pick.  With a ring of K + 3 = 5 slots
(batches of at most 2 scans): full scans 0, 1 (scan 1's slot becomes the
snapshot), three degenerate scans (a 3-degree sector: fewer than 100
less-flat points, no rebuild) that walk the ring past the snapshot, then a
batch whose first scan rebuilds and whose second scan's pick reaches the old
snapshot's slot.  Before round 5 the kernel skipped the snapshot as it stood
at that moment (the new one) while k_ring_prep had skipped the old one, so
the second scan used a slot whose control words still held an old launch's
claims: wrong clouds, no error.  Every pose is compared bit for
bit with the oracle's."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _sector(p, half_deg):
    a = np.degrees(np.arctan2(p["y"], p["x"]))
    return np.ascontiguousarray(p[np.abs(a - 90.0) < half_deg])


def test_snapshot_slot_after_degenerate_scans(L):
    sensor = "HDL-64E"
    sc = L.synth_cfg(sensor, 2)
    full = [L.synth_scan(sc, k) for k in range(12)]
    plan = [[0, 1], [2, 3], [4], [5, 6], [7, 8], [9], [10, 11]]
    degenerate = {2, 3, 4, 9}
    scans = [(_sector(p, 1.5), s) if k in degenerate else (p, s) for k, (p, s) in enumerate(full)]
    ora = L.Oracle(L.sensor_cfg(sensor))
    ref, counts = [], []
    for p, s in scans:
        ora.ip(p, s)
        f = ora.fa()
        ref.append(f["transform_sum"].astype(np.float32))
        counts.append((len(f["less_sharp"]), len(f["less_flat"])))
    # the premise: the degenerate scans do not rebuild, the full ones do
    for k in range(len(scans)):
        rebuild = counts[k][0] > 10 and counts[k][1] > 100
        assert rebuild == (k not in degenerate), (k, counts[k])
    g = L.Lego(L.sensor_cfg(sensor, L.hip_lib()), max_points=max(len(p) for p, _ in scans) + 16, max_batch=2)
    recs = []
    try:
        for b in plan:
            pts = np.concatenate([scans[k][0] for k in b])
            off = np.zeros(len(b) + 1, np.int64)
            off[1:] = np.cumsum([len(scans[k][0]) for k in b])
            recs.extend(g.odom_batch(pts, off, np.array([scans[k][1] for k in b])))
    finally:
        g.close()
    assert len(recs) == len(scans)
    for k, r in enumerate(recs):
        got = np.array(list(r.transform_sum), np.float32)
        assert (r.n_less_sharp, r.n_less_flat) == counts[k], k
        assert np.array_equal(got.view(np.uint32), ref[k].view(np.uint32)), (k, got, ref[k])
