"""The exchanges' steal-on-timeout paths (lego_odom.hip, "exchange" and the
hand-off exchange): nothing assumes the workgroups of an odometry launch are
resident together, so a workgroup that never publishes (lego_ctx_opts::odom_silent_wg,
a diagnostic read at context creation) must only cost time: the others wait
kStealTicks, then compute its NN queries and its share of TransformToEnd
themselves.  The records must equal a normal context's byte for byte:
VLP-16 (LDS-resident: NN exchange) and HDL-64E (HBM-resident: NN and
hand-off exchanges)."""

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pack(scans):
    pts = np.concatenate([p for p, _ in scans])
    off = np.zeros(len(scans) + 1, np.int64)
    off[1:] = np.cumsum([len(p) for p, _ in scans])
    return pts, off, np.array([t for _, t in scans])


@pytest.mark.parametrize("sensor,seed,n,cap", [("VLP-16", 7, 10, 40000), ("HDL-64E", 2, 4, 140000)])
def test_silent_workgroup_is_stolen(L, sensor, seed, n, cap):
    cfg = L.sensor_cfg(sensor, L.hip_lib())
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(n)]
    g = L.Lego(cfg, max_points=cap, max_batch=n)
    want = bytes(g.odom_batch(*_pack(scans)))
    g.close()
    s = L.Lego(cfg, max_points=cap, max_batch=n, opts={"odom_silent_wg": 3})
    got = bytes(s.odom_batch(*_pack(scans)))
    s.close()
    assert [got[64 * k:64 * k + 60] for k in range(n)] == [want[64 * k:64 * k + 60] for k in range(n)]


@pytest.mark.parametrize("sensor,seed,n,cap", [("VLP-16", 7, 12, 40000), ("HDL-64E", 2, 6, 140000)])
def test_late_workgroup_reads_input_state(L, sensor, seed, n, cap):
    """A workgroup dispatched after its stream's lead has finished (and written
    the launch's final OdomState) must still start from the launch's input
    state (OdomBufs::stIn): lego_ctx_opts::odom_late_wg holds one workgroup until the
    lead is done.  Three launches, so the late workgroup's private last clouds
    of launch k feed the NN results it publishes in launch k+1."""
    cfg = L.sensor_cfg(sensor, L.hip_lib())
    sc = L.synth_cfg(sensor, seed)
    scans = [L.synth_scan(sc, k) for k in range(n)]
    per = n // 3

    def run(ctx):
        out = b""
        for b in range(3):
            out += bytes(ctx.odom_batch(*_pack(scans[b * per:(b + 1) * per])))
        return [out[64 * k:64 * k + 60] for k in range(n)]

    g = L.Lego(cfg, max_points=cap, max_batch=per)
    want = run(g)
    g.close()
    s = L.Lego(cfg, max_points=cap, max_batch=per, opts={"odom_late_wg": 5})
    got = run(s)
    s.close()
    assert got == want
