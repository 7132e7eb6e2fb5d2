"""GPU loop closure (lego_mo_loop_closure, mapOptmization.cpp:875-945) vs the
oracle's restatement on the same stream: a synthetic VLP-16 drive in a tight
circle (15 deg/s, 1 m/s: radius 3.8 m) so that after 30 s the robot is back
among keyframes older than the history time window.  Mapping runs on the
keyframe-built map (no fixed map), as loop closure requires.

Bar: detection, keyframe ids and cloud sizes exact; convergence, acceptance
and the ICP iteration count equal; the final transformation, the fitness and
the constraint within 1e-4 (the ICP's reductions run in a different order on
the device)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-4


def test_loop_closure_matches_oracle(L):
    sc = L.synth_cfg("VLP-16", 6, yaw_rate_dps=15.0, speed_mps=1.0)
    cap = L.synth_lib().lego_synth_max_points(L.C.byref(sc))
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=cap)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    checked = accepted = 0
    for k in range(340):
        pts, stamp = L.synth_scan(sc, k)
        gpu.ip(pts, stamp)
        ora.ip(pts, stamp)
        gpu.fa()
        ora.fa()
        gm, om = gpu.mo(), ora.mo()
        assert gm["processed"] == om["processed"]
        if k not in (289, 309, 324, 339):
            continue
        g, o = gpu.loop_closure(), ora.loop_closure()
        for key in ("detected", "latest_id", "closest_id", "n_source", "n_target", "converged", "accepted",
                    "iterations"):
            assert g[key] == o[key], (k, key, g[key], o[key])
        checked += 1
        if not o["detected"]:
            assert k == 289  # no keyframe is 30 s old yet
            continue
        assert abs(g["fitness"] - o["fitness"]) <= TOL * max(1.0, abs(o["fitness"])), (k, g["fitness"], o["fitness"])
        assert np.max(np.abs(g["icp_transform"] - o["icp_transform"])) <= TOL, k
        if o["accepted"]:
            accepted += 1
            for key in ("from_rotation", "from_translation", "to_rotation", "to_translation", "between_rotation",
                        "between_translation"):
                assert np.max(np.abs(g[key] - o[key])) <= TOL, (k, key)
        print(f"scan {k}: keyframes {o['latest_id']} -> {o['closest_id']}, {o['iterations']} ICP iterations, "
              f"fitness {o['fitness']:.4g} (gpu {g['fitness']:.4g}), "
              f"max |dT| {np.max(np.abs(g['icp_transform'] - o['icp_transform'])):.2g}")
    assert checked == 4 and accepted >= 2
    gpu.close()


@pytest.mark.parametrize("search_num", [50, 5])
def test_loop_closure_mode_matches_oracle(L, search_num):
    """loopClosureEnableFlag on (lego_mo_configure): the surrounding map is
    the queue of the most recent keyframes (mapOptmization.cpp:961-999,
    including the refill / pop-push bookkeeping and its duplicate after a
    refill), every keyframe goes into the pose graph, accepted loop closures
    add their factor and the next mapping step re-optimises and corrects every
    keyframe pose (correctPoses :1456-1478).  The product (GPU map and
    keyframe store, host graph) against the oracle's restatement (its own
    cached transformed clouds) over the whole drive, performLoopClosure every
    ten scans once keyframes are 30 s old: decisions and map sizes exact,
    mapped poses within 1e-4 (the loop factor carries the ICP's 1e-6-level
    reduction-order differences into the graph, so after the first loop the
    corrected keyframes can move a boundary point to the next voxel: map sizes
    then within 0.5%)."""
    sc = L.synth_cfg("VLP-16", 6, yaw_rate_dps=15.0, speed_mps=1.0)
    cap = L.synth_lib().lego_synth_max_points(L.C.byref(sc))
    gpu = L.Lego(L.sensor_cfg("VLP-16", L.hip_lib()), max_points=cap)
    ora = L.Oracle(L.sensor_cfg("VLP-16"))
    gpu.mo_configure(loop_closure=True, keyframe_search_num=search_num)
    ora.mo_configure(loop_closure=True, keyframe_search_num=search_num)
    steps = exact = accepted = after = 0
    worst = 0.0
    for k in range(340):
        pts, stamp = L.synth_scan(sc, k)
        gpu.ip(pts, stamp)
        ora.ip(pts, stamp)
        gpu.fa()
        ora.fa()
        gm, om = gpu.mo(), ora.mo()
        assert gm["processed"] == om["processed"], k
        if om["processed"]:
            steps += 1
            after += int(accepted > 0)
            for key in ("optimized", "n_corner_scan_ds", "n_surf_scan_ds"):
                assert gm[key] == om[key], (k, key, gm[key], om[key])
            for key in ("n_corner_map_ds", "n_surf_map_ds"):  # exact until a loop factor enters the graph
                assert abs(gm[key] - om[key]) <= (0 if not accepted else 0.005 * om[key]), (k, key, gm[key], om[key])
            d = float(np.max(np.abs(gm["transform_aft_mapped"].astype(np.float64) - om["transform_aft_mapped"])))
            worst = max(worst, d)
            assert d <= TOL, (k, gm["transform_aft_mapped"], om["transform_aft_mapped"])
            exact += int(np.array_equal(gm["transform_aft_mapped"].view(np.uint32),
                                        om["transform_aft_mapped"].view(np.uint32)))
        if k >= 289 and k % 10 == 9:
            g, o = gpu.loop_closure(), ora.loop_closure()
            for key in ("detected", "latest_id", "closest_id", "accepted"):
                assert g[key] == o[key], (k, key, g[key], o[key])
            accepted += int(o["accepted"])
    gpu.close()
    print(f"loop-closure mode (search num {search_num}): {steps} mapping steps ({after} after the first loop), "
          f"{accepted} loops accepted, worst |dpose| {worst:.3g}, bit-exact {exact}/{steps}")
    assert exact == steps, f"only {exact}/{steps} mapped poses bit-exact"
    assert accepted >= 1 and after >= 3
