"""Host-side bench.py logic (CPU): the kernel-timing sample interval and the roofline fields
built from a timed region (one definition of the algorithmic bytes,
percentiles only from enough samples)."""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


@pytest.mark.parametrize("steps,every", [(1, 1), (10, 1), (19, 1), (20, 2), (50, 5), (500, 5)])
def test_timing_every(steps, every):
    assert bench.timing_every(steps) == every
    # the driver's 20 steps sample 10 launches, the default 50 steps 10
    assert steps // every >= min(steps, bench.MIN_TIMED)


def test_roofline_from_timed_region():
    W, H, F, K = 1920, 1080, 512, 2_000_000
    in_bytes = F * W * H
    alg = in_bytes + 8 * K + 4 * F
    # 3 lanes, 20 launches spanning 8.0 ms of GPU time, each launch 1.2 ms long on its own
    t = bench.Timed(elapsed=0.0081, span_ms=8.0, det=[1.2] * 20, com=[0.015] * 20, last=1,
                    steps=20, lanes=3)
    r = bench.roofline_of(t, alg, in_bytes, (None, None))
    assert r["kernel_ms_avg"] == pytest.approx(0.4)
    assert r["achieved"] == pytest.approx(alg / 0.4e-3 / 1e9, rel=1e-4)
    assert r["frac"] == pytest.approx(r["achieved"] / 8000.0, rel=1e-3)
    assert r["frac_input_bytes_only"] < r["frac"]
    assert r["alg_bytes_per_launch"] == alg and r["input_bytes_per_launch"] == in_bytes
    assert r["launches_in_flight_avg"] == pytest.approx(3.0)
    assert r["launch_ms"] is not None and r["timed_launches"] == 20
    few = bench.Timed(0.001, 1.0, [0.4] * 4, [0.01] * 4, 0, 4, 1)
    r4 = bench.roofline_of(few, alg, in_bytes, (None, None))
    assert r4["launch_ms"] is None and r4["compaction_kernel_ms"] is None    # mean only
