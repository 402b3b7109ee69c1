"""PCIe-inclusive throughput of the streaming host pipeline (fdf_pipeline_*): host frames in,
host keypoints out, 1080p, the bench workload's content (workloads.s1_frame).

Two producer models:
  in_place  -- the producer writes straight into the pinned staging (acquire/submit), so
               the host-side cost is only the collect copy of the keypoints;
  push      -- frames come from ordinary (pageable) memory and are memcpy'd into staging.
Prints one JSON line per (mode, nms).  Not the bench `value` (that is HBM-resident input).

    python tools/stream_bench.py [--frames-per-batch 32] [--batches 24] [--depth 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import workloads  # noqa: E402
from feature_detector_fast_amd import Config, NonMaximalSuppression  # noqa: E402
from feature_detector_fast_amd.stream import Pipeline  # noqa: E402


def run(mode, nms, fpb, batches, depth, src):
    W, H = 1920, 1080
    cfg = Config(16, 9, NonMaximalSuppression(nms))
    with Pipeline(W, H, fpb, cfg, depth=depth, max_points_per_frame=200_000) as pipe:
        if mode == "in_place":     # fill every slot's staging once, then reuse it
            staged = []
            for _ in range(depth):
                t, stage = pipe.acquire()
                stage[:] = src[:fpb]
                pipe.submit(t, fpb)
                staged.append(t)
            for t in staged:
                pipe.collect(t)

        def issue():
            if mode == "push":
                return pipe.push(src[:fpb])
            t, _ = pipe.acquire()
            pipe.submit(t, fpb)
            return t

        pending, points = [], 0
        for _ in range(depth):     # warm-up
            pending.append(issue())
        for t in pending:
            pipe.collect(t)
        pending = []
        t0 = time.perf_counter()
        for _ in range(batches):
            if len(pending) == depth:
                points += len(pipe.collect(pending.pop(0))[0])
            pending.append(issue())
        for t in pending:
            points += len(pipe.collect(t)[0])
        dt = time.perf_counter() - t0
    px = batches * fpb * W * H
    return {"tool": "stream_bench", "mode": mode, "nms": nms, "frames_per_batch": fpb,
            "batches": batches, "depth": depth, "Mpix_per_s": round(px / dt / 1e6, 1),
            "frames_per_s": round(batches * fpb / dt, 1),
            "h2d_GBps": round(px / dt / 1e9, 2), "keypoints": points}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames-per-batch", type=int, default=32)
    ap.add_argument("--batches", type=int, default=24)
    ap.add_argument("--depth", type=int, default=3)
    a = ap.parse_args()
    src = np.stack([workloads.s1_frame(i) for i in range(a.frames_per_batch)])
    for mode in ("in_place", "push"):
        for nms in (1, 0):
            print(json.dumps(run(mode, nms, a.frames_per_batch, a.batches, a.depth, src)),
                  flush=True)


if __name__ == "__main__":
    main()
