"""Per-launch detector time against time under load, from a cold start: the bench's workload
launched back to back for --seconds, every --every-th launch timed with HIP events (the
library's dispatch-stamped events).  Prints JSON: [(seconds since start, ms), ...] and the
rocm-smi clocks at the end.

    python tools/settle_curve.py --nms maxt --seconds 3
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--nms", default="maxt")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--every", type=int, default=20)
    args = ap.parse_args()
    import torch

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip

    nms = {"off": 0, "maxt": 1, "sad": 2}[args.nms]
    cfg = Config(16, 9, NonMaximalSuppression(nms))
    frames = workloads.s1_frames_torch(0, args.frames)
    out = torch.empty((args.frames * 50_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(args.frames + 1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    ctx = fast_hip.context(0)
    fast_hip.detect_device(frames, cfg, out, offs, stream=stream)
    torch.cuda.synchronize()
    ctx.set_timing(True, every=args.every)
    t0 = time.perf_counter()
    marks = []
    k = 0
    while time.perf_counter() - t0 < args.seconds:
        for _ in range(args.every):
            fast_hip.detect_device(frames, cfg, out, offs, stream=stream)
            k += 1
        torch.cuda.synchronize()
        marks.append(time.perf_counter() - t0)
    det, _ = ctx.timing_samples()
    ctx.set_timing(False)
    n = min(len(det), len(marks))
    curve = [(round(marks[i], 4), round(float(det[i]), 4)) for i in range(n)]
    print(json.dumps({"nms": args.nms, "launches": k, "curve": curve,
                      "first_10_ms": [c[1] for c in curve[:10]],
                      "last_10_ms_mean": round(float(np.mean([c[1] for c in curve[-10:]])), 4)}))


if __name__ == "__main__":
    main()
