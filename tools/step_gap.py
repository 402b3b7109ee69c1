"""Wall time per bench step against the kernels' own durations: how much of a step is the
gap between launches, with the library's per-kernel timing on and off (interleaved rounds).

    python tools/step_gap.py [--frames 512] [--steps 50] [--rounds 3] [--nms maxt]
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
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--nms", default="maxt")
    ap.add_argument("--lib", default="", help="another build of libfdf.so (FDF_LIB_PATH)")
    args = ap.parse_args()
    if args.lib:
        os.environ["FDF_LIB_PATH"] = args.lib
    import torch

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip

    nms = {"off": 0, "maxt": 1, "sad": 2}[args.nms]
    cfg = Config(16, 9, NonMaximalSuppression(nms))
    frames = workloads.s1_frames_torch(0, args.frames, args.width, args.height)
    copies = [frames] + [frames.clone() for _ in range(max(0, (1 << 29) // frames.numel()))]
    out = torch.empty((args.frames * 20_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(args.frames + 1, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    ctx = fast_hip.context(0)
    for k in range(10):
        fast_hip.detect_device(copies[k % len(copies)], cfg, out, offs, stream=stream)
    torch.cuda.synchronize()
    res = {"timing_off": [], "timing_on": [], "kernels_on": []}
    for _ in range(args.rounds):
        for timing in (False, True):
            ctx.set_timing(timing)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                fast_hip.detect_device(copies[k % len(copies)], cfg, out, offs, stream=stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / args.steps
            if timing:
                det, com = ctx.timing_samples()
                res["timing_on"].append(round(ms, 4))
                res["kernels_on"].append(round(float(np.mean(det) + np.mean(com)), 4))
            else:
                res["timing_off"].append(round(ms, 4))
            ctx.set_timing(False)
    summary = {k + "_median": float(np.median(v)) for k, v in res.items()}
    summary["gap_ms_timing_on"] = summary["timing_on_median"] - summary["kernels_on_median"]
    summary["gap_ms_timing_off"] = summary["timing_off_median"] - summary["kernels_on_median"]
    print(json.dumps({"config": vars(args), "rounds": res, "summary": summary}, indent=1))


if __name__ == "__main__":
    main()
