"""Single device-resident 1080p frame, repeated: for rocprofv3 --kernel-trace (kernel
durations and the gaps between them) and HIP-event latency per call.
    python tools/single_frame.py [--nms off|maxt] [--iters 200]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nms", default="maxt")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--rows", type=int, default=0, help="fdf_ctx_set_band_rows (0 = automatic)")
    args = ap.parse_args()
    import torch

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip

    nms = {"off": 0, "maxt": 1, "sad": 2}[args.nms]
    one = workloads.s1_frames_torch(0, 1)
    out = torch.empty((200_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(2, dtype=torch.int64, device="cuda")
    cfg = Config(16, 9, NonMaximalSuppression(nms))
    stream = torch.cuda.current_stream()
    fast_hip.context(0).set_band_rows(args.rows)
    for _ in range(20):
        fast_hip.detect_device(one, cfg, out, offs, stream=stream)
    torch.cuda.synchronize()
    ctx = fast_hip.context(0)
    ctx.set_timing(True)
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    s.record(stream)
    for _ in range(args.iters):
        fast_hip.detect_device(one, cfg, out, offs, stream=stream)
    e.record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.iters * 1e3
    det, com = ctx.timing_samples()
    ctx.set_timing(False)
    # back-to-back calls: the stream never idles, so the event span / calls is the throughput
    # latency; each call alone is bounded below by its two kernels
    print(json.dumps({"nms": args.nms, "calls": args.iters, "rows": args.rows,
                      "event_ms_per_call": round(s.elapsed_time(e) / args.iters, 4),
                      "host_wall_ms_per_call": round(wall, 4),
                      "sweep_ms_p50": round(float(sorted(det)[len(det) // 2]), 4),
                      "compact_ms_p50": round(float(sorted(com)[len(com) // 2]), 4),
                      "keypoints": int(offs[1].item())}))


if __name__ == "__main__":
    main()
