"""Single-frame latency, direct output (look-back, one launch) against detector + compaction
(two launches), interleaved in one process on the debug build (FDF_DIRECT=0/1 is read at
every enqueue).  Per call: HIP events around it on the stream, isolated calls (the stream
idles between them) and back-to-back calls.
    FDF_LIB_PATH=build/libfdf_debug.so python tools/direct_ab.py [--rounds 5]"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FDF_LIB_PATH", os.path.join(ROOT, "build", "libfdf_debug.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    args = ap.parse_args()
    import torch

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip

    one = workloads.s1_frames_torch(0, 1, args.width, args.height)
    out = torch.empty((400_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(2, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    res = {}
    for r in range(args.rounds):
        for nms in (0, 1):
            for direct in ("1", "0"):
                os.environ["FDF_DIRECT"] = direct
                cfg = Config(16, 9, NonMaximalSuppression(nms))
                for _ in range(5):
                    fast_hip.detect_device(one, cfg, out, offs, stream=stream)
                torch.cuda.synchronize()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(args.iters)]
                for s, e in ev:            # isolated: the host waits between calls
                    s.record(stream)
                    fast_hip.detect_device(one, cfg, out, offs, stream=stream)
                    e.record(stream)
                    e.synchronize()
                iso = sorted(s.elapsed_time(e) for s, e in ev)[args.iters // 2]
                s = torch.cuda.Event(enable_timing=True)
                e = torch.cuda.Event(enable_timing=True)
                s.record(stream)
                for _ in range(args.iters):
                    fast_hip.detect_device(one, cfg, out, offs, stream=stream)
                e.record(stream)
                torch.cuda.synchronize()
                key = f"{'maxt' if nms else 'off'}_direct{direct}"
                d = res.setdefault(key, {"isolated_ms_p50": [], "back_to_back_ms": [],
                                         "keypoints": int(offs[1].item())})
                d["isolated_ms_p50"].append(round(iso, 4))
                d["back_to_back_ms"].append(round(s.elapsed_time(e) / args.iters, 4))
    os.environ.pop("FDF_DIRECT", None)
    for d in res.values():
        d["isolated_median"] = float(np.median(d["isolated_ms_p50"]))
        d["back_to_back_median"] = float(np.median(d["back_to_back_ms"]))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
