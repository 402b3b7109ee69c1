"""In-process A/B timing of detector variants (cdna_hip_programming.md §5.4 rule 24).

Variants are selected through FDF_DEBUG_FLAGS (internal ablation switches of the band
kernel, fdf_kernels.h) and the NMS mode; rounds are interleaved in one process on one
device, and the median/min per variant are printed as JSON.
    python tools/ablate.py [--frames 512] [--rounds 5] [--iters 10]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# the ablation switches exist only in the debug build (make debug)
os.environ.setdefault("FDF_LIB_PATH", os.path.join(ROOT, "build", "libfdf_debug.so"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--threshold", type=int, default=16)
    ap.add_argument("--count", type=int, default=9)
    ap.add_argument("--variants", default="maxt:0,maxt:2,maxt:3,off:0,off:2,off:3,sad:0")
    ap.add_argument("--log-geometry", action="store_true",
                    help="debug build: print each launch's band geometry to stderr")
    args = ap.parse_args()
    if args.log_geometry:
        os.environ["FDF_GEOMETRY_LOG"] = "1"
    import torch

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip

    frames = workloads.s1_frames_torch(0, args.frames, args.width, args.height)
    out = torch.empty((args.frames * 50_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(args.frames + 1, dtype=torch.int64, device="cuda")
    modes = {"off": 0, "maxt": 1, "sad": 2}
    # mode:flags[:lds_budget[:nsub[:rows[:margin]]]] -- budget (bytes per workgroup), sub-bands
    # per band, band rows (fdf_ctx_set_band_rows) and the NMS density margin (debug build)
    # override the geometry pick (0 = default)
    variants = [tuple(v.split(":")) for v in args.variants.split(",")]
    times = {v: [] for v in variants}
    stream = torch.cuda.current_stream()
    ctx = fast_hip.context(0)
    for r in range(args.rounds):
        for v in variants:
            mode, flags = v[0], v[1]
            os.environ["FDF_DEBUG_FLAGS"] = str(int(flags, 0))
            for k, name in ((2, "FDF_LDS_BUDGET"), (3, "FDF_NSUB"), (5, "FDF_DENSITY_MARGIN")):
                if len(v) > k and v[k] != "0":
                    os.environ[name] = v[k]
                else:
                    os.environ.pop(name, None)
            ctx.set_band_rows(int(v[4]) if len(v) > 4 else 0)
            cfg = Config(args.threshold, args.count, NonMaximalSuppression(modes[mode]))
            fast_hip.detect_device(frames, cfg, out, offs, stream=stream)
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record(stream)
            for _ in range(args.iters):
                fast_hip.detect_device(frames, cfg, out, offs, stream=stream)
            e.record(stream)
            torch.cuda.synchronize()
            times[v].append(s.elapsed_time(e) / args.iters)
    os.environ.pop("FDF_DEBUG_FLAGS", None)
    ctx.set_band_rows(0)
    px = args.frames * args.width * args.height
    res = {}
    for v, ts in times.items():
        med = float(np.median(ts))
        res[":".join(v)] = {"ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                                       "Gpix_s": round(px / med / 1e6, 1)}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
