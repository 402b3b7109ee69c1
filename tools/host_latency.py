"""End-to-end fdf_detect on one host 1080p frame (the literal fast_simd::detector replacement:
H2D, detection, D2H, synchronous), pinned and pageable, p5/p50/p95 per mode.  Under
rocprofv3 --kernel-trace --memory-copy-trace it shows where a call's time goes.
    python tools/host_latency.py [--iters 200] [--modes off,maxt] [--mem pinned,pageable]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--modes", default="off,maxt")
    ap.add_argument("--mem", default="pinned,pageable")
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--chunks", default="0,1",
                    help="fdf_ctx_set_upload_chunks values to time (0 = default, 1 = one copy)")
    ap.add_argument("--rows", default="0",
                    help="fdf_ctx_set_band_rows values to time (0 = automatic)")
    args = ap.parse_args()
    import torch

    import workloads
    from feature_detector_fast_amd import _native, fast_hip

    frame = workloads.s1_frame(0, args.width, args.height)
    H, W = frame.shape
    lib = _native.load()
    ctx = fast_hip.context(0)
    cap = W * H // 8
    pin_in = torch.from_numpy(frame).pin_memory()
    pin_out = torch.empty((cap, 2), dtype=torch.int32).pin_memory()
    np_out = np.empty((cap, 2), dtype=np.uint32)
    res = {}
    for name, mem, ch, rows in [(n, m, c, r) for n in args.modes.split(",")
                                for m in args.mem.split(",") for c in args.chunks.split(",")
                                for r in args.rows.split(",")]:
        mode = {"off": 0, "maxt": 1, "sad": 2}[name]
        c = _native.FdfConfig(16, 9, mode)
        ctx.set_upload_chunks(int(ch))
        ctx.set_band_rows(int(rows))
        src, dst = ((pin_in.data_ptr(), pin_out.data_ptr()) if mem == "pinned"
                    else (frame.ctypes.data, np_out.ctypes.data))
        n = ctypes.c_size_t(0)
        ts = []
        for k in range(20 + args.iters):
            t0 = time.perf_counter()
            rc = lib.fdf_detect(ctx.handle, src, W, H, W, ctypes.byref(c), dst, cap,
                                ctypes.byref(n))
            t1 = time.perf_counter()
            _native.check(rc, "fdf_detect")
            if k >= 20:
                ts.append((t1 - t0) * 1e3)
        ts = np.sort(ts)
        q = lambda p: round(float(ts[int(p * (len(ts) - 1))]), 4)
        key = (f"{name}_{mem}" + ("" if ch == "0" else f"_chunks{ch}") +
               ("" if rows == "0" else f"_rows{rows}"))
        res[key] = {"p5": q(0.05), "p50": q(0.5), "p95": q(0.95), "keypoints": n.value}
    ctx.set_band_rows(0)
    ctx.set_upload_chunks(0)
    res["recoveries"] = list(ctx.recoveries())    # (upload fallbacks, look-back recoveries)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
