"""Probe: do consecutive detector calls gain from running on two streams at once?

Times K back-to-back fdf_detect_device calls over the bench's 512-frame 1080p batch in three
shapes (same frames, same config):
  one_ctx      one context, one stream (the bench's shape: detector, compaction, detector ...)
  two_ctx_1s   two contexts alternating on one stream (same serialisation, two workspaces)
  two_ctx_2s   two contexts on two streams, alternating, no dependency between the streams:
               a call's detector can fill the CUs the other call's tail and compaction leave
Prints one JSON object: ms per call (wall, between synchronizes) per shape.
    python tools/overlap_probe.py [--frames 512] [--steps 50] [--nms maxt]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--nms", default="maxt")
    ap.add_argument("--only", default="", help="time one shape only (under a kernel trace)")
    ap.add_argument("--settle", type=float, default=1.0)
    args = ap.parse_args()
    import torch

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, _native
    import ctypes

    nms = {"off": 0, "maxt": 1, "sad": 2}[args.nms]
    F, W, H = args.frames, 1920, 1080
    frames = workloads.s1_frames_torch(0, F, W, H)
    lib = _native.load()
    ctxs = [_native.Context(0), _native.Context(0)]
    outs = [torch.empty((F * 20_000, 2), dtype=torch.int32, device="cuda") for _ in ctxs]
    offs = [torch.zeros(F + 1, dtype=torch.int64, device="cuda") for _ in ctxs]
    # torch's streams, and the contexts' own HIP streams (created by fdf_ctx_create)
    streams = [torch.cuda.Stream().cuda_stream, torch.cuda.Stream().cuda_stream,
               ctxs[0].stream, ctxs[1].stream]
    cfg = _native.FdfConfig(16, 9, nms)

    def call(i, s):
        rc = lib.fdf_detect_device(ctxs[i].handle, frames.data_ptr(), F, W, H, W * H,
                                   ctypes.byref(cfg), outs[i].data_ptr(), outs[i].shape[0],
                                   offs[i].data_ptr(), ctypes.c_void_p(streams[s]))
        _native.check(rc, "fdf_detect_device")

    shapes = {"one_ctx": lambda k: call(0, 0), "two_ctx_1s": lambda k: call(k & 1, 0),
              "two_ctx_2s": lambda k: call(k & 1, k & 1),
              "two_ctx_own_streams": lambda k: call(k & 1, 2 + (k & 1))}
    if args.only:
        shapes = {args.only: shapes[args.only]}
    # settle: ~1 s of back-to-back launches
    t_end = time.perf_counter() + args.settle
    while time.perf_counter() < t_end:
        for k in range(20):
            call(0, 0)
        torch.cuda.synchronize()
    res = {name: [] for name in shapes}
    for _ in range(args.rounds):
        for name, fn in shapes.items():
            for k in range(4):
                fn(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                fn(k)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) * 1e3 / args.steps)
    same = bool(torch.equal(offs[0], offs[1])) if len(shapes) > 1 else None
    print(json.dumps({"frames": F, "nms": args.nms, "steps": args.steps,
                      "ms_per_call": {k: sorted(v) for k, v in res.items()},
                      "outputs_equal": same}))
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
