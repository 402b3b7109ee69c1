"""Probe: do consecutive detector calls gain from running on several streams at once?

Times K back-to-back fdf_detect_device calls over a batch of S1 frames, call k on lane
k % L, each lane = its own context (workspace) + the HIP stream fdf_ctx_create made for it,
with no dependency between the lanes: a launch's tail and its compaction leave CUs idle that
the next lane's detector fills.  L = 1 is the bench's one-stream shape.  Also the two-lane
shape on torch streams (`torch2`), which measured no overlap (r04 t1/t2).  Prints one JSON
object: ms per call (wall, between synchronizes) per shape, median of --rounds.
    python tools/overlap_probe.py [--frames 512] [--steps 50] [--nms maxt] [--lanes 1,2,3]
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
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--threshold", type=int, default=16)
    ap.add_argument("--count", type=int, default=9)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--nms", default="maxt")
    ap.add_argument("--lanes", default="1,2", help="comma-separated lane counts to time")
    ap.add_argument("--torch-streams", action="store_true", help="also time 2 lanes on torch streams")
    ap.add_argument("--settle", type=float, default=1.0)
    ap.add_argument("--cap", type=int, default=20_000, help="output points per frame")
    ap.add_argument("--rows", default="0",
                    help="band heights to time (fdf_ctx_set_band_rows on every lane; 0 = automatic)")
    args = ap.parse_args()
    import ctypes

    import torch

    import workloads
    from feature_detector_fast_amd import _native

    nms = {"off": 0, "maxt": 1, "sad": 2}[args.nms]
    F, W, H = args.frames, args.width, args.height
    frames = workloads.s1_frames_torch(0, F, W, H)
    # a batch below 512 MiB rotates through copies (HBM reads, as bench.py)
    copies = [frames] + [frames.clone() for _ in range(max(0, (1 << 29) // frames.numel()))]
    lanes = sorted({int(x) for x in args.lanes.split(",")})
    L = max(lanes + ([2] if args.torch_streams else []))
    lib = _native.load()
    ctxs = [_native.Context(0) for _ in range(L)]
    outs = [torch.empty((F * args.cap, 2), dtype=torch.int32, device="cuda") for _ in ctxs]
    offs = [torch.zeros(F + 1, dtype=torch.int64, device="cuda") for _ in ctxs]
    tstreams = [torch.cuda.Stream().cuda_stream for _ in range(2)]
    cfg = _native.FdfConfig(args.threshold, args.count, nms)

    def call(k, i, stream):
        fr = copies[k % len(copies)]
        rc = lib.fdf_detect_device(ctxs[i].handle, fr.data_ptr(), F, W, H, W * H,
                                   ctypes.byref(cfg), outs[i].data_ptr(), outs[i].shape[0],
                                   offs[i].data_ptr(), ctypes.c_void_p(stream))
        _native.check(rc, "fdf_detect_device")

    def with_rows(r, fn):
        def run(k):
            if k == 0:
                for c in ctxs:
                    c.set_band_rows(r)
            fn(k)
        return run

    shapes = {}
    for r in [int(x) for x in args.rows.split(",")]:
        tag = "" if r == 0 else f"_rows{r}"
        for n in lanes:
            shapes[f"lanes{n}{tag}"] = with_rows(r, (lambda n: lambda k: call(k, k % n, ctxs[k % n].stream))(n))
        if args.torch_streams:
            shapes[f"torch2{tag}"] = with_rows(r, lambda k: call(k, k & 1, tstreams[k & 1]))
    t_end = time.perf_counter() + args.settle
    while time.perf_counter() < t_end:
        for k in range(20):
            call(k, 0, ctxs[0].stream)
        torch.cuda.synchronize()
    res = {name: [] for name in shapes}
    for _ in range(args.rounds):
        for name, fn in shapes.items():
            for k in range(6):
                fn(k)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(args.steps):
                fn(k)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) * 1e3 / args.steps)
    same = all(bool(torch.equal(offs[0], o)) for o in offs[1:])
    total = int(offs[0][-1])
    print(json.dumps({"frames": F, "shape": f"{W}x{H}", "nms": args.nms, "steps": args.steps,
                      "ms_per_call": {k: round(sorted(v)[len(v) // 2], 4) for k, v in res.items()},
                      "ms_per_call_all": {k: [round(x, 4) for x in sorted(v)] for k, v in res.items()},
                      "outputs_equal": same, "points": total,
                      "points_fit": total <= outs[0].shape[0]}))
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
