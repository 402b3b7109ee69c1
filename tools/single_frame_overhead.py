"""Where a single device-resident frame's per-call time goes: host enqueue cost versus GPU
time, through fast_hip.detect_device (the Python wrapper) and through a bare ctypes call of
fdf_detect_device with prebuilt arguments.
    python tools/single_frame_overhead.py [--iters 400]
Prints one JSON line per (path, nms): host_us_per_call = wall time of enqueueing the calls
(no synchronisation inside the loop), gpu_us_per_call = event span of the same calls back to
back / calls, event_pair_us_p50 = the bench's protocol (an event pair around every call),
kernel_us_p50 = the detector's own dispatch-timestamped duration (separate run)."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=400)
    args = ap.parse_args()
    import numpy as np
    import torch

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, _native, fast_hip

    one = workloads.s1_frames_torch(0, 1)
    out = torch.empty((200_000, 2), dtype=torch.int32, device="cuda")
    offs = torch.zeros(2, dtype=torch.int64, device="cuda")
    stream = torch.cuda.current_stream()
    ctx = fast_hip.context(0)
    lib = _native.load()
    H, W = one.shape[1], one.shape[2]
    for nms in (0, 1):
        cfg = Config(16, 9, NonMaximalSuppression(nms))
        ccfg = fast_hip._to_c_config(cfg)
        raw_args = (ctx.handle, ctypes.c_void_p(one.data_ptr()), 1, W, H, W * H,
                    ctypes.byref(ccfg), ctypes.c_void_p(out.data_ptr()), out.shape[0],
                    ctypes.c_void_p(offs.data_ptr()), ctypes.c_void_p(stream.cuda_stream))
        fn = lib.fdf_detect_device

        def wrapped():
            fast_hip.detect_device(one, cfg, out, offs, stream=stream)

        def bare():
            fn(*raw_args)

        for name, call in (("fast_hip.detect_device", wrapped), ("ctypes fdf_detect_device", bare)):
            for _ in range(30):
                call()
            torch.cuda.synchronize()
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record(stream)
            t0 = time.perf_counter()
            for _ in range(args.iters):
                call()
            host = (time.perf_counter() - t0) / args.iters * 1e6
            e.record(stream)
            torch.cuda.synchronize()
            gpu = s.elapsed_time(e) / args.iters * 1e3
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(100)]
            for a, b in ev:
                a.record(stream)
                call()
                b.record(stream)
            torch.cuda.synchronize()
            pair = sorted(a.elapsed_time(b) * 1e3 for a, b in ev)
            print(json.dumps({"path": name, "nms": nms, "host_us_per_call": round(host, 2),
                              "gpu_us_per_call": round(gpu, 2),
                              "event_pair_us_p50": round(pair[len(pair) // 2], 2),
                              "keypoints": int(offs[1].item())}), flush=True)
        ctx.set_timing(True)
        for _ in range(100):
            fast_hip.detect_device(one, cfg, out, offs, stream=stream)
        torch.cuda.synchronize()
        det, _ = ctx.timing_samples()
        ctx.set_timing(False)
        print(json.dumps({"path": "kernel (dispatch-timestamped)", "nms": nms,
                          "kernel_us_p50": round(float(np.median(det)) * 1e3, 2)}), flush=True)


if __name__ == "__main__":
    main()
