"""Workgroup timeline of the detector kernel from the debug build's stamps (s_memtime /
s_memrealtime at each workgroup's start and end, its XCD and CU; fdf_kernels.h kStampWords).

    FDF_LIB_PATH=build/libfdf_debug.so python tools/stamps.py --frames 64 512 --nms maxt

For each batch size: the launch's span (first start to last end, real time), the ramp (time
until every CU has started a workgroup), the tail (time from the 90th-percentile end to the
last), workgroup durations, per-XCD spans, the in-kernel shader clock (Δmemtime / Δrealtime x
100 MHz) and the HIP-event duration of the same launches.  Stamps go to their own buffer; this
build's times are for shares, not for quoting.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FDF_LIB_PATH", os.path.join(ROOT, "build", "libfdf_debug.so"))
os.environ["FDF_STAMPS"] = "1"
WORDS = 12


def summarize(st, ntasks_expected):
    t0, t1, r0, r1, ids, task = (st[:, k] for k in range(6))
    ph = st[:, 6:10]
    xcc = (ids >> 32) & 0xF
    hw = ids & 0xFFFFFFFF
    cu = (hw >> 8) & 0xF
    sh = (hw >> 12) & 0x1
    se = (hw >> 13) & 0x7
    cu_key = xcc * 1000 + se * 100 + sh * 16 + cu
    base = r0.min()
    s_us = (r0 - base) / 100.0          # s_memrealtime ticks at 100 MHz
    e_us = (r1 - base) / 100.0
    span = float(e_us.max())
    clocks = (t1 - t0) / np.maximum(r1 - r0, 1) * 100.0   # MHz
    dur = e_us - s_us
    first_per_cu = {}
    for k, s in zip(cu_key, s_us):
        first_per_cu[k] = min(first_per_cu.get(k, 1e18), s)
    xcds = {}
    for x in sorted(set(xcc.tolist())):
        m = xcc == x
        xcds[int(x)] = {"wg": int(m.sum()), "start_us": round(float(s_us[m].min()), 2),
                        "end_us": round(float(e_us[m].max()), 2),
                        "wg_us_mean": round(float(dur[m].mean()), 2)}
    order = np.sort(e_us)
    # phases in shader cycles from the workgroup's start: setup, wave 0's sweep, the rest of
    # the band's sweep (barrier), NMS, look-back (direct output), emit + end
    marks = np.concatenate([t0[:, None], np.where(ph > 0, ph, 0), t1[:, None]], axis=1)
    phases = {}
    names = ["setup", "sweep_wave0", "sweep_rest_and_nms", "lookback", "emit_end"]
    prev = marks[:, 0]
    for k, name in enumerate(names[:-1]):
        m = marks[:, k + 1]
        ok = m > 0
        if ok.any():
            phases[name] = round(float(np.median((m - prev)[ok])), 0)
            prev = np.where(ok, m, prev)
    phases["emit_end"] = round(float(np.median(marks[:, -1] - prev)), 0)
    phases["total_cycles"] = round(float(np.median(t1 - t0)), 0)
    # the four waves' sweep ends (low 32 bits of the shader clock) relative to the start
    ends = np.stack([st[:, 10] & 0xFFFFFFFF, st[:, 10] >> 32, st[:, 11] & 0xFFFFFFFF,
                     st[:, 11] >> 32], axis=1)
    rel = (ends - (t0[:, None] & 0xFFFFFFFF)) % (1 << 32)
    spread = rel.max(axis=1) - rel.min(axis=1)
    waves = {"sweep_end_spread_cycles_p50_p90": [round(float(np.percentile(spread, q)), 0) for q in (50, 90)],
             "spread_over_slowest_sweep_p50": round(float(np.median(spread / np.maximum(rel.max(axis=1), 1))), 3),
             "slowest_wave_share": [round(float(np.mean(rel.argmax(axis=1) == w)), 3) for w in range(4)]}
    # bands running at once (a persistent grid's workgroups run several bands each)
    ev = np.concatenate([np.stack([s_us, np.ones_like(s_us)], 1), np.stack([e_us, -np.ones_like(e_us)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    run = np.cumsum(ev[:, 1])
    dt = np.diff(ev[:, 0], append=ev[-1, 0])
    conc = {"max": int(run.max()), "time_mean": round(float((run * dt).sum() / max(dt.sum(), 1e-9)), 1)}
    return {"phases_cycles_p50": phases, "waves": waves, "concurrent_bands": conc,
        "workgroups": int(len(st)), "ntasks": int(ntasks_expected),
        "span_us": round(span, 2),
        "cus_seen": len(first_per_cu),
        "ramp_us": round(float(max(first_per_cu.values())), 2),
        "start_us_p50_p90_max": [round(float(np.percentile(s_us, q)), 2) for q in (50, 90, 100)],
        "end_us_p10_p50_p90": [round(float(np.percentile(e_us, q)), 2) for q in (10, 50, 90)],
        "tail_us_p90_to_last": round(float(order[-1] - np.percentile(e_us, 90)), 2),
        "wg_us_p5_p50_p95": [round(float(np.percentile(dur, q)), 2) for q in (5, 50, 95)],
        "busy_fraction": round(float(dur.sum() / (span * len(first_per_cu) * 4)), 3),
        "clock_mhz_p50": round(float(np.median(clocks)), 1),
        "xcd": xcds,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, nargs="+", default=[64, 512])
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--threshold", type=int, default=16)
    ap.add_argument("--count", type=int, default=9)
    ap.add_argument("--nms", default="maxt")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--raw", default="", help="write the raw stamps of each batch size here (.npz)")
    ap.add_argument("--host", default="", choices=["", "pinned", "copy"],
                    help="one frame through fdf_detect instead: 'pinned' = read in place from "
                         "pinned host memory, 'copy' = the same buffer copied to the device first")
    args = ap.parse_args()
    import torch

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, _native, fast_hip

    lib = _native.load()
    if not hasattr(lib, "fdf_debug_stamps"):
        sys.exit("fdf_debug_stamps missing: use the debug build (make debug)")
    lib.fdf_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.POINTER(ctypes.c_uint64)]
    lib.fdf_debug_stamps.restype = ctypes.c_int
    nms = {"off": 0, "maxt": 1, "sad": 2}[args.nms]
    cfg = Config(args.threshold, args.count, NonMaximalSuppression(nms))
    stream = torch.cuda.current_stream()
    ctx = fast_hip.context(0)
    res = {}
    raw = {}
    if args.host:
        frame = workloads.s1_frame(0, args.width, args.height)
        pin = torch.from_numpy(frame).pin_memory()
        cap = args.width * args.height // 8
        pout = torch.empty((cap, 2), dtype=torch.int32).pin_memory()
        c = _native.FdfConfig(args.threshold, args.count, nms)
        ctx.set_upload_chunks(1 if args.host == "copy" else 0)
        per = []
        for k in range(5 + args.iters):
            n = ctypes.c_size_t(0)
            _native.check(lib.fdf_detect(ctx.handle, pin.data_ptr(), args.width, args.height,
                                         args.width, ctypes.byref(c), pout.data_ptr(), cap,
                                         ctypes.byref(n)), "fdf_detect")
            if k < 5:
                continue
            m = ctypes.c_uint64(0)
            _native.check(lib.fdf_debug_stamps(ctx.handle, None, 0, ctypes.byref(m)), "stamps")
            buf = np.zeros(m.value, dtype=np.uint64)
            _native.check(lib.fdf_debug_stamps(ctx.handle, buf.ctypes.data, m.value,
                                               ctypes.byref(m)), "stamps")
            st = buf.reshape(-1, WORDS).astype(np.int64)
            per.append(summarize(st, st.shape[0]))
        ctx.set_upload_chunks(0)
        med = sorted(per, key=lambda d: d["span_us"])[len(per) // 2]
        med["span_us_all"] = [p["span_us"] for p in per]
        print(json.dumps({"config": vars(args), "host_frame": med}, indent=1))
        return
    for F in args.frames:
        frames = workloads.s1_frames_torch(0, F, args.width, args.height)
        # copies so that the batch comes from HBM, not the Infinity Cache (as bench.py)
        copies = [frames] + [frames.clone() for _ in range(max(0, (1 << 29) // frames.numel()))]
        out = torch.empty((F * 50_000, 2), dtype=torch.int32, device="cuda")
        offs = torch.zeros(F + 1, dtype=torch.int64, device="cuda")
        for k in range(5):
            fast_hip.detect_device(copies[k % len(copies)], cfg, out, offs, stream=stream)
        torch.cuda.synchronize()
        ctx.set_timing(True)
        per = []
        for k in range(args.iters):
            fast_hip.detect_device(copies[k % len(copies)], cfg, out, offs, stream=stream)
            torch.cuda.synchronize()
            n = ctypes.c_uint64(0)
            _native.check(lib.fdf_debug_stamps(ctx.handle, None, 0, ctypes.byref(n)), "stamps")
            buf = np.zeros(n.value, dtype=np.uint64)
            _native.check(lib.fdf_debug_stamps(ctx.handle, buf.ctypes.data, n.value,
                                               ctypes.byref(n)), "stamps")
            st = buf.reshape(-1, WORDS).astype(np.int64)
            per.append(summarize(st, st.shape[0]))
            if k == args.iters - 1:
                raw[f"f{F}"] = st
        det, _ = ctx.timing_samples()
        ctx.set_timing(False)
        med = sorted(per, key=lambda d: d["span_us"])[len(per) // 2]
        med["event_ms_p50"] = round(float(np.median(det)), 4)
        med["span_us_all"] = [p["span_us"] for p in per]
        res[F] = med
        del copies, frames, out
    if args.raw:
        np.savez_compressed(args.raw, **raw)
    print(json.dumps({"config": vars(args), "by_frames": res}, indent=1))


if __name__ == "__main__":
    main()
