"""Throughput benchmark of the HIP FAST detector (driver contract: one JSON line on rank 0).

A step = one launch of the fused detector over a device-resident batch of synthetic 1080p
frames (S1 "tiled media", workloads.py) per GPU, t=16 n=9 with max-t NMS (BASELINE.json
config 4's per-frame work; weak scaling: every rank owns its own batch, no collective on
the data path).  Inputs are already in HBM when the timed region starts.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames B] [--nms off|maxt|sad]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Besides the headline value the line carries: the roofline of the detector kernel (HIP
events on the launch stream; algorithmic bytes = W*H + 8*K + 4 per frame),
single-frame latencies, a parity check of sampled frames against the CPU oracle, and the
CPU baseline (the AVX2 port of the reference path, oracle/fast_avx2.cpp, rank 0, N=1).
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpixels/sec 1920x1080 t=16 n=9 (+NMS) at 1/2/4/8 GPUs; keypoints bit-exact"
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s spec (6.29 TB/s measured copy)
NMS_NAMES = {"off": 0, "maxt": 1, "sad": 2}


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--frames", type=int, default=512, help="frames per GPU per step")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--threshold", type=int, default=16)
    p.add_argument("--count", type=int, default=9)
    p.add_argument("--nms", choices=sorted(NMS_NAMES), default="maxt")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="budget for the single-thread CPU baseline sample (0 = skip)")
    p.add_argument("--no-extras", action="store_true", help="skip latency/parity extras")
    return p.parse_args(argv)


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def shard_frames(rank, frames_per_rank):
    """Frame indices owned by `rank` (weak scaling: a contiguous block per rank)."""
    return rank * frames_per_rank, frames_per_rank


def reduce_max(value, world, device):
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(value, world, device):
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def load_traffic(cfg_key):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary, if one matches."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            data = json.load(f)
        return data.get(cfg_key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def cpu_baseline(args, nms):
    """Single-thread AVX2 port of the reference path on a bounded S1 sample (rank 0, N=1)."""
    import workloads
    from oracle import oracle

    frames = np.stack([workloads.s1_frame(i, args.width, args.height) for i in range(8)])
    secs1, _ = oracle.avx2_time(frames[:1], args.threshold, args.count, nms, 1, 1)
    reps = max(1, int(args.cpu_seconds / max(secs1, 1e-6) / len(frames)))
    secs, kp = oracle.avx2_time(frames, args.threshold, args.count, nms, 1, reps)
    px = float(args.width * args.height) * len(frames) * reps
    base = {"value": px / secs / 1e6, "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": f"{len(frames)} S1 {args.width}x{args.height} frames x {reps} reps, "
                      f"t={args.threshold} n={args.count} nms={args.nms}, 1 thread, "
                      f"AVX2 port of src/fast_simd.rs (oracle/fast_avx2.cpp), {secs:.1f} s",
            "ms_per_frame": secs * 1e3 / (len(frames) * reps)}
    threads = min(16, os.cpu_count() or 1)
    reps_mt = max(1, reps * threads // 4)
    secs_mt, _ = oracle.avx2_time(frames, args.threshold, args.count, nms, threads, reps_mt)
    mt = {"value": px / reps * reps_mt / secs_mt / 1e6, "unit": "Mpixels/s", "cores": threads,
          "kind": "port", "cpu": platform.processor() or platform.machine(),
          "nproc": os.cpu_count()}
    return base, mt


def config5_4k(fast_hip, Config, NonMaximalSuppression, workloads, out, stream, device,
               oracle_detect, frames=128, steps=10):
    """BASELINE.json config 5 on this GPU: 3840x2160 S1 frames, t=8 n=12 (3-of-4 cardinal
    pre-filter), SAD NMS; 128 frames = 1.06 GB, the same bytes per launch as config 4."""
    import torch

    W, H = 3840, 2160
    batch = workloads.s1_frames_torch(0, frames, W, H, device=device)
    offs = torch.zeros(frames + 1, dtype=torch.int64, device=device)
    cfg = Config(8, 12, NonMaximalSuppression.SumAbsolute)
    for _ in range(3):
        fast_hip.detect_device(batch, cfg, out, offs, stream=stream)
    ctx = fast_hip.context(device.index or 0)
    ctx.set_timing(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fast_hip.detect_device(batch, cfg, out, offs, stream=stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    calls, sweep_ms, compact_ms = ctx.timing()
    ctx.set_timing(False)
    kernel_ms = sweep_ms / max(calls, 1)
    alg = frames * W * H
    # parity outside the timed region: one more launch must repeat the last one exactly, and
    # frame 0 and the densest frame must equal the CPU oracle
    total = int(offs[-1].item())
    o1 = offs.cpu().numpy().copy()
    p1 = out[: min(total, out.shape[0])].cpu().numpy().copy()
    fast_hip.detect_device(batch, cfg, out, offs, stream=stream)
    torch.cuda.synchronize()
    repeat_ok = bool(np.array_equal(offs.cpu().numpy(), o1)) and bool(
        np.array_equal(out[: len(p1)].cpu().numpy(), p1))
    checked = sorted({0, int(np.argmax(np.diff(o1)))})
    exact = all(np.array_equal(p1[o1[f]:o1[f + 1]].astype(np.uint32),
                               oracle_detect(batch[f].cpu().numpy(), 8, 12, 2)) for f in checked)
    res = {"workload": f"batch of {frames} {W}x{H} S1 frames, t=8 n=12 nms=sad",
           "Mpix_s": round(alg * steps / elapsed / 1e6, 1),
           "ms_per_step": round(elapsed * 1e3 / steps, 4),
           "kernel_ms_avg": round(kernel_ms, 4),
           "compaction_kernel_ms_avg": round(compact_ms / max(calls, 1), 4),
           "roofline_frac": round(alg / (kernel_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "keypoints_per_step": total,
           "parity": {"oracle_frames": checked, "bit_exact": exact, "repeat_identical": repeat_ok}}
    del batch
    return res


def rgb_path(fast_hip, cfg, frames, out, offs, stream, nframes=256, steps=10):
    """SURVEY.md §8 row f4 on this GPU: device-resident RGB8 frames -> rgb_to_luma_kernel ->
    detector.  The RGB frames repeat each grey frame's byte in all three channels, so their
    luma is the grey frame itself and the keypoints must equal the grey path's.  The luma
    kernel moves 4 algorithmic bytes per pixel (3 read, 1 written)."""
    import torch

    F, H, W = min(nframes, frames.shape[0]), frames.shape[1], frames.shape[2]
    grey_in = frames[:F]
    rgb = grey_in.unsqueeze(-1).expand(F, H, W, 3).contiguous()
    grey = torch.empty((F, H, W), dtype=torch.uint8, device=frames.device)
    offs_rgb = torch.zeros(F + 1, dtype=torch.int64, device=frames.device)
    for _ in range(3):
        fast_hip.rgb_to_luma(rgb, grey, stream=stream)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    torch.cuda.synchronize()
    for s, e in ev:
        s.record(stream)
        fast_hip.rgb_to_luma(rgb, grey, stream=stream)
        e.record(stream)
    torch.cuda.synchronize()
    luma_ms = sorted(s.elapsed_time(e) for s, e in ev)[steps // 2]
    for _ in range(3):
        fast_hip.rgb_to_luma(rgb, grey, stream=stream)
        fast_hip.detect_device(grey, cfg, out, offs_rgb, stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fast_hip.rgb_to_luma(rgb, grey, stream=stream)
        fast_hip.detect_device(grey, cfg, out, offs_rgb, stream=stream)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    same = bool(torch.equal(grey, grey_in))
    n_rgb = int(offs_rgb[-1].item())
    pts_rgb = out[:n_rgb].clone()
    fast_hip.detect_device(grey_in, cfg, out, offs, stream=stream)
    torch.cuda.synchronize()
    n_grey = int(offs[F].item())
    gbps = 4.0 * F * H * W / (luma_ms * 1e-3) / 1e9
    res = {"workload": f"batch of {F} {W}x{H} RGB8 frames (grey repeated per channel)",
           "Mpix_s": round(F * H * W * steps / elapsed / 1e6, 1),
           "ms_per_step": round(elapsed * 1e3 / steps, 4),
           "luma_kernel_ms_p50": round(luma_ms, 4),
           "luma_kernel_GBps": round(gbps, 1),
           "luma_roofline_frac": round(gbps / HBM_PEAK_GBS, 4),
           "luma_equals_grey": same,
           "keypoints_per_step": n_rgb,
           "keypoints_equal_grey_path": n_rgb == n_grey and bool(torch.equal(pts_rgb, out[:n_grey]))}
    del rgb, grey, pts_rgb
    return res


def main(argv=None):
    args = parse_args(argv)
    world, rank, local = dist_env()
    import torch

    if world > 1:
        import torch.distributed as dist

        dist.init_process_group(backend="nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip
    from oracle import oracle

    nms = NMS_NAMES[args.nms]
    cfg = Config(args.threshold, args.count, NonMaximalSuppression(nms))
    W, H, B = args.width, args.height, args.frames
    first, count = shard_frames(rank, B)
    frames = workloads.s1_frames_torch(first, count, W, H, device=device)
    cap = B * 200_000
    out = torch.empty((cap, 2), dtype=torch.int32, device=device)
    offs = torch.zeros(B + 1, dtype=torch.int64, device=device)
    stream = torch.cuda.current_stream(device)

    for _ in range(args.warmup):
        fast_hip.detect_device(frames, cfg, out, offs, stream=stream)
    torch.cuda.synchronize()

    # HIP events recorded by the library on the launch stream around each of its two kernels
    # (fdf_ctx_set_timing): the detector kernel's own duration, live in the timed region
    ctx = fast_hip.context(local)
    ctx.set_timing(True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        fast_hip.detect_device(frames, cfg, out, offs, stream=stream)
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    elapsed = reduce_max(elapsed, world, device)
    calls, sweep_ms_total, compact_ms_total = ctx.timing()
    ctx.set_timing(False)
    sweep_ms_avg = sweep_ms_total / max(calls, 1)
    compact_ms_avg = compact_ms_total / max(calls, 1)

    total_kp = int(offs[-1].item())
    offsets = offs.cpu().numpy()

    # ---- parity of sampled frames against the CPU oracle (outside the timed region)
    parity = {}
    if not args.no_extras:
        pts = out[: min(total_kp, cap)].cpu().numpy().astype(np.uint32)
        ok = True
        checked = []
        for f in sorted({0, count // 2, count - 1}):
            want = oracle.detect(frames[f].cpu().numpy(), args.threshold, args.count, nms)
            ok &= bool(np.array_equal(pts[offsets[f]:offsets[f + 1]], want))
            checked.append(first + f)
        order_ok = True
        for f in range(count):   # raster order inside every frame (size-independent property)
            seg = pts[offsets[f]:offsets[f + 1]].astype(np.int64)
            if len(seg) > 1:
                key = seg[:, 1] * W + seg[:, 0]
                order_ok &= bool(np.all(np.diff(key) > 0))
        parity = {"oracle_frames": checked, "bit_exact": ok, "raster_order": order_ok}

    frames_total = reduce_sum(float(count), world, device)
    kp_total = reduce_sum(float(total_kp), world, device)
    pixels = frames_total * W * H
    value = pixels / elapsed * args.steps / 1e6
    ms_per_step = elapsed * 1e3 / args.steps

    # algorithmic bytes of one detector launch: every pixel of every frame read once
    # (DESIGN.md §5); the whole call adds the output points and frame offsets
    alg_bytes = count * W * H
    call_bytes = alg_bytes + 8 * total_kp + 8 * (count + 1)
    achieved = alg_bytes / (sweep_ms_avg * 1e-3) / 1e9
    cfg_key = f"{W}x{H}_b{B}_t{args.threshold}_n{args.count}_{args.nms}"
    roofline = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(cfg_key), "kernel": "fast_sweep_kernel",
                "kernel_ms_avg": round(sweep_ms_avg, 4), "timed_launches": calls,
                "alg_bytes_per_launch": alg_bytes,
                "compaction_kernel_ms_avg": round(compact_ms_avg, 4),
                "call_GBps": round(call_bytes / ((sweep_ms_avg + compact_ms_avg) * 1e-3) / 1e9, 1),
                "measured_achievable_peak": 6290.0}

    extras = {}
    cpu = None
    if rank == 0 and not args.no_extras:
        # single-frame latency (device-resident frame, one launch, HIP events)
        one = frames[:1].contiguous()
        for name, mode in (("off", 0), ("maxt", 1)):
            c1 = Config(args.threshold, args.count, NonMaximalSuppression(mode))
            for _ in range(10):
                fast_hip.detect_device(one, c1, out, offs, stream=stream)
            torch.cuda.synchronize()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                  for _ in range(50)]
            for s, e in ev:
                s.record(stream)
                fast_hip.detect_device(one, c1, out, offs, stream=stream)
                e.record(stream)
            torch.cuda.synchronize()
            lat = sorted(s.elapsed_time(e) for s, e in ev)
            extras[f"single_frame_{name}_ms_p50"] = round(lat[len(lat) // 2], 4)
            extras[f"single_frame_{name}_Mpix_s"] = round(W * H / (lat[len(lat) // 2] * 1e-3) / 1e6, 1)
            extras[f"single_frame_{name}_kp"] = int(offs[1].item())
        extras["config5_4k"] = config5_4k(fast_hip, Config, NonMaximalSuppression, workloads,
                                          out, stream, device, oracle.detect)
        extras["rgb_path"] = rgb_path(fast_hip, cfg, frames, out, offs, stream)
        if world == 1 and args.cpu_seconds > 0:
            cpu, cpu_mt = cpu_baseline(args, nms)
            extras["cpu_baseline_all_cores"] = cpu_mt

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "Mpixels/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic S1 (committed 300x200 golden fixture tiled, rolled per frame)",
            "config": {"workload": f"batch of {B} {W}x{H} frames per GPU, t={args.threshold} "
                                   f"n={args.count} nms={args.nms}",
                       "frames_per_gpu": B, "width": W, "height": H,
                       "threshold": args.threshold, "count": args.count, "nms": args.nms,
                       "parallelism": f"frame-sharded x{world} (no collective)"},
            "keypoints_per_step": int(kp_total),
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
            "extras": extras,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.destroy_process_group()


if __name__ == "__main__":
    main()
