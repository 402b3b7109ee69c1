"""Throughput benchmark of the HIP FAST detector (driver contract: one JSON line on rank 0).

A step = one fdf_detect_device call (detector + compaction) over a device-resident batch of
synthetic 1080p frames (S1 "tiled media", workloads.py) per GPU, t=16 n=9 with max-t NMS
(BASELINE.json config 4's per-frame work; weak scaling: every rank owns its own batch, no
collective on the data path).  Inputs are already in HBM when the timed region starts.
Step k runs on launch lane k % L (fast_hip.Lanes, --lanes, default 3): each lane is a
context with its own HIP stream, so consecutive calls overlap on the GPU the way a caller
streaming batches through the public API would run them (extras.single_lane keeps the
one-stream protocol of rounds 1-3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames B] [--nms off|maxt|sad]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

Besides the headline value the line carries: the roofline of the detector (HIP events on the
lane streams; algorithmic bytes = W*H + 8*K + 4 per frame), single-frame
latencies, whole-batch parity (every frame of every input copy against the CPU checker, on
every rank, all-reduced), and the CPU baseline (the AVX2 port of the reference path,
oracle/fast_avx2.cpp, rank 0, N=1).  Each lane reads its own copy of the batch (different
rolls of the S1 frames), so no two launches in flight share input bytes.
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
# launch-duration percentiles need at least this many samples (timed_steps samples the
# launches' own durations in a region of their own: a timestamped dispatch costs queue time)
MIN_TIMED = 10
NMS_NAMES = {"off": 0, "maxt": 1, "sad": 2}


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=10)
    p.add_argument("--settle-seconds", type=float, default=1.0,
                   help="untimed back-to-back launches before the warm-up steps (sustained clocks)")
    p.add_argument("--frames", type=int, default=512, help="frames per GPU per step")
    p.add_argument("--frames-total", type=int, default=0,
                   help="strong scaling: this many frames per step in total, sharded "
                        "contiguously over the ranks (BASELINE config 4: 512); 0 = --frames "
                        "per GPU (weak scaling)")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--threshold", type=int, default=16)
    p.add_argument("--count", type=int, default=9)
    p.add_argument("--nms", choices=sorted(NMS_NAMES), default="maxt")
    p.add_argument("--cpu-seconds", type=float, default=10.0,
                   help="budget for the single-thread CPU baseline sample (0 = skip)")
    p.add_argument("--no-extras", action="store_true", help="skip the latency/leg extras")
    p.add_argument("--no-parity", action="store_true",
                   help="skip the whole-batch parity check of the headline (experiments only)")
    p.add_argument("--copies", type=int, default=0,
                   help="input copies of the shard (0 = one per lane and >= 512 MiB in all; "
                        "1 = every lane reads the same copy, the rounds-1-4 protocol, for A/Bs)")
    p.add_argument("--inline-timing", action="store_true",
                   help="timestamp the timed region's own dispatches (the rounds-1-5 protocol, "
                        "for A/Bs) instead of sampling launch durations in a region of their own")
    p.add_argument("--lanes", type=int, default=3,
                   help="launch lanes: step k runs on lane k %% L, each lane a context with its "
                        "own HIP stream and no dependency between lanes (fast_hip.Lanes)")
    p.add_argument("--ranks-share-device", action="store_true",
                   help="multi-rank runs on a one-GPU box: every rank uses cuda:0, and the "
                        "barrier and reductions go over gloo (the line composes as on N GPUs)")
    p.add_argument("--no-strong-leg", action="store_true",
                   help="N>1: skip extras.config4_strong (BASELINE config 4 as 512 frames in total)")
    p.add_argument("--input", default=os.environ.get("INPUT_FILE", ""),
                   help="an image (PNG/PGM, converted as image 0.24.6 to_luma8) for the "
                        "single-frame GPU and CPU legs, as the reference's bench takes "
                        "INPUT_FILE (benches/benchmark.rs:6-7); the batch stays synthetic")
    return p.parse_args(argv)


# torch.distributed's reductions run on this device ("cpu" under gloo when ranks share a GPU)
_REDUCE_DEVICE = None


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return world, rank, local


def shard_frames(rank, frames_per_rank):
    """Frame indices owned by `rank` (weak scaling: a contiguous block per rank)."""
    return rank * frames_per_rank, frames_per_rank


def strong_shard(rank, world, frames_total):
    """(first, count) of `rank`'s contiguous shard of a `frames_total` batch (strong
    scaling: shard sizes differ by at most one frame)."""
    first = frames_total * rank // world
    return first, frames_total * (rank + 1) // world - first


def percentiles(v):
    v = np.sort(np.asarray(v, dtype=np.float64))
    if len(v) == 0:
        return {}
    q = lambda p: float(v[min(len(v) - 1, int(round(p * (len(v) - 1))))])
    return {"p5": round(q(0.05), 4), "p50": round(q(0.5), 4), "p95": round(q(0.95), 4)}


def median_ci95(v):
    """Median and its distribution-free 95% confidence interval (order statistics)."""
    v = np.sort(np.asarray(v, dtype=np.float64))
    n = len(v)
    lo = max(0, int(np.floor(n / 2 - 1.96 * np.sqrt(n) / 2)) - 1)
    hi = min(n - 1, int(np.ceil(n / 2 + 1.96 * np.sqrt(n) / 2)))
    return float(np.median(v)), [float(v[lo]), float(v[hi])]


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or platform.machine()


def cpu_quota():
    """The cgroup CPU quota in cores (None when unlimited / unknown)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        return None


def reduce_max(value, world, device):
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=_REDUCE_DEVICE or device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def reduce_sum(value, world, device):
    if world == 1:
        return value
    import torch
    import torch.distributed as dist

    t = torch.tensor([value], dtype=torch.float64, device=_REDUCE_DEVICE or device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def barrier(world):
    if world > 1:
        import torch.distributed as dist

        dist.barrier()


def load_traffic(cfg_key, lanes=1):
    """Per-launch HBM bytes from the committed rocprofv3 PMC summary (profiles/
    pmc_traffic.json), and the entry's stamp: (bytes, {"src_sha16", "rev", "stale", "key"}).
    With lanes > 1 the entry profiled under that many lanes (each reading its own input copy,
    tools/profile_round.sh) is preferred.  An entry profiled from other kernel sources than
    the ones in this tree is stale: its bytes are not reported (None) and the stamp says so."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            data = json.load(f)
    except (OSError, ValueError):
        data = {}
    key = f"{cfg_key}_lanes{lanes}" if lanes > 1 and f"{cfg_key}_lanes{lanes}" in data else cfg_key
    entry = data.get(key, {})
    if not entry:
        return None, None
    import workloads
    now = workloads.kernel_source_sha16()
    stamp = {"src_sha16": entry.get("src_sha16"), "rev": entry.get("rev"),
             "stale": entry.get("src_sha16") != now, "key": key}
    return (None if stamp["stale"] else entry.get("hbm_bytes_per_launch")), stamp

def gpu_clocks(device_index):
    """The GPU's current sclk / mclk and package power from rocm-smi (None fields when it
    is missing): taken while the detector runs back to back (see clock_probe)."""
    import subprocess
    res = {"sclk_mhz": None, "mclk_mhz": None, "power_w": None}
    try:
        out = subprocess.run(["rocm-smi", "-d", str(device_index), "--showclocks", "--showpower",
                              "--json"], capture_output=True, text=True, timeout=20).stdout
        card = next(iter(json.loads(out).values()))
    except Exception:                       # noqa: BLE001 -- a missing tool is not an error
        return res
    def mhz(v):
        try:
            return float(str(v).strip("()").lower().replace("mhz", "").split()[0])
        except (ValueError, IndexError):
            return None
    for k, v in card.items():
        kl = k.lower()
        if "sclk" in kl and "clock" in kl and res["sclk_mhz"] is None:
            res["sclk_mhz"] = mhz(v)
        elif "mclk" in kl and "clock" in kl and res["mclk_mhz"] is None:
            res["mclk_mhz"] = mhz(v)
        elif "power" in kl and res["power_w"] is None:
            try:
                res["power_w"] = float(str(v).split()[0])
            except ValueError:
                pass
    return res


def clock_probe(fast_hip, copies, cfg, out, offs, stream, device, seconds=2.0):
    """rocm-smi's clocks and power sampled halfway through ~`seconds` of back-to-back
    detector launches (the bench's own workload), from a helper thread."""
    import threading

    import torch

    sample = {}
    stop = threading.Event()

    def probe():
        stop.wait(seconds / 2)
        sample.update(gpu_clocks(device.index or 0))

    th = threading.Thread(target=probe)
    t0 = time.perf_counter()
    th.start()
    k = 0
    while time.perf_counter() - t0 < seconds:
        for _ in range(10):
            fast_hip.detect_device(copies[k % len(copies)], cfg, out, offs, stream=stream)
            k += 1
        torch.cuda.synchronize()
    th.join()
    idle = gpu_clocks(device.index or 0)
    return {"under_load": sample, "after": idle, "launches": k}


def cpu_baseline(args, nms, single_img=None):
    """The AVX2 port of the reference path (oracle/fast_avx2.cpp) on the host cores, rank 0,
    N=1 (benches/benchmark.rs:18-50 protocol):
      * single frame, 1 thread: NMS off / max-t / SAD, 10 warm-up calls then 100 timed calls
        each, median and its 95% CI (config 1 is the off leg), on `single_img` (--input)
        or one S1 frame;
      * throughput, 1 thread (the headline `cpu_baseline`): 8 S1 frames x N repetitions in
        the bench's NMS mode, ~args.cpu_seconds of CPU work;
      * all cores: the bench's whole S1 batch (args.frames frames), one
        frame at a time per thread, with min(CPUs this process may use, cgroup CPU quota)
        threads, each pinned to its own CPU -- no more threads than the quota runs at once."""
    import workloads
    from oracle import oracle

    W, H = args.width, args.height
    frame = workloads.s1_frame(0, W, H) if single_img is None else single_img
    fh, fw = frame.shape
    single = {}
    for name, mode in (("off", 0), ("maxt", 1), ("sad", 2)):
        ms, kp = oracle.avx2_samples(frame, args.threshold, args.count, mode, 10, 100)
        med, ci = median_ci95(ms)
        single[name] = {"ms_median": round(med, 4), "ms_ci95": [round(ci[0], 4), round(ci[1], 4)],
                        "Mpix_s": round(fw * fh / (med * 1e-3) / 1e6, 1), "keypoints": kp,
                        "warmup": 10, "samples": 100}
    frames = np.stack([workloads.s1_frame(i, W, H) for i in range(8)])
    secs1, _ = oracle.avx2_time(frames[:1], args.threshold, args.count, nms, 1, 1)
    reps = max(1, int(args.cpu_seconds / max(secs1, 1e-6) / len(frames)))
    secs, kp = oracle.avx2_time(frames, args.threshold, args.count, nms, 1, reps)
    px = float(W * H) * len(frames) * reps
    nproc = os.cpu_count() or 1
    base = {"value": round(px / secs / 1e6, 1), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": f"{len(frames)} S1 {W}x{H} frames x {reps} reps, "
                      f"t={args.threshold} n={args.count} nms={args.nms}, 1 thread, "
                      f"AVX2 port of src/fast_simd.rs (oracle/fast_avx2.cpp), {secs:.1f} s",
            "ms_per_frame": round(secs * 1e3 / (len(frames) * reps), 4),
            "cpu": cpu_model(), "nproc": nproc,
            "single_frame_image": args.input or "S1 frame 0",
            "single_frame": single}
    try:
        allowed = sorted(os.sched_getaffinity(0))
    except AttributeError:
        allowed = list(range(nproc))
    quota = cpu_quota()
    threads = max(1, min(len(allowed), int(quota) if quota else len(allowed)))
    cpus = allowed[:threads]
    nb = max(1, args.frames)
    batch = np.stack([workloads.s1_frame(i, W, H) for i in range(nb)])
    per_pass = secs1 * nb / threads
    reps_mt = max(1, int(3.0 / max(per_pass, 1e-6)))
    secs_mt, _ = oracle.avx2_time(batch, args.threshold, args.count, nms, threads, reps_mt,
                                  cpus=cpus)
    del batch
    mt = {"kind": "port", "cpu": cpu_model(), "nproc": nproc, "affinity_cpus": len(allowed),
          "cgroup_cpu_quota": quota, "threads": threads, "pinned": True,
          "cpus": [cpus[0], cpus[-1]], "nms": args.nms,
          "sample": f"{nb} S1 {W}x{H} frames x {reps_mt} passes, frame f on thread f % {threads}, "
                    f"thread i pinned to CPU cpus[i] (sched_setaffinity)",
          "value": round(float(W * H) * nb * reps_mt / secs_mt / 1e6, 1), "unit": "Mpixels/s",
          "seconds": round(secs_mt, 2)}
    return base, mt


def host_latency(fast_hip, _native, frame, cfgs, samples=50):
    """End-to-end fdf_detect on one host 1080p frame -- the literal replacement of
    fast_simd::detector: H2D + detector + compaction + offsets/points D2H, synchronous --
    from pageable numpy memory and from pinned (page-locked) host buffers."""
    import ctypes

    import torch

    lib = _native.load()
    ctx = fast_hip.context(0)
    H, W = frame.shape
    cap = W * H // 8
    res = {}
    pin_in = torch.from_numpy(frame).pin_memory()
    pin_out = torch.empty((cap, 2), dtype=torch.int32).pin_memory()
    np_out = np.empty((cap, 2), dtype=np.uint32)
    for name, (cfg, mode) in cfgs.items():
        c = _native.FdfConfig(cfg.threshold, cfg.count, mode)
        for mem, (src, dst) in (("pageable", (frame.ctypes.data, np_out.ctypes.data)),
                                ("pinned", (pin_in.data_ptr(), pin_out.data_ptr()))):
            n = ctypes.c_size_t(0)
            ts = []
            for k in range(10 + samples):
                t0 = time.perf_counter()
                rc = lib.fdf_detect(ctx.handle, src, W, H, W, ctypes.byref(c), dst, cap,
                                    ctypes.byref(n))
                t1 = time.perf_counter()
                _native.check(rc, "fdf_detect")
                if k >= 10:
                    ts.append((t1 - t0) * 1e3)
            res[f"{name}_{mem}"] = {**percentiles(ts), "keypoints": n.value}
    return res


def config5_4k(fast_hip, Config, NonMaximalSuppression, workloads, lanes, device,
               frames=128, steps=10, warmup=3, settle=0.0):
    """BASELINE.json config 5 on this GPU: 3840x2160 S1 frames, t=8 n=12 (3-of-4 cardinal
    pre-filter), SAD NMS; 128 frames = 1.06 GB, the same bytes per launch as config 4.  Same
    protocol as the headline (timed_steps over `lanes`), plus one lane for the isolated
    kernel."""
    import torch

    from oracle import oracle

    W, H = 3840, 2160
    copies = make_batch(workloads, 0, frames, W, H, device, lanes=len(lanes))
    cfg = Config(8, 12, NonMaximalSuppression.SumAbsolute)
    bufs = LaneBufs(len(lanes), frames * 120_000, frames, device)
    sums_before = [int(c.sum(dtype=torch.int64)) for c in copies]
    t = timed_steps(fast_hip, lanes, bufs, copies, cfg, steps, warmup, 1, settle=settle)
    # parity outside the timed region: every frame of every copy against the CPU checker
    parity, kp_step = batch_parity(oracle, copies, bufs, t, 8, 12, 2, W)
    lanes1 = fast_hip.Lanes(1, device.index or 0)
    buf1 = LaneBufs.__new__(LaneBufs)
    buf1.out, buf1.offs = bufs.out[:1], bufs.offs[:1]
    # (the same sustained-clock settle as the lanes leg: without it this leg read 0.70-0.72 ms
    # per launch against 0.641 settled, profiles/r06/t4_c5ab/)
    t1 = timed_steps(fast_hip, lanes1, buf1, copies, cfg, steps, warmup, 1, settle=settle)
    parity["input_checksums"] = sums_before
    parity["inputs_unchanged"] = [int(c.sum(dtype=torch.int64)) for c in copies] == sums_before
    in_bytes = frames * W * H
    # algorithmic bytes as the headline's: W*H + 8K + 4 per frame
    alg = in_bytes + 8 * kp_step + 4 * frames
    per_launch = t.span_ms / steps
    tbytes, tstamp = load_traffic(f"{W}x{H}_b{frames}_t8_n12_sad", len(lanes))
    det1 = float(np.mean(t1.det)) if len(t1.det) else None
    res = {"workload": f"batch of {frames} {W}x{H} S1 frames, t=8 n=12 nms=sad, "
                       f"{len(copies)} distinct copies (one per lane)",
           "Mpix_s": round(in_bytes * steps / t.elapsed / 1e6, 1),
           "ms_per_step": round(t.elapsed * 1e3 / steps, 4),
           "lanes": t.lanes, "hbm_copies": len(copies),
           "kernel_ms_avg": round(per_launch, 4),
           "launch_ms_avg": round(float(np.mean(t.det)), 4) if len(t.det) else None,
           "launch_ms": percentiles(t.det) if len(t.det) >= MIN_TIMED else None,
           "alg_bytes_per_launch": int(round(alg)),
           "roofline_frac": round(alg / (per_launch * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "roofline_frac_input_bytes_only": round(in_bytes / (per_launch * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "traffic": tbytes, "traffic_stamp": tstamp,
           "traffic_over_alg": round(tbytes / alg, 3) if tbytes else None,
           "single_lane": {"ms_per_step": round(t1.elapsed * 1e3 / steps, 4),
                           "kernel_ms_avg": round(det1, 4) if det1 else None,
                           "kernel_ms": percentiles(t1.det) if len(t1.det) >= MIN_TIMED else None,
                           "compaction_kernel_ms_avg": round(float(np.mean(t1.com)), 4) if len(t1.com) else None,
                           "roofline_frac": round(alg / (det1 * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                           if det1 else None},
           "keypoints_per_step": int(round(kp_step)),
           "parity": parity}
    del copies, bufs
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
    grey_same = n_rgb == n_grey and bool(torch.equal(pts_rgb, out[:n_grey]))
    # the fused path: luma converted in the detector's loads (fdf_detect_device_rgb)
    offs_f = torch.zeros(F + 1, dtype=torch.int64, device=frames.device)
    for _ in range(3):
        fast_hip.detect_device_rgb(rgb, cfg, out, offs_f, stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fast_hip.detect_device_rgb(rgb, cfg, out, offs_f, stream=stream)
    torch.cuda.synchronize()
    elapsed_f = time.perf_counter() - t0
    n_f = int(offs_f[-1].item())
    fused_same = n_f == n_rgb and bool(torch.equal(out[:n_f], pts_rgb))
    gbps = 4.0 * F * H * W / (luma_ms * 1e-3) / 1e9
    res = {"workload": f"batch of {F} {W}x{H} RGB8 frames (grey repeated per channel)",
           "Mpix_s": round(F * H * W * steps / elapsed / 1e6, 1),
           "ms_per_step": round(elapsed * 1e3 / steps, 4),
           "luma_kernel_ms_p50": round(luma_ms, 4),
           "luma_kernel_GBps": round(gbps, 1),
           "luma_roofline_frac": round(gbps / HBM_PEAK_GBS, 4),
           "luma_equals_grey": same,
           "keypoints_per_step": n_rgb,
           "keypoints_equal_grey_path": grey_same,
           "fused_Mpix_s": round(F * H * W * steps / elapsed_f / 1e6, 1),
           "fused_ms_per_step": round(elapsed_f * 1e3 / steps, 4),
           "fused_keypoints_equal_two_pass": fused_same}
    del rgb, grey, pts_rgb
    return res


def input_file_checks(fast_hip, Config, NonMaximalSuppression, workloads, oracle, path, grey,
                      rgb):
    """tests/compare.rs on --input: the five configurations, GPU against the CPU oracle (keypoint
    counts stated, so the README's 23 184 / 7 646 / 8 307 can be checked on its image), and the
    reference's hash guard (compare.rs:83-89: if the RGB bytes hash to its test image's hash,
    the max-t keypoints must hash to 0x8bf9cd0f9ca9ebec)."""
    res = {"path": path, "width": int(grey.shape[1]), "height": int(grey.shape[0]), "configs": {}}
    for name, t, n, m in (("non_max_suppression_t16_c_9", 16, 9, 0), ("max_threshold_t16_c_9", 16, 9, 1),
                          ("sum_absolute_t16_c_9", 16, 9, 2), ("sum_absolute_t16_c_12", 16, 12, 2),
                          ("sum_absolute_t32_c_16", 32, 12, 2)):
        got = fast_hip.detect_array(grey, Config(t, n, NonMaximalSuppression(m)))
        want = oracle.detect(grey, t, n, m)
        res["configs"][name] = {"keypoints": int(len(got)), "bit_exact": bool(np.array_equal(got, want))}
        if m == 1:
            h = workloads.rust_hash_points(got)
            img_h = workloads.rust_hash_bytes(rgb)
            res["hash_keypoints"] = f"0x{h:x}"
            res["reference_test_image"] = img_h == workloads.REF_IMAGE_HASH
            res["hash_guard_ok"] = img_h != workloads.REF_IMAGE_HASH or h == workloads.REF_MAXT_HASH
    return res


COPY_ROLL = 211   # copy c's frame k is S1 frame first + k + 211 c (a different roll)


def n_copies(batch_bytes, lanes, min_bytes):
    """Distinct input copies of a shard: at least one per lane, so no two launches in flight
    read the same bytes, enough to hold >= min_bytes together (a shard
    smaller than the 256 MiB Infinity Cache is still read from HBM on every step), and a
    multiple of the lane count, so lane i always reads copies i, i + L, ..."""
    need = max(1, -(-min_bytes // max(1, batch_bytes))) if min_bytes else 1
    need = max(need, lanes)
    return -(-need // lanes) * lanes


def make_batch(workloads, first, count, W, H, device, min_bytes=0, lanes=1, copies=0):
    """`count` S1 frames from global index `first` in n_copies(...) distinct copies (or
    `copies` when given): copy c holds frames first + 211 c ... (each frame rolled differently
    from the same position in every other copy).  Step k reads copy k % len(copies) on lane
    k % lanes."""
    nc = copies if copies > 0 else n_copies(count * W * H, lanes, min_bytes)
    return [workloads.s1_frames_torch(first + COPY_ROLL * c, count, W, H, device=device)
            for c in range(nc)]


class LaneBufs:
    """Each lane's own output buffers (a lane's call may still run while the next lane's
    writes): `cap` points and count + 1 offsets per lane."""

    def __init__(self, n, cap, count, device):
        import torch

        self.out = [torch.empty((cap, 2), dtype=torch.int32, device=device) for _ in range(n)]
        self.offs = [torch.zeros(count + 1, dtype=torch.int64, device=device) for _ in range(n)]


class Timed:
    """One timed region: wall seconds between barriers + synchronizes, the GPU span of its
    launches from HIP events (lane streams wait on a start event, each records an end event),
    the per-launch detector / compaction durations the library's dispatches timestamped, and
    the lane that ran the last step (its buffers hold the last result)."""

    def __init__(self, elapsed, span_ms, det, com, last, steps, lanes, lane_copy=None,
                 copy_steps=None):
        self.elapsed, self.span_ms, self.det, self.com = elapsed, span_ms, det, com
        self.last, self.steps, self.lanes = last, steps, lanes
        # lane -> the input copy its last call read (its buffers hold that copy's result);
        # copy -> timed steps that read it
        self.lane_copy = lane_copy or {}
        self.copy_steps = copy_steps or {}


def timed_steps(fast_hip, lanes, bufs, copies, cfg, steps, warmup, world, settle=0.0,
                sample=True, inline=False):
    """W warm-up steps, then K timed steps between barriers + synchronizes; one step = one
    fdf_detect_device call over a batch, step k on lane k % L (fast_hip.Lanes: a context and
    its own HIP stream per lane, no dependency between lanes, so a call's detector runs beside
    the previous calls' last workgroups and compaction).  `settle` > 0: before the warm-up
    steps, the same launches back to back for that many seconds (untimed), so the timed steps
    run at the GPU's sustained clocks -- a cold GPU's launches speed up over the first
    ~30 ms of load.  `sample`: the launches' own durations (t.det, t.com) from
    the same calls in a region of their own before the timed one."""
    import torch

    n = len(lanes)
    lane_copy = {}

    def call(k):
        lanes.detect_device(k, copies[k % len(copies)], cfg, bufs.out[k % n], bufs.offs[k % n],
                            after_current=False)
        lane_copy[k % n] = k % len(copies)

    # the lanes do not wait on torch's stream: the inputs and buffers it just made must be done
    torch.cuda.synchronize()

    if settle > 0:
        t_end = time.perf_counter() + settle
        k = 0
        while time.perf_counter() < t_end:
            for _ in range(20):
                call(k)
                k += 1
            torch.cuda.synchronize()
    for k in range(warmup):
        call(k)
    torch.cuda.synchronize()
    # the launches' own durations: HIP events the library's dispatches timestamp on each
    # lane's stream (fdf_ctx_set_timing), sampled in a region of their own before the timed
    # one -- a timestamped dispatch costs queue time (one stream: 0.4367 -> 0.4478 ms per
    # 512-frame step, profiles/r03/l10_gap_*.json), so the timed region runs without them
    det, com = [], []

    def collect():
        for ctx in lanes.ctxs:
            d, c = ctx.timing_samples()
            det.extend(d.tolist())
            com.extend(c.tolist())
            ctx.set_timing(False)

    if sample and not inline:
        for ctx in lanes.ctxs:
            ctx.set_timing(True)
        for k in range(steps):
            call(k)
        torch.cuda.synchronize()
        collect()
    elif sample:
        for ctx in lanes.ctxs:
            ctx.set_timing(True)
    start = torch.cuda.Event(enable_timing=True)
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    start.record(torch.cuda.current_stream())
    for i in range(n):
        lanes.stream(i).wait_event(start)
    for k in range(steps):
        call(k)
    for i in range(n):
        ends[i].record(lanes.stream(i))
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    span_ms = max(start.elapsed_time(e) for e in ends)
    if sample and inline:
        collect()
    copy_steps = {}
    for k in range(steps):
        copy_steps[k % len(copies)] = copy_steps.get(k % len(copies), 0) + 1
    return Timed(elapsed, span_ms, det, com, (steps - 1) % n, steps, n, dict(lane_copy),
                 copy_steps)


def roofline_of(t, alg_bytes, in_bytes, traffic):
    """Roofline of the detector from a timed region `t`: `alg_bytes` = W*H + 8K + 4 per
    frame, `in_bytes` = the input pixels alone; `traffic` is
    load_traffic()'s (bytes, stamp).
      kernel_ms_avg: the detector's GPU time per launch -- the HIP-event span of the timed
        region's launches / launches.  With L > 1 lanes the launches overlap (each one's
        own duration covers the others' beside it), so the span is what a launch costs the
        GPU; with one lane it is each launch's duration plus its compaction and the gaps.
      launch_ms_avg: the mean of the launches' own HIP-event durations (the isolated
        kernel's duration with one lane; with L lanes ~L launches share the GPU in it),
        from the same calls in a sampling region before the timed one (timed_steps).
    Percentiles only from >= MIN_TIMED samples (fewer: the mean alone)."""
    per_launch = t.span_ms / t.steps
    launch = float(np.mean(t.det)) if len(t.det) else float("nan")
    comp = float(np.mean(t.com)) if len(t.com) else float("nan")
    achieved = alg_bytes / (per_launch * 1e-3) / 1e9
    tbytes, tstamp = traffic
    enough = len(t.det) >= MIN_TIMED
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": tbytes,
            "traffic_stamp": tstamp,
            "traffic_over_alg": round(tbytes / alg_bytes, 3) if tbytes else None,
            "kernel": "fast_sweep_kernel", "kernel_ms_avg": round(per_launch, 4),
            "kernel_ms_basis": f"HIP-event span of {t.steps} launches on {t.lanes} lane stream(s) / launches",
            "lanes": t.lanes,
            "launch_ms_avg": round(launch, 4),
            "launch_ms": percentiles(t.det) if enough else None,
            "launches_in_flight_avg": round(launch / per_launch, 3) if per_launch > 0 else None,
            "timed_launches": int(len(t.det)),
            "alg_bytes_per_launch": int(alg_bytes),
            "input_bytes_per_launch": int(in_bytes),
            "frac_input_bytes_only": round(in_bytes / (per_launch * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "compaction_kernel_ms_avg": round(comp, 4),
            "compaction_kernel_ms": percentiles(t.com) if enough else None,
            "measured_achievable_peak": 6290.0}


def raster_order_ok(pts, offsets, W):
    """Keypoints strictly increasing in raster order inside every frame."""
    if len(pts) < 2:
        return True
    key = pts[:, 1].astype(np.int64) * W + pts[:, 0].astype(np.int64)
    inc = np.diff(key) > 0
    # a frame boundary may step back: position offsets[f] - 1 -> offsets[f]
    starts = np.asarray(offsets[1:-1], dtype=np.int64) - 1
    starts = starts[(starts >= 0) & (starts < len(inc))]
    inc[starts] = True
    return bool(np.all(inc))


def batch_parity(oracle, copies, bufs, tm, t, n, nms, W, redo=None):
    """Whole-batch parity outside the timed region (the reference's
    integration test compares the whole output Vec, tests/compare.rs:45-61): every frame of
    every input copy goes through the CPU checker (oracle.avx2_detect_batch: the AVX2 port of
    src/fast_simd.rs over a thread pool, itself pinned to the scalar oracle by
    tests/test_oracle.py), and every copy's GPU result -- offsets and points of all its
    frames -- must equal the checker's: the lanes' last results for the copies they read last,
    and for every other copy one more call after the timed region (`redo(copy)` -> the lane
    whose buffers hold it; ADVICE r05: with more copies than lanes the timed region leaves
    only the last L copies' results).  The scalar oracle (oracle/fast_oracle.c) also checks the
    first, middle and last frame of the last lane's copy directly.  Returns the record and the
    keypoints per timed step (the copies' exact totals weighted by the steps that read them)."""
    ref = {}
    for c in range(len(copies)):
        ref[c] = oracle.avx2_detect_batch(copies[c], t, n, nms)
    count = copies[0].shape[0]
    ok, order_ok, compared = True, True, []

    def compare(lane, c, how):
        nonlocal ok, order_ok
        o = bufs.offs[lane][: count + 1].cpu().numpy().astype(np.uint64)
        total = int(o[-1])
        rp, ro = ref[c]
        if total > bufs.out[lane].shape[0]:
            ok = False
            return
        p = bufs.out[lane][:total].cpu().numpy().astype(np.uint32)
        ok &= bool(np.array_equal(o, ro)) and bool(np.array_equal(p, rp))
        order_ok &= raster_order_ok(p, o, W)
        compared.append({"lane": lane, "copy": c, "frames": count, "keypoints": total,
                         "result": how})

    for lane, c in sorted(tm.lane_copy.items()):
        compare(lane, c, "timed")
    c_last = tm.lane_copy.get(tm.last, 0)
    rp, ro = ref[c_last]
    sampled = sorted({0, count // 2, count - 1})
    scalar_ok = all(bool(np.array_equal(rp[ro[f]:ro[f + 1]],
                                         oracle.detect(copies[c_last][f].cpu().numpy(), t, n, nms)))
                    for f in sampled)
    if redo is not None:
        for c in sorted(set(range(len(copies))) - set(tm.lane_copy.values())):
            compare(redo(c), c, "after")
    kp_per_copy = [int(ref[c][1][-1]) for c in range(len(copies))]
    steps = sum(tm.copy_steps.values()) or 1
    kp_step = sum(kp_per_copy[c] * s for c, s in tm.copy_steps.items()) / steps
    rec = {"oracle_frames": "all", "frames_per_copy": count, "copies_checked": len(copies),
           "copies_compared": len({x["copy"] for x in compared}),
           "lanes_compared": compared, "bit_exact": bool(ok and scalar_ok),
           "gpu_equals_checker_all_frames": bool(ok), "raster_order": order_ok,
           "checker": "oracle.avx2_detect_batch (AVX2 port, pinned to fast_oracle.c)",
           "scalar_oracle_frames": sampled, "scalar_oracle_copy": c_last,
           "scalar_oracle_equal": bool(scalar_ok), "keypoints_per_copy": kp_per_copy}
    return rec, kp_step


def redo_on_lane0(lanes, bufs, copies, cfg):
    """batch_parity's `redo`: copy c once more on lane 0 (synchronised), its result in lane
    0's buffers."""
    import torch

    def redo(c):
        torch.cuda.synchronize()
        lanes.detect_device(0, copies[c], cfg, bufs.out[0], bufs.offs[0], after_current=False)
        torch.cuda.synchronize()
        return 0
    return redo


def shard_leg(fast_hip, workloads, oracle, lanes, cfg, args, world, device, first, count, nms):
    """One frame-sharded leg: `count` frames per call from global frame `first` on the lanes,
    distinct copies, whole-batch parity, its own roofline.  Serves config 4's strong split
    (N > 1) and, at N = 1, the 64-frame shard one GPU of the 8-way split runs (VERDICT r05
    item 6)."""
    W, H = args.width, args.height
    cop = make_batch(workloads, first, count, W, H, device, min_bytes=1 << 29, lanes=args.lanes)
    buf = LaneBufs(len(lanes), max(count, 1) * 200_000, count, device)
    t = timed_steps(fast_hip, lanes, buf, cop, cfg, args.steps, args.warmup, world,
                    settle=args.settle_seconds)
    e = reduce_max(t.elapsed, world, device)
    par, kpf = batch_parity(oracle, cop, buf, t, args.threshold, args.count, nms, W,
                            redo=redo_on_lane0(lanes, buf, cop, cfg))
    kp = int(round(kpf))
    in_bytes = count * W * H
    roof = roofline_of(t, in_bytes + 8 * kp + 4 * count, in_bytes, (None, None))
    del cop, buf
    return t, e, par, kp, roof


def select_device(ranks_share_device, world, local):
    """(GPU index, process-group backend or None) of this rank: one process per GPU, rank
    with LOCAL_RANK r on cuda:r over the default backend ("nccl" = RCCL on ROCm); with
    --ranks-share-device every rank on cuda:0 over gloo (RCCL wants one rank per device)."""
    if ranks_share_device:
        return 0, ("gloo" if world > 1 else None)
    return local, ("nccl" if world > 1 else None)


def main(argv=None):
    args = parse_args(argv)
    world, rank, local = dist_env()
    import torch

    gpu, backend = select_device(args.ranks_share_device, world, local)
    if world > 1:
        import torch.distributed as dist

        global _REDUCE_DEVICE
        if backend == "gloo":
            # several ranks on one GPU: RCCL wants one rank per device, so the barrier and
            # the reductions go over gloo on host tensors (the data path has no collective)
            dist.init_process_group(backend="gloo")
            _REDUCE_DEVICE = "cpu"
        else:
            dist.init_process_group(backend=backend, device_id=torch.device("cuda", gpu))
    torch.cuda.set_device(gpu)
    device = torch.device("cuda", gpu)

    import workloads
    from feature_detector_fast_amd import Config, NonMaximalSuppression, _native, fast_hip
    from oracle import oracle

    nms = NMS_NAMES[args.nms]
    cfg = Config(args.threshold, args.count, NonMaximalSuppression(nms))
    W, H = args.width, args.height
    strong = args.frames_total > 0
    if strong:
        first, count = strong_shard(rank, world, args.frames_total)
    else:
        first, count = shard_frames(rank, args.frames)
    # one distinct copy of the shard per lane at least (no two launches in flight read the
    # same bytes), and >= 512 MiB in all, so that its frames come from HBM, not the 256 MiB
    # Infinity Cache
    copies = make_batch(workloads, first, count, W, H, device, min_bytes=1 << 29,
                        lanes=args.lanes, copies=args.copies)
    frames = copies[0]
    cap = max(count, 1) * 200_000
    stream = torch.cuda.current_stream(device)
    lanes = fast_hip.Lanes(args.lanes, gpu)
    bufs = LaneBufs(len(lanes), cap, count, device)
    ctx = lanes.ctxs[0]
    # lane 0's buffers serve the one-stream extras below
    out, offs = bufs.out[0], bufs.offs[0]

    tm = timed_steps(fast_hip, lanes, bufs, copies, cfg, args.steps, args.warmup, world,
                     settle=args.settle_seconds, inline=args.inline_timing)
    elapsed = reduce_max(tm.elapsed, world, device)

    # ---- whole-batch parity against the CPU checker (outside the timed region), on every
    # rank for its own shard, all-reduced
    parity = {}
    if args.no_parity:
        kp_step = float(np.mean([int(bufs.offs[i][count].item()) for i in tm.lane_copy]))
    else:
        parity, kp_step = batch_parity(oracle, copies, bufs, tm, args.threshold, args.count,
                                       nms, W, redo=redo_on_lane0(lanes, bufs, copies, cfg))
        bad = reduce_sum(0.0 if parity["bit_exact"] else 1.0, world, device)
        parity["ranks"] = {"world": world, "ranks_bit_exact": int(world - bad),
                           "all_ranks_bit_exact": bad == 0,
                           "frames_checked_all_ranks": int(reduce_sum(
                               float(count * len(parity["lanes_compared"])), world, device))}
    total_kp = int(round(kp_step))

    frames_total = reduce_sum(float(count), world, device)
    kp_total = reduce_sum(float(total_kp), world, device)
    pixels = frames_total * W * H
    value = pixels / elapsed * args.steps / 1e6
    ms_per_step = elapsed * 1e3 / args.steps

    # algorithmic bytes of one detector launch: every pixel of every frame
    # read once, plus 8 B per output point and a 4 B count per frame -- W*H + 8K + 4 per
    # frame; the input bytes alone are reported beside it
    in_bytes = count * W * H
    alg_bytes = in_bytes + 8 * total_kp + 4 * count
    cfg_key = f"{W}x{H}_b{count}_t{args.threshold}_n{args.count}_{args.nms}"
    roofline = roofline_of(tm, alg_bytes, in_bytes, load_traffic(cfg_key, len(lanes)))
    roofline["launch_ms_source"] = ("the timed region's own dispatches, timestamped" if args.inline_timing
                                    else "the same calls in a sampling region before the timed one "
                                         "(the timed region's dispatches are not timestamped)")

    extras = {}
    cpu = None
    if not args.no_extras:
        # the GPU's clocks and power while this workload runs back to back (rocm-smi), so a
        # box-to-box difference in kernel time can be told apart from a clock difference
        extras["gpu_clock"] = clock_probe(fast_hip, copies, cfg, out, offs, stream, device)
        # the other NMS modes on the same batch, same protocol: the headline metric is "with
        # and without NMS", and the reference's bench times all three (benches/benchmark.rs:18-50)
        for other in [m for m in ("off", "maxt", "sad") if m != args.nms]:
            ocfg = Config(args.threshold, args.count, NonMaximalSuppression(NMS_NAMES[other]))
            t2 = timed_steps(fast_hip, lanes, bufs, copies, ocfg, args.steps, args.warmup,
                             world, settle=args.settle_seconds)
            e2 = reduce_max(t2.elapsed, world, device)
            par2, kp2f = batch_parity(oracle, copies, bufs, t2, args.threshold, args.count,
                                      NMS_NAMES[other], W,
                                      redo=redo_on_lane0(lanes, bufs, copies, ocfg))
            kp2 = int(round(kp2f))
            leg = {"workload": f"same batch, nms={other}",
                   "value": round(pixels / e2 * args.steps / 1e6, 1), "unit": "Mpixels/s",
                   "ms_per_step": round(e2 * 1e3 / args.steps, 4),
                   "keypoints_per_step": int(reduce_sum(float(kp2), world, device)),
                   "roofline": roofline_of(t2, in_bytes + 8 * kp2 + 4 * count, in_bytes,
                                           load_traffic(f"{W}x{H}_b{count}_t{args.threshold}_n{args.count}_{other}",
                                                        len(lanes))),
                   "parity": par2}
            extras[f"nms_{other}"] = leg
        # the same batch on one lane (one stream: every launch waits for the previous call's
        # compaction): the protocol of rounds 1-3, and the isolated kernel's own duration
        lanes1 = fast_hip.Lanes(1, gpu)
        buf1 = LaneBufs.__new__(LaneBufs)
        buf1.out, buf1.offs = bufs.out[:1], bufs.offs[:1]
        t1 = timed_steps(fast_hip, lanes1, buf1, copies, cfg, args.steps, args.warmup, world,
                         settle=args.settle_seconds)
        e1 = reduce_max(t1.elapsed, world, device)
        kp1 = int(bufs.offs[0][count].item())
        want1 = parity.get("keypoints_per_copy", [None] * len(copies))[t1.lane_copy.get(0, 0)]
        extras["single_lane"] = {
            "workload": "same batch and config, one lane (one stream), the same copies",
            "value": round(pixels / e1 * args.steps / 1e6, 1), "unit": "Mpixels/s",
            "ms_per_step": round(e1 * 1e3 / args.steps, 4),
            "keypoints_equal": want1 is None or kp1 == want1,
            "roofline": roofline_of(t1, in_bytes + 8 * total_kp + 4 * count, in_bytes,
                                    load_traffic(cfg_key))}
    if world > 1 and not strong and not args.no_strong_leg:
        # BASELINE config 4 as defined: 512 frames in total, contiguous shard per GPU (run
        # with --no-extras too: it is the multi-GPU line's own strong-scaling number)
        f4, c4 = strong_shard(rank, world, 512)
        t4, e4, par4, kp4r, roof4 = shard_leg(fast_hip, workloads, oracle, lanes, cfg, args,
                                              world, device, f4, c4, nms)
        kp4 = int(reduce_sum(float(kp4r), world, device))
        bad4 = reduce_sum(0.0 if par4["bit_exact"] else 1.0, world, device)
        extras["config4_strong"] = {
            "workload": f"512 {W}x{H} frames in total, {c4} per GPU (rank {rank}), "
                        f"nms={args.nms}; distinct copies per lane (HBM reads)",
            "value": round(512 * W * H / e4 * args.steps / 1e6, 1), "unit": "Mpixels/s",
            "ms_per_step": round(e4 * 1e3 / args.steps, 4), "scaling": "strong",
            "frames_total": 512, "keypoints_per_step": kp4,
            "lanes": t4.lanes,
            "kernel_ms_avg": round(t4.span_ms / t4.steps, 4),
            "launch_ms_avg": round(float(np.mean(t4.det)), 4) if len(t4.det) else None,
            "roofline_rank0": roof4,
            "parity": {"oracle_frames": "all", "all_ranks_bit_exact": bad4 == 0,
                       "rank0": par4}}
    if world == 1 and not strong and not args.no_extras and not args.no_strong_leg:
        # the per-GPU shard of config 4 split over 8 GPUs (64 frames per call), on this one
        # GPU: the measured basis of the 8-way strong-scaling projection
        c64 = max(1, 512 // 8)
        t6, e6, par6, kp6, roof6 = shard_leg(fast_hip, workloads, oracle, lanes, cfg, args,
                                             world, device, 0, c64, nms)
        ms64 = e6 * 1e3 / args.steps
        extras["shard64"] = {
            "workload": f"{c64} {W}x{H} frames per call (config 4's per-GPU shard at 8 GPUs), "
                        f"nms={args.nms}, {t6.lanes} lanes, distinct copies",
            "value": round(c64 * W * H / e6 * args.steps / 1e6, 1), "unit": "Mpixels/s",
            "ms_per_step": round(ms64, 4), "keypoints_per_step": kp6,
            "roofline": roof6, "parity": par6,
            # 8 GPUs each running this shard against one GPU's 512-frame step / 8
            "projected_8gpu_strong_efficiency": round(ms_per_step / 8 / ms64, 4),
            "projection_basis": "headline ms_per_step / 8 over this leg's ms_per_step; "
                                "the 8-GPU curve itself is unmeasured on hardware"}
    if rank == 0 and not args.no_extras:
        # single-frame latency (device-resident frame, one launch, HIP events), on --input
        # when given (the reference's bench image, benches/benchmark.rs:6-16), else S1 frame 0
        single_img = None
        if args.input:
            import workloads
            single_img, rgb_in = workloads.input_image(args.input)
            extras["input_file"] = input_file_checks(fast_hip, Config, NonMaximalSuppression,
                                                     workloads, oracle, args.input, single_img,
                                                     rgb_in)
            one = torch.from_numpy(single_img).to(device).unsqueeze(0).contiguous()
        else:
            one = frames[:1].contiguous()
        oh, ow = one.shape[1], one.shape[2]
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
            extras[f"single_frame_{name}_Mpix_s"] = round(ow * oh / (lat[len(lat) // 2] * 1e-3) / 1e6, 1)
            extras[f"single_frame_{name}_kp"] = int(offs[1].item())
            # the detector's own duration per call (dispatch-timestamped events, no packets
            # between the kernels): the events above also hold each call's dispatch gap
            sf_ctx = fast_hip.context(device.index or 0)
            sf_ctx.set_timing(True)
            for _ in range(50):
                fast_hip.detect_device(one, c1, out, offs, stream=stream)
            torch.cuda.synchronize()
            det, _ = sf_ctx.timing_samples()
            sf_ctx.set_timing(False)
            if len(det):
                extras[f"single_frame_{name}_kernel_ms_p50"] = round(float(np.median(det)), 4)
        host = one[0].cpu().numpy()
        extras["host_fdf_detect_ms"] = host_latency(
            fast_hip, _native, host,
            {"off": (cfg, 0), "maxt": (cfg, 1)})
        extras["config5_4k"] = config5_4k(fast_hip, Config, NonMaximalSuppression, workloads,
                                          lanes, device,
                                          settle=args.settle_seconds)
        extras["rgb_path"] = rgb_path(fast_hip, cfg, frames, out, offs, stream)
        if world == 1 and args.cpu_seconds > 0:
            cpu, cpu_mt = cpu_baseline(args, nms, single_img)
            extras["cpu_baseline_all_cores"] = cpu_mt
            sf = cpu["single_frame"]
            extras["gpu_vs_cpu_single_frame"] = {
                k: {"cpu_avx2_ms_median": sf[k]["ms_median"],
                    "gpu_fdf_detect_pinned_ms_p50": extras["host_fdf_detect_ms"].get(f"{k}_pinned", {}).get("p50"),
                    "gpu_device_resident_ms_p50": extras.get(f"single_frame_{k}_ms_p50")}
                for k in ("off", "maxt")}

    if rank == 0:
        work = (f"{args.frames_total} {W}x{H} frames per step in total, {count} per GPU"
                if strong else f"batch of {count} {W}x{H} frames per GPU")
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "Mpixels/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "settle_seconds": args.settle_seconds,
            "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "u8",
            "data": "synthetic S1 (committed 300x200 golden fixture tiled, rolled per frame; one distinct copy of the batch per lane)",
            "config": {"workload": f"{work}, t={args.threshold} n={args.count} nms={args.nms}",
                       "frames_per_gpu": count, "width": W, "height": H,
                       "threshold": args.threshold, "count": args.count, "nms": args.nms,
                       "hbm_copies": len(copies),
                       "lanes": len(lanes),
                       "workspace_bytes": sum(c.workspace_bytes() for c in lanes.ctxs),
                       "parallelism": f"frame-sharded x{world} (no collective)",
                       "ranks_share_device": bool(args.ranks_share_device)},
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
