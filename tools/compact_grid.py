"""Compaction-kernel time across resolutions / NMS modes / thresholds (GPU box, one process).
Prints one line per config: detector ms, compaction ms, keypoints per step."""
import contextlib
import io
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

GRID = [
    ("1920", "1080", "512", "16", "9", "off"),
    ("1920", "1080", "512", "8", "12", "sad"),
    ("1920", "1080", "512", "8", "12", "off"),
    ("3840", "2160", "128", "8", "12", "sad"),
    ("3840", "2160", "128", "8", "12", "off"),
    ("3840", "2160", "128", "16", "9", "off"),
    ("3840", "2160", "128", "16", "9", "maxt"),
]
for w, h, f, t, n, nms in GRID:
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        bench.main(["--width", w, "--height", h, "--frames", f, "--threshold", t, "--count", n,
                    "--nms", nms, "--steps", "10", "--warmup", "3", "--cpu-seconds", "0",
                    "--no-extras"])
    d = json.loads(buf.getvalue().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"{w}x{h} b{f} t{t} n{n} {nms}: sweep {r['kernel_ms_avg']} ms, compact "
          f"{r['compaction_kernel_ms_avg']} ms, step {d['ms_per_step']} ms, kp {d['keypoints_per_step']}", flush=True)
