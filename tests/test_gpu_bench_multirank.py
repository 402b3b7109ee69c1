"""bench.py's multi-rank path, end to end.

The driver launches `torch.distributed.run --nproc-per-node N bench.py --gpus N` on a whole
node; this pool gives one GPU, so the test runs two ranks on it with --ranks-share-device
(every rank on cuda:0, barrier and reductions over gloo instead of RCCL) as a fresh child
process, and checks the one JSON line rank 0 prints: two ranks, both shards' frames summed
into the value, and BASELINE config 4's strong-scaling leg (512 frames in total) present."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_torchrun_two_ranks_share_device():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--frames", "64", "--steps", "5",
           "--warmup", "2", "--settle-seconds", "0", "--no-extras", "--ranks-share-device"]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    if res.returncode != 0:       # the ranks' own tracebacks, not torchrun's summary
        err = res.stderr
        i = err.find("Traceback")
        raise AssertionError(err[i:i + 4000] if i >= 0 else err[-4000:])
    lines = [l for l in res.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]           # rank 0 alone prints the line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["scaling"] == "weak"
    assert d["config"]["frames_per_gpu"] == 64 and d["config"]["ranks_share_device"]
    # value = all ranks' pixels / the slowest rank's time
    px = 2 * 64 * 1920 * 1080 * 5
    assert d["value"] == pytest.approx(px / (d["ms_per_step"] * 5 * 1e-3) / 1e6, rel=2e-3)
    assert d["keypoints_per_step"] > 0
    strong = d["extras"]["config4_strong"]
    assert strong["frames_total"] == 512 and strong["scaling"] == "strong"
    assert strong["value"] > 0 and strong["keypoints_per_step"] > 0
    assert d["roofline"]["timed_launches"] >= 1
    # every rank checked every frame of every input copy of its own shard (the GPU result of
    # each copy against the CPU checker, plus sampled frames against the scalar oracle),
    # all-reduced
    par = d["parity"]
    assert par["oracle_frames"] == "all" and par["bit_exact"] and par["raster_order"]
    assert par["copies_compared"] == par["copies_checked"] == d["config"]["hbm_copies"]
    assert par["ranks"] == {"world": 2, "ranks_bit_exact": 2, "all_ranks_bit_exact": True,
                            "frames_checked_all_ranks": 2 * 64 * par["copies_compared"]}
    assert d["config"]["hbm_copies"] >= 3
    assert strong["parity"]["all_ranks_bit_exact"] and strong["parity"]["oracle_frames"] == "all"
