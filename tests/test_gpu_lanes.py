"""Back-to-back overlapped device calls: fast_hip.Lanes runs call k on
lane k % L -- a context of its own and that context's HIP stream -- with no dependency
between lanes, so consecutive calls' detectors and compactions run beside each other on the
GPU (bench.py's protocol).  50 calls alternate an S1 batch and a dense mixed batch over 3
lanes, each into its own output buffers; every result must equal the batch's one-lane
result, which equals the CPU oracle (oracle/fast_oracle.c, pinned to the reference's
goldens) on sampled frames.  Both a compaction-sized batch (> 1 024 bands) and a small
direct-output batch are covered."""
import numpy as np
import pytest

import workloads
from feature_detector_fast_amd import Config, NonMaximalSuppression, fast_hip
from oracle import oracle

pytestmark = pytest.mark.gpu


def _batches(nf):
    a = [workloads.s1_frame(3 * i + 1) for i in range(nf)]
    b = [(workloads.s3_frame, workloads.s2_frame, workloads.s1_frame)[i % 3](40 + i) for i in range(nf)]
    return a, b


@pytest.mark.parametrize("nf,nms", [(24, 1), (24, 0), (2, 1)])
def test_lanes_back_to_back(nf, nms):
    import torch

    hosts = _batches(nf)
    frames = [torch.from_numpy(np.stack(h)).cuda() for h in hosts]
    cfg = Config(16, 9, NonMaximalSuppression(nms))
    lanes = fast_hip.Lanes(3)
    try:
        # each batch once, alone: the reference result of the loop below
        ref = []
        for b in range(2):
            cap = nf * 600_000
            out = torch.empty((cap, 2), dtype=torch.int32, device="cuda")
            offs = torch.zeros(nf + 1, dtype=torch.int64, device="cuda")
            lane = lanes.detect_device(b, frames[b], cfg, out, offs)
            lanes.wait(lane)
            torch.cuda.synchronize()
            o = offs.cpu().numpy().copy()
            assert o[-1] <= cap
            ref.append((o, out[: o[-1]].cpu().numpy().astype(np.uint32)))
        for b in range(2):
            o, p = ref[b]
            for f in sorted({0, nf // 2, nf - 1}):
                want = oracle.detect(hosts[b][f], 16, 9, nms)
                assert np.array_equal(p[o[f]:o[f + 1]], want), (b, f)
        # 50 calls back to back over the 3 lanes, every call into its own buffers
        outs, offs = [], []
        for k in range(50):
            n = int(ref[k % 2][0][-1])
            outs.append(torch.full((n + 64, 2), -1, dtype=torch.int32, device="cuda"))
            offs.append(torch.zeros(nf + 1, dtype=torch.int64, device="cuda"))
        for k in range(50):
            lanes.detect_device(k, frames[k % 2], cfg, outs[k], offs[k])
        lanes.wait()
        torch.cuda.synchronize()
        for k in range(50):
            o, p = ref[k % 2]
            assert np.array_equal(offs[k].cpu().numpy(), o), k
            got = outs[k].cpu().numpy()
            assert np.array_equal(got[: o[-1]].astype(np.uint32), p), k
            assert np.all(got[o[-1]:] == -1), k                  # nothing past the total
    finally:
        lanes.close()
