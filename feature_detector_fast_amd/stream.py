"""Streaming host pipeline over ``fdf_pipeline_*`` (include/fdf.h): host frames in, host
keypoints out, with H2D copies, detection and D2H copies of consecutive batches overlapped
on per-slot HIP streams.

    pipe = Pipeline(1920, 1080, max_frames=64, depth=3, config=Config(16, 9, MaxThreshold))
    ticket, stage = pipe.acquire()          # pinned (max_frames, H, W) numpy view
    stage[:n] = frames                      # fill in place (no extra copy)
    pipe.submit(ticket, n)
    ...
    points, offsets = pipe.collect(ticket)  # frame f: points[offsets[f]:offsets[f+1]]

``push(frames)`` is acquire + copy + submit.  Tickets are issued in order; ticket k reuses
slot k % depth, so at most ``depth`` batches are outstanding (``FdfError`` with status
FDF_ERR_BUSY beyond that).
"""
import ctypes

import numpy as np

from . import _native
from ._native import FdfError, check
from .fast_hip import _to_c_config


class Pipeline:
    def __init__(self, width, height, max_frames, config, depth=3, rgb=False, scores=False,
                 max_points_per_frame=0, device=0):
        lib = _native.load()
        self._lib = lib
        self.width, self.height, self.max_frames = int(width), int(height), int(max_frames)
        self.rgb, self.scores = bool(rgb), bool(scores)
        flags = (_native.FDF_PIPE_RGB if rgb else 0) | (_native.FDF_PIPE_SCORES if scores else 0)
        self._cfg = _to_c_config(config)
        handle = ctypes.c_void_p()
        check(lib.fdf_pipeline_create(int(device), self.width, self.height, self.max_frames,
                                      int(depth), int(max_points_per_frame), flags,
                                      ctypes.byref(self._cfg), ctypes.byref(handle)),
              "fdf_pipeline_create")
        self.handle = handle
        self._frames = {}                   # ticket -> frames submitted

    @property
    def frame_shape(self):
        return (self.height, self.width, 3) if self.rgb else (self.height, self.width)

    def acquire(self):
        """(ticket, pinned staging array of shape (max_frames,) + frame_shape)."""
        ptr = ctypes.c_void_p()
        ticket = ctypes.c_uint64()
        check(self._lib.fdf_pipeline_acquire(self.handle, ctypes.byref(ptr), ctypes.byref(ticket)),
              "fdf_pipeline_acquire")
        shape = (self.max_frames,) + self.frame_shape
        buf = (ctypes.c_uint8 * int(np.prod(shape))).from_address(ptr.value)
        return ticket.value, np.frombuffer(buf, dtype=np.uint8).reshape(shape)

    def submit(self, ticket, n_frames):
        check(self._lib.fdf_pipeline_submit(self.handle, int(ticket), int(n_frames)),
              "fdf_pipeline_submit")
        self._frames[int(ticket)] = int(n_frames)

    def push(self, frames):
        """Copy (F,) + frame_shape uint8 frames into the next slot and submit; -> ticket."""
        frames = np.ascontiguousarray(frames, dtype=np.uint8)
        if frames.shape[1:] != self.frame_shape:
            raise ValueError(f"frames must be (F,) + {self.frame_shape}")
        ticket = ctypes.c_uint64()
        check(self._lib.fdf_pipeline_push(self.handle, frames.ctypes.data, frames.shape[0],
                                          frames[0].size if frames.shape[0] else 0,
                                          ctypes.byref(ticket)), "fdf_pipeline_push")
        self._frames[ticket.value] = frames.shape[0]
        return ticket.value

    def collect(self, ticket, allow_dropped=False):
        """Wait for ``ticket``: (points (K, 2) uint32, offsets (F+1,) uint64), plus scores
        (K,) uint16 when created with ``scores=True``."""
        ticket = int(ticket)
        nf = self._frames.get(ticket)
        if nf is None:
            raise FdfError(_native.FDF_ERR_ARG, "fdf_pipeline_collect: unknown ticket")
        offsets = np.zeros(nf + 1, dtype=np.uint64)
        n = ctypes.c_size_t(0)
        out = np.empty((0, 2), dtype=np.uint32)
        sc = np.empty(0, dtype=np.uint16)
        rc = self._lib.fdf_pipeline_collect(self.handle, ticket, None, None, 0,
                                            offsets.ctypes.data, ctypes.byref(n))
        if rc == _native.FDF_ERR_CAPACITY:
            out = np.empty((n.value, 2), dtype=np.uint32)
            sc = np.empty(n.value, dtype=np.uint16)
            rc = self._lib.fdf_pipeline_collect(
                self.handle, ticket, out.ctypes.data, sc.ctypes.data if self.scores else None,
                out.shape[0], offsets.ctypes.data, ctypes.byref(n))
        if rc == _native.FDF_ERR_DROPPED and allow_dropped:
            rc = _native.FDF_OK
        self._frames.pop(ticket, None)
        check(rc, "fdf_pipeline_collect")
        out = out[: min(n.value, out.shape[0])]
        if self.scores:
            return out, offsets, sc[: out.shape[0]]
        return out, offsets

    def close(self):
        if self.handle:
            self._lib.fdf_pipeline_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def detect_stream(frame_batches, config, width, height, max_frames, depth=3, rgb=False,
                  scores=False, device=0):
    """Generator: push each (F,) + frame_shape batch, yield its results in order, keeping up
    to ``depth`` batches in flight."""
    with Pipeline(width, height, max_frames, config, depth=depth, rgb=rgb, scores=scores,
                  device=device) as pipe:
        pending = []
        for batch in frame_batches:
            if len(pending) == depth:
                yield pipe.collect(pending.pop(0))
            pending.append(pipe.push(batch))
        for t in pending:
            yield pipe.collect(t)
