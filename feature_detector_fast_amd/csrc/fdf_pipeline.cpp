// fdf_pipeline.cpp -- streaming host pipeline (include/fdf.h fdf_pipeline_*), built only on
// the public device entry points (fdf_detect_device, fdf_rgb_to_luma_device,
// fdf_score_device).
//
// Each slot owns pinned staging, device buffers and a context with its own HIP stream, so
// the copy engines move batch k+1 in (and batch k-1's offsets out) while the detector runs
// batch k.  A submitted batch is, on its slot's stream:
//   H2D frames -> [RGB -> luma] -> detect (+ compaction) -> [scores] -> D2H offsets -> event.
// Collecting waits on the event, then copies exactly the points found (the count is only
// known on the device until then).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/fdf.h"

namespace {

enum SlotState { kFree = 0, kAcquired = 1, kSubmitted = 2, kWaiting = 3 };

struct Slot {
    fdf_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint8_t* h_frames = nullptr;          // pinned staging (grey or RGB)
    uint64_t* h_offsets = nullptr;        // pinned, max_frames + 1
    uint8_t* d_frames = nullptr;          // as staged
    uint8_t* d_grey = nullptr;            // == d_frames unless RGB
    fdf_point* d_points = nullptr;
    uint16_t* d_scores = nullptr;
    uint64_t* d_offsets = nullptr;
    uint64_t ticket = 0;
    uint32_t n_frames = 0;
    int state = kFree;
    int error = FDF_OK;                   // a failed enqueue, reported by collect
};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

struct fdf_pipeline {
    int device = 0;
    uint32_t width = 0, height = 0, max_frames = 0, depth = 0, flags = 0;
    uint64_t frame_px = 0, frame_in_bytes = 0, cap_points = 0;   // cap per slot
    fdf_config cfg{};
    int empty = 0;                        // shape the reference answers with no points
    uint64_t next_ticket = 0;
    std::mutex mu;
    std::vector<Slot> slots;
};

namespace {

void free_slot(Slot& s) {
    if (s.stream) (void)hipStreamSynchronize(s.stream);
    if (s.done) (void)hipEventDestroy(s.done);
    if (s.h_frames) (void)hipHostFree(s.h_frames);
    if (s.h_offsets) (void)hipHostFree(s.h_offsets);
    if (s.d_grey && s.d_grey != s.d_frames) (void)hipFree(s.d_grey);
    if (s.d_frames) (void)hipFree(s.d_frames);
    if (s.d_points) (void)hipFree(s.d_points);
    if (s.d_scores) (void)hipFree(s.d_scores);
    if (s.d_offsets) (void)hipFree(s.d_offsets);
    if (s.ctx) fdf_ctx_destroy(s.ctx);
    s = Slot{};
}

int alloc_slot(fdf_pipeline* p, Slot& s) {
    int rc = fdf_ctx_create(p->device, &s.ctx);
    if (rc) return rc;
    s.stream = reinterpret_cast<hipStream_t>(fdf_ctx_stream(s.ctx));
    if (hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) return FDF_ERR_DEVICE;
    const uint64_t in_bytes = p->frame_in_bytes * p->max_frames;
    if (hipHostMalloc(reinterpret_cast<void**>(&s.h_frames), std::max<uint64_t>(in_bytes, 1),
                      hipHostMallocDefault) != hipSuccess ||
        hipHostMalloc(reinterpret_cast<void**>(&s.h_offsets),
                      sizeof(uint64_t) * (p->max_frames + 1ull), hipHostMallocDefault) != hipSuccess)
        return FDF_ERR_ALLOC;
    if (p->empty) return FDF_OK;          // nothing is ever sent to the device
    if (hipMalloc(reinterpret_cast<void**>(&s.d_frames), in_bytes) != hipSuccess) return FDF_ERR_ALLOC;
    s.d_grey = s.d_frames;
    if ((p->flags & FDF_PIPE_RGB) &&
        hipMalloc(reinterpret_cast<void**>(&s.d_grey), p->frame_px * p->max_frames) != hipSuccess) {
        s.d_grey = nullptr;
        return FDF_ERR_ALLOC;
    }
    if (hipMalloc(reinterpret_cast<void**>(&s.d_points), sizeof(fdf_point) * p->cap_points) !=
            hipSuccess ||
        hipMalloc(reinterpret_cast<void**>(&s.d_offsets), sizeof(uint64_t) * (p->max_frames + 1ull)) !=
            hipSuccess)
        return FDF_ERR_ALLOC;
    if ((p->flags & FDF_PIPE_SCORES) &&
        hipMalloc(reinterpret_cast<void**>(&s.d_scores), sizeof(uint16_t) * p->cap_points) != hipSuccess)
        return FDF_ERR_ALLOC;
    return FDF_OK;
}

// Enqueue one batch on its slot's stream (lock held by the caller).
int enqueue_batch(fdf_pipeline* p, Slot& s, uint32_t n) {
    if (p->empty) {                       // offsets are all zero; no device work
        std::memset(s.h_offsets, 0, sizeof(uint64_t) * (n + 1ull));
        return hipEventRecord(s.done, s.stream) == hipSuccess ? FDF_OK : FDF_ERR_DEVICE;
    }
    const uint64_t cap = p->cap_points / p->max_frames * n;
    if (hipMemcpyAsync(s.d_frames, s.h_frames, p->frame_in_bytes * n, hipMemcpyHostToDevice,
                       s.stream) != hipSuccess)
        return FDF_ERR_DEVICE;
    int rc;
    if (p->flags & FDF_PIPE_RGB) {
        rc = fdf_rgb_to_luma_device(s.ctx, s.d_frames, n, p->width, p->height, p->frame_in_bytes,
                                    s.d_grey, s.stream);
        if (rc) return rc;
    }
    rc = fdf_detect_device(s.ctx, s.d_grey, n, p->width, p->height, p->frame_px, &p->cfg,
                           s.d_points, cap, s.d_offsets, s.stream);
    if (rc) return rc;
    if (p->flags & FDF_PIPE_SCORES) {
        rc = fdf_score_device(s.ctx, s.d_grey, n, p->width, p->height, p->frame_px, &p->cfg,
                              s.d_points, cap, s.d_offsets, s.d_scores, s.stream);
        if (rc) return rc;
    }
    if (hipMemcpyAsync(s.h_offsets, s.d_offsets, sizeof(uint64_t) * (n + 1ull),
                       hipMemcpyDeviceToHost, s.stream) != hipSuccess ||
        hipEventRecord(s.done, s.stream) != hipSuccess)
        return FDF_ERR_DEVICE;
    return FDF_OK;
}

Slot* slot_of(fdf_pipeline* p, uint64_t ticket) {
    Slot& s = p->slots[ticket % p->depth];
    return s.state != kFree && s.ticket == ticket ? &s : nullptr;
}

}  // namespace

extern "C" {

int fdf_pipeline_create(int device, uint32_t width, uint32_t height, uint32_t max_frames,
                        uint32_t depth, uint64_t max_points_per_frame, uint32_t flags,
                        const fdf_config* cfg, fdf_pipeline** out) {
    if (!out) return FDF_ERR_ARG;
    *out = nullptr;
    int empty = 0;
    int rc = fdf_validate(width, height, cfg, &empty);
    if (rc) return rc;
    if (max_frames == 0 || max_frames > 65535u || depth == 0 || depth > 16 ||
        (flags & ~(uint32_t)(FDF_PIPE_RGB | FDF_PIPE_SCORES)))
        return FDF_ERR_ARG;
    const uint64_t px = (uint64_t)width * height;
    if (px > 0xffffffffull / 3) return FDF_ERR_ARG;
    auto* p = new (std::nothrow) fdf_pipeline;
    if (!p) return FDF_ERR_ALLOC;
    p->device = device;
    p->width = width;
    p->height = height;
    p->max_frames = max_frames;
    p->depth = depth;
    p->flags = flags;
    p->cfg = *cfg;
    p->empty = empty;
    p->frame_px = px;
    p->frame_in_bytes = (flags & FDF_PIPE_RGB) ? 3 * px : px;
    const uint64_t most = empty ? 0 : (uint64_t)(width - 6) * (height - 6);
    const uint64_t per_frame = max_points_per_frame ? std::min(max_points_per_frame, most) : most;
    p->cap_points = std::max<uint64_t>(per_frame, 1) * max_frames;
    DeviceGuard guard(device);
    p->slots.resize(depth);
    for (auto& s : p->slots) {
        if ((rc = alloc_slot(p, s))) {
            fdf_pipeline_destroy(p);
            return rc;
        }
    }
    *out = p;
    return FDF_OK;
}

void fdf_pipeline_destroy(fdf_pipeline* p) {
    if (!p) return;
    {
        DeviceGuard guard(p->device);
        for (auto& s : p->slots) free_slot(s);
    }
    delete p;
}

int fdf_pipeline_acquire(fdf_pipeline* p, uint8_t** frames, uint64_t* ticket) {
    if (!p || !frames || !ticket) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(p->mu);
    Slot& s = p->slots[p->next_ticket % p->depth];
    if (s.state != kFree) return FDF_ERR_BUSY;
    s.state = kAcquired;
    s.ticket = p->next_ticket++;
    s.error = FDF_OK;
    *frames = s.h_frames;
    *ticket = s.ticket;
    return FDF_OK;
}

int fdf_pipeline_submit(fdf_pipeline* p, uint64_t ticket, uint32_t n_frames) {
    if (!p || n_frames == 0) return FDF_ERR_ARG;
    std::lock_guard<std::mutex> lock(p->mu);
    Slot* s = slot_of(p, ticket);
    if (!s || s->state != kAcquired || n_frames > p->max_frames) return FDF_ERR_ARG;
    DeviceGuard guard(p->device);
    s->n_frames = n_frames;
    s->state = kSubmitted;
    s->error = enqueue_batch(p, *s, n_frames);   // reported by collect
    // a batch that failed part-way may still have its frame copy in flight: drain the slot's
    // stream, so that its staging buffer is free once collect releases the slot (the
    // batch's done event was not recorded for this ticket)
    if (s->error) (void)hipStreamSynchronize(s->stream);
    return FDF_OK;
}

int fdf_pipeline_push(fdf_pipeline* p, const uint8_t* frames, uint32_t n_frames,
                      size_t frame_stride_bytes, uint64_t* ticket) {
    if (!p || !frames || !ticket || n_frames == 0 || n_frames > p->max_frames) return FDF_ERR_ARG;
    if (n_frames > 1 && frame_stride_bytes < p->frame_in_bytes) return FDF_ERR_ARG;
    uint8_t* stage = nullptr;
    uint64_t t = 0;
    int rc = fdf_pipeline_acquire(p, &stage, &t);
    if (rc) return rc;
    for (uint32_t f = 0; f < n_frames; ++f)
        std::memcpy(stage + (size_t)f * p->frame_in_bytes, frames + (size_t)f * frame_stride_bytes,
                    p->frame_in_bytes);
    *ticket = t;
    return fdf_pipeline_submit(p, t, n_frames);
}

int fdf_pipeline_collect(fdf_pipeline* p, uint64_t ticket, fdf_point* out,
                         uint16_t* out_scores, size_t cap, uint64_t* frame_offsets,
                         size_t* n_out) {
    if (!p || !n_out || (cap && !out)) return FDF_ERR_ARG;
    Slot* s;
    hipEvent_t done;
    {
        std::lock_guard<std::mutex> lock(p->mu);
        s = slot_of(p, ticket);
        if (!s || (s->state != kSubmitted)) return FDF_ERR_ARG;
        s->state = kWaiting;              // a second collector of this ticket gets FDF_ERR_ARG
        done = s->done;
    }
    DeviceGuard guard(p->device);
    const hipError_t we = s->error ? hipSuccess : hipEventSynchronize(done);
    std::lock_guard<std::mutex> lock(p->mu);
    s->state = kSubmitted;
    if (s->error || we != hipSuccess) {   // a failed batch is dropped with its error
        const int err = s->error ? s->error : FDF_ERR_DEVICE;
        s->state = kFree;
        return err;
    }
    const uint32_t n = s->n_frames;
    const uint64_t total = s->h_offsets[n];
    const uint64_t held = std::min<uint64_t>(total, p->cap_points / p->max_frames * n);
    *n_out = (size_t)total;
    if (frame_offsets) std::memcpy(frame_offsets, s->h_offsets, sizeof(uint64_t) * (n + 1ull));
    if (held > cap) {
        *n_out = (size_t)held;            // what one collect can return
        return FDF_ERR_CAPACITY;
    }
    if (held) {
        hipError_t e = hipMemcpyAsync(out, s->d_points, held * sizeof(fdf_point),
                                      hipMemcpyDeviceToHost, s->stream);
        if (e == hipSuccess && out_scores && (p->flags & FDF_PIPE_SCORES))
            e = hipMemcpyAsync(out_scores, s->d_scores, held * sizeof(uint16_t),
                               hipMemcpyDeviceToHost, s->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
        if (e != hipSuccess) {
            s->state = kFree;
            return FDF_ERR_DEVICE;
        }
    }
    s->state = kFree;
    return held < total ? FDF_ERR_DROPPED : FDF_OK;
}

}  // extern "C"
