// fdf.hpp -- header-only C++ mirror of the reference crate API over the C ABI (fdf.h).
//
//   reference (iwanders/feature_detector_fast)          here
//   --------------------------------------------       -----------------------------------
//   Point {x: u32, y: u32}          src/lib.rs:17-20     fdf::Point
//   NonMaximalSuppression           src/lib.rs:26-36     fdf::NonMaximalSuppression
//   Config {threshold,count,nms}    src/lib.rs:40-52     fdf::Config
//   Config::detect(&img)            src/lib.rs:56-58     fdf::Config::detect(img)
//   detect(&img, &config)           src/lib.rs:62-64     fdf::detect(img, config)
//   fast_simd::detector(img, cfg)   src/fast_simd.rs:847 fdf::fast_hip::detector(img, cfg)
//   fast_simd::NORTH..WEST          src/fast_simd.rs:69  fdf::fast_hip::NORTH..WEST
//   fast_simd::circle()             src/fast_simd.rs:79  fdf::fast_hip::circle()
//   fast_simd::calculate_offsets(w) src/fast_simd.rs:104 fdf::fast_hip::calculate_offsets(w)
//   keypoint_score_max_threshold    src/fast_simd.rs:623 fdf::fast_hip::keypoint_score_max_threshold
//   keypoint_score_sum_abs_difference :722               fdf::fast_hip::keypoint_score_sum_abs_difference
//   image::GrayImage                (image 0.24.6)       fdf::GrayView (borrowed row-major u8)
//
// Where the reference panics (n < 9, n > 16, degenerate sizes) these throw fdf::Error.
// Each thread lazily owns one device context per HIP device (device 0 unless
// fdf::set_device() was called), so the free functions stay pure calls like the reference's.
#pragma once

#include <array>
#include <cstdint>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "fdf.h"

namespace fdf {

struct Point {
    uint32_t x = 0;
    uint32_t y = 0;
    bool operator==(const Point& o) const { return x == o.x && y == o.y; }
    bool operator!=(const Point& o) const { return !(*this == o); }
};
static_assert(sizeof(Point) == sizeof(fdf_point), "Point must match the C ABI layout");

enum class NonMaximalSuppression : uint8_t {
    Off = FDF_NMS_OFF,
    MaxThreshold = FDF_NMS_MAX_THRESHOLD,
    SumAbsolute = FDF_NMS_SUM_ABSOLUTE,
};

// A borrowed 8-bit grayscale image: `stride` bytes between rows (GrayImage: == width).
struct GrayView {
    const uint8_t* data = nullptr;
    uint32_t width = 0;
    uint32_t height = 0;
    size_t stride = 0;
    GrayView() = default;
    GrayView(const uint8_t* d, uint32_t w, uint32_t h, size_t s = 0)
        : data(d), width(w), height(h), stride(s ? s : w) {}
};

class Error : public std::runtime_error {
public:
    Error(int status, const std::string& what) : std::runtime_error(what), status_(status) {}
    int status() const { return status_; }

private:
    int status_;
};

inline void check(int status, const char* where) {
    if (status != FDF_OK)
        throw Error(status, std::string(where) + ": " + fdf_status_string(status));
}

// RAII device context (one device, one stream).
class Context {
public:
    explicit Context(int device = 0) {
        fdf_ctx* c = nullptr;
        check(fdf_ctx_create(device, &c), "fdf_ctx_create");
        ctx_.reset(c);
    }
    fdf_ctx* get() const { return ctx_.get(); }

private:
    struct Del {
        void operator()(fdf_ctx* c) const { fdf_ctx_destroy(c); }
    };
    std::unique_ptr<fdf_ctx, Del> ctx_;
};

inline int& current_device() {
    thread_local int dev = 0;
    return dev;
}
inline void set_device(int device) { current_device() = device; }

inline Context& thread_context() {
    thread_local std::vector<std::unique_ptr<Context>> per_device;
    const int dev = current_device();
    if ((int)per_device.size() <= dev) per_device.resize(dev + 1);
    if (!per_device[dev]) per_device[dev].reset(new Context(dev));
    return *per_device[dev];
}

struct Config;
std::vector<Point> detect(const GrayView& img, const Config& config);

struct Config {
    uint8_t threshold = 16;
    uint8_t count = 9;
    NonMaximalSuppression non_maximal_supression = NonMaximalSuppression::Off;

    fdf_config to_c() const {
        fdf_config c;
        c.threshold = threshold;
        c.count = count;
        c.nms = static_cast<uint8_t>(non_maximal_supression);
        return c;
    }
    std::vector<Point> detect(const GrayView& img) const { return fdf::detect(img, *this); }
};

namespace fast_hip {
// First capacity of the two-call pattern: 1 keypoint per 64 pixels (real images have
// 0.5-1.5 per 100).  A denser result is copied out of the context by fdf_fetch_last, so the
// detection runs once either way.
inline size_t capacity_guess(const GrayView& img) {
    const size_t px = (size_t)img.width * img.height;
    return px / 64 > 4096 ? px / 64 : 4096;
}

constexpr size_t NORTH = FDF_NORTH;
constexpr size_t EAST = FDF_EAST;
constexpr size_t SOUTH = FDF_SOUTH;
constexpr size_t WEST = FDF_WEST;

using CircleOffsets = std::array<int32_t, 16>;

inline std::array<std::pair<int32_t, int32_t>, 16> circle() {
    int32_t dx[16], dy[16];
    fdf_circle(dx, dy);
    std::array<std::pair<int32_t, int32_t>, 16> c;
    for (int i = 0; i < 16; ++i) c[i] = {dx[i], dy[i]};
    return c;
}

inline CircleOffsets calculate_offsets(uint32_t width) {
    CircleOffsets o;
    fdf_calculate_offsets(width, o.data());
    return o;
}

// Ring scores on the GPU (fdf_score_rings), one ring per call as the reference's functions;
// batch through fdf_score_rings for many.  `pixels` are the 16 circle pixels in circle() order.
inline uint16_t keypoint_score_max_threshold(uint8_t base_v, const std::array<uint8_t, 16>& pixels,
                                             uint8_t consecutive) {
    fdf_config c{0, consecutive, FDF_NMS_MAX_THRESHOLD};
    uint16_t s = 0;
    check(fdf_score_rings(thread_context().get(), &base_v, pixels.data(), 1, &c, &s),
          "fdf_score_rings");
    return s;
}
inline uint16_t keypoint_score_sum_abs_difference(const std::array<uint8_t, 16>& pixels,
                                                  uint8_t center, uint8_t threshold) {
    fdf_config c{threshold, 9, FDF_NMS_SUM_ABSOLUTE};
    uint16_t s = 0;
    check(fdf_score_rings(thread_context().get(), &center, pixels.data(), 1, &c, &s),
          "fdf_score_rings");
    return s;
}

// Drop-in for fast_simd::detector: result in raster order, bit-identical to the reference.
inline std::vector<Point> detector(const GrayView& img, const Config& config, Context& ctx) {
    const fdf_config c = config.to_c();
    std::vector<Point> out(capacity_guess(img));
    size_t n = 0;
    int rc = fdf_detect(ctx.get(), img.data, img.width, img.height, img.stride, &c,
                        reinterpret_cast<fdf_point*>(out.data()), out.size(), &n);
    if (rc == FDF_ERR_CAPACITY) {   // two-call pattern: copy the retained result
        out.resize(n);
        rc = fdf_fetch_last(ctx.get(), reinterpret_cast<fdf_point*>(out.data()), nullptr,
                            out.size(), &n);
    }
    check(rc, "fdf_detect");
    out.resize(n);
    return out;
}
inline std::vector<Point> detector(const GrayView& img, const Config& config) {
    return detector(img, config, thread_context());
}
}  // namespace fast_hip

inline std::vector<Point> detect(const GrayView& img, const Config& config) {
    return fast_hip::detector(img, config);
}

}  // namespace fdf
