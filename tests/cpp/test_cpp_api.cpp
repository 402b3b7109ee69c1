// C++ API smoke test (include/fdf.hpp), run by tests/test_gpu_parity.py on a GPU box.
// Usage: test_cpp_api <image.pgm> <expected_off.txt> <expected_maxt.txt>
// Mirrors tests/compare.rs:66-81 of the reference: detect with t=16 n=9 off and max-t and
// compare the Vec<Point> for exact (ordered) equality with the golden lists.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "fdf.hpp"

static bool read_pgm(const char* path, std::vector<uint8_t>& px, uint32_t& w, uint32_t& h) {
    std::ifstream f(path, std::ios::binary);
    std::string magic;
    int maxv = 0;
    if (!(f >> magic >> w >> h >> maxv) || magic != "P5" || maxv != 255) return false;
    f.get();
    px.resize((size_t)w * h);
    return (bool)f.read(reinterpret_cast<char*>(px.data()), px.size());
}

static std::vector<fdf::Point> read_points(const char* path) {
    std::vector<fdf::Point> pts;
    std::ifstream f(path);
    fdf::Point p;
    while (f >> p.x >> p.y) pts.push_back(p);
    return pts;
}

int main(int argc, char** argv) {
    if (argc != 4) {
        std::fprintf(stderr, "usage: %s image.pgm off.txt maxt.txt\n", argv[0]);
        return 2;
    }
    std::vector<uint8_t> px;
    uint32_t w = 0, h = 0;
    if (!read_pgm(argv[1], px, w, h)) {
        std::fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    const fdf::GrayView img(px.data(), w, h);
    int failures = 0;

    fdf::Config off{16, 9, fdf::NonMaximalSuppression::Off};
    const auto got_off = fdf::detect(img, off);
    if (got_off != read_points(argv[2])) {
        std::fprintf(stderr, "NMS off: %zu points differ from golden\n", got_off.size());
        ++failures;
    }
    fdf::Config maxt{16, 9, fdf::NonMaximalSuppression::MaxThreshold};
    const auto got_maxt = maxt.detect(img);
    if (got_maxt != read_points(argv[3])) {
        std::fprintf(stderr, "max-t: %zu points differ from golden\n", got_maxt.size());
        ++failures;
    }
    // the reference panics for n < 9; here that is an exception carrying FDF_ERR_COUNT
    try {
        fdf::Config bad{16, 8, fdf::NonMaximalSuppression::Off};
        (void)fdf::detect(img, bad);
        std::fprintf(stderr, "count 8 did not throw\n");
        ++failures;
    } catch (const fdf::Error& e) {
        if (e.status() != FDF_ERR_COUNT) ++failures;
    }
    // ring helpers: circle / offsets (src/fast_simd.rs:79-110) and the score KAT of
    // test_47_115_score_calc (src/fast_simd.rs:919-948): centre 17, n = 9 -> 20
    namespace fh = fdf::fast_hip;
    if (fh::circle()[fh::EAST] != std::make_pair(3, 0) || fh::calculate_offsets(w)[fh::NORTH] != -3 * (int32_t)w) {
        std::fprintf(stderr, "circle / offsets differ\n");
        ++failures;
    }
    const std::array<uint8_t, 16> ring{37, 37, 39, 39, 37, 42, 43, 16, 14, 13, 15, 16, 15, 38, 37, 38};
    if (fh::keypoint_score_max_threshold(17, ring, 9) != 20) {
        std::fprintf(stderr, "max-t KAT: %u != 20\n", fh::keypoint_score_max_threshold(17, ring, 9));
        ++failures;
    }
    std::printf("off=%zu maxt=%zu failures=%d\n", got_off.size(), got_maxt.size(), failures);
    return failures ? 1 : 0;
}
