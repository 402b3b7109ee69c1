// Host round trip of one tiny launch on this runtime: launch + blocking
// hipStreamSynchronize, launch + hipStreamQuery poll, the cost of hipPointerGetAttributes, and
// how fast kernels read a 1080p frame (2 073 600 B) of pinned host memory over the link, each
// byte once, by grid size.
//   hipcc --offload-arch=gfx950 -O2 tools/microbench/sync_latency.hip -o build/sync_latency
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void touch(uint32_t* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

// writes `seq` to a host-mapped word with a system-scope release (a vector store)
__global__ void touch_flag(uint32_t* flag, uint32_t seq) {
    if (threadIdx.x == 0 && blockIdx.x == 0)
        __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// each thread reads 16-byte words i, i + stride, ... of the buffer and folds them into one
// word per thread (written, so the loads are not dead)
__global__ void read_all(const uint4* __restrict__ p, size_t n16, uint32_t* sink) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    sink[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(
               std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void report(const char* name, std::vector<double>& v) {
    std::sort(v.begin(), v.end());
    std::printf("{\"case\": \"%s\", \"p5_us\": %.2f, \"p50_us\": %.2f, \"p95_us\": %.2f}\n", name,
                v[v.size() / 20], v[v.size() / 2], v[v.size() * 19 / 20]);
}

int main() {
    uint32_t* d = nullptr;
    hipStream_t s;
    if (hipMalloc(&d, 4) != hipSuccess || hipStreamCreate(&s) != hipSuccess) return 1;
    uint8_t* h = nullptr;
    if (hipHostMalloc(&h, 1 << 21, hipHostMallocNonCoherent) != hipSuccess) return 1;
    const int iters = 2000;
    for (int mode = 0; mode < 2; ++mode) {
        std::vector<double> t;
        for (int i = 0; i < iters + 100; ++i) {
            const double t0 = now_us();
            touch<<<1, 64, 0, s>>>(d);
            if (mode == 0) {
                (void)hipStreamSynchronize(s);
            } else {
                while (hipStreamQuery(s) == hipErrorNotReady) __builtin_ia32_pause();
            }
            if (i >= 100) t.push_back(now_us() - t0);
        }
        report(mode == 0 ? "launch+hipStreamSynchronize" : "launch+hipStreamQuery_poll", t);
    }
    {
        // round 6: the host waits for a word the kernel writes to pinned host memory instead
        // of the runtime's completion (the stream is drained afterwards, untimed)
        uint32_t* hf = nullptr;
        uint32_t* df = nullptr;
        if (hipHostMalloc(&hf, 64, hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer(reinterpret_cast<void**>(&df), hf, 0) != hipSuccess)
            return 1;
        *hf = 0;
        std::vector<double> t, tsync;
        for (int i = 0; i < iters + 100; ++i) {
            const uint32_t seq = (uint32_t)i + 1;
            const double t0 = now_us();
            touch_flag<<<1, 64, 0, s>>>(df, seq);
            while (__atomic_load_n(reinterpret_cast<volatile uint32_t*>(hf), __ATOMIC_ACQUIRE) != seq)
                __builtin_ia32_pause();
            const double t1 = now_us();
            (void)hipStreamSynchronize(s);
            const double t2 = now_us();
            if (i >= 100) {
                t.push_back(t1 - t0);
                tsync.push_back(t2 - t0);
            }
        }
        report("launch+host_flag_seen", t);
        report("launch+host_flag_then_sync", tsync);
        (void)hipHostFree(hf);
    }
    {
        std::vector<double> t;
        hipPointerAttribute_t a;
        for (int i = 0; i < iters; ++i) {
            const double t0 = now_us();
            (void)hipPointerGetAttributes(&a, h + (i & 1023));
            t.push_back(now_us() - t0);
        }
        report("hipPointerGetAttributes", t);
    }
    {
        std::vector<double> t;
        hipEvent_t e;
        (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
        for (int i = 0; i < iters; ++i) {
            const double t0 = now_us();
            (void)hipEventRecord(e, s);
            t.push_back(now_us() - t0);
        }
        (void)hipStreamSynchronize(s);
        report("hipEventRecord", t);
    }
    {
        std::vector<double> t;
        for (int i = 0; i < iters; ++i) {
            const double t0 = now_us();
            touch<<<1, 64, 0, s>>>(d);
            t.push_back(now_us() - t0);
            (void)hipStreamSynchronize(s);
        }
        report("launch_call_only", t);
    }
    {
        const size_t bytes = 1920 * 1080, n16 = bytes / 16;
        uint8_t* dbuf = nullptr;
        uint32_t* sink = nullptr;
        if (hipMalloc(&dbuf, bytes) != hipSuccess || hipMalloc(&sink, 4096 * 256 * 4) != hipSuccess)
            return 1;
        uint8_t* hdev = nullptr;
        (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&hdev), h, 0);
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        for (int src = 0; src < 2; ++src) {
            for (int grid : {32, 64, 128, 256, 512, 1024, 2048}) {
                std::vector<double> t;
                for (int i = 0; i < 230; ++i) {
                    (void)hipEventRecord(e0, s);
                    read_all<<<grid, 256, 0, s>>>(reinterpret_cast<const uint4*>(src ? dbuf : hdev),
                                                  n16, sink);
                    (void)hipEventRecord(e1, s);
                    (void)hipStreamSynchronize(s);
                    float ms = 0;
                    (void)hipEventElapsedTime(&ms, e0, e1);
                    if (i >= 30) t.push_back(ms * 1e3);
                }
                char name[96];
                std::snprintf(name, sizeof name, "read_1080p_%s_grid%d", src ? "hbm" : "pinned_host", grid);
                report(name, t);
            }
        }
    }
    return 0;
}
