// Host <-> HBM transfer probe for the host-resident path (DESIGN.md §5 "end-to-end").
// Measures, on one MI355X, what the staging copies of a host-resident transform can reach:
// pageable vs registered (pinned) host memory, one direction alone vs H2D and D2H at the same
// time on two streams (PCIe full duplex), chunked copies, strided (2D) copies, and a
// multi-threaded host memcpy into a pinned staging buffer.
//   build: hipcc --offload-arch=gfx950 -O2 -std=c++17 tools/pcie_probe.hip -o tools/pcie_probe
//   run:   tools/pcie_probe [MiB]     (default 2048 MiB per direction)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                        \
    do {                                                                             \
        hipError_t e_ = (x);                                                         \
        if (e_ != hipSuccess) {                                                      \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x,            \
                         hipGetErrorString(e_));                                     \
            std::exit(2);                                                            \
        }                                                                            \
    } while (0)

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// best and median wall time of `reps` runs of f (f synchronises itself)
static void timeit(const char* name, double bytes, int reps, const std::function<void()>& f) {
    std::vector<double> t;
    for (int r = 0; r < reps; ++r) {
        double t0 = now();
        f();
        t.push_back(now() - t0);
    }
    std::sort(t.begin(), t.end());
    std::printf("%-58s best %8.2f ms  med %8.2f ms  %7.2f GB/s (best)\n", name, t[0] * 1e3,
                t[t.size() / 2] * 1e3, bytes / t[0] / 1e9);
    std::fflush(stdout);
}

static void par_memcpy(char* dst, const char* src, size_t n, int threads) {
    std::vector<std::thread> th;
    const size_t per = (n + threads - 1) / threads;
    for (int i = 0; i < threads; ++i) {
        const size_t lo = std::min(n, i * per), hi = std::min(n, lo + per);
        th.emplace_back([=] { std::memcpy(dst + lo, src + lo, hi - lo); });
    }
    for (auto& t : th) t.join();
}

int main(int argc, char** argv) {
    const size_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 2048;
    const size_t N = mib << 20;
    const int reps = 3;
    std::printf("bytes per direction: %zu MiB\n", mib);
    char* hA = static_cast<char*>(std::aligned_alloc(4096, N));
    char* hC = static_cast<char*>(std::aligned_alloc(4096, N));
    std::memset(hA, 1, N);
    std::memset(hC, 2, N);
    char *dA, *dC;
    CK(hipMalloc(&dA, N));
    CK(hipMalloc(&dC, N));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const double D = double(N);

    auto h2d = [&](char* h, hipStream_t s, size_t chunk) {
        for (size_t o = 0; o < N; o += chunk)
            CK(hipMemcpyAsync(dA + o, h + o, std::min(chunk, N - o), hipMemcpyHostToDevice, s));
    };
    auto d2h = [&](char* h, hipStream_t s, size_t chunk) {
        for (size_t o = 0; o < N; o += chunk)
            CK(hipMemcpyAsync(h + o, dC + o, std::min(chunk, N - o), hipMemcpyDeviceToHost, s));
    };
    auto sync2 = [&] {
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
    };
    // warm up both directions (first-touch of the runtime's staging)
    h2d(hA, s1, N);
    d2h(hC, s1, N);
    sync2();

    std::printf("-- pageable\n");
    timeit("H2D pageable, one call", D, reps, [&] { h2d(hA, s1, N); sync2(); });
    timeit("D2H pageable, one call", D, reps, [&] { d2h(hC, s1, N); sync2(); });
    timeit("H2D + D2H pageable, two streams (bytes = both)", 2 * D, reps,
           [&] { h2d(hA, s1, N); d2h(hC, s2, N); sync2(); });
    timeit("H2D 64 MiB chunks pageable", D, reps, [&] { h2d(hA, s1, 64 << 20); sync2(); });
    timeit("H2D + D2H 64 MiB chunks pageable, two streams", 2 * D, reps,
           [&] { h2d(hA, s1, 64 << 20); d2h(hC, s2, 64 << 20); sync2(); });
    // strided: 16 KiB rows at a 128 KiB pitch (a 2048-row slab of a 16384-row fp64 matrix)
    {
        const size_t w = 16 << 10, pitch = 128 << 10, h = N / pitch;
        timeit("H2D 2D pageable (16 KiB rows, 128 KiB pitch)", double(w * h), reps, [&] {
            CK(hipMemcpy2DAsync(dA, w, hA, pitch, w, h, hipMemcpyHostToDevice, s1));
            sync2();
        });
        timeit("D2H 2D pageable (16 KiB rows, 128 KiB pitch)", double(w * h), reps, [&] {
            CK(hipMemcpy2DAsync(hC, pitch, dC, w, w, h, hipMemcpyDeviceToHost, s1));
            sync2();
        });
    }

    std::printf("-- registered (hipHostRegister of the same buffers)\n");
    {
        double t0 = now();
        CK(hipHostRegister(hA, N, hipHostRegisterDefault));
        double t1 = now();
        CK(hipHostRegister(hC, N, hipHostRegisterDefault));
        double t2 = now();
        std::printf("hipHostRegister: A %.2f ms, C %.2f ms\n", (t1 - t0) * 1e3, (t2 - t1) * 1e3);
    }
    timeit("H2D registered, one call", D, reps, [&] { h2d(hA, s1, N); sync2(); });
    timeit("D2H registered, one call", D, reps, [&] { d2h(hC, s1, N); sync2(); });
    timeit("H2D + D2H registered, two streams", 2 * D, reps,
           [&] { h2d(hA, s1, N); d2h(hC, s2, N); sync2(); });
    timeit("H2D + D2H registered 64 MiB chunks, two streams", 2 * D, reps,
           [&] { h2d(hA, s1, 64 << 20); d2h(hC, s2, 64 << 20); sync2(); });
    {
        const size_t w = 16 << 10, pitch = 128 << 10, h = N / pitch;
        timeit("H2D 2D registered (16 KiB rows, 128 KiB pitch)", double(w * h), reps, [&] {
            CK(hipMemcpy2DAsync(dA, w, hA, pitch, w, h, hipMemcpyHostToDevice, s1));
            sync2();
        });
        timeit("D2H 2D registered (16 KiB rows, 128 KiB pitch)", double(w * h), reps, [&] {
            CK(hipMemcpy2DAsync(hC, pitch, dC, w, w, h, hipMemcpyDeviceToHost, s1));
            sync2();
        });
    }
    {
        double t0 = now();
        CK(hipHostUnregister(hA));
        CK(hipHostUnregister(hC));
        std::printf("hipHostUnregister both: %.2f ms\n", (now() - t0) * 1e3);
    }

    std::printf("-- mixed: one direction pageable (the runtime's path), the other pinned\n");
    {
        char* pin;
        CK(hipHostMalloc(reinterpret_cast<void**>(&pin), N, hipHostMallocDefault));
        std::memset(pin, 3, N);
        auto d2h_pin = [&](hipStream_t s, size_t chunk) {
            for (size_t o = 0; o < N; o += chunk)
                CK(hipMemcpyAsync(pin + o, dC + o, std::min(chunk, N - o), hipMemcpyDeviceToHost, s));
        };
        auto h2d_pin = [&](hipStream_t s, size_t chunk) {
            for (size_t o = 0; o < N; o += chunk)
                CK(hipMemcpyAsync(dA + o, pin + o, std::min(chunk, N - o), hipMemcpyHostToDevice, s));
        };
        timeit("H2D pageable + D2H pinned, two streams", 2 * D, reps,
               [&] { h2d(hA, s1, N); d2h_pin(s2, N); sync2(); });
        timeit("H2D pageable + D2H pinned, 64 MiB chunks", 2 * D, reps,
               [&] { h2d(hA, s1, 64 << 20); d2h_pin(s2, 64 << 20); sync2(); });
        timeit("H2D pinned + D2H pageable, two streams", 2 * D, reps,
               [&] { h2d_pin(s1, N); d2h(hC, s2, N); sync2(); });
        timeit("H2D pinned + D2H pinned, two streams", 2 * D, reps,
               [&] { h2d_pin(s1, N); d2h_pin(s2, N); sync2(); });
        // does an async D2H into pageable memory return before it completes?  (the host
        // pipeline's issuing thread must not stall on it)
        {
            const size_t c = size_t(64) << 20;
            double ret = 0, done = 0;
            for (int r = 0; r < 5; ++r) {
                CK(hipDeviceSynchronize());
                const double t0 = now();
                CK(hipMemcpyAsync(hC, dC, c, hipMemcpyDeviceToHost, s2));
                const double t1 = now();
                CK(hipStreamSynchronize(s2));
                const double t2 = now();
                if (r) ret += t1 - t0, done += t2 - t0;
            }
            std::printf("D2H pageable 64 MiB hipMemcpyAsync: call returns after %.3f ms, done after %.3f ms\n",
                        ret / 4 * 1e3, done / 4 * 1e3);
            for (int r = 0; r < 5; ++r) {
                CK(hipDeviceSynchronize());
                const double t0 = now();
                CK(hipMemcpyAsync(pin, dC, c, hipMemcpyDeviceToHost, s2));
                const double t1 = now();
                CK(hipStreamSynchronize(s2));
                const double t2 = now();
                if (r) ret += t1 - t0, done += t2 - t0;
            }
        }
        timeit("H2D pinned + D2H pageable, 64 MiB chunks", 2 * D, reps,
               [&] { h2d_pin(s1, 64 << 20); d2h(hC, s2, 64 << 20); sync2(); });
        timeit("H2D pinned + D2H pageable 64 MiB chunks + 16-thread host copy of 2 GiB", 2 * D, reps, [&] {
            h2d_pin(s1, 64 << 20);
            std::thread t([&] { par_memcpy(pin, hA, N, 15); });
            d2h(hC, s2, 64 << 20);
            t.join();
            sync2();
        });
        // strided (2D) DMA straight from / to pinned host memory: column bands of w bytes of a
        // 2 GiB matrix with 128 KiB rows (16384 rows), one call per band: the direct-DMA staging
        // of a host pipeline over pinned caller memory
        char* pin2;
        CK(hipHostMalloc(reinterpret_cast<void**>(&pin2), N, hipHostMallocDefault));
        std::memset(pin2, 4, N);
        for (size_t w : {size_t(1) << 10, size_t(2) << 10, size_t(4) << 10, size_t(16) << 10}) {
            const size_t pitch = 128 << 10, h = N / pitch, calls = pitch / w;
            std::string nm = "H2D 2D pinned, " + std::to_string(w) + " B rows x 16384";
            timeit(nm.c_str(), D, reps, [&] {
                for (size_t c = 0; c < calls; ++c)
                    CK(hipMemcpy2DAsync(dA + c * h * w, w, pin + c * w, pitch, w, h, hipMemcpyHostToDevice, s1));
                sync2();
            });
            nm = "D2H 2D pinned, " + std::to_string(w) + " B rows x 16384";
            timeit(nm.c_str(), D, reps, [&] {
                for (size_t c = 0; c < calls; ++c)
                    CK(hipMemcpy2DAsync(pin + c * w, pitch, dC + c * h * w, w, w, h, hipMemcpyDeviceToHost, s2));
                sync2();
            });
            nm = "H2D 1D pinned + D2H 2D pinned " + std::to_string(w) + " B rows, together";
            timeit(nm.c_str(), 2 * D, reps, [&] {
                for (size_t c = 0; c < calls; ++c) {
                    CK(hipMemcpyAsync(dA + c * h * w, pin2 + c * h * w, h * w, hipMemcpyHostToDevice, s1));
                    CK(hipMemcpy2DAsync(pin + c * w, pitch, dC + c * h * w, w, w, h, hipMemcpyDeviceToHost, s2));
                }
                sync2();
            });
        }
        CK(hipHostFree(pin2));
        {
            const double t0 = now();
            for (int i = 0; i < 1000; ++i)
                CK(hipMemcpy2DAsync(dA, 2048, pin, 131072, 2048, 16, hipMemcpyHostToDevice, s1));
            const double t1 = now();
            sync2();
            std::printf("hipMemcpy2DAsync issue cost (pinned, 32 KiB): %.2f us per call\n", (t1 - t0) * 1e3);
        }
        // the pinned D2H while 16 host threads copy pinned -> pageable (the scatter) at once
        timeit("H2D pageable + D2H pinned + 16-thread host copy of 2 GiB", 2 * D, reps, [&] {
            h2d(hA, s1, 64 << 20);
            d2h_pin(s2, 64 << 20);
            par_memcpy(hC, pin, N, 16);
            sync2();
        });
        CK(hipHostFree(pin));
    }

    std::printf("-- pinned staging ring (hipHostMalloc) + host threads\n");
    {
        const size_t ring = 256 << 20;
        char* pin;
        CK(hipHostMalloc(reinterpret_cast<void**>(&pin), ring, hipHostMallocDefault));
        for (int th : {1, 4, 8, 16}) {
            std::string nm = "host memcpy pageable -> pinned, " + std::to_string(th) + " threads";
            timeit(nm.c_str(), double(ring), reps, [&] { par_memcpy(pin, hA, ring, th); });
        }
        timeit("H2D from pinned 256 MiB", double(ring), reps, [&] {
            CK(hipMemcpyAsync(dA, pin, ring, hipMemcpyHostToDevice, s1));
            sync2();
        });
        CK(hipHostFree(pin));
    }
    std::printf("done\n");
    return 0;
}
