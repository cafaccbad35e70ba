// FETCH_SIZE / WRITE_SIZE calibration by access width.
// MI355X_MICROARCH.md calibrates FETCH_SIZE for wide (16 B a lane) streaming reads only: it
// reports half of their bytes.  The wavefront and destination-block kernels of cfg 5 read one
// dword a lane, over short column runs at arbitrary alignment.  Each kernel below moves a byte
// count known on the host; `rocprofv3 --pmc FETCH_SIZE` (or WRITE_SIZE) over this program then
// gives the factor per access kind.
//   flat16   1 GiB read, 16 B a lane, fully coalesced
//   flat4    1 GiB read, 4 B a lane, fully coalesced
//   runs4    cfg 5-like column runs (8-96 floats, start at any 4-byte offset, one run per
//            512-byte slot so no two runs share a line), lanes along the run, 4 B a lane
//   runs16   the same runs read as the aligned 16-byte chunks that cover them
//   wr16     1 GiB written, 16 B a lane
//   wr4      1 GiB written, 4 B a lane
// Prints one JSON line per kind: bytes useful, 64-byte granules and 128-byte lines touched.
// Build: hipcc -O3 --offload-arch=gfx950 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
            std::exit(1);                                                                       \
        }                                                                                       \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void flat16(const f4* __restrict__ a, int64_t n4, float* out) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    float s = 0.f;
    if (i < n4) {
        const f4 v = a[i];
        s = v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;  // keeps the load
}

__global__ void flat4(const float* __restrict__ a, int64_t n, float* out) {
    const int64_t i = (int64_t(blockIdx.x) * blockDim.x) * 4 + threadIdx.x;
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (i + u * blockDim.x < n) s += a[i + u * blockDim.x];
    if (s == 12345.f) out[0] = s;
}

// one wavefront per run of floats: start (in floats) and length
__global__ void runs4(const float* __restrict__ a, const int64_t* __restrict__ start, const int* __restrict__ len,
                      int64_t nruns, float* out) {
    const int64_t w = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const int lane = threadIdx.x % 64;
    if (w >= nruns) return;
    const float* p = a + start[w];
    float s = 0.f;
    for (int e = lane; e < len[w]; e += 64) s += p[e];
    if (s == 12345.f) out[0] = s;
}

__global__ void runs16(const float* __restrict__ a, const int64_t* __restrict__ start, const int* __restrict__ len,
                       int64_t nruns, float* out) {
    const int64_t w = (int64_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
    const int lane = threadIdx.x % 64;
    if (w >= nruns) return;
    const int64_t c0 = start[w] / 4, c1 = (start[w] + len[w] + 3) / 4;  // aligned chunks covering it
    const f4* p = reinterpret_cast<const f4*>(a);
    float s = 0.f;
    for (int64_t c = c0 + lane; c < c1; c += 64) {
        const f4 v = p[c];
        s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.f) out[0] = s;
}

__global__ void wr16(f4* __restrict__ a, int64_t n4) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n4) a[i] = f4{1.f, 2.f, 3.f, float(i)};
}

__global__ void wr4(float* __restrict__ a, int64_t n) {
    const int64_t i = (int64_t(blockIdx.x) * blockDim.x) * 4 + threadIdx.x;
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (i + u * blockDim.x < n) a[i + u * blockDim.x] = float(i);
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    const int64_t bytes = int64_t(1) << 30, n = bytes / 4;
    float *a, *out;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(a, 0, bytes));
    // runs: one per 512-byte slot (128 floats), length 8..96, start 0..(128 - len) floats into it
    const int64_t nruns = n / 128;
    std::vector<int64_t> st(nruns);
    std::vector<int> ln(nruns);
    std::mt19937_64 g(0xCA11B);
    int64_t useful = 0, gran = 0, lines = 0;
    for (int64_t k = 0; k < nruns; ++k) {
        const int L = 8 + int(g() % 89);
        const int64_t s0 = k * 128 + int64_t(g() % uint64_t(128 - L + 1));
        st[k] = s0;
        ln[k] = L;
        useful += 4 * L;
        gran += (4 * (s0 + L) - 1) / 64 - (4 * s0) / 64 + 1;
        lines += (4 * (s0 + L) - 1) / 128 - (4 * s0) / 128 + 1;
    }
    int64_t chunks16 = 0;
    for (int64_t k = 0; k < nruns; ++k) chunks16 += (st[k] + ln[k] + 3) / 4 - st[k] / 4;
    int64_t* dst_;
    int* dln;
    CK(hipMalloc(&dst_, nruns * 8));
    CK(hipMalloc(&dln, nruns * 4));
    CK(hipMemcpy(dst_, st.data(), nruns * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dln, ln.data(), nruns * 4, hipMemcpyHostToDevice));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, auto launch, int64_t alg, int64_t g64, int64_t l128) {
        float best = 1e30f;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            launch();
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            best = ms < best ? ms : best;
        }
        std::printf("{\"kind\": \"%s\", \"bytes_useful\": %lld, \"bytes_64B_granules\": %lld, "
                    "\"bytes_128B_lines\": %lld, \"best_ms\": %.4f}\n",
                    name, (long long)alg, (long long)(64 * g64), (long long)(128 * l128), best);
    };
    const int64_t n4 = n / 4;
    timed("flat16", [&] { hipLaunchKernelGGL(flat16, dim3(unsigned(n4 / 256)), dim3(256), 0, 0, (const f4*)a, n4, out); },
          bytes, bytes / 64, bytes / 128);
    timed("flat4", [&] { hipLaunchKernelGGL(flat4, dim3(unsigned(n / 1024)), dim3(256), 0, 0, a, n, out); }, bytes,
          bytes / 64, bytes / 128);
    const unsigned rb = unsigned((nruns * 64 + 255) / 256);
    timed("runs4", [&] { hipLaunchKernelGGL(runs4, dim3(rb), dim3(256), 0, 0, a, dst_, dln, nruns, out); }, useful, gran,
          lines);
    timed("runs16", [&] { hipLaunchKernelGGL(runs16, dim3(rb), dim3(256), 0, 0, a, dst_, dln, nruns, out); },
          16 * chunks16, gran, lines);
    timed("wr16", [&] { hipLaunchKernelGGL(wr16, dim3(unsigned(n4 / 256)), dim3(256), 0, 0, (f4*)a, n4); }, bytes,
          bytes / 64, bytes / 128);
    timed("wr4", [&] { hipLaunchKernelGGL(wr4, dim3(unsigned(n / 1024)), dim3(256), 0, 0, a, n); }, bytes, bytes / 64,
          bytes / 128);
    CK(hipDeviceSynchronize());
    return 0;
}
