// Probe (not product): does a plain strided copy lose when the column stride is a large power
// of two plus 64 B .. 4 KiB, as the transposes do (profiles/r4l/)?  The source and
// destination are 16384 columns of 8192 fp64 rows (64 KiB) at a stride of 128 KiB + delta bytes;
// a 256-thread workgroup copies 16 column segments of 1 KiB, consecutive workgroups continue down
// the same 16 columns (tools/copy_ceiling.hip "seg 1024"), nt loads and stores.  Modes: both
// sides strided, only the source strided (destination dense), only the destination strided.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/stride_probe.hip -o /tmp/sp && /tmp/sp
// `/tmp/sp strides`: both sides strided at 128 / 192 / 256 / 384 / 512 KiB (delta 0, 64 B), with
// 1 KiB and 512-byte segments (the fp64 transposes' read segment; DESIGN §3b, fp64 32768^2);
// `/tmp/sp windows`: 1 KiB segments from each column's start against 1 KiB windows aligned to the
// address grid, strides 128 / 256 / 384 KiB + 0 / 64 / 256 / 512 B; `/tmp/sp segsizes`: segment
// length 512 B - 4 KiB (1024 B / 16 columns per workgroup) at strides of 128 - 384 KiB;
// `/tmp/sp three [n]`: the three-stream C = A + C (cfg 4's reads and writes) against the copy, on
// the c128 n^2 geometry (columns of 16 n bytes; n = 16384 by default); `/tmp/sp runs`: runs of
// 64 B - 1 KiB at 1 - 2x their length apart (cfg 5's access shape), copy and C = A + C;
// `/tmp/sp inflight`: cfg 2's copy ceiling under other workgroup sizes and column counts;
// `/tmp/sp segu`: segment length against loads in flight per thread
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// column c, segment q (1 KiB = 64 x 16 B): element e of the segment at base + c * stride16 + q * 64 + e
// SEG16: 16-byte vectors per segment (64: 1 KiB, 32: 512 B); 1024 / SEG16 columns per workgroup
template <int SEG16>
__global__ __launch_bounds__(256) void seg(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                           long sa, long sc, long segs_per_col) {
    constexpr int COLS = 1024 / SEG16;
    const long w = blockIdx.x;
    const long g = w / segs_per_col, q = w % segs_per_col;
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + int(threadIdx.x);
        const long col = g * COLS + e / SEG16;
        x[u] = __builtin_nontemporal_load(a + col * sa + q * SEG16 + e % SEG16);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + int(threadIdx.x);
        const long col = g * COLS + e / SEG16;
        __builtin_nontemporal_store(x[u], c + col * sc + q * SEG16 + e % SEG16);
    }
}

template <int SEG16>
static float time_seg(const char* a, char* c, long cols, long col_bytes, long sa, long sc) {
    const long segs = col_bytes / (SEG16 * 16);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(seg<SEG16>, dim3(unsigned(cols / (1024 / SEG16) * segs)), dim3(256), 0, 0,
                           reinterpret_cast<const u32x4*>(a), reinterpret_cast<u32x4*>(c), sa / 16, sc / 16, segs);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return t[t.size() / 2];
}

// 1 KiB windows aligned to the address grid: window q of column col covers the 16-byte vectors of
// [align_down(base, 1 KiB) + q KiB, + 1 KiB) inside the column (base = col * stride, the same on
// both sides); ragged windows at each column's two ends
__global__ __launch_bounds__(256) void win(const u32x4* __restrict__ a, u32x4* __restrict__ c, long s16,
                                           long col16, long wins_per_col) {
    const long w = blockIdx.x;
    const long g = w / wins_per_col, q = w % wins_per_col;
    u32x4 x[4];
    long idx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + int(threadIdx.x);
        const long col = g * 16 + e / 64;
        const long base = col * s16, lo = base / 64 * 64;
        const long v = lo + q * 64 + e % 64;
        idx[u] = (v >= base && v < base + col16) ? v : -1;
        if (idx[u] >= 0) x[u] = __builtin_nontemporal_load(a + idx[u]);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
        if (idx[u] >= 0) __builtin_nontemporal_store(x[u], c + idx[u]);
}

static float time_win(const char* a, char* c, long cols, long col_bytes, long stride) {
    const long wins = col_bytes / 1024 + 1;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(win, dim3(unsigned(cols / 16 * wins)), dim3(256), 0, 0, reinterpret_cast<const u32x4*>(a),
                           reinterpret_cast<u32x4*>(c), stride / 16, col_bytes / 16, wins);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return t[t.size() / 2];
}

static int windows() {
    const long cols = 16384, col_bytes = 65536;
    const long max_stride = 393216 + 1024;
    char *a, *c;
    CK(hipMalloc(&a, cols * max_stride));
    CK(hipMalloc(&c, cols * max_stride));
    CK(hipMemset(a, 1, cols * max_stride));
    CK(hipMemset(c, 0, cols * max_stride));
    const double bytes = 2.0 * cols * col_bytes;
    for (long kib : {128, 256, 384})
        for (long d : {0, 64, 256, 512}) {
            const long stride = kib * 1024 + d;
            const float m1 = time_seg<64>(a, c, cols, col_bytes, stride, stride);
            const float m2 = time_win(a, c, cols, col_bytes, stride);
            printf("stride %3ld KiB + %3ld B: segments from the column start %.4f ms %.2f TB/s   1 KiB-aligned windows %.4f ms %.2f TB/s\n",
                   kib, d, m1, bytes / (m1 * 1e-3) / 1e12, m2, bytes / (m2 * 1e-3) / 1e12);
        }
    return 0;
}

static int segsizes() {
    const long cols = 16384, col_bytes = 65536;
    const long max_stride = 393216;
    char *a, *c;
    CK(hipMalloc(&a, cols * max_stride));
    CK(hipMalloc(&c, cols * max_stride));
    CK(hipMemset(a, 1, cols * max_stride));
    CK(hipMemset(c, 0, cols * max_stride));
    const double bytes = 2.0 * cols * col_bytes;
    for (long kib : {128, 160, 192, 256, 320, 384}) {
        const long stride = kib * 1024;
        const float m0 = time_seg<32>(a, c, cols, col_bytes, stride, stride);
        const float m1 = time_seg<64>(a, c, cols, col_bytes, stride, stride);
        const float m2 = time_seg<128>(a, c, cols, col_bytes, stride, stride);
        const float m3 = time_seg<256>(a, c, cols, col_bytes, stride, stride);
        printf("stride %3ld KiB: TB/s with 512 B / 1 / 2 / 4 KiB segments: %.2f %.2f %.2f %.2f\n", kib,
               bytes / (m0 * 1e-3) / 1e12, bytes / (m1 * 1e-3) / 1e12, bytes / (m2 * 1e-3) / 1e12,
               bytes / (m3 * 1e-3) / 1e12);
    }
    return 0;
}

// C = A + C over 1 KiB column segments (reads A and C, writes C: cfg 4's three streams), against
// the two-stream copy of the same geometry: c128 16384^2 (columns of 256 KiB, dense)
__global__ __launch_bounds__(256) void axpy_seg(const u32x4* __restrict__ a, u32x4* __restrict__ c, long s16,
                                                long segs_per_col) {
    const long w = blockIdx.x;
    const long g = w / segs_per_col, q = w % segs_per_col;
    u32x4 x[4], y[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + int(threadIdx.x);
        const long col = g * 16 + e / 64;
        x[u] = __builtin_nontemporal_load(a + col * s16 + q * 64 + e % 64);
        y[u] = __builtin_nontemporal_load(c + col * s16 + q * 64 + e % 64);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + int(threadIdx.x);
        const long col = g * 16 + e / 64;
        __builtin_nontemporal_store(x[u] ^ y[u], c + col * s16 + q * 64 + e % 64);
    }
}

static int three(long n) {
    const long cols = n, col_bytes = n * 16;
    char *a, *c;
    CK(hipMalloc(&a, cols * col_bytes));
    CK(hipMalloc(&c, cols * col_bytes));
    CK(hipMemset(a, 1, cols * col_bytes));
    CK(hipMemset(c, 0, cols * col_bytes));
    const long segs = col_bytes / 1024;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(axpy_seg, dim3(unsigned(cols / 16 * segs)), dim3(256), 0, 0,
                           reinterpret_cast<const u32x4*>(a), reinterpret_cast<u32x4*>(c), col_bytes / 16, segs);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    const float m3 = t[t.size() / 2];
    const float m2 = time_seg<64>(a, c, cols, col_bytes, col_bytes, col_bytes);
    printf("c128 %ld^2 geometry, 1 KiB segments: C = A + C (3 x %ld MiB) %.4f ms %.2f TB/s; copy (2 x %ld MiB) %.4f ms %.2f TB/s\n",
           n, cols * col_bytes >> 20, m3, 3.0 * cols * col_bytes / (m3 * 1e-3) / 1e12, cols * col_bytes >> 20, m2, 2.0 * cols * col_bytes / (m2 * 1e-3) / 1e12);
    return 0;
}

// Short runs (cfg 5's access shape: ~130-byte column runs of small blocks, dense-ish): run r of
// L bytes at r * S on both sides, one dword per lane, consecutive lanes along a run; the copy
// (two streams) and C = A + C (three, cfg 5 'T' with beta != 0); 16 dwords per thread in flight, nt
template <bool THREE>
__global__ __launch_bounds__(256) void runs_k(const unsigned* __restrict__ a, unsigned* __restrict__ c, long L4,
                                              long S4, long n) {
    constexpr int K = 16;  // dwords per thread, all loads in flight before the stores
    const long base = long(blockIdx.x) * 256 * K + threadIdx.x;
    unsigned v[K];
    long idx[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const long t = base + long(j) * 256;
        idx[j] = t < n ? (t / L4) * S4 + t % L4 : -1;
        if (idx[j] >= 0) v[j] = __builtin_nontemporal_load(a + idx[j]);
    }
    if (THREE) {
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (idx[j] >= 0) v[j] ^= __builtin_nontemporal_load(c + idx[j]);
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (idx[j] >= 0) __builtin_nontemporal_store(v[j], c + idx[j]);
}

// the same C = A + C with A read as 16-byte vectors (aligned runs: the upper bound of wider source
// loads) and C read and written as dwords
__global__ __launch_bounds__(256) void runs_wide_a(const u32x4* __restrict__ a, unsigned* __restrict__ c, long L4,
                                                   long S4, long n) {
    constexpr int K = 16;
    const long base = long(blockIdx.x) * 256 * K + threadIdx.x;
    unsigned v[K];
    long idx[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const long t = base + long(j) * 256;
        idx[j] = t < n ? (t / L4) * S4 + t % L4 : -1;
    }
    // A: 4 of this thread's dwords (j = 4q .. 4q+3 are 256 dwords apart) come from one vector
    // at the position of dword 4q's lane group: re-map so that lane l of pass q loads vector l
#pragma unroll
    for (int q = 0; q < K / 4; ++q) {
        const long t4 = (long(blockIdx.x) * 256 * K) / 4 + q * 256 + threadIdx.x;  // vector index
        const long e = t4 * 4;                                                     // first dword
        const long i = e < n ? (e / L4) * S4 + e % L4 : -1;
        u32x4 x = {0, 0, 0, 0};
        if (i >= 0) x = __builtin_nontemporal_load(a + i / 4);
        v[4 * q] = x[0];
        v[4 * q + 1] = x[1];
        v[4 * q + 2] = x[2];
        v[4 * q + 3] = x[3];
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (idx[j] >= 0) v[j] ^= __builtin_nontemporal_load(c + idx[j]);
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (idx[j] >= 0) __builtin_nontemporal_store(v[j], c + idx[j]);
}

// C = A + C with every stream in 16-byte vectors, C's runs OFF bytes past the 16-byte grid
// (unaligned vector loads and stores: cfg 5's destination runs start on any dword)
typedef unsigned u32x4u __attribute__((ext_vector_type(4), aligned(4)));
template <int OFF>
__global__ __launch_bounds__(256) void runs_x4(const u32x4* __restrict__ a, unsigned* __restrict__ c, long L16,
                                               long S16, long n16) {
    constexpr int K = 4;
    const long base = long(blockIdx.x) * 256 * K + threadIdx.x;
    u32x4 v[K];
    long idx[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        const long t = base + long(j) * 256;
        idx[j] = t < n16 ? (t / L16) * S16 + t % L16 : -1;
        if (idx[j] >= 0) v[j] = __builtin_nontemporal_load(a + idx[j]);
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (idx[j] >= 0) {
            const u32x4u* p = reinterpret_cast<const u32x4u*>(reinterpret_cast<const char*>(c) + idx[j] * 16 + OFF);
            v[j] ^= *p;
        }
#pragma unroll
    for (int j = 0; j < K; ++j)
        if (idx[j] >= 0) *reinterpret_cast<u32x4u*>(reinterpret_cast<char*>(c) + idx[j] * 16 + OFF) = v[j];
}

template <int OFF>
static float time_x4(const char* a, char* c, long L, long S, long bytes) {
    const long n16 = bytes / 16;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL(runs_x4<OFF>, dim3(unsigned((n16 + 1023) / 1024)), dim3(256), 0, 0,
                           reinterpret_cast<const u32x4*>(a), reinterpret_cast<unsigned*>(c), L / 16, S / 16, n16);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return t[t.size() / 2];
}

static int runs() {
    const long bytes = 1L << 30;  // moved per stream
    const long max_span = bytes * 4;
    char *a, *c;
    CK(hipMalloc(&a, max_span));
    CK(hipMalloc(&c, max_span));
    CK(hipMemset(a, 1, max_span));
    CK(hipMemset(c, 0, max_span));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (long L : {64, 128, 192, 256, 1024})
        for (long S : {L, L * 3 / 2, L * 2}) {
            const long n = bytes / 4;
            float med[2];
            for (int three = 0; three < 2; ++three) {
                std::vector<float> t;
                for (int r = 0; r < 12; ++r) {
                    CK(hipEventRecord(e0));
                    if (three)
                        hipLaunchKernelGGL(runs_k<true>, dim3(unsigned((n + 4095) / 4096)), dim3(256), 0, 0,
                                           reinterpret_cast<const unsigned*>(a), reinterpret_cast<unsigned*>(c), L / 4, S / 4, n);
                    else
                        hipLaunchKernelGGL(runs_k<false>, dim3(unsigned((n + 4095) / 4096)), dim3(256), 0, 0,
                                           reinterpret_cast<const unsigned*>(a), reinterpret_cast<unsigned*>(c), L / 4, S / 4, n);
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float ms;
                    CK(hipEventElapsedTime(&ms, e0, e1));
                    if (r >= 2) t.push_back(ms);
                }
                std::sort(t.begin(), t.end());
                med[three] = t[t.size() / 2];
            }
            std::vector<float> tw;
            for (int r = 0; r < 12; ++r) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(runs_wide_a, dim3(unsigned((n + 4095) / 4096)), dim3(256), 0, 0,
                                   reinterpret_cast<const u32x4*>(a), reinterpret_cast<unsigned*>(c), L / 4, S / 4, n);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) tw.push_back(ms);
            }
            std::sort(tw.begin(), tw.end());
            const float mw = tw[tw.size() / 2];
            const float x0 = time_x4<0>(a, c, L, S, bytes), x4 = time_x4<4>(a, c, L, S, bytes);
            printf("runs of %4ld B every %4ld B: copy %.2f TB/s   C = A + C dwords %.2f TB/s, A as 16 B %.2f, all 16 B %.2f, "
                   "C 4 B off the grid %.2f\n",
                   L, S, 2.0 * bytes / (med[0] * 1e-3) / 1e12, 3.0 * bytes / (med[1] * 1e-3) / 1e12,
                   3.0 * bytes / (mw * 1e-3) / 1e12, 3.0 * bytes / (x0 * 1e-3) / 1e12, 3.0 * bytes / (x4 * 1e-3) / 1e12);
        }
    return 0;
}

// the strided nt copy with more bytes in flight per workgroup: NT threads, COLS column segments of
// 1 KiB per workgroup, U 16-byte vectors per thread (U = COLS * 64 / NT), consecutive workgroups
// continuing down the same columns
template <int NT, int COLS>
__global__ __launch_bounds__(NT) void segw(const u32x4* __restrict__ a, u32x4* __restrict__ c, long s16,
                                          long segs_per_col) {
    constexpr int U = COLS * 64 / NT;
    const long w = blockIdx.x;
    const long g = w / segs_per_col, q = w % segs_per_col;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = u * NT + int(threadIdx.x);
        x[u] = __builtin_nontemporal_load(a + (g * COLS + e / 64) * s16 + q * 64 + e % 64);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = u * NT + int(threadIdx.x);
        __builtin_nontemporal_store(x[u], c + (g * COLS + e / 64) * s16 + q * 64 + e % 64);
    }
}

template <int NT, int COLS>
static float time_segw(const char* a, char* c, long cols, long col_bytes) {
    const long segs = col_bytes / 1024;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((segw<NT, COLS>), dim3(unsigned(cols / COLS * segs)), dim3(NT), 0, 0,
                           reinterpret_cast<const u32x4*>(a), reinterpret_cast<u32x4*>(c), col_bytes / 16, segs);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return t[t.size() / 2];
}

// cfg 2's bytes (16384 columns of 128 KiB, 2 GiB per side) under several workgroup shapes
static int inflight() {
    const long cols = 16384, col_bytes = 131072;
    char *a, *c;
    CK(hipMalloc(&a, cols * col_bytes));
    CK(hipMalloc(&c, cols * col_bytes));
    CK(hipMemset(a, 1, cols * col_bytes));
    CK(hipMemset(c, 0, cols * col_bytes));
    const double bytes = 2.0 * cols * col_bytes;
    auto show = [&](const char* name, float ms) {
        printf("%-36s %.4f ms %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    for (int rep = 0; rep < 2; ++rep) {
        show("256 threads, 16 columns (shipped ceiling)", time_segw<256, 16>(a, c, cols, col_bytes));
        show("64 threads, 1 column (U 1)", time_segw<64, 1>(a, c, cols, col_bytes));
        show("256 threads, 4 columns (U 1)", time_segw<256, 4>(a, c, cols, col_bytes));
        show("512 threads, 8 columns (U 1)", time_segw<512, 8>(a, c, cols, col_bytes));
        show("1024 threads, 16 columns (U 1)", time_segw<1024, 16>(a, c, cols, col_bytes));
        show("64 threads, 2 columns (U 2)", time_segw<64, 2>(a, c, cols, col_bytes));
        show("256 threads, 8 columns (U 2)", time_segw<256, 8>(a, c, cols, col_bytes));
        show("512 threads, 16 columns (U 2)", time_segw<512, 16>(a, c, cols, col_bytes));
        show("1024 threads, 32 columns (U 2)", time_segw<1024, 32>(a, c, cols, col_bytes));
        show("512 threads, 64 columns (U 8)", time_segw<512, 64>(a, c, cols, col_bytes));
    }
    return 0;
}

// segw with SEGB-byte segments (SEGB / 16 lanes per column)
template <int NT, int COLS, int SEGB>
__global__ __launch_bounds__(NT) void segv(const u32x4* __restrict__ a, u32x4* __restrict__ c, long s16,
                                          long segs_per_col) {
    constexpr int L = SEGB / 16, U = COLS * L / NT;
    const long w = blockIdx.x;
    const long g = w / segs_per_col, q = w % segs_per_col;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = u * NT + int(threadIdx.x);
        x[u] = __builtin_nontemporal_load(a + (g * COLS + e / L) * s16 + q * L + e % L);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const int e = u * NT + int(threadIdx.x);
        __builtin_nontemporal_store(x[u], c + (g * COLS + e / L) * s16 + q * L + e % L);
    }
}
template <int NT, int COLS, int SEGB>
static float time_segv(const char* a, char* c, long cols, long col_bytes) {
    const long segs = col_bytes / SEGB;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> t;
    for (int r = 0; r < 12; ++r) {
        CK(hipEventRecord(e0));
        hipLaunchKernelGGL((segv<NT, COLS, SEGB>), dim3(unsigned(cols / COLS * segs)), dim3(NT), 0, 0,
                           reinterpret_cast<const u32x4*>(a), reinterpret_cast<u32x4*>(c), col_bytes / 16, segs);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r >= 2) t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return t[t.size() / 2];
}
// segment length against loads per thread on cfg 2's bytes
static int segu() {
    const long cols = 16384, col_bytes = 131072;
    char *a, *c;
    CK(hipMalloc(&a, cols * col_bytes));
    CK(hipMalloc(&c, cols * col_bytes));
    CK(hipMemset(a, 1, cols * col_bytes));
    CK(hipMemset(c, 0, cols * col_bytes));
    const double bytes = 2.0 * cols * col_bytes;
    auto show = [&](const char* name, float ms) {
        printf("%-44s %.4f ms %.2f TB/s\n", name, ms, bytes / (ms * 1e-3) / 1e12);
    };
    for (int rep = 0; rep < 2; ++rep) {
        show("256 B segments, 256 threads, 16 cols (U 1)", time_segv<256, 16, 256>(a, c, cols, col_bytes));
        show("512 B segments, 256 threads, 8 cols (U 1)", time_segv<256, 8, 512>(a, c, cols, col_bytes));
        show("1 KiB segments, 256 threads, 4 cols (U 1)", time_segv<256, 4, 1024>(a, c, cols, col_bytes));
        show("256 B segments, 256 threads, 32 cols (U 2)", time_segv<256, 32, 256>(a, c, cols, col_bytes));
        show("512 B segments, 256 threads, 16 cols (U 2)", time_segv<256, 16, 512>(a, c, cols, col_bytes));
        show("512 B segments, 1024 threads, 64 cols (U 2)", time_segv<1024, 64, 512>(a, c, cols, col_bytes));
        show("512 B segments, 512 threads, 64 cols (U 4)", time_segv<512, 64, 512>(a, c, cols, col_bytes));
        show("512 B segments, 512 threads, 128 cols (U 8)", time_segv<512, 128, 512>(a, c, cols, col_bytes));
    }
    return 0;
}

static int strides() {
    const long cols = 16384, col_bytes = 65536;
    const long max_stride = 524288 + 64;
    char *a, *c;
    CK(hipMalloc(&a, cols * max_stride));
    CK(hipMalloc(&c, cols * max_stride));
    CK(hipMemset(a, 1, cols * max_stride));
    CK(hipMemset(c, 0, cols * max_stride));
    const double bytes = 2.0 * cols * col_bytes;
    for (long kib : {128, 192, 256, 384, 512})
        for (long d : {0, 64}) {
            const long stride = kib * 1024 + d;
            const float m1 = time_seg<64>(a, c, cols, col_bytes, stride, stride);
            const float m2 = time_seg<32>(a, c, cols, col_bytes, stride, stride);
            printf("stride %3ld KiB + %2ld B: 1 KiB segments %.4f ms %.2f TB/s   512 B segments %.4f ms %.2f TB/s\n",
                   kib, d, m1, bytes / (m1 * 1e-3) / 1e12, m2, bytes / (m2 * 1e-3) / 1e12);
        }
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "strides") return strides();
    if (argc > 1 && std::string(argv[1]) == "windows") return windows();
    if (argc > 1 && std::string(argv[1]) == "segsizes") return segsizes();
    if (argc > 1 && std::string(argv[1]) == "three") return three(argc > 2 ? std::atol(argv[2]) : 16384);
    if (argc > 1 && std::string(argv[1]) == "runs") return runs();
    if (argc > 1 && std::string(argv[1]) == "inflight") return inflight();
    if (argc > 1 && std::string(argv[1]) == "segu") return segu();
    const long cols = 16384, col_bytes = 65536;  // 8192 fp64 rows per column, 1 GiB per side
    const long segs = col_bytes / 1024;
    const long max_stride = 131072 + 8192;
    char *a, *c;
    CK(hipMalloc(&a, cols * max_stride));
    CK(hipMalloc(&c, cols * max_stride));
    CK(hipMemset(a, 1, cols * max_stride));
    CK(hipMemset(c, 0, cols * max_stride));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const long deltas[] = {0, 16, 64, 128, 256, 512, 1024, 2048, 4096, 8192};
    for (int mode = 0; mode < 3; ++mode) {
        for (long d : deltas) {
            const long stride = 131072 + d;
            const long sa = (mode == 2 ? col_bytes : stride) / 16, sc = (mode == 1 ? col_bytes : stride) / 16;
            std::vector<float> t;
            for (int r = 0; r < 12; ++r) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(seg<64>, dim3(unsigned(cols / 16 * segs)), dim3(256), 0, 0,
                                   reinterpret_cast<const u32x4*>(a), reinterpret_cast<u32x4*>(c), sa, sc, segs);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (r >= 2) t.push_back(ms);
            }
            std::sort(t.begin(), t.end());
            const double bytes = 2.0 * cols * col_bytes;
            printf("%-22s stride 128 KiB + %5ld B: %.4f ms  %.2f TB/s\n",
                   mode == 0 ? "both strided" : mode == 1 ? "source strided" : "destination strided", d,
                   t[t.size() / 2], bytes / (t[t.size() / 2] * 1e-3) / 1e12);
        }
    }
    return 0;
}
