// Tuning probe (not part of the product): does a destination whose 128-byte lines are split
// between two workgroups cost bandwidth on MI355X?  Copies 2 GiB as cfg 2's transposes write it:
// 16 columns of 128 KiB per workgroup in 1 KiB segments, consecutive workgroups continuing the
// same columns (tools/copy_ceiling.hip k_seg).  The destination base is shifted by OFF bytes:
//   OFF = 0 / 128   every line written whole by one workgroup
//   OFF = 16 / 64   16-byte aligned stores, but the first and last line of every segment are
//                   shared with the neighbouring workgroup's segment
//   OFF = 8         the same with 8-byte stores (an odd fp64 lld)
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/partial_line_probe.hip -o /tmp/plp && /tmp/plp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
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
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr long COLB = 131072;  // column bytes
constexpr long SEG = 1024;     // segment bytes
constexpr int S = 16;          // columns per workgroup

// W = 16: 16-byte stores, W = 8: 8-byte stores (two per loaded vector)
// XCD: 0 = blocks in order (round-robin over the 8 XCDs), -1 = each XCD a contiguous slice of
// the grid, R > 0 = runs of R consecutive segments per XCD inside every group of 8 R (the
// in-flight window stays one contiguous range; neighbours inside a run meet in one L2)
template <int W, bool NT, int XCD = 0>
__global__ __launch_bounds__(256) void k_copy(const char* a, char* c) {
    constexpr long SPC = COLB / SEG;
    long w = blockIdx.x;
    if (XCD < 0) {
        const long nb = gridDim.x, x = w % 8, per = nb / 8, i = w / 8;
        w = x * per + i;
    } else if (XCD > 0) {
        const long grp = w / (8 * XCD), in = w % (8 * XCD), x = in % 8, slot = in / 8;
        w = grp * (8 * XCD) + x * XCD + slot;
    }
    const long g = w / SPC, q = w % SPC;
    const long base = g * S * COLB + q * SEG;
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + threadIdx.x;  // 64 lanes per 1 KiB segment
        const u32x4* p = reinterpret_cast<const u32x4*>(a + base + (e / 64) * COLB + (e % 64) * 16);
        x[u] = __builtin_nontemporal_load(p);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + threadIdx.x;
        char* p = c + base + (e / 64) * COLB + (e % 64) * 16;
        if constexpr (W == 16) {
            if (NT) __builtin_nontemporal_store(x[u], reinterpret_cast<u32x4*>(p));
            else *reinterpret_cast<u32x4*>(p) = x[u];
        } else {
            u32x2 lo = {x[u].x, x[u].y}, hi = {x[u].z, x[u].w};
            if (NT) {
                __builtin_nontemporal_store(lo, reinterpret_cast<u32x2*>(p));
                __builtin_nontemporal_store(hi, reinterpret_cast<u32x2*>(p + 8));
            } else {
                *reinterpret_cast<u32x2*>(p) = lo;
                *reinterpret_cast<u32x2*>(p + 8) = hi;
            }
        }
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const long n = 2L << 30;
    char *A, *C;
    CK(hipMalloc(&A, n + 4096));
    CK(hipMalloc(&C, n + 4096));
    CK(hipMemset(A, 1, n + 4096));
    CK(hipMemset(C, 0, n + 4096));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned blocks = unsigned(n / (S * SEG));
    struct variant {
        const char* name;
        int off;
        void (*run)(const char*, char*, unsigned);
    };
    auto r16nt = [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, true>), dim3(b), dim3(256), 0, 0, a, c); };
    auto r16 = [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, false>), dim3(b), dim3(256), 0, 0, a, c); };
    auto r8nt = [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<8, true>), dim3(b), dim3(256), 0, 0, a, c); };
    auto r8 = [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<8, false>), dim3(b), dim3(256), 0, 0, a, c); };
    std::vector<variant> vs = {
        {"16B nt  off 0", 0, r16nt},   {"16B nt  off 128", 128, r16nt}, {"16B nt  off 16", 16, r16nt},
        {"16B nt  off 64", 64, r16nt}, {"16B def off 0", 0, r16},       {"16B def off 16", 16, r16},
        {"16B nt  off 32", 32, r16nt}, {"16B nt  off 48", 48, r16nt},   {"16B nt  off 96", 96, r16nt},
        {"8B  nt  off 0", 0, r8nt},    {"8B  nt  off 8", 8, r8nt},      {"8B  def off 8", 8, r8},
        {"16B xcd nt off 0", 0, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, true, -1>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B xcd def off 16", 16, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, false, -1>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B r2 nt off 0", 0, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, true, 2>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B r2 def off 16", 16, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, false, 2>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B r4 nt off 0", 0, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, true, 4>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B r4 def off 0", 0, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, false, 4>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B r4 def off 16", 16, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, false, 4>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B r4 nt off 16", 16, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, true, 4>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B r8 def off 16", 16, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, false, 8>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"16B r16 def off 16", 16, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<16, false, 16>), dim3(b), dim3(256), 0, 0, a, c); }},
        {"8B r4 def off 8", 8, [](const char* a, char* c, unsigned b) { hipLaunchKernelGGL((k_copy<8, false, 4>), dim3(b), dim3(256), 0, 0, a, c); }},
    };
    std::vector<std::vector<float>> t(vs.size());
    for (int r = 0; r < reps; ++r)
        for (size_t v = 0; v < vs.size(); ++v) {
            CK(hipEventRecord(e0));
            vs[v].run(A, C + vs[v].off, blocks);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            t[v].push_back(ms);
        }
    for (size_t v = 0; v < vs.size(); ++v) {
        std::sort(t[v].begin(), t[v].end());
        const float med = t[v][t[v].size() / 2];
        printf("%-18s median %.4f ms  %.1f GB/s (algorithmic read + write)\n", vs[v].name, med,
               2.0 * n / (med * 1e-3) / 1e9);
    }
    return 0;
}
