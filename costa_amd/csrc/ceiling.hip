// Measurement support for bench.py (not part of the transform path): what a plain device copy
// of the headline workload's bytes reaches on THIS box, so that the tile kernel's roofline
// fraction can be read against a ceiling the same run measured ("also report a
// measured hipMemcpyDtoD ceiling").  Built as its own library, libcosta_ceiling.so; the product
// library does not link it.
//
//   kind 0  hipMemcpyDtoD of `bytes` (one call)
//   kind 1  strided column-segment copy: the source and destination are column-major matrices of
//           `col_bytes`-byte columns; a 256-thread workgroup copies 16 KiB as 16 segments of
//           1 KiB (one per column), consecutive workgroups continue down the same 16 columns,
//           nontemporal 16-byte loads and stores.  This is the fastest copy of cfg 2's bytes
//           measured on MI355X (tools/copy_ceiling.hip "seg 1024 nt/nt").
//   kind 2  flat copy, one 16 KiB chunk per 256-thread workgroup, nontemporal loads and stores
//   kind 3  flat copy, one 1 KiB chunk per 64-thread workgroup (one 16-byte vector per thread)
//   kind 4  the strided segment copy of kind 1 with one vector per thread: a 256-thread
//           workgroup copies 4 columns' 1 KiB segments.  Kinds 3 and 4 keep fewer loads in flight
//           per thread (1 against 4) and ran 6.6-6.7 TB/s against kind 1's 6.2-6.3 on MI355X
//           (profiles/r4zj/)
//   kind 5  the headline transpose's access pattern without its LDS exchange (a probe, not a
//           ceiling: tools/pairs_probe.py): src and dst square column-major fp64 matrices of
//           `col_bytes`-byte columns, 512-thread workgroups on 64 x 128 sub-tiles in destination
//           order; each thread loads 8 16-byte vectors where the transpose loads them (128 source
//           columns x 512 B) and stores 8 where it stores (64 destination columns x 1 KiB),
//           the data merely moved, not transposed
//   kind 6  the same pattern for 128 x 128 sub-tiles (1 KiB segments on both sides), 1024 threads
//   kind 7  kind 5's loads with flat stores; kind 8  flat loads with kind 5's stores
//   kinds 100 + 10 g + m  the pattern of other sub-tile geometries (pat_g below)
//   kinds 200 + p  kind 5 with other store cache policies (tr_pattern_pol below)
//   kinds 300 + o  kind 5 with other sub-tile orders (tr_pattern_ord below)
//
// costa_ceiling_copy_ms runs `reps` timed repetitions (HIP events on its own stream) after one
// untimed one and writes every repetition's milliseconds to ms_out[0..reps).  Returns 0, or a
// negative code: -1 bad arguments, -2 a HIP error.
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kSegBytes = 1024;
constexpr int kSegs = 16;  // 16 KiB per workgroup
constexpr int kLanesPerSeg = kSegBytes / 16;

__global__ __launch_bounds__(kThreads) void seg_copy(const u32x4* __restrict__ a,
                                                     u32x4* __restrict__ c, long col16,
                                                     long segs_per_col) {
    const long w = blockIdx.x;
    const long g = w / segs_per_col, q = w % segs_per_col;
    const long base = g * kSegs * col16 + q * kLanesPerSeg;
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * kThreads + int(threadIdx.x);
        x[u] = __builtin_nontemporal_load(a + base + (e / kLanesPerSeg) * col16 + e % kLanesPerSeg);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * kThreads + int(threadIdx.x);
        __builtin_nontemporal_store(x[u], c + base + (e / kLanesPerSeg) * col16 + e % kLanesPerSeg);
    }
}

__global__ __launch_bounds__(kThreads) void flat_copy(const u32x4* __restrict__ a,
                                                      u32x4* __restrict__ c) {
    const long base = long(blockIdx.x) * 4 * kThreads;
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
        x[u] = __builtin_nontemporal_load(a + base + u * kThreads + threadIdx.x);
#pragma unroll
    for (int u = 0; u < 4; ++u)
        __builtin_nontemporal_store(x[u], c + base + u * kThreads + threadIdx.x);
}

// kinds 3 and 4: one 16-byte vector per thread
__global__ __launch_bounds__(64) void flat_copy_1k(const u32x4* __restrict__ a, u32x4* __restrict__ c) {
    const long i = long(blockIdx.x) * 64 + threadIdx.x;
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), c + i);
}

constexpr int kSegs1 = 4;  // kind 4: columns per 256-thread workgroup
__global__ __launch_bounds__(kThreads) void seg_copy_1(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                       long col16, long segs_per_col) {
    const long w = blockIdx.x;
    const long g = w / segs_per_col, q = w % segs_per_col;
    const int e = int(threadIdx.x);
    const long i = (g * kSegs1 + e / kLanesPerSeg) * col16 + q * kLanesPerSeg + e % kLanesPerSeg;
    __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), c + i);
}

// kind 5: the transpose's loads and stores without LDS (fp64, 64 x 128 sub-tiles, 512 threads)
__global__ __launch_bounds__(512) void tr_pattern(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                  long n, long sblocks) {
    const long w = blockIdx.x;
    const long f0 = (w / sblocks) * 64, s0 = (w % sblocks) * 128;  // band-major destination order
    const int t = int(threadIdx.x);
    u32x4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // source column s0 + t / 32 + 16 k, rows f0 + 2 (t % 32) ..
        const long s = s0 + t / 32 + 16 * k;
        x[k] = __builtin_nontemporal_load(a + (s * n + f0) / 2 + t % 32);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // destination column f0 + 8 (t / 64) + k, rows s0 + 2 (t % 64) ..
        const long f = f0 + 8 * (t / 64) + k;
        __builtin_nontemporal_store(x[k], c + (f * n + s0) / 2 + t % 64);
    }
}

// kind 6: the same for 128 x 128 sub-tiles (1 KiB segments on both sides), 1024 threads
__global__ __launch_bounds__(1024) void tr_pattern_sq(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                      long n, long sblocks) {
    const long w = blockIdx.x;
    const long f0 = (w / sblocks) * 128, s0 = (w % sblocks) * 128;
    const int t = int(threadIdx.x);
    u32x4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // source column s0 + t / 64 + 16 k, rows f0 + 2 (t % 64) ..
        const long s = s0 + t / 64 + 16 * k;
        x[k] = __builtin_nontemporal_load(a + (s * n + f0) / 2 + t % 64);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // destination column f0 + 8 (t / 64) + k, rows s0 + 2 (t % 64) ..
        const long f = f0 + 8 * (t / 64) + k;
        __builtin_nontemporal_store(x[k], c + (f * n + s0) / 2 + t % 64);
    }
}

// kinds 7 / 8: half of kind 5's pattern each -- 7: its loads, stores flat (workgroup w writes
// the 64 KiB at w * 64 KiB); 8: loads flat, its stores
template <bool TR_LOADS>
__global__ __launch_bounds__(512) void tr_half_pattern(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                       long n, long sblocks) {
    const long w = blockIdx.x;
    const long f0 = (w / sblocks) * 64, s0 = (w % sblocks) * 128;
    const int t = int(threadIdx.x);
    u32x4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long s = s0 + t / 32 + 16 * k;
        x[k] = __builtin_nontemporal_load(TR_LOADS ? a + (s * n + f0) / 2 + t % 32 : a + w * 4096 + k * 512 + t);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long f = f0 + 8 * (t / 64) + k;
        __builtin_nontemporal_store(x[k], TR_LOADS ? c + w * 4096 + k * 512 + t : c + (f * n + s0) / 2 + t % 64);
    }
}

// kinds 100 + 10 g + m (probes): the transposing access pattern of BF x BS fp64 sub-tiles (64 KiB,
// 512 threads, 8 16-byte vectors a thread each way, destination order), geometry g: 0 64 x 128,
// 1 32 x 256, 2 16 x 512, 3 128 x 64, 4 256 x 32; m 0: transposed loads and stores, 1: flat
// loads (workgroup w reads the 64 KiB at w * 64 KiB) with transposed stores, 2: transposed loads
// with flat stores
template <int BF, int BS, int M>
__global__ __launch_bounds__(512) void pat_g(const u32x4* __restrict__ a, u32x4* __restrict__ c, long n) {
    constexpr int LPC = BF / 2, CPP = 512 / LPC, LPD = BS / 2, CPD = 512 / LPD;
    static_assert(BF * BS == 8192 && CPP * 8 == BS && CPD * 8 == BF, "geometry");
    const long sblocks = n / BS, w = blockIdx.x;
    const long f0 = (w / sblocks) * BF, s0 = (w % sblocks) * BS;
    const int t = int(threadIdx.x);
    u32x4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long s = s0 + t / LPC + CPP * k;
        x[k] = __builtin_nontemporal_load(M == 1 ? a + w * 4096 + k * 512 + t : a + (s * n + f0) / 2 + t % LPC);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long f = f0 + t / LPD + CPD * k;
        __builtin_nontemporal_store(x[k], M == 2 ? c + w * 4096 + k * 512 + t : c + (f * n + s0) / 2 + t % LPD);
    }
}
template <int BF, int BS>
hipError_t launch_pat(int m, const u32x4* a, u32x4* c, long n, hipStream_t s) {
    const unsigned grid = unsigned((n / BF) * (n / BS));
    if (m == 0) hipLaunchKernelGGL((pat_g<BF, BS, 0>), dim3(grid), dim3(512), 0, s, a, c, n);
    if (m == 1) hipLaunchKernelGGL((pat_g<BF, BS, 1>), dim3(grid), dim3(512), 0, s, a, c, n);
    if (m == 2) hipLaunchKernelGGL((pat_g<BF, BS, 2>), dim3(grid), dim3(512), 0, s, a, c, n);
    return hipGetLastError();
}

// kinds 200 + p (probes): kind 5's pattern with the stores' cache policy p: 0 nt, 1 default,
// 2 sc1, 3 sc1 nt, 4 sc0 nt, 5 sc0 sc1 nt (vector stores through inline asm)
template <int P>
__device__ __forceinline__ void st_pol(u32x4* p, u32x4 v) {
    if constexpr (P == 0) __builtin_nontemporal_store(v, p);
    if constexpr (P == 1) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(p), "v"(v) : "memory");
    if constexpr (P == 2) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
    if constexpr (P == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
    if constexpr (P == 4) asm volatile("global_store_dwordx4 %0, %1, off sc0 nt" ::"v"(p), "v"(v) : "memory");
    if constexpr (P == 5) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
}
template <int P>
__global__ __launch_bounds__(512) void tr_pattern_pol(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                      long n, long sblocks) {
    const long w = blockIdx.x;
    const long f0 = (w / sblocks) * 64, s0 = (w % sblocks) * 128;
    const int t = int(threadIdx.x);
    u32x4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long s = s0 + t / 32 + 16 * k;
        x[k] = __builtin_nontemporal_load(a + (s * n + f0) / 2 + t % 32);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long f = f0 + 8 * (t / 64) + k;
        st_pol<P>(c + (f * n + s0) / 2 + t % 64, x[k]);
    }
}

// kinds 300 + o (probes): kind 5's pattern with another order of the sub-tiles (workgroup i ->
// band, s-block; nb bands of 64 destination columns, sb s-blocks of 128 rows):
// 0 band-major (shipped), 1 each band bottom to top, 2 the bands in reverse, 3 boustrophedon,
// 4 one band per XCD (workgroups are dealt round-robin over 8 XCDs: 8 bands in flight, XCD x on
// band 8 j + x), 5 four bands advancing together one s-block at a time, 6 (r6) band-major with
// a per-XCD row-band rotation: XCD x = i mod 8 starts its share of each band x eighths of the
// column further down (s-block (j + x sb / 8) mod sb), so the workgroups resident at one time on
// different XCDs write different in-column offsets
__global__ __launch_bounds__(512) void tr_pattern_ord(const u32x4* __restrict__ a, u32x4* __restrict__ c,
                                                      long n, int o) {
    const long sb = n / 128, nb = n / 64, i = blockIdx.x;
    long band = i / sb, blk = i % sb;
    if (o == 1) blk = sb - 1 - blk;
    if (o == 2) band = nb - 1 - band;
    if (o == 3 && band % 2) blk = sb - 1 - blk;
    if (o == 4) band = 8 * (i / (8 * sb)) + i % 8, blk = (i / 8) % sb;
    if (o == 5) band = 4 * (i / (4 * sb)) + i % 4, blk = (i % (4 * sb)) / 4;
    if (o == 6) blk = (blk + (i % 8) * (sb / 8)) % sb;  // a permutation of the band when 8 | sb
    const long f0 = band * 64, s0 = blk * 128;
    const int t = int(threadIdx.x);
    u32x4 x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long s = s0 + t / 32 + 16 * k;
        x[k] = __builtin_nontemporal_load(a + (s * n + f0) / 2 + t % 32);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const long f = f0 + 8 * (t / 64) + k;
        __builtin_nontemporal_store(x[k], c + (f * n + s0) / 2 + t % 64);
    }
}

// kinds 400 / 401 (probes, r6): 64 x 256 fp64 sub-tiles (128 KiB), destination order; each
// wavefront writes whole 2 KiB destination column segments, a column's two 1 KiB halves by two
// back-to-back instructions.  400: 1024 threads x 8 vectors; 401: 512 threads x 16
template <int NT>
__global__ __launch_bounds__(NT) void tr_pattern_2k(const u32x4* __restrict__ a, u32x4* __restrict__ c, long n) {
    constexpr int PL = 8192 / NT;  // 16-byte vectors a thread
    const long sb = n / 256, w = blockIdx.x;
    const long f0 = (w / sb) * 64, s0 = (w % sb) * 256;
    const int t = int(threadIdx.x), lane = t % 64, wave = t / 64;
    u32x4 x[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) {  // source column s0 + t / 32 + (NT / 32) k, rows f0 + 2 (t % 32) ..
        const long s = s0 + t / 32 + (NT / 32) * k;
        x[k] = __builtin_nontemporal_load(a + (s * n + f0) / 2 + t % 32);
    }
#pragma unroll
    for (int k = 0; k < PL; ++k) {  // column f0 + (PL / 2) wave + k / 2, rows s0 + 128 (k % 2) + 2 lane ..
        const long f = f0 + (PL / 2) * wave + k / 2;
        __builtin_nontemporal_store(x[k], c + (f * n + s0) / 2 + 64 * (k % 2) + lane);
    }
}

}  // namespace

extern "C" int costa_ceiling_copy_ms(int kind, const void* src, void* dst, uint64_t bytes,
                                     uint64_t col_bytes, int reps, float* ms_out) {
    if (!src || !dst || !ms_out || reps <= 0 || bytes == 0 || bytes % (kSegs * kSegBytes))
        return -1;
    long grid = long(bytes / (kSegs * kSegBytes));
    if (kind == 1 || kind == 4) {
        // whole 16-column groups of whole 1 KiB segments only: no tail handling needed
        if (col_bytes == 0 || col_bytes % kSegBytes || bytes % (kSegs * col_bytes)) return -1;
    } else if (kind == 6) {
        const uint64_t n = col_bytes / 8;
        if (col_bytes % 1024 || bytes != n * col_bytes) return -1;
        grid = long((n / 128) * (n / 128));
    } else if (kind >= 100 && kind < 150 && kind % 10 < 3) {
        const uint64_t n = col_bytes / 8;
        if (col_bytes % 4096 || bytes != n * col_bytes) return -1;
        grid = 1;
    } else if (kind == 400 || kind == 401) {
        const uint64_t n = col_bytes / 8;
        if (col_bytes % 2048 || bytes != n * col_bytes) return -1;
        grid = long((n / 64) * (n / 256));
    } else if (kind == 5 || kind == 7 || kind == 8 || (kind >= 200 && kind <= 205) ||
               (kind >= 300 && kind <= 306)) {
        // square fp64: n = col_bytes / 8 columns of n elements, n a multiple of 128
        const uint64_t n = col_bytes / 8;
        if (col_bytes % 1024 || bytes != n * col_bytes) return -1;
        grid = long((n / 64) * (n / 128));
    } else if (kind != 0 && kind != 2 && kind != 3) {
        return -1;
    }
    if (kind == 3) grid = long(bytes / kSegBytes);            // one 1 KiB chunk per workgroup
    if (kind == 4) grid = long(bytes / (kSegs1 * kSegBytes));  // four 1 KiB segments per workgroup
    if (grid > 0x7fffffffL) return -1;
    hipStream_t s;
    hipEvent_t e0, e1;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -2;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return -2;
    const u32x4* a = static_cast<const u32x4*>(src);
    u32x4* c = static_cast<u32x4*>(dst);
    const long col16 = long(col_bytes / 16), spc = long(col_bytes / kSegBytes);
    auto once = [&]() -> hipError_t {
        if (kind == 0) return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s);
        if (kind >= 400) {
            const long n = long(col_bytes / 8);
            if (kind == 400)
                hipLaunchKernelGGL(tr_pattern_2k<1024>, dim3(unsigned(grid)), dim3(1024), 0, s, a, c, n);
            else
                hipLaunchKernelGGL(tr_pattern_2k<512>, dim3(unsigned(grid)), dim3(512), 0, s, a, c, n);
            return hipGetLastError();
        }
        if (kind >= 300) {
            const long n = long(col_bytes / 8);
            hipLaunchKernelGGL(tr_pattern_ord, dim3(unsigned((n / 64) * (n / 128))), dim3(512), 0, s, a, c, n,
                               kind - 300);
            return hipGetLastError();
        }
        if (kind >= 200) {
            const long n = long(col_bytes / 8), sb = n / 128;
            const dim3 gr(unsigned((n / 64) * (n / 128)));
            switch (kind - 200) {
            case 0: hipLaunchKernelGGL(tr_pattern_pol<0>, gr, dim3(512), 0, s, a, c, n, sb); break;
            case 1: hipLaunchKernelGGL(tr_pattern_pol<1>, gr, dim3(512), 0, s, a, c, n, sb); break;
            case 2: hipLaunchKernelGGL(tr_pattern_pol<2>, gr, dim3(512), 0, s, a, c, n, sb); break;
            case 3: hipLaunchKernelGGL(tr_pattern_pol<3>, gr, dim3(512), 0, s, a, c, n, sb); break;
            case 4: hipLaunchKernelGGL(tr_pattern_pol<4>, gr, dim3(512), 0, s, a, c, n, sb); break;
            default: hipLaunchKernelGGL(tr_pattern_pol<5>, gr, dim3(512), 0, s, a, c, n, sb); break;
            }
            return hipGetLastError();
        }
        if (kind >= 100) {
            const long n = long(col_bytes / 8);
            const int g = (kind - 100) / 10, m = kind % 10;
            if (g == 0) return launch_pat<64, 128>(m, a, c, n, s);
            if (g == 1) return launch_pat<32, 256>(m, a, c, n, s);
            if (g == 2) return launch_pat<16, 512>(m, a, c, n, s);
            if (g == 3) return launch_pat<128, 64>(m, a, c, n, s);
            return launch_pat<256, 32>(m, a, c, n, s);
        }
        if (kind == 1)
            hipLaunchKernelGGL(seg_copy, dim3(unsigned(grid)), dim3(kThreads), 0, s, a, c, col16, spc);
        else if (kind == 2)
            hipLaunchKernelGGL(flat_copy, dim3(unsigned(grid)), dim3(kThreads), 0, s, a, c);
        else if (kind == 3)
            hipLaunchKernelGGL(flat_copy_1k, dim3(unsigned(grid)), dim3(64), 0, s, a, c);
        else if (kind == 4)
            hipLaunchKernelGGL(seg_copy_1, dim3(unsigned(grid)), dim3(kThreads), 0, s, a, c, col16, spc);
        else if (kind == 5)
            hipLaunchKernelGGL(tr_pattern, dim3(unsigned(grid)), dim3(512), 0, s, a, c, long(col_bytes / 8),
                               long(col_bytes / 8 / 128));
        else if (kind == 7)
            hipLaunchKernelGGL(tr_half_pattern<true>, dim3(unsigned(grid)), dim3(512), 0, s, a, c,
                               long(col_bytes / 8), long(col_bytes / 8 / 128));
        else if (kind == 8)
            hipLaunchKernelGGL(tr_half_pattern<false>, dim3(unsigned(grid)), dim3(512), 0, s, a, c,
                               long(col_bytes / 8), long(col_bytes / 8 / 128));
        else
            hipLaunchKernelGGL(tr_pattern_sq, dim3(unsigned(grid)), dim3(1024), 0, s, a, c, long(col_bytes / 8),
                               long(col_bytes / 8 / 128));
        return hipGetLastError();
    };
    int rc = 0;
    if (once() != hipSuccess) rc = -2;
    for (int r = 0; r < reps && rc == 0; ++r) {
        if (hipEventRecord(e0, s) != hipSuccess || once() != hipSuccess ||
            hipEventRecord(e1, s) != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
            hipEventElapsedTime(&ms_out[r], e0, e1) != hipSuccess)
            rc = -2;
    }
    if (hipStreamSynchronize(s) != hipSuccess) rc = -2;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipStreamDestroy(s);
    return rc;
}
