// Tuning probe (not part of the product): what a plain device copy of BASELINE cfg 2's bytes
// (2 GiB read + 2 GiB written) reaches on this MI355X, against MI355X_MICROARCH.md's "6.29 TB/s
// measured (float4 copy)" and its LDS-DMA read rates (6.4 default, 6.5-6.8 nt).  Every variant
// runs interleaved in one process (median of R repetitions); copies are verified.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/copy_ceiling.hip -o /tmp/cc && /tmp/cc [R] [filter]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <type_traits>
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

// buffer resource of one region (wave-uniform base), offsets < 2^31
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}

// ---- A: grid-stride, U 16-B loads per thread then U stores; cache-policy bits via buffer ops
// LA / SA: aux bits of loads / stores (0 default, 2 nt, 16 sc1, 3 sc0+nt ...)
template <int U, int LA, int SA>
__global__ __launch_bounds__(256) void k_stride(const u32x4* a, u32x4* c, long n) {
    const long per = long(U) * 256;
    for (long base = blockIdx.x * per; base < n; base += long(gridDim.x) * per) {
        const auto ra = rsrc(a + base);
        const auto rc = rsrc(c + base);
        u32x4 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u)
            x[u] = __builtin_amdgcn_raw_buffer_load_b128(ra, (u * 256 + threadIdx.x) * 16, 0, LA);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(x[u], rc, (u * 256 + threadIdx.x) * 16, 0, SA);
    }
}

// ---- B: one chunk per workgroup (no grid-stride): CH = U * NT * 16 bytes per WG
template <int U, int NT, int NTL = 0, int NTS = 0>
__global__ __launch_bounds__(NT) void k_chunk(const u32x4* a, u32x4* c) {
    const long base = long(blockIdx.x) * U * NT;
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        const u32x4* p = a + base + u * NT + threadIdx.x;
        x[u] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
        u32x4* p = c + base + u * NT + threadIdx.x;
        if (NTS) __builtin_nontemporal_store(x[u], p); else *p = x[u];
    }
}

// ---- C: software-pipelined grid-stride: chunk k+1's loads are issued before chunk k's stores
template <int U>
__global__ __launch_bounds__(256) void k_pipe(const u32x4* a, u32x4* c, long n) {
    const long per = long(U) * 256, step = long(gridDim.x) * per;
    long base = blockIdx.x * per;
    if (base >= n) return;
    u32x4 x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = a[base + u * 256 + threadIdx.x];
    for (;;) {
        const long nb = base + step;
        const bool more = nb < n;
        if (more) {
#pragma unroll
            for (int u = 0; u < U; ++u) y[u] = a[nb + u * 256 + threadIdx.x];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) c[base + u * 256 + threadIdx.x] = x[u];
        if (!more) break;
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = y[u];
        base = nb;
    }
}

// ---- D: LDS-DMA copy: every wave streams its own chunks through a private LDS ring of NB slots
// of 1 KiB x K (K global_load_lds_dwordx4 per slot), then reads the slot back and stores it.
template <int K, int NB, int AUX>
__global__ __launch_bounds__(256) void k_ldsdma(const u32x4* a, u32x4* c, long n) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x % 64;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / 64);
    unsigned char* ring = smem + size_t(wave) * NB * K * 1024;
    const long per = long(K) * 64;  // 16-B elements per slot
    const long nw = long(gridDim.x) * 4;
    const long w0 = long(blockIdx.x) * 4 + wave;
    const long nchunks = n / per;
    auto issue = [&](long ch, int slot) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void*)(a + ch * per + k * 64 + lane),
                (__attribute__((address_space(3))) void*)(ring + (slot * K + k) * 1024), 16, 0, AUX);
    };
    long ch = w0;
    int head = 0;
    for (int q = 0; q < NB - 1; ++q)
        if (ch + q * nw < nchunks) issue(ch + q * nw, q);
    for (long it = 0; ch + it * nw < nchunks; ++it) {
        const long cur = ch + it * nw;
        // wait for everything older than the NB-2 newer slots' loads (and this slot's stores)
        __builtin_amdgcn_s_waitcnt(0);  // simple form: drain (the loads of later slots too)
        const long nxt = cur + (NB - 1) * nw;
        if (nxt < nchunks) issue(nxt, (head + NB - 1) % NB);
        u32x4 v[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
            v[k] = *reinterpret_cast<const u32x4*>(ring + (head * K + k) * 1024 + lane * 16);
#pragma unroll
        for (int k = 0; k < K; ++k) c[cur * per + k * 64 + lane] = v[k];
        head = (head + 1) % NB;
    }
}

// ---- F: strided 2-D copy (no transpose): the source and destination are 16384 x 16384 fp64
// column-major (a column = 128 KiB); every 256-thread WG copies 16 KiB = S column segments of L
// bytes.  Consecutive WGs take consecutive segments of the same S columns.
template <int L, int NTL, int NTS>
__global__ __launch_bounds__(256) void k_seg(const u32x4* a, u32x4* c) {
    constexpr int S = 16384 / L, LPS = L / 16;  // segments per WG, lanes per segment
    constexpr long COL = 131072 / 16;           // column length in 16-B units
    constexpr int SPC = 131072 / L;             // segments per column
    const long w = blockIdx.x;
    const long g = w / SPC, q = w % SPC;
    const long base = g * S * COL + q * LPS;
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + threadIdx.x;
        const u32x4* p = a + base + (e / LPS) * COL + e % LPS;
        x[u] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + threadIdx.x;
        u32x4* p = c + base + (e / LPS) * COL + e % LPS;
        if (NTS) __builtin_nontemporal_store(x[u], p); else *p = x[u];
    }
}

// ---- G: the HBM access pattern of a BF x BS fp64 tile transpose (cfg 2: 16384^2, 256^2 blocks,
// sub-tiles of a block consecutive, blocks in column-major order), WITHOUT the transpose: every
// thread stores the vectors it loaded at the addresses the real kernel's stores use (the data land
// in the wrong places; only the traffic is the same).  No LDS, no barrier.
// ORD: order of the 64 x 64 blocks in the grid: 0 column-major (block row fastest, the
// product's r01 order), SB > 1: super-blocks of SB x SB blocks (column-major inside and
// between super-blocks), -1 row-major
template <int BF, int BS, int NT, int NTL, int NTS, int ORD = 0>
__global__ __launch_bounds__(NT) void k_pat(const double* a, double* c) {
    constexpr long LD = 16384;
    constexpr int SUBF = 256 / BF, SUBS = 256 / BS;
    const long w = blockIdx.x;
    const long b = w / (SUBF * SUBS), sub = w % (SUBF * SUBS);
    long bi, bj;
    if (ORD == 0) {
        bi = b % 64, bj = b / 64;
    } else if (ORD == -1) {
        bj = b % 64, bi = b / 64;
    } else if (ORD == -2) {  // diagonals: block k of diagonal d is (k, k + d)
        bi = b % 64, bj = (b % 64 + b / 64) % 64;
    } else if (ORD == -3) {  // anti-diagonal stripes with stride 8 in bj
        bi = b % 64, bj = (b / 64 + 8 * (b % 64)) % 64;
    } else if (ORD <= -10 && ORD > -20) {  // S = -10 - ORD interleaved write streams, each
        // walking down its own C column band (= along its own A block-row)
        constexpr long S = ORD <= -10 && ORD > -20 ? -10 - ORD : 1;
        const long g = b % S, t = b / S;
        bi = g * (64 / S) + t / 64, bj = t % 64;
    } else if (ORD <= -20) {  // the same, stream g starting at block column g * 64 / S
        constexpr long S = ORD <= -20 ? -20 - ORD : 1;
        const long g = b % S, t = b / S;
        bi = g * (64 / S) + t / 64, bj = (t + g * (64 / S)) % 64;
    } else {
        constexpr long SB = ORD > 0 ? ORD : 1, NSB = 64 / SB;
        const long sb = b / (SB * SB), in = b % (SB * SB);
        bi = (sb % NSB) * SB + in % SB;
        bj = (sb / NSB) * SB + in / SB;
    }
    const long f0 = bi * 256 + (sub % SUBF) * BF, s0 = bj * 256 + (sub / SUBF) * BS;
    constexpr int LPC = BF / 2, CPP = NT / LPC, PL = BS / CPP;
    const int lf = (threadIdx.x % LPC) * 2, c0 = threadIdx.x / LPC;
    typedef double d2 __attribute__((ext_vector_type(2)));
    d2 x[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
        const d2* p = reinterpret_cast<const d2*>(a + (s0 + c0 + CPP * k) * LD + f0 + lf);
        x[k] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
    // store k of a thread: 16-B vector e = k * NT + thread in destination order (rows f of BS
    // s-values), i.e. consecutive lanes store consecutive 16 B of a row, as the real kernel does
#pragma unroll
    for (int k = 0; k < PL; ++k) {
        const int e = k * NT + int(threadIdx.x);
        const int f = e / (BS / 2), so = (e % (BS / 2)) * 2;
        d2* q = reinterpret_cast<d2*>(c + (f0 + f) * LD + s0 + so);
        if (NTS) __builtin_nontemporal_store(x[k], q); else *q = x[k];
    }
}

// ---- F2: strided copy where consecutive WGs take the SAME segment of the next 16 columns
// (the in-flight WGs then all read / write one in-column offset range of many columns)
template <int L, int NTL, int NTS>
__global__ __launch_bounds__(256) void k_seg_camp(const u32x4* a, u32x4* c) {
    constexpr int S = 16384 / L, LPS = L / 16;
    constexpr long COL = 131072 / 16;
    constexpr long NG = 16384 / S;  // column groups
    const long w = blockIdx.x;
    const long g = w % NG, q = w / NG;
    const long base = g * S * COL + q * LPS;
    u32x4 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + threadIdx.x;
        const u32x4* p = a + base + (e / LPS) * COL + e % LPS;
        x[u] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = u * 256 + threadIdx.x;
        u32x4* p = c + base + (e / LPS) * COL + e % LPS;
        if (NTS) __builtin_nontemporal_store(x[u], p); else *p = x[u];
    }
}

// ---- H: flat copy with narrow lanes: W-byte accesses (4, 8, 16), U per thread, 16 KiB per
// 256-thread WG for W = 16 (the same bytes per WG for every W: U = 64 / W * 4)
template <int W, int NTL, int NTS>
__global__ __launch_bounds__(256) void k_narrow(const unsigned char* a, unsigned char* c) {
    typedef unsigned int u1 __attribute__((ext_vector_type(1)));
    typedef unsigned int u2 __attribute__((ext_vector_type(2)));
    using T = typename std::conditional<W == 4, unsigned int,
              typename std::conditional<W == 8, u2, u32x4>::type>::type;
    constexpr int U = 16384 / (256 * W);
    const T* s = reinterpret_cast<const T*>(a) + long(blockIdx.x) * U * 256;
    T* d = reinterpret_cast<T*>(c) + long(blockIdx.x) * U * 256;
    T x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) x[u] = NTL ? __builtin_nontemporal_load(s + u * 256 + threadIdx.x) : s[u * 256 + threadIdx.x];
#pragma unroll
    for (int u = 0; u < U; ++u) {
        if (NTS) __builtin_nontemporal_store(x[u], d + u * 256 + threadIdx.x); else d[u * 256 + threadIdx.x] = x[u];
    }
}

// ---- E: read-only and write-only streams
template <int U, int LA>
__global__ __launch_bounds__(256) void k_read(const u32x4* a, long n, u32x4* sink) {
    u32x4 acc = {0, 0, 0, 0};
    const long per = long(U) * 256;
    for (long base = blockIdx.x * per; base < n; base += long(gridDim.x) * per) {
        const auto ra = rsrc(a + base);
#pragma unroll
        for (int u = 0; u < U; ++u)
            acc ^= __builtin_amdgcn_raw_buffer_load_b128(ra, (u * 256 + threadIdx.x) * 16, 0, LA);
    }
    if (acc.x == 0x12345678u && acc.y == 0x9abcdef0u) sink[threadIdx.x] = acc;
}
template <int K, int AUX>
__global__ __launch_bounds__(256) void k_read_lds(const u32x4* a, long n, u32x4* sink) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x % 64;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / 64);
    unsigned char* slot = smem + size_t(wave) * K * 1024;
    const long per = long(K) * 64, nw = long(gridDim.x) * 4;
    for (long ch = long(blockIdx.x) * 4 + wave; ch < n / per; ch += nw) {
#pragma unroll
        for (int k = 0; k < K; ++k)
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void*)(a + ch * per + k * 64 + lane),
                (__attribute__((address_space(3))) void*)(slot + k * 1024), 16, 0, AUX);
    }
    __builtin_amdgcn_s_waitcnt(0);
    const u32x4 v = *reinterpret_cast<const u32x4*>(slot + lane * 16);
    if (v.x == 0x12345678u && v.y == 0x9abcdef0u) sink[threadIdx.x] = v;
}
template <int U, int SA>
__global__ __launch_bounds__(256) void k_write(u32x4* c, long n) {
    const long per = long(U) * 256;
    const u32x4 v = {1u, 2u, 3u, 4u};
    for (long base = blockIdx.x * per; base < n; base += long(gridDim.x) * per) {
        const auto rc = rsrc(c + base);
#pragma unroll
        for (int u = 0; u < U; ++u)
            __builtin_amdgcn_raw_buffer_store_b128(v, rc, (u * 256 + threadIdx.x) * 16, 0, SA);
    }
}

__global__ void fill(u32x4* a, long n) {
    for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x)
        a[i] = u32x4{unsigned(i), unsigned(i >> 32) ^ 0x5au, unsigned(i * 2654435761u), 7u};
}
__global__ void check(const u32x4* a, const u32x4* c, long n, unsigned long long* bad) {
    for (long i = blockIdx.x * long(blockDim.x) + threadIdx.x; i < n; i += long(gridDim.x) * blockDim.x) {
        const u32x4 x = a[i], y = c[i];
        if (x.x != y.x || x.y != y.y || x.z != y.z || x.w != y.w) atomicAdd(bad, 1ull);
    }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const std::string filt = argc > 2 ? argv[2] : "";
    const long bytes1 = 2L << 30;  // one side of cfg 2
    const long n = bytes1 / 16;
    u32x4 *A, *Cm, *sink;
    CK(hipMalloc(&A, bytes1));
    CK(hipMalloc(&Cm, bytes1));
    CK(hipMalloc(&sink, 4096));
    unsigned long long* bad;
    CK(hipMalloc(&bad, 8));
    hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, A, n);
    CK(hipDeviceSynchronize());
    const int cus = 256;
    struct var {
        std::string name;
        std::function<void()> run;
        double traffic;  // bytes
        bool verify;
        std::vector<float> ms;
    };
    std::vector<var> V;
    const double T = 2.0 * bytes1;
    auto add = [&](std::string name, std::function<void()> f, double tr, bool ver) {
        if (filt.empty() || name.find(filt) != std::string::npos) V.push_back({name, f, tr, ver, {}});
    };
#define STRIDE(U, LA, SA, G)                                                                      \
    add("stride U" #U " ld" #LA " st" #SA " " #G "/CU",                                          \
        [&] { hipLaunchKernelGGL((k_stride<U, LA, SA>), dim3(cus * G), dim3(256), 0, 0, A, Cm, n); }, T, true)
    STRIDE(8, 0, 0, 8);
    STRIDE(8, 0, 0, 4);
    STRIDE(8, 0, 0, 16);
    STRIDE(4, 0, 0, 8);
    STRIDE(16, 0, 0, 4);
    STRIDE(8, 2, 0, 8);
    STRIDE(8, 0, 2, 8);
    STRIDE(8, 2, 2, 8);
    STRIDE(8, 0, 16, 8);
    STRIDE(8, 2, 16, 8);
    STRIDE(8, 0, 3, 8);
    STRIDE(8, 0, 1, 8);
#define CHUNK(U, NT)                                                                              \
    add("chunk U" #U " t" #NT, [&] {                                                              \
        hipLaunchKernelGGL((k_chunk<U, NT>), dim3(unsigned(n / (U * NT))), dim3(NT), 0, 0, A, Cm); \
    }, T, true)
#define CHUNKNT(U, NT)                                                                            \
    add("chunk U" #U " t" #NT " nt-both", [&] {                                                    \
        hipLaunchKernelGGL((k_chunk<U, NT, 1, 1>), dim3(unsigned(n / (U * NT))), dim3(NT), 0, 0, A, Cm); \
    }, T, true)
    CHUNKNT(4, 256);
    CHUNKNT(8, 256);
    CHUNKNT(8, 1024);
    CHUNKNT(4, 1024);
    CHUNKNT(8, 512);
    CHUNKNT(16, 256);
    STRIDE(8, 2, 2, 16);
    STRIDE(8, 2, 2, 4);
    STRIDE(4, 2, 2, 16);
    STRIDE(16, 2, 2, 4);
    STRIDE(8, 2, 18, 8);
    CHUNK(4, 256);
    CHUNK(8, 256);
    CHUNK(16, 256);
    CHUNK(8, 512);
    CHUNK(4, 1024);
    CHUNK(8, 1024);
    add("pipe U4 8/CU", [&] { hipLaunchKernelGGL((k_pipe<4>), dim3(cus * 8), dim3(256), 0, 0, A, Cm, n); }, T, true);
    add("pipe U8 4/CU", [&] { hipLaunchKernelGGL((k_pipe<8>), dim3(cus * 4), dim3(256), 0, 0, A, Cm, n); }, T, true);
    add("pipe U8 8/CU", [&] { hipLaunchKernelGGL((k_pipe<8>), dim3(cus * 8), dim3(256), 0, 0, A, Cm, n); }, T, true);
#define LDSDMA(K, NB, AUX, G)                                                                     \
    add("ldsdma K" #K " nb" #NB " aux" #AUX " " #G "/CU", [&] {                                  \
        hipLaunchKernelGGL((k_ldsdma<K, NB, AUX>), dim3(cus * G), dim3(256), 4 * NB * K * 1024, 0, A, Cm, n); \
    }, T, true)
    LDSDMA(8, 2, 0, 2);
    LDSDMA(8, 2, 2, 2);
    LDSDMA(4, 3, 2, 2);
    LDSDMA(8, 2, 2, 1);
#define SEG(L, NTL, NTS)                                                                          \
    add("seg L" #L " ntl" #NTL " nts" #NTS, [&] {                                                 \
        hipLaunchKernelGGL((k_seg<L, NTL, NTS>), dim3(unsigned(n / 1024)), dim3(256), 0, 0, A, Cm); \
    }, T, true)
    SEG(64, 0, 0);
    SEG(128, 0, 0);
    SEG(128, 1, 1);
    SEG(256, 0, 0);
    SEG(256, 1, 1);
    SEG(512, 1, 1);
    SEG(1024, 1, 1);
    SEG(2048, 1, 1);
    SEG(4096, 1, 1);
    SEG(16384, 1, 1);
    SEG(1024, 0, 0);
    SEG(2048, 0, 0);
#define PAT(BF, BS, NT, NTL, NTS)                                                                 \
    add("pat " #BF "x" #BS " t" #NT " ntl" #NTL " nts" #NTS, [&] {                                \
        hipLaunchKernelGGL((k_pat<BF, BS, NT, NTL, NTS>), dim3(unsigned(n * 2 / (BF * BS))), dim3(NT), 0, 0, \
                           (const double*)A, (double*)Cm);                                         \
    }, T, false)
#define PATO(BF, BS, NT, NTL, NTS, O)                                                             \
    add("pat " #BF "x" #BS " t" #NT " ntl" #NTL " nts" #NTS " ord" #O, [&] {                      \
        hipLaunchKernelGGL((k_pat<BF, BS, NT, NTL, NTS, O>), dim3(unsigned(n * 2 / (BF * BS))), dim3(NT), 0, 0, \
                           (const double*)A, (double*)Cm);                                         \
    }, T, false)
    PATO(128, 128, 1024, 1, 1, -12);
    PATO(128, 128, 1024, 1, 1, -14);
    PATO(128, 128, 1024, 1, 1, -18);
    PATO(128, 128, 1024, 1, 1, -22);
    PATO(128, 128, 1024, 1, 1, -24);
    PATO(128, 128, 1024, 1, 1, -28);
    PATO(128, 128, 1024, 0, 0, -1);
    PATO(128, 128, 1024, 1, 1, -1);
    PATO(128, 128, 1024, 0, 0, -2);
    PATO(128, 128, 1024, 1, 1, -2);
    PATO(128, 128, 1024, 1, 1, -3);
    PATO(64, 64, 256, 1, 1, -2);
    PATO(64, 64, 256, 0, 0, -2);
    PATO(128, 64, 512, 1, 1, -2);
    PATO(128, 32, 256, 1, 1, -2);
    PATO(64, 32, 256, 1, 1, -2);
    add("segcamp L1024 nt", [&] {
        hipLaunchKernelGGL((k_seg_camp<1024, 1, 1>), dim3(unsigned(n / 1024)), dim3(256), 0, 0, A, Cm);
    }, T, true);
    add("segcamp L1024 plain", [&] {
        hipLaunchKernelGGL((k_seg_camp<1024, 0, 0>), dim3(unsigned(n / 1024)), dim3(256), 0, 0, A, Cm);
    }, T, true);
    PATO(128, 128, 1024, 0, 0, 2);
    PATO(128, 128, 1024, 0, 0, 4);
    PATO(128, 128, 1024, 0, 0, 8);
    PATO(128, 128, 1024, 0, 0, 16);
    PATO(128, 128, 1024, 1, 1, 4);
    PATO(128, 128, 1024, 1, 1, 8);
    PATO(128, 128, 1024, 1, 1, 16);
    PATO(64, 64, 256, 0, 0, 8);
    PATO(64, 64, 256, 1, 1, 8);
    PATO(128, 64, 512, 1, 1, 8);
    PATO(128, 64, 512, 0, 0, 8);
    PAT(128, 128, 1024, 0, 0);
    PAT(128, 128, 1024, 1, 1);
    PAT(128, 16, 256, 0, 0);
    PAT(128, 16, 256, 1, 1);
    PAT(64, 32, 256, 0, 0);
    PAT(64, 32, 256, 1, 1);
    PAT(128, 32, 256, 1, 1);
    PAT(64, 64, 256, 0, 0);
    PAT(64, 64, 256, 1, 1);
    PAT(128, 64, 512, 1, 1);
#define NARROW(W, NTL, NTS)                                                                       \
    add("narrow W" #W " ntl" #NTL " nts" #NTS, [&] {                                              \
        hipLaunchKernelGGL((k_narrow<W, NTL, NTS>), dim3(unsigned(bytes1 / 16384)), dim3(256), 0, 0, \
                           (const unsigned char*)A, (unsigned char*)Cm);                           \
    }, T, true)
    NARROW(4, 0, 0);
    NARROW(4, 1, 1);
    NARROW(8, 0, 0);
    NARROW(8, 1, 1);
    NARROW(16, 0, 0);
    NARROW(16, 1, 1);
    add("hipMemcpyDtoD", [&] { CK(hipMemcpyAsync(Cm, A, bytes1, hipMemcpyDeviceToDevice, 0)); }, T, true);
    // reads and writes alone (4 GiB of traffic each, like the copy)
    add("read U8 ld0 8/CU x2", [&] {
        hipLaunchKernelGGL((k_read<8, 0>), dim3(cus * 8), dim3(256), 0, 0, A, n, sink);
        hipLaunchKernelGGL((k_read<8, 0>), dim3(cus * 8), dim3(256), 0, 0, Cm, n, sink);
    }, T, false);
    add("read U8 nt 8/CU x2", [&] {
        hipLaunchKernelGGL((k_read<8, 2>), dim3(cus * 8), dim3(256), 0, 0, A, n, sink);
        hipLaunchKernelGGL((k_read<8, 2>), dim3(cus * 8), dim3(256), 0, 0, Cm, n, sink);
    }, T, false);
    add("read ldsdma K16 nt 2/CU x2", [&] {
        hipLaunchKernelGGL((k_read_lds<16, 2>), dim3(cus * 2), dim3(256), 4 * 16 * 1024, 0, A, n, sink);
        hipLaunchKernelGGL((k_read_lds<16, 2>), dim3(cus * 2), dim3(256), 4 * 16 * 1024, 0, Cm, n, sink);
    }, T, false);
    add("read ldsdma K16 ld0 2/CU x2", [&] {
        hipLaunchKernelGGL((k_read_lds<16, 0>), dim3(cus * 2), dim3(256), 4 * 16 * 1024, 0, A, n, sink);
        hipLaunchKernelGGL((k_read_lds<16, 0>), dim3(cus * 2), dim3(256), 4 * 16 * 1024, 0, Cm, n, sink);
    }, T, false);
    add("write U8 st0 8/CU x2", [&] {
        hipLaunchKernelGGL((k_write<8, 0>), dim3(cus * 8), dim3(256), 0, 0, Cm, n);
        hipLaunchKernelGGL((k_write<8, 0>), dim3(cus * 8), dim3(256), 0, 0, Cm, n);
    }, T, false);
    add("write U8 nt 8/CU x2", [&] {
        hipLaunchKernelGGL((k_write<8, 2>), dim3(cus * 8), dim3(256), 0, 0, Cm, n);
        hipLaunchKernelGGL((k_write<8, 2>), dim3(cus * 8), dim3(256), 0, 0, Cm, n);
    }, T, false);
    add("write U8 sc1 8/CU x2", [&] {
        hipLaunchKernelGGL((k_write<8, 16>), dim3(cus * 8), dim3(256), 0, 0, Cm, n);
        hipLaunchKernelGGL((k_write<8, 16>), dim3(cus * 8), dim3(256), 0, 0, Cm, n);
    }, T, false);
    // smaller footprints of the best-known plain copy (the 256 MiB Infinity Cache)
    for (long mb : {64L, 256L, 1024L}) {
        const long nn = (mb << 20) / 16;
        add("stride U8 8/CU " + std::to_string(mb) + "MiB", [&, nn] {
            hipLaunchKernelGGL((k_stride<8, 0, 0>), dim3(cus * 8), dim3(256), 0, 0, A, Cm, nn);
        }, 2.0 * nn * 16, false);
    }

    for (auto& v : V) {  // warm + verify
        CK(hipMemset(Cm, 0, bytes1));
        v.run();
        CK(hipDeviceSynchronize());
        if (v.verify) {
            CK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(check, dim3(8192), dim3(256), 0, 0, A, Cm, n, bad);
            unsigned long long h = 0;
            CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
            printf("%-34s verify: %s\n", v.name.c_str(), h ? "FAIL" : "ok");
        }
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int r = 0; r < reps; ++r)
        for (auto& v : V) {
            CK(hipEventRecord(e0, 0));
            v.run();
            CK(hipEventRecord(e1, 0));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            v.ms.push_back(ms);
        }
    printf("%-34s %9s %9s %9s %7s\n", "variant", "min ms", "med ms", "GB/s med", "%8TB/s");
    for (auto& v : V) {
        std::sort(v.ms.begin(), v.ms.end());
        const float med = v.ms[v.ms.size() / 2];
        printf("%-34s %9.4f %9.4f %9.1f %7.2f\n", v.name.c_str(), v.ms[0], med, v.traffic / med / 1e6,
               v.traffic / med / 1e6 / 80.0);
    }
    return 0;
}
