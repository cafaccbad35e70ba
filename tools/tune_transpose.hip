// Tuning harness (not part of the product): structural variants of the fp64 tile transpose
// on BASELINE cfg 2 geometry (16384^2, 4096 tiles of 256^2, ld 16384), timed interleaved in
// one process with hipEvents.  Each variant is verified against C == A^T.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/tune_transpose.hip -o /tmp/tune && /tmp/tune
#include <hip/hip_runtime.h>

#include <algorithm>
#include <functional>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e = (x);                                                             \
        if (e != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                    \
        }                                                                               \
    } while (0)

struct op_t {
    uint64_t src, dst;
    int nf, ns, lds, ldd;
    uint32_t flags, pad;
};

typedef double d2 __attribute__((ext_vector_type(2)));

// ----------------------------------------------------------------------------------
// V0: one 64x64 sub-tile per WG, 256 threads, padded LDS, 8-B row stores (product r01)
template <int BS, int NTS>
__global__ __launch_bounds__(256) void v_basic(const op_t* ops, const uint64_t* work) {
    constexpr int BF = 64, P = BF + 1;
    __shared__ double tile[BS * P];
    const uint64_t w = work[blockIdx.x];
    const op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = op.nf / BF;
    const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
    const double* src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
    double* dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
    const int lf = (threadIdx.x % 32) * 2, c0 = threadIdx.x / 32;
    d2 x[BS / 8];
#pragma unroll
    for (int k = 0; k < BS / 8; ++k)
        x[k] = *reinterpret_cast<const d2*>(src + int64_t(c0 + 8 * k) * op.lds + lf);
#pragma unroll
    for (int k = 0; k < BS / 8; ++k) {
        tile[(c0 + 8 * k) * P + lf] = x[k].x;
        tile[(c0 + 8 * k) * P + lf + 1] = x[k].y;
    }
    __syncthreads();
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    if (NTS) {
#pragma unroll
        for (int j = 0; j < BS / 64; ++j)
#pragma unroll
            for (int f = wave; f < BF; f += 4)
                __builtin_nontemporal_store(tile[(lane + 64 * j) * P + f],
                                            dst + int64_t(f) * op.ldd + lane + 64 * j);
    } else {
        for (int j = 0; j < BS / 64; ++j)
            for (int f = wave; f < BF; f += 4)
                dst[int64_t(f) * op.ldd + lane + 64 * j] = tile[(lane + 64 * j) * P + f];
    }
}

// ----------------------------------------------------------------------------------
// V1: unrolled store phase with 16-B stores via a 2x2 lane-pair exchange.
// LDS rows are s, pitch 66 doubles (conflict-free b128 reads and writes); a lane reads
// slot (s, f..f+1) and swaps with its xor-1 neighbour so it holds (s, f),(s+1, f) [even
// lane] or (s, f+1),(s+1, f+1) [odd lane] -> one 16-B store each.
template <int BS, int NTS, int NTL>
__global__ __launch_bounds__(256) void v_pair(const op_t* ops, const uint64_t* work) {
    constexpr int BF = 64, P = BF + 2;
    __shared__ __attribute__((aligned(16))) double tile[BS * P];
    const uint64_t w = work[blockIdx.x];
    const op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = op.nf / BF;
    const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
    const double* src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
    double* dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
    const int lf = (threadIdx.x % 32) * 2, c0 = threadIdx.x / 32;
    d2 x[BS / 8];
#pragma unroll
    for (int k = 0; k < BS / 8; ++k) {
        const d2* p = reinterpret_cast<const d2*>(src + int64_t(c0 + 8 * k) * op.lds + lf);
        x[k] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int k = 0; k < BS / 8; ++k) *reinterpret_cast<d2*>(&tile[(c0 + 8 * k) * P + lf]) = x[k];
    __syncthreads();
    // store phase: a wave covers rows f, f+1 (BS s-values each): lane -> s = lane (for 64)
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    const bool odd = lane & 1;
    constexpr int SW = BS / 64;  // s-chunks of 64
    d2 y[BF / 8 * SW];
#pragma unroll
    for (int j = 0; j < SW; ++j)
#pragma unroll
        for (int q = 0; q < BF / 8; ++q) {  // slot pairs: rows f = 2*(wave + 4q)
            const int f = 2 * (wave + 4 * q);
            y[j * (BF / 8) + q] = *reinterpret_cast<const d2*>(&tile[(lane + 64 * j) * P + f]);
        }
#pragma unroll
    for (int j = 0; j < SW; ++j)
#pragma unroll
        for (int q = 0; q < BF / 8; ++q) {
            d2 v = y[j * (BF / 8) + q];
            // even lane keeps (s,f) and takes neighbour's (s+1,f); odd keeps (s+1,f+1)...
            double give = odd ? v.x : v.y;
            double got = __shfl_xor(give, 1);
            d2 o;
            if (!odd) { o.x = v.x; o.y = got; }   // (s, f), (s+1, f)
            else      { o.x = got; o.y = v.y; }   // (s-1, f+1), (s, f+1)
            const int f = 2 * (wave + 4 * q) + (odd ? 1 : 0);
            const int s = (lane & ~1) + 64 * j;
            d2* p = reinterpret_cast<d2*>(dst + int64_t(f) * op.ldd + s);
            if (NTS) __builtin_nontemporal_store(o, p); else *p = o;
        }
}

// ----------------------------------------------------------------------------------
// V2: persistent WGs with software pipelining: the next sub-tile's loads are in flight
// while the current one is stored.
template <int BS>
__global__ __launch_bounds__(256) void v_persist(const op_t* ops, const uint64_t* work, int64_t n) {
    constexpr int BF = 64, P = BF + 2;
    __shared__ __attribute__((aligned(16))) double tile[BS * P];
    const int lf = (threadIdx.x % 32) * 2, c0 = threadIdx.x / 32;
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    const bool odd = lane & 1;
    int64_t i = blockIdx.x;
    if (i >= n) return;
    auto geo = [&](int64_t wi, const double*& src, double*& dst, int& ldd) {
        const uint64_t w = work[wi];
        const op_t op = ops[w >> 32];
        const uint32_t sub = uint32_t(w);
        const int nbf = op.nf / BF;
        const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
        src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
        dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
        ldd = op.ldd;
        return op.lds;
    };
    const double* src;
    double* dst;
    int ldd;
    int lds = geo(i, src, dst, ldd);
    d2 x[BS / 8];
#pragma unroll
    for (int k = 0; k < BS / 8; ++k)
        x[k] = *reinterpret_cast<const d2*>(src + int64_t(c0 + 8 * k) * lds + lf);
    while (true) {
#pragma unroll
        for (int k = 0; k < BS / 8; ++k) *reinterpret_cast<d2*>(&tile[(c0 + 8 * k) * P + lf]) = x[k];
        __syncthreads();
        double* cdst = dst;
        const int cldd = ldd;
        const int64_t nxt = i + gridDim.x;
        if (nxt < n) {
            lds = geo(nxt, src, dst, ldd);
#pragma unroll
            for (int k = 0; k < BS / 8; ++k)
                x[k] = *reinterpret_cast<const d2*>(src + int64_t(c0 + 8 * k) * lds + lf);
        }
        constexpr int SW = BS / 64;
        d2 y[BF / 8 * SW];
#pragma unroll
        for (int j = 0; j < SW; ++j)
#pragma unroll
            for (int q = 0; q < BF / 8; ++q)
                y[j * (BF / 8) + q] =
                    *reinterpret_cast<const d2*>(&tile[(lane + 64 * j) * P + 2 * (wave + 4 * q)]);
        __syncthreads();  // tile free for the next iteration's writes
#pragma unroll
        for (int j = 0; j < SW; ++j)
#pragma unroll
            for (int q = 0; q < BF / 8; ++q) {
                d2 v = y[j * (BF / 8) + q];
                double got = __shfl_xor(odd ? v.x : v.y, 1);
                d2 o;
                if (!odd) { o.x = v.x; o.y = got; } else { o.x = got; o.y = v.y; }
                const int f = 2 * (wave + 4 * q) + (odd ? 1 : 0);
                const int s = (lane & ~1) + 64 * j;
                *reinterpret_cast<d2*>(cdst + int64_t(f) * cldd + s) = o;
            }
        if (nxt >= n) break;
        i = nxt;
    }
}

// ----------------------------------------------------------------------------------
// V3: generic BF x BS tile, NT threads, pair-exchange 16-B stores, optional nt loads.
// Load: LPC = BF/2 lanes per column; store: 32 lane-pairs cover 64 s per row pair.
template <int BF, int BS, int NT, int NTL, int NTS = 0>
__global__ __launch_bounds__(NT) void v_gen(const op_t* ops, const uint64_t* work) {
    constexpr int P = BF + 2;
    __shared__ __attribute__((aligned(16))) double tile[BS * P];
    const uint64_t w = work[blockIdx.x];
    const op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = op.nf / BF;
    const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
    const double* src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
    double* dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
    constexpr int LPC = BF / 2, CPP = NT / LPC, PL = BS / CPP;
    const int lf = (threadIdx.x % LPC) * 2, c0 = threadIdx.x / LPC;
    d2 x[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
        const d2* p = reinterpret_cast<const d2*>(src + int64_t(c0 + CPP * k) * op.lds + lf);
        x[k] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int k = 0; k < PL; ++k) *reinterpret_cast<d2*>(&tile[(c0 + CPP * k) * P + lf]) = x[k];
    __syncthreads();
    // store: a wave = 64 lanes = 64 s values x one row pair (f, f+1); NT/64 waves
    constexpr int NW = NT / 64, SC = BS / 64, RP = BF / 2;  // row pairs
    constexpr int PS = SC * RP / NW;
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    const bool odd = lane & 1;
    d2 y[PS];
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int t = wave + NW * k, j = t / RP, rp = t % RP;
        y[k] = *reinterpret_cast<const d2*>(&tile[(lane + 64 * j) * P + 2 * rp]);
    }
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int t = wave + NW * k, j = t / RP, rp = t % RP;
        d2 v = y[k];
        double got = __shfl_xor(odd ? v.x : v.y, 1);
        d2 o;
        if (!odd) { o.x = v.x; o.y = got; } else { o.x = got; o.y = v.y; }
        d2* q = reinterpret_cast<d2*>(dst + int64_t(2 * rp + (odd ? 1 : 0)) * op.ldd + (lane & ~1) + 64 * j);
        if (NTS) __builtin_nontemporal_store(o, q); else *q = o;
    }
}

// ----------------------------------------------------------------------------------
// V5: 128x128 / 1024 threads, row stores: one wave instruction writes a whole 1 KiB row
// segment (128 s values of one f): lane l holds (2l, f), (2l+1, f) from two 8-byte LDS reads.
// PAD selects the LDS row pitch in doubles (BF + PAD).
template <int PAD, int NTL>
__global__ __launch_bounds__(1024) void v_rowstore(const op_t* ops, const uint64_t* work) {
    constexpr int BF = 128, BS = 128, NT = 1024, P = BF + PAD;
    __shared__ __attribute__((aligned(16))) double tile[BS * P];
    const uint64_t w = work[blockIdx.x];
    const op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = op.nf / BF;
    const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
    const double* src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
    double* dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
    constexpr int LPC = BF / 2, CPP = NT / LPC, PL = BS / CPP;
    const int lf = (threadIdx.x % LPC) * 2, c0 = threadIdx.x / LPC;
    d2 x[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
        const d2* p = reinterpret_cast<const d2*>(src + int64_t(c0 + CPP * k) * op.lds + lf);
        x[k] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int k = 0; k < PL; ++k) {
        if (PAD % 2 == 0) {
            *reinterpret_cast<d2*>(&tile[(c0 + CPP * k) * P + lf]) = x[k];
        } else {
            tile[(c0 + CPP * k) * P + lf] = x[k].x;
            tile[(c0 + CPP * k) * P + lf + 1] = x[k].y;
        }
    }
    __syncthreads();
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    constexpr int PS = BF / (NT / 64);  // rows per wave
    d2 y[PS];
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int f = wave + 16 * k;
        y[k].x = tile[(2 * lane) * P + f];
        y[k].y = tile[(2 * lane + 1) * P + f];
    }
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int f = wave + 16 * k;
        *reinterpret_cast<d2*>(dst + int64_t(f) * op.ldd + 2 * lane) = y[k];
    }
}

// ----------------------------------------------------------------------------------
// V4: v_gen as a persistent loop: the next sub-tile's loads are issued before the current
// sub-tile's LDS read-out and stores (register double buffering).
template <int BF, int BS, int NT, int NTL = 0, int NTS = 0>
__global__ __launch_bounds__(NT) void v_gen_persist(const op_t* ops, const uint64_t* work,
                                                    int64_t n) {
    constexpr int P = BF + 2;
    __shared__ __attribute__((aligned(16))) double tile[BS * P];
    constexpr int LPC = BF / 2, CPP = NT / LPC, PL = BS / CPP;
    constexpr int NW = NT / 64, SC = BS / 64, RP = BF / 2, PS = SC * RP / NW;
    const int lf = (threadIdx.x % LPC) * 2, c0 = threadIdx.x / LPC;
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    const bool odd = lane & 1;
    int64_t i = blockIdx.x;
    if (i >= n) return;
    const double* src;
    double* dst;
    int lds, ldd;
    auto geo = [&](int64_t wi) {
        const uint64_t w = work[wi];
        const op_t op = ops[w >> 32];
        const uint32_t sub = uint32_t(w);
        const int nbf = op.nf / BF;
        const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
        src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
        dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
        lds = op.lds;
        ldd = op.ldd;
    };
    geo(i);
    d2 x[PL];
    auto ld = [&](int k) {
        const d2* p = reinterpret_cast<const d2*>(src + int64_t(c0 + CPP * k) * lds + lf);
        return NTL ? __builtin_nontemporal_load(p) : *p;
    };
#pragma unroll
    for (int k = 0; k < PL; ++k) x[k] = ld(k);
    while (true) {
#pragma unroll
        for (int k = 0; k < PL; ++k) *reinterpret_cast<d2*>(&tile[(c0 + CPP * k) * P + lf]) = x[k];
        __syncthreads();
        double* cdst = dst;
        const int cldd = ldd;
        const int64_t nxt = i + gridDim.x;
        if (nxt < n) {
            geo(nxt);
#pragma unroll
            for (int k = 0; k < PL; ++k) x[k] = ld(k);
        }
        d2 y[PS];
#pragma unroll
        for (int k = 0; k < PS; ++k) {
            const int t = wave + NW * k, j = t / RP, rp = t % RP;
            y[k] = *reinterpret_cast<const d2*>(&tile[(lane + 64 * j) * P + 2 * rp]);
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < PS; ++k) {
            const int t = wave + NW * k, j = t / RP, rp = t % RP;
            d2 v = y[k];
            double got = __shfl_xor(odd ? v.x : v.y, 1);
            d2 o;
            if (!odd) { o.x = v.x; o.y = got; } else { o.x = got; o.y = v.y; }
            d2* q = reinterpret_cast<d2*>(cdst + int64_t(2 * rp + (odd ? 1 : 0)) * cldd + (lane & ~1) + 64 * j);
            if (NTS) __builtin_nontemporal_store(o, q); else *q = o;
        }
        if (nxt >= n) break;
        i = nxt;
    }
}


// ----------------------------------------------------------------------------------
// V7: copy-shaped transpose: 128 (f) x 32 (s) fp64 per 256-thread WG (32 KiB, like the best
// flat copy's one 32 KiB chunk per WG); 4 WGs per CU interleave load and store phases.
// Store: half-waves of 32 lanes cover the 32 s values of one row pair (pair exchange).
template <int NTL>
__global__ __launch_bounds__(256) void v_copyshape(const op_t* ops, const uint64_t* work) {
    constexpr int BF = 128, BS = 32, NT = 256, P = BF + 2;
    __shared__ __attribute__((aligned(16))) double tile[BS * P];
    const uint64_t w = work[blockIdx.x];
    const op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = op.nf / BF;
    const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
    const double* src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
    double* dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
    constexpr int LPC = BF / 2, CPP = NT / LPC, PL = BS / CPP;  // 64 lanes/col, 4 cols, 8 passes
    const int lf = (threadIdx.x % LPC) * 2, c0 = threadIdx.x / LPC;
    d2 x[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
        const d2* p = reinterpret_cast<const d2*>(src + int64_t(c0 + CPP * k) * op.lds + lf);
        x[k] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int k = 0; k < PL; ++k) *reinterpret_cast<d2*>(&tile[(c0 + CPP * k) * P + lf]) = x[k];
    __syncthreads();
    // 64 row pairs; a wave does 2 per pass (one per half), 4 waves -> 8 passes
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    const int half = lane / 32, sl = lane % 32;
    const bool odd = sl & 1;
    constexpr int PS = (BF / 2) / (2 * (NT / 64));
    d2 y[PS];
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int rp = 2 * (wave + 4 * k) + half;
        y[k] = *reinterpret_cast<const d2*>(&tile[sl * P + 2 * rp]);
    }
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int rp = 2 * (wave + 4 * k) + half;
        d2 v = y[k];
        double got = __shfl_xor(odd ? v.x : v.y, 1);
        d2 o;
        if (!odd) { o.x = v.x; o.y = got; } else { o.x = got; o.y = v.y; }
        *reinterpret_cast<d2*>(dst + int64_t(2 * rp + (odd ? 1 : 0)) * op.ldd + (sl & ~1)) = o;
    }
}

// ----------------------------------------------------------------------------------
// V6: persistent, double-buffered LDS filled by global_load_lds_dwordx4: a 128 (f) x 64 (s)
// fp64 sub-tile per buffer, one 1 KiB source column per wave instruction into one padded LDS
// row; the next sub-tile's loads are in flight while the current one is stored.
template <int NTL>
__global__ __launch_bounds__(512) void v_glds(const op_t* ops, const uint64_t* work, int64_t n) {
    constexpr int BF = 128, BS = 64, NT = 512, P = BF + 2;
    extern __shared__ __attribute__((aligned(16))) double lds_buf[];  // 2 x BS x P
    const int lane = threadIdx.x % 64;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / 64);
    constexpr int NW = NT / 64, CPW = BS / NW;  // columns per wave per tile
    auto geo = [&](int64_t wi, const double*& src, double*& dst, int& ld_s, int& ld_d) {
        const uint64_t w = work[wi];
        const op_t op = ops[w >> 32];
        const uint32_t sub = uint32_t(w);
        const int nbf = op.nf / BF;
        const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
        src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
        dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
        ld_s = op.lds;
        ld_d = op.ldd;
    };
    auto issue = [&](const double* src, int ld_s, int b) {
#pragma unroll
        for (int k = 0; k < CPW; ++k) {
            const int c = wave + NW * k;
            const double* g = src + int64_t(c) * ld_s + 2 * lane;
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void*)(g),
                (__attribute__((address_space(3))) void*)(&lds_buf[(b * BS + c) * P]), 16, 0,
                NTL ? 2 : 0);
        }
    };
    int64_t i = blockIdx.x;
    if (i >= n) return;
    const double* src;
    double* dst;
    int ls, ld;
    geo(i, src, dst, ls, ld);
    issue(src, ls, 0);
    int b = 0;
    constexpr int RP = BF / 2, PS = RP / NW;  // row pairs per wave (BS = 64 = one wave of s)
    const bool odd = lane & 1;
    while (true) {
        const int64_t nxt = i + gridDim.x;
        double* cdst = dst;
        const int cld = ld;
        __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) expcnt(0) lgkmcnt(0): own DMA + stores done
        __syncthreads();
        if (nxt < n) {
            geo(nxt, src, dst, ls, ld);
            issue(src, ls, b ^ 1);
        }
        const double* t = &lds_buf[b * BS * P];
        d2 y[PS];
#pragma unroll
        for (int k = 0; k < PS; ++k) {
            const int rp = wave + NW * k;
            y[k] = *reinterpret_cast<const d2*>(&t[lane * P + 2 * rp]);
        }
#pragma unroll
        for (int k = 0; k < PS; ++k) {
            const int rp = wave + NW * k;
            d2 v = y[k];
            double got = __shfl_xor(odd ? v.x : v.y, 1);
            d2 o;
            if (!odd) { o.x = v.x; o.y = got; } else { o.x = got; o.y = v.y; }
            *reinterpret_cast<d2*>(cdst + int64_t(2 * rp + (odd ? 1 : 0)) * cld + (lane & ~1)) = o;
        }
        if (nxt >= n) break;
        i = nxt;
        b ^= 1;
    }
}

// V8: persistent LDS-DMA ring.  One workgroup per CU walks sub-tiles i = blockIdx.x + k*grid;
// each source column of a BF x BS sub-tile (BF = 128 fp64 = 1 KiB) arrives by one
// global_load_lds_dwordx4 wave instruction straight into an LDS row (pitch BF + 2); NB buffers,
// NB - 1 sub-tiles of loads in flight.  The wait before reading sub-tile i counts only the loads
// of sub-tile i: the stores of earlier sub-tiles and the loads of later ones stay in flight
// (vmcnt counts in issue order).  Store: lane pairs swap halves so every lane writes 16 B
// along s (BS s-values per row pair, 64 / BS row pairs per instruction).
template <int BS, int NT, int NB, int NTL, int NTS = 0>
__global__ __launch_bounds__(NT) void v_ring(const op_t* ops, const uint64_t* work, int64_t n) {
    constexpr int BF = 128, P = BF + 2;
    constexpr int NW = NT / 64;
    constexpr int CPW = BS / NW;             // load instructions (columns) per wave per sub-tile
    constexpr int RPI = 64 / BS;             // row pairs per store instruction
    constexpr int SI = (BF / 2) / RPI;       // store instructions per sub-tile
    constexpr int PS = SI / NW;              // per wave
    static_assert(BS % NW == 0 && SI % NW == 0 && CPW >= 1 && PS >= 1, "mapping");
    constexpr int WAIT = (NB - 1) * PS + (NB - 2) * CPW;  // vmcnt allowed while sub-tile i lands
    static_assert(WAIT < 64, "vmcnt range");
    extern __shared__ __attribute__((aligned(16))) double lds_buf[];  // NB x BS x P
    const int lane = threadIdx.x % 64;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / 64);
    auto geo = [&](int64_t wi, const double*& src, double*& dst, int& ld_s, int& ld_d) {
        const uint64_t w = work[wi];
        const op_t op = ops[w >> 32];
        const uint32_t sub = uint32_t(w);
        const int nbf = op.nf / BF;
        const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
        src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
        dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
        ld_s = op.lds;
        ld_d = op.ldd;
    };
    auto issue = [&](int64_t wi, int b) {
        const double* src;
        double* dst;
        int ls, ld;
        geo(wi, src, dst, ls, ld);
#pragma unroll
        for (int k = 0; k < CPW; ++k) {
            const int c = wave + NW * k;
            __builtin_amdgcn_global_load_lds(
                (__attribute__((address_space(1))) void*)(src + int64_t(c) * ls + 2 * lane),
                (__attribute__((address_space(3))) void*)(&lds_buf[(b * BS + c) * P]), 16, 0,
                NTL ? 2 : 0);
        }
    };
    const int64_t G = gridDim.x;
    int64_t i = blockIdx.x;
    if (i >= n) return;
    // prologue: NB - 1 sub-tiles in flight
#pragma unroll
    for (int q = 0; q < NB - 1; ++q)
        if (i + q * G < n) issue(i + q * G, q);
    int b = 0;
    const bool odd = lane & 1;
    const int sl = lane % BS, rq = lane / BS;  // s of this lane, row pair within the instruction
    for (int64_t it = 0;; ++it) {
        const int64_t cur = i + it * G;
        if (cur >= n) break;
        // loads of sub-tile `cur` done; later loads and earlier stores may stay in flight.
        // Near the end fewer later loads exist: wait for everything then.
        // (the first NB - 1 sub-tiles have fewer stores behind them: wait for everything)
        if (it >= NB - 1 && cur + (NB - 2) * G < n)
            __builtin_amdgcn_s_waitcnt((WAIT & 0xF) | ((WAIT >> 4) << 14) | (0x7 << 4) | (0xF << 8));
        else
            __builtin_amdgcn_s_waitcnt(0);
        __syncthreads();  // every wave's DMA into this buffer landed; the oldest buffer is free
        const int64_t nxt = cur + (NB - 1) * G;
        if (nxt < n) issue(nxt, (b + NB - 1) % NB);
        const double* src;
        double* cdst;
        int ls, cld;
        geo(cur, src, cdst, ls, cld);
        const double* t = &lds_buf[b * BS * P];
        d2 y[PS];
#pragma unroll
        for (int k = 0; k < PS; ++k) {
            const int rp = (wave + NW * k) * RPI + rq;
            y[k] = *reinterpret_cast<const d2*>(&t[sl * P + 2 * rp]);
        }
#pragma unroll
        for (int k = 0; k < PS; ++k) {
            const int rp = (wave + NW * k) * RPI + rq;
            d2 v = y[k];
            double got = __shfl_xor(odd ? v.x : v.y, 1);
            d2 o;
            if (!odd) { o.x = v.x; o.y = got; } else { o.x = got; o.y = v.y; }
            d2* q = reinterpret_cast<d2*>(cdst + int64_t(2 * rp + (odd ? 1 : 0)) * cld + (sl & ~1));
            if (NTS) __builtin_nontemporal_store(o, q); else *q = o;
        }
        b = (b + 1) % NB;
    }
}

// ----------------------------------------------------------------------------------
// V9: generic BF (f) x BS (s) sub-tile per NT-thread WG, BS <= 64: one store instruction covers
// 64 / BS row pairs of BS s-values (pair exchange), optional nt loads / stores.  Small tiles
// (16-32 KiB) keep up to 8 WGs per CU resident, so load and store phases of different WGs overlap
// on every CU (the flat copy's best shape: 16 KiB per 256-thread WG, nt both ways).
template <int BF, int BS, int NT, int NTL, int NTS>
__global__ __launch_bounds__(NT) void v_tr(const op_t* ops, const uint64_t* work) {
    constexpr int P = BF + 2;
    __shared__ __attribute__((aligned(16))) double tile[BS * P];
    const uint64_t w = work[blockIdx.x];
    const op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = op.nf / BF;
    const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
    const double* src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
    double* dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
    constexpr int LPC = BF / 2, CPP = NT / LPC, PL = BS / CPP;
    static_assert(NT % LPC == 0 && BS % CPP == 0 && BS <= 64, "mapping");
    const int lf = (threadIdx.x % LPC) * 2, c0 = threadIdx.x / LPC;
    d2 x[PL];
#pragma unroll
    for (int k = 0; k < PL; ++k) {
        const d2* p = reinterpret_cast<const d2*>(src + int64_t(c0 + CPP * k) * op.lds + lf);
        x[k] = NTL ? __builtin_nontemporal_load(p) : *p;
    }
#pragma unroll
    for (int k = 0; k < PL; ++k) *reinterpret_cast<d2*>(&tile[(c0 + CPP * k) * P + lf]) = x[k];
    __syncthreads();
    constexpr int NW = NT / 64, RPI = 64 / BS, SI = (BF / 2) / RPI, PS = SI / NW;
    static_assert(SI % NW == 0 && PS >= 1, "store mapping");
    const int lane = threadIdx.x % 64, wave = threadIdx.x / 64;
    const bool odd = lane & 1;
    const int sl = lane % BS, rq = lane / BS;
    d2 y[PS];
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int rp = (wave + NW * k) * RPI + rq;
        y[k] = *reinterpret_cast<const d2*>(&tile[sl * P + 2 * rp]);
    }
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int rp = (wave + NW * k) * RPI + rq;
        d2 v = y[k];
        double got = __shfl_xor(odd ? v.x : v.y, 1);
        d2 o;
        if (!odd) { o.x = v.x; o.y = got; } else { o.x = got; o.y = v.y; }
        d2* q = reinterpret_cast<d2*>(dst + int64_t(2 * rp + (odd ? 1 : 0)) * op.ldd + (sl & ~1));
        if (NTS) __builtin_nontemporal_store(o, q); else *q = o;
    }
}

// ----------------------------------------------------------------------------------
// V10: v_gen 128x128 / 1024 threads with the loads done by LDS-DMA (global_load_lds_dwordx4):
// every source column (1 KiB) lands in one padded LDS row without passing through VGPRs and
// without ds_write (the most expensive LDS instruction of the VGPR-staged form).
template <int AUX, int NTS>
__global__ __launch_bounds__(1024) void v_glds1(const op_t* ops, const uint64_t* work) {
    constexpr int BF = 128, BS = 128, NT = 1024, P = BF + 2;
    extern __shared__ __attribute__((aligned(16))) double tile[];
    const uint64_t w = work[blockIdx.x];
    const op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = op.nf / BF;
    const int f0 = int(sub % nbf) * BF, s0 = int(sub / nbf) * BS;
    const double* src = reinterpret_cast<const double*>(op.src) + int64_t(s0) * op.lds + f0;
    double* dst = reinterpret_cast<double*>(op.dst) + int64_t(f0) * op.ldd + s0;
    const int lane = threadIdx.x % 64;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / 64);
    constexpr int NW = NT / 64;
#pragma unroll
    for (int k = 0; k < BS / NW; ++k) {
        const int c = wave + NW * k;
        __builtin_amdgcn_global_load_lds(
            (__attribute__((address_space(1))) void*)(src + int64_t(c) * op.lds + 2 * lane),
            (__attribute__((address_space(3))) void*)(&tile[c * P]), 16, 0, AUX);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    constexpr int SC = BS / 64, RP = BF / 2, PS = SC * RP / NW;
    const bool odd = lane & 1;
    d2 y[PS];
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int t = wave + NW * k, j = t / RP, rp = t % RP;
        y[k] = *reinterpret_cast<const d2*>(&tile[(lane + 64 * j) * P + 2 * rp]);
    }
#pragma unroll
    for (int k = 0; k < PS; ++k) {
        const int t = wave + NW * k, j = t / RP, rp = t % RP;
        d2 v = y[k];
        double got = __shfl_xor(odd ? v.x : v.y, 1);
        d2 o;
        if (!odd) { o.x = v.x; o.y = got; } else { o.x = got; o.y = v.y; }
        d2* q = reinterpret_cast<d2*>(dst + int64_t(2 * rp + (odd ? 1 : 0)) * op.ldd + (lane & ~1) + 64 * j);
        if (NTS) __builtin_nontemporal_store(o, q); else *q = o;
    }
}

// ----------------------------------------------------------------------------------
// ceiling: flat 16-B copy of the same bytes (grid-stride)
__global__ __launch_bounds__(256) void v_copy(const d2* a, d2* c, int64_t n) {
    for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256)
        c[i] = a[i];
}

// ceiling probes: each WG moves U*256 contiguous 16-B chunks per iteration, loads first
template <int U, int NTL, int NTS>
__global__ __launch_bounds__(256) void v_copy_ilp(const d2* a, d2* c, int64_t n) {
    const int64_t per = int64_t(U) * 256;
    for (int64_t base = blockIdx.x * per; base < n; base += int64_t(gridDim.x) * per) {
        d2 x[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const d2* p = a + base + u * 256 + threadIdx.x;
            x[u] = NTL ? __builtin_nontemporal_load(p) : *p;
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            d2* p = c + base + u * 256 + threadIdx.x;
            if (NTS) __builtin_nontemporal_store(x[u], p); else *p = x[u];
        }
    }
}
template <int U>
__global__ __launch_bounds__(256) void v_read(const d2* a, int64_t n, d2* sink) {
    d2 acc = {0, 0};
    const int64_t per = int64_t(U) * 256;
    for (int64_t base = blockIdx.x * per; base < n; base += int64_t(gridDim.x) * per) {
#pragma unroll
        for (int u = 0; u < U; ++u) acc += a[base + u * 256 + threadIdx.x];
    }
    if (acc.x == 12345.678) sink[threadIdx.x] = acc;
}
template <int U>
__global__ __launch_bounds__(256) void v_write(d2* c, int64_t n) {
    const int64_t per = int64_t(U) * 256;
    d2 v = {1.0, 2.0};
    for (int64_t base = blockIdx.x * per; base < n; base += int64_t(gridDim.x) * per) {
#pragma unroll
        for (int u = 0; u < U; ++u) c[base + u * 256 + threadIdx.x] = v;
    }
}

__global__ void fill(double* a, int64_t n) {
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
         i += int64_t(gridDim.x) * blockDim.x)
        a[i] = double(i % 1000003) * 0.5 + double(i / 1000003);
}

__global__ void check(const double* a, const double* c, int n, unsigned long long* bad) {
    int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x;
    if (k >= int64_t(n) * n) return;
    int i = int(k % n), j = int(k / n);  // C(i, j) at i + j*n must be A(j, i) at j + i*n
    if (c[k] != a[j + int64_t(i) * n]) atomicAdd(bad, 1ull);
}

int main(int argc, char** argv) {
    const int n = 16384, b = 256;
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    double *A, *Cm;
    CK(hipMalloc(&A, sizeof(double) * n * n));
    CK(hipMalloc(&Cm, sizeof(double) * n * n));
    hipLaunchKernelGGL(fill, dim3(4096), dim3(256), 0, 0, A, int64_t(n) * n);
    std::vector<op_t> ops;
    for (int j = 0; j < n / b; ++j)
        for (int i = 0; i < n / b; ++i) {
            op_t o{};
            o.src = uint64_t(A + i * b + int64_t(j) * b * n);
            o.dst = uint64_t(Cm + j * b + int64_t(i) * b * n);
            o.nf = o.ns = b;
            o.lds = o.ldd = n;
            ops.push_back(o);
        }
    op_t* d_ops;
    CK(hipMalloc(&d_ops, ops.size() * sizeof(op_t)));
    CK(hipMemcpy(d_ops, ops.data(), ops.size() * sizeof(op_t), hipMemcpyHostToDevice));
    // tord: ops in the order of the product's locality hint (target column-major: consecutive
    // ops continue down the same C columns); otherwise source column-major (ops[] order)
    auto mkwork = [&](int BS, int BF = 64, bool xcd = false, bool tord = false) {
        std::vector<uint64_t> w;
        const int nb = n / b;
        for (size_t q = 0; q < ops.size(); ++q) {
            const size_t o = tord ? (q % nb) * nb + q / nb : q;
            for (uint64_t k = 0; k < uint64_t(b / BF) * (b / BS); ++k) w.push_back((uint64_t(o) << 32) | k);
        }
        if (xcd) {  // blockIdx p -> XCD p%8: give each XCD a contiguous run of the list
            std::vector<uint64_t> v(w.size());
            const size_t per = w.size() / 8;
            for (size_t p = 0; p < w.size(); ++p) v[p] = w[(p % 8) * per + p / 8];
            w.swap(v);
        }
        uint64_t* d;
        CK(hipMalloc(&d, w.size() * 8));
        CK(hipMemcpy(d, w.data(), w.size() * 8, hipMemcpyHostToDevice));
        return std::make_pair(d, int64_t(w.size()));
    };
    auto w64 = mkwork(64), w128 = mkwork(128);
    auto w64x = mkwork(64, 64, true);
    auto g128x64 = mkwork(64, 128), g128x128 = mkwork(128, 128), g64x128 = mkwork(128, 64);
    auto g128x32 = mkwork(32, 128);
    auto g64x32 = mkwork(32, 64), g32x64 = mkwork(64, 32), g128x16 = mkwork(16, 128);
    auto g256x16 = mkwork(16, 256), g256x32 = mkwork(32, 256);
    auto t128x128 = mkwork(128, 128, false, true), t128x64 = mkwork(64, 128, false, true);
    auto t64x128 = mkwork(128, 64, false, true), t64x64 = mkwork(64, 64, false, true);
    auto t128x32 = mkwork(32, 128, false, true);
    unsigned long long* bad;
    CK(hipMalloc(&bad, 8));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double bytes = 2.0 * sizeof(double) * n * n;
    int cus = 256;

    struct var {
        std::string name;
        std::function<void()> run;
        bool verify;
        std::vector<float> ms;
    };
    std::vector<var> V;
    // ---- r2: hint (target column-major) order, nt loads and stores
    V.push_back({"H gen 128x128 t1024", [&] { hipLaunchKernelGGL((v_gen<128, 128, 1024, 1, 1>), dim3(t128x128.second), dim3(1024), 0, 0, d_ops, t128x128.first); }, true, {}});
    V.push_back({"H gen 128x128 t1024 plain", [&] { hipLaunchKernelGGL((v_gen<128, 128, 1024, 0, 0>), dim3(t128x128.second), dim3(1024), 0, 0, d_ops, t128x128.first); }, true, {}});
    V.push_back({"H gen 128x64 t512", [&] { hipLaunchKernelGGL((v_gen<128, 64, 512, 1, 1>), dim3(t128x64.second), dim3(512), 0, 0, d_ops, t128x64.first); }, true, {}});
    V.push_back({"H gen 64x128 t512", [&] { hipLaunchKernelGGL((v_gen<64, 128, 512, 1, 1>), dim3(t64x128.second), dim3(512), 0, 0, d_ops, t64x128.first); }, true, {}});
    V.push_back({"H gen 64x64 t256", [&] { hipLaunchKernelGGL((v_gen<64, 64, 256, 1, 1>), dim3(t64x64.second), dim3(256), 0, 0, d_ops, t64x64.first); }, true, {}});
    V.push_back({"H gen 128x128 t512", [&] { hipLaunchKernelGGL((v_gen<128, 128, 512, 1, 1>), dim3(t128x128.second), dim3(512), 0, 0, d_ops, t128x128.first); }, true, {}});
    V.push_back({"H tr 128x32 t256", [&] { hipLaunchKernelGGL((v_tr<128, 32, 256, 1, 1>), dim3(t128x32.second), dim3(256), 0, 0, d_ops, t128x32.first); }, true, {}});
    V.push_back({"H tr 64x64 t256", [&] { hipLaunchKernelGGL((v_tr<64, 64, 256, 1, 1>), dim3(t64x64.second), dim3(256), 0, 0, d_ops, t64x64.first); }, true, {}});
    V.push_back({"H tr 128x64 t512", [&] { hipLaunchKernelGGL((v_tr<128, 64, 512, 1, 1>), dim3(t128x64.second), dim3(512), 0, 0, d_ops, t128x64.first); }, true, {}});
    V.push_back({"H tr 128x64 t256", [&] { hipLaunchKernelGGL((v_tr<128, 64, 256, 1, 1>), dim3(t128x64.second), dim3(256), 0, 0, d_ops, t128x64.first); }, true, {}});
    {
        const int gb = 128 * 130 * 8;
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&v_glds1<2, 1>), hipFuncAttributeMaxDynamicSharedMemorySize, gb));
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&v_glds1<0, 1>), hipFuncAttributeMaxDynamicSharedMemorySize, gb));
        V.push_back({"H glds1 128x128 t1024 nt", [&, gb] { hipLaunchKernelGGL((v_glds1<2, 1>), dim3(t128x128.second), dim3(1024), gb, 0, d_ops, t128x128.first); }, true, {}});
        V.push_back({"H glds1 128x128 t1024 ldplain", [&, gb] { hipLaunchKernelGGL((v_glds1<0, 1>), dim3(t128x128.second), dim3(1024), gb, 0, d_ops, t128x128.first); }, true, {}});
    }
    for (int k : {1, 2}) {
        V.push_back({"H gpersist 128x128 t1024 x" + std::to_string(k), [&, k] { hipLaunchKernelGGL((v_gen_persist<128, 128, 1024, 1, 1>), dim3(cus * k), dim3(1024), 0, 0, d_ops, t128x128.first, t128x128.second); }, true, {}});
    }
    for (int k : {2, 3}) {
        V.push_back({"H gpersist 128x64 t512 x" + std::to_string(k), [&, k] { hipLaunchKernelGGL((v_gen_persist<128, 64, 512, 1, 1>), dim3(cus * k), dim3(512), 0, 0, d_ops, t128x64.first, t128x64.second); }, true, {}});
    }
    {
        auto hring = [&](auto kern, const char* name, int bs, int nt, int nb) {
            const int bytes = nb * bs * 130 * 8;
            CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
            auto w = bs == 64 ? t128x64 : t128x32;
            V.push_back({name, [=] { hipLaunchKernelGGL(kern, dim3(cus), dim3(nt), bytes, 0, d_ops,
                                                        w.first, w.second); }, true, {}});
        };
        hring(&v_ring<64, 512, 2, 1, 1>, "H ring 128x64 t512 nb2", 64, 512, 2);
        hring(&v_ring<64, 1024, 2, 1, 1>, "H ring 128x64 t1024 nb2", 64, 1024, 2);
        hring(&v_ring<32, 512, 4, 1, 1>, "H ring 128x32 t512 nb4", 32, 512, 4);
        hring(&v_ring<32, 512, 3, 1, 1>, "H ring 128x32 t512 nb3", 32, 512, 3);
    }
#define VTR(BF, BS, NT, NTL, NTS, W)                                                              \
    V.push_back({"tr " #BF "x" #BS " t" #NT " ntl" #NTL " nts" #NTS, [&] {                       \
        hipLaunchKernelGGL((v_tr<BF, BS, NT, NTL, NTS>), dim3(W.second), dim3(NT), 0, 0, d_ops,    \
                           W.first); }, true, {}})
    VTR(64, 32, 256, 1, 1, g64x32);
    VTR(64, 32, 256, 0, 0, g64x32);
    VTR(64, 32, 256, 1, 0, g64x32);
    VTR(32, 64, 256, 1, 1, g32x64);
    VTR(32, 64, 256, 0, 0, g32x64);
    VTR(128, 16, 256, 1, 1, g128x16);
    VTR(128, 32, 256, 1, 1, g128x32);
    VTR(128, 32, 256, 0, 0, g128x32);
    VTR(64, 64, 256, 1, 1, w64);
    VTR(256, 16, 256, 1, 1, g256x16);
    VTR(256, 32, 512, 1, 1, g256x32);
    VTR(128, 64, 512, 1, 1, g128x64);
    VTR(64, 32, 128, 1, 1, g64x32);
    V.push_back({"basic 64x64", [&] { hipLaunchKernelGGL((v_basic<64, 0>), dim3(w64.second), dim3(256), 0, 0, d_ops, w64.first); }, true, {}});
    V.push_back({"basic 64x64 nt-store", [&] { hipLaunchKernelGGL((v_basic<64, 1>), dim3(w64.second), dim3(256), 0, 0, d_ops, w64.first); }, true, {}});
    V.push_back({"basic 64x128", [&] { hipLaunchKernelGGL((v_basic<128, 0>), dim3(w128.second), dim3(256), 0, 0, d_ops, w128.first); }, true, {}});
    V.push_back({"pair 64x64", [&] { hipLaunchKernelGGL((v_pair<64, 0, 0>), dim3(w64.second), dim3(256), 0, 0, d_ops, w64.first); }, true, {}});
    V.push_back({"pair 64x64 nt-store", [&] { hipLaunchKernelGGL((v_pair<64, 1, 0>), dim3(w64.second), dim3(256), 0, 0, d_ops, w64.first); }, true, {}});
    V.push_back({"pair 64x64 nt-load", [&] { hipLaunchKernelGGL((v_pair<64, 0, 1>), dim3(w64.second), dim3(256), 0, 0, d_ops, w64.first); }, true, {}});
    V.push_back({"pair 64x128", [&] { hipLaunchKernelGGL((v_pair<128, 0, 0>), dim3(w128.second), dim3(256), 0, 0, d_ops, w128.first); }, true, {}});
    for (int k : {4, 8, 16}) {
        V.push_back({"persist 64x64 x" + std::to_string(k), [&, k] { hipLaunchKernelGGL((v_persist<64>), dim3(cus * k), dim3(256), 0, 0, d_ops, w64.first, w64.second); }, true, {}});
    }
    V.push_back({"persist 64x128 x4", [&] { hipLaunchKernelGGL((v_persist<128>), dim3(cus * 4), dim3(256), 0, 0, d_ops, w128.first, w128.second); }, true, {}});
    V.push_back({"flat copy 16B (ceiling)", [&] { hipLaunchKernelGGL(v_copy, dim3(cus * 16), dim3(256), 0, 0, (const d2*)A, (d2*)Cm, int64_t(n) * n / 2); }, false, {}});
    V.push_back({"hipMemcpyDtoD (ceiling)", [&] { CK(hipMemcpyAsync(Cm, A, sizeof(double) * n * n, hipMemcpyDeviceToDevice, 0)); }, false, {}});
    V.push_back({"gen 64x64 t256 nt-load", [&] { hipLaunchKernelGGL((v_gen<64, 64, 256, 1>), dim3(w64.second), dim3(256), 0, 0, d_ops, w64.first); }, true, {}});
    V.push_back({"gen 64x64 t256 nt-load xcd", [&] { hipLaunchKernelGGL((v_gen<64, 64, 256, 1>), dim3(w64x.second), dim3(256), 0, 0, d_ops, w64x.first); }, true, {}});
    V.push_back({"gen 128x64 t512", [&] { hipLaunchKernelGGL((v_gen<128, 64, 512, 0>), dim3(g128x64.second), dim3(512), 0, 0, d_ops, g128x64.first); }, true, {}});
    V.push_back({"gen 128x64 t512 nt-load", [&] { hipLaunchKernelGGL((v_gen<128, 64, 512, 1>), dim3(g128x64.second), dim3(512), 0, 0, d_ops, g128x64.first); }, true, {}});
    V.push_back({"gen 128x64 t256", [&] { hipLaunchKernelGGL((v_gen<128, 64, 256, 0>), dim3(g128x64.second), dim3(256), 0, 0, d_ops, g128x64.first); }, true, {}});
    V.push_back({"gen 64x128 t512", [&] { hipLaunchKernelGGL((v_gen<64, 128, 512, 0>), dim3(g64x128.second), dim3(512), 0, 0, d_ops, g64x128.first); }, true, {}});
    V.push_back({"gen 128x128 t1024", [&] { hipLaunchKernelGGL((v_gen<128, 128, 1024, 0>), dim3(g128x128.second), dim3(1024), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"gen 128x128 t1024 nt-load", [&] { hipLaunchKernelGGL((v_gen<128, 128, 1024, 1>), dim3(g128x128.second), dim3(1024), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"rowstore 128x128 pad2", [&] { hipLaunchKernelGGL((v_rowstore<2, 0>), dim3(g128x128.second), dim3(1024), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"rowstore 128x128 pad1", [&] { hipLaunchKernelGGL((v_rowstore<1, 0>), dim3(g128x128.second), dim3(1024), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"rowstore 128x128 pad1 nt-load", [&] { hipLaunchKernelGGL((v_rowstore<1, 1>), dim3(g128x128.second), dim3(1024), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"rowstore 128x128 pad3", [&] { hipLaunchKernelGGL((v_rowstore<3, 0>), dim3(g128x128.second), dim3(1024), 0, 0, d_ops, g128x128.first); }, true, {}});
    for (int k : {1, 2}) {
        V.push_back({"gpersist 128x128 t1024 x" + std::to_string(k), [&, k] { hipLaunchKernelGGL((v_gen_persist<128, 128, 1024>), dim3(cus * k), dim3(1024), 0, 0, d_ops, g128x128.first, g128x128.second); }, true, {}});
    }
    for (int k : {2, 3}) {
        V.push_back({"gpersist 128x64 t512 x" + std::to_string(k), [&, k] { hipLaunchKernelGGL((v_gen_persist<128, 64, 512>), dim3(cus * k), dim3(512), 0, 0, d_ops, g128x64.first, g128x64.second); }, true, {}});
    }
    V.push_back({"gpersist 64x64 t256 x4", [&] { hipLaunchKernelGGL((v_gen_persist<64, 64, 256>), dim3(cus * 4), dim3(256), 0, 0, d_ops, w64.first, w64.second); }, true, {}});
    V.push_back({"gen 128x128 t1024 nt-both", [&] { hipLaunchKernelGGL((v_gen<128, 128, 1024, 1, 1>), dim3(g128x128.second), dim3(1024), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"gen 128x128 t1024 nt-store", [&] { hipLaunchKernelGGL((v_gen<128, 128, 1024, 0, 1>), dim3(g128x128.second), dim3(1024), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"gen 128x64 t512 nt-both", [&] { hipLaunchKernelGGL((v_gen<128, 64, 512, 1, 1>), dim3(g128x64.second), dim3(512), 0, 0, d_ops, g128x64.first); }, true, {}});
    V.push_back({"gen 64x128 t512 nt-both", [&] { hipLaunchKernelGGL((v_gen<64, 128, 512, 1, 1>), dim3(g64x128.second), dim3(512), 0, 0, d_ops, g64x128.first); }, true, {}});
    V.push_back({"gen 64x64 t256 nt-both", [&] { hipLaunchKernelGGL((v_gen<64, 64, 256, 1, 1>), dim3(w64.second), dim3(256), 0, 0, d_ops, w64.first); }, true, {}});
    V.push_back({"gen 128x64 t256 nt-both", [&] { hipLaunchKernelGGL((v_gen<128, 64, 256, 1, 1>), dim3(g128x64.second), dim3(256), 0, 0, d_ops, g128x64.first); }, true, {}});
    V.push_back({"gen 128x128 t512 nt-both", [&] { hipLaunchKernelGGL((v_gen<128, 128, 512, 1, 1>), dim3(g128x128.second), dim3(512), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"gen 128x128 t512", [&] { hipLaunchKernelGGL((v_gen<128, 128, 512, 0>), dim3(g128x128.second), dim3(512), 0, 0, d_ops, g128x128.first); }, true, {}});
    V.push_back({"copyshape 128x32 t256", [&] { hipLaunchKernelGGL((v_copyshape<0>), dim3(g128x32.second), dim3(256), 0, 0, d_ops, g128x32.first); }, true, {}});
    V.push_back({"copyshape 128x32 t256 nt-load", [&] { hipLaunchKernelGGL((v_copyshape<1>), dim3(g128x32.second), dim3(256), 0, 0, d_ops, g128x32.first); }, true, {}});
    {
        const int glds_bytes = 2 * 64 * 130 * 8;
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&v_glds<0>), hipFuncAttributeMaxDynamicSharedMemorySize, glds_bytes));
        CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&v_glds<1>), hipFuncAttributeMaxDynamicSharedMemorySize, glds_bytes));
        V.push_back({"glds 128x64 t512 x1", [&, glds_bytes] { hipLaunchKernelGGL((v_glds<0>), dim3(cus), dim3(512), glds_bytes, 0, d_ops, g128x64.first, g128x64.second); }, true, {}});
        V.push_back({"glds 128x64 t512 x1 nt-load", [&, glds_bytes] { hipLaunchKernelGGL((v_glds<1>), dim3(cus), dim3(512), glds_bytes, 0, d_ops, g128x64.first, g128x64.second); }, true, {}});
    }
    {
        auto ring = [&](auto kern, const char* name, int bs, int nt, int nb) {
            const int bytes = nb * bs * 130 * 8;
            CK(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                   hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
            auto w = bs == 64 ? g128x64 : g128x32;
            V.push_back({name, [=] { hipLaunchKernelGGL(kern, dim3(cus), dim3(nt), bytes, 0, d_ops,
                                                        w.first, w.second); }, true, {}});
        };
        ring(&v_ring<64, 512, 2, 0>, "ring 128x64 t512 nb2", 64, 512, 2);
        ring(&v_ring<64, 512, 2, 1>, "ring 128x64 t512 nb2 nt", 64, 512, 2);
        ring(&v_ring<64, 1024, 2, 0>, "ring 128x64 t1024 nb2", 64, 1024, 2);
        ring(&v_ring<64, 1024, 2, 1>, "ring 128x64 t1024 nb2 nt", 64, 1024, 2);
        ring(&v_ring<32, 512, 4, 0>, "ring 128x32 t512 nb4", 32, 512, 4);
        ring(&v_ring<32, 512, 4, 1>, "ring 128x32 t512 nb4 nt", 32, 512, 4);
        ring(&v_ring<32, 256, 4, 1>, "ring 128x32 t256 nb4 nt", 32, 256, 4);
        ring(&v_ring<32, 512, 3, 1>, "ring 128x32 t512 nb3 nt", 32, 512, 3);
    }
    const int64_t n2 = int64_t(n) * n / 2;
    for (int g : {2, 4, 8, 32}) {
        V.push_back({"copy U8 grid " + std::to_string(g) + "/CU", [&, g] { hipLaunchKernelGGL((v_copy_ilp<8, 0, 0>), dim3(cus * g), dim3(256), 0, 0, (const d2*)A, (d2*)Cm, n2); }, false, {}});
    }
    V.push_back({"copy U4 grid 8/CU", [&] { hipLaunchKernelGGL((v_copy_ilp<4, 0, 0>), dim3(cus * 8), dim3(256), 0, 0, (const d2*)A, (d2*)Cm, n2); }, false, {}});
    V.push_back({"copy U16 grid 4/CU", [&] { hipLaunchKernelGGL((v_copy_ilp<16, 0, 0>), dim3(cus * 4), dim3(256), 0, 0, (const d2*)A, (d2*)Cm, n2); }, false, {}});
    V.push_back({"copy U8 nt-load", [&] { hipLaunchKernelGGL((v_copy_ilp<8, 1, 0>), dim3(cus * 8), dim3(256), 0, 0, (const d2*)A, (d2*)Cm, n2); }, false, {}});
    V.push_back({"copy U8 nt-both", [&] { hipLaunchKernelGGL((v_copy_ilp<8, 1, 1>), dim3(cus * 8), dim3(256), 0, 0, (const d2*)A, (d2*)Cm, n2); }, false, {}});
    V.push_back({"copy U8 nt-store", [&] { hipLaunchKernelGGL((v_copy_ilp<8, 0, 1>), dim3(cus * 8), dim3(256), 0, 0, (const d2*)A, (d2*)Cm, n2); }, false, {}});
    V.push_back({"copy U8 one-shot grid", [&] { hipLaunchKernelGGL((v_copy_ilp<8, 0, 0>), dim3(n2 / 2048), dim3(256), 0, 0, (const d2*)A, (d2*)Cm, n2); }, false, {}});
    V.push_back({"read-only 2GiB x2 (as 4GiB)", [&] { hipLaunchKernelGGL((v_read<8>), dim3(cus * 8), dim3(256), 0, 0, (const d2*)A, n2, (d2*)Cm); hipLaunchKernelGGL((v_read<8>), dim3(cus * 8), dim3(256), 0, 0, (const d2*)Cm, n2, (d2*)A); }, false, {}});
    V.push_back({"write-only 2GiB x2 (as 4GiB)", [&] { hipLaunchKernelGGL((v_write<8>), dim3(cus * 8), dim3(256), 0, 0, (d2*)Cm, n2); hipLaunchKernelGGL((v_write<8>), dim3(cus * 8), dim3(256), 0, 0, (d2*)Cm, n2); }, false, {}});

    if (argc > 2) {  // keep variants whose name contains one of the comma-separated tokens
        std::vector<std::string> toks;
        std::string f = argv[2];
        for (size_t a = 0, b; a <= f.size(); a = b + 1) {
            b = f.find(',', a);
            if (b == std::string::npos) b = f.size();
            if (b > a) toks.push_back(f.substr(a, b - a));
        }
        std::vector<var> keep;
        for (auto& v : V)
            for (auto& t : toks)
                if (v.name.find(t) != std::string::npos) {
                    keep.push_back(v);
                    break;
                }
        V.swap(keep);
    }
    for (auto& v : V) {  // warm + verify
        CK(hipMemset(Cm, 0, sizeof(double) * n * n));
        v.run();
        CK(hipDeviceSynchronize());
        if (v.verify) {
            CK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(check, dim3((int64_t(n) * n + 255) / 256), dim3(256), 0, 0, A, Cm, n, bad);
            unsigned long long h = 0;
            CK(hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost));
            printf("%-28s verify: %s\n", v.name.c_str(), h ? "FAIL" : "ok");
        }
    }
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
    printf("%-28s %9s %9s %9s %7s\n", "variant", "min ms", "med ms", "GB/s med", "%peak");
    for (auto& v : V) {
        std::sort(v.ms.begin(), v.ms.end());
        float med = v.ms[v.ms.size() / 2];
        printf("%-28s %9.4f %9.4f %9.1f %7.2f\n", v.name.c_str(), v.ms[0], med, bytes / med / 1e6,
               bytes / med / 1e6 / 80.0);
    }
    return 0;
}
