// Batched tile kernels for CDNA4 (gfx950): one launch runs a whole list of tile ops
// (pack, local or unpack), one workgroup per sub-tile of one op.
//
// What each op computes is the reference's copy_and_transform
// (eth-cscs/COSTA src/costa/grid2grid/memory_utils.hpp:339-412):
//   copy mode       dst(f, s) = g(src(f, s))                 copy2D / copy           :20-98
//   transpose mode  dst(s, f) = g(src(f, s))                 transpose_{col,row}_major :101-291
//   g(x) = x | 0 | alpha*op(x) | beta*dst + alpha*op(x)      (op = conj for 'C' on complex)
// evaluated in the reference's order with contraction OFF: results are bit-identical to the
// reference's x86 build (which has no FMA: SURVEY §8c).
//
// Memory path (HBM-bound, no MFMA: <= 0.5 flop/byte):
//   load   every lane fetches 16-byte vectors along the source's contiguous dimension; all
//          of a thread's loads are issued before any is consumed
//   LDS    the sub-tile is staged as rows s with a 16-byte pad per row, so both the
//          ds_write_b128 of the load phase and the ds_read_b128 of the store phase are
//          bank-conflict free
//   store  a lane reads one 16-byte LDS slot (V elements along f for one s); V lanes then
//          transpose their V x V block through cross-lane shuffles, so every lane stores one
//          16-byte vector along the destination's contiguous dimension
// Two paths: the "large" shape (512 or 1024 threads, 64 or 128 KiB sub-tiles, 512 B - 1 KiB load
// segments; `shapes` below) for ops with at least half a large sub-tile of data, aligned on both
// sides; the wavefront path (one op per wavefront, ops cut to wavefront size on the host) for
// the rest.  Measured on MI355X: cfg 2's transposes run at the rate a plain copy with the same
// access pattern reaches (tools/copy_ceiling.hip "pat").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "engine.hpp"

#pragma clang fp contract(off)

namespace costa {
namespace engine {
namespace {

template <typename R>
struct cpx {
    R re, im;
};

// ---- element arithmetic, written out so the rounding sequence is explicit ----
template <typename T> __device__ __forceinline__ T e_mul(T a, T b) { return a * b; }
template <typename T> __device__ __forceinline__ T e_add(T a, T b) { return a + b; }
template <typename T> __device__ __forceinline__ T e_conj(T a) { return a; }
template <typename T> __device__ __forceinline__ T e_zero() { return T(0); }

// (a + i b)(c + i d): the reference's std::complex product as GCC compiles it (C99 Annex G):
// the naive (ac - bd, ad + bc) -- 4 products, 2 sums, no fma -- and, only when BOTH parts come
// out NaN, libgcc's __muldc3 / __mulsc3 recovery of infinities (GCC 11.4 libgcc2.c; restated in
// oracle/costa_oracle.c ANNEX_G_MUL and pinned to GCC there): an infinite factor is "boxed" to
// +-1 / +-0 with the other factor's NaNs zeroed, or, when a partial product overflowed, every
// NaN is zeroed; then the product is recomputed and scaled by infinity.  The branch is never
// taken on finite data: (inf + inf i)(1 + 0i) = inf + inf i, not NaN + NaN i.
// (the partial products are recomputed inside the rare branch rather than kept live: fewer
// registers on the common path)
template <typename R>
__device__ __attribute__((cold)) cpx<R> annex_g_recover(R a, R b, R c, R d) {
    const R one = R(1), zero = R(0), inf = __builtin_huge_val();
    const bool ovf = __builtin_isinf(a * c) || __builtin_isinf(b * d) || __builtin_isinf(a * d) ||
                     __builtin_isinf(b * c);
    bool recalc = false;
    if (__builtin_isinf(a) || __builtin_isinf(b)) {
        a = __builtin_copysign(__builtin_isinf(a) ? one : zero, a);
        b = __builtin_copysign(__builtin_isinf(b) ? one : zero, b);
        if (__builtin_isnan(c)) c = __builtin_copysign(zero, c);
        if (__builtin_isnan(d)) d = __builtin_copysign(zero, d);
        recalc = true;
    }
    if (__builtin_isinf(c) || __builtin_isinf(d)) {
        c = __builtin_copysign(__builtin_isinf(c) ? one : zero, c);
        d = __builtin_copysign(__builtin_isinf(d) ? one : zero, d);
        if (__builtin_isnan(a)) a = __builtin_copysign(zero, a);
        if (__builtin_isnan(b)) b = __builtin_copysign(zero, b);
        recalc = true;
    }
    if (!recalc && ovf) {
        if (__builtin_isnan(a)) a = __builtin_copysign(zero, a);
        if (__builtin_isnan(b)) b = __builtin_copysign(zero, b);
        if (__builtin_isnan(c)) c = __builtin_copysign(zero, c);
        if (__builtin_isnan(d)) d = __builtin_copysign(zero, d);
        recalc = true;
    }
    const R p = a * c, q = b * d, r = a * d, t = b * c;
    if (!recalc) return {p - q, r + t};
    return {inf * (p - q), inf * (r + t)};
}
#ifndef COSTA_ANNEX_G  // 0: naive complex products only (tuning builds: the recovery's cost)
#define COSTA_ANNEX_G 1
#endif
template <typename R>
__device__ __forceinline__ cpx<R> cmul(cpx<R> z, cpx<R> w) {
    const R x = z.re * w.re - z.im * w.im, y = z.re * w.im + z.im * w.re;
    if (COSTA_ANNEX_G && __builtin_expect(__builtin_isnan(x) && __builtin_isnan(y), 0))
        return annex_g_recover(z.re, z.im, w.re, w.im);
    return {x, y};
}
template <> __device__ __forceinline__ cpx<float> e_mul(cpx<float> a, cpx<float> b) { return cmul(a, b); }
template <> __device__ __forceinline__ cpx<double> e_mul(cpx<double> a, cpx<double> b) { return cmul(a, b); }
template <> __device__ __forceinline__ cpx<float> e_add(cpx<float> a, cpx<float> b) {
    return {a.re + b.re, a.im + b.im};
}
template <> __device__ __forceinline__ cpx<double> e_add(cpx<double> a, cpx<double> b) {
    return {a.re + b.re, a.im + b.im};
}
template <> __device__ __forceinline__ cpx<float> e_conj(cpx<float> a) { return {a.re, -a.im}; }
template <> __device__ __forceinline__ cpx<double> e_conj(cpx<double> a) { return {a.re, -a.im}; }
template <> __device__ __forceinline__ cpx<float> e_zero() { return {0.f, 0.f}; }
template <> __device__ __forceinline__ cpx<double> e_zero() { return {0.0, 0.0}; }

// g(x) for one element; `y` is the old destination value (read only for AXPBY)
template <typename T>
__device__ __forceinline__ T scale(T x, T y, uint32_t kind, bool conj, T alpha, T beta) {
    if (conj) x = e_conj(x);
    if (kind == COSTA_SCALE_ZERO) return e_zero<T>();
    if (kind == COSTA_SCALE_ALPHA) return e_mul(alpha, x);
    if (kind == COSTA_SCALE_AXPBY) return e_add(e_mul(beta, y), e_mul(alpha, x));
    return x;  // BITCOPY
}

// The same with the naive complex product only: `bad` is set when a product needs the Annex G
// recovery (both parts NaN), and the caller then redoes that vector with scale() out of the
// hot loop (run_tile): the recovery code stays off the register-hungry large shapes' main path
// (inlined per element it made the 1024-thread c64 shape spill to scratch).
template <typename T> struct is_cpx { static constexpr bool value = false; };
template <typename R> struct is_cpx<cpx<R>> { static constexpr bool value = true; };
// (a product whose parts are both NaN leaves both parts of the result NaN, beta * y + alpha * x
// included, so checking the result suffices; a NaN result for another reason is redone too,
// with the same outcome).  Costs cfg 4 (c128 'T', alpha, beta) ~3 %: 2.234 against 2.170 ms
// with naive products only (COSTA_ANNEX_G=0, profiles/r3/annex_ab.txt); storing unconditionally
// and fixing up afterwards would keep the old values live and spill.
template <typename T> __device__ __forceinline__ T e_mul_naive(T a, T b) { return a * b; }
template <typename R>
__device__ __forceinline__ cpx<R> e_mul_naive(cpx<R> z, cpx<R> w) {
    return {z.re * w.re - z.im * w.im, z.re * w.im + z.im * w.re};
}
template <typename T> __device__ __forceinline__ bool both_nan(const T&) { return false; }
template <typename R> __device__ __forceinline__ bool both_nan(const cpx<R>& v) {
    return COSTA_ANNEX_G && (v.re != v.re) & (v.im != v.im);
}
template <typename T>
__device__ __forceinline__ T scale_naive(T x, T y, uint32_t kind, bool conj, T alpha, T beta,
                                         bool& bad) {
    if (conj) x = e_conj(x);
    T r = x;  // BITCOPY
    if (kind == COSTA_SCALE_ZERO) r = e_zero<T>();
    else if (kind == COSTA_SCALE_ALPHA) r = e_mul_naive(alpha, x);
    else if (kind == COSTA_SCALE_AXPBY) r = e_add(e_mul_naive(beta, y), e_mul_naive(alpha, x));
    bad = bad | both_nan(r);
    return r;
}

// ---- cross-lane moves ----
[[maybe_unused]] __device__ __forceinline__ float shfl(float v, int l) { return __shfl(v, l); }
[[maybe_unused]] __device__ __forceinline__ int shfl(int v, int l) { return __shfl(v, l); }
[[maybe_unused]] __device__ __forceinline__ double shfl(double v, int l) { return __shfl(v, l); }
[[maybe_unused]] __device__ __forceinline__ cpx<float> shfl(cpx<float> v, int l) {
    return {__shfl(v.re, l), __shfl(v.im, l)};
}

// V elements = one 16-byte vector
template <typename T>
struct vec {
    static constexpr int V = 16 / int(sizeof(T));
    T e[V];
};
struct __attribute__((aligned(16))) raw16 {
    uint32_t w[4];
};

// 16-byte vector accesses of the tile kernels are non-temporal (`nt`): every byte of a
// transform is read once and written once, and on MI355X the nt policy moves such streams
// faster (tools/copy_ceiling.hip, profiles/r2/: a strided 2 GiB copy in 1 KiB column segments
// 6.37-6.49 TB/s with nt loads and stores against 6.02-6.23 without; cfg 2's transposed access
// pattern 6.27 against 5.73).
typedef uint32_t u32x4a __attribute__((ext_vector_type(4)));
// 16-byte loads need only dword alignment on gfx950 (global_load_dwordx4): sources of 4-byte
// elements off the 16-byte grid are read this way too (engine.cpp build_work marks them
// COSTA_TILE_VEC_SRC), so the load goes through a type that promises 4-byte alignment only
typedef uint32_t u32x4d __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ raw16 ld16(const void* p) {
    raw16 r;
    const u32x4d v = __builtin_nontemporal_load(reinterpret_cast<const u32x4d*>(p));
    __builtin_memcpy(&r, &v, 16);
    return r;
}
template <bool NT = true>
__device__ __forceinline__ void st16(void* p, const raw16& r) {
    if constexpr (NT) {
        u32x4a v;
        __builtin_memcpy(&v, &r, 16);
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4a*>(p));
    } else {
        *reinterpret_cast<raw16*>(p) = r;
    }
}

template <typename T, bool NT = true>
__device__ __forceinline__ void vload(vec<T>& out, const T* p, int n, bool vec_ok) {
    constexpr int V = vec<T>::V;
    if (vec_ok && n >= V) {
        raw16 r;
        if constexpr (NT) {
            r = ld16(p);
        } else {
            const u32x4d v = *reinterpret_cast<const u32x4d*>(p);
            __builtin_memcpy(&r, &v, 16);
        }
        __builtin_memcpy(&out, &r, 16);
    } else {
#pragma unroll
        for (int k = 0; k < V; ++k)
            if (k < n) out.e[k] = p[k];
    }
}

template <typename T, bool NT = true>
__device__ __forceinline__ void vstore(T* p, const vec<T>& in, int n, bool vec_ok) {
    constexpr int V = vec<T>::V;
    if (vec_ok && n >= V) {
        raw16 r;
        __builtin_memcpy(&r, &in, 16);
        st16<NT>(p, r);
    } else {
#pragma unroll
        for (int k = 0; k < V; ++k)
            if (k < n) p[k] = in.e[k];
    }
}

// Lanes k = 0..V-1 of an aligned group hold in[.] = row k of a V x V block; afterwards
// lane k holds column k.  Round r: every lane offers element (k - r) mod V and reads the
// offer of lane (k + r) mod V.  All indices are compile-time after unrolling.  The cross-lane
// read is a DPP quad permutation (a VALU move; V <= 4 lanes sit in one quad), not an LDS
// permute: the large shape spends its non-overlapped LDS time on the tile itself (the
// ds_bpermute form ran equally fast, 0.7063 ms both, with the LDS busier).
template <int V, int R>
constexpr int quad_ctrl() {  // quad_perm: lane q of each quad reads lane sel(q)
    int c = 0;
    for (int q = 0; q < 4; ++q) {
        const int base = q & ~(V - 1), k = q & (V - 1);
        c |= (base + ((k + R) & (V - 1))) << (2 * q);
    }
    return c;
}
template <int CTRL, typename T>
__device__ __forceinline__ T dpp_move(T v) {
    static_assert(sizeof(T) % 4 == 0, "32-bit words");
    uint32_t w[sizeof(T) / 4];
    __builtin_memcpy(w, &v, sizeof(T));
#pragma unroll
    for (unsigned i = 0; i < sizeof(T) / 4; ++i)
        w[i] = uint32_t(__builtin_amdgcn_mov_dpp(int(w[i]), CTRL, 0xF, 0xF, true));
    T out;
    __builtin_memcpy(&out, w, sizeof(T));
    return out;
}
template <typename T, int R>
__device__ __forceinline__ void xround(const vec<T>& in, vec<T>& out, int lane) {
    constexpr int V = vec<T>::V;
    const int k = lane & (V - 1);
    const int give = (k - R) & (V - 1), from = (k + R) & (V - 1);
    T offer = in.e[0];
#pragma unroll
    for (int e = 1; e < V; ++e)
        if (e == give) offer = in.e[e];
    T got = offer;
    if constexpr (R != 0) got = dpp_move<quad_ctrl<V, R>()>(offer);
#pragma unroll
    for (int e = 0; e < V; ++e)
        if (e == from) out.e[e] = got;
}
// a[k] for a lane-dependent k in 0..3, as selects (a runtime-indexed vec<T> lives in scratch)
template <typename T>
__device__ __forceinline__ T sel4(int k, T a0, T a1, T a2, T a3) {
    return k == 0 ? a0 : k == 1 ? a1 : k == 2 ? a2 : a3;
}
template <typename T>
__device__ __forceinline__ vec<T> lane_transpose(const vec<T>& in, int lane) {
    constexpr int V = vec<T>::V;
    static_assert(V == 1 || V == 2 || V == 4, "one quad");
    vec<T> out;
    if constexpr (V == 1) {
        out = in;
    } else if constexpr (V == 2) {
        xround<T, 0>(in, out, lane);
        xround<T, 1>(in, out, lane);
    } else {
        // V = 4 (4-byte elements), every index compile-time: lane k rotates its row by k
        // (r[e] = in[(e + k) & 3]), so in round R every lane offers r[R] and lane k receives
        // in_{k-R}[k]; out[e] = g[(k - e) & 3] un-rotates (r13: the runtime-indexed form of
        // xround kept 144 bytes per lane in scratch and ran fp32 transposes at 3.3 TB/s)
        const int k = lane & 3;
        const T r0 = sel4(k, in.e[0], in.e[1], in.e[2], in.e[3]);
        const T r1 = sel4(k, in.e[1], in.e[2], in.e[3], in.e[0]);
        const T r2 = sel4(k, in.e[2], in.e[3], in.e[0], in.e[1]);
        const T r3 = sel4(k, in.e[3], in.e[0], in.e[1], in.e[2]);
        const T g0 = r0;
        const T g1 = dpp_move<quad_ctrl<4, 3>()>(r1);  // from lane (k - 1) & 3
        const T g2 = dpp_move<quad_ctrl<4, 2>()>(r2);  // from lane (k - 2) & 3
        const T g3 = dpp_move<quad_ctrl<4, 1>()>(r3);  // from lane (k - 3) & 3
        out.e[0] = sel4(k, g0, g1, g2, g3);
        out.e[1] = sel4(k, g3, g0, g1, g2);
        out.e[2] = sel4(k, g2, g3, g0, g1);
        out.e[3] = sel4(k, g1, g2, g3, g0);
    }
    return out;
}

// A lane of the transposing store phase holds V consecutive destination elements d[0, V) of one
// destination column (s values sb .. sb + V - 1); with an odd ld those columns start off the
// 16-byte grid: d sits eps elements past an aligned address.  Element-wise stores there ran
// 8-byte fp64 columns at ~4 TB/s against 6.1 aligned (HBM traffic equal: 1.035x), misaligned
// 16-byte stores no faster.  Instead every aligned chunk [d - eps, d - eps + V) is stored whole,
// by the lane whose own elements fill its top V - eps slots, the bottom eps taken from the lane V
// below (which holds d[-V, 0) of the same column: same f, s values sb - V ..).  The lowest lane
// group of a store unit has no such neighbour in its wavefront and stores its own part element by
// element; so does a lane whose upper eps elements no lane above will cover (top of the unit or of
// the tile).  Every lane that is valid here runs the shuffle (the lane V below a valid lane is
// valid: same column, earlier s).
template <typename T, int V, int EPS>
__device__ __forceinline__ vec<T> shifted_chunk(const vec<T>& below, const vec<T>& o) {
    vec<T> c;
#pragma unroll
    for (int e = 0; e < V; ++e)
        c.e[e] = e < EPS ? below.e[V - EPS + e < V ? V - EPS + e : V - 1] : o.e[e >= EPS ? e - EPS : 0];
    return c;
}
template <typename T, typename S, bool NT>
__device__ __forceinline__ void store_shifted(T* d, const vec<T>& o, int n, int lane) {
    constexpr int V = S::V;
    vec<T> below;
#pragma unroll
    for (int e = 0; e < V; ++e) below.e[e] = __shfl_up(o.e[e], unsigned(V), 64);
    const int eps = int((reinterpret_cast<uintptr_t>(d) / sizeof(T)) & uintptr_t(V - 1));
    if (eps == 0) {
        vstore<T, NT>(d, o, n, true);
        return;
    }
    const int ls = lane % S::SW;
    const int own = V - eps;  // own elements in the chunk that starts eps below d
    if (ls >= V && n >= own) {
        // (every register index compile-time: one branch per eps)
        vec<T> c;
        if (eps == 1) c = shifted_chunk<T, V, 1>(below, o);
        if constexpr (V > 2) {
            if (eps == 2) c = shifted_chunk<T, V, 2>(below, o);
            if (eps == 3) c = shifted_chunk<T, V, 3>(below, o);
        }
        vstore<T, NT>(d - eps, c, V, true);
    } else {
#pragma unroll
        for (int e = 0; e < V; ++e)
            if (e < own && e < n) d[e] = o.e[e];
    }
    // the upper eps elements go with the chunk of the lane V above, unless there is none
    if (ls + V >= S::SW || n - V < own) {
#pragma unroll
        for (int e = 0; e < V; ++e)
            if (e >= own && e < n) d[e] = o.e[e];
    }
}

// sub-tile geometry of one kernel shape
template <typename T, int NT_, int BF_, int BS_>
struct shape {
    static constexpr int NT = NT_;
    static constexpr int V = vec<T>::V;
    static constexpr int BF = BF_;                  // elements along the source's fast dim
    static constexpr int BS = BS_;                  // elements along the source's slow dim
    static constexpr int P = BF + V;                // LDS row pitch (16-byte pad)
    static constexpr int LPC = BF / V;              // lanes per source column (load)
    static constexpr int CPP = NT / LPC;            // source columns per load pass
    static constexpr int PL = BS / CPP;             // load passes
    static constexpr int NW = NT / 64;              // wavefronts
    static constexpr int SW = BS < 64 ? BS : 64;    // s values of one store unit per f slot
    static constexpr int FW = 64 / SW;              // f slots of one store unit (a wavefront)
    static constexpr int UNITS = (BS / SW) * (BF / V) / FW;  // store units: SW s x FW f slots
    static constexpr int PS = UNITS / NW;           // store passes
    static_assert(LPC <= NT && NT % LPC == 0 && BS % CPP == 0, "load mapping");
    static_assert(BS % SW == 0 && SW % V == 0 && (BF / V) % FW == 0 && UNITS % NW == 0, "store mapping");
    static constexpr size_t lds_bytes = size_t(BS) * P * sizeof(T);
};

// the large shapes per element size: `large` for copy-only lists, `large_tr` for lists that
// transpose.  Transposes of fp64 / fp32 / int32 take 512 threads and 64 KiB sub-tiles (~67 KiB
// of LDS: two workgroups per CU, whose load and store phases overlap); c64 / c128 1024 threads
// and 128 KiB.  Measured on 16384^2 (r2, profiles/r2/shapes/): fp64 'T' 64 x 128 against
// 128 x 128 / 1024 threads 0.698 against 0.712 ms with 256^2 and 128^2 blocks, 0.779 against
// 1.057 with 64^2 blocks (those went to the wavefront path); 128 x 64 slower (0.765-0.811); fp32
// 'T' 128 x 128 against 256 x 128 / 1024 threads 0.367 against 0.578 ms with 128^2 blocks
// (half-filled sub-tiles before), 0.397 against 0.402 with 256^2.
// Copies (r5): 512 threads, two 16-byte loads a thread, 1 KiB column segments (16 KiB
// sub-tiles of 1 KiB x 16 columns; no LDS, so many workgroups a CU).  A plain copy runs fastest
// with few loads a thread in flight (profiles/r4zj/); side by side against r4's
// 128 KiB sub-tiles with 8-32 loads a thread (profiles/r5v/, r5w/): BASELINE cfg 3's copy slice
// (fp64 32768^2, 128^2 blocks) 2.797 -> 2.620 ms (6.56 TB/s), fp64 16384^2 256^2 blocks 0.68 ->
// 0.65 ms (beta != 0: 1.07 -> 1.01), fp32 0.36 -> 0.322, c64 0.695 -> 0.650, c128 (128^2 blocks)
// 1.45 -> 1.29; one load a thread (1024 threads) 3.13 ms on cfg 3, 128 x 8 sub-tiles 2.72-2.77,
// 1024 threads x 2 loads 2.66.  Copy-only lists still classify and merge their ops by r4's
// sub-tile sizes (copy_class below).
// `medium_tr`: 256 threads, 16 KiB sub-tiles, for aligned transposing ops of at least half of
// one that are below half a large sub-tile (before: cut into wavefront pieces of ~128-byte
// runs): fp32 64^2 blocks 3.60 -> 4.77 TB/s, 96^2 4.18 -> 4.60; fp64 32^2 4.27 -> 4.97, 48^2
// 4.27 -> 5.26 (profiles/r2/shapes/medium.log).  None for c64 / c128 (has_medium).
template <typename T> struct shapes;
// the sub-tile dimensions by which copy-only lists classify and merge their ops (engine.cpp
// build_work: the large class = ops of at least half of one; merge_filled): r4's copy sub-tiles,
// so that the r5 copy shapes change how the large class runs, not which ops it holds
template <typename T> struct copy_class;
template <> struct copy_class<float> { static constexpr int BF = 256, BS = 128; };
template <> struct copy_class<int> { static constexpr int BF = 256, BS = 128; };
template <> struct copy_class<double> { static constexpr int BF = 128, BS = 128; };
template <> struct copy_class<cpx<float>> { static constexpr int BF = 128, BS = 128; };
template <> struct copy_class<cpx<double>> { static constexpr int BF = 64, BS = 128; };
// `small_tr` (fp64): the square 64 x 64 variant of the large transposing shape, 512 threads, for
// transposing lists whose large ops all fit in it (engine.cpp build_work): a 64^2 block then fills
// one sub-tile instead of half of a 64 x 128 one, and four workgroups fit a CU.  fp64 16384^2 'T'
// with 64^2 blocks 0.683-0.726 ms against 0.783 (profiles/r2d/small_blocks/).
// medium shapes: 256 threads.  4-byte types take 128 threads when every medium op
// of the list is a whole number of sub-tiles (`medium_tr_full`, engine.cpp work_split::med_full):
// fp32 64^2 blocks 0.455 -> 0.408 ms (beta = 0 only: with C read 0.628 against 0.610); with
// ragged ops 128 / 512 threads lost 12-21 % (48^2, 80^2)
// and fp64 lost 12-14 % at 32^2 / 48^2 (profiles/r2d/medium_threads.log)
template <> struct shapes<float> {
    using large = shape<float, 512, 256, 16>;
    using large_tr = shape<float, 512, 128, 128>;
    using medium_tr = shape<float, 256, 64, 64>;
    static constexpr bool has_medium = true;
    using small_tr = large_tr;
    static constexpr bool has_small = false;
    using large_tr_full = large_tr;
    using medium_tr_full = shape<float, 128, 64, 64>;
    using small32_tr = shape<float, 128, 32, 32>;
};
template <> struct shapes<int> {
    using large = shape<int, 512, 256, 16>;
    using large_tr = shape<int, 512, 128, 128>;
    using medium_tr = shape<int, 256, 64, 64>;
    static constexpr bool has_medium = true;
    using small_tr = large_tr;
    static constexpr bool has_small = false;
    using large_tr_full = large_tr;
    using medium_tr_full = shape<int, 128, 64, 64>;
    using small32_tr = shape<int, 128, 32, 32>;
};
template <> struct shapes<double> {
    using large = shape<double, 512, 128, 16>;
    using large_tr = shape<double, 512, 64, 128>;
    using medium_tr = shape<double, 256, 32, 64>;
    static constexpr bool has_medium = true;
    using small_tr = shape<double, 512, 64, 64>;
    static constexpr bool has_small = true;
    using large_tr_full = large_tr;
    using medium_tr_full = medium_tr;
    using small32_tr = shape<double, 128, 32, 32>;
};
// c128 transposes: 1024 threads.  256 gain 3 % when every op is a whole number of sub-tiles (cfg
// 4's 128^2 blocks: 2.19 against 2.26 ms; the `large_tr_full` launch, engine.cpp
// work_split::full) and lose 35-55 % with blocks that half-fill them (80^2 3.05 against 1.98 ms,
// 96^2 2.35 against 1.74; profiles/r2c/tr_shapes/, profiles/r2d/c128_threads.log).  The square
// 64 x 64 sub-tile (cfg 4's destination-ordered lists, r4) takes 1024 threads since r5: 4 loads a
// thread, one workgroup a CU (72 VGPRs); cfg 4's 32768^2 slice 8.58-8.64 -> 8.38-8.44 ms against
// 256 threads (512: 8.61-8.64; profiles/r5y/)
template <> struct shapes<cpx<float>> {
    using large = shape<cpx<float>, 512, 128, 16>;
    using large_tr = shape<cpx<float>, 1024, 128, 128>;
    using medium_tr = large_tr;
    static constexpr bool has_medium = false;
    using small_tr = shape<cpx<float>, 512, 64, 64>;
    static constexpr bool has_small = true;
    using large_tr_full = large_tr;
    using medium_tr_full = medium_tr;
    using small32_tr = shape<cpx<float>, 128, 32, 32>;
};
template <> struct shapes<cpx<double>> {
    using large = shape<cpx<double>, 512, 64, 16>;
    using large_tr = shape<cpx<double>, 1024, 64, 128>;
    using medium_tr = large_tr;
    static constexpr bool has_medium = false;
    using small_tr = shape<cpx<double>, 1024, 64, 64>;
    static constexpr bool has_small = true;
    using large_tr_full = shape<cpx<double>, 256, 64, 128>;
    using medium_tr_full = medium_tr;
    using small32_tr = shape<cpx<double>, 128, 32, 32>;
};

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void glob_void;

// One sub-tile.  FULL: the sub-tile is a whole BF x BS block with 16-byte aligned rows on
// both sides, so every guard below folds away and each thread issues its loads and stores
// back to back with no per-lane branches (the common case: block-cyclic tiles).
template <typename T, typename S, bool FULL, bool NT = true>
__device__ __forceinline__ void run_tile(const costa_tile_op_t& op, int f0, int s0, int tf_, int ts_,
                                         const char* src_base, char* dst_base, T alpha, T beta,
                                         T* tile) {
    constexpr int V = S::V, BF = S::BF, P = S::P;
    const int tf = FULL ? S::BF : tf_;
    const int ts = FULL ? S::BS : ts_;
    const uint32_t flags = op.flags;
    const uint32_t kind = (flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
    const bool conj = flags & COSTA_TILE_CONJ;
    const bool vs = FULL || (flags & COSTA_TILE_VEC_SRC);
    const bool vd = FULL || (flags & COSTA_TILE_VEC_DST);
    const int64_t lds = op.lds, ldd = op.ldd;
    const T* src = reinterpret_cast<const T*>(src_base + op.src) + int64_t(s0) * lds + f0;

    // ---- load phase: lane -> (16-byte strip along f, column s); all loads issued first
    const int lf = (int(threadIdx.x) % S::LPC) * V;
    const int c0 = int(threadIdx.x) / S::LPC;
    auto col_of = [&](int k) { return c0 + k * S::CPP; };  // source column of load k
    const int nf_lane = FULL ? V : tf - lf;  // elements of this lane's strip inside the tile
    vec<T> x[S::PL];
#pragma unroll
    for (int k = 0; k < S::PL; ++k) {
        const int s = col_of(k);
        if (FULL || (nf_lane > 0 && s < ts)) vload(x[k], src + s * lds + lf, nf_lane, vs);
    }

    if (!(flags & COSTA_TILE_TRANSPOSE)) {
        // ---- copy mode: dst(f, s) = g(src(f, s)), no LDS
        T* dst = reinterpret_cast<T*>(dst_base + op.dst) + int64_t(s0) * ldd + f0;
        // beta != 0: every old value is requested before the first store (a load behind a
        // store to the same array would otherwise wait for it: one round trip per strip)
        vec<T> y[S::PL];
        if (kind == COSTA_SCALE_AXPBY) {
#pragma unroll
            for (int k = 0; k < S::PL; ++k) {
                const int s = col_of(k);
                if (FULL || (nf_lane > 0 && s < ts)) vload(y[k], dst + s * ldd + lf, nf_lane, vd);
            }
        }
        uint32_t redo = 0;  // complex vectors left for the Annex G path (bit k: strip k)
#pragma unroll
        for (int k = 0; k < S::PL; ++k) {
            const int s = col_of(k);
            if (!FULL && (nf_lane <= 0 || s >= ts)) continue;
            T* d = dst + s * ldd + lf;
            if (kind != COSTA_SCALE_BITCOPY) {
                bool bad = false;
#pragma unroll
                for (int e = 0; e < V; ++e)
                    x[k].e[e] = scale_naive(x[k].e[e], kind == COSTA_SCALE_AXPBY ? y[k].e[e] : e_zero<T>(),
                                            kind, conj, alpha, beta, bad);
                if (is_cpx<T>::value && bad) {
                    redo |= 1u << k;
                    continue;
                }
            }
            vstore<T, NT>(d, x[k], nf_lane, vd);
        }
        if constexpr (is_cpx<T>::value) {
            static_assert(S::PL <= 32, "redo mask");
            // strips whose naive products needed the recovery: source and (not yet written)
            // destination are read again and every element goes through scale()
            if (__builtin_expect(redo != 0, 0)) {
#pragma unroll 1
                for (int k = 0; k < S::PL; ++k) {
                    if (!((redo >> k) & 1u)) continue;
                    const int s = col_of(k);
                    const T* a = src + s * lds + lf;
                    T* d = dst + s * ldd + lf;
                    const int n = FULL ? V : min(V, nf_lane);
#pragma unroll 1
                    for (int e = 0; e < n; ++e)
                        d[e] = scale(a[e], kind == COSTA_SCALE_AXPBY ? d[e] : e_zero<T>(), kind, conj,
                                     alpha, beta);
                }
            }
        }
        return;
    }

    // ---- transpose mode: dst(s, f) = g(src(f, s)) through LDS
    T* dst = reinterpret_cast<T*>(dst_base + op.dst) + int64_t(f0) * ldd + s0;
    const int lane = int(threadIdx.x) % 64, wave = int(threadIdx.x) / 64;
    constexpr int SW = S::SW, FW = S::FW, QG = BF / V / FW;  // QG: f-slot groups per s chunk
    // store unit u -> (s chunk, f-slot group): s chunk slowest, units NW apart per wavefront.
    // PAIR (r5, the fp64 64 x 128 shape of BASELINE cfg 2): a wavefront stores its own column
    // pairs, the two s chunks of a pair back to back, so each destination column's 1 KiB segment
    // is written in one go.  Side by side on the same buffers (tools/libs_probe.py,
    // profiles/r5l/): fp64 0.6990 -> 0.6934 ms; fp32 128 x 128 +2 %, c128 64 x 64 +4.5 %: those
    // keep the strided order
    constexpr int NSC = S::BS / SW;
    constexpr bool PAIR = FULL && std::is_same<T, double>::value && S::BF == 64 && S::BS == 128 && S::NT == 512;
    auto unit_u = [&](int k) {
        if constexpr (PAIR) return wave * S::PS + k;
        return wave + S::NW * k;
    };
    auto unit_sc = [&](int u) {
        if constexpr (PAIR) return u % NSC;
        return u / QG;
    };
    auto unit_q = [&](int u) {
        if constexpr (PAIR) return u / NSC;
        return u % QG;
    };
    // store unit k of this lane: SW s values x FW f slots (64 x 1 for BS >= 64); after the lane
    // exchange lane (base + j) stores f = q*V + j for s = sc*SW + base .. +V-1
    auto unit = [&](int k, int& f, int& sb, int& n) {
        const int u = unit_u(k);
        const int sc = unit_sc(u), q = unit_q(u) * FW + lane / SW;
        const int j = lane & (V - 1);
        f = q * V + j;
        sb = sc * SW + (lane % SW - j);
        n = FULL ? V : ts - sb;
        return FULL || (f < tf && n > 0);
    };
    // beta != 0: the old destination values are requested now, overlapping the source loads
    // still in flight (not after the LDS exchange, one round trip per store unit)
    vec<T> old[S::PS];
    if (kind == COSTA_SCALE_AXPBY) {
#pragma unroll
        for (int k = 0; k < S::PS; ++k) {
            int f, sb, n;
            if (unit(k, f, sb, n)) vload(old[k], dst + f * ldd + sb, n, vd);
        }
    }
#pragma unroll
    for (int k = 0; k < S::PL; ++k) {
        const int s = col_of(k);
        if (FULL || (nf_lane > 0 && s < ts)) {  // partial strips: the tail is junk, never stored
            raw16 r;
            __builtin_memcpy(&r, &x[k], 16);
            *reinterpret_cast<raw16*>(tile + s * P + lf) = r;
        }
    }
    __syncthreads();

    vec<T> y[S::PS];
#pragma unroll
    for (int k = 0; k < S::PS; ++k) {
        const int u = unit_u(k);                         // store unit
        const int sc = unit_sc(u), q = unit_q(u) * FW + lane / SW;   // s chunk, f slot
        const int s = sc * SW + lane % SW;
        if (FULL || (s < ts && q * V < tf)) {
            raw16 r = *reinterpret_cast<const raw16*>(tile + s * P + q * V);
            __builtin_memcpy(&y[k], &r, 16);
        }
    }
    uint32_t redo = 0;  // complex store units left for the Annex G path (bit k: unit k)
    // destination columns not 16-byte aligned but element aligned (an odd ScaLAPACK lld): the
    // stores are re-cut into aligned 16-byte chunks across lanes (store_shifted)
    const bool shift_dst = !vd && op.dst % sizeof(T) == 0;
#pragma unroll
    for (int k = 0; k < S::PS; ++k) {
        vec<T> o = lane_transpose(y[k], lane);
        int f, sb, n;
        if (!unit(k, f, sb, n)) continue;
        T* d = dst + f * ldd + sb;
        if (kind != COSTA_SCALE_BITCOPY) {
            bool bad = false;
#pragma unroll
            for (int e = 0; e < V; ++e)
                o.e[e] = scale_naive(o.e[e], kind == COSTA_SCALE_AXPBY ? old[k].e[e] : e_zero<T>(),
                                     kind, conj, alpha, beta, bad);
            if (is_cpx<T>::value && bad) {
                redo |= 1u << k;
                continue;
            }
        }
        if constexpr (!FULL && !is_cpx<T>::value && V > 1) {
            if (shift_dst) {
                store_shifted<T, S, NT>(d, o, n, lane);
                continue;
            }
        }
        vstore<T, NT>(d, o, n, vd);
    }
    if constexpr (is_cpx<T>::value) {
        static_assert(S::PS <= 32, "redo mask");
        // units whose naive products needed the recovery: element e of the unit is source row
        // sb + e, column f of the staged tile (read straight from LDS: no lane exchange with
        // part of the wavefront inactive), its old value is still in the destination
        if (__builtin_expect(redo != 0, 0)) {
#pragma unroll 1
            for (int k = 0; k < S::PS; ++k) {
                if (!((redo >> k) & 1u)) continue;
                int f, sb, n;
                unit(k, f, sb, n);
                T* d = dst + f * ldd + sb;
                n = FULL ? V : min(V, n);
#pragma unroll 1
                for (int e = 0; e < n; ++e)
                    d[e] = scale(tile[(sb + e) * P + f], kind == COSTA_SCALE_AXPBY ? d[e] : e_zero<T>(),
                                 kind, conj, alpha, beta);
            }
        }
    }
}

template <typename T, typename S>
__global__ __launch_bounds__(S::NT) void tile_kernel(const costa_tile_op_t* __restrict__ ops,
                                                     const uint64_t* __restrict__ work,
                                                     const char* src_base, char* dst_base,
                                                     const T* __restrict__ scalars) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* tile = reinterpret_cast<T*>(smem);
    // which sub-tile of which op (wave-uniform: scalar loads)
    const uint64_t w = work[blockIdx.x];
    const costa_tile_op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = (op.nf + S::BF - 1) / S::BF;
    const int f0 = int(sub % uint32_t(nbf)) * S::BF;
    const int s0 = int(sub / uint32_t(nbf)) * S::BS;
    const int tf = min(S::BF, op.nf - f0);
    const int ts = min(S::BS, op.ns - s0);
    const uint32_t slot = op.flags >> COSTA_SLOT_SHIFT;
    const T alpha = scalars[2 * slot];
    const T beta = scalars[2 * slot + 1];
    const uint32_t vec_both = COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST;
    constexpr bool NT = true;
    if (tf == S::BF && ts == S::BS && (op.flags & vec_both) == vec_both)
        run_tile<T, S, true, NT>(op, f0, s0, tf, ts, src_base, dst_base, alpha, beta, tile);
    else
        run_tile<T, S, false, NT>(op, f0, s0, tf, ts, src_base, dst_base, alpha, beta, tile);
}

// ---------------------------------------------------------------- skew shape
// Transposing ops whose destination columns are off the 16-byte grid (an odd ScaLAPACK lld;
// engine.cpp build_work routes them here, real types).  A partial 64-byte granule written by two
// workgroups costs the HBM a read-modify-write: a copy with its lines split at 16-byte granularity
// between neighbouring workgroups ran 0.808 against 0.672 ms (tools/partial_line_probe.hip).  So
// the cut between sub-tiles follows the granules of each destination column instead of the source
// rows: in column f, sub-tile (f0, s0) writes [s0 - eps_f, s0 + BS - eps_f), eps_f being how far
// d(f, s0) lies past a granule boundary (the same for every s0 of the column: BS * sizeof(T) is a
// multiple of 64), the first sub-tile of the op from 0, the last one up to ns.  Every element is
// written by exactly one workgroup, every granule inside the op by one: no duplicated bytes, and
// ops that read C (beta != 0) are as safe here as anywhere.  The source rows [s0 - G, s0 + BS)
// are staged (odd pitch: the column-wise LDS reads of the store phase are conflict-free); lanes
// then walk each destination column in 16-byte chunks, 64 consecutive chunks per instruction.
// Sub-tiles: 4-byte types 32 x 512, fp64 64 x 128.
// WIDE (4-byte types, lists whose skew ops also read sources off the 16-byte grid): 64 x 256
// instead of 32 x 512, so every misaligned source run is 256 bytes, not 128 (its two partial
// lines shared with the f-neighbour sub-tiles, which engine.cpp build_work then puts on one XCD);
// fp32 16384^2 'T' lld 16385 both sides 0.456 -> 0.419-0.424 ms with that grouping, while
// destination-only lists lost with it (0.384 -> 0.430: they keep 32 x 512, no grouping;
// profiles/r3b/README.md §skew)
template <typename T, bool WIDE = false>
struct skew_shape {
    static constexpr int NT = 512;
    static constexpr int BF = sizeof(T) == 4 ? (WIDE ? 64 : 32) : 64;
    static constexpr int BS = sizeof(T) == 4 ? (WIDE ? 256 : 512) : 128;
    static constexpr int E = int(sizeof(T)), G = 64 / E, RS = BS + G, P = BF + 1;
    static constexpr int V = 16 / E, LPC = BF / V, CPP = NT / LPC, PL = (RS + CPP - 1) / CPP;
    static constexpr int NW = NT / 64;
    static constexpr size_t lds_bytes = size_t(RS) * P * sizeof(T);
    static_assert(BS * E % 64 == 0, "sub-tile rows: whole granules");
};

template <typename T, bool WIDE>
__global__ __launch_bounds__(512) void skew_kernel(const costa_tile_op_t* __restrict__ ops,
                                                   const uint64_t* __restrict__ work,
                                                   const char* src_base, char* dst_base,
                                                   const T* __restrict__ scalars) {
    using K = skew_shape<T, WIDE>;
    constexpr int V = K::V, BF = K::BF, BS = K::BS, G = K::G, P = K::P;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* tile = reinterpret_cast<T*>(smem);
    const uint64_t w = work[blockIdx.x];
    const costa_tile_op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = (op.nf + BF - 1) / BF;
    const int f0 = int(sub % uint32_t(nbf)) * BF;
    const int s0 = int(sub / uint32_t(nbf)) * BS;
    const int tf = min(BF, op.nf - f0), ns = op.ns;
    const uint32_t kind = (op.flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
    const uint32_t slot = op.flags >> COSTA_SLOT_SHIFT;
    const T alpha = kind >= COSTA_SCALE_ALPHA ? scalars[2 * slot] : T(0);
    const T beta = kind == COSTA_SCALE_AXPBY ? scalars[2 * slot + 1] : T(0);
    const bool vs = op.flags & COSTA_TILE_VEC_SRC;
    const int64_t lds = op.lds, ldd = op.ldd;
    const T* src = reinterpret_cast<const T*>(src_base + op.src) + f0;
    // ---- rows s = s0 - G + r, r < RS, inside the op: all loads first (16-byte vectors when the
    // source allows, else element loads: shifted aligned chunks measured slower here, 0.954
    // against 0.843 ms with both sides off the grid)
    const int lf = (int(threadIdx.x) % K::LPC) * V;
    const int c0 = int(threadIdx.x) / K::LPC;
    const int nf_lane = tf - lf;
    const int s_lo = s0 > 0 ? s0 - G : 0, s_hi = min(ns, s0 + BS);
    vec<T> x[K::PL];
#pragma unroll
    for (int k = 0; k < K::PL; ++k) {
        const int r = c0 + k * K::CPP, s = s0 - G + r;
        // (default cache policy: the G rows above s0 are also the previous sub-tile's, which
        // reads them from L2 then; non-temporal loads ran fp64 dst-odd 'T' 0.750-0.764 against
        // 0.780-0.782 ms, fp32 both sides odd 1-1.5 % slower, the rest level: profiles/r6j/)
        if (r < K::RS && s >= s_lo && s < s_hi && nf_lane > 0)
            vload<T, false>(x[k], src + s * lds + lf, nf_lane, vs);
    }
#pragma unroll
    for (int k = 0; k < K::PL; ++k) {
        const int r = c0 + k * K::CPP, s = s0 - G + r;
        if (r < K::RS && s >= s_lo && s < s_hi && nf_lane > 0) {
#pragma unroll
            for (int e = 0; e < V; ++e)
                if (e < nf_lane) tile[r * P + lf + e] = x[k].e[e];
        }
    }
    __syncthreads();
    // ---- destination column f0 + f, 16-byte chunks between granule boundaries
    const int lane = int(threadIdx.x) % 64, wave = int(threadIdx.x) / 64;
    T* dst = reinterpret_cast<T*>(dst_base + op.dst);
    const bool last = s0 + BS >= ns;
    for (int f = wave; f < tf; f += K::NW) {
        T* col = dst + int64_t(f0 + f) * ldd;
        const int eps = int((reinterpret_cast<uintptr_t>(col + s0) / sizeof(T)) & uintptr_t(G - 1));
        const int lo = s0 > 0 ? s0 - eps : 0;
        const int hi = last ? ns : s0 + BS - eps;
        // [lo, hi) is whole granules except where it meets the op's edges: 16-byte chunks from the
        // first aligned element a to b, single elements before and after
        const int mis = int((reinterpret_cast<uintptr_t>(col + lo) / sizeof(T)) & uintptr_t(V - 1));
        const int a = min(hi, lo + ((V - mis) & (V - 1)));
        const int b = a + (hi - a) / V * V;
        const T* tcol = tile + (G - s0) * P + f;  // element s of the column at tcol[s * P]
        if (lo + lane < a) {
            T* d = col + lo + lane;
            *d = scale(tcol[(lo + lane) * P], kind == COSTA_SCALE_AXPBY ? *d : T(0), kind, false, alpha, beta);
        }
        if (b + lane < hi) {
            T* d = col + b + lane;
            *d = scale(tcol[(b + lane) * P], kind == COSTA_SCALE_AXPBY ? *d : T(0), kind, false, alpha, beta);
        }
        for (int c = a + V * lane; c < b; c += 64 * V) {
            vec<T> y, o;
            if (kind == COSTA_SCALE_AXPBY) vload(y, col + c, V, true);
#pragma unroll
            for (int e = 0; e < V; ++e)
                o.e[e] = scale(tcol[(c + e) * P], kind == COSTA_SCALE_AXPBY ? y.e[e] : T(0), kind, false,
                               alpha, beta);
            vstore<T, true>(col + c, o, V, true);
        }
    }
}

template <typename T, bool WIDE>
void launch_skew_w(const launch_args& a, const uint64_t* work, int64_t n, hipStream_t stream) {
    using K = skew_shape<T, WIDE>;
    const int64_t max_grid = 1LL << 30;
    for (int64_t off = 0; off < n; off += max_grid) {
        const int64_t m = std::min(max_grid, n - off);
        hipLaunchKernelGGL((skew_kernel<T, WIDE>), dim3(unsigned(m)), dim3(K::NT), K::lds_bytes, stream,
                           a.ops, work + off, a.src_base, a.dst_base, static_cast<const T*>(a.scalars));
    }
}
template <typename T>
void launch_skew(const launch_args& a, const uint64_t* work, int64_t n, hipStream_t stream) {
    if constexpr (std::is_same<T, float>::value || std::is_same<T, double>::value ||
                  std::is_same<T, int>::value) {
        if (a.skew_wide && sizeof(T) == 4)
            launch_skew_w<T, true>(a, work, n, stream);
        else
            launch_skew_w<T, false>(a, work, n, stream);
    } else if (n > 0) {
        throw error(COSTA_ERR_INTERNAL, "costa: skew shape for a complex type");
    }
}

// ---------------------------------------------------------------- wavefront path
// Every op below the large shape, cut on the host into wave-sized rectangles (engine.cpp
// wave_pieces), runs on one wavefront.  Lanes walk the tile in linear order: source order (f
// fastest) for loads, destination order for stores, with (f, s) advanced by a constant per step
// (no per-element division).  Copy mode needs no LDS; transpose mode stages the tile in the
// wave's own LDS region with an odd row pitch (conflict-free column reads).
// Measured on BASELINE cfg 5 (242k tiles of ~33x33 fp32, 'N'): 1.8 TB/s with one 256-thread
// workgroup per tile, 2.65 TB/s with one wavefront per op, 3.35-3.5 TB/s with the directly
// indexed, destination-sorted list and the host split, 4.3-4.5 with the r11 XCD remap and
// budgets.  What bounds it now is the access shape itself: a strided copy in whole, aligned
// 128-byte cache lines reaches 4.8-4.9 TB/s, 256-byte runs 5.4-5.5, 1 KiB runs 6.3
// (tools/copy_ceiling.hip "seg L*", profiles/r2/); cfg 5's column runs are ~132 bytes with
// ragged edges.  Variants measured slower and removed: 16-byte copy accesses,
// several ops per wavefront (strided, chunked, moved together), a persistent pipelined kernel
// (next op's loads in flight while this op stores: 2.9 against 4.4 TB/s), nt cache policy here.
// r3: transposing ops stage through LDS-DMA and request their old destination values before
// the one wait (tiny_transpose_glds): cfg 5 'T' 0.781 -> 0.743 ms on one lease (4 waves per
// workgroup), 0.722 with 8; without the early old-value loads 0.948 (profiles/r3b/README.md §glds).
// Wavefronts per workgroup: 8 (4 KiB of LDS each for lists that transpose; copy-only lists
// without LDS: profiles/r06/c5_knobs.log).
// r3 (LDS-DMA staging): cfg 5 'T' 0.736-0.738 ms with 4 wavefronts per workgroup, 0.721-0.723
// with 8, 0.728-0.729 with 16, 0.759-0.761 with 2 (profiles/r3b/README.md §glds)
constexpr int TINY_WAVES_TR = 8;
constexpr int TINY_WAVES_COPY = 8;
// the same for the copy path (engine.hpp tiny_copy_lane_bytes): 64 for every type since r11
template <typename T> constexpr int tiny_copy_bytes() { return tiny_copy_lane_bytes(sizeof(T)); }

template <typename T>
struct lin {  // (f, s) of linear element index e = f + s*n, stepped by 64
    int f, s, df, ds, n;
    __device__ __forceinline__ lin(int lane, int n_) : n(n_) {
        f = lane % n;
        s = lane / n;
        df = 64 % n;
        ds = 64 / n;
    }
    __device__ __forceinline__ void step() {
        f += df;
        s += ds;
        if (f >= n) {
            f -= n;
            ++s;
        }
    }
};

// Transpose mode with the staging loads going straight to LDS (global_load_lds_dword: no VGPR
// destination), so a wavefront has its whole staged tile and, for ops that read C, every old
// destination value (16 VGPRs at most: the tile is at most tiny_lds_budget() bytes) in flight at
// once, and waits once: one memory round trip per op instead of one per 64 x U elements of each
// phase (register staging holds U elements per lane and pass).  The LDS image is the same
// (element (f, s) at s * pitch + f, pitch odd): an LDS-DMA instruction writes its 64 dwords
// lane-linearly from a wave-uniform base, so lane j of instruction k takes dword 64 k + j of the
// padded image and loads whatever source word belongs there (pad words: lane inactive).
template <typename T>
__device__ __forceinline__ void tiny_stage(const T* src, int nf, int ns, int64_t lds, int pitch, int lane,
                                           T* t) {
    constexpr int W = int(sizeof(T)) / 4;  // dwords per element
    constexpr int DP = 64 / W;             // image positions per instruction
    const int nd = pitch * ns * W;
    {
        const int w = lane % W;
        int f = (lane / W) % pitch, s = (lane / W) / pitch;
        const int df = DP % pitch, ds = DP / pitch;
        const char* sb = reinterpret_cast<const char*>(src) + 4 * w;
        char* tb = reinterpret_cast<char*>(t);
        for (int d0 = 0; d0 < nd; d0 += 64) {
            if (f < nf && d0 + lane < nd)
                __builtin_amdgcn_global_load_lds((glob_void*)(sb + (int64_t(s) * lds + f) * int64_t(sizeof(T))),
                                                 (lds_void*)(tb + 4 * d0), 4, 0, 0);
            f += df;
            s += ds;
            if (f >= pitch) {
                f -= pitch;
                ++s;
            }
        }
    }
}

template <typename T, bool AX>
__device__ __forceinline__ void tiny_transpose_glds(const T* src, T* dst, int nf, int ns, int64_t lds,
                                                    int64_t ldd, uint32_t kind, bool conj, T alpha, T beta,
                                                    int lane, T* t) {
    constexpr int NY = kTinyLdsDefault / (64 * int(sizeof(T)));  // passes with old values held
    constexpr int NP = kTinyLdsBytes / (64 * int(sizeof(T)));    // destination passes at most
    const int pitch = nf | 1, total = nf * ns;
    tiny_stage(src, nf, ns, lds, pitch, lane, t);
    // the old destination values of the whole op, requested before the wait
    T y[AX && NY > 0 ? NY : 1];
    if constexpr (AX) {
        if (kind == COSTA_SCALE_AXPBY) {
            lin<T> q(lane, ns);  // destination order: q.f walks s, q.s walks f
#pragma unroll
            for (int u = 0; u < NY; ++u) {
                if (u * 64 >= total) break;
                if (u * 64 + lane < total) y[u] = dst[int64_t(q.s) * ldd + q.f];
                q.step();
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the LDS-DMA writes (and y) have landed
    lin<T> q(lane, ns);
#pragma unroll
    for (int u = 0; u < NP; ++u) {
        if (u * 64 >= total) break;
        if (u * 64 + lane < total) {
            const T v = t[q.f * pitch + q.s];
            T* d = dst + int64_t(q.s) * ldd + q.f;
            T old = e_zero<T>();
            if (AX && kind == COSTA_SCALE_AXPBY) old = u < NY ? y[AX && u < NY ? u : 0] : *d;
            *d = scale(v, old, kind, conj, alpha, beta);
        }
        q.step();
    }
}

// TR = false: the list has no transposing op (the transpose path and its registers are
// compiled out, so copy-only lists keep a high occupancy).  AX = false: no op of the list reads
// its destination (beta == 0 everywhere), so the copy path holds no old values.  UC: bytes per
// lane of one copy pass.
template <typename T, bool TR, bool AX, int UC>
__device__ __forceinline__ void tiny_op(const costa_tile_op_t& op, int lane, T* t,
                                        const char* src_base, char* dst_base,
                                        const T* __restrict__ scalars) {
    const uint32_t flags = op.flags;
    const uint32_t kind = (flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
    const bool conj = flags & COSTA_TILE_CONJ;
    const uint32_t slot = flags >> COSTA_SLOT_SHIFT;
    T alpha = e_zero<T>(), beta = e_zero<T>();
    if (kind >= COSTA_SCALE_ALPHA) {  // BITCOPY / ZERO never read the scalars
        alpha = scalars[2 * slot];
        beta = scalars[2 * slot + 1];
    }
    const T* src = reinterpret_cast<const T*>(src_base + op.src);
    T* dst = reinterpret_cast<T*>(dst_base + op.dst);
    const int nf = op.nf, ns = op.ns, total = nf * ns;
    const int64_t lds = op.lds, ldd = op.ldd;

    if (!TR || !(flags & COSTA_TILE_TRANSPOSE)) {
        // copy mode: dst(f, s) = g(src(f, s)).  Every load of a pass is issued before the first
        // store; passes end where the op ends (wave-uniform tests), and the store walk repeats
        // the load walk instead of keeping every element's address in registers.
        constexpr int UCE = UC / int(sizeof(T)) > 0 ? UC / int(sizeof(T)) : 1;
        lin<T> p(lane, nf);
        for (int e0 = 0; e0 < total; e0 += 64 * UCE) {
            T x[UCE];
            T y[AX ? UCE : 1];
            const lin<T> q0 = p;
#pragma unroll
            for (int u = 0; u < UCE; ++u) {
                if (e0 + u * 64 >= total) break;
                if (e0 + u * 64 + lane < total) x[u] = src[p.s * lds + p.f];
                p.step();
            }
            if constexpr (AX) {
                if (kind == COSTA_SCALE_AXPBY) {
                    lin<T> r = q0;
#pragma unroll
                    for (int u = 0; u < UCE; ++u) {
                        if (e0 + u * 64 >= total) break;
                        if (e0 + u * 64 + lane < total) y[u] = dst[r.s * ldd + r.f];
                        r.step();
                    }
                }
            }
            lin<T> q = q0;
#pragma unroll
            for (int u = 0; u < UCE; ++u) {
                if (e0 + u * 64 >= total) break;
                if (e0 + u * 64 + lane < total) {
                    T v = x[u];
                    if (kind != COSTA_SCALE_BITCOPY)
                        v = scale(v, AX && kind == COSTA_SCALE_AXPBY ? y[AX ? u : 0] : e_zero<T>(),
                                  kind, conj, alpha, beta);
                    dst[q.s * ldd + q.f] = v;
                }
                q.step();
            }
        }
        return;
    }
    // transpose mode: staged in LDS by LDS-DMA (pitch odd), then written in destination order
    // (the destination side in aligned 16-byte chunks, element-wise heads and tails, halved the
    // vector-memory instructions of cfg 5 'T' and ran 10 % slower with 25 % more L2 requests:
    // profiles/r4a/cfg5T_chunk_ab.txt, profiles/r4b/)
    tiny_transpose_glds<T, AX>(src, dst, nf, ns, lds, ldd, kind, conj, alpha, beta, lane, t);
}

// ---------------------------------------------------------------- destination blocks (r5)
// A group = the ops of a list that together write one contiguous destination range: R rows x K
// columns of a column-major buffer whose leading dimension is R (a custom layout's own block
// buffer, or a column band of it; engine.cpp cblock_groups).  One workgroup per group:
//   load   every wavefront walks its share of the group's ops in source order (lanes along the
//          source's contiguous dimension, U elements a lane in flight) and writes each element
//          to its destination position in an LDS image of the range (column pitch R | 1: the
//          transposed writes are conflict-free)
//   store  the range in 16-byte vectors at 16-byte aligned addresses, old values (beta != 0)
//          requested before the barrier, element-wise only at the two ends
// Every destination granule inside the range is written by this workgroup alone, in whole
// 16-byte vectors: the wavefront path writes cfg 5's destination columns one element a lane,
// each granule shared by the tiles of two source blocks (cfg 5).
// Header op (work item): src = number of ops that follow it, dst = the range, nf = R, ns = K,
// flags = the transform of every op of the group.
constexpr int CB_NT = kCblockThreads;              // threads per workgroup
constexpr int CB_CHUNKS = kCblockChunks;           // 16-byte destination vectors per thread
constexpr int CB_U = 16;                           // source elements a lane has in flight
constexpr int CB_UV = 8;                           // ... 16-byte chunks, for 4-byte copy groups

template <typename T, bool TR, bool AX>
__global__ __launch_bounds__(CB_NT) void cblock_kernel(const costa_tile_op_t* __restrict__ ops,
                                                       const uint64_t* __restrict__ work,
                                                       const char* src_base, char* dst_base,
                                                       const T* __restrict__ scalars, int map, int chunk,
                                                       int64_t n_groups, const costa_tile_op_t* __restrict__ pieces,
                                                       int64_t n_pieces, int piece_lds) {
    constexpr int V = 16 / int(sizeof(T)), NW = CB_NT / 64;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* img = reinterpret_cast<T*>(smem);
    if (int64_t(blockIdx.x) >= n_groups) {
        // the list's wavefront pieces (tiny_kernel's work), one a wavefront, as workgroups after
        // the groups in the same launch: dispatched last, they run in the groups' tail instead of
        // a launch of their own (launch_cblock: fuse)
        const int64_t b = xcd_slice_order(int64_t(blockIdx.x) - n_groups, int64_t(gridDim.x) - n_groups);
        const int wv = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / 64);
        const int64_t w = b * NW + wv;
        if (w >= n_pieces) return;
        tiny_op<T, TR, AX, tiny_copy_bytes<T>()>(pieces[w], int(threadIdx.x) % 64, img + int64_t(wv) * piece_lds,
                                                 src_base, dst_base, scalars);
        return;
    }
    // Transposing lists: workgroups are dealt round-robin over the 8 XCDs; renumbered so that
    // each XCD takes `chunk` (kCblockXcdChunk) consecutive groups of the destination order and
    // the 8 XCDs work on 8 adjacent such chunks -- neighbouring groups read the other parts of the
    // same source cache lines, now in one L2.  cfg 5 'T' 0.634 -> 0.600 ms with chunks of 4 (r5;
    // one contiguous slice per XCD 0.625, its L2 -> memory reads -36 %); r6: 16, the source lines
    // shared across a chunk boundary a quarter as often -- reads 1.190x -> 1.065x their bytes,
    // traffic 1.134x -> 1.050x, for +0.7 % in-run (8: 1.107x at +0.2 %, 32 / 64 1.044x / 1.033x
    // at +1.4 / +2.6 %; profiles/r6m/, r6n/).  The copy ('N') uses the XCD column bands
    // (map == cb_xcd_bands: XCD x walks the x-th slice of the list, one band of target columns;
    // engine.cpp cblock_groups)
    uint64_t g = blockIdx.x;
    if (map == cb_xcd_chunks) g = uint64_t(cblock_xcd_order(int64_t(blockIdx.x), n_groups, chunk));
    else if (map == cb_xcd_bands) g = uint64_t(xcd_slice_order(int64_t(blockIdx.x), n_groups));
    const uint64_t h = work[g];
    const costa_tile_op_t hd = ops[h];
    const int n_ops = int(hd.src), R = hd.nf, K = hd.ns, P = R | 1;
    const uint32_t flags = hd.flags;
    const uint32_t kind = (flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
    const bool conj = flags & COSTA_TILE_CONJ;
    const bool tr = TR && (flags & COSTA_TILE_TRANSPOSE);
    const uint32_t slot = flags >> COSTA_SLOT_SHIFT;
    T alpha = e_zero<T>(), beta = e_zero<T>();
    if (kind >= COSTA_SCALE_ALPHA) {
        alpha = scalars[2 * slot];
        beta = scalars[2 * slot + 1];
    }
    const int lane = int(threadIdx.x) % 64;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / 64);
    T* dst = reinterpret_cast<T*>(dst_base + hd.dst);
    const int total = R * K;
    // 16-byte vectors of the range: vector c holds elements [V c - mis, V c - mis + V)
    const int mis = int((reinterpret_cast<uintptr_t>(dst) / sizeof(T)) & uintptr_t(V - 1));
    const int nvec = (total + mis + V - 1) / V;
    vec<T> old[CB_CHUNKS];
    if (AX && kind == COSTA_SCALE_AXPBY) {  // old values, in flight with the source loads
#pragma unroll
        for (int k = 0; k < CB_CHUNKS; ++k) {
            const int c = int(threadIdx.x) + CB_NT * k;
            const int e0 = V * c - mis;
            if (c >= nvec) break;
            if (e0 >= 0 && e0 + V <= total) {
                raw16 r = *reinterpret_cast<const raw16*>(dst + e0);
                __builtin_memcpy(&old[k], &r, 16);
            } else {
#pragma unroll
                for (int e = 0; e < V; ++e)
                    if (e0 + e >= 0 && e0 + e < total) old[k].e[e] = dst[e0 + e];
            }
        }
    }
    // ---- sources -> image (element (r, c) of the range at c * P + r)
    for (int i = wave; i < n_ops; i += NW) {
        const costa_tile_op_t op = ops[h + 1 + uint64_t(i)];
        const T* src = reinterpret_cast<const T*>(src_base + op.src);
        const int64_t e0 = int64_t(op.dst - hd.dst) / int64_t(sizeof(T));
        const int r0 = int(e0 % R), c0 = int(e0 / R);
        const int nf = op.nf, n = op.nf * op.ns;
        const int64_t lds = op.lds;
        // image position of source element (f, s): transpose (r0 + s, c0 + f), copy (r0 + f, c0 + s)
        const int di_f = tr ? P : 1, di_s = tr ? 1 : P;
        const int ibase = c0 * P + r0;
        if constexpr (sizeof(T) == 4 && !TR) {
            // copy-only lists of 4-byte elements (r6): each source column run read as the aligned
            // 16-byte chunks covering it -- a quarter of the load instructions: ncm chunk slots a
            // column (enough for any alignment), slot (k, s) -> the k-th chunk from the one
            // holding the column's first element; elements outside the run are dropped.  An
            // aligned chunk never crosses a page, and holds at least one element of the run.
            // cfg 5 'N', with the XCD column bands (engine.cpp cblock_groups): 0.436 -> 0.427 ms,
            // 0.402 with default-policy chunk loads
            // (CB_UV chunks a lane in flight: 2 / 4 / 8 0.438 / 0.429 / 0.427; 32 KiB groups 0.523;
            // each change alone +1 %; 8 KiB groups 0.484, 128 / 512 threads 0.452 / 0.641:
            // profiles/r6c/, r6d/, r6f/, r6h/).  Transposing groups keep dword loads: a chunk's
            // four elements land P x 4 apart in the transposed image, 'T' 0.600 -> 0.857 ms, 0.775
            // with the writes in lane-rotated order
            const int ncm = (nf + 6) / 4, nq = ncm * op.ns;
            lin<T> q(lane, ncm);
            for (int b = 0; b < nq; b += 64 * CB_UV) {
                raw16 x[CB_UV];
                int fb[CB_UV], sv[CB_UV];
#pragma unroll
                for (int u = 0; u < CB_UV; ++u) {
                    fb[u] = nf;
                    if (b + u * 64 + lane < nq) {
                        const T* col = src + int64_t(q.s) * lds;
                        const int mis = int((reinterpret_cast<uintptr_t>(col) >> 2) & 3);
                        const int f = 4 * q.f - mis;  // the chunk's first element, relative to the run
                        if (f < nf) {
                            // default cache policy, not non-temporal: the edge lines a run shares
                            // with its neighbours (the next column, the group of the next band or
                            // block-row) stay in L2 for them -- nt chunks read 1.32x the run bytes
                            // at 0.428 ms, these 1.03x at 0.402 (profiles/r6i/)
                            const u32x4a v = *reinterpret_cast<const u32x4a*>(col + f);
                            __builtin_memcpy(&x[u], &v, 16);
                            fb[u] = f;
                            sv[u] = q.s;
                        }
                    }
                    q.step();
                }
#pragma unroll
                for (int u = 0; u < CB_UV; ++u) {
                    if (fb[u] >= nf) continue;
                    T v[4];
                    __builtin_memcpy(v, &x[u], 16);
                    // (in element order: the 4-way bank conflicts of one write step -- lanes 4
                    // elements apart -- cost less than a lane-rotated order's selects, 'N' 0.428
                    // against 0.441 ms; profiles/r6h/)
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int f = fb[u] + e;
                        if (f >= 0 && f < nf) img[ibase + f * di_f + sv[u] * di_s] = v[e];
                    }
                }
            }
            continue;
        }
        lin<T> p(lane, nf);
        for (int b = 0; b < n; b += 64 * CB_U) {
            T x[CB_U];
            int at[CB_U];
#pragma unroll
            for (int u = 0; u < CB_U; ++u) {
                if (b + u * 64 >= n) break;
                at[u] = -1;
                if (b + u * 64 + lane < n) {
                    x[u] = src[p.s * lds + p.f];
                    at[u] = ibase + p.f * di_f + p.s * di_s;
                }
                p.step();
            }
#pragma unroll
            for (int u = 0; u < CB_U; ++u) {
                if (b + u * 64 >= n) break;
                if (at[u] >= 0) img[at[u]] = x[u];
            }
        }
    }
    __syncthreads();
    // ---- image -> the range, 16-byte vectors
#pragma unroll
    for (int k = 0; k < CB_CHUNKS; ++k) {
        const int c = int(threadIdx.x) + CB_NT * k;
        if (c >= nvec) break;
        const int e0 = V * c - mis;
        const int first = e0 < 0 ? -e0 : 0;  // elements of the vector inside the range
        int r = (e0 + first) % R, col = (e0 + first) / R;
        vec<T> o;
#pragma unroll
        for (int e = 0; e < V; ++e) {
            if (e < first || e0 + e >= total) continue;
            T v = img[col * P + r];
            if (kind != COSTA_SCALE_BITCOPY)
                v = scale(v, AX && kind == COSTA_SCALE_AXPBY ? old[k].e[e] : e_zero<T>(), kind, conj,
                          alpha, beta);
            o.e[e] = v;
            if (++r == R) {
                r = 0;
                ++col;
            }
        }
        if (e0 >= 0 && e0 + V <= total) {
            raw16 w;
            __builtin_memcpy(&w, &o, 16);
            st16<true>(dst + e0, w);
        } else {
#pragma unroll
            for (int e = 0; e < V; ++e)
                if (e0 + e >= 0 && e0 + e < total) dst[e0 + e] = o.e[e];
        }
    }
}

template <typename T, bool TR, bool AX>
void launch_cblock_v(const launch_args& a, const uint64_t* work, int64_t n, bool fuse, hipStream_t stream) {
    static const int chunk = [] {  // COSTA_CB_CHUNK (tuning): groups per XCD chunk
        const char* v = tuning_env("COSTA_CB_CHUNK");
        return v ? std::max(1, std::atoi(v)) : int(kCblockXcdChunk);
    }();
    const int64_t max_grid = 1LL << 30;
    // the wavefront pieces fused into the launch (launch_t decides): CB_NT / 64 a workgroup, each
    // wavefront its tiny_lds_budget() of the LDS when the list transposes
    const int64_t pb = fuse ? (a.n_tiny + CB_NT / 64 - 1) / (CB_NT / 64) : 0;
    const int piece_lds = TR ? int(tiny_lds_budget() / int64_t(sizeof(T))) : 0;
    size_t lds = size_t(a.cblock_lds) * sizeof(T);
    if (fuse) lds = std::max(lds, size_t(piece_lds) * sizeof(T) * size_t(CB_NT / 64));
    for (int64_t off = 0; off < n; off += max_grid) {
        const int64_t m = std::min(max_grid, n - off);
        const int64_t extra = off + m >= n ? pb : 0;  // the pieces ride on the last launch
        hipLaunchKernelGGL((cblock_kernel<T, TR, AX>), dim3(unsigned(m + extra)), dim3(CB_NT), lds, stream, a.ops,
                           work + off, a.src_base, a.dst_base, static_cast<const T*>(a.scalars), a.cb_map,
                           chunk, m, a.ops + a.tiny_first, extra ? a.n_tiny : int64_t(0), piece_lds);
    }
}
template <typename T>
void launch_cblock(const launch_args& a, const uint64_t* work, int64_t n, bool fuse, hipStream_t stream) {
    if (n <= 0) return;
    if constexpr (is_cpx<T>::value) {  // real types only (engine.cpp cblock_groups)
        throw error(COSTA_ERR_INTERNAL, "costa: destination-block groups of a complex type");
    } else if (a.any_transpose)
        a.any_axpby ? launch_cblock_v<T, true, true>(a, work, n, fuse, stream)
                    : launch_cblock_v<T, true, false>(a, work, n, fuse, stream);
    else
        a.any_axpby ? launch_cblock_v<T, false, true>(a, work, n, fuse, stream)
                    : launch_cblock_v<T, false, false>(a, work, n, fuse, stream);
}

// One op per wavefront.  Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md,
// workgroup dispatch); they are renumbered so that each XCD walks one contiguous slice of the
// locality-ordered list, and neighbouring ops (which share partially written cache lines) meet
// in one L2 (r11: cfg 5 'N' 3.77 against 3.58 TB/s, 'T' 3.07 against 3.00;
// profiles/r11/c5_order.log).  Placement only changes speed, never results.
// Real types: 8 wavefronts per SIMD.  The transposing, beta-reading variant needed 66 VGPRs,
// one over the 8-wave budget, so 7 fitted (cfg 5 'T' 0.790 -> 0.774 ms with the bound, no
// spills; profiles/r2/w8ab/).  Complex types would spill under it (tests/test_kernel_resources.py).
template <typename T> struct tiny_min_waves { static constexpr int value = 8; };
template <typename R> struct tiny_min_waves<cpx<R>> { static constexpr int value = 1; };
template <typename T, int W, bool TR, bool AX, int UC>
__global__ __launch_bounds__(64 * W, tiny_min_waves<T>::value) void tiny_kernel(const costa_tile_op_t* __restrict__ ops,
                                                      int64_t n_ops, const char* src_base,
                                                      char* dst_base, const T* __restrict__ scalars,
                                                      int lds_per_wave) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = int(threadIdx.x) % 64;
    const int wave = __builtin_amdgcn_readfirstlane(int(threadIdx.x) / 64);
    const int64_t b = xcd_slice_order(int64_t(blockIdx.x), int64_t(gridDim.x));
    const int64_t w = b * W + wave;
    if (w >= n_ops) return;
    T* t = reinterpret_cast<T*>(smem) + int64_t(wave) * lds_per_wave;
    tiny_op<T, TR, AX, UC>(ops[w], lane, t, src_base, dst_base, scalars);
}

template <typename T, int W, bool TR, bool AX>
void launch_tiny_v(const launch_args& a, hipStream_t stream) {
    constexpr int UC = tiny_copy_bytes<T>();
    const int64_t n = a.n_tiny;
    const int per_wave = TR ? int(tiny_lds_budget() / int64_t(sizeof(T))) : 0;
    const size_t lds = size_t(per_wave) * sizeof(T) * W;
    const int64_t blocks = (n + W - 1) / W;
    if (blocks >= (int64_t(1) << 31)) throw error(COSTA_ERR_ARG, "costa: tile list too long");
    hipLaunchKernelGGL((tiny_kernel<T, W, TR, AX, UC>), dim3(unsigned(blocks)),
                       dim3(64 * W), lds, stream, a.ops + a.tiny_first, n, a.src_base, a.dst_base,
                       static_cast<const T*>(a.scalars), per_wave);
}

template <typename T>
void launch_tiny(const launch_args& a, hipStream_t stream) {
    if (a.n_tiny <= 0) return;
    // transposing lists: TINY_WAVES_TR wavefronts per workgroup; copy-only: TINY_WAVES_COPY
    if (a.any_transpose)
        return a.any_axpby ? launch_tiny_v<T, TINY_WAVES_TR, true, true>(a, stream)
                           : launch_tiny_v<T, TINY_WAVES_TR, true, false>(a, stream);
    a.any_axpby ? launch_tiny_v<T, TINY_WAVES_COPY, false, true>(a, stream)
                : launch_tiny_v<T, TINY_WAVES_COPY, false, false>(a, stream);
}

template <typename T, typename S>
void launch_shape(const launch_args& a, const uint64_t* work, int64_t n, hipStream_t stream) {
    const int64_t max_grid = 1LL << 30;
    for (int64_t off = 0; off < n; off += max_grid) {
        const int64_t m = std::min(max_grid, n - off);
        // copy-only lists need no LDS tile: more workgroups per CU
        const size_t lds = a.any_transpose ? S::lds_bytes : 0;
        hipLaunchKernelGGL((tile_kernel<T, S>), dim3(unsigned(m)), dim3(S::NT), lds, stream,
                           a.ops, work + off, a.src_base, a.dst_base,
                           static_cast<const T*>(a.scalars));
    }
}
template <typename T>
void launch_t(const launch_args& a, hipStream_t stream) {
    // work list: the large shape's sub-tiles (the list's shape: build_work cut them with
    // tile_shapes(dtype, tr_shape)), then the wavefront ops
    if (a.sq) {
        if (!shapes<T>::has_small || !a.tr_shape) throw error(COSTA_ERR_INTERNAL, "costa: square shape");
        launch_shape<T, typename shapes<T>::small_tr>(a, a.work, a.n_large, stream);
    } else if (a.tr_shape && a.full)
        launch_shape<T, typename shapes<T>::large_tr_full>(a, a.work, a.n_large, stream);
    else if (a.tr_shape)
        launch_shape<T, typename shapes<T>::large_tr>(a, a.work, a.n_large, stream);
    else
        launch_shape<T, typename shapes<T>::large>(a, a.work, a.n_large, stream);
    if (a.n_medium > 0 && a.med_sq) {  // the medium class on 32 x 32 sub-tiles (nb = 32 blocks)
        if (!a.tr_shape) throw error(COSTA_ERR_INTERNAL, "costa: 32 x 32 shape");
        launch_shape<T, typename shapes<T>::small32_tr>(a, a.work + a.n_large, a.n_medium, stream);
    } else if (a.n_medium > 0) {
        if (!shapes<T>::has_medium || !a.tr_shape) throw error(COSTA_ERR_INTERNAL, "costa: medium shape");
        if (a.med_full && !a.any_axpby)  // every medium op a whole number of sub-tiles, C not read
            launch_shape<T, typename shapes<T>::medium_tr_full>(a, a.work + a.n_large, a.n_medium, stream);
        else
            launch_shape<T, typename shapes<T>::medium_tr>(a, a.work + a.n_large, a.n_medium, stream);
    }
    if (a.n_skew > 0) launch_skew<T>(a, a.work + a.n_large + a.n_medium, a.n_skew, stream);
    // the wavefront pieces ride in the group launch's tail when there is one (COSTA_FUSE_PIECES=0,
    // tuning: a launch of their own)
    const bool fuse = !is_cpx<T>::value && pieces_in_group_launch(a.n_cblock, a.n_tiny);
    launch_cblock<T>(a, a.work + a.n_large + a.n_medium + a.n_skew, a.n_cblock, fuse, stream);
    if (!fuse) launch_tiny<T>(a, stream);
}

template <typename T>
void shape_of(bool tr, shape_dims* d) {
    d->bf = tr ? shapes<T>::large_tr::BF : shapes<T>::large::BF;
    d->bs = tr ? shapes<T>::large_tr::BS : shapes<T>::large::BS;
    d->cf = tr ? shapes<T>::large_tr::BF : copy_class<T>::BF;
    d->cs = tr ? shapes<T>::large_tr::BS : copy_class<T>::BS;
    const bool med = tr && shapes<T>::has_medium;
    d->bf_m = med ? shapes<T>::medium_tr::BF : 0;
    d->bs_m = med ? shapes<T>::medium_tr::BS : 0;
    const bool sq = tr && shapes<T>::has_small;
    d->bf_q = sq ? shapes<T>::small_tr::BF : 0;
    d->bs_q = sq ? shapes<T>::small_tr::BS : 0;
    d->bf_s = tr ? shapes<T>::small32_tr::BF : 0;
    d->bs_s = tr ? shapes<T>::small32_tr::BS : 0;
    constexpr bool skew = std::is_same<T, float>::value || std::is_same<T, double>::value ||
                          std::is_same<T, int>::value;
    d->bf_k = tr && skew ? skew_shape<T>::BF : 0;
    d->bs_k = tr && skew ? skew_shape<T>::BS : 0;
    d->bf_kw = tr && skew ? skew_shape<T, true>::BF : 0;
    d->bs_kw = tr && skew ? skew_shape<T, true>::BS : 0;
}

template <typename T, typename S>
void set_lds_limit() {
    // the large shapes need more than the default dynamic-LDS limit
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&tile_kernel<T, S>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(S::lds_bytes));
}
template <typename T>
void set_lds_limits() {
    if constexpr (std::is_same<T, float>::value || std::is_same<T, double>::value ||
                  std::is_same<T, int>::value)
    {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&skew_kernel<T, false>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  int(skew_shape<T, false>::lds_bytes));
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&skew_kernel<T, true>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  int(skew_shape<T, true>::lds_bytes));
    }
    if constexpr (!is_cpx<T>::value)
        for (void* f : {reinterpret_cast<void*>(&cblock_kernel<T, true, true>),
                        reinterpret_cast<void*>(&cblock_kernel<T, true, false>),
                        reinterpret_cast<void*>(&cblock_kernel<T, false, true>),
                        reinterpret_cast<void*>(&cblock_kernel<T, false, false>)})
            (void)hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      int((cblock_max_elems(int64_t(sizeof(T))) + 4096) * int64_t(sizeof(T))));
    set_lds_limit<T, typename shapes<T>::large>();
    set_lds_limit<T, typename shapes<T>::large_tr>();
    set_lds_limit<T, typename shapes<T>::medium_tr>();
    set_lds_limit<T, typename shapes<T>::small_tr>();
    set_lds_limit<T, typename shapes<T>::large_tr_full>();
    set_lds_limit<T, typename shapes<T>::medium_tr_full>();
    set_lds_limit<T, typename shapes<T>::small32_tr>();
}

}  // namespace

bool pieces_in_group_launch(int64_t n_cblock, int64_t n_tiny) {
    static const bool on = [] {  // COSTA_FUSE_PIECES=0 (tuning): a launch of their own
        const char* v = tuning_env("COSTA_FUSE_PIECES");
        return !v || std::atoi(v) != 0;
    }();
    return on && n_cblock > 0 && n_tiny > 0 && n_cblock + n_tiny / (CB_NT / 64) + 1 < (int64_t(1) << 30);
}

void tile_shapes(costa_dtype_t dtype, bool transposing_list, shape_dims* d) {
    const bool t = transposing_list;
    switch (dtype) {
    case COSTA_FLOAT: shape_of<float>(t, d); return;
    case COSTA_DOUBLE: shape_of<double>(t, d); return;
    case COSTA_CFLOAT: shape_of<cpx<float>>(t, d); return;
    case COSTA_CDOUBLE: shape_of<cpx<double>>(t, d); return;
    case COSTA_INT32: shape_of<int>(t, d); return;
    }
    throw error(COSTA_ERR_ARG, "unknown dtype");
}

void launch_tiles(costa_dtype_t dtype, const launch_args& a, void* stream) {
    if (a.n_large + a.n_medium + a.n_skew + a.n_cblock + a.n_tiny <= 0) return;
    static bool once = [] {
        set_lds_limits<float>();
        set_lds_limits<double>();
        set_lds_limits<cpx<float>>();
        set_lds_limits<cpx<double>>();
        set_lds_limits<int>();
        return true;
    }();
    (void)once;
    hipStream_t s = static_cast<hipStream_t>(stream);
    switch (dtype) {
    case COSTA_FLOAT: launch_t<float>(a, s); break;
    case COSTA_DOUBLE: launch_t<double>(a, s); break;
    case COSTA_CFLOAT: launch_t<cpx<float>>(a, s); break;
    case COSTA_CDOUBLE: launch_t<cpx<double>>(a, s); break;
    case COSTA_INT32: launch_t<int>(a, s); break;
    }
    hipError_t e = hipGetLastError();
    if (e != hipSuccess)
        throw error(COSTA_ERR_HIP, std::string("tile kernel launch failed: ") + hipGetErrorString(e));
}

}  // namespace engine
}  // namespace costa
