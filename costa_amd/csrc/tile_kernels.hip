// Batched tile kernels for CDNA4 (gfx950): one launch runs a whole list of tile ops
// (pack, local or unpack), one 256-thread workgroup per sub-tile.
//
// What each op computes is the reference's copy_and_transform
// (eth-cscs/COSTA src/costa/grid2grid/memory_utils.hpp:339-412):
//   copy mode       dst(f, s) = g(src(f, s))            copy2D / copy         :20-98
//   transpose mode  dst(s, f) = g(src(f, s))            transpose_{col,row}_major :101-291
//   g(x) = x | 0 | alpha*op(x) | beta*dst + alpha*op(x) (op = conj for 'C' on complex)
// evaluated in the same order as the reference with contraction OFF, so results are
// bit-identical to the x86 build (which has no FMA: SURVEY §8c).
//
// Memory path: the transpose stages each BF x BS sub-tile through LDS. Global loads are
// 16-byte vectors along the source's contiguous dimension, global stores are whole
// wavefront rows along the destination's contiguous dimension.  No MFMA: the op is
// purely HBM-bound (<= 0.5 flop/byte).
#include <hip/hip_runtime.h>

#include "engine.hpp"

#pragma clang fp contract(off)

namespace costa {
namespace engine {
namespace {

constexpr int NT = 256;  // threads per workgroup = 4 wavefronts

template <typename R>
struct cpx {
    R re, im;
};

// ---- element arithmetic, written out so the rounding sequence is explicit ----
template <typename T> __device__ __forceinline__ T e_mul(T a, T b) { return a * b; }
template <typename T> __device__ __forceinline__ T e_add(T a, T b) { return a + b; }
template <typename T> __device__ __forceinline__ T e_conj(T a) { return a; }
template <typename T> __device__ __forceinline__ T e_zero() { return T(0); }

// (a.re + i a.im)(b.re + i b.im) = (a.re b.re - a.im b.im) + i (a.re b.im + a.im b.re):
// libstdc++/GCC's complex product for finite operands (4 products, 2 sums, no fma)
template <> __device__ __forceinline__ cpx<float> e_mul(cpx<float> a, cpx<float> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
template <> __device__ __forceinline__ cpx<double> e_mul(cpx<double> a, cpx<double> b) {
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
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

// sub-tile shape: BF elements along the source's contiguous dim (one 512-byte strip per
// 32 lanes), BS = 64 along the strided dim; V elements per 16-byte vector
template <typename T>
struct shape {
    static constexpr int V = 16 / sizeof(T);
    static constexpr int BF = 32 * V;
    static constexpr int BS = 64;
};

struct __attribute__((aligned(16))) vec16 {
    uint32_t w[4];
};

template <typename T>
union pack16 {
    vec16 v;
    T e[shape<T>::V];
};

template <typename T>
__device__ __forceinline__ void load_strip(const T* p, int n, bool vec, pack16<T>& out) {
    constexpr int V = shape<T>::V;
    if (vec && n == V) {
        out.v = *reinterpret_cast<const vec16*>(p);
    } else {
#pragma unroll
        for (int k = 0; k < V; ++k)
            if (k < n) out.e[k] = p[k];
    }
}

template <typename T>
__device__ __forceinline__ void store_strip(T* p, int n, bool vec, const pack16<T>& in) {
    constexpr int V = shape<T>::V;
    if (vec && n == V) {
        *reinterpret_cast<vec16*>(p) = in.v;
    } else {
#pragma unroll
        for (int k = 0; k < V; ++k)
            if (k < n) p[k] = in.e[k];
    }
}

// ---- copy mode: dst(f, s) = g(src(f, s)); no LDS ----
template <typename T>
__device__ __forceinline__ void copy_tile(const T* __restrict__ src, T* __restrict__ dst, int tf,
                                          int ts, int64_t lds, int64_t ldd, uint32_t flags,
                                          T alpha, T beta) {
    constexpr int V = shape<T>::V;
    constexpr int LPC = shape<T>::BF / V;  // lanes per column (32)
    constexpr int CPP = NT / LPC;          // columns per pass (8)
    const int lane_f = (threadIdx.x % LPC) * V;
    const int col0 = threadIdx.x / LPC;
    const uint32_t kind = (flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
    const bool conj = flags & COSTA_TILE_CONJ;
    const bool vs = flags & COSTA_TILE_VEC_SRC, vd = flags & COSTA_TILE_VEC_DST;
    const int n = min(V, tf - lane_f);
    if (n <= 0) return;
    constexpr int P = shape<T>::BS / CPP;  // passes
    pack16<T> x[P];
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int s = col0 + k * CPP;
        if (s < ts) load_strip(src + s * lds + lane_f, n, vs, x[k]);
    }
#pragma unroll
    for (int k = 0; k < P; ++k) {
        const int s = col0 + k * CPP;
        if (s >= ts) continue;
        T* d = dst + s * ldd + lane_f;
        if (kind != COSTA_SCALE_BITCOPY) {
            pack16<T> y;
            if (kind == COSTA_SCALE_AXPBY) load_strip(d, n, vd, y);
#pragma unroll
            for (int e = 0; e < V; ++e) x[k].e[e] = scale(x[k].e[e], y.e[e], kind, conj, alpha, beta);
        }
        store_strip(d, n, vd, x[k]);
    }
}

// ---- transpose mode: dst(s, f) = g(src(f, s)), staged through LDS ----
template <typename T>
__device__ __forceinline__ void transpose_tile(const T* __restrict__ src, T* __restrict__ dst,
                                               int tf, int ts, int64_t lds, int64_t ldd,
                                               uint32_t flags, T alpha, T beta, T* tile) {
    constexpr int V = shape<T>::V;
    constexpr int BF = shape<T>::BF;
    constexpr int BS = shape<T>::BS;
    constexpr int PITCH = BF + 1;          // +1 element: conflict-free column reads
    constexpr int LPC = BF / V;            // lanes per source column (32)
    constexpr int CPP = NT / LPC;          // source columns per pass (8)
    constexpr int P = BS / CPP;            // load passes (8)
    const uint32_t kind = (flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
    const bool conj = flags & COSTA_TILE_CONJ;
    const bool vs = flags & COSTA_TILE_VEC_SRC;

    // load: 16-byte strips along f, all loads issued before any LDS write
    {
        const int lane_f = (threadIdx.x % LPC) * V;
        const int col0 = threadIdx.x / LPC;
        const int n = min(V, tf - lane_f);
        pack16<T> x[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const int s = col0 + k * CPP;
            if (n > 0 && s < ts) load_strip(src + s * lds + lane_f, n, vs, x[k]);
        }
#pragma unroll
        for (int k = 0; k < P; ++k) {
            const int s = col0 + k * CPP;
            if (n > 0 && s < ts) {
#pragma unroll
                for (int e = 0; e < V; ++e)
                    if (e < n) tile[s * PITCH + lane_f + e] = x[k].e[e];
            }
        }
    }
    __syncthreads();
    // store: destination row f is contiguous along s; one wavefront row per f
    {
        const int lane = threadIdx.x % 64;  // s within the row
        const int wave = threadIdx.x / 64;
        if (lane < ts) {
            for (int f = wave; f < tf; f += NT / 64) {
                T v = tile[lane * PITCH + f];
                T* d = dst + f * ldd + lane;
                T y = e_zero<T>();
                if (kind == COSTA_SCALE_AXPBY) y = *d;
                *d = scale(v, y, kind, conj, alpha, beta);
            }
        }
    }
}

template <typename T>
__global__ __launch_bounds__(NT) void tile_kernel(const costa_tile_op_t* __restrict__ ops,
                                                  const uint64_t* __restrict__ work,
                                                  const char* src_base, char* dst_base,
                                                  const T* __restrict__ scalars) {
    constexpr int BF = shape<T>::BF;
    constexpr int BS = shape<T>::BS;
    __shared__ T tile[BS * (BF + 1)];

    const uint64_t w = work[blockIdx.x];
    const costa_tile_op_t op = ops[w >> 32];
    const uint32_t sub = uint32_t(w);
    const int nbf = (op.nf + BF - 1) / BF;
    const int f0 = int(sub % uint32_t(nbf)) * BF;
    const int s0 = int(sub / uint32_t(nbf)) * BS;
    const int tf = min(BF, op.nf - f0);
    const int ts = min(BS, op.ns - s0);
    const uint32_t slot = op.flags >> COSTA_SLOT_SHIFT;
    const T alpha = scalars[2 * slot];
    const T beta = scalars[2 * slot + 1];
    const T* src = reinterpret_cast<const T*>(src_base + op.src) + int64_t(s0) * op.lds + f0;
    if (op.flags & COSTA_TILE_TRANSPOSE) {
        T* dst = reinterpret_cast<T*>(dst_base + op.dst) + int64_t(f0) * op.ldd + s0;
        transpose_tile<T>(src, dst, tf, ts, op.lds, op.ldd, op.flags, alpha, beta, tile);
    } else {
        T* dst = reinterpret_cast<T*>(dst_base + op.dst) + int64_t(s0) * op.ldd + f0;
        copy_tile<T>(src, dst, tf, ts, op.lds, op.ldd, op.flags, alpha, beta);
    }
}

template <typename T>
void launch_t(const launch_args& a, hipStream_t stream) {
    const int64_t max_grid = 1LL << 30;
    for (int64_t off = 0; off < a.n_work; off += max_grid) {
        const int64_t n = std::min(max_grid, a.n_work - off);
        hipLaunchKernelGGL(tile_kernel<T>, dim3(unsigned(n)), dim3(NT), 0, stream, a.ops,
                           a.work + off, a.src_base, a.dst_base,
                           static_cast<const T*>(a.scalars));
    }
}

}  // namespace

void tile_shape(costa_dtype_t dtype, int* bf, int* bs) {
    switch (dtype) {
    case COSTA_FLOAT: *bf = shape<float>::BF; *bs = shape<float>::BS; return;
    case COSTA_DOUBLE: *bf = shape<double>::BF; *bs = shape<double>::BS; return;
    case COSTA_CFLOAT: *bf = shape<cpx<float>>::BF; *bs = shape<cpx<float>>::BS; return;
    case COSTA_CDOUBLE: *bf = shape<cpx<double>>::BF; *bs = shape<cpx<double>>::BS; return;
    case COSTA_INT32: *bf = shape<int>::BF; *bs = shape<int>::BS; return;
    }
    throw error(COSTA_ERR_ARG, "unknown dtype");
}

void launch_tiles(costa_dtype_t dtype, const launch_args& a, void* stream) {
    if (a.n_work <= 0) return;
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
