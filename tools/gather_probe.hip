// Tuning probe (not part of the product): cfg 5's bytes moved DESTINATION-BLOCK-WISE.
// The product's wavefront path gives each A∩C piece to one wave, so both the read and the write
// stream are ~130-byte column runs (a 128-B-segment copy peaks at 4.8-4.9 TB/s).
// Here one 256-thread workgroup owns a strip of whole columns of one C block (contiguous in
// memory: every block is its own column-major buffer with ld = rows, as in bench.py's cfg 5):
//   phase 1: its waves copy every A piece of the strip into an LDS image of the strip
//            ('T': transposed on the way in, odd LDS pitch);
//   phase 2: the workgroup streams the image out as one contiguous run ('T': C read, beta*C +
//            alpha*image, written back).
// Geometry: fp32 16384^2, A edges uniform 8-96, C edges 16-160 (mt19937_64, not bench's PCG64
// streams: the same distributions), every block owned. Verified on a 1M-element sample.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 tools/gather_probe.hip -o /tmp/gp && /tmp/gp [reps]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <cstring>
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

struct strip_t {
    uint64_t c_off;  // float index of the strip's first element in the C arena
    int h, k;        // rows (= ld) and columns of the strip
    int pitch;       // LDS pitch of the image (floats)
    int p0, p1;      // pieces [p0, p1)
};
struct piece_t {
    uint64_t a_off;       // float index of the piece's first element in the A arena
    int lda, nf, ns;      // A leading dim; run length (A rows) and runs (A cols)
    int img, fstep, sstep;  // image offset of (f, s) = img + f * fstep + s * sstep
};

template <bool NT>
__device__ __forceinline__ float ldg(const float* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    else return *p;
}
template <bool NT>
__device__ __forceinline__ void stg(float* p, float v) {
    if constexpr (NT) __builtin_nontemporal_store(v, p);
    else *p = v;
}

// U: elements per thread in flight per batch
template <bool TR, bool NT, int U>
__global__ __launch_bounds__(256) void k_gather(const strip_t* strips, const piece_t* pieces, const float* A,
                                                float* C, float alpha, float beta) {
    extern __shared__ float img[];
    const strip_t st = strips[blockIdx.x];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int p = st.p0 + wave; p < st.p1; p += 4) {
        const piece_t q = pieces[p];
        const int total = q.nf * q.ns;
        // element e = lane + 64 t: f = e % nf, s = e / nf, advanced incrementally
        int f = lane % q.nf, s = lane / q.nf;
        const int df = 64 % q.nf, ds = 64 / q.nf;
        for (int e0 = 0; e0 < total; e0 += 64 * U) {
            float v[U];
            int o[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const bool in = e0 + u * 64 + lane < total;
                v[u] = in ? ldg<NT>(A + q.a_off + uint64_t(s) * q.lda + f) : 0.f;
                o[u] = in ? q.img + f * q.fstep + s * q.sstep : -1;
                f += df;
                s += ds;
                if (f >= q.nf) {
                    f -= q.nf;
                    ++s;
                }
            }
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (o[u] >= 0) img[o[u]] = v[u];
        }
    }
    __syncthreads();
    const int total = st.h * st.k;
    float* c = C + st.c_off;
    int r = threadIdx.x % st.h, col = threadIdx.x / st.h;
    const int dr = 256 % st.h, dc = 256 / st.h;
    for (int e0 = 0; e0 < total; e0 += 256 * U) {
        float v[U], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = e0 + u * 256 + threadIdx.x;
            v[u] = e < total ? img[col * st.pitch + r] : 0.f;
            if constexpr (TR) w[u] = e < total ? ldg<NT>(c + e) : 0.f;
            r += dr;
            col += dc;
            if (r >= st.h) {
                r -= st.h;
                ++col;
            }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int e = e0 + u * 256 + threadIdx.x;
            if (e < total) stg<NT>(c + e, TR ? beta * w[u] + alpha * v[u] : v[u]);
        }
    }
}

static std::vector<int> splits(uint64_t seed, int lo, int hi, int n) {
    std::mt19937_64 g(seed);
    std::uniform_int_distribution<int> d(lo, hi);
    std::vector<int> s{0};
    while (s.back() < n) s.push_back(std::min(n, s.back() + d(g)));
    return s;
}

struct arena_t {
    std::vector<int> rs, cs;
    std::vector<uint64_t> off;  // per block, row-major over (i, j)
    uint64_t size = 0;
    int nbr() const { return int(rs.size()) - 1; }
    int nbc() const { return int(cs.size()) - 1; }
    int h(int i) const { return rs[size_t(i) + 1] - rs[size_t(i)]; }
    int w(int j) const { return cs[size_t(j) + 1] - cs[size_t(j)]; }
    uint64_t at(int gi, int gj) const {  // float index of global (gi, gj)
        const int i = int(std::upper_bound(rs.begin(), rs.end(), gi) - rs.begin()) - 1;
        const int j = int(std::upper_bound(cs.begin(), cs.end(), gj) - cs.begin()) - 1;
        return off[size_t(i) * nbc() + j] + uint64_t(gj - cs[size_t(j)]) * h(i) + (gi - rs[size_t(i)]);
    }
};

static arena_t arena(std::vector<int> rs, std::vector<int> cs) {
    arena_t a;
    a.rs = std::move(rs);
    a.cs = std::move(cs);
    for (int i = 0; i < a.nbr(); ++i)
        for (int j = 0; j < a.nbc(); ++j) {
            a.off.push_back(a.size);
            a.size += (uint64_t(a.h(i)) * a.w(j) + 63) / 64 * 64;
        }
    return a;
}

// strips of <= max_floats per C block (whole columns), and their A pieces
static void build(const arena_t& A, const arena_t& C, bool tr, int max_floats, std::vector<strip_t>& S,
                  std::vector<piece_t>& P) {
    S.clear();
    P.clear();
    for (int bj = 0; bj < C.nbc(); ++bj)
        for (int bi = 0; bi < C.nbr(); ++bi) {  // blocks column-major (the planner's hint order)
            const int h = C.h(bi), w = C.w(bj), r0 = C.rs[size_t(bi)];
            const int kmax = std::max(1, max_floats / (tr ? (h | 1) : h));
            for (int c0 = 0; c0 < w; c0 += kmax) {
                strip_t s;
                s.h = h;
                s.k = std::min(kmax, w - c0);
                s.pitch = tr ? (h | 1) : h;
                s.c_off = C.off[size_t(bi) * C.nbc() + bj] + uint64_t(c0) * h;
                s.p0 = int(P.size());
                const int gc0 = C.cs[size_t(bj)] + c0, gc1 = gc0 + s.k;  // global C cols
                // the A region: 'N' rows [r0, r0+h) x cols [gc0, gc1); 'T' rows [gc0, gc1) x cols [r0, r0+h)
                const int ar0 = tr ? gc0 : r0, ar1 = tr ? gc1 : r0 + h;
                const int ac0 = tr ? r0 : gc0, ac1 = tr ? r0 + h : gc1;
                const int ai0 = int(std::upper_bound(A.rs.begin(), A.rs.end(), ar0) - A.rs.begin()) - 1;
                const int aj0 = int(std::upper_bound(A.cs.begin(), A.cs.end(), ac0) - A.cs.begin()) - 1;
                for (int aj = aj0; aj < A.nbc() && A.cs[size_t(aj)] < ac1; ++aj)
                    for (int ai = ai0; ai < A.nbr() && A.rs[size_t(ai)] < ar1; ++ai) {
                        const int x0 = std::max(ar0, A.rs[size_t(ai)]), x1 = std::min(ar1, A.rs[size_t(ai) + 1]);
                        const int y0 = std::max(ac0, A.cs[size_t(aj)]), y1 = std::min(ac1, A.cs[size_t(aj) + 1]);
                        piece_t q;
                        q.lda = A.h(ai);
                        q.a_off = A.off[size_t(ai) * A.nbc() + aj] + uint64_t(y0 - A.cs[size_t(aj)]) * q.lda +
                                  (x0 - A.rs[size_t(ai)]);
                        q.nf = x1 - x0;
                        q.ns = y1 - y0;
                        if (!tr) {  // A (x, y) -> C (x, y): image (y - gc0) * pitch + (x - r0)
                            q.img = (y0 - gc0) * s.pitch + (x0 - r0);
                            q.fstep = 1;
                            q.sstep = s.pitch;
                        } else {  // A (x, y) -> C (y, x): image (x - gc0) * pitch + (y - r0)
                            q.img = (x0 - gc0) * s.pitch + (y0 - r0);
                            q.fstep = s.pitch;
                            q.sstep = 1;
                        }
                        P.push_back(q);
                    }
                s.p1 = int(P.size());
                S.push_back(s);
            }
        }
}


// ---- band tables: the strip's A region (rows [ar0, ar1) x cols [ac0, ac1) of A) cut by A's
// block rows into x-bands and by A's block columns into y-bands; region element (x, y) lives at
// pb[i * ny + j] + y * lda[i] + x for its bands (i, j).  'N': x = strip row, y = strip column
// (the strip is written as it is read: no image); 'T': x = strip column, y = strip row, through
// the LDS image.
struct bstrip_t {
    uint64_t c_off;
    int h, k, pitch;
    int nx, ny;          // region extent (x, y)
    int nbx, nby;        // band counts
    int tab;             // int offset of this strip's tables in the blob
};
// blob per strip: xband[nx] (uint8), yband[ny] (uint8) packed 4 per int; lda[nbx]; pb[nbx*nby] (int64 as 2 ints)

template <bool TR, bool NT>
__global__ __launch_bounds__(256) void k_band(const bstrip_t* strips, const int* blob, const float* A, float* C,
                                              float alpha, float beta) {
    extern __shared__ int lds[];
    const bstrip_t st = strips[blockIdx.x];
    const int nxw = (st.nx + 3) / 4, nyw = (st.ny + 3) / 4;
    const int pbo = (nxw + nyw + st.nbx + 1) & ~1;  // int64s 8-B aligned
    const int nint = pbo + 2 * st.nbx * st.nby;
    for (int t = threadIdx.x; t < nint; t += 256) lds[t] = blob[st.tab + t];
    const unsigned char* xb = reinterpret_cast<const unsigned char*>(lds);
    const unsigned char* yb = reinterpret_cast<const unsigned char*>(lds + nxw);
    const int* lda = lds + nxw + nyw;
    const long long* pb = reinterpret_cast<const long long*>(lds + pbo);
    float* img = reinterpret_cast<float*>(lds + ((nint + 3) & ~3));
    __syncthreads();
    float* c = C + st.c_off;
    const int total = st.h * st.k;
    if constexpr (!TR) {
        // contiguous output: thread t owns elements t, t+256, ...; x = e % h, y = e / h
        int x = threadIdx.x % st.h, y = threadIdx.x / st.h;
        const int dx = 256 % st.h, dy = 256 / st.h;
        for (int e0 = 0; e0 < total; e0 += 256 * 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * 256 + threadIdx.x;
                if (e < total) {
                    const int i = xb[x], j = yb[y];
                    v[u] = ldg<NT>(A + pb[i * st.nby + j] + (long long)y * lda[i] + x);
                }
                x += dx;
                y += dy;
                if (x >= st.h) { x -= st.h; ++y; }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * 256 + threadIdx.x;
                if (e < total) stg<NT>(c + e, v[u]);
            }
        }
    } else {
        // phase 1: region order (x fastest: A columns), x = strip column, y = strip row
        const int nx = st.nx;
        int x = threadIdx.x % nx, y = threadIdx.x / nx;
        const int dx = 256 % nx, dy = 256 / nx;
        for (int e0 = 0; e0 < total; e0 += 256 * 8) {
            float v[8];
            int o[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * 256 + threadIdx.x;
                o[u] = -1;
                if (e < total) {
                    const int i = xb[x], j = yb[y];
                    v[u] = ldg<NT>(A + pb[i * st.nby + j] + (long long)y * lda[i] + x);
                    o[u] = x * st.pitch + y;
                }
                x += dx;
                y += dy;
                if (x >= nx) { x -= nx; ++y; }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u)
                if (o[u] >= 0) img[o[u]] = v[u];
        }
        __syncthreads();
        int r = threadIdx.x % st.h, col = threadIdx.x / st.h;
        const int dr = 256 % st.h, dc = 256 / st.h;
        for (int e0 = 0; e0 < total; e0 += 256 * 8) {
            float v[8], w[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * 256 + threadIdx.x;
                v[u] = e < total ? img[col * st.pitch + r] : 0.f;
                w[u] = e < total ? ldg<NT>(c + e) : 0.f;
                r += dr;
                col += dc;
                if (r >= st.h) { r -= st.h; ++col; }
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * 256 + threadIdx.x;
                if (e < total) stg<NT>(c + e, beta * w[u] + alpha * v[u]);
            }
        }
    }
}

static void build_band(const arena_t& A, const arena_t& C, bool tr, int max_floats, std::vector<bstrip_t>& S,
                       std::vector<int>& blob, int& lds_max) {
    S.clear();
    blob.clear();
    lds_max = 0;
    for (int bj = 0; bj < C.nbc(); ++bj)
        for (int bi = 0; bi < C.nbr(); ++bi) {
            const int h = C.h(bi), w = C.w(bj), r0 = C.rs[size_t(bi)];
            const int pitch = tr ? (h | 1) : h;
            const int kmax = std::max(1, max_floats / pitch);
            for (int c0 = 0; c0 < w; c0 += kmax) {
                bstrip_t s;
                s.h = h;
                s.k = std::min(kmax, w - c0);
                s.pitch = pitch;
                s.c_off = C.off[size_t(bi) * C.nbc() + bj] + uint64_t(c0) * h;
                const int gc0 = C.cs[size_t(bj)] + c0, gc1 = gc0 + s.k;
                const int ar0 = tr ? gc0 : r0, ar1 = tr ? gc1 : r0 + h;
                const int ac0 = tr ? r0 : gc0, ac1 = tr ? r0 + h : gc1;
                s.nx = ar1 - ar0;
                s.ny = ac1 - ac0;
                const int ai0 = int(std::upper_bound(A.rs.begin(), A.rs.end(), ar0) - A.rs.begin()) - 1;
                const int aj0 = int(std::upper_bound(A.cs.begin(), A.cs.end(), ac0) - A.cs.begin()) - 1;
                std::vector<int> xs, ys;  // band starts (region coordinates)
                int ai1 = ai0, aj1 = aj0;
                while (ai1 < A.nbr() && A.rs[size_t(ai1)] < ar1) ++ai1;
                while (aj1 < A.nbc() && A.cs[size_t(aj1)] < ac1) ++aj1;
                s.nbx = ai1 - ai0;
                s.nby = aj1 - aj0;
                s.tab = int(blob.size());
                std::vector<unsigned char> xb(size_t((s.nx + 3) / 4 * 4)), yb(size_t((s.ny + 3) / 4 * 4));
                for (int x = 0; x < s.nx; ++x)
                    xb[size_t(x)] = (unsigned char)(int(std::upper_bound(A.rs.begin(), A.rs.end(), ar0 + x) - A.rs.begin()) - 1 - ai0);
                for (int y = 0; y < s.ny; ++y)
                    yb[size_t(y)] = (unsigned char)(int(std::upper_bound(A.cs.begin(), A.cs.end(), ac0 + y) - A.cs.begin()) - 1 - aj0);
                const size_t base = blob.size();
                blob.resize(base + xb.size() / 4 + yb.size() / 4);
                std::memcpy(&blob[base], xb.data(), xb.size());
                std::memcpy(&blob[base + xb.size() / 4], yb.data(), yb.size());
                for (int i = 0; i < s.nbx; ++i) blob.push_back(A.h(ai0 + i));
                if ((blob.size() - size_t(s.tab)) % 2) blob.push_back(0);
                for (int i = 0; i < s.nbx; ++i)
                    for (int j = 0; j < s.nby; ++j) {
                        const int ai = ai0 + i, aj = aj0 + j;
                        // region (x, y) -> A.off + (ac0 + y - cs[aj]) * lda + (ar0 + x - rs[ai])
                        const long long lda = A.h(ai);
                        const long long pb = (long long)A.off[size_t(ai) * A.nbc() + aj] +
                                             (long long)(ac0 - A.cs[size_t(aj)]) * lda + (ar0 - A.rs[size_t(ai)]);
                        blob.push_back(int(pb & 0xffffffff));
                        blob.push_back(int(pb >> 32));
                    }
                const int nint = int(blob.size()) - s.tab;
                const int lds = ((nint + 3) & ~3) * 4 + (tr ? s.k * s.pitch * 4 : 0);
                lds_max = std::max(lds_max, lds);
                S.push_back(s);
            }
        }
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 10;
    const int n = 16384;
    const arena_t A = arena(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n));
    const arena_t C = arena(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n));
    printf("A %dx%d blocks, C %dx%d blocks, arenas %.1f / %.1f MiB\n", A.nbr(), A.nbc(), C.nbr(), C.nbc(),
           A.size * 4.0 / 1048576, C.size * 4.0 / 1048576);
    std::vector<float> ha(A.size), hc(C.size);
    for (uint64_t k = 0; k < A.size; ++k) ha[k] = float(k % 1000003) * 0.5f;
    for (uint64_t k = 0; k < C.size; ++k) hc[k] = float(k % 999983) * 0.25f;
    float *dA, *dC;
    CK(hipMalloc(&dA, A.size * 4));
    CK(hipMalloc(&dC, C.size * 4));
    CK(hipMemcpy(dA, ha.data(), A.size * 4, hipMemcpyHostToDevice));
    const float alpha = -0.5f, beta = 2.f;
    std::mt19937_64 g(7);
    std::vector<std::pair<int, int>> sample(1 << 20);
    for (auto& x : sample) x = {int(g() % n), int(g() % n)};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<float> out(C.size);
    for (int tr = 0; tr < 2; ++tr)
        for (int maxf : {2048, 4096, 8192}) {
            std::vector<strip_t> S;
            std::vector<piece_t> P;
            build(A, C, tr, maxf, S, P);
            strip_t* dS;
            piece_t* dP;
            CK(hipMalloc(&dS, S.size() * sizeof(strip_t)));
            CK(hipMalloc(&dP, P.size() * sizeof(piece_t)));
            CK(hipMemcpy(dS, S.data(), S.size() * sizeof(strip_t), hipMemcpyHostToDevice));
            CK(hipMemcpy(dP, P.data(), P.size() * sizeof(piece_t), hipMemcpyHostToDevice));
            int lds = 0;
            for (const auto& s : S) lds = std::max(lds, s.k * s.pitch * 4);
            const double bytes = double(n) * n * 4 * (tr ? 3 : 2);
            auto launch = [&](int nt, int u) {
#define L(T, N, U)                                                                                      \
    hipLaunchKernelGGL((k_gather<T, N, U>), dim3(S.size()), dim3(256), lds, 0, dS, dP, dA, dC, alpha, beta)
                if (tr) {
                    if (nt) { if (u == 4) L(true, true, 4); else L(true, true, 8); }
                    else { if (u == 4) L(true, false, 4); else L(true, false, 8); }
                } else {
                    if (nt) { if (u == 4) L(false, true, 4); else L(false, true, 8); }
                    else { if (u == 4) L(false, false, 4); else L(false, false, 8); }
                }
#undef L
            };
            for (int nt = 0; nt < 2; ++nt)
                for (int u : {4, 8}) {
                    CK(hipMemcpy(dC, hc.data(), C.size * 4, hipMemcpyHostToDevice));
                    launch(nt, u);
                    CK(hipDeviceSynchronize());
                    CK(hipMemcpy(out.data(), dC, C.size * 4, hipMemcpyDeviceToHost));
                    long bad = 0;
                    for (const auto& x : sample) {
                        const uint64_t kc = C.at(x.first, x.second);
                        const float a = tr ? ha[A.at(x.second, x.first)] : ha[A.at(x.first, x.second)];
                        const float want = tr ? beta * hc[kc] + alpha * a : a;
                        bad += out[kc] != want;
                    }
                    std::vector<float> ms;
                    for (int r = 0; r < reps; ++r) {
                        CK(hipEventRecord(e0));
                        launch(nt, u);
                        CK(hipEventRecord(e1));
                        CK(hipEventSynchronize(e1));
                        float t = 0;
                        CK(hipEventElapsedTime(&t, e0, e1));
                        ms.push_back(t);
                    }
                    std::sort(ms.begin(), ms.end());
                    const double med = ms[ms.size() / 2];
                    printf("%s strip<=%5d floats nt%d U%d: %zu strips %zu pieces lds %6d B  %.4f ms  %.3f TB/s  %s\n",
                           tr ? "T" : "N", maxf, nt, u, S.size(), P.size(), lds, med, bytes / med / 1e9,
                           bad ? "BAD" : "ok");
                    fflush(stdout);
                }
            CK(hipFree(dS));
            CK(hipFree(dP));
            // band-table variant on the same strips
            std::vector<bstrip_t> B;
            std::vector<int> blob;
            int blds = 0;
            build_band(A, C, tr, maxf, B, blob, blds);
            bstrip_t* dB;
            int* dblob;
            CK(hipMalloc(&dB, B.size() * sizeof(bstrip_t)));
            CK(hipMalloc(&dblob, blob.size() * 4));
            CK(hipMemcpy(dB, B.data(), B.size() * sizeof(bstrip_t), hipMemcpyHostToDevice));
            CK(hipMemcpy(dblob, blob.data(), blob.size() * 4, hipMemcpyHostToDevice));
            for (int nt = 0; nt < 2; ++nt) {
                auto blaunch = [&] {
                    if (tr) {
                        if (nt) hipLaunchKernelGGL((k_band<true, true>), dim3(B.size()), dim3(256), blds, 0, dB, dblob, dA, dC, alpha, beta);
                        else hipLaunchKernelGGL((k_band<true, false>), dim3(B.size()), dim3(256), blds, 0, dB, dblob, dA, dC, alpha, beta);
                    } else {
                        if (nt) hipLaunchKernelGGL((k_band<false, true>), dim3(B.size()), dim3(256), blds, 0, dB, dblob, dA, dC, alpha, beta);
                        else hipLaunchKernelGGL((k_band<false, false>), dim3(B.size()), dim3(256), blds, 0, dB, dblob, dA, dC, alpha, beta);
                    }
                };
                CK(hipMemcpy(dC, hc.data(), C.size * 4, hipMemcpyHostToDevice));
                blaunch();
                CK(hipDeviceSynchronize());
                CK(hipMemcpy(out.data(), dC, C.size * 4, hipMemcpyDeviceToHost));
                long bad = 0;
                for (const auto& x : sample) {
                    const uint64_t kc = C.at(x.first, x.second);
                    const float a = tr ? ha[A.at(x.second, x.first)] : ha[A.at(x.first, x.second)];
                    const float want = tr ? beta * hc[kc] + alpha * a : a;
                    bad += out[kc] != want;
                }
                std::vector<float> ms;
                for (int r = 0; r < reps; ++r) {
                    CK(hipEventRecord(e0));
                    blaunch();
                    CK(hipEventRecord(e1));
                    CK(hipEventSynchronize(e1));
                    float t = 0;
                    CK(hipEventElapsedTime(&t, e0, e1));
                    ms.push_back(t);
                }
                std::sort(ms.begin(), ms.end());
                const double med = ms[ms.size() / 2];
                printf("%s strip<=%5d floats BAND nt%d: %zu strips blob %zu KiB lds %6d B  %.4f ms  %.3f TB/s  %s\n",
                       tr ? "T" : "N", maxf, nt, B.size(), blob.size() * 4 / 1024, blds, med, bytes / med / 1e9,
                       bad ? "BAD" : "ok");
                fflush(stdout);
            }
            CK(hipFree(dB));
            CK(hipFree(dblob));
        }
    return 0;
}
