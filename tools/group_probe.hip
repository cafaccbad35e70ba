// Tuning probe (not product): BASELINE cfg 5's geometry moved group-wise through LDS, so that
// both the reads and the writes are long contiguous runs.
//
// Every block of the cfg 5 layouts is its own column-major buffer (ld = rows), so the columns
// [c0, c1) of one block, all its rows, are one contiguous range ("chunk").
//   'T' (C = beta C + alpha A^T): a group is one C row block k (C rows r0..r1) x one A row block i
//       (C cols).  Its C part is whole column bands of the C blocks (k, l) it meets, its A part
//       whole column bands of the A blocks (i, j): every chunk on both sides is contiguous.
//   'N' (C = A): a group is a merged column band x a run of C row blocks; the C chunks are
//       contiguous, the A chunks at the two ends of the run are partial column runs.
// A workgroup stages its group in LDS (C coordinates, column-major, odd pitch for 'T'), every
// thread issuing all its loads before its LDS writes; then it writes the C chunks in memory order.
// The result is checked on the host against the definition, element by element.
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 tools/group_probe.hip -o tools/group_probe
//   tools/group_probe [N|T] [cap elements] [steps] [waves per workgroup 4|8] [elements per lane 8|16] [group order 0|1|2]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                            \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            std::printf("HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__);  \
            std::exit(2);                                                                \
        }                                                                                \
    } while (0)

struct chunk {
    int64_t addr;  // element offset from the array base
    int ld, nf, ns, ioff, isf, iss, start;
    float inv;
};
// a wavefront's share of one chunk: elements [l0, l0 + cnt) of the chunk in its memory order
struct piece {
    int64_t addr;
    int ld, nf, ioff, isf, iss, l0, cnt, pad;
};
struct group {
    int pa, na, pc, nc;  // A pieces [pa, pa + na), C pieces [pc, pc + nc)
};

// lanes walk a piece in memory order, (f, s) advanced by a constant per step (no division
// after the first element)
template <int U>
__device__ __forceinline__ void walk(const piece& q, int lane, int64_t* ad, int* id) {
    const int l = q.l0 + lane;
    int s = l / q.nf, f = l - s * q.nf;
    const int df = 64 % q.nf, ds = 64 / q.nf;
#pragma unroll
    for (int u = 0; u < U; ++u) {
        id[u] = -1;
        if (u * 64 + lane < q.cnt) {
            ad[u] = q.addr + int64_t(s) * q.ld + f;
            id[u] = q.ioff + f * q.isf + s * q.iss;
        }
        f += df;
        s += ds;
        if (f >= q.nf) { f -= q.nf; ++s; }
    }
}

template <int U, int NW, bool AX>
__global__ __launch_bounds__(64 * NW) void group_kernel(const group* __restrict__ groups,
                                                        const piece* __restrict__ pieces, int64_t n_groups,
                                                        const float* __restrict__ A, float* __restrict__ C,
                                                        float alpha, float beta) {
    extern __shared__ float img[];
    // XCD-contiguous slices of the group list (blocks are dealt round-robin over 8 XCDs)
    const int64_t nb = gridDim.x, x8 = int64_t(blockIdx.x) % 8, per = nb / 8, rem = nb % 8;
    const int64_t i8 = int64_t(blockIdx.x) / 8;
    const int64_t b = x8 < rem ? x8 * (per + 1) + i8 : rem * (per + 1) + (x8 - rem) * per + i8;
    if (b >= n_groups) return;
    const group g = groups[b];
    const int lane = threadIdx.x % 64, wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    for (int p = wave; p < g.na; p += NW) {
        const piece q = pieces[g.pa + p];
        int64_t ad[U];
        int id[U];
        float v[U];
        walk<U>(q, lane, ad, id);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (id[u] >= 0) v[u] = __builtin_nontemporal_load(A + ad[u]);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (id[u] >= 0) img[id[u]] = v[u];
    }
    __syncthreads();
    for (int p = wave; p < g.nc; p += NW) {
        const piece q = pieces[g.pc + p];
        int64_t ad[U];
        int id[U];
        float y[U];
        walk<U>(q, lane, ad, id);
        if (AX) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (id[u] >= 0) y[u] = C[ad[u]];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (id[u] < 0) continue;
            const float a = img[id[u]];
            const float r = AX ? beta * y[u] + alpha * a : a;
            __builtin_nontemporal_store(r, C + ad[u]);
        }
    }
}

static std::vector<int> splits(uint64_t seed, int lo, int hi, int n) {
    std::mt19937_64 r(seed);
    std::uniform_int_distribution<int> d(lo, hi);
    std::vector<int> s{0};
    while (s.back() < n) s.push_back(std::min(n, s.back() + d(r)));
    return s;
}
struct arena {
    std::vector<int> rs, cs;
    std::vector<int64_t> base;  // per block (i, j) row-major over the grid
    int64_t size = 0;
    int nr() const { return int(rs.size()) - 1; }
    int nc() const { return int(cs.size()) - 1; }
    int rows(int i) const { return rs[i + 1] - rs[i]; }
    int64_t at(int i, int j) const { return base[size_t(i) * nc() + j]; }
    arena(std::vector<int> r, std::vector<int> c) : rs(std::move(r)), cs(std::move(c)) {
        for (int i = 0; i < nr(); ++i)
            for (int j = 0; j < nc(); ++j) {
                base.push_back(size);
                size += (int64_t(rows(i)) * (cs[j + 1] - cs[j]) + 63) / 64 * 64;
            }
        size = std::max<int64_t>(size, 64);
    }
    // block index of global coordinate x along splits v
    static std::vector<int> owner(const std::vector<int>& v) {
        std::vector<int> o(size_t(v.back()));
        for (size_t b = 0; b + 1 < v.size(); ++b)
            for (int x = v[b]; x < v[b + 1]; ++x) o[size_t(x)] = int(b);
        return o;
    }
};

static int g_piece = 1024;  // elements per wavefront piece (64 * U)
static void finish(std::vector<group>& G, std::vector<piece>& PC, std::vector<chunk> a, std::vector<chunk> c) {
    group g{};
    auto cut = [&](const std::vector<chunk>& v) {
        for (const auto& x : v) {
            const int n = x.nf * x.ns;
            for (int l0 = 0; l0 < n; l0 += g_piece)
                PC.push_back(piece{x.addr, x.ld, x.nf, x.ioff, x.isf, x.iss, l0, std::min(g_piece, n - l0), 0});
        }
    };
    g.pa = int(PC.size());
    cut(a);
    g.na = int(PC.size()) - g.pa;
    g.pc = int(PC.size());
    cut(c);
    g.nc = int(PC.size()) - g.pc;
    G.push_back(g);
}

int main(int argc, char** argv) {
    const char op = argc > 1 ? argv[1][0] : 'T';
    const int cap = argc > 2 ? std::atoi(argv[2]) : 8192;
    const int steps = argc > 3 ? std::atoi(argv[3]) : 20;
    const int NW = argc > 4 ? std::atoi(argv[4]) : 4;   // wavefronts per workgroup: 4 or 8
    const int U = argc > 5 ? std::atoi(argv[5]) : 16;   // elements per lane per piece: 8 or 16
    g_piece = 64 * U;
    const int n = 16384;
    arena A(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n));
    arena Cb(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n));
    std::vector<group> G;
    std::vector<piece> PC;
    if (op == 'T') {
        // group (k, i, part): C rows [r0, r1) of C row block k x C cols = A rows of A row block i
        for (int i = 0; i < A.nr(); ++i) {
            const int c0 = A.rs[i], c1 = A.rs[i + 1], S = c1 - c0;
            for (int k = 0; k < Cb.nr(); ++k) {
                const int R = Cb.rows(k);
                int q = 1;
                while (((R + q - 1) / q | 1) * S > cap) ++q;
                for (int p = 0; p < q; ++p) {
                    const int r0 = Cb.rs[k] + p * R / q, r1 = Cb.rs[k] + (p + 1) * R / q;
                    const int P = (r1 - r0) | 1;
                    std::vector<chunk> ca, cc;
                    for (int l = 0; l < Cb.nc(); ++l) {
                        const int l0 = std::max(Cb.cs[l], c0), l1 = std::min(Cb.cs[l + 1], c1);
                        if (l0 >= l1) continue;
                        chunk x{};
                        x.addr = Cb.at(k, l) + int64_t(l0 - Cb.cs[l]) * R + (r0 - Cb.rs[k]);
                        x.ld = R; x.nf = r1 - r0; x.ns = l1 - l0;
                        x.ioff = (l0 - c0) * P; x.isf = 1; x.iss = P;
                        cc.push_back(x);
                    }
                    for (int j = 0; j < A.nc(); ++j) {
                        const int j0 = std::max(A.cs[j], r0), j1 = std::min(A.cs[j + 1], r1);
                        if (j0 >= j1) continue;
                        chunk x{};
                        x.addr = A.at(i, j) + int64_t(j0 - A.cs[j]) * S;
                        x.ld = S; x.nf = S; x.ns = j1 - j0;
                        x.ioff = j0 - r0; x.isf = P; x.iss = 1;
                        ca.push_back(x);
                    }
                    finish(G, PC, ca, cc);
                }
            }
        }
    } else {
        std::vector<int> m;  // merged column splits
        std::merge(A.cs.begin(), A.cs.end(), Cb.cs.begin(), Cb.cs.end(), std::back_inserter(m));
        m.erase(std::unique(m.begin(), m.end()), m.end());
        const auto aj = arena::owner(A.cs), cl = arena::owner(Cb.cs), ai = arena::owner(A.rs);
        const int wmax = std::max(1, cap / 160);
        for (size_t b = 0; b + 1 < m.size(); ++b) {
            for (int c0 = m[b]; c0 < m[b + 1]; c0 += wmax) {
                const int W = std::min(wmax, m[b + 1] - c0), j = aj[size_t(c0)], l = cl[size_t(c0)];
                int k = 0;
                while (k < Cb.nr()) {
                    int k1 = k, R = 0;  // C row blocks k..k1-1
                    while (k1 < Cb.nr() && (R + Cb.rows(k1)) * W <= cap && k1 - k < 12) R += Cb.rows(k1++);
                    if (k1 == k) { std::printf("C block over cap\n"); return 1; }
                    const int r0 = Cb.rs[k], r1 = Cb.rs[k1];
                    std::vector<chunk> ca, cc;
                    for (int kk = k; kk < k1; ++kk) {
                        chunk x{};
                        x.addr = Cb.at(kk, l) + int64_t(c0 - Cb.cs[l]) * Cb.rows(kk);
                        x.ld = Cb.rows(kk); x.nf = Cb.rows(kk); x.ns = W;
                        x.ioff = Cb.rs[kk] - r0; x.isf = 1; x.iss = R;
                        cc.push_back(x);
                    }
                    for (int i = ai[size_t(r0)]; i < A.nr() && A.rs[i] < r1; ++i) {
                        const int i0 = std::max(A.rs[i], r0), i1 = std::min(A.rs[i + 1], r1);
                        chunk x{};
                        x.addr = A.at(i, j) + int64_t(c0 - A.cs[j]) * A.rows(i) + (i0 - A.rs[i]);
                        x.ld = A.rows(i); x.nf = i1 - i0; x.ns = W;
                        x.ioff = i0 - r0; x.isf = 1; x.iss = R;
                        ca.push_back(x);
                    }
                    finish(G, PC, ca, cc);
                    k = k1;
                }
            }
        }
    }
    // group order: 0 as built, 1 by the address of the first C piece, 2 by the first A piece
    const int order = argc > 6 ? std::atoi(argv[6]) : 0;
    if (order) {
        std::stable_sort(G.begin(), G.end(), [&](const group& x, const group& y) {
            return order == 1 ? PC[size_t(x.pc)].addr < PC[size_t(y.pc)].addr
                              : PC[size_t(x.pa)].addr < PC[size_t(y.pa)].addr;
        });
    }
    const int64_t el = int64_t(n) * n;
    const bool ax = op == 'T';
    const float alpha = ax ? -0.5f : 1.f, beta = ax ? 2.f : 0.f;
    const double bytes = double(el) * (ax ? 12 : 8);
    std::printf("op %c cap %d waves %d U %d: %zu groups, %zu pieces, %.3f GB per launch\n", op, cap, NW, U,
                G.size(), PC.size(), bytes / 1e9);

    std::vector<float> ha(size_t(A.size)), hc(size_t(Cb.size));
    std::mt19937 rg(7);
    std::uniform_real_distribution<float> ud(-1.f, 1.f);
    for (auto& x : ha) x = ud(rg);
    for (auto& x : hc) x = ud(rg);
    float *da, *dc;
    group* dg;
    piece* dch;
    CK(hipMalloc(&da, ha.size() * 4));
    CK(hipMalloc(&dc, hc.size() * 4));
    CK(hipMalloc(&dg, G.size() * sizeof(group)));
    CK(hipMalloc(&dch, PC.size() * sizeof(piece)));
    CK(hipMemcpy(da, ha.data(), ha.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dg, G.data(), G.size() * sizeof(group), hipMemcpyHostToDevice));
    CK(hipMemcpy(dch, PC.data(), PC.size() * sizeof(piece), hipMemcpyHostToDevice));
    auto launch = [&]() {
        const size_t lds = size_t(cap) * 4;
        const unsigned blocks = unsigned(G.size());
#define GK(U_, NW_, AX_) hipLaunchKernelGGL((group_kernel<U_, NW_, AX_>), dim3(blocks), dim3(64 * NW_), lds, 0, \
                                            dg, dch, int64_t(G.size()), da, dc, alpha, beta)
        if (U == 16 && NW == 4) { if (ax) GK(16, 4, true); else GK(16, 4, false); }
        else if (U == 16 && NW == 8) { if (ax) GK(16, 8, true); else GK(16, 8, false); }
        else if (U == 8 && NW == 4) { if (ax) GK(8, 4, true); else GK(8, 4, false); }
        else { if (ax) GK(8, 8, true); else GK(8, 8, false); }
        CK(hipGetLastError());
    };
    if ((U != 8 && U != 16) || (NW != 4 && NW != 8) || cap > 16384) { std::printf("bad args\n"); return 1; }
    if (cap > 8192) CK(hipFuncSetAttribute(reinterpret_cast<const void*>(&group_kernel<16, 8, true>),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, cap * 4));
    // correctness: one launch on known C
    CK(hipMemcpy(dc, hc.data(), hc.size() * 4, hipMemcpyHostToDevice));
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> out(hc.size());
    CK(hipMemcpy(out.data(), dc, out.size() * 4, hipMemcpyDeviceToHost));
    {
        const auto ari = arena::owner(A.rs), acj = arena::owner(A.cs);
        int64_t bad = 0;
        for (int k = 0; k < Cb.nr(); ++k)
            for (int l = 0; l < Cb.nc(); ++l) {
                const int R = Cb.rows(k);
                for (int c = Cb.cs[l]; c < Cb.cs[l + 1]; ++c)
                    for (int r = Cb.rs[k]; r < Cb.rs[k + 1]; ++r) {
                        const int ar = ax ? c : r, ac = ax ? r : c;
                        const int i = ari[size_t(ar)], j = acj[size_t(ac)];
                        const float a = ha[size_t(A.at(i, j) + int64_t(ac - A.cs[j]) * A.rows(i) + (ar - A.rs[i]))];
                        const size_t ci = size_t(Cb.at(k, l) + int64_t(c - Cb.cs[l]) * R + (r - Cb.rs[k]));
                        const float want = ax ? beta * hc[ci] + alpha * a : a;
                        if (std::memcmp(&want, &out[ci], 4) != 0 && bad++ < 5)
                            std::printf("mismatch at C(%d,%d): %g vs %g\n", r, c, out[ci], want);
                    }
            }
        std::printf("check: %s (%lld mismatches)\n", bad ? "WRONG" : "ok", (long long)bad);
        if (bad) return 1;
    }
    for (int w = 0; w < 3; ++w) launch();
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, 0));
    for (int s = 0; s < steps; ++s) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= float(steps);
    std::printf("op %c cap %d waves %d U %d order %d: kernel %.4f ms  %.1f GB/s\n", op, cap, NW, U, order, ms,
                bytes / (ms * 1e-3) / 1e9);
    return 0;
}
