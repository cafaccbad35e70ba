// TEST INFRASTRUCTURE ONLY — drives the REFERENCE COSTA library (compiled from
// /root/reference sources into oracle/_ref/ by oracle/Makefile) to produce golden vectors.
// Run by tests/golden/make_fixtures.py under `mpiexec -n P`; never shipped, never run on
// the GPU box.
//
//   ref_harness kat <outdir>             the 4 copy_and_transform known-answer tests of
//                                        tests/unit/test_utils.cpp, inputs + outputs dumped
//   ref_harness case <spec> <outdir>     one transform case (spec written by
//                                        make_fixtures.py); every rank dumps its C buffer
//   ref_harness bench <m> <n> <nb> <s>   CPU baseline: the reference's own transform 'T'
//                                        (alpha 1, beta 0) of an m x n fp64 matrix in nb x nb
//                                        blocks on one rank, repeated for ~s seconds (OpenMP
//                                        threads: OMP_NUM_THREADS); prints one JSON line.
//                                        Run by bench.py (cpu_baseline, rank 0, N = 1) on the
//                                        GPU box as a child process, as the timed baseline.
//   ref_harness bench_cfg3 <n> <nb> <s> | bench_c128 <n> <nb> <s> | bench_custom <spec> <N|T> <s>
//                                        the same for BASELINE cfg 3 / 4 / 5 (run_bench_cfg3 ...)
//   ref_harness relabel <spec>           rank relabelling of two grids (spec: P, trans, then
//                                        per grid its row splits, col splits, owners): prints
//                                        the communication volume, the reference's proposed
//                                        permutation and the volume after relabelling (JSON)
#include <costa/layout.hpp>
#include <costa/grid2grid/transform.hpp>
#include <costa/grid2grid/transformer.hpp>
#include <costa/grid2grid/memory_utils.hpp>
#include <costa/grid2grid/workspace.hpp>
#include <costa/grid2grid/ranks_reordering.hpp>
#include <mpi.h>

#include <algorithm>
#include <tuple>

#include <omp.h>

#include <chrono>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <iostream>
#include <limits>
#include <memory>
#include <string>
#include <vector>

namespace {

uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
// the synthetic-data generator shared with tests/golden/gen.py
uint64_t draw(uint64_t seed, int rank, uint64_t k) {
    return splitmix64(seed ^ (uint64_t(rank) << 48) ^ k);
}
double unif(uint64_t z) { return double(z >> 11) * 0x1.0p-52 - 1.0; }

template <typename T> T gen(uint64_t seed, int rank, uint64_t k);
template <> double gen<double>(uint64_t s, int r, uint64_t k) { return unif(draw(s, r, k)); }
template <> float gen<float>(uint64_t s, int r, uint64_t k) { return float(unif(draw(s, r, k))); }
template <> int gen<int>(uint64_t s, int r, uint64_t k) {
    return int((draw(s, r, k) >> 33) % 2001) - 1000;
}
template <> std::complex<double> gen<std::complex<double>>(uint64_t s, int r, uint64_t k) {
    return {unif(draw(s, r, 2 * k)), unif(draw(s, r, 2 * k + 1))};
}
template <> std::complex<float> gen<std::complex<float>>(uint64_t s, int r, uint64_t k) {
    return {float(unif(draw(s, r, 2 * k))), float(unif(draw(s, r, 2 * k + 1)))};
}

// optional "specials 1" on a pair line: about one element in 8 of A and of C gets non-finite or
// extreme parts from a fixed table (the same rule as oracle.add_specials in Python)
template <typename R> R special_part(uint64_t sel);
template <> double special_part<double>(uint64_t sel) {
    const double t[8] = {std::numeric_limits<double>::infinity(), -std::numeric_limits<double>::infinity(),
                         std::numeric_limits<double>::quiet_NaN(), -0.0, 0.0, 1e308, -3.0, 0.5};
    return t[sel & 7];
}
template <> float special_part<float>(uint64_t sel) {
    const float t[8] = {std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
                        std::numeric_limits<float>::quiet_NaN(), -0.0f, 0.0f, 3e38f, -3.0f, 0.5f};
    return t[sel & 7];
}
template <typename T> struct part { using type = T; };
template <typename R> struct part<std::complex<R>> { using type = R; };
template <typename T>
void add_specials(std::vector<T>& v, uint64_t seed, int rank) {
    using R = typename part<T>::type;
    for (size_t k = 0; k < v.size(); ++k) {
        const uint64_t z = draw(seed ^ 0x5EC1A1ull, rank, k);
        if (z & 7) continue;
        if constexpr (std::is_same<T, R>::value)
            v[k] = special_part<R>(z >> 3);
        else
            v[k] = T(special_part<R>(z >> 3), special_part<R>(z >> 6));
    }
}

template <typename T>
void dump(const std::string& path, const std::vector<T>& v) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(v.data()), std::streamsize(v.size() * sizeof(T)));
}

struct lspec {
    std::string kind;
    // bc
    int m, n, mb, nb, ia, ja, subm, subn, pm, pn, rsrc, csrc, lld;
    char order, ord;
    long long buf_elems;
    // custom
    int nbr, nbc;
    std::vector<int> rs, cs, owners;
    std::vector<long long> bufs;                      // per rank
    std::vector<std::vector<long long>> blocks;       // per rank: row col off ld ...
};

lspec read_layout(std::istream& in, int P) {
    lspec L;
    std::string tok;
    in >> tok >> L.kind;  // "kind" <bc|custom>
    if (L.kind == "bc") {
        in >> L.m >> L.n >> L.mb >> L.nb >> L.ia >> L.ja >> L.subm >> L.subn >> L.pm >> L.pn >>
            L.order >> L.rsrc >> L.csrc >> L.ord >> L.lld >> L.buf_elems;
    } else {
        in >> L.nbr >> L.nbc;
        L.rs.resize(size_t(L.nbr + 1));
        L.cs.resize(size_t(L.nbc + 1));
        L.owners.resize(size_t(L.nbr) * size_t(L.nbc));
        for (auto& x : L.rs) in >> x;
        for (auto& x : L.cs) in >> x;
        for (auto& x : L.owners) in >> x;
        in >> L.ord;
        L.bufs.resize(size_t(P));
        for (auto& x : L.bufs) in >> x;
        L.blocks.resize(size_t(P));
        for (int r = 0; r < P; ++r) {
            int nb;
            in >> nb;
            L.blocks[size_t(r)].resize(size_t(nb) * 4);
            for (auto& x : L.blocks[size_t(r)]) in >> x;
        }
    }
    return L;
}

template <typename T>
costa::grid_layout<T> build(const lspec& L, std::vector<T>& buf, int rank) {
    if (L.kind == "bc") {
        return costa::block_cyclic_layout<T>(L.m, L.n, L.mb, L.nb, L.ia, L.ja, L.subm, L.subn, L.pm,
                                             L.pn, L.order, L.rsrc, L.csrc, buf.data(), L.lld,
                                             L.ord, rank);
    }
    const auto& bl = L.blocks[size_t(rank)];
    std::vector<costa::block_t> loc;
    for (size_t k = 0; k + 3 < bl.size(); k += 4) {
        costa::block_t b;
        b.row = int(bl[k]);
        b.col = int(bl[k + 1]);
        b.data = buf.data() + bl[k + 2];
        b.ld = int(bl[k + 3]);
        loc.push_back(b);
    }
    return costa::custom_layout<T>(L.nbr, L.nbc, L.rs.data(), L.cs.data(), L.owners.data(),
                                   int(loc.size()), loc.data(), L.ord);
}

long long buf_size(const lspec& L, int rank) {
    long long n = L.kind == "bc" ? L.buf_elems : L.bufs[size_t(rank)];
    return n > 0 ? n : 1;
}

template <typename T>
int run_case(std::istream& in, const std::string& out, int rank, int P) {
    int npairs;
    std::string tok;
    in >> tok >> npairs;
    const size_t np = size_t(npairs);
    std::vector<char> trans(np);
    std::vector<T> alpha(np), beta(np);
    std::vector<int> noscale(np);
    std::vector<uint64_t> seedA(np), seedC(np);
    std::vector<std::vector<int>> relabel(np);  // target-layout rank relabelling (may be empty)
    std::vector<int> specials(np, 0);
    std::vector<lspec> A, C;
    for (int p = 0; p < npairs; ++p) {
        double ar, ai, br, bi;
        in >> tok >> trans[size_t(p)] >> tok >> ar >> ai >> tok >> br >> bi >> tok >>
            noscale[size_t(p)] >> tok >> seedA[size_t(p)] >> tok >> seedC[size_t(p)];
        // optional "relabelC k p0 .. p(k-1)": the target grid is relabelled by reorder_ranks(p)
        // (grid_layout.hpp:32-34, grid2D.hpp:219-229: a cell of base owner o belongs to rank
        // p[o]), so the target layout of rank r holds the local blocks of base rank p^-1[r]
        // (README.md:343-362 states it for the pair swaps optimal_reordering proposes: p^-1 = p)
        in >> std::ws;
        if (in.peek() == 'r') {
            int k;
            in >> tok >> k;
            relabel[size_t(p)].resize(size_t(k));
            for (auto& x : relabel[size_t(p)]) in >> x;
        }
        in >> std::ws;
        if (in.peek() == 's') in >> tok >> specials[size_t(p)];
        if constexpr (std::is_same<T, std::complex<double>>::value ||
                      std::is_same<T, std::complex<float>>::value) {
            alpha[size_t(p)] = T(ar, ai);
            beta[size_t(p)] = T(br, bi);
        } else {
            alpha[size_t(p)] = T(ar);
            beta[size_t(p)] = T(br);
        }
        A.push_back(read_layout(in, P));
        C.push_back(read_layout(in, P));
    }
    std::vector<std::vector<T>> abuf(np), cbuf(np);
    std::vector<costa::grid_layout<T>> la, lc;
    la.reserve(np);
    lc.reserve(np);
    for (int p = 0; p < npairs; ++p) {
        auto& a = abuf[size_t(p)];
        auto& c = cbuf[size_t(p)];
        auto& rl = relabel[size_t(p)];
        int crank = rank;
        for (size_t q = 0; q < rl.size(); ++q)
            if (rl[q] == rank) crank = int(q);
        a.resize(size_t(buf_size(A[size_t(p)], rank)));
        c.resize(size_t(buf_size(C[size_t(p)], crank)));
        for (size_t k = 0; k < a.size(); ++k) a[k] = gen<T>(seedA[size_t(p)], rank, k);
        for (size_t k = 0; k < c.size(); ++k) c[k] = gen<T>(seedC[size_t(p)], rank, k);
        if (specials[size_t(p)]) {
            add_specials(a, seedA[size_t(p)], rank);
            add_specials(c, seedC[size_t(p)], rank);
        }
        la.push_back(build<T>(A[size_t(p)], a, rank));
        lc.push_back(build<T>(C[size_t(p)], c, crank));
        if (!rl.empty()) lc.back().reorder_ranks(rl);
    }
    if (npairs == 1) {
        if (noscale[0])
            costa::transform<T>(la[0], lc[0], MPI_COMM_WORLD);
        else
            costa::transform<T>(la[0], lc[0], trans[0], alpha[0], beta[0], MPI_COMM_WORLD);
    } else {
        costa::transformer<T> tf(MPI_COMM_WORLD);
        for (int p = 0; p < npairs; ++p) {
            if (noscale[0])
                tf.schedule(la[size_t(p)], lc[size_t(p)]);
            else
                tf.schedule(la[size_t(p)], lc[size_t(p)], trans[size_t(p)], alpha[size_t(p)],
                            beta[size_t(p)]);
        }
        tf.transform();
    }
    for (int p = 0; p < npairs; ++p)
        dump(out + "/C" + std::to_string(p) + "_rank" + std::to_string(rank) + ".bin",
             cbuf[size_t(p)]);
    return 0;
}

// the four known-answer tests of the reference (tests/unit/test_utils.cpp:7, 75, 143, 208)
int run_kat(const std::string& out) {
    auto& ws = *costa::memory::get_costa_context_instance<int>();
    std::vector<int> in8x4 = {9, 1, 1, -1, 7, 3, 4, -1, 5, 5, 1, -1, 9, 2, 3, -1,
                              7, 6, 5, -1, 2, 2, 4, -1, 3, 7, 4, -1, 3, 8, 1, -1};
    {  // copy2D.row_major
        std::vector<int> o(40);
        costa::memory::copy_and_transform(8, 3, in8x4.data(), 4, false, o.data(), 5, false, false,
                                          false, 1, 0, ws);
        dump(out + "/kat_copy2D_row_major_out.bin", o);
    }
    {  // copy2D.col_major: in 3x8 col-major, ld 4 -> ld 5
        std::vector<int> o(40);
        costa::memory::copy_and_transform(3, 8, in8x4.data(), 4, true, o.data(), 5, true, false,
                                          false, 1, 0, ws);
        dump(out + "/kat_copy2D_col_major_out.bin", o);
    }
    {  // transpose.row_to_col_major
        std::vector<int> o(30);
        costa::memory::copy_and_transform(8, 3, in8x4.data(), 4, false, o.data(), 10, true, false,
                                          false, 1, 0, ws);
        dump(out + "/kat_row_to_col_major_out.bin", o);
    }
    {  // transpose.col_to_row_major with srand(100), in[i] = i + rand()
        srand(100);
        const int n_rows = 1000, n_cols = 500, in_stride = 1100, out_stride = 501;
        std::vector<int> in(size_t(n_cols) * in_stride);
        for (size_t i = 0; i < in.size(); ++i) in[i] = int(i) + rand();
        std::vector<int> o(size_t(n_rows) * out_stride);
        costa::memory::copy_and_transform(n_rows, n_cols, in.data(), in_stride, true, o.data(),
                                          out_stride, false, false, false, 1, 0, ws);
        dump(out + "/kat_col_to_row_major_in.bin", in);
        dump(out + "/kat_col_to_row_major_out.bin", o);
    }
    dump(out + "/kat_in8x4.bin", in8x4);
    return 0;
}

int run_bench(int m, int n, int nb, double seconds) {
    std::vector<double> a(size_t(m) * n), c(size_t(n) * m, 0.0);
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < a.size(); ++k) a[k] = gen<double>(0xC057A0, 0, k);
    auto A = costa::block_cyclic_layout<double>(m, n, nb, nb, 1, 1, m, n, 1, 1, 'R', 0, 0,
                                                a.data(), m, 'C', 0);
    auto C = costa::block_cyclic_layout<double>(n, m, nb, nb, 1, 1, n, m, 1, 1, 'R', 0, 0,
                                                c.data(), n, 'C', 0);
    costa::transform<double>(A, C, 'T', 1.0, 0.0, MPI_COMM_WORLD);  // warm-up: first touch
    int reps = 0;
    const auto t0 = std::chrono::steady_clock::now();
    double el = 0;
    do {
        costa::transform<double>(A, C, 'T', 1.0, 0.0, MPI_COMM_WORLD);
        ++reps;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } while (el < seconds && reps < 100000);
    bool ok = true;
    for (int j = 0; j < n && ok; ++j)
        for (int i = 0; i < m; ++i)
            if (c[size_t(i) * n + j] != a[size_t(j) * m + i]) {
                ok = false;
                break;
            }
    const double bytes = 2.0 * sizeof(double) * double(m) * n;  // read A + write C
    std::printf("{\"GBps\": %.3f, \"reps\": %d, \"seconds\": %.3f, \"threads\": %d, "
                "\"verified\": %s}\n",
                bytes * reps / el / 1e9, reps, el, omp_get_max_threads(), ok ? "true" : "false");
    return ok ? 0 : 1;
}

// CPU baselines of BASELINE cfg 3 / 4 / 5 (bench.py cpu_baseline of each baseline_configs
// entry; one rank, the reference's own OpenMP transform, timed like run_bench):
//   cfg3  pxgemr2d slice: fp64 'N' no-scale copy of an n x n matrix, nb x nb blocks, 1 x 1 grid
//   c128  pztranu slice: complex<double> 'T', alpha = (0.75, -0.5), beta = (1.25, 0.25), n x n,
//         nb x nb blocks (C changes every call; the first call's result is checked)
//   spec  custom layouts (cfg 5): `spec` holds A's row and column splits, then C's (each: count,
//         values); every block its own column-major buffer; op N (alpha 1, beta 0) or T
//         (alpha -0.5, beta 2)
// Each prints one JSON line {GBps (algorithmic bytes: read + write of every element, + read of C
// when beta != 0), reps, seconds, threads, verified}.
template <typename T>
double bench_loop(const std::function<void()>& call, double seconds, int& reps) {
    call();  // warm-up: first touch (the checked call where C changes)
    reps = 0;
    const auto t0 = std::chrono::steady_clock::now();
    double el = 0;
    do {
        call();
        ++reps;
        el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    } while (el < seconds && reps < 100000);
    return el;
}

void print_bench(double bytes, int reps, double el, bool ok) {
    std::printf("{\"GBps\": %.3f, \"reps\": %d, \"seconds\": %.3f, \"threads\": %d, \"verified\": %s}\n",
                bytes * reps / el / 1e9, reps, el, omp_get_max_threads(), ok ? "true" : "false");
}

int run_bench_cfg3(int n, int nb, double seconds) {
    std::vector<double> a(size_t(n) * n), c(size_t(n) * n, 0.0);
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < a.size(); ++k) a[k] = gen<double>(0xC057A0, 0, k);
    auto A = costa::block_cyclic_layout<double>(n, n, nb, nb, 1, 1, n, n, 1, 1, 'R', 0, 0, a.data(), n, 'C', 0);
    auto C = costa::block_cyclic_layout<double>(n, n, nb, nb, 1, 1, n, n, 1, 1, 'R', 0, 0, c.data(), n, 'C', 0);
    int reps = 0;
    const double el = bench_loop<double>([&] { costa::transform<double>(A, C, MPI_COMM_WORLD); }, seconds, reps);
    const bool ok = a == c;
    print_bench(2.0 * sizeof(double) * double(n) * n, reps, el, ok);
    return ok ? 0 : 1;
}

int run_bench_c128(int n, int nb, double seconds) {
    using z = std::complex<double>;
    std::vector<z> a(size_t(n) * n), c(size_t(n) * n);
#pragma omp parallel for schedule(static)
    for (size_t k = 0; k < a.size(); ++k) {
        a[k] = gen<z>(0xC057A0, 0, k);
        c[k] = gen<z>(0xC057C0, 0, k);
    }
    const std::vector<z> c0 = c;
    const z alpha(0.75, -0.5), beta(1.25, 0.25);
    auto A = costa::block_cyclic_layout<z>(n, n, nb, nb, 1, 1, n, n, 1, 1, 'R', 0, 0, a.data(), n, 'C', 0);
    auto C = costa::block_cyclic_layout<z>(n, n, nb, nb, 1, 1, n, n, 1, 1, 'R', 0, 0, c.data(), n, 'C', 0);
    costa::transform<z>(A, C, 'T', alpha, beta, MPI_COMM_WORLD);
    bool ok = true;  // the first call: C(i, j) = beta C0(i, j) + alpha A(j, i), every 97th element
    for (size_t k = 0; k < c.size() && ok; k += 97) {
        const size_t i = k % size_t(n), j = k / size_t(n);
        ok = c[k] == beta * c0[k] + alpha * a[i * size_t(n) + j];
    }
    int reps = 0;
    const double el = bench_loop<z>([&] { costa::transform<z>(A, C, 'T', alpha, beta, MPI_COMM_WORLD); },
                                    seconds, reps);
    print_bench(3.0 * sizeof(z) * double(n) * n, reps, el, ok);
    return ok ? 0 : 1;
}

int run_bench_custom(const char* spec, char op, double seconds) {
    std::ifstream in(spec);
    auto vec = [&]() {
        int k;
        in >> k;
        std::vector<int> v(static_cast<size_t>(k));
        for (auto& x : v) in >> x;
        return v;
    };
    const std::vector<int> ars = vec(), acs = vec(), crs = vec(), ccs = vec();
    struct arena {
        std::vector<float> buf;
        std::vector<costa::block_t> blocks;
        std::vector<size_t> off;
        std::vector<int> owners;
    };
    // every block its own column-major buffer (ld = rows), 256-byte aligned offsets
    auto make = [](const std::vector<int>& rs, const std::vector<int>& cs, uint64_t seed) {
        arena r;
        size_t off = 0;
        for (size_t i = 0; i + 1 < rs.size(); ++i)
            for (size_t j = 0; j + 1 < cs.size(); ++j) {
                r.off.push_back(off);
                off += (size_t(rs[i + 1] - rs[i]) * size_t(cs[j + 1] - cs[j]) + 63) / 64 * 64;
            }
        r.buf.assign(std::max<size_t>(off, 64), 0.f);
#pragma omp parallel for schedule(static)
        for (size_t k = 0; k < r.buf.size(); ++k) r.buf[k] = gen<float>(seed, 0, k);
        size_t b = 0;
        for (size_t i = 0; i + 1 < rs.size(); ++i)
            for (size_t j = 0; j + 1 < cs.size(); ++j, ++b)
                r.blocks.push_back({r.buf.data() + r.off[b], rs[i + 1] - rs[i], int(i), int(j)});
        r.owners.assign(r.blocks.size(), 0);
        return r;
    };
    arena a = make(ars, acs, 0xC057A0), c = make(crs, ccs, 0xC057C0);
    const std::vector<float> c0 = c.buf;
    auto A = costa::custom_layout<float>(int(ars.size()) - 1, int(acs.size()) - 1, ars.data(), acs.data(),
                                         a.owners.data(), int(a.blocks.size()), a.blocks.data(), 'C');
    auto C = costa::custom_layout<float>(int(crs.size()) - 1, int(ccs.size()) - 1, crs.data(), ccs.data(),
                                         c.owners.data(), int(c.blocks.size()), c.blocks.data(), 'C');
    const float alpha = op == 'N' ? 1.f : -0.5f, beta = op == 'N' ? 0.f : 2.f;
    costa::transform<float>(A, C, op, alpha, beta, MPI_COMM_WORLD);
    // the first call against the definition, element by element: C(i, j) = beta C0 + alpha op(A)
    auto at = [](const arena& r, const std::vector<int>& rs, const std::vector<int>& cs, int i, int j) {
        const size_t bi = size_t(std::upper_bound(rs.begin(), rs.end(), i) - rs.begin()) - 1;
        const size_t bj = size_t(std::upper_bound(cs.begin(), cs.end(), j) - cs.begin()) - 1;
        const size_t b = bi * (cs.size() - 1) + bj;
        return r.off[b] + size_t(j - cs[bj]) * size_t(rs[bi + 1] - rs[bi]) + size_t(i - rs[bi]);
    };
    const int M = crs.back(), N = ccs.back();
    long bad = 0;
#pragma omp parallel for schedule(dynamic, 16) reduction(+ : bad)
    for (int j = 0; j < N; j += 7)
        for (int i = 0; i < M; ++i) {
            const size_t kc = at(c, crs, ccs, i, j);
            const float x = op == 'N' ? a.buf[at(a, ars, acs, i, j)] : a.buf[at(a, ars, acs, j, i)];
            const float want = op == 'N' ? x : beta * c0[kc] + alpha * x;
            bad += c.buf[kc] != want;
        }
    const bool ok = bad == 0;
    int reps = 0;
    const double el = bench_loop<float>([&] { costa::transform<float>(A, C, op, alpha, beta, MPI_COMM_WORLD); },
                                        seconds, reps);
    print_bench((op == 'N' ? 2.0 : 3.0) * sizeof(float) * double(M) * N, reps, el, ok);
    return ok ? 0 : 1;
}

// ---- multi-rank CPU baselines (bench.py cpu_baseline at N > 1)
// Every rank of `mpiexec -n P` holds its share of the layouts and runs the reference's own
// costa::transform (pack -> MPI Isend / Irecv -> unpack, local tiles on the side;
// transform.cpp:46-128).  Each call is bracketed by MPI_Barrier, as the reference's miniapps time
// pxgemr2d (utils/pxgemr2d_utils.hpp:284-292); calls repeat until rank 0 has spent ~s seconds in
// them (its sum, broadcast, so every rank stops together).  Values are a function of the GLOBAL
// position (gen at i + j * M), so every rank checks sampled local elements of C after the first
// call against the definition; the mismatch counts are summed over the ranks.
//   bench_mr pxtran <n> <nb> <pm> <pn> <s>  fp64 'T' alpha 1 beta 0: A (n pm) x (n pn) on the pm x pn
//                                           'R' grid, C = A^T on the same grid (bench.py's N-rank
//                                           headline, n per rank)
//   bench_mr cfg3 <n> <nb> <pm> <pn> <s>    fp64 'N' copy (no scale): A (n pm) x (n pn) on pm x pn ->
//                                           C on a P x 1 grid (BASELINE configs[2]'s remap)
//   bench_mr cfg4 <e> <nb> <pm> <pn> <s>    complex<double> 'T' alpha (0.75, -0.5), beta (1.25, 0.25),
//                                           e x e on pm x pn (BASELINE configs[3])
//   bench_mr custom <spec> <N|T> <s>        custom layouts (BASELINE configs[4]); spec: A's row and
//                                           column splits and owners (row-major), then C's; every
//                                           owned block its own column-major buffer
// Rank 0 prints one JSON line {GBps (algorithmic bytes of all ranks: read + write of every
// element, + read of C when beta != 0, per call / rank 0's time), reps, seconds, ranks, threads
// (OpenMP threads per rank), verified}.
int bc_global(int l, int nb, int p, int pr) { return (l / nb) * p * nb + pr * nb + l % nb; }

template <typename T>
int bench_mr_bc(const std::string& kind, int n, int nb, int pm, int pn, double seconds, int rank, int P) {
    const bool c4 = kind == "cfg4", c3 = kind == "cfg3";
    const int M = c4 ? n : n * pm, N = c4 ? n : n * pn;  // A is M x N
    const int pr = rank / pn, pc = rank % pn;             // 'R' rank order
    const int lr_a = M / pm, lc_a = N / pn;
    // C: cfg3 M x N on P x 1; else N x M on pm x pn
    const int cpm = c3 ? P : pm, cpn = c3 ? 1 : pn, cpr = c3 ? rank : pr, cpc = c3 ? 0 : pc;
    const int Mc = c3 ? M : N, Nc = c3 ? N : M;
    const int lr_c = Mc / cpm, lc_c = Nc / cpn;
    if (M % (pm * nb) || N % (pn * nb) || Mc % (cpm * nb) || Nc % (cpn * nb)) {
        if (rank == 0) std::fprintf(stderr, "bench_mr: sizes not multiples of the grid blocks\n");
        return 2;
    }
    const uint64_t sa = 0xC057A0, sc = 0xC057C0;
    std::vector<T> a(size_t(lr_a) * lc_a), c(size_t(lr_c) * lc_c);
#pragma omp parallel for schedule(static)
    for (int lj = 0; lj < lc_a; ++lj)
        for (int li = 0; li < lr_a; ++li)
            a[size_t(lj) * lr_a + li] =
                gen<T>(sa, 0, uint64_t(bc_global(li, nb, pm, pr)) + uint64_t(bc_global(lj, nb, pn, pc)) * uint64_t(M));
#pragma omp parallel for schedule(static)
    for (int lj = 0; lj < lc_c; ++lj)
        for (int li = 0; li < lr_c; ++li)
            c[size_t(lj) * lr_c + li] = gen<T>(
                sc, 0, uint64_t(bc_global(li, nb, cpm, cpr)) + uint64_t(bc_global(lj, nb, cpn, cpc)) * uint64_t(Mc));
    auto A = costa::block_cyclic_layout<T>(M, N, nb, nb, 1, 1, M, N, pm, pn, 'R', 0, 0, a.data(), lr_a, 'C', rank);
    auto C = costa::block_cyclic_layout<T>(Mc, Nc, nb, nb, 1, 1, Mc, Nc, cpm, cpn, 'R', 0, 0, c.data(), lr_c, 'C',
                                           rank);
    T alpha = T(1), beta = T(0);
    if constexpr (std::is_same<T, std::complex<double>>::value) {
        alpha = T(0.75, -0.5);
        beta = T(1.25, 0.25);
    }
    const char op = c3 ? 'N' : 'T';
    auto call = [&] {
        if (c3)
            costa::transform<T>(A, C, MPI_COMM_WORLD);
        else
            costa::transform<T>(A, C, op, alpha, beta, MPI_COMM_WORLD);
    };
    call();  // warm-up (first touch, the MPI buffers); checked
    long bad = 0;
    for (size_t k = 0; k < c.size(); k += 97) {
        const int li = int(k % size_t(lr_c)), lj = int(k / size_t(lr_c));
        const int i = bc_global(li, nb, cpm, cpr), j = bc_global(lj, nb, cpn, cpc);
        const T x = op == 'N' ? gen<T>(sa, 0, uint64_t(i) + uint64_t(j) * M) : gen<T>(sa, 0, uint64_t(j) + uint64_t(i) * M);
        const T want = beta == T(0) ? alpha * x : beta * gen<T>(sc, 0, uint64_t(i) + uint64_t(j) * Mc) + alpha * x;
        bad += !(c[k] == want);
    }
    long bad_all = 0;
    MPI_Allreduce(&bad, &bad_all, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
    int reps = 0;
    double tsum = 0;
    for (;;) {
        MPI_Barrier(MPI_COMM_WORLD);
        const auto t0 = std::chrono::steady_clock::now();
        call();
        MPI_Barrier(MPI_COMM_WORLD);
        tsum += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        ++reps;
        double el = tsum;
        MPI_Bcast(&el, 1, MPI_DOUBLE, 0, MPI_COMM_WORLD);
        if (el >= seconds || reps >= 100000) {
            tsum = el;
            break;
        }
    }
    const double bytes = (beta == T(0) ? 2.0 : 3.0) * sizeof(T) * double(M) * N;
    if (rank == 0)
        std::printf("{\"GBps\": %.3f, \"reps\": %d, \"seconds\": %.3f, \"ranks\": %d, \"threads\": %d, "
                    "\"verified\": %s}\n",
                    bytes * reps / tsum / 1e9, reps, tsum, P, omp_get_max_threads(), bad_all == 0 ? "true" : "false");
    return bad_all == 0 ? 0 : 1;
}

int bench_mr_custom(const char* spec, char op, double seconds, int rank, int P) {
    std::ifstream in(spec);
    auto vec = [&]() {
        int k;
        in >> k;
        std::vector<int> v(static_cast<size_t>(k));
        for (auto& x : v) in >> x;
        return v;
    };
    struct grid {
        std::vector<int> rs, cs, owners;
        std::vector<float> buf;
        std::vector<costa::block_t> blocks;
    };
    auto read = [&] {
        grid g;
        g.rs = vec();
        g.cs = vec();
        g.owners.resize((g.rs.size() - 1) * (g.cs.size() - 1));
        for (auto& x : g.owners) in >> x;
        return g;
    };
    grid ga = read(), gc = read();
    const uint64_t sa = 0xC057A0, sc = 0xC057C0;
    const int M = ga.rs.back(), N = ga.cs.back();
    // this rank's blocks, each its own column-major buffer (ld = rows) at 256-byte aligned offsets
    auto make = [&](grid& g, uint64_t seed, int rows) {
        std::vector<size_t> off;
        std::vector<int> bi, bj;
        size_t o = 0;
        for (size_t i = 0; i + 1 < g.rs.size(); ++i)
            for (size_t j = 0; j + 1 < g.cs.size(); ++j)
                if (g.owners[i * (g.cs.size() - 1) + j] == rank) {
                    off.push_back(o);
                    bi.push_back(int(i));
                    bj.push_back(int(j));
                    o += (size_t(g.rs[i + 1] - g.rs[i]) * size_t(g.cs[j + 1] - g.cs[j]) + 63) / 64 * 64;
                }
        g.buf.assign(std::max<size_t>(o, 64), 0.f);
#pragma omp parallel for schedule(dynamic, 16)
        for (size_t b = 0; b < off.size(); ++b) {
            const int r0 = g.rs[size_t(bi[b])], r1 = g.rs[size_t(bi[b]) + 1];
            const int c0 = g.cs[size_t(bj[b])], c1 = g.cs[size_t(bj[b]) + 1];
            for (int j = c0; j < c1; ++j)
                for (int i = r0; i < r1; ++i)
                    g.buf[off[b] + size_t(j - c0) * size_t(r1 - r0) + size_t(i - r0)] =
                        gen<float>(seed, 0, uint64_t(i) + uint64_t(j) * uint64_t(rows));
        }
        for (size_t b = 0; b < off.size(); ++b)
            g.blocks.push_back({g.buf.data() + off[b], g.rs[size_t(bi[b]) + 1] - g.rs[size_t(bi[b])], bi[b], bj[b]});
    };
    make(ga, sa, M);
    const int Mc = gc.rs.back();
    make(gc, sc, Mc);
    auto A = costa::custom_layout<float>(int(ga.rs.size()) - 1, int(ga.cs.size()) - 1, ga.rs.data(), ga.cs.data(),
                                         ga.owners.data(), int(ga.blocks.size()), ga.blocks.data(), 'C');
    auto C = costa::custom_layout<float>(int(gc.rs.size()) - 1, int(gc.cs.size()) - 1, gc.rs.data(), gc.cs.data(),
                                         gc.owners.data(), int(gc.blocks.size()), gc.blocks.data(), 'C');
    const float alpha = op == 'N' ? 1.f : -0.5f, beta = op == 'N' ? 0.f : 2.f;
    auto call = [&] { costa::transform<float>(A, C, op, alpha, beta, MPI_COMM_WORLD); };
    call();
    long bad = 0;  // every 7th column of every local C block against the definition
    for (const auto& b : gc.blocks) {
        const int r0 = gc.rs[size_t(b.row)], r1 = gc.rs[size_t(b.row) + 1];
        const int c0 = gc.cs[size_t(b.col)], c1 = gc.cs[size_t(b.col) + 1];
        const float* p = static_cast<const float*>(b.data);
        for (int j = c0; j < c1; j += 7)
            for (int i = r0; i < r1; ++i) {
                const float x = op == 'N' ? gen<float>(sa, 0, uint64_t(i) + uint64_t(j) * uint64_t(M))
                                          : gen<float>(sa, 0, uint64_t(j) + uint64_t(i) * uint64_t(M));
                const float want = op == 'N' ? x : beta * gen<float>(sc, 0, uint64_t(i) + uint64_t(j) * uint64_t(Mc)) + alpha * x;
                bad += p[size_t(j - c0) * size_t(r1 - r0) + size_t(i - r0)] != want;
            }
    }
    long bad_all = 0;
    MPI_Allreduce(&bad, &bad_all, 1, MPI_LONG, MPI_SUM, MPI_COMM_WORLD);
    int reps = 0;
    double tsum = 0;
    for (;;) {
        MPI_Barrier(MPI_COMM_WORLD);
        const auto t0 = std::chrono::steady_clock::now();
        call();
        MPI_Barrier(MPI_COMM_WORLD);
        tsum += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        ++reps;
        double el = tsum;
        MPI_Bcast(&el, 1, MPI_DOUBLE, 0, MPI_COMM_WORLD);
        if (el >= seconds || reps >= 100000) {
            tsum = el;
            break;
        }
    }
    const double bytes = (op == 'N' ? 2.0 : 3.0) * sizeof(float) * double(M) * N;
    if (rank == 0)
        std::printf("{\"GBps\": %.3f, \"reps\": %d, \"seconds\": %.3f, \"ranks\": %d, \"threads\": %d, "
                    "\"verified\": %s}\n",
                    bytes * reps / tsum / 1e9, reps, tsum, P, omp_get_max_threads(), bad_all == 0 ? "true" : "false");
    return bad_all == 0 ? 0 : 1;
}

// spec: P trans / per grid: n_rs rs... n_cs cs... owners (row-major)
costa::assigned_grid2D read_grid(std::istream& in, int P) {
    auto vec = [&]() {
        int n;
        in >> n;
        std::vector<int> v(static_cast<size_t>(n));
        for (auto& x : v) in >> x;
        return v;
    };
    std::vector<int> rs = vec(), cs = vec();
    const int nbr = int(rs.size()) - 1, nbc = int(cs.size()) - 1;
    std::vector<std::vector<int>> own(static_cast<size_t>(nbr), std::vector<int>(static_cast<size_t>(nbc)));
    for (auto& row : own)
        for (auto& x : row) in >> x;
    return costa::assigned_grid2D(costa::grid2D(std::move(rs), std::move(cs)), std::move(own), P);
}

void print_volume(const char* key, const costa::comm_volume& cv) {
    std::vector<std::tuple<int, int, size_t>> e;
    for (const auto& kv : cv.volume)
        if (kv.second) e.emplace_back(kv.first.src, kv.first.dest, kv.second);
    std::sort(e.begin(), e.end());
    std::printf("\"%s\": [", key);
    for (size_t i = 0; i < e.size(); ++i)
        std::printf("%s[%d, %d, %zu]", i ? ", " : "", std::get<0>(e[i]), std::get<1>(e[i]), std::get<2>(e[i]));
    std::printf("]");
}

int run_relabel(const char* spec) {
    std::ifstream in(spec);
    int P;
    char trans;
    in >> P >> trans;
    auto gi = read_grid(in, P);
    auto gf = read_grid(in, P);
    auto cv = costa::communication_volume(gi, gf, trans);
    bool reordered = false;
    auto perm = costa::optimal_reordering(cv, P, reordered);
    gf.reorder_ranks(perm);
    auto cv2 = costa::communication_volume(gi, gf, trans);
    std::printf("{\"total\": %zu, \"new_total\": %zu, \"reordered\": %s, \"perm\": [", cv.total_volume(),
                cv2.total_volume(), reordered ? "true" : "false");
    for (size_t i = 0; i < perm.size(); ++i) std::printf("%s%d", i ? ", " : "", perm[i]);
    std::printf("], ");
    print_volume("volume", cv);
    std::printf("}\n");
    return 0;
}

}  // namespace

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int rank = 0, P = 1;
    MPI_Comm_rank(MPI_COMM_WORLD, &rank);
    MPI_Comm_size(MPI_COMM_WORLD, &P);
    int rc = 1;
    if (argc >= 3 && std::string(argv[1]) == "kat") {
        rc = rank == 0 ? run_kat(argv[2]) : 0;
    } else if (argc >= 4 && std::string(argv[1]) == "case") {
        std::ifstream in(argv[2]);
        std::string tok;
        int dtype;
        in >> tok >> dtype;
        switch (dtype) {
        case 0: rc = run_case<float>(in, argv[3], rank, P); break;
        case 1: rc = run_case<double>(in, argv[3], rank, P); break;
        case 2: rc = run_case<std::complex<float>>(in, argv[3], rank, P); break;
        case 3: rc = run_case<std::complex<double>>(in, argv[3], rank, P); break;
        default: break;  // the reference instantiates transform for the 4 FP types only
        }
    } else if (argc >= 6 && std::string(argv[1]) == "bench") {
        rc = rank == 0 ? run_bench(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]),
                                   std::atof(argv[5]))
                       : 0;
    } else if (argc >= 5 && std::string(argv[1]) == "bench_cfg3") {
        rc = rank == 0 ? run_bench_cfg3(std::atoi(argv[2]), std::atoi(argv[3]), std::atof(argv[4])) : 0;
    } else if (argc >= 5 && std::string(argv[1]) == "bench_c128") {
        rc = rank == 0 ? run_bench_c128(std::atoi(argv[2]), std::atoi(argv[3]), std::atof(argv[4])) : 0;
    } else if (argc >= 5 && std::string(argv[1]) == "bench_custom") {
        rc = rank == 0 ? run_bench_custom(argv[2], argv[3][0], std::atof(argv[4])) : 0;
    } else if (argc >= 6 && std::string(argv[1]) == "bench_mr" && std::string(argv[2]) == "custom") {
        rc = bench_mr_custom(argv[3], argv[4][0], std::atof(argv[5]), rank, P);
    } else if (argc >= 8 && std::string(argv[1]) == "bench_mr") {
        const std::string kind = argv[2];
        const int n = std::atoi(argv[3]), nb = std::atoi(argv[4]), pm = std::atoi(argv[5]), pn = std::atoi(argv[6]);
        const double s = std::atof(argv[7]);
        if (pm * pn != P)
            rc = 2;
        else if (kind == "pxtran" || kind == "cfg3")
            rc = bench_mr_bc<double>(kind, n, nb, pm, pn, s, rank, P);
        else if (kind == "cfg4")
            rc = bench_mr_bc<std::complex<double>>(kind, n, nb, pm, pn, s, rank, P);
    } else if (argc >= 3 && std::string(argv[1]) == "relabel") {
        rc = rank == 0 ? run_relabel(argv[2]) : 0;
    } else {
        if (rank == 0)
            std::cerr << "usage: ref_harness kat <out> | case <spec> <out> | bench <m> <n> <nb> <s>"
                         " | relabel <spec>\n";
    }
    MPI_Finalize();
    return rc;
}
