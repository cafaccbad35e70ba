// The host side of the path under AddressSanitizer + UndefinedBehaviorSanitizer (the
// reference runs no sanitizers; the build runs its host code under them).  No GPU: layouts are
// built by the product's layout builders (layout.cpp), every rank of a P-rank job is planned by
// the product's planner (plan.cpp), and the three op lists of every rank are executed here by a
// plain element loop, the exchange done by memcpy between the ranks' package buffers.  An op
// that reaches outside its buffers trips ASan; every element of C is then checked exactly against
// op(A) with alpha / beta (contraction off: 0 ulp).
//
// Built and run by tests/test_sanitizers.py; prints "OK <cases>" or FAIL lines.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <random>
#include <vector>

#include "../../costa_amd/csrc/engine.hpp"

using namespace costa;
using namespace costa::engine;

static int failures = 0;
#define CHECK(c, ...)                                         \
    do {                                                      \
        if (!(c)) {                                           \
            std::printf("FAIL %s:%d: ", __FILE__, __LINE__);  \
            std::printf(__VA_ARGS__);                         \
            std::printf("\n");                                \
            ++failures;                                       \
        }                                                     \
    } while (0)

// one tile op on the host: dst(f, s) or dst(s, f) = g(src(f, s)) (the kernels' contract)
static void exec_op(const costa_tile_op_t& op, const char* src_base, char* dst_base, double alpha,
                    double beta) {
    const double* src = reinterpret_cast<const double*>(src_base + op.src);
    double* dst = reinterpret_cast<double*>(dst_base + op.dst);
    const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
    const uint32_t kind = (op.flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
    for (int s = 0; s < op.ns; ++s)
        for (int f = 0; f < op.nf; ++f) {
            const double x = src[int64_t(s) * op.lds + f];
            double& y = dst[tr ? int64_t(f) * op.ldd + s : int64_t(s) * op.ldd + f];
            if (kind == COSTA_SCALE_BITCOPY)
                y = x;
            else if (kind == COSTA_SCALE_ZERO)
                y = 0.0;
            else if (kind == COSTA_SCALE_ALPHA)
                y = alpha * x;
            else
                y = beta * y + alpha * x;
        }
}

static double a_val(int i, int j) { return 1.0 + i * 7919.0 + j * 0.5; }
static double c_val(int i, int j) { return -3.0 + i * 0.25 - j * 104729.0; }

// one job on P ranks; make_a / make_c(rank, buffer) build each rank's layout
// `relabel` (a rank permutation, involution): rank r builds C with the blocks of rank
// relabel[r] and every C layout gets reorder_ranks(relabel), as README.md:343-362 prescribes
template <typename MA, typename MC>
static void run_case(const char* name, int P, MA make_a, MC make_c, size_t a_elems, size_t c_elems,
                     char op, double alpha, double beta, int loopback = 0,
                     const std::vector<int>& relabel = {}) {
    std::vector<std::vector<double>> abuf, cbuf;
    std::vector<grid_layout<double>> la, lc;
    std::vector<elayout> ea, ec;
    for (int r = 0; r < P; ++r) {
        abuf.emplace_back(a_elems, -1.0);
        cbuf.emplace_back(c_elems, 0.0);
    }
    for (int r = 0; r < P; ++r) {
        la.push_back(make_a(r, abuf[size_t(r)].data()));
        lc.push_back(make_c(relabel.empty() ? r : relabel[size_t(r)], cbuf[size_t(r)].data()));
        if (!relabel.empty()) lc.back().reorder_ranks(relabel);
        la.back().initialize(a_val);
        lc.back().initialize(c_val);
    }
    for (int r = 0; r < P; ++r) {
        ea.push_back(erase(la[size_t(r)]));
        ec.push_back(erase(lc[size_t(r)]));
    }
    std::vector<std::unique_ptr<plan>> plans;
    for (int r = 0; r < P; ++r) {
        job j;
        j.A = &ea[size_t(r)];
        j.C = &ec[size_t(r)];
        j.trans = op;
        std::memcpy(j.s.alpha.data(), &alpha, 8);
        std::memcpy(j.s.beta.data(), &beta, 8);
        plans.push_back(make_plan({j}, r, P, loopback));
    }
    for (int r = 0; r < P; ++r)  // package geometry agrees across ranks
        for (int q = 0; q < P; ++q)
            CHECK(plans[size_t(r)]->send_counts[size_t(q)] == plans[size_t(q)]->recv_counts[size_t(r)],
                  "%s: send %d->%d differs from the receive", name, r, q);
    std::vector<std::vector<char>> sendb(static_cast<size_t>(P)), recvb(static_cast<size_t>(P));
    for (int r = 0; r < P; ++r) {
        sendb[size_t(r)].resize(size_t(plans[size_t(r)]->send_elems) * 8 + 8);
        recvb[size_t(r)].resize(size_t(plans[size_t(r)]->recv_elems) * 8 + 8);
    }
    for (int r = 0; r < P; ++r)  // PACK
        for (const auto& o : plans[size_t(r)]->pack_ops) exec_op(o, nullptr, sendb[size_t(r)].data(), alpha, beta);
    for (int r = 0; r < P; ++r)  // the exchange
        for (int q = 0; q < P; ++q) {
            const auto& pr = *plans[size_t(r)];
            const auto& pq = *plans[size_t(q)];
            const size_t n = size_t(pr.send_counts[size_t(q)]) * 8;
            if (n)
                std::memcpy(recvb[size_t(q)].data() + pq.recv_displs[size_t(r)] * 8,
                            sendb[size_t(r)].data() + pr.send_displs[size_t(q)] * 8, n);
        }
    for (int r = 0; r < P; ++r) {  // UNPACK, LOCAL
        for (const auto& o : plans[size_t(r)]->unpack_ops)
            exec_op(o, recvb[size_t(r)].data(), nullptr, alpha, beta);
        for (const auto& o : plans[size_t(r)]->local_ops) exec_op(o, nullptr, nullptr, alpha, beta);
    }
    for (int r = 0; r < P; ++r) {
        const bool ok = lc[size_t(r)].validate(
            [&](int i, int j) {
                const double x = op == 'N' ? a_val(i, j) : a_val(j, i);
                return beta == 0.0 ? alpha * x : beta * c_val(i, j) + alpha * x;
            },
            0.0);
        CHECK(ok, "%s: rank %d C differs from op(A)", name, r);
    }
}

struct bc {
    int m, n, mb, nb, ia, ja, sm, sn, pm, pn;
    char order, ord;
};

// local leading dimension (+3 padding) and slow extent of a block-cyclic rank's buffer
static std::pair<int, int> local_dims(const bc& g, int rank) {
    const int pr = g.order == 'R' ? rank / g.pn : rank % g.pm;
    const int pc = g.order == 'R' ? rank % g.pn : rank / g.pm;
    const int lr = scalapack::numroc(g.m, g.mb, pr, 0, g.pm);
    const int lc = scalapack::numroc(g.n, g.nb, pc, 0, g.pn);
    return {std::max(1, g.ord == 'C' ? lr : lc) + 3, std::max(1, g.ord == 'C' ? lc : lr)};
}

static int cases = 0;

static void run_bc(const char* name, bc a, bc c, char op, double alpha, double beta, int loop = 0,
                   const std::vector<int>& relabel = {}) {
    const int P = std::max(a.pm * a.pn, c.pm * c.pn);
    size_t ae = 0, ce = 0;
    for (int r = 0; r < P; ++r) {
        const auto da = local_dims(a, r), dc = local_dims(c, r);
        ae = std::max(ae, size_t(da.first) * size_t(da.second));
        ce = std::max(ce, size_t(dc.first) * size_t(dc.second));
    }
    auto mk = [](const bc& g) {
        return [g](int r, double* p) {
            return block_cyclic_layout<double>(g.m, g.n, g.mb, g.nb, g.ia, g.ja, g.sm, g.sn, g.pm, g.pn,
                                               g.order, 0, 0, p, local_dims(g, r).first, g.ord, r);
        };
    };
    run_case(name, P, mk(a), mk(c), ae, ce, op, alpha, beta, loop, relabel);
    ++cases;
}

int main() {
    // block-cyclic -> block-cyclic (ScaLAPACK p?gemr2d / p?tran): grids, blocks, sub-matrices,
    // orderings, alpha / beta, and the one-rank loopback routings
    run_bc("same 2x2", {300, 280, 64, 64, 1, 1, 300, 280, 2, 2, 'R', 'C'},
           {300, 280, 64, 64, 1, 1, 300, 280, 2, 2, 'R', 'C'}, 'N', 1.0, 0.0);
    run_bc("2x2 -> 4x1 gemr2d", {300, 280, 64, 64, 1, 1, 300, 280, 2, 2, 'R', 'C'},
           {300, 280, 50, 70, 1, 1, 300, 280, 4, 1, 'R', 'C'}, 'N', 1.0, 0.0);
    run_bc("2x3 -> 3x2 tran axpby", {257, 190, 32, 48, 1, 1, 257, 190, 2, 3, 'C', 'C'},
           {190, 257, 40, 24, 1, 1, 190, 257, 3, 2, 'R', 'R'}, 'T', 2.0, 0.5);
    run_bc("row-major source, sub-matrices", {260, 240, 30, 20, 5, 7, 200, 180, 2, 2, 'R', 'R'},
           {190, 210, 16, 48, 3, 2, 180, 200, 1, 4, 'C', 'C'}, 'T', -0.75, 0.0);
    run_bc("2x2 -> 4x1 relabelled target", {300, 280, 64, 64, 1, 1, 300, 280, 2, 2, 'R', 'C'},
           {300, 280, 50, 70, 1, 1, 300, 280, 4, 1, 'R', 'C'}, 'N', 1.0, 0.0, 0, {2, 3, 0, 1});
    run_bc("1 rank, loopback all", {200, 150, 32, 48, 1, 1, 200, 150, 1, 1, 'R', 'C'},
           {150, 200, 40, 24, 1, 1, 150, 200, 1, 1, 'R', 'C'}, 'T', 1.0, 0.0, 1);
    run_bc("1 rank, loopback half", {200, 150, 32, 48, 1, 1, 200, 150, 1, 1, 'R', 'C'},
           {200, 150, 40, 24, 1, 1, 200, 150, 1, 1, 'R', 'R'}, 'N', 1.5, 2.0, 2);

    // custom layouts: irregular splits, random owners over 3 ranks, blocks one after another in
    // a rank's buffer with ld = rows + 2
    std::mt19937 g(7);
    auto splits = [&](int n, int lo, int hi) {
        std::vector<int> s{0};
        while (s.back() < n) s.push_back(std::min(n, s.back() + lo + int(g() % unsigned(hi - lo + 1))));
        return s;
    };
    const int m = 230, n = 170, P = 3;
    for (char op : {'N', 'T'}) {
        const int am = op == 'N' ? m : n, an = op == 'N' ? n : m;
        const auto ars = splits(am, 5, 40), acs = splits(an, 5, 40);
        const auto crs = splits(m, 8, 60), ccs = splits(n, 8, 60);
        std::vector<int> aown, cown;
        for (size_t i = 0; i + 1 < ars.size(); ++i)
            for (size_t j = 0; j + 1 < acs.size(); ++j) aown.push_back(int(g() % P));
        for (size_t i = 0; i + 1 < crs.size(); ++i)
            for (size_t j = 0; j + 1 < ccs.size(); ++j) cown.push_back(int(g() % P));
        auto make = [](const std::vector<int>& rs, const std::vector<int>& cs,
                       const std::vector<int>& own) {
            return [&rs, &cs, &own](int r, double* p) {
                std::vector<block_t> bl;
                size_t off = 0;
                const int nbc = int(cs.size()) - 1;
                for (int i = 0; i + 1 < int(rs.size()); ++i)
                    for (int j = 0; j < nbc; ++j) {
                        if (own[size_t(i * nbc + j)] != r) continue;
                        const int rows = rs[size_t(i + 1)] - rs[size_t(i)];
                        const int cols = cs[size_t(j + 1)] - cs[size_t(j)];
                        bl.push_back({p + off, rows + 2, i, j});
                        off += size_t(rows + 2) * size_t(cols);
                    }
                return custom_layout<double>(int(rs.size()) - 1, nbc, rs.data(), cs.data(), own.data(),
                                             int(bl.size()), bl.data(), 'C');
            };
        };
        const size_t ae = size_t(am + 2 * int(ars.size())) * size_t(an);
        const size_t ce = size_t(m + 2 * int(crs.size())) * size_t(n);
        run_case(op == 'N' ? "custom N" : "custom T axpby", P, make(ars, acs, aown),
                 make(crs, ccs, cown), ae, ce, op, op == 'N' ? 1.0 : 0.5, op == 'N' ? 0.0 : -1.25);
        ++cases;
    }
    if (failures == 0) std::printf("OK %d\n", cases);
    return failures ? 1 : 0;
}
