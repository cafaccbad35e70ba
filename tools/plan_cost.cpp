// Host cost of a plan-cache miss on BASELINE cfg 5's geometry (fp32 16384^2 custom layouts, A
// edges 8-96, C edges 16-160, one rank), without a GPU: the host planner (make_plan) and the
// work-list build (build_work) timed separately, best of 5.  Block addresses are never touched.
//   g++ -O2 -std=c++17 -Iinclude -Icosta_amd/csrc tools/plan_cost.cpp -Lcosta_amd/lib \
//       -lcosta_amd -Wl,-rpath,$PWD/costa_amd/lib -o /tmp/plan_cost && /tmp/plan_cost
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>

#include "engine.hpp"

using namespace costa;
using namespace costa::engine;

static std::vector<int> splits(uint64_t seed, int lo, int hi, int n) {
    std::mt19937_64 r(seed);
    std::uniform_int_distribution<int> d(lo, hi);
    std::vector<int> s{0};
    while (s.back() < n) s.push_back(std::min(n, s.back() + d(r)));
    return s;
}

static grid_layout<float> layout(const std::vector<int>& rs, const std::vector<int>& cs, uint64_t base) {
    const int nr = int(rs.size()) - 1, nc = int(cs.size()) - 1;
    std::vector<int> own(size_t(nr) * size_t(nc), 0);
    std::vector<block_t> blocks;
    uint64_t off = 0;
    for (int i = 0; i < nr; ++i)
        for (int j = 0; j < nc; ++j) {
            const int rows = rs[size_t(i) + 1] - rs[size_t(i)], cols = cs[size_t(j) + 1] - cs[size_t(j)];
            blocks.push_back({reinterpret_cast<void*>(base + 4 * off), rows, i, j});
            off += (uint64_t(rows) * uint64_t(cols) + 63) / 64 * 64;
        }
    return custom_layout<float>(nr, nc, rs.data(), cs.data(), own.data(), int(blocks.size()),
                                blocks.data(), 'C');
}

int main() {
    const int n = 16384;
    auto LA = layout(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n), uint64_t(1) << 40);
    auto LC = layout(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n), uint64_t(1) << 41);
    elayout a = erase(LA), c = erase(LC);
    for (char op : {'N', 'T'}) {
        job j;
        j.A = &a;
        j.C = &c;
        j.trans = op;
        const float alpha = op == 'N' ? 1.f : -0.5f, beta = op == 'N' ? 0.f : 2.f;
        std::copy_n(reinterpret_cast<const unsigned char*>(&alpha), 4, j.s.alpha.begin());
        std::copy_n(reinterpret_cast<const unsigned char*>(&beta), 4, j.s.beta.begin());
        double best_plan = 1e30, best_work = 1e30;
        size_t ops = 0, items = 0;
        for (int rep = 0; rep < 5; ++rep) {
            auto t0 = std::chrono::steady_clock::now();
            auto p = make_plan({j}, 0, 1);
            auto t1 = std::chrono::steady_clock::now();
            std::vector<costa_tile_op_t> ord;
            std::vector<uint64_t> work;
            const work_split w = build_work(p->dtype, p->local_ops, ord, work);
            auto t2 = std::chrono::steady_clock::now();
            best_plan = std::min(best_plan, std::chrono::duration<double, std::milli>(t1 - t0).count());
            best_work = std::min(best_work, std::chrono::duration<double, std::milli>(t2 - t1).count());
            ops = p->local_ops.size();
            items = size_t(w.n_items());
        }
        std::printf("cfg5 %c: %zu ops -> %zu work items: make_plan %.2f ms, build_work %.2f ms\n", op,
                    ops, items, best_plan, best_work);
    }
    return 0;
}
