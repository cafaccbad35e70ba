// Rank relabelling: the communication graph of a transformation and the greedy matching that
// proposes a rank permutation keeping more data local.  Host-only.
//
// Behaviour follows the reference:
//   communication_volume   src/costa/grid2grid/transform.cpp:9-44
//     (per block of the initial grid: utils.cpp:90-140 rank_to_comm_vol_for_block)
//   optimal_reordering     src/costa/grid2grid/ranks_reordering.cpp:4-61
// with 64-bit weights (the reference narrows each edge's volume to int) and ties between equal
// weights broken by rank ids (the reference's order there follows its hash map's iteration).
#include <costa/grid2grid/ranks_reordering.hpp>
#include <costa/transform.hpp>

#include <algorithm>
#include <cctype>
#include <cstdint>
#include <stdexcept>
#include <tuple>
#include <vector>

namespace costa {

namespace {
// index range [first, last) of the cells of `split` that overlap [lo, hi)
std::pair<int, int> cover(const std::vector<int>& split, int lo, int hi) {
    const int first = int(std::upper_bound(split.begin(), split.end(), lo) - split.begin()) - 1;
    const int last = int(std::lower_bound(split.begin(), split.end(), hi) - split.begin());
    return {std::max(first, 0), last};
}
}  // namespace

comm_volume communication_volume(assigned_grid2D& g_init, assigned_grid2D& g_final, char trans) {
    assigned_grid2D gi = g_init;  // the caller's grid is left as it is
    const char op = char(std::toupper(static_cast<unsigned char>(trans)));
    if (op != 'N') gi.transpose();
    const auto& ri = gi.grid().rows_split;
    const auto& ci = gi.grid().cols_split;
    const auto& rf = g_final.grid().rows_split;
    const auto& cf = g_final.grid().cols_split;
    if (ri.empty() || ci.empty() || rf.empty() || cf.empty()) return {};
    if (ri.back() != rf.back() || ci.back() != cf.back())
        throw std::runtime_error("costa::communication_volume: grids of different matrix sizes");
    comm_volume::volume_t w;
    for (int i = 0; i + 1 < int(ri.size()); ++i) {
        const auto rc = cover(rf, ri[size_t(i)], ri[size_t(i) + 1]);
        for (int j = 0; j + 1 < int(ci.size()); ++j) {
            const int a = gi.owner(i, j);
            const auto cc = cover(cf, ci[size_t(j)], ci[size_t(j) + 1]);
            for (int p = rc.first; p < rc.second; ++p) {
                const int64_t rows = std::min(ri[size_t(i) + 1], rf[size_t(p) + 1]) -
                                     std::max(ri[size_t(i)], rf[size_t(p)]);
                if (rows <= 0) continue;
                for (int q = cc.first; q < cc.second; ++q) {
                    const int64_t cols = std::min(ci[size_t(j) + 1], cf[size_t(q) + 1]) -
                                         std::max(ci[size_t(j)], cf[size_t(q)]);
                    if (cols <= 0) continue;
                    const int b = g_final.owner(p, q);
                    w[edge_t{std::min(a, b), std::max(a, b)}] += size_t(rows * cols);
                }
            }
        }
    }
    return comm_volume(std::move(w));
}

std::vector<int> optimal_reordering(comm_volume& cv, int n_ranks, bool& reordered) {
    std::vector<int> perm(size_t(std::max(n_ranks, 0)));
    for (int k = 0; k < n_ranks; ++k) perm[size_t(k)] = k;
    reordered = false;
    auto vol = [&](int a, int b) -> int64_t {
        const auto it = cv.volume.find(edge_t{a, b});
        return it == cv.volume.end() ? 0 : int64_t(it->second);
    };
    // worth of taking pair {a, b}: what swapping keeps local beyond what already stays (a self
    // edge is worth 1, so a rank without a better partner keeps its label)
    std::vector<std::tuple<int64_t, int, int>> edges;
    edges.reserve(cv.volume.size());
    for (const auto& kv : cv.volume) {
        const int a = kv.first.src, b = kv.first.dest;
        if (a < 0 || b < 0 || a >= n_ranks || b >= n_ranks) continue;
        int64_t w = int64_t(kv.second);
        if (a == b) w = 2 * w + 1;
        w -= vol(a, a) + vol(b, b);
        if (w > 0) edges.emplace_back(w, a, b);
    }
    std::sort(edges.begin(), edges.end(), [](const auto& x, const auto& y) {
        if (std::get<0>(x) != std::get<0>(y)) return std::get<0>(x) > std::get<0>(y);
        return std::make_pair(std::get<1>(x), std::get<2>(x)) < std::make_pair(std::get<1>(y), std::get<2>(y));
    });
    std::vector<bool> taken(size_t(std::max(n_ranks, 0)), false);
    for (const auto& e : edges) {
        const int a = std::get<1>(e), b = std::get<2>(e);
        if (taken[size_t(a)] || taken[size_t(b)]) continue;
        perm[size_t(a)] = b;
        perm[size_t(b)] = a;
        if (a != b) reordered = true;
        taken[size_t(a)] = taken[size_t(b)] = true;
    }
    return perm;
}

}  // namespace costa
