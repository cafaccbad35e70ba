// Our rank relabelling (costa::communication_volume + costa::optimal_reordering through the
// drop-in headers) on one spec of tests/relabel/relabel_cases.py; prints the same JSON as the
// reference harness (oracle/ref_harness.cpp relabel).  Built and run by tests/test_relabel.py.
#include <costa/grid2grid/ranks_reordering.hpp>
#include <costa/layout.hpp>
#include <costa/transform.hpp>

#include <algorithm>
#include <cstdio>
#include <fstream>
#include <tuple>
#include <vector>

static costa::assigned_grid2D read_grid(std::istream& in, int P) {
    auto vec = [&]() {
        int n = 0;
        in >> n;
        std::vector<int> v(static_cast<size_t>(n));
        for (auto& x : v) in >> x;
        return v;
    };
    std::vector<int> rs = vec(), cs = vec();
    const size_t nbr = rs.size() - 1, nbc = cs.size() - 1;
    std::vector<std::vector<int>> own(nbr, std::vector<int>(nbc));
    for (auto& row : own)
        for (auto& x : row) in >> x;
    return costa::assigned_grid2D(costa::grid2D(std::move(rs), std::move(cs)), std::move(own), P);
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    std::ifstream in(argv[1]);
    int P = 0;
    char trans = 'N';
    in >> P >> trans;
    auto gi = read_grid(in, P);
    auto gf = read_grid(in, P);
    auto cv = costa::communication_volume(gi, gf, trans);
    bool reordered = false;
    auto perm = costa::optimal_reordering(cv, P, reordered);
    gf.reorder_ranks(perm);
    auto cv2 = costa::communication_volume(gi, gf, trans);
    std::vector<std::tuple<int, int, size_t>> e;
    for (const auto& kv : cv.volume)
        if (kv.second) e.emplace_back(kv.first.src, kv.first.dest, kv.second);
    std::sort(e.begin(), e.end());
    std::printf("{\"total\": %zu, \"new_total\": %zu, \"reordered\": %s, \"perm\": [", cv.total_volume(),
                cv2.total_volume(), reordered ? "true" : "false");
    for (size_t i = 0; i < perm.size(); ++i) std::printf("%s%d", i ? ", " : "", perm[i]);
    std::printf("], \"volume\": [");
    for (size_t i = 0; i < e.size(); ++i)
        std::printf("%s[%d, %d, %zu]", i ? ", " : "", std::get<0>(e[i]), std::get<1>(e[i]), std::get<2>(e[i]));
    std::printf("]}\n");
    return 0;
}
