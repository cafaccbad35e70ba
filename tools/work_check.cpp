// Invariants of the wavefront work lists (engine.cpp build_work) on BASELINE cfg 5's geometry,
// without a GPU (block addresses are never touched).  Run by tests/test_work_lists.py.
// For op 'N' (copy list) and 'T' (transposing list):
//   * no op takes the large or small shapes (every cfg 5 tile is below the large threshold);
//   * every piece fits the wavefront budget (3 KiB copy, 4 KiB staged with pitch nf | 1);
//   * the pieces of every op (found by its unique locality hint) lie inside it and add up to it;
//   * order: copy lists by hint, transposing lists by the op's destination address;
//   * two builds give byte-identical lists (the threaded cut is deterministic).
// Prints "ok" and exits 0, or prints the first violation and exits 1.
#include <cstdio>
#include <cstring>
#include <map>
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

#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            std::printf("FAIL %c: ", op);              \
            std::printf(__VA_ARGS__);                  \
            std::printf("\n");                         \
            return 1;                                  \
        }                                              \
    } while (0)

int main() {
    const int n = 16384;
    auto LA = layout(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n), uint64_t(1) << 40);
    auto LC = layout(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n), uint64_t(1) << 41);
    elayout a = erase(LA), c = erase(LC);
    const int64_t E = 4;
    for (char op : {'N', 'T'}) {
        job j;
        j.A = &a;
        j.C = &c;
        j.trans = op;
        const float alpha = op == 'N' ? 1.f : -0.5f, beta = op == 'N' ? 0.f : 2.f;
        std::memcpy(j.s.alpha.data(), &alpha, 4);
        std::memcpy(j.s.beta.data(), &beta, 4);
        auto p = make_plan({j}, 0, 1);
        const auto& ops = p->local_ops;
        std::vector<costa_tile_op_t> ord, ord2;
        std::vector<uint64_t> work, work2;
        const work_split w = build_work(p->dtype, ops, ord, work);
        build_work(p->dtype, ops, ord2, work2);
        CHECK(w.n_large == 0 && w.n_small == 0, "large %lld small %lld", (long long)w.n_large,
              (long long)w.n_small);
        CHECK(ord.size() == ord2.size() &&
                  std::memcmp(ord.data(), ord2.data(), ord.size() * sizeof(costa_tile_op_t)) == 0,
              "two builds differ");
        std::map<uint32_t, const costa_tile_op_t*> parent;
        for (const auto& o : ops) {
            CHECK(o.order > 0 && parent.emplace(o.order, &o).second, "hint %u not unique", o.order);
        }
        std::map<uint32_t, int64_t> area;
        uint64_t last_key = 0;
        for (int64_t i = w.tiny_first; i < w.tiny_first + w.n_tiny; ++i) {
            const costa_tile_op_t& s = ord[size_t(i)];
            const bool tr = s.flags & COSTA_TILE_TRANSPOSE;
            const int64_t bytes = tr ? int64_t(s.nf | 1) * s.ns * E : int64_t(s.nf) * s.ns * E;
            CHECK(bytes <= (tr ? 4096 : 3072), "piece %lld over budget (%lld B)", (long long)i,
                  (long long)bytes);
            auto it = parent.find(s.order);
            CHECK(it != parent.end(), "piece %lld has no parent", (long long)i);
            const costa_tile_op_t& q = *it->second;
            CHECK(s.lds == q.lds && s.ldd == q.ldd && s.src >= q.src, "piece %lld strides", (long long)i);
            const int64_t off = int64_t(s.src - q.src) / E, s0 = off / q.lds, f0 = off % q.lds;
            CHECK(f0 + s.nf <= q.nf && s0 + s.ns <= q.ns, "piece %lld outside its op", (long long)i);
            const uint64_t dst = q.dst + uint64_t((tr ? f0 * q.ldd + s0 : s0 * q.ldd + f0) * E);
            CHECK(s.dst == dst, "piece %lld destination", (long long)i);
            area[s.order] += int64_t(s.nf) * s.ns;
            const uint64_t key = tr ? q.dst : uint64_t(q.order);
            CHECK(key >= last_key, "piece %lld out of order", (long long)i);
            last_key = key;
        }
        for (const auto& o : ops)
            CHECK(area[o.order] == int64_t(o.nf) * o.ns, "op %u: pieces cover %lld of %lld", o.order,
                  (long long)area[o.order], (long long)(int64_t(o.nf) * o.ns));
        std::printf("%c: %zu ops -> %lld pieces\n", op, ops.size(), (long long)w.n_tiny);
    }
    std::printf("ok\n");
    return 0;
}
