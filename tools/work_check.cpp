// Invariants of the work lists (engine.cpp build_work), without a GPU (block addresses are never
// touched).  Run by tests/test_work_lists.py.
//   cfg 5 'N' (copy list) and 'T' (transposing list) on BASELINE cfg 5's geometry:
//     * the ops that take a sub-tiled shape are the ones the classification rules name (the
//       'T' list's aligned ops of at least half a medium sub-tile);
//     * every piece fits the wavefront budget the library uses (tiny_copy_budget,
//       tiny_lds_budget; staged pitch nf | 1);
//     * the pieces of every op (found by its unique locality hint) lie inside it and add up to it;
//     * order: by the op's destination address within at most 8 column bands (copy and
//       transposing lists alike), pack lists by the op's source address;
//     * two builds give byte-identical lists (the threaded cut is deterministic).
//   a sub-list of every 8th cfg 5 op (what one exchange round's pack / unpack list looks like:
//     hints sparse in the list, so the comparison sort replaces the counting sort): the same.
//   unaligned large ops (fp32, lld % 4 != 0): transposes into unaligned destinations take the
//     skew shape; other ops up to kUnalignedWaveCap large sub-tiles are cut into wavefront
//     pieces (the same checks), bigger ones stay on the large shape.
//   run with COSTA_MERGE=0 (ops that continue each other stay apart: every op has one parent);
//   `work_check merge` checks the merging itself; `work_check cover` that the sub-tiled work items
//   of the default lists (panels, skew XCD groups, merged ragged blocks) cover their ops exactly.
// Prints "ok" and exits 0, or prints the first violation and exits 1.
#include <chrono>
#include <complex>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <random>
#include <string>
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

template <typename T = float>
static grid_layout<T> layout(const std::vector<int>& rs, const std::vector<int>& cs, uint64_t base,
                             uint64_t gap = 0) {
    const int nr = int(rs.size()) - 1, nc = int(cs.size()) - 1;
    std::vector<int> own(size_t(nr) * size_t(nc), 0);
    std::vector<block_t> blocks;
    uint64_t off = 0;
    for (int i = 0; i < nr; ++i)
        for (int j = 0; j < nc; ++j) {
            const int rows = rs[size_t(i) + 1] - rs[size_t(i)], cols = cs[size_t(j) + 1] - cs[size_t(j)];
            blocks.push_back({reinterpret_cast<void*>(base + sizeof(T) * off), rows, i, j});
            off += (uint64_t(rows) * uint64_t(cols) + 63) / 64 * 64 + gap;
        }
    return custom_layout<T>(nr, nc, rs.data(), cs.data(), own.data(), int(blocks.size()),
                                blocks.data(), 'C');
}

#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            std::printf("FAIL %s: ", name.c_str());    \
            std::printf(__VA_ARGS__);                  \
            std::printf("\n");                         \
            return false;                              \
        }                                              \
    } while (0)

// hints of the ops the classification rules put on a sub-tiled shape: aligned ops of at least
// half a large sub-tile, unaligned ones above kUnalignedWaveCap sub-tiles, transposes into
// unaligned destinations (the skew shape, engine.cpp build_work), and in lists that transpose,
// aligned transposing ops of at least half a medium sub-tile
static std::set<uint32_t> expected_shaped(costa_dtype_t dt, const std::vector<costa_tile_op_t>& ops,
                                          bool pack = false) {
    bool tr = false;
    for (const auto& o : ops) tr = tr || (o.flags & COSTA_TILE_TRANSPOSE);
    shape_dims sh;
    tile_shapes(dt, tr, &sh);
    const int64_t E = int64_t(dtype_size(dt)), big = int64_t(sh.cf) * sh.cs, med = int64_t(sh.bf_m) * sh.bs_m;
    const uint32_t both = COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST;
    const int64_t skew_elems = int64_t(sh.bf_k) * sh.bs_k;
    std::set<uint32_t> large, medium;
    for (const auto& o0 : ops) {
        costa_tile_op_t o = o0;
        const int64_t e = int64_t(o.nf) * o.ns;
        // 4-byte sources off the grid read as 16-byte vectors (engine.cpp build_work), ops of at
        // least one large sub-tile
        if (E == 4 && e >= big && o.src % 4 == 0) o.flags |= COSTA_TILE_VEC_SRC;
        const bool al = (o.flags & both) == both, t = o.flags & COSTA_TILE_TRANSPOSE;
        const uint32_t kind = (o.flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
        const bool off_granule = o.dst % 64 != 0 || (uint64_t(o.ldd) * uint64_t(E)) % 64 != 0;
        if (skew_elems > 0 && e > 0 && t && (!(o.flags & COSTA_TILE_VEC_DST) || off_granule) &&
            o.dst % uint64_t(E) == 0 && 2 * e >= skew_elems) {
            large.insert(o.order);
            continue;
        }
        const bool tiny = (t ? int64_t(o.nf | 1) * o.ns * E <= tiny_lds_budget() : e * E <= tiny_copy_budget(E, !pack));
        const bool lg = 2 * e >= big && (al || e > kUnalignedWaveCap * big) && !tiny;
        if (lg) large.insert(o.order);
        else if (med > 0 && al && t && 2 * e >= med) medium.insert(o.order);
    }
    if (medium.size() >= 4096) large.insert(medium.begin(), medium.end());  // engine.cpp kMinMediumOps
    return large;
}

static int64_t big_elems(costa_dtype_t dt, const std::vector<costa_tile_op_t>& ops) {
    bool tr = false;
    for (const auto& o : ops) tr = tr || (o.flags & COSTA_TILE_TRANSPOSE);
    shape_dims sh;
    tile_shapes(dt, tr, &sh);
    return int64_t(sh.cf) * sh.cs;  // the large class (engine.cpp build_work)
}

// `ops` must carry unique, non-zero hints; expect_large: ops that must go to a sub-tiled shape
static bool check_list(const std::string& name, costa_dtype_t dt, const std::vector<costa_tile_op_t>& ops,
                       const std::set<uint32_t>& shaped, bool pack = false) {
    const int64_t E = int64_t(dtype_size(dt));
    std::vector<costa_tile_op_t> ord, ord2;
    std::vector<uint64_t> work, work2;
    const list_kind kind = pack ? list_pack : list_local;
    const work_split w = build_work(dt, ops, ord, work, kind);
    build_work(dt, ops, ord2, work2, kind);
    // (skew ops that continue each other are merged: fewer shaped ops than parents)
    CHECK(w.tiny_first <= int64_t(shaped.size()) && (w.tiny_first == 0) == shaped.empty(),
          "%lld ops on the sub-tiled shapes, expected %zu", (long long)w.tiny_first, shaped.size());
    CHECK(ord.size() == ord2.size() && work == work2 &&
              std::memcmp(ord.data(), ord2.data(), ord.size() * sizeof(costa_tile_op_t)) == 0,
          "two builds differ");
    std::map<uint32_t, const costa_tile_op_t*> parent;
    for (const auto& o : ops) CHECK(o.order > 0 && parent.emplace(o.order, &o).second, "hint %u not unique", o.order);
    std::map<uint32_t, int64_t> area;
    int restarts = 0;  // the large ops, then the medium ones: each run whole, in hint order
    int64_t shaped_area = 0, want_area = 0;
    for (const auto& o : ops)
        if (shaped.count(o.order)) want_area += int64_t(o.nf) * o.ns;
    for (int64_t i = 0; i < w.tiny_first; ++i) {
        const costa_tile_op_t& s = ord[size_t(i)];
        CHECK(parent.count(s.order) && shaped.count(s.order), "shaped op %lld has no shaped parent", (long long)i);
        costa_tile_op_t q = *parent[s.order];
        if (E == 4 && int64_t(q.nf) * q.ns >= big_elems(dt, ops) && q.src % 4 == 0) q.flags |= COSTA_TILE_VEC_SRC;
        // an op merged from tiles that continue each other (merge_filled / merge_adjacent, copy or
        // transpose mode) starts at the tile whose hint it keeps
        const bool merged = s.src == q.src && s.dst == q.dst && s.flags == q.flags && s.lds == q.lds &&
                            s.ldd == q.ldd && s.nf >= q.nf && s.ns >= q.ns;
        CHECK(std::memcmp(&s, &q, sizeof(s)) == 0 || merged, "shaped op %lld", (long long)i);
        restarts += i > 0 && ord[size_t(i) - 1].order > s.order;
        CHECK(restarts <= 2, "shaped op %lld out of hint order", (long long)i);
        shaped_area += int64_t(s.nf) * s.ns;
    }
    CHECK(shaped_area == want_area, "shaped ops cover %lld of %lld elements", (long long)shaped_area,
          (long long)want_area);
    uint64_t last_key = 0;
    int band_restarts = 0;
    for (int64_t i = w.tiny_first; i < w.tiny_first + w.n_tiny; ++i) {
        const costa_tile_op_t& s = ord[size_t(i)];
        const bool tr = s.flags & COSTA_TILE_TRANSPOSE;
        const int64_t bytes = tr ? int64_t(s.nf | 1) * s.ns * E : int64_t(s.nf) * s.ns * E;
        CHECK(bytes <= (tr ? tiny_lds_budget() : tiny_copy_budget(E, !pack)), "piece %lld over budget (%lld B)",
              (long long)i, (long long)bytes);
        auto it = parent.find(s.order);
        CHECK(it != parent.end(), "piece %lld has no parent", (long long)i);
        const costa_tile_op_t& q = *it->second;
        CHECK(s.lds == q.lds && s.ldd == q.ldd && s.src >= q.src, "piece %lld strides", (long long)i);
        const int64_t off = int64_t(s.src - q.src) / E, s0 = off / q.lds, f0 = off % q.lds;
        CHECK(f0 + s.nf <= q.nf && s0 + s.ns <= q.ns, "piece %lld outside its op", (long long)i);
        const uint64_t dst = q.dst + uint64_t((tr ? f0 * q.ldd + s0 : s0 * q.ldd + f0) * E);
        CHECK(s.dst == dst, "piece %lld destination", (long long)i);
        area[s.order] += int64_t(s.nf) * s.ns;
        // wave_knobs::sort 5; other lists in 8 XCD column bands (wave_knobs::xcd_bands), each
        // in destination order
        const uint64_t key = pack ? q.src : q.dst;
        if (key < last_key) ++band_restarts;
        CHECK(band_restarts <= (pack ? 0 : 7), "piece %lld out of order", (long long)i);
        last_key = key;
    }
    for (const auto& o : ops)
        CHECK(shaped.count(o.order) || area[o.order] == int64_t(o.nf) * o.ns, "op %u: pieces cover %lld of %lld",
              o.order, (long long)area[o.order], (long long)(int64_t(o.nf) * o.ns));
    std::printf("%s: %zu ops -> %lld large, %lld pieces\n", name.c_str(), ops.size(),
                (long long)w.tiny_first, (long long)w.n_tiny);
    return true;
}

static std::unique_ptr<plan> plan_of(const elayout& a, const elayout& c, char op, float alpha, float beta) {
    job j;
    j.A = &a;
    j.C = &c;
    j.trans = op;
    std::memcpy(j.s.alpha.data(), &alpha, 4);
    std::memcpy(j.s.beta.data(), &beta, 4);
    return make_plan({j}, 0, 1);
}

// merging (engine.cpp merge_adjacent, run with COSTA_MERGE unset): a 4096^2 matrix on one rank
// with 24^2 blocks, 'T' and 'N', fp32 and fp64: every tile continues its neighbours in source and
// destination, so the list becomes one op on the large shape; with a ragged last block row
// (4100^2: blocks of 24 and 20 rows) the ops still cover every element once
static bool check_merge() {
    const std::string name = "merge";
    for (int m : {4096, 4100})
        for (char op : {'T', 'N'}) {
            auto A = block_cyclic_layout<float>(m, m, 24, 24, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                                reinterpret_cast<float*>(uint64_t(1) << 40), m, 'C', 0);
            auto C = block_cyclic_layout<float>(m, m, 24, 24, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                                reinterpret_cast<float*>(uint64_t(1) << 41), m, 'C', 0);
            elayout ea = erase(A), ec = erase(C);
            auto p = plan_of(ea, ec, op, 1.f, 0.f);
            std::vector<costa_tile_op_t> ord;
            std::vector<uint64_t> work;
            const work_split w = build_work(p->dtype, p->local_ops, ord, work, list_local);
            int64_t area = 0;
            for (const auto& o : ord) area += int64_t(o.nf) * o.ns;
            // (pieces of wavefront ops are in `ord` after tiny_first; shaped ops before)
            CHECK(area == int64_t(m) * m, "%c %d: ops cover %lld of %lld elements", op, m, (long long)area,
                  (long long)int64_t(m) * m);
            // ('N' with columns off the 64-byte grid: the merged op is then cut at the granules,
            // engine.cpp granule_split -- 4 column classes, their heads as wavefront pieces)
            const bool gran = op == 'N' && (int64_t(m) * 4) % 64 != 0;
            CHECK(p->local_ops.size() > 1000 && w.tiny_first <= (gran ? 8 : 2) && (gran || w.n_tiny == 0) &&
                      w.n_large + w.n_skew > 0,
                  "%c %d: %zu tiles -> %lld shaped ops, %lld pieces", op, m, p->local_ops.size(),
                  (long long)w.tiny_first, (long long)w.n_tiny);
            std::printf("merge %c %d: %zu tiles -> %lld op(s), %lld large / %lld skew sub-tiles\n", op, m,
                        p->local_ops.size(), (long long)w.tiny_first, (long long)w.n_large, (long long)w.n_skew);
        }
    // tiles that continue each other along s only (each strip's destination elsewhere): merged
    // they would be 24-wide strips, a third of the fp64 sub-tile, so they stay apart
    std::vector<costa_tile_op_t> strips;
    const int64_t lda = 4096;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 170; ++j) {
            costa_tile_op_t o{};
            o.src = (uint64_t(1) << 40) + uint64_t((j * 24 * lda + i * 24) * 8);
            o.dst = (uint64_t(1) << 41) + (uint64_t(i) << 32) + uint64_t(j * 24 * 8);
            o.nf = o.ns = 24;
            o.lds = int32_t(lda);
            o.ldd = 8192;
            o.flags = COSTA_TILE_TRANSPOSE | COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST;
            o.order = uint32_t(strips.size() + 1);
            strips.push_back(o);
        }
    std::vector<costa_tile_op_t> ord;
    std::vector<uint64_t> work;
    const work_split w = build_work(COSTA_DOUBLE, strips, ord, work, list_unpack);
    CHECK(w.tiny_first == 0 && w.n_large == 0, "thin strips: %lld shaped ops", (long long)w.tiny_first);
    std::printf("merge: %zu tiles continuing along s only -> %lld shaped ops, %lld pieces\n", strips.size(),
                (long long)w.tiny_first, (long long)w.n_tiny);
    return true;
}

// the sub-tiled work items cover their ops exactly: every (op, sub-tile) of ordered[0, tiny_first)
// once, each class's items naming only its own ops, whatever order the sorts (hint, destination
// address, 128 KiB panels, XCD groups of the skew shape) left them in; with panels, the items walk
// the destination panel by panel
static bool check_cover(const std::string& name, costa_dtype_t dt, const std::vector<costa_tile_op_t>& ops,
                        bool expect_panels = false) {
    std::vector<costa_tile_op_t> ord;
    std::vector<uint64_t> work;
    const work_split w = build_work(dt, ops, ord, work, list_local);
    shape_dims sh;
    tile_shapes(dt, w.tr_shape, &sh);
    const int64_t E = int64_t(dtype_size(dt));
    CHECK(w.n_cblock == 0, "%lld destination-block groups (run with COSTA_CBLOCK=0)", (long long)w.n_cblock);
    CHECK(int64_t(work.size()) == w.n_large + w.n_medium + w.n_skew, "%zu work items, split %lld + %lld + %lld",
          work.size(), (long long)w.n_large, (long long)w.n_medium, (long long)w.n_skew);
    const int bfs[3][2] = {{w.sq ? sh.bf_q : sh.bf, w.sq ? sh.bs_q : sh.bs},
                           {w.med_sq ? sh.bf_s : sh.bf_m, w.med_sq ? sh.bs_s : sh.bs_m},
                           {w.skew_wide ? sh.bf_kw : sh.bf_k, w.skew_wide ? sh.bs_kw : sh.bs_k}};
    const int64_t ends[3] = {w.n_large, w.n_large + w.n_medium, w.n_large + w.n_medium + w.n_skew};
    std::vector<int> cls(size_t(w.tiny_first), -1);
    std::vector<std::vector<char>> seen(size_t(w.tiny_first));
    int64_t covered = 0, want = 0, panel_back = 0;
    for (int64_t i = 0; i < w.tiny_first; ++i) want += int64_t(ord[size_t(i)].nf) * ord[size_t(i)].ns;
    uint64_t last_panel = 0, lo = ~uint64_t(0);
    for (int64_t i = 0; i < w.tiny_first; ++i) lo = std::min(lo, ord[size_t(i)].dst);
    for (int64_t x = 0; x < int64_t(work.size()); ++x) {
        const int c = x < ends[0] ? 0 : x < ends[1] ? 1 : 2;
        const int bf = bfs[c][0], bs = bfs[c][1];
        CHECK(bf > 0 && bs > 0, "item %lld in class %d without a shape", (long long)x, c);
        const uint64_t i = work[size_t(x)] >> 32, q = work[size_t(x)] & 0xFFFFFFFFull;
        CHECK(int64_t(i) < w.tiny_first, "item %lld names op %llu past the shaped ops", (long long)x,
              (unsigned long long)i);
        const costa_tile_op_t& op = ord[size_t(i)];
        const uint64_t nbf = uint64_t((op.nf + bf - 1) / bf), n = nbf * uint64_t((op.ns + bs - 1) / bs);
        CHECK(cls[i] == -1 || cls[i] == c, "op %llu in two classes", (unsigned long long)i);
        cls[i] = c;
        if (seen[i].empty()) seen[i].assign(size_t(n), 0);
        CHECK(q < n && !seen[i][q], "op %llu sub-tile %llu (of %llu) twice or out of range", (unsigned long long)i,
              (unsigned long long)q, (unsigned long long)n);
        seen[i][q] = 1;
        const int64_t f0 = int64_t(q % nbf) * bf, s0 = int64_t(q / nbf) * bs;
        covered += std::min<int64_t>(bf, op.nf - f0) * std::min<int64_t>(bs, op.ns - s0);
        if (expect_panels && c == 0) {  // engine.cpp build_work: 128 KiB panels of destination rows
            const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
            const uint64_t e = (op.dst - lo) / uint64_t(E) +uint64_t(tr ? f0 * op.ldd + s0 : s0 * op.ldd + f0);
            const uint64_t panel = (e % uint64_t(op.ldd)) / uint64_t((int64_t(128) << 10) / E);
            panel_back += panel < last_panel;
            last_panel = panel;
        }
    }
    CHECK(covered == want, "sub-tiles cover %lld of %lld elements", (long long)covered, (long long)want);
    for (int64_t i = 0; i < w.tiny_first; ++i) CHECK(cls[size_t(i)] >= 0, "op %lld has no work item", (long long)i);
    CHECK(!expect_panels || panel_back == 0,"%lld steps back to an earlier panel", (long long)panel_back);
    std::printf("cover %s: %lld shaped ops -> %zu items (%lld large, %lld medium, %lld skew)%s\n", name.c_str(),
                (long long)w.tiny_first, work.size(), (long long)w.n_large, (long long)w.n_medium,
                (long long)w.n_skew, expect_panels ? ", panels" : "");
    return true;
}

// destination-block groups (engine.cpp cblock_groups): every group's ops tile its R x K range
// exactly once (ldd = R, inside the range, no element twice, one transform), and together with
// the shaped ops and the wavefront pieces every op of the list is covered exactly (by its hint)
static bool check_cblock(const std::string& name, costa_dtype_t dt, const std::vector<costa_tile_op_t>& ops,
                         list_kind kind, bool expect_groups) {
    std::vector<costa_tile_op_t> ord;
    std::vector<uint64_t> work;
    const work_split w = build_work(dt, ops, ord, work, kind);
    const int64_t E = int64_t(dtype_size(dt));
    const uint32_t vec_bits = COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST;
    CHECK(int64_t(work.size()) == w.n_large + w.n_medium + w.n_skew + w.n_cblock, "%zu work items", work.size());
    CHECK(!expect_groups || w.n_cblock > 0, "no destination-block group");
    std::map<uint32_t, int64_t> area;
    int64_t lds = 0, grouped = 0, first = INT64_MAX;
    uint64_t last = 0;
    for (int64_t x = w.n_large + w.n_medium + w.n_skew; x < int64_t(work.size()); ++x) {
        const uint64_t h = work[size_t(x)];
        CHECK(h < uint64_t(w.tiny_first), "group header %llu past the groups", (unsigned long long)h);
        first = std::min(first, int64_t(h));
        const costa_tile_op_t& hd = ord[size_t(h)];
        const int64_t R = hd.nf, K = hd.ns, n = int64_t(hd.src);
        // (a range off the 16-byte grid needs up to V - 1 more elements of whole vectors)
        CHECK(R > 0 && K > 0 && n >= 1 && hd.ldd == R && R * K + 16 / E - 1 <= cblock_max_elems(E),
              "group %lld shape", (long long)x);
        // destination order (with XCD column bands: inside each of the 8 slices of the kernel's sizes)
        const int64_t gi = x - (w.n_large + w.n_medium + w.n_skew), ng = w.n_cblock;
        const bool slice_start = w.cb_map == cb_xcd_bands &&
                                 (gi < (ng % 8) * (ng / 8 + 1) ? gi % (ng / 8 + 1) == 0
                                                               : ng / 8 > 0 && (gi - (ng % 8) * (ng / 8 + 1)) % (ng / 8) == 0);
        CHECK(slice_start || hd.dst >= last, "group %lld out of destination order", (long long)x);
        last = hd.dst;
        lds = std::max(lds, (R | 1) * K);
        std::vector<char> cov(size_t(R * K), 0);
        for (int64_t i = 0; i < n; ++i) {
            const costa_tile_op_t& op = ord[size_t(h) + 1 + size_t(i)];
            const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
            const int64_t run = tr ? op.ns : op.nf, runs = tr ? op.nf : op.ns;
            CHECK(op.ldd == R && (op.flags & ~vec_bits) == hd.flags && op.dst >= hd.dst, "group %lld op %lld", (long long)x,
                  (long long)i);
            const int64_t e = int64_t(op.dst - hd.dst) / E, r0 = e % R, c0 = e / R;
            CHECK(r0 + run <= R && c0 + runs <= K, "group %lld op %lld outside the range", (long long)x, (long long)i);
            for (int64_t c = c0; c < c0 + runs; ++c)
                for (int64_t r = r0; r < r0 + run; ++r) {
                    CHECK(!cov[size_t(c * R + r)], "group %lld: element (%lld, %lld) twice", (long long)x, (long long)r,
                          (long long)c);
                    cov[size_t(c * R + r)] = 1;
                }
            area[op.order] += int64_t(op.nf) * op.ns;
            grouped += int64_t(op.nf) * op.ns;
        }
        for (char v : cov) CHECK(v, "group %lld not covered", (long long)x);
    }
    CHECK(lds == w.cblock_lds, "LDS image %lld, split says %lld", (long long)lds, (long long)w.cblock_lds);
    for (int64_t i = 0; i < std::min<int64_t>(first, w.tiny_first); ++i) area[ord[size_t(i)].order] += int64_t(ord[size_t(i)].nf) * ord[size_t(i)].ns;
    for (int64_t i = w.tiny_first; i < w.tiny_first + w.n_tiny; ++i) area[ord[size_t(i)].order] += int64_t(ord[size_t(i)].nf) * ord[size_t(i)].ns;
    for (const auto& o : ops)
        CHECK(area[o.order] == int64_t(o.nf) * o.ns, "op %u covered %lld of %lld", o.order, (long long)area[o.order],
              (long long)(int64_t(o.nf) * o.ns));
    std::printf("cblock %s: %zu ops -> %lld groups holding %lld elements, %lld pieces, LDS %lld elements\n", name.c_str(),
                ops.size(), (long long)w.n_cblock, (long long)grouped, (long long)w.n_tiny, (long long)lds);
    return true;
}

// the destination-block groups' XCD chunk order (engine.hpp cblock_xcd_order) is a permutation of
// the launch, whatever its size
static bool check_xcd() {
    const std::string name = "xcd order";
    for (int64_t nb = 1; nb <= 4096; ++nb) {
        std::vector<char> seen(size_t(nb), 0);
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t g = cblock_xcd_order(b, nb);
            CHECK(g >= 0 && g < nb && !seen[size_t(g)], "nb %lld, b %lld -> %lld", (long long)nb, (long long)b,
                  (long long)g);
            seen[size_t(g)] = 1;
        }
        // and so is the slice order (xcd_slice_order), XCD b mod 8 inside slice b mod 8
        std::vector<char> seen2(size_t(nb), 0);
        for (int64_t b = 0; b < nb; ++b) {
            const int64_t g = xcd_slice_order(b, nb);
            const int64_t x = b % 8, lo = x < nb % 8 ? x * (nb / 8 + 1) : (nb % 8) * (nb / 8 + 1) + (x - nb % 8) * (nb / 8);
            CHECK(g >= 0 && g < nb && !seen2[size_t(g)] && g >= lo && g < lo + nb / 8 + (x < nb % 8),
                  "slice order: nb %lld, b %lld -> %lld", (long long)nb, (long long)b, (long long)g);
            seen2[size_t(g)] = 1;
        }
    }
    return true;
}

static bool check_cblocks() {
    const int n = 16384;
    auto LA = layout(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n), uint64_t(1) << 40);
    auto LC = layout(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n), uint64_t(1) << 41);
    elayout a = erase(LA), c = erase(LC);
    for (char op : {'N', 'T'}) {
        auto p = plan_of(a, c, op, op == 'N' ? 1.f : -0.5f, op == 'N' ? 0.f : 2.f);
        if (!check_cblock(std::string("cfg5 ") + op, p->dtype, p->local_ops, list_local, true)) return false;
        if (!check_cblock(std::string("cfg5 unpack-list ") + op, p->dtype, p->local_ops, list_unpack, true)) return false;
        // every 8th op: the ranges are no longer covered, so no group forms
        std::vector<costa_tile_op_t> sub;
        for (size_t i = 0; i < p->local_ops.size(); i += 8) sub.push_back(p->local_ops[i]);
        if (!check_cblock(std::string("cfg5 sub-list ") + op, p->dtype, sub, list_local, false)) return false;
    }
    // C blocks of 200 x 200 fp64 (over the budget: cut into column bands) and blocks separated by
    // gaps, fed by 24 x 24 A blocks
    // (gap 3: every block after the first starts off the 16-byte grid, as in test_gpu_cblock.py)
    auto LA2 = layout<double>(splits(7, 20, 28, 2000), splits(8, 20, 28, 2000), uint64_t(1) << 40);
    auto LC2 = layout<double>(splits(9, 150, 250, 2000), splits(10, 150, 250, 2000), uint64_t(1) << 41, 3);
    elayout a2 = erase(LA2), c2 = erase(LC2);
    for (char op : {'N', 'T'}) {
        job j{&a2, &c2, op, {}};
        const double one = 1.0, zero = 0.0;
        std::memcpy(j.s.alpha.data(), &one, 8);
        std::memcpy(j.s.beta.data(), &zero, 8);
        auto p = make_plan({j}, 0, 1);
        if (!check_cblock(std::string("fp64 bands ") + op, p->dtype, p->local_ops, list_local, true)) return false;
    }
    return true;
}

template <typename T>
static std::unique_ptr<plan> square_plan(int m, int nb, int lld, char op) {
    auto A = block_cyclic_layout<T>(m, m, nb, nb, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                    reinterpret_cast<T*>(uint64_t(1) << 40), lld, 'C', 0);
    auto C = block_cyclic_layout<T>(m, m, nb, nb, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                    reinterpret_cast<T*>(uint64_t(1) << 42), lld, 'C', 0);
    elayout ea = erase(A), ec = erase(C);
    job j{&ea, &ec, op, {}};
    const T one = T(1), zero = T(0);
    std::memcpy(j.s.alpha.data(), &one, sizeof(T));
    std::memcpy(j.s.beta.data(), &zero, sizeof(T));
    return make_plan({j}, 0, 1);
}

// copies into destinations off the 64-byte grid cut at the granules (engine.cpp granule_split,
// run with COSTA_TUNING=1 COSTA_COPY_GRANULE=1): every destination element is written exactly once,
// from the source element of the same (row, column); the sub-tiled ops start every destination
// column on a 64-byte granule
template <typename T>
static bool check_granule_case(int m, int nb, int lda, int ldc, T beta) {
    const std::string name = "granule";
    const int64_t E = int64_t(sizeof(T));
    const uint64_t A0 = uint64_t(1) << 40, C0 = uint64_t(1) << 42;
    auto A = block_cyclic_layout<T>(m, m, nb, nb, 1, 1, m, m, 1, 1, 'R', 0, 0, reinterpret_cast<T*>(A0), lda, 'C', 0);
    auto C = block_cyclic_layout<T>(m, m, nb, nb, 1, 1, m, m, 1, 1, 'R', 0, 0, reinterpret_cast<T*>(C0), ldc, 'C', 0);
    elayout ea = erase(A), ec = erase(C);
    job j{&ea, &ec, 'N', {}};
    const T one = T(1);
    std::memcpy(j.s.alpha.data(), &one, sizeof(T));
    std::memcpy(j.s.beta.data(), &beta, sizeof(T));
    auto p = make_plan({j}, 0, 1);
    std::vector<costa_tile_op_t> ord;
    std::vector<uint64_t> work;
    const work_split w = build_work(p->dtype, p->local_ops, ord, work, list_local);
    std::vector<char> hit(size_t(ldc) * size_t(m), 0);
    int64_t aligned_ops = 0;
    auto walk = [&](const costa_tile_op_t& o) {
        CHECK(!(o.flags & COSTA_TILE_TRANSPOSE), "a copy became a transpose");
        for (int64_t s = 0; s < o.ns; ++s)
            for (int64_t f = 0; f < o.nf; ++f) {
                const int64_t ea_ = int64_t(o.src - A0) / E + s * o.lds + f;
                const int64_t ec_ = int64_t(o.dst - C0) / E + s * o.ldd + f;
                const int64_t i = ea_ % lda, jj = ea_ / lda;
                CHECK(i < m && jj < m && ec_ == i + jj * int64_t(ldc), "element (%lld, %lld) misplaced", (long long)i,
                      (long long)jj);
                CHECK(!hit[size_t(ec_)], "element (%lld, %lld) written twice", (long long)i, (long long)jj);
                hit[size_t(ec_)] = 1;
            }
        return true;
    };
    for (int64_t i = 0; i < w.tiny_first; ++i) {
        const costa_tile_op_t& o = ord[size_t(i)];
        if (!walk(o)) return false;
        // every sub-tiled op's destination columns start on a granule
        CHECK(o.dst % 64 == 0 && (uint64_t(o.ldd) * uint64_t(E)) % 64 == 0, "sub-tiled op %lld off the granules",
              (long long)i);
        ++aligned_ops;
    }
    for (int64_t i = w.tiny_first; i < w.tiny_first + w.n_tiny; ++i)
        if (!walk(ord[size_t(i)])) return false;
    int64_t n_hit = 0;
    for (char h : hit) n_hit += h;
    CHECK(n_hit == int64_t(m) * m, "%lld of %lld elements written", (long long)n_hit, (long long)int64_t(m) * m);
    CHECK(aligned_ops > 0, "no sub-tiled op");
    std::printf("granule E=%lld lda %d ldc %d: %lld sub-tiled ops (granule-aligned), %lld large items, %lld pieces\n",
                (long long)E, lda, ldc, (long long)aligned_ops, (long long)w.n_large, (long long)w.n_tiny);
    return true;
}

static bool check_granule() {
    for (int pad : {1, 2, 3, 8})
        if (!check_granule_case<double>(2048, 256, 2048, 2048 + pad, 0.0) ||
            !check_granule_case<double>(2048, 256, 2048 + pad, 2048 + pad, 2.0))
            return false;
    for (int pad : {1, 4, 8, 24})
        if (!check_granule_case<float>(2048, 256, 2048, 2048 + pad, 0.f) ||
            !check_granule_case<float>(2048, 200, 2048 + 3, 2048 + pad, 0.5f))
            return false;
    return check_granule_case<int>(2048, 256, 2048, 2051, 0);
}

static bool check_covers() {
    using z = std::complex<double>;
    struct g {
        const char* name;
        std::unique_ptr<plan> p;
        bool panels;
    };
    std::vector<g> gs;
    gs.push_back({"fp64 32768^2 256^2 'T'", square_plan<double>(32768, 256, 32768, 'T'), true});
    gs.push_back({"fp64 16384^2 256^2 'T'", square_plan<double>(16384, 256, 16384, 'T'), false});
    gs.push_back({"c128 32768^2 128^2 'T'", square_plan<z>(32768, 128, 32768, 'T'), true});
    gs.push_back({"c128 8192^2 80^2 'T' (merged)", square_plan<z>(8192, 80, 8192, 'T'), false});
    gs.push_back({"fp64 8192^2 100^2 'N' (merged)", square_plan<double>(8192, 100, 8192, 'N'), false});
    gs.push_back({"fp32 4096^2 256^2 'T' lld 4097 (skew)", square_plan<float>(4096, 256, 4097, 'T'), false});
    gs.push_back({"fp64 8192^2 32^2 'T' lld 8196 (skew)", square_plan<double>(8192, 32, 8196, 'T'), false});
    {
        // eight separate 32768 x 4096 column strips of A (no merging) into one 32768^2 C: 'T'
        // writes 256 KiB destination columns, walked in panels across the eight ops
        std::vector<int> rs{0, 32768}, cs;
        for (int j = 0; j <= 8; ++j) cs.push_back(4096 * j);
        auto A = layout<double>(rs, cs, uint64_t(1) << 40, 64);
        auto C = block_cyclic_layout<double>(32768, 32768, 32768, 32768, 1, 1, 32768, 32768, 1, 1, 'R', 0, 0,
                                             reinterpret_cast<double*>(uint64_t(1) << 42), 32768, 'C', 0);
        elayout ea = erase(A), ec = erase(C);
        job j{&ea, &ec, 'T', {}};
        const double one = 1.0, zero = 0.0;
        std::memcpy(j.s.alpha.data(), &one, 8);
        std::memcpy(j.s.beta.data(), &zero, 8);
        gs.push_back({"fp64 8 strips 32768 x 4096 'T'", make_plan({j}, 0, 1), true});
    }
    for (const auto& x : gs)
        if (!check_cover(x.name, x.p->dtype, x.p->local_ops, x.panels)) return false;
    const int n = 16384;
    auto LA = layout(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n), uint64_t(1) << 40);
    auto LC = layout(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n), uint64_t(1) << 41);
    elayout a = erase(LA), c = erase(LC);
    for (char op : {'N', 'T'}) {
        auto p = plan_of(a, c, op, 1.f, 0.f);
        if (!check_cover(std::string("cfg5 ") + op, p->dtype, p->local_ops)) return false;
    }
    return true;
}

// FNV-1a over the work lists of a set of geometries (cfg 5 'N' / 'T', cfg 2's 256^2 fp64 'T',
// cfg 4's 128^2 c128 'T' with alpha / beta, 24^2 fp32 blocks that merge, fp32 with lld 4097):
// `work_check digest` prints it, so that tests/test_work_lists.py can compare builds of the
// library under different environments
static uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}
static uint64_t digest_of(uint64_t h, const plan& p) {
    for (int kind = 0; kind < 3; ++kind) {
        const auto& ops = kind == 0 ? p.local_ops : kind == 1 ? p.pack_ops : p.unpack_ops;
        std::vector<costa_tile_op_t> ord;
        std::vector<uint64_t> work;
        const work_split w = build_work(p.dtype, ops, ord, work, kind == 0 ? list_local : kind == 1 ? list_pack : list_unpack);
        h = fnv(h, ord.data(), ord.size() * sizeof(costa_tile_op_t));
        h = fnv(h, work.data(), work.size() * sizeof(uint64_t));
        h = fnv(h, &w, sizeof(w));
    }
    return h;
}
static int digest() {
    uint64_t h = 0xcbf29ce484222325ull;
    const int n = 16384;
    auto LA = layout(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n), uint64_t(1) << 40);
    auto LC = layout(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n), uint64_t(1) << 41);
    elayout a = erase(LA), c = erase(LC);
    for (char op : {'N', 'T'}) h = digest_of(h, *plan_of(a, c, op, op == 'N' ? 1.f : -0.5f, op == 'N' ? 0.f : 2.f));
    {
        auto A = block_cyclic_layout<double>(n, n, 256, 256, 1, 1, n, n, 1, 1, 'R', 0, 0,
                                             reinterpret_cast<double*>(uint64_t(1) << 40), n, 'C', 0);
        auto C = block_cyclic_layout<double>(n, n, 256, 256, 1, 1, n, n, 1, 1, 'R', 0, 0,
                                             reinterpret_cast<double*>(uint64_t(1) << 41), n, 'C', 0);
        elayout ea = erase(A), ec = erase(C);
        job j{&ea, &ec, 'T', {}};
        const double one = 1.0, zero = 0.0;
        std::memcpy(j.s.alpha.data(), &one, 8);
        std::memcpy(j.s.beta.data(), &zero, 8);
        h = digest_of(h, *make_plan({j}, 0, 1));
    }
    {
        using z = std::complex<double>;
        const int m = 8192;
        auto A = block_cyclic_layout<z>(m, m, 128, 128, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                        reinterpret_cast<z*>(uint64_t(1) << 40), m, 'C', 0);
        auto C = block_cyclic_layout<z>(m, m, 128, 128, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                        reinterpret_cast<z*>(uint64_t(1) << 41), m, 'C', 0);
        elayout ea = erase(A), ec = erase(C);
        job j{&ea, &ec, 'T', {}};
        const z al(0.75, -0.5), be(1.25, 0.25);
        std::memcpy(j.s.alpha.data(), &al, 16);
        std::memcpy(j.s.beta.data(), &be, 16);
        h = digest_of(h, *make_plan({j}, 0, 1));
    }
    for (int lld : {4096, 4097}) {
        const int m = 4096, nb = lld == m ? 24 : 256;
        auto A = block_cyclic_layout<float>(m, m, nb, nb, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                            reinterpret_cast<float*>(uint64_t(1) << 40), lld, 'C', 0);
        auto C = block_cyclic_layout<float>(m, m, nb, nb, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                            reinterpret_cast<float*>(uint64_t(1) << 41), lld, 'C', 0);
        elayout ea = erase(A), ec = erase(C);
        for (char op : {'T', 'N'}) h = digest_of(h, *plan_of(ea, ec, op, 1.f, 0.f));
    }
    std::printf("digest %016llx\n", (unsigned long long)h);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && std::string(argv[1]) == "digest") return digest();
    if (argc > 1 && std::string(argv[1]) == "time") {  // build_work on cfg 5's 'N' list (host cost)
        const int n = 16384;
        auto LA = layout(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n), uint64_t(1) << 40);
        auto LC = layout(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n), uint64_t(1) << 41);
        elayout a = erase(LA), c = erase(LC);
        auto p = plan_of(a, c, 'N', 1.f, 0.f);
        std::vector<costa_tile_op_t> ord;
        std::vector<uint64_t> work;
        build_work(p->dtype, p->local_ops, ord, work, list_local);
        const auto t0 = std::chrono::steady_clock::now();
        for (int k = 0; k < 5; ++k) build_work(p->dtype, p->local_ops, ord, work, list_local);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count() / 5;
        std::printf("build_work cfg 5 'N' (%zu ops): %.2f ms\n", p->local_ops.size(), ms);
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "cover") {
        if (!check_covers()) return 1;
        std::printf("ok\n");
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "granule") {
        if (!check_granule()) return 1;
        std::printf("ok\n");
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "xcd") {
        if (!check_xcd()) return 1;
        std::printf("ok\n");
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "cblock") {
        if (!check_cblocks()) return 1;
        std::printf("ok\n");
        return 0;
    }
    if (argc > 1 && std::string(argv[1]) == "merge") {
        if (!check_merge()) return 1;
        std::printf("ok\n");
        return 0;
    }
    const int n = 16384;
    auto LA = layout(splits(0xC5A1, 8, 96, n), splits(0xC5A2, 8, 96, n), uint64_t(1) << 40);
    auto LC = layout(splits(0xC5A3, 16, 160, n), splits(0xC5A4, 16, 160, n), uint64_t(1) << 41);
    elayout a = erase(LA), c = erase(LC);
    for (char op : {'N', 'T'}) {
        auto p = plan_of(a, c, op, op == 'N' ? 1.f : -0.5f, op == 'N' ? 0.f : 2.f);
        const std::set<uint32_t> shaped = expected_shaped(p->dtype, p->local_ops);
        if (!check_list(std::string("cfg5 ") + op, p->dtype, p->local_ops, shaped)) return 1;
        // one exchange round's share of a list: every 8th op (hints sparse)
        std::vector<costa_tile_op_t> sub;
        for (size_t i = 0; i < p->local_ops.size(); i += 8) sub.push_back(p->local_ops[i]);
        if (!check_list(std::string("cfg5 sub-list ") + op, p->dtype, sub, expected_shaped(p->dtype, sub)))
            return 1;
        // the same as a pack list (wavefront ops by source address)
        if (!check_list(std::string("cfg5 pack sub-list ") + op, p->dtype, sub, expected_shaped(p->dtype, sub, true), true))
            return 1;
    }
    // unaligned large ops: fp32 4096^2 'T' with lld = 4097 (columns 4-byte aligned only)
    for (int nb : {256, 1024}) {
        const int m = 4096, lld = m + 1;
        auto A = block_cyclic_layout<float>(m, m, nb, nb, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                            reinterpret_cast<float*>(uint64_t(1) << 40), lld, 'C', 0);
        auto C = block_cyclic_layout<float>(m, m, nb, nb, 1, 1, m, m, 1, 1, 'R', 0, 0,
                                            reinterpret_cast<float*>(uint64_t(1) << 41), lld, 'C', 0);
        elayout ea = erase(A), ec = erase(C);
        auto p = plan_of(ea, ec, 'T', 1.f, 0.f);
        shape_dims sh;
        tile_shapes(COSTA_FLOAT, true, &sh);  // a transposing list
        // every op transposes into unaligned destination columns: the skew shape, whatever its size
        const std::set<uint32_t> expect = expected_shaped(p->dtype, p->local_ops);
        if (expect.size() != p->local_ops.size()) {
            std::printf("FAIL unaligned %d^2 blocks: %zu of %zu ops expected on the skew shape\n", nb,
                        expect.size(), p->local_ops.size());
            return 1;
        }
        if (!check_list("unaligned " + std::to_string(nb) + "^2 blocks", p->dtype, p->local_ops, expect))
            return 1;
    }
    std::printf("ok\n");
    return 0;
}
