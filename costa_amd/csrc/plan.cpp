// Tile planner: turns (A layout, C layout, op, alpha, beta) into the pack / local / unpack
// tile-op lists of one rank.
//
// Reference algorithm followed (eth-cscs/COSTA):
//   transform(): transpose A's view when op != 'N'        grid2grid/transform.cpp:162-200
//   decompose_blocks / decompose_block                     grid2grid/utils.hpp:26-115
//     cover of a block by the other grid                   grid2grid/grid_cover.cpp:54-121
//     sub-tile pointer (stored orientation)                grid2grid/block.cpp:72-111
//   message sort key (peer, tag, rows, cols, |a|,|b|,...)  communication_data.cpp:67-82,
//                                                          block.cpp:121-125
//   communication_data: local vs remote split, running     communication_data.cpp:103-164
//     offsets, per-peer counts, displacements
//   copy_to_buffer / copy_from_buffer / copy_local_blocks  communication_data.cpp:191-302
//     -> copy_and_transform normalisation                  memory_utils.hpp:330-412
// The cover is found by binary search instead of the reference's merged linear scan;
// the resulting tile set and order are identical.
#include "engine.hpp"
#include "tile_op.hpp"

#include <algorithm>
#include <cctype>
#include <complex>
#include <cstring>
#include <exception>
#include <thread>

namespace costa {
namespace engine {

size_t dtype_size(costa_dtype_t t) {
    switch (t) {
    case COSTA_FLOAT: return 4;
    case COSTA_DOUBLE: return 8;
    case COSTA_CFLOAT: return 8;
    case COSTA_CDOUBLE: return 16;
    case COSTA_INT32: return 4;
    }
    throw error(COSTA_ERR_ARG, "unknown dtype");
}

bool dtype_is_complex(costa_dtype_t t) { return t == COSTA_CFLOAT || t == COSTA_CDOUBLE; }

template <> costa_dtype_t dtype_of<float>() { return COSTA_FLOAT; }
template <> costa_dtype_t dtype_of<double>() { return COSTA_DOUBLE; }
template <> costa_dtype_t dtype_of<std::complex<float>>() { return COSTA_CFLOAT; }
template <> costa_dtype_t dtype_of<std::complex<double>>() { return COSTA_CDOUBLE; }
template <> costa_dtype_t dtype_of<int>() { return COSTA_INT32; }

template <typename T>
elayout erase(const grid_layout<T>& L) {
    elayout e;
    e.dtype = dtype_of<T>();
    const auto& g = L.grid;
    if (g.is_transposed())
        throw error(COSTA_ERR_ARG, "costa: layouts must not be left transposed by the caller");
    e.rows_split = g.grid().rows_split;
    e.cols_split = g.grid().cols_split;
    e.owners = g.reordered_owners_row_major();  // with a rank relabelling applied
    e.n_ranks = g.num_ranks();
    e.ordering = L.ordering;
    e.blocks.reserve(size_t(L.blocks.num_blocks()));
    for (int i = 0; i < L.blocks.num_blocks(); ++i) {
        const auto& b = L.blocks.get_block(i);
        if (b.transposed)
            throw error(COSTA_ERR_ARG, "costa: layouts must not be left transposed by the caller");
        e.blocks.push_back({b.rows_interval, b.cols_interval,
                            reinterpret_cast<char*>(const_cast<T*>(b.data)), b.stride});
    }
    return e;
}
template elayout erase<float>(const grid_layout<float>&);
template elayout erase<double>(const grid_layout<double>&);
template elayout erase<std::complex<float>>(const grid_layout<std::complex<float>>&);
template elayout erase<std::complex<double>>(const grid_layout<std::complex<double>>&);
template elayout erase<int>(const grid_layout<int>&);

namespace {

// ---- scalar predicates evaluated exactly as the reference does, in T's arithmetic ----
template <typename T>
T load(const std::array<unsigned char, 16>& b) {
    T v;
    std::memcpy(&v, b.data(), sizeof(T));
    return v;
}

template <typename T>
uint32_t kind_t(const scal& s, bool copy_mode, bool conj) {
    const T a = load<T>(s.alpha), b = load<T>(s.beta);
    // memcpy fast path of memory::copy (memory_utils.hpp:29-33): copy mode only
    if (copy_mode && !conj && !(std::abs(a - T{1}) > 0 || std::abs(b - T{0}) > 0))
        return COSTA_SCALE_BITCOPY;
    if (a == T{0} && b == T{0}) return COSTA_SCALE_ZERO;  // memory_utils.hpp:42-43
    if (b == T{0}) return COSTA_SCALE_ALPHA;               // :44-45
    return COSTA_SCALE_AXPBY;                              // :46-47
}

struct side_tile {
    int peer, tag;
    interval rows, cols;  // target (C) coordinates
    char* ptr;            // first element, stored orientation
    int ld;
    int n_rows, n_cols;   // stored orientation
};

bool key_less(const side_tile& x, const side_tile& y) {
    return std::tie(x.peer, x.tag, x.rows, x.cols) < std::tie(y.peer, y.tag, y.rows, y.cols);
}
bool key_equal(const side_tile& x, const side_tile& y) {
    return x.tag == y.tag && x.rows == y.rows && x.cols == y.cols;
}

// first cell of `split` overlapping index `a` (split[k] <= a < split[k+1])
int cell_of(const std::vector<int>& split, int a) {
    auto it = std::upper_bound(split.begin(), split.end(), a);
    return int(it - split.begin()) - 1;
}

// A layout seen in transform coordinates: transposed (rows <-> cols) when `t`.
struct view {
    const elayout* L;
    bool t;
    const std::vector<int>& rsplit() const { return t ? L->cols_split : L->rows_split; }
    const std::vector<int>& csplit() const { return t ? L->rows_split : L->cols_split; }
    int owner(int i, int j) const {
        int r = t ? j : i, c = t ? i : j;
        return L->owners[size_t(r) * size_t(L->nbc()) + size_t(c)];
    }
};

// decompose every local block of `src` (seen through `sv`) by the grid of `dst` (seen
// through `dv`) and append the tiles (utils.hpp:26-115)
void decompose(const view& sv, const view& dv, int tag, size_t elem, std::vector<side_tile>& out) {
    out.reserve(out.size() + sv.L->blocks.size() * 4);
    const auto& drs = dv.rsplit();
    const auto& dcs = dv.csplit();
    if (sv.rsplit().back() != drs.back() || sv.csplit().back() != dcs.back())
        throw error(COSTA_ERR_ARG, "costa::transform: layouts describe matrices of different sizes");
    const bool row_major = sv.L->ordering == 'R';
    for (const eblock& b : sv.L->blocks) {
        // block intervals in transform coordinates
        const interval vr = sv.t ? b.cols : b.rows;
        const interval vc = sv.t ? b.rows : b.cols;
        if (!vr.non_empty() || !vc.non_empty()) continue;
        const int i0 = cell_of(drs, vr.start), i1 = cell_of(drs, vr.end - 1) + 1;
        const int j0 = cell_of(dcs, vc.start), j1 = cell_of(dcs, vc.end - 1) + 1;
        for (int j = j0; j < j1; ++j) {
            const interval c(std::max(vc.start, dcs[j]), std::min(vc.end, dcs[j + 1]));
            if (c.empty()) continue;
            for (int i = i0; i < i1; ++i) {
                const interval r(std::max(vr.start, drs[i]), std::min(vr.end, drs[i + 1]));
                if (r.empty()) continue;
                // back to the stored orientation of the block (block.cpp:85-99)
                const tile_side ts = sub_tile(reinterpret_cast<uint64_t>(b.data), b.ld, b.rows.start,
                                              b.cols.start, row_major, sv.t, r.start, r.end,
                                              c.start, c.end, elem);
                out.push_back({dv.owner(i, j), tag, r, c, reinterpret_cast<char*>(ts.ptr), b.ld,
                               ts.n_rows, ts.n_cols});
            }
        }
    }
}

char upper(char c) { return char(std::toupper(static_cast<unsigned char>(c))); }

// costa_tile_op_t::order = 1 + rank of the tile in column-major order of its target
// coordinates (per tag): consecutive ranks walk down a column band, so each tile shares the
// partially used cache lines at its edges with the next one, on the source side (same source
// block) or on the destination side (same target block).
void set_order(std::vector<costa_tile_op_t>& ops, const std::vector<const side_tile*>& at) {
    // packed key (tag:16 | col start:24 | row start:24; matrix edges < 2^24) + index
    std::vector<std::pair<uint64_t, uint32_t>> k(ops.size());
    for (size_t i = 0; i < k.size(); ++i) {
        const side_tile& t = *at[i];
        k[i] = {(uint64_t(uint32_t(t.tag)) << 48) | (uint64_t(uint32_t(t.cols.start)) << 24) |
                    uint64_t(uint32_t(t.rows.start)),
                uint32_t(i)};
    }
    std::sort(k.begin(), k.end());
    for (size_t r = 0; r < k.size(); ++r) ops[k[r].second].order = uint32_t(r + 1);
}

}  // namespace

uint32_t scale_kind(costa_dtype_t dtype, const scal& s, bool copy_mode, bool conj) {
    switch (dtype) {
    case COSTA_FLOAT: return kind_t<float>(s, copy_mode, conj);
    case COSTA_DOUBLE: return kind_t<double>(s, copy_mode, conj);
    case COSTA_CFLOAT: return kind_t<std::complex<float>>(s, copy_mode, conj);
    case COSTA_CDOUBLE: return kind_t<std::complex<double>>(s, copy_mode, conj);
    case COSTA_INT32: return kind_t<int>(s, copy_mode, conj);
    }
    throw error(COSTA_ERR_ARG, "unknown dtype");
}

costa_tile_op_t make_tile_op(int n_rows, int n_cols, uint64_t src, int src_stride, bool src_cm,
                             uint64_t dst, int dst_stride, bool dst_cm, bool transpose, bool conj,
                             uint32_t kind, uint32_t slot, size_t elem) {
    return tile_op(n_rows, n_cols, src, src_stride, src_cm, dst, dst_stride, dst_cm, transpose, conj,
                   kind, slot, elem);
}

std::vector<job_params> check_jobs(const std::vector<job>& jobs, int n_ranks, costa_dtype_t& dtype) {
    if (jobs.empty()) throw error(COSTA_ERR_ARG, "costa::transform: nothing scheduled");
    if (jobs.size() > 0xFFFF) throw error(COSTA_ERR_ARG, "costa::transform: too many layout pairs");
    dtype = jobs[0].A->dtype;
    const bool cplx = dtype_is_complex(dtype);
    std::vector<job_params> out;
    for (const job& jb : jobs) {
        if (jb.A->dtype != dtype || jb.C->dtype != dtype)
            throw error(COSTA_ERR_ARG, "costa::transform: all layouts must share one element type");
        for (const elayout* L : {jb.A, jb.C})
            for (int o : L->owners)
                if (o < 0 || o >= n_ranks)
                    throw error(COSTA_ERR_ARG,
                                "costa::transform: a block owner is outside the communicator");
        const char op = upper(jb.trans);
        if (op != 'N' && op != 'T' && op != 'C')
            throw error(COSTA_ERR_ARG, "costa::transform: trans must be 'N', 'T' or 'C'");
        const bool tr = op != 'N';            // utils.cpp:9 (if_should_transpose)
        const bool cj = op == 'C' && cplx;    // communication_data.cpp:31-33
        out.push_back({tr, cj, jb.A->ordering == 'C', jb.C->ordering == 'C',
                       scale_kind(dtype, jb.s, true, cj), scale_kind(dtype, jb.s, false, cj)});
    }
    return out;
}

std::unique_ptr<plan> make_plan(const std::vector<job>& jobs, int rank, int n_ranks,
                                int loopback) {
    // loopback test mode: which of the rank's own tiles stay local
    auto stays_local = [&](const side_tile& m) {
        if (m.peer != rank) return false;
        if (loopback == 1) return false;
        if (loopback == 2) return ((m.rows.start / 7 + m.cols.start / 5) & 1) == 0;
        return true;
    };
    auto p = std::make_unique<plan>();
    p->rank = rank;
    p->n_ranks = n_ranks;
    using tag_info = job_params;
    const std::vector<tag_info> tags = check_jobs(jobs, n_ranks, p->dtype);
    const size_t E = dtype_size(p->dtype);
    std::vector<side_tile> send, recv;
    for (const job& jb : jobs) p->slots.push_back(jb.s);
    // prepare_to_send and prepare_to_recv are independent: the receive side runs on a second
    // thread when there are enough blocks to pay for it
    auto side = [&](bool send_side, std::vector<side_tile>& out) {
        for (size_t t = 0; t < jobs.size(); ++t) {
            const job& jb = jobs[t];
            const bool tr = tags[t].transpose;
            if (send_side)
                decompose(view{jb.A, tr}, view{jb.C, false}, int(t), E, out);  // prepare_to_send
            else
                decompose(view{jb.C, false}, view{jb.A, tr}, int(t), E, out);  // prepare_to_recv
        }
        std::sort(out.begin(), out.end(), key_less);
    };
    size_t n_blocks = 0;
    for (const job& jb : jobs) n_blocks += jb.A->blocks.size() + jb.C->blocks.size();
    if (n_blocks >= 4096) {
        std::exception_ptr err;
        std::thread th([&] {
            try {
                side(false, recv);
            } catch (...) {
                err = std::current_exception();
            }
        });
        try {
            side(true, send);
        } catch (...) {
            th.join();
            throw;
        }
        th.join();
        if (err) std::rethrow_exception(err);
    } else {
        side(true, send);
        side(false, recv);
    }

    p->send_counts.assign(size_t(n_ranks), 0);
    p->recv_counts.assign(size_t(n_ranks), 0);
    p->send_displs.assign(size_t(n_ranks), 0);
    p->recv_displs.assign(size_t(n_ranks), 0);

    auto kind_of = [&](const tag_info& ti, bool n_rows_cols_transposes) {
        return n_rows_cols_transposes ? ti.kind_tr : ti.kind_copy;
    };
    auto will_tr = [](const tag_info& ti, bool src_cm, bool dst_cm) {
        return (ti.transpose && src_cm == dst_cm) || (!ti.transpose && src_cm != dst_cm);
    };
    auto op_bytes = [&](const costa_tile_op_t& op) { return op_alg_bytes(op, E); };

    // target coordinates of every op, for the locality hint (costa_tile_op_t::order)
    std::vector<const side_tile*> at_pack, at_unpack, at_local;

    // ---- send side: local tiles stay, remote tiles are packed in sorted order ----
    std::vector<const side_tile*> local_src;
    int64_t off = 0;
    for (const side_tile& m : send) {
        if (stays_local(m)) {
            local_src.push_back(&m);
            continue;
        }
        const tag_info& ti = tags[size_t(m.tag)];
        const int64_t n = int64_t(m.n_rows) * m.n_cols;
        // copy_to_buffer: stored shape and ordering, dense, no transform (cpp:191-217)
        p->pack_ops.push_back(make_tile_op(m.n_rows, m.n_cols, uint64_t(m.ptr), m.ld, ti.a_cm,
                                           uint64_t(off) * E, 0, ti.a_cm, false, false,
                                           COSTA_SCALE_BITCOPY, 0, E));
        at_pack.push_back(&m);
        p->send_counts[size_t(m.peer)] += n;
        off += n;
    }
    p->send_elems = off;

    // ---- receive side ----
    std::vector<const side_tile*> local_dst;
    off = 0;
    for (const side_tile& m : recv) {
        if (stays_local(m)) {
            local_dst.push_back(&m);
            continue;
        }
        const tag_info& ti = tags[size_t(m.tag)];
        const int64_t n = int64_t(m.n_rows) * m.n_cols;
        // copy_from_buffer(idx): the buffer holds the tile in A's stored shape/ordering
        // (cpp:219-244); dims swapped back when transposing
        const int nr = ti.transpose ? m.n_cols : m.n_rows;
        const int nc = ti.transpose ? m.n_rows : m.n_cols;
        const bool wt = will_tr(ti, ti.a_cm, ti.c_cm);
        p->unpack_ops.push_back(make_tile_op(nr, nc, uint64_t(off) * E, 0, ti.a_cm, uint64_t(m.ptr),
                                             m.ld, ti.c_cm, ti.transpose, ti.conj,
                                             kind_of(ti, wt), uint32_t(m.tag), E));
        at_unpack.push_back(&m);
        p->recv_counts[size_t(m.peer)] += n;
        off += n;
    }
    p->recv_elems = off;

    // ---- local pairs (copy_local_blocks, cpp:251-302): same key order on both sides ----
    if (local_src.size() != local_dst.size())
        throw error(COSTA_ERR_INTERNAL, "costa: local tile lists of the two sides differ");
    for (size_t k = 0; k < local_src.size(); ++k) {
        const side_tile& s = *local_src[k];
        const side_tile& d = *local_dst[k];
        if (!key_equal(s, d) || int64_t(s.n_rows) * s.n_cols != int64_t(d.n_rows) * d.n_cols)
            throw error(COSTA_ERR_INTERNAL, "costa: local tiles do not pair up");
        const tag_info& ti = tags[size_t(s.tag)];
        const bool wt = will_tr(ti, ti.a_cm, ti.c_cm);
        p->local_ops.push_back(make_tile_op(s.n_rows, s.n_cols, uint64_t(s.ptr), s.ld, ti.a_cm,
                                            uint64_t(d.ptr), d.ld, ti.c_cm, ti.transpose, ti.conj,
                                            kind_of(ti, wt), uint32_t(s.tag), E));
        at_local.push_back(&d);
        p->local_elems += int64_t(s.n_rows) * s.n_cols;
    }

    for (int r = 1; r < n_ranks; ++r) {
        p->send_displs[size_t(r)] = p->send_displs[size_t(r - 1)] + p->send_counts[size_t(r - 1)];
        p->recv_displs[size_t(r)] = p->recv_displs[size_t(r - 1)] + p->recv_counts[size_t(r - 1)];
    }
    set_order(p->pack_ops, at_pack);
    set_order(p->unpack_ops, at_unpack);
    set_order(p->local_ops, at_local);
    for (auto& op : p->local_ops) p->local_bytes += op_bytes(op);
    for (auto& op : p->pack_ops) p->pack_bytes += op_bytes(op);
    for (auto& op : p->unpack_ops) p->unpack_bytes += op_bytes(op);
    return p;
}

}  // namespace engine
}  // namespace costa
