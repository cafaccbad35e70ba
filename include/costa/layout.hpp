// costa-mi355x — public C++ layout API (drop-in for COSTA's <costa/layout.hpp>).
//
// Mirrors the reference surface:
//   block_t                      reference src/costa/layout.hpp:14-19
//   custom_layout / custom_grid  reference src/costa/layout.hpp:34-49, layout.cpp:4-62
//   block_cyclic_layout / _grid  reference src/costa/layout.hpp:70-99, layout.cpp:64-138
//   grid_layout<T>               reference src/costa/grid2grid/grid_layout.hpp:8-189
//   block<T>, interval, grid2D,  reference grid2grid/block.hpp:94-170, interval.hpp,
//   assigned_grid2D                         grid2D.hpp:17-121
//
// Differences that are deliberate:
//   * all local offsets are computed in 64 bits (the reference overflows at 2^31 local
//     elements, scalapack_layout.cpp:259-266, block.cpp:92-99);
//   * the data pointers may be host memory (staged through HBM by the engine) or
//     device memory (used in place: the "device-resident" path).
#pragma once

#include <algorithm>
#include <cassert>
#include <complex>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <stdexcept>
#include <tuple>
#include <utility>
#include <vector>

namespace costa {

// half-open [start, end) range of global row or column indices
struct interval {
    int start = 0;
    int end = 0;

    interval() = default;
    interval(int s, int e) : start(s), end(e) {
        if (s < 0 || e < 0 || s > e)
            throw std::runtime_error("costa::interval: need 0 <= start <= end");
    }
    int length() const { return end - start; }
    bool contains(interval o) const { return start <= o.start && o.end <= end; }
    bool contains(int idx) const { return start <= idx && idx < end; }
    bool non_empty() const { return end > start; }
    bool empty() const { return end == start; }
    interval intersection(const interval& o) const {
        int s = std::max(start, o.start), e = std::min(end, o.end);
        if (!non_empty() || !o.non_empty() || s >= e) return {};
        return {s, e};
    }
    bool operator==(const interval& o) const {
        return empty() ? o.empty() : (start == o.start && end == o.end);
    }
    bool operator!=(const interval& o) const { return !(*this == o); }
    // lexicographic (start, end): the order the reference sorts tiles by (interval.cpp:53-56)
    bool operator<(const interval& o) const {
        return start < o.start || (start == o.start && end < o.end);
    }
};

struct block_coordinates {
    int row = 0;
    int col = 0;
    block_coordinates() = default;
    block_coordinates(int r, int c) : row(r), col(c) {}
    void transpose() { std::swap(row, col); }
};

// matrix split into an irregular grid: block (i, j) covers rows [rows_split[i], rows_split[i+1])
struct grid2D {
    int n_rows = 0;  // number of block rows
    int n_cols = 0;  // number of block columns
    std::vector<int> rows_split;
    std::vector<int> cols_split;

    grid2D() = default;
    grid2D(std::vector<int>&& r, std::vector<int>&& c)
        : n_rows(r.empty() ? 0 : int(r.size()) - 1),
          n_cols(c.empty() ? 0 : int(c.size()) - 1),
          rows_split(std::move(r)),
          cols_split(std::move(c)) {}
    interval row_interval(int i) const {
        if (i < 0 || i >= n_rows) throw std::runtime_error("costa::grid2D: row index out of range");
        return {rows_split[i], rows_split[i + 1]};
    }
    interval col_interval(int j) const {
        if (j < 0 || j >= n_cols) throw std::runtime_error("costa::grid2D: col index out of range");
        return {cols_split[j], cols_split[j + 1]};
    }
    void transpose() {
        std::swap(rows_split, cols_split);
        std::swap(n_rows, n_cols);
    }
};

// grid2D plus the owning rank of every block; owners are stored row-major
class assigned_grid2D {
  public:
    assigned_grid2D() = default;
    assigned_grid2D(grid2D&& g, std::vector<int>&& owners_row_major, int n_ranks)
        : g_(std::move(g)), owners_(std::move(owners_row_major)), n_ranks_(n_ranks) {
        if (owners_.size() != size_t(g_.n_rows) * size_t(g_.n_cols))
            throw std::runtime_error("costa::assigned_grid2D: owners size mismatch");
    }
    // reference-style constructor (grid2D.hpp:49-51)
    assigned_grid2D(grid2D&& g, std::vector<std::vector<int>>&& proc, int n_ranks)
        : g_(std::move(g)), n_ranks_(n_ranks) {
        owners_.reserve(size_t(g_.n_rows) * size_t(g_.n_cols));
        for (auto& row : proc) owners_.insert(owners_.end(), row.begin(), row.end());
        if (owners_.size() != size_t(g_.n_rows) * size_t(g_.n_cols))
            throw std::runtime_error("costa::assigned_grid2D: owners size mismatch");
    }

    // owner of block (i, j) in the CURRENT (possibly transposed) orientation, relabelled when
    // reorder_ranks was called (reference grid2D.hpp:186)
    int owner(int i, int j) const {
        int r = transposed_ ? j : i;
        int c = transposed_ ? i : j;
        int stored_cols = transposed_ ? g_.n_rows : g_.n_cols;
        return reordered_rank(owners_[size_t(r) * size_t(stored_cols) + size_t(c)]);
    }
    // rank relabelling (reference grid2D.hpp:75-79, 219-233): rank k of the grid becomes
    // reordering[k], a permutation (costa::optimal_reordering proposes one); the process of rank
    // r then holds the blocks of the rank k with reordering[k] == r (costa_hip.h)
    void reorder_ranks(const std::vector<int>& reordering) {
        if (!reordering.empty() && int(reordering.size()) < n_ranks_)
            throw std::runtime_error("costa::assigned_grid2D: reordering shorter than the ranks");
        std::vector<char> seen(reordering.size(), 0);
        for (int k : reordering) {
            if (k < 0 || k >= int(reordering.size()))
                throw std::runtime_error("costa::assigned_grid2D: reordering out of range");
            if (seen[size_t(k)]++)
                throw std::runtime_error("costa::assigned_grid2D: reordering is not a permutation");
        }
        reordering_ = reordering;
    }
    int reordered_rank(int rank) const {
        return reordering_.empty() ? rank : reordering_[size_t(rank)];
    }
    bool ranks_reordered() const noexcept { return !reordering_.empty(); }
    const grid2D& grid() const noexcept { return g_; }
    int num_ranks() const noexcept { return n_ranks_; }
    interval rows_interval(int i) const { return g_.row_interval(i); }
    interval cols_interval(int j) const { return g_.col_interval(j); }
    int block_size(int i, int j) const { return rows_interval(i).length() * cols_interval(j).length(); }
    void transpose() {
        g_.transpose();
        transposed_ = !transposed_;
    }
    bool is_transposed() const noexcept { return transposed_; }
    int num_blocks_row() const noexcept { return g_.n_rows; }
    int num_blocks_col() const noexcept { return g_.n_cols; }
    int num_rows() const noexcept { return g_.rows_split.empty() ? 0 : g_.rows_split.back(); }
    int num_cols() const noexcept { return g_.cols_split.empty() ? 0 : g_.cols_split.back(); }
    // stored owners, row-major in the stored (untransposed) orientation, before relabelling
    const std::vector<int>& owners_row_major() const noexcept { return owners_; }
    // the same with the relabelling applied (what the planner uses)
    std::vector<int> reordered_owners_row_major() const {
        if (reordering_.empty()) return owners_;
        std::vector<int> o(owners_.size());
        for (size_t k = 0; k < o.size(); ++k) o[k] = reordering_[size_t(owners_[k])];
        return o;
    }

  private:
    grid2D g_;
    std::vector<int> owners_;
    std::vector<int> reordering_;  // empty: identity
    int n_ranks_ = 0;
    bool transposed_ = false;
};

// one locally stored block: global intervals + pointer to its first element
template <typename T>
struct block {
    int tag = 0;
    interval rows_interval;
    interval cols_interval;
    block_coordinates coordinates;
    T* data = nullptr;
    int stride = 0;         // leading dimension of the local storage
    char _ordering = 'C';   // 'C' column-major, 'R' row-major local storage
    bool transposed = false;

    block() = default;
    block(interval r, interval c, block_coordinates coord, T* ptr, int ld)
        : rows_interval(r), cols_interval(c), coordinates(coord), data(ptr), stride(ld) {}

    int n_rows() const { return rows_interval.length(); }
    int n_cols() const { return cols_interval.length(); }
    std::pair<int, int> size() const { return {n_rows(), n_cols()}; }
    size_t total_size() const { return size_t(n_rows()) * size_t(n_cols()); }
    bool non_empty() const { return rows_interval.non_empty() && cols_interval.non_empty(); }

    void transpose() {
        std::swap(rows_interval, cols_interval);
        coordinates.transpose();
        transposed = !transposed;
    }
    void set_ordering(char o) {
        o = char(std::toupper(static_cast<unsigned char>(o)));
        if (o != 'R' && o != 'C') throw std::runtime_error("costa::block: ordering must be 'R' or 'C'");
        _ordering = o;
    }
    // 64-bit element offset of stored-local (li, lj) (block.cpp:127-161 semantics)
    size_t local_offset(int li, int lj) const {
        return _ordering == 'R' ? size_t(li) * size_t(stride) + size_t(lj)
                                : size_t(lj) * size_t(stride) + size_t(li);
    }
    T& local_element(int li, int lj) { return data[local_offset(li, lj)]; }
    T local_element(int li, int lj) const { return data[local_offset(li, lj)]; }
    // stored-local -> global coordinates (block.cpp:163-180)
    std::pair<int, int> local_to_global(int li, int lj) const {
        interval r = transposed ? cols_interval : rows_interval;
        interval c = transposed ? rows_interval : cols_interval;
        return {r.start + li, c.start + lj};
    }
    bool operator<(const block& o) const {
        return std::tie(tag, rows_interval, cols_interval) < std::tie(o.tag, o.rows_interval, o.cols_interval);
    }
};

template <typename T>
class local_blocks {
  public:
    local_blocks() = default;
    explicit local_blocks(std::vector<block<T>>&& b) : blocks_(std::move(b)) {
        for (const auto& x : blocks_) total_ += x.total_size();
    }
    block<T>& get_block(int i) { return blocks_[size_t(i)]; }
    const block<T>& get_block(int i) const { return blocks_[size_t(i)]; }
    int num_blocks() const { return int(blocks_.size()); }
    size_t size() const { return total_; }
    void transpose() {
        for (auto& b : blocks_) b.transpose();
    }

  private:
    std::vector<block<T>> blocks_;
    size_t total_ = 0;
};

// assigned grid + this rank's blocks + their local storage ordering
template <typename T>
class grid_layout {
  public:
    grid_layout() = default;
    grid_layout(assigned_grid2D&& g, local_blocks<T>&& b, char order)
        : grid(std::move(g)), blocks(std::move(b)) {
        ordering = char(std::toupper(static_cast<unsigned char>(order)));
        if (ordering != 'R' && ordering != 'C')
            throw std::runtime_error("costa::grid_layout: ordering must be 'R' or 'C'");
        for (int i = 0; i < blocks.num_blocks(); ++i) blocks.get_block(i).set_ordering(ordering);
    }

    int num_ranks() const { return grid.num_ranks(); }
    void transpose() {
        grid.transpose();
        blocks.transpose();
    }
    // rank relabelling of the grid (reference grid_layout.hpp:32-42)
    void reorder_ranks(const std::vector<int>& reordering) { grid.reorder_ranks(reordering); }
    int reordered_rank(int rank) const { return grid.reordered_rank(rank); }
    bool ranks_reordered() const { return grid.ranks_reordered(); }
    int num_cols() const noexcept { return grid.num_cols(); }
    int num_rows() const noexcept { return grid.num_rows(); }
    int num_blocks_col() const noexcept { return grid.num_blocks_col(); }
    int num_blocks_row() const noexcept { return grid.num_blocks_row(); }

    // host-side helpers (the data must be host-accessible), grid_layout.hpp:76-185
    template <typename F>
    void initialize(F f) {
        for_each_local([&](int gi, int gj, T& x) { x = T(f(gi, gj)); });
    }
    template <typename F>
    void apply(F f) {
        for_each_local([&](int gi, int gj, T& x) { x = T(f(gi, gj, x)); });
    }
    template <typename F>
    bool validate(F f, double tolerance = 1e-12) {
        bool ok = true;
        for_each_local([&](int gi, int gj, T& x) {
            if (std::abs(x - T(f(gi, gj))) > tolerance) ok = false;
        });
        return ok;
    }
    template <typename F>
    T accumulate(F f, T init) {
        for_each_local([&](int, int, T& x) { init = f(init, x); });
        return init;
    }

    assigned_grid2D grid;
    local_blocks<T> blocks;
    char ordering = 'C';

  private:
    template <typename F>
    void for_each_local(F&& fn) {
        for (int b = 0; b < blocks.num_blocks(); ++b) {
            auto& blk = blocks.get_block(b);
            int nr = blk.transposed ? blk.n_cols() : blk.n_rows();
            int nc = blk.transposed ? blk.n_rows() : blk.n_cols();
            for (int li = 0; li < nr; ++li)
                for (int lj = 0; lj < nc; ++lj) {
                    auto g = blk.local_to_global(li, lj);
                    fn(g.first, g.second, blk.local_element(li, lj));
                }
        }
    }
};

template <typename T>
using layout_ref = std::reference_wrapper<grid_layout<T>>;

// user description of one local block (layout.hpp:14-19)
struct block_t {
    void* data;
    int ld;
    int row;
    int col;
};

// ---- layout builders (defined in costa_amd/csrc/layout.cpp, instantiated for
//      float, double, std::complex<float>, std::complex<double>, int) ----

template <typename T>
grid_layout<T> custom_layout(int rowblocks, int colblocks, const int* rowsplit, const int* colsplit,
                             const int* owners, int nlocalblocks, const block_t* localblocks,
                             char ordering);

assigned_grid2D custom_grid(int rowblocks, int colblocks, const int* rowsplit, const int* colsplit,
                            const int* owners);

template <typename T>
grid_layout<T> block_cyclic_layout(int m, int n, int block_m, int block_n, int i, int j, int sub_m,
                                   int sub_n, int p_m, int p_n, char rank_grid_ordering, int rsrc,
                                   int csrc, T* ptr, int lld, char data_ordering, int rank);

assigned_grid2D block_cyclic_grid(int m, int n, int block_m, int block_n, int i, int j, int sub_m,
                                  int sub_n, int p_m, int p_n, char rank_grid_ordering, int rsrc,
                                  int csrc);

// ScaLAPACK helpers used by the layouts and the p?gemr2d / p?tran wrappers
namespace scalapack {
// number of rows/cols of a block-cyclically distributed dimension owned by iproc
// (same contract as ScaLAPACK NUMROC; reference scalapack.cpp:56-94)
int numroc(int n, int nb, int iproc, int isrcproc, int nprocs);
// rank id of grid coordinate (prow, pcol) for a row- ('R') or column-major ('C') rank grid
int rank_from_grid(int prow, int pcol, int p_m, int p_n, char rank_grid_ordering);
}  // namespace scalapack

}  // namespace costa
