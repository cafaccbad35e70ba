// Layout builders: ScaLAPACK block-cyclic and user-defined ("custom") layouts.
//
// Behaviour follows the reference:
//   custom_grid / custom_layout       src/costa/layout.cpp:4-62
//   block_cyclic_grid / _layout       src/costa/layout.cpp:64-138
//     -> get_scalapack_layout         src/costa/grid2grid/scalapack_layout.cpp:178-285
//     -> line_split                   scalapack_layout.cpp:152-177
//     -> rank_from_grid               scalapack_layout.cpp:40-56
//   numroc                            src/costa/scalapack.cpp:56-94
// but every local offset is 64-bit.
#include <costa/layout.hpp>

#include <cctype>
#include <complex>
#include <string>

namespace costa {
namespace {

char upper(char c) { return char(std::toupper(static_cast<unsigned char>(c))); }

// Split ticks of the rows (or columns) of a submatrix that starts at 0-based global
// index `begin` and ends (exclusive) at `end`, relative to `begin`: the first tick
// is 0, the first block may be partial (begin not on a block edge), the last too.
std::vector<int> submatrix_ticks(int begin, int end, int nb) {
    std::vector<int> t{0};
    const int len = end - begin;
    const int first = nb - begin % nb;  // rows left in the block `begin` falls in
    if (first >= len) {
        t.push_back(len);
        return t;
    }
    t.push_back(first);
    while (t.back() + nb < len) t.push_back(t.back() + nb);
    if (t.back() != len) t.push_back(len);
    return t;
}

struct bc_geometry {
    std::vector<int> rows, cols;   // submatrix-relative split ticks
    std::vector<int> owners;       // row-major owners of the submatrix blocks
    int first_blk_row = 0;         // global block index of the submatrix's first block row
    int first_blk_col = 0;
    int ia0 = 0, ja0 = 0;          // 0-based submatrix start
};

bc_geometry bc_build(int m, int n, int mb, int nb, int ia, int ja, int sub_m, int sub_n, int p_m,
                     int p_n, char rank_order, int rsrc, int csrc) {
    if (mb <= 0 || nb <= 0 || p_m <= 0 || p_n <= 0)
        throw std::runtime_error("costa::block_cyclic: block and grid sizes must be positive");
    if (ia < 1 || ja < 1) throw std::runtime_error("costa::block_cyclic: i, j are 1-based");
    if (sub_m < 0 || sub_n < 0 || ia - 1 + sub_m > m || ja - 1 + sub_n > n)
        throw std::runtime_error("costa::block_cyclic: submatrix outside the global matrix");
    rank_order = upper(rank_order);
    if (rank_order != 'R' && rank_order != 'C')
        throw std::runtime_error("costa::block_cyclic: rank grid ordering must be 'R' or 'C'");
    if (rsrc < 0 || rsrc >= p_m || csrc < 0 || csrc >= p_n)
        throw std::runtime_error("costa::block_cyclic: rsrc/csrc outside the rank grid");

    bc_geometry g;
    g.ia0 = ia - 1;
    g.ja0 = ja - 1;
    g.rows = submatrix_ticks(g.ia0, g.ia0 + sub_m, mb);
    g.cols = submatrix_ticks(g.ja0, g.ja0 + sub_n, nb);
    g.first_blk_row = g.ia0 / mb;
    g.first_blk_col = g.ja0 / nb;
    const int nbr = int(g.rows.size()) - 1, nbc = int(g.cols.size()) - 1;
    // rank coordinate owning the submatrix's first block (scalapack_layout.cpp:220-226)
    const int prow0 = (g.first_blk_row % p_m + rsrc) % p_m;
    const int pcol0 = (g.first_blk_col % p_n + csrc) % p_n;
    g.owners.resize(size_t(nbr) * size_t(nbc));
    for (int i = 0; i < nbr; ++i)
        for (int j = 0; j < nbc; ++j)
            g.owners[size_t(i) * nbc + j] =
                scalapack::rank_from_grid((i % p_m + prow0) % p_m, (j % p_n + pcol0) % p_n, p_m,
                                          p_n, rank_order);
    return g;
}

}  // namespace

namespace scalapack {

int numroc(int n, int nb, int iproc, int isrcproc, int nprocs) {
    const int dist = (nprocs + iproc - isrcproc) % nprocs;  // distance from the source process
    const int nblocks = n / nb;
    int len = (nblocks / nprocs) * nb;
    const int extra = nblocks % nprocs;
    if (dist < extra)
        len += nb;
    else if (dist == extra)
        len += n % nb;
    return len;
}

int rank_from_grid(int prow, int pcol, int p_m, int p_n, char order) {
    if (prow < 0 || prow >= p_m || pcol < 0 || pcol >= p_n)
        throw std::runtime_error("costa::rank_from_grid: coordinates outside the rank grid");
    return upper(order) == 'C' ? pcol * p_m + prow : prow * p_n + pcol;
}

}  // namespace scalapack

assigned_grid2D custom_grid(int rowblocks, int colblocks, const int* rowsplit, const int* colsplit,
                            const int* owners) {
    if (rowblocks < 0 || colblocks < 0)
        throw std::runtime_error("costa::custom_grid: negative block counts");
    std::vector<int> r(rowsplit, rowsplit + rowblocks + 1);
    std::vector<int> c(colsplit, colsplit + colblocks + 1);
    for (size_t k = 1; k < r.size(); ++k)
        if (r[k] < r[k - 1]) throw std::runtime_error("costa::custom_grid: rowsplit not sorted");
    for (size_t k = 1; k < c.size(); ++k)
        if (c[k] < c[k - 1]) throw std::runtime_error("costa::custom_grid: colsplit not sorted");
    std::vector<int> own(owners, owners + size_t(rowblocks) * size_t(colblocks));
    int n_ranks = 1;  // as the reference: max owner + 1, at least 1 (layout.cpp:16-24)
    for (int o : own) {
        if (o < 0) throw std::runtime_error("costa::custom_grid: negative owner");
        n_ranks = std::max(n_ranks, o + 1);
    }
    return assigned_grid2D(grid2D(std::move(r), std::move(c)), std::move(own), n_ranks);
}

template <typename T>
grid_layout<T> custom_layout(int rowblocks, int colblocks, const int* rowsplit, const int* colsplit,
                             const int* owners, int nlocalblocks, const block_t* localblocks,
                             char ordering) {
    auto grid = custom_grid(rowblocks, colblocks, rowsplit, colsplit, owners);
    std::vector<block<T>> blks;
    blks.reserve(size_t(std::max(nlocalblocks, 0)));
    for (int k = 0; k < nlocalblocks; ++k) {
        const block_t& b = localblocks[k];
        if (b.row < 0 || b.row >= rowblocks || b.col < 0 || b.col >= colblocks)
            throw std::runtime_error("costa::custom_layout: block coordinates outside the grid");
        blks.emplace_back(interval(rowsplit[b.row], rowsplit[b.row + 1]),
                          interval(colsplit[b.col], colsplit[b.col + 1]),
                          block_coordinates(b.row, b.col), static_cast<T*>(b.data), b.ld);
    }
    return grid_layout<T>(std::move(grid), local_blocks<T>(std::move(blks)), ordering);
}

assigned_grid2D block_cyclic_grid(int m, int n, int mb, int nb, int ia, int ja, int sub_m,
                                  int sub_n, int p_m, int p_n, char rank_order, int rsrc,
                                  int csrc) {
    auto g = bc_build(m, n, mb, nb, ia, ja, sub_m, sub_n, p_m, p_n, rank_order, rsrc, csrc);
    return assigned_grid2D(grid2D(std::move(g.rows), std::move(g.cols)), std::move(g.owners),
                           p_m * p_n);
}

template <typename T>
grid_layout<T> block_cyclic_layout(int m, int n, int mb, int nb, int ia, int ja, int sub_m,
                                   int sub_n, int p_m, int p_n, char rank_order, int rsrc, int csrc,
                                   T* ptr, int lld, char data_ordering, int rank) {
    auto g = bc_build(m, n, mb, nb, ia, ja, sub_m, sub_n, p_m, p_n, rank_order, rsrc, csrc);
    data_ordering = upper(data_ordering);
    if (data_ordering != 'R' && data_ordering != 'C')
        throw std::runtime_error("costa::block_cyclic_layout: data ordering must be 'R' or 'C'");
    const int nbr = int(g.rows.size()) - 1, nbc = int(g.cols.size()) - 1;
    std::vector<block<T>> blks;
    for (int j = 0; j < nbc; ++j) {  // column-major traversal, as scalapack_layout.cpp:229
        for (int i = 0; i < nbr; ++i) {
            if (g.owners[size_t(i) * nbc + j] != rank) continue;
            // global block index -> local block index and offset inside it
            const int gbr = g.first_blk_row + i, gbc = g.first_blk_col + j;
            const int64_t loc_row = int64_t(gbr / p_m) * mb + (g.ia0 + g.rows[i] - int64_t(gbr) * mb);
            const int64_t loc_col = int64_t(gbc / p_n) * nb + (g.ja0 + g.cols[j] - int64_t(gbc) * nb);
            const int64_t off = data_ordering == 'R' ? loc_col + int64_t(lld) * loc_row
                                                     : loc_row + int64_t(lld) * loc_col;
            blks.emplace_back(interval(g.rows[i], g.rows[i + 1]), interval(g.cols[j], g.cols[j + 1]),
                              block_coordinates(i, j), ptr + off, lld);
        }
    }
    assigned_grid2D grid(grid2D(std::move(g.rows), std::move(g.cols)), std::move(g.owners),
                         p_m * p_n);
    return grid_layout<T>(std::move(grid), local_blocks<T>(std::move(blks)), data_ordering);
}

#define COSTA_INSTANTIATE_LAYOUTS(T)                                                              \
    template grid_layout<T> custom_layout<T>(int, int, const int*, const int*, const int*, int,     \
                                             const block_t*, char);                                 \
    template grid_layout<T> block_cyclic_layout<T>(int, int, int, int, int, int, int, int, int, int, \
                                                   char, int, int, T*, int, char, int);

COSTA_INSTANTIATE_LAYOUTS(float)
COSTA_INSTANTIATE_LAYOUTS(double)
COSTA_INSTANTIATE_LAYOUTS(std::complex<float>)
COSTA_INSTANTIATE_LAYOUTS(std::complex<double>)
COSTA_INSTANTIATE_LAYOUTS(int)

}  // namespace costa
