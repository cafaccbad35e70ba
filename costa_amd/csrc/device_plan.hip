// Device-side planning: the tile-op lists of make_plan (plan.cpp) built on the
// GPU from the two grids' split points and owner maps, so that a plan-cache miss on a large
// layout pair does not pay the host decomposition and sort (the reference re-plans on the host
// at every call: utils.hpp:87-206, communication_data.cpp:67-164).
//
// Every tile is the intersection of one source block with one target block, i.e. one cell of
// the MERGED grid of a layout pair (the union of both grids' split points, A's grid seen
// transposed when op != 'N'): no split point of either grid falls inside such a cell, and every
// non-empty intersection is one.  With one thread per merged cell:
//   classify  the owners of the cell's A block and C block make it a local tile (both this rank),
//             a pack tile (A here; peer = C's owner), an unpack tile (C here; peer = A's owner),
//             or nothing
//   order     the reference's message order (peer, tag, rows, cols) (communication_data.cpp:
//             67-82) is row-major cell order inside each peer: a stable radix sort of the cell
//             ids by peer gives it, and the package offsets are an exclusive scan of the sorted
//             tiles' sizes (communication_data.cpp:103-164)
//   hint      costa_tile_op_t::order (plan.cpp set_order: the rank in column-major target
//             order) is an exclusive scan of each list's flags in column-major cell order
//   emit      one thread per tile writes its op through tile_op.hpp, the normalisation the
//             host planner uses
// The host does O(split points + blocks) work (merging split points, cell -> block tables).
// Layouts whose local blocks are not exactly their rank's grid cells (possible with hand-made
// custom layouts) are left to the host planner.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <iterator>

#include "engine.hpp"
#include "tile_op.hpp"

namespace costa {
namespace engine {

#define DP_CHECK(x)                                                                    \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
            throw error(COSTA_ERR_HIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

namespace {

struct dp_block {  // one local block
    uint64_t data;
    int32_t ld, row0, col0, pad;
};

// one layout pair: its merged grid and where its tables sit in the shared arrays
struct dp_job {
    int64_t base;          // first cell id (the cells of earlier pairs come first)
    int32_t nr, nc;        // merged grid: rows, columns
    int32_t sr, sc;        // offsets of its merged row / column split points in `splits`; `amap`
                           // and `cmap` hold at the same offsets the A-view / C cell of each
    int32_t a_nbc, c_nbc;  // owner-matrix row lengths
    int64_t a_own, c_own;  // owner matrices (row-major) in `owners`
    int64_t a_tab, c_tab;  // cell -> local block tables in `tab` (-1: not local)
    int32_t tr, cj;        // the op transposes / conjugates
    int32_t a_cm, c_cm;    // column-major ('C') storage
    int32_t a_rm, c_rm;    // row-major ('R') storage
    uint32_t kind_copy, kind_tr;
    int32_t tag;
};

struct dp_args {
    const dp_job* jobs;
    int n_jobs;
    int64_t n_cells;
    const int32_t* splits;
    const int32_t* amap;
    const int32_t* cmap;
    const int32_t* owners;
    const int32_t* tab;
    const dp_block* blocks;
    int rank, n_ranks, loopback;
    uint64_t elem;
};

struct dp_cell {
    const dp_job* j;
    int i, k;            // merged row, column
    int r0, r1, c0, c1;  // target coordinates
    int ar, ac;          // A's own cell (row, column)
    int cr, cc;          // C's cell
};

__device__ inline dp_cell locate(const dp_args& a, int64_t g) {
    int lo = 0, hi = a.n_jobs - 1;
    while (lo < hi) {  // last pair starting at or before g
        const int mid = (lo + hi + 1) / 2;
        if (a.jobs[mid].base <= g)
            lo = mid;
        else
            hi = mid - 1;
    }
    dp_cell c;
    c.j = a.jobs + lo;
    const dp_job& J = *c.j;
    const int64_t q = g - J.base;
    c.i = int(q / J.nc);
    c.k = int(q - int64_t(c.i) * J.nc);
    c.r0 = a.splits[J.sr + c.i];
    c.r1 = a.splits[J.sr + c.i + 1];
    c.c0 = a.splits[J.sc + c.k];
    c.c1 = a.splits[J.sc + c.k + 1];
    const int vi = a.amap[J.sr + c.i], vk = a.amap[J.sc + c.k];  // cell of A's view
    c.ar = J.tr ? vk : vi;
    c.ac = J.tr ? vi : vk;
    c.cr = a.cmap[J.sr + c.i];
    c.cc = a.cmap[J.sc + c.k];
    return c;
}

__device__ inline int64_t cm_index(const dp_cell& c) {
    return c.j->base + int64_t(c.k) * c.j->nr + c.i;
}

// the send side's tile of a cell (prepare_to_send: A's block, seen transposed when op != 'N')
__device__ inline tile_side a_side(const dp_args& a, const dp_cell& c) {
    const dp_job& J = *c.j;
    const dp_block& b = a.blocks[a.tab[J.a_tab + int64_t(c.ar) * J.a_nbc + c.ac]];
    return sub_tile(b.data, b.ld, b.row0, b.col0, J.a_rm, J.tr, c.r0, c.r1, c.c0, c.c1, a.elem);
}
// the receive side's tile (prepare_to_recv: C's block)
__device__ inline tile_side c_side(const dp_args& a, const dp_cell& c) {
    const dp_job& J = *c.j;
    const dp_block& b = a.blocks[a.tab[J.c_tab + int64_t(c.cr) * J.c_nbc + c.cc]];
    return sub_tile(b.data, b.ld, b.row0, b.col0, J.c_rm, false, c.r0, c.r1, c.c0, c.c1, a.elem);
}

enum { L_LOCAL = 0, L_PACK = 1, L_UNPACK = 2 };

__global__ void dp_iota(uint32_t* v, int64_t n) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k < n) v[k] = uint32_t(k);
}

// per cell: its key in each list (the peer; n_ranks = not in the list; local: 0 / 1) in cell
// order, and its membership flags in column-major cell order
__global__ void dp_classify(dp_args a, uint32_t* keys, uint32_t* flags) {
    const int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g >= a.n_cells) return;
    const int64_t n = a.n_cells;
    const dp_cell c = locate(a, g);
    const dp_job& J = *c.j;
    const int ao = a.owners[J.a_own + int64_t(c.ar) * J.a_nbc + c.ac];
    const int co = a.owners[J.c_own + int64_t(c.cr) * J.c_nbc + c.cc];
    // make_plan's stays_local (loopback is a test mode)
    const bool stays = a.loopback == 0   ? true
                       : a.loopback == 1 ? false
                                         : ((c.r0 / 7 + c.c0 / 5) & 1) == 0;
    const bool local = ao == a.rank && co == a.rank && stays;
    const bool pack = ao == a.rank && !local;
    const bool unpack = co == a.rank && !local;
    const uint32_t none = uint32_t(a.n_ranks);
    keys[L_LOCAL * n + g] = local ? 0u : 1u;
    keys[L_PACK * n + g] = pack ? uint32_t(co) : none;
    keys[L_UNPACK * n + g] = unpack ? uint32_t(ao) : none;
    const int64_t m = cm_index(c);
    flags[L_LOCAL * n + m] = local;
    flags[L_PACK * n + m] = pack;
    flags[L_UNPACK * n + m] = unpack;
}

// members of each list: the last exclusive-scan value plus the last flag
__global__ void dp_totals(const uint32_t* flags, const uint32_t* ranks, int64_t n, uint32_t* tot) {
    const int l = int(threadIdx.x);
    if (l < 3) tot[l] = ranks[l * n + n - 1] + flags[l * n + n - 1];
}

// sizes (elements) of the sorted tiles of one list
__global__ void dp_sizes(dp_args a, const uint32_t* cells, int64_t n, int64_t* size) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const dp_cell c = locate(a, cells[k]);
    size[k] = int64_t(c.r1 - c.r0) * (c.c1 - c.c0);
}

// the ops of one list in the reference's message order; for pack / unpack also each peer's
// element range in the package (first offset of its run, one past its last element)
template <int L>
__global__ void dp_emit(dp_args a, const uint32_t* cells, const uint32_t* keys, int64_t n,
                        const int64_t* off, const uint32_t* rank_cm, costa_tile_op_t* out,
                        int64_t* run_lo, int64_t* run_hi) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= n) return;
    const dp_cell c = locate(a, cells[k]);
    const dp_job& J = *c.j;
    const bool wt = (J.tr && J.a_cm == J.c_cm) || (!J.tr && J.a_cm != J.c_cm);
    const uint32_t kind = wt ? J.kind_tr : J.kind_copy;
    costa_tile_op_t op;
    if (L == L_PACK) {  // copy_to_buffer: stored shape and ordering, dense, no transform
        const tile_side s = a_side(a, c);
        op = tile_op(s.n_rows, s.n_cols, s.ptr, s.ld, J.a_cm, uint64_t(off[k]) * a.elem, 0, J.a_cm,
                     false, false, COSTA_SCALE_BITCOPY, 0, a.elem);
    } else if (L == L_UNPACK) {  // copy_from_buffer: A's stored shape, dims swapped back
        const tile_side d = c_side(a, c);
        const int nr = J.tr ? d.n_cols : d.n_rows, nc = J.tr ? d.n_rows : d.n_cols;
        op = tile_op(nr, nc, uint64_t(off[k]) * a.elem, 0, J.a_cm, d.ptr, d.ld, J.c_cm, J.tr, J.cj,
                     kind, uint32_t(J.tag), a.elem);
    } else {  // copy_local_blocks
        const tile_side s = a_side(a, c), d = c_side(a, c);
        op = tile_op(s.n_rows, s.n_cols, s.ptr, s.ld, J.a_cm, d.ptr, d.ld, J.c_cm, J.tr, J.cj, kind,
                     uint32_t(J.tag), a.elem);
    }
    op.order = rank_cm[cm_index(c)] + 1;
    out[k] = op;
    if (L != L_LOCAL) {
        const uint32_t p = keys[k];
        const int64_t size = int64_t(c.r1 - c.r0) * (c.c1 - c.c0);
        if (k == 0 || keys[k - 1] != p) run_lo[p] = off[k];
        if (k == n - 1 || keys[k + 1] != p) run_hi[p] = off[k] + size;
    }
}

int32_t cell_index(const std::vector<int>& split, int x) {
    return int32_t(std::upper_bound(split.begin(), split.end(), x) - split.begin()) - 1;
}

// the distinct split points of two grids (same first and last point), each with the cell of
// either grid the merged interval starting there lies in
void merge_splits(const std::vector<int>& a, const std::vector<int>& b, std::vector<int32_t>& out,
                  std::vector<int32_t>& amap, std::vector<int32_t>& bmap) {
    std::vector<int> m;
    m.reserve(a.size() + b.size());
    std::set_union(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(m));
    m.erase(std::unique(m.begin(), m.end()), m.end());
    for (size_t t = 0; t < m.size(); ++t) {
        const bool last = t + 1 == m.size();
        out.push_back(m[t]);
        amap.push_back(last ? 0 : cell_index(a, m[t]));
        bmap.push_back(last ? 0 : cell_index(b, m[t]));
    }
}

// cell -> local block table of one layout; false when its local blocks are not exactly the
// non-empty cells the owner matrix gives this rank
bool block_table(const elayout& L, int rank, std::vector<int32_t>& tab, std::vector<dp_block>& blocks,
                 int64_t& at) {
    const int nbr = L.nbr(), nbc = L.nbc();
    at = int64_t(tab.size());
    tab.resize(tab.size() + size_t(nbr) * size_t(nbc), -1);
    int32_t* t = tab.data() + at;
    for (const eblock& b : L.blocks) {
        if (!b.rows.non_empty() || !b.cols.non_empty()) continue;
        const int i = cell_index(L.rows_split, b.rows.start), j = cell_index(L.cols_split, b.cols.start);
        if (i < 0 || j < 0 || i >= nbr || j >= nbc) return false;
        if (L.rows_split[size_t(i)] != b.rows.start || L.rows_split[size_t(i) + 1] != b.rows.end ||
            L.cols_split[size_t(j)] != b.cols.start || L.cols_split[size_t(j) + 1] != b.cols.end)
            return false;
        const size_t cell = size_t(i) * size_t(nbc) + size_t(j);
        if (L.owners[cell] != rank || t[cell] >= 0) return false;
        t[cell] = int32_t(blocks.size());
        blocks.push_back({reinterpret_cast<uint64_t>(b.data), b.ld, b.rows.start, b.cols.start, 0});
    }
    for (int i = 0; i < nbr; ++i) {
        if (L.rows_split[size_t(i)] == L.rows_split[size_t(i) + 1]) continue;
        for (int j = 0; j < nbc; ++j) {
            if (L.cols_split[size_t(j)] == L.cols_split[size_t(j) + 1]) continue;
            const size_t cell = size_t(i) * size_t(nbc) + size_t(j);
            if (L.owners[cell] == rank && t[cell] < 0) return false;
        }
    }
    return true;
}

struct dmem {
    void* p = nullptr;
    explicit dmem(size_t n) {
        if (n) DP_CHECK(hipMalloc(&p, n));
    }
    dmem(const dmem&) = delete;
    dmem& operator=(const dmem&) = delete;
    ~dmem() {
        if (p) (void)hipFree(p);
    }
    template <typename T>
    T* at(size_t off) const {
        return reinterpret_cast<T*>(static_cast<char*>(p) + off);
    }
};

// bump allocator over one device allocation (256-byte aligned pieces)
struct carver {
    size_t top = 0;
    size_t take(size_t bytes) {
        const size_t o = top;
        top += (bytes + 255) & ~size_t(255);
        return o;
    }
};

unsigned grid_of(int64_t n) { return unsigned((n + 255) / 256); }

template <typename T>
void upload(const dmem& m, size_t off, const std::vector<T>& v, hipStream_t s) {
    if (!v.empty())
        DP_CHECK(hipMemcpyAsync(m.at<char>(off), v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, s));
}

}  // namespace

std::unique_ptr<plan> make_plan_device(const std::vector<job>& jobs, int rank, int n_ranks,
                                       int loopback, int device, void* stream) {
    // COSTA_PLAN_TRACE=1: where the time goes (stderr)
    static const bool trace = std::getenv("COSTA_PLAN_TRACE") != nullptr;
    auto now = [] {
        return std::chrono::duration<double, std::milli>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const double t0 = now();
    auto p = std::make_unique<plan>();
    const std::vector<job_params> prm = check_jobs(jobs, n_ranks, p->dtype);
    const uint64_t E = dtype_size(p->dtype);

    // ---- host: merged grids and tables, O(split points + blocks) ----
    std::vector<dp_job> J;
    std::vector<int32_t> splits, amap, cmap, owners, tab;
    std::vector<dp_block> blocks;
    int64_t n = 0;
    for (size_t t = 0; t < jobs.size(); ++t) {
        const elayout& A = *jobs[t].A;
        const elayout& C = *jobs[t].C;
        const bool tr = prm[t].transpose;
        const auto& ra = tr ? A.cols_split : A.rows_split;
        const auto& ca = tr ? A.rows_split : A.cols_split;
        if (ra.back() != C.rows_split.back() || ca.back() != C.cols_split.back())
            throw error(COSTA_ERR_ARG, "costa::transform: layouts describe matrices of different sizes");
        if (ra.front() != C.rows_split.front() || ca.front() != C.cols_split.front()) return nullptr;
        dp_job d{};
        d.base = n;
        d.sr = int32_t(splits.size());
        merge_splits(ra, C.rows_split, splits, amap, cmap);
        d.nr = int32_t(splits.size()) - d.sr - 1;
        d.sc = int32_t(splits.size());
        merge_splits(ca, C.cols_split, splits, amap, cmap);
        d.nc = int32_t(splits.size()) - d.sc - 1;
        d.a_nbc = A.nbc();
        d.c_nbc = C.nbc();
        d.a_own = int64_t(owners.size());
        owners.insert(owners.end(), A.owners.begin(), A.owners.end());
        d.c_own = int64_t(owners.size());
        owners.insert(owners.end(), C.owners.begin(), C.owners.end());
        if (!block_table(A, rank, tab, blocks, d.a_tab) || !block_table(C, rank, tab, blocks, d.c_tab))
            return nullptr;
        d.tr = tr;
        d.cj = prm[t].conj;
        d.a_cm = prm[t].a_cm;
        d.c_cm = prm[t].c_cm;
        d.a_rm = A.ordering == 'R';
        d.c_rm = C.ordering == 'R';
        d.kind_copy = prm[t].kind_copy;
        d.kind_tr = prm[t].kind_tr;
        d.tag = int32_t(t);
        n += int64_t(std::max(d.nr, 0)) * std::max(d.nc, 0);
        J.push_back(d);
        p->slots.push_back(jobs[t].s);
    }
    if (n == 0 || n > int64_t(UINT32_MAX) || n_ranks > (1 << 24)) return nullptr;
    p->rank = rank;
    p->n_ranks = n_ranks;

    DP_CHECK(hipSetDevice(device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    unsigned bits = 1;  // key bits of the pack / unpack lists: peers 0..n_ranks-1 and "none"
    while ((uint64_t(1) << bits) <= uint64_t(n_ranks)) ++bits;
    const size_t N = size_t(n);

    // rocprim scratch: the largest need of the sorts and scans
    size_t tmp = 0, q = 0;
    {
        uint32_t* u = nullptr;
        int64_t* w = nullptr;
        DP_CHECK(rocprim::radix_sort_pairs(nullptr, q, u, u, u, u, N, 0, bits, s));
        tmp = std::max(tmp, q);
        DP_CHECK(rocprim::radix_sort_pairs(nullptr, q, u, u, u, u, N, 0, 1, s));
        tmp = std::max(tmp, q);
        DP_CHECK(rocprim::exclusive_scan(nullptr, q, u, u, uint32_t(0), N, rocprim::plus<uint32_t>(), s));
        tmp = std::max(tmp, q);
        DP_CHECK(rocprim::exclusive_scan(nullptr, q, w, w, int64_t(0), N, rocprim::plus<int64_t>(), s));
        tmp = std::max(tmp, q);
    }
    carver cv;
    const size_t o_jobs = cv.take(J.size() * sizeof(dp_job));
    const size_t o_splits = cv.take(splits.size() * 4), o_amap = cv.take(amap.size() * 4),
                 o_cmap = cv.take(cmap.size() * 4);
    const size_t o_owners = cv.take(owners.size() * 4), o_tab = cv.take(tab.size() * 4);
    const size_t o_blocks = cv.take(blocks.size() * sizeof(dp_block));
    const size_t o_keys = cv.take(3 * N * 4), o_iota = cv.take(N * 4), o_skeys = cv.take(3 * N * 4),
                 o_cells = cv.take(3 * N * 4), o_flags = cv.take(3 * N * 4), o_ranks = cv.take(3 * N * 4);
    const size_t o_size = cv.take(2 * N * 8), o_off = cv.take(2 * N * 8);
    const size_t o_runs = cv.take(4 * size_t(n_ranks + 1) * 8), o_tot = cv.take(16);
    const size_t o_tmp = cv.take(tmp);
    const double t1 = now();
    dmem m(cv.top);
    const double t2 = now();
    upload(m, o_jobs, J, s);
    upload(m, o_splits, splits, s);
    upload(m, o_amap, amap, s);
    upload(m, o_cmap, cmap, s);
    upload(m, o_owners, owners, s);
    upload(m, o_tab, tab, s);
    upload(m, o_blocks, blocks, s);

    dp_args a;
    a.jobs = m.at<dp_job>(o_jobs);
    a.n_jobs = int(J.size());
    a.n_cells = n;
    a.splits = m.at<int32_t>(o_splits);
    a.amap = m.at<int32_t>(o_amap);
    a.cmap = m.at<int32_t>(o_cmap);
    a.owners = m.at<int32_t>(o_owners);
    a.tab = m.at<int32_t>(o_tab);
    a.blocks = m.at<dp_block>(o_blocks);
    a.rank = rank;
    a.n_ranks = n_ranks;
    a.loopback = loopback;
    a.elem = E;
    uint32_t* keys = m.at<uint32_t>(o_keys);
    uint32_t* iota = m.at<uint32_t>(o_iota);
    uint32_t* skeys = m.at<uint32_t>(o_skeys);
    uint32_t* cells = m.at<uint32_t>(o_cells);
    uint32_t* flags = m.at<uint32_t>(o_flags);
    uint32_t* ranks = m.at<uint32_t>(o_ranks);
    void* scratch = m.at<void>(o_tmp);

    hipLaunchKernelGGL(dp_iota, dim3(grid_of(n)), dim3(256), 0, s, iota, n);
    hipLaunchKernelGGL(dp_classify, dim3(grid_of(n)), dim3(256), 0, s, a, keys, flags);
    DP_CHECK(hipGetLastError());
    for (int l = 0; l < 3; ++l) {
        q = tmp;
        DP_CHECK(rocprim::exclusive_scan(scratch, q, flags + l * N, ranks + l * N, uint32_t(0), N,
                                         rocprim::plus<uint32_t>(), s));
        q = tmp;  // stable: row-major cell order survives inside each peer
        DP_CHECK(rocprim::radix_sort_pairs(scratch, q, keys + l * N, skeys + l * N, iota, cells + l * N,
                                           N, 0, l == L_LOCAL ? 1u : bits, s));
    }
    uint32_t* d_tot = m.at<uint32_t>(o_tot);
    hipLaunchKernelGGL(dp_totals, dim3(1), dim3(64), 0, s, flags, ranks, n, d_tot);
    DP_CHECK(hipGetLastError());
    uint32_t tot[3] = {0, 0, 0};
    DP_CHECK(hipMemcpyAsync(tot, d_tot, sizeof(tot), hipMemcpyDeviceToHost, s));
    DP_CHECK(hipStreamSynchronize(s));
    const double t3 = now();

    // ---- the three lists ----
    const int64_t cnt[3] = {int64_t(tot[0]), int64_t(tot[1]), int64_t(tot[2])};
    dmem ops(size_t(cnt[0] + cnt[1] + cnt[2]) * sizeof(costa_tile_op_t));
    costa_tile_op_t* d_ops[3];
    d_ops[0] = ops.at<costa_tile_op_t>(0);
    d_ops[1] = d_ops[0] + cnt[0];
    d_ops[2] = d_ops[1] + cnt[1];
    int64_t* sizes = m.at<int64_t>(o_size);
    int64_t* offs = m.at<int64_t>(o_off);
    int64_t* runs = m.at<int64_t>(o_runs);  // [list-1][lo | hi][peer]
    const size_t R = size_t(n_ranks + 1);
    DP_CHECK(hipMemsetAsync(runs, 0, 4 * R * 8, s));
    for (int l = L_PACK; l <= L_UNPACK; ++l) {
        if (!cnt[l]) continue;
        int64_t* sz = sizes + (l - 1) * N;
        int64_t* of = offs + (l - 1) * N;
        hipLaunchKernelGGL(dp_sizes, dim3(grid_of(cnt[l])), dim3(256), 0, s, a, cells + l * N, cnt[l], sz);
        q = tmp;
        DP_CHECK(rocprim::exclusive_scan(scratch, q, sz, of, int64_t(0), size_t(cnt[l]),
                                         rocprim::plus<int64_t>(), s));
    }
    if (cnt[L_LOCAL])
        hipLaunchKernelGGL(dp_emit<L_LOCAL>, dim3(grid_of(cnt[0])), dim3(256), 0, s, a, cells,
                           skeys, cnt[0], static_cast<const int64_t*>(nullptr), ranks, d_ops[0],
                           static_cast<int64_t*>(nullptr), static_cast<int64_t*>(nullptr));
    if (cnt[L_PACK])
        hipLaunchKernelGGL(dp_emit<L_PACK>, dim3(grid_of(cnt[1])), dim3(256), 0, s, a, cells + N,
                           skeys + N, cnt[1], offs, ranks + N, d_ops[1], runs, runs + R);
    if (cnt[L_UNPACK])
        hipLaunchKernelGGL(dp_emit<L_UNPACK>, dim3(grid_of(cnt[2])), dim3(256), 0, s, a, cells + 2 * N,
                           skeys + 2 * N, cnt[2], offs + N, ranks + 2 * N, d_ops[2], runs + 2 * R,
                           runs + 3 * R);
    DP_CHECK(hipGetLastError());
    p->local_ops.resize(size_t(cnt[0]));
    p->pack_ops.resize(size_t(cnt[1]));
    p->unpack_ops.resize(size_t(cnt[2]));
    std::vector<int64_t> run(4 * R);
    auto down = [&](void* dst, const void* src, size_t bytes) {
        if (bytes) DP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s));
    };
    down(p->local_ops.data(), d_ops[0], size_t(cnt[0]) * sizeof(costa_tile_op_t));
    down(p->pack_ops.data(), d_ops[1], size_t(cnt[1]) * sizeof(costa_tile_op_t));
    down(p->unpack_ops.data(), d_ops[2], size_t(cnt[2]) * sizeof(costa_tile_op_t));
    down(run.data(), runs, run.size() * 8);
    DP_CHECK(hipStreamSynchronize(s));
    const double t4 = now();

    // ---- exchange geometry and byte counts (as make_plan) ----
    p->send_counts.assign(size_t(n_ranks), 0);
    p->recv_counts.assign(size_t(n_ranks), 0);
    p->send_displs.assign(size_t(n_ranks), 0);
    p->recv_displs.assign(size_t(n_ranks), 0);
    for (size_t r = 0; r < size_t(n_ranks); ++r) {
        p->send_counts[r] = run[R + r] - run[r];
        p->recv_counts[r] = run[3 * R + r] - run[2 * R + r];
    }
    for (size_t r = 1; r < size_t(n_ranks); ++r) {
        p->send_displs[r] = p->send_displs[r - 1] + p->send_counts[r - 1];
        p->recv_displs[r] = p->recv_displs[r - 1] + p->recv_counts[r - 1];
    }
    for (size_t r = 0; r < size_t(n_ranks); ++r) {
        p->send_elems += p->send_counts[r];
        p->recv_elems += p->recv_counts[r];
    }
    for (const auto& op : p->local_ops) {
        p->local_elems += int64_t(op.nf) * op.ns;
        p->local_bytes += op_alg_bytes(op, E);
    }
    for (const auto& op : p->pack_ops) p->pack_bytes += op_alg_bytes(op, E);
    for (const auto& op : p->unpack_ops) p->unpack_bytes += op_alg_bytes(op, E);
    if (trace)
        std::fprintf(stderr,
                     "[costa device plan] %lld cells, %lld / %lld / %lld ops: host tables %.2f ms, "
                     "alloc %.2f, classify+sort %.2f, emit+download %.2f, tail %.2f\n",
                     (long long)n, (long long)cnt[0], (long long)cnt[1], (long long)cnt[2], t1 - t0,
                     t2 - t1, t3 - t2, t4 - t3, now() - t4);
    return p;
}

}  // namespace engine
}  // namespace costa

// The work lists' destination-block groups on the GPU: in this translation unit so that both share
// one code object and their rocPRIM kernels (the first GPU plan of a process loads both).
#include "device_lists.hip"
