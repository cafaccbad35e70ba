// CPU check of the ScaLAPACK shims' process mapping (costa_amd/csrc/scalapack.cpp), no GPU:
// the shim is compiled into this program with COSTA_SCALAPACK_TEST_HOOK, which hands the two
// layouts a call would transform to check_layouts() below instead of running the transform.
// Runs under `mpiexec -n 4` with MKL BLACS over MPICH (tests/test_scalapack_dropin.py).
//
// Cases (grids made with Cblacs_gridmap, so grid cells and MPI ranks differ):
//   1. pdgemr2d, A on a 2x2 grid of every rank, C on a 1x2 grid of ranks {3, 1} only (ranks 0
//      and 2 pass descc[CTXT] = -1 and junk in the other fields), ictxt a 1x4 grid of ranks
//      {2, 0, 3, 1}: sub-matrices at ia, ja != 1, rank sources != 0.
//   2. pdtran on a column-major 2x2 grid of ranks {1, 3, 0, 2}.
//   3. communicator reuse across grids whose BLACS process numbers coincide: pdtran
//      on a 1x2 grid of world ranks {0, 1}; then on a 1x2 grid over a sub-communicator of
//      world ranks {0, 2} (the same process numbers {0, 1}, possibly the same handle); then on
//      {0, 1} again.  Every member of each grid must make the same create-or-reuse choice: a
//      cache keyed by handle and process numbers had world rank 0 create a communicator while
//      rank 1 reused one, and the two hung in different collectives.
// For every block of both layouts: its owner must be the rank, in the call's communicator
// (= the call context's grid cells, row-major), of the process the BLACS grid puts it on;
// every process's local blocks must be exactly the blocks it owns, inside its local array.
#include <mpi.h>

#include <cstdio>
#include <vector>

#include <costa/layout.hpp>

template <typename T>
void check_layouts(costa::grid_layout<T>& A, costa::grid_layout<T>& C, char op, MPI_Comm comm);
#define COSTA_SCALAPACK_TEST_HOOK(A, C, op, alpha, beta, comm) check_layouts(A, C, op, comm)
#include "../../costa_amd/csrc/scalapack.cpp"

extern "C" {
void Cblacs_pinfo(int*, int*);
void Cblacs_gridmap(int*, int*, int, int, int);
void Cblacs_gridexit(int);
void Cblacs_gridinit(int*, const char*, int, int);
int Csys2blacs_handle(MPI_Comm);
void Cfree_blacs_system_handle(int);
int numroc_(const int*, const int*, const int*, const int*, const int*);
}

namespace {
int g_fail = 0, g_me = 0;

struct expect_t {  // what the test knows about one matrix
    int M, N, MB, NB, rsrc, csrc, ia, ja, sub_m, sub_n;
    int pm, pn;
    std::vector<int> world;  // world rank of grid cell (r, c) at r * pn + c
    const void* base;        // this process's local array (nullptr outside the grid)
    size_t bytes;
};
expect_t g_exp[2];
std::vector<int> g_call_world;  // world rank of each cell of the call's context (row-major)

void fail(const char* what, int a, int b) {
    std::printf("rank %d: FAIL %s (%d vs %d)\n", g_me, what, a, b);
    g_fail++;
}

int comm_rank_of_world(int w) {
    for (size_t k = 0; k < g_call_world.size(); ++k)
        if (g_call_world[k] == w) return int(k);
    return -1;
}

template <typename T>
void check_one(const costa::grid_layout<T>& L, const expect_t& x, int me_comm, const char* name) {
    const int first_r = (x.ia - 1) / x.MB, first_c = (x.ja - 1) / x.NB;
    int owned = 0;
    for (int bi = 0; bi < L.num_blocks_row(); ++bi)
        for (int bj = 0; bj < L.num_blocks_col(); ++bj) {
            const int pr = (first_r + bi + x.rsrc) % x.pm, pc = (first_c + bj + x.csrc) % x.pn;
            const int want = comm_rank_of_world(x.world[size_t(pr) * x.pn + pc]);
            const int got = L.grid.owner(bi, bj);
            if (got != want) fail(name, got, want);
            owned += got == me_comm;
        }
    if (L.blocks.num_blocks() != owned) fail(name, L.blocks.num_blocks(), owned);
    for (int b = 0; b < L.blocks.num_blocks(); ++b) {
        const auto& blk = L.blocks.get_block(b);
        const char* p = reinterpret_cast<const char*>(blk.data);
        const char* lo = static_cast<const char*>(x.base);
        if (!lo || p < lo || p >= lo + x.bytes) fail(name, b, -1);
        if (L.grid.owner(blk.coordinates.row, blk.coordinates.col) != me_comm) fail(name, b, me_comm);
    }
}
}  // namespace

template <typename T>
void check_layouts(costa::grid_layout<T>& A, costa::grid_layout<T>& C, char op, MPI_Comm comm) {
    int r = 0;
    MPI_Comm_rank(comm, &r);
    int w = 0;
    MPI_Comm_rank(MPI_COMM_WORLD, &w);
    if (comm_rank_of_world(w) != r) fail("comm rank = call-context cell", r, comm_rank_of_world(w));
    check_one(A, g_exp[0], r, op == 'N' ? "gemr2d A" : "tran A");
    check_one(C, g_exp[1], r, op == 'N' ? "gemr2d C" : "tran C");
}

static int make_grid(const std::vector<int>& world, int pm, int pn) {  // cells row-major
    int ctxt = 0;
    Cblacs_get(-1, 0, &ctxt);
    std::vector<int> map(size_t(pm) * pn);  // Cblacs_gridmap wants column-major (ld = pm)
    for (int r = 0; r < pm; ++r)
        for (int c = 0; c < pn; ++c) map[size_t(c) * pm + r] = world[size_t(r) * pn + c];
    Cblacs_gridmap(&ctxt, map.data(), pm, pm, pn);
    return ctxt;
}

static void desc_for(int* d, int ctxt, const expect_t& x, int me_world, std::vector<double>& buf) {
    int myr = -1, myc = -1;
    for (int k = 0; k < x.pm * x.pn; ++k)
        if (x.world[size_t(k)] == me_world) myr = k / x.pn, myc = k % x.pn;
    if (myr < 0) {  // outside this matrix's grid
        for (int k = 0; k < 9; ++k) d[k] = -99;
        d[1] = -1;
        buf.assign(1, 0.0);
        return;
    }
    const int lr = numroc_(&x.M, &x.MB, &myr, &x.rsrc, &x.pm);
    const int lc = numroc_(&x.N, &x.NB, &myc, &x.csrc, &x.pn);
    const int lld = lr > 1 ? lr : 1;
    buf.assign(size_t(lld) * size_t(lc > 1 ? lc : 1), 0.0);
    const int v[9] = {1, ctxt, x.M, x.N, x.MB, x.NB, x.rsrc, x.csrc, lld};
    for (int k = 0; k < 9; ++k) d[k] = v[k];
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int np = 0;
    Cblacs_pinfo(&g_me, &np);
    if (np != 4) {
        if (g_me == 0) std::printf("needs 4 ranks\n");
        MPI_Finalize();
        return 2;
    }
    std::vector<double> abuf, cbuf;
    int desca[9], descc[9];
    {  // 1. pdgemr2d between different grids
        const std::vector<int> wa = {0, 1, 2, 3}, wc = {3, 1}, wi = {2, 0, 3, 1};
        const int ca = make_grid(wa, 2, 2);
        int cc = make_grid(wc, 1, 2);  // every process calls; those outside get no grid
        if (g_me != 1 && g_me != 3) cc = -1;
        const int ci = make_grid(wi, 1, 4);
        const int m = 150, n = 130;
        g_exp[0] = {170, 160, 16, 12, 1, 1, 11, 7, m, n, 2, 2, wa, nullptr, 0};
        g_exp[1] = {165, 140, 20, 9, 0, 1, 3, 5, m, n, 1, 2, wc, nullptr, 0};
        desc_for(desca, ca, g_exp[0], g_me, abuf);
        desc_for(descc, cc, g_exp[1], g_me, cbuf);
        g_exp[0].base = desca[1] >= 0 ? abuf.data() : nullptr;
        g_exp[0].bytes = abuf.size() * sizeof(double);
        g_exp[1].base = descc[1] >= 0 ? cbuf.data() : nullptr;
        g_exp[1].bytes = cbuf.size() * sizeof(double);
        g_call_world = wi;
        const int ia = g_exp[0].ia, ja = g_exp[0].ja, ic = g_exp[1].ia, jc = g_exp[1].ja;
        costa_pdgemr2d(&m, &n, abuf.data(), &ia, &ja, desca, cbuf.data(), &ic, &jc, descc, &ci);
    }
    {  // 2. pdtran on a column-major grid with permuted ranks
        const std::vector<int> wt = {1, 3, 0, 2};  // row-major cells of a 2x2 grid
        const int ct = make_grid(wt, 2, 2);
        const int m = 90, n = 70;  // sub(C) m x n, sub(A) n x m
        g_exp[0] = {80, 100, 8, 16, 1, 0, 3, 2, n, m, 2, 2, wt, nullptr, 0};
        g_exp[1] = {95, 75, 16, 8, 0, 1, 1, 4, m, n, 2, 2, wt, nullptr, 0};
        desc_for(desca, ct, g_exp[0], g_me, abuf);
        desc_for(descc, ct, g_exp[1], g_me, cbuf);
        g_exp[0].base = abuf.data();
        g_exp[0].bytes = abuf.size() * sizeof(double);
        g_exp[1].base = cbuf.data();
        g_exp[1].bytes = cbuf.size() * sizeof(double);
        g_call_world = wt;
        double alpha = 0.5, beta = 0.25;
        const int ia = g_exp[0].ia, ja = g_exp[0].ja, ic = g_exp[1].ia, jc = g_exp[1].ja;
        costa_pdtran(&m, &n, &alpha, abuf.data(), &ia, &ja, desca, &beta, cbuf.data(), &ic, &jc, descc);
    }
    {  // 3. grids with equal process numbers over different system communicators
        MPI_Comm sub = MPI_COMM_NULL;  // world ranks {0, 2}
        MPI_Comm_split(MPI_COMM_WORLD, (g_me == 0 || g_me == 2) ? 0 : MPI_UNDEFINED, g_me, &sub);
        const int m = 40, n = 30;
        for (int round = 0; round < 3; ++round) {
            const bool via_sub = round == 1;
            const std::vector<int> w = via_sub ? std::vector<int>{0, 2} : std::vector<int>{0, 1};
            int ctxt = -1;
            if (via_sub) {
                if (sub != MPI_COMM_NULL) {
                    const int h = Csys2blacs_handle(sub);
                    ctxt = h;
                    Cblacs_gridinit(&ctxt, "R", 1, 2);
                }
            } else {
                ctxt = make_grid(w, 1, 2);  // every process calls; those outside get no grid
                if (g_me != 0 && g_me != 1) ctxt = -1;
            }
            g_exp[0] = {n, m, 8, 8, 0, 0, 1, 1, n, m, 1, 2, w, nullptr, 0};
            g_exp[1] = {m, n, 8, 8, 0, 0, 1, 1, m, n, 1, 2, w, nullptr, 0};
            desc_for(desca, ctxt, g_exp[0], g_me, abuf);
            desc_for(descc, ctxt, g_exp[1], g_me, cbuf);
            g_exp[0].base = desca[1] >= 0 ? abuf.data() : nullptr;
            g_exp[0].bytes = abuf.size() * sizeof(double);
            g_exp[1].base = descc[1] >= 0 ? cbuf.data() : nullptr;
            g_exp[1].bytes = cbuf.size() * sizeof(double);
            g_call_world = w;
            double alpha = 1.0, beta = 0.0;
            const int one = 1;
            if (ctxt >= 0) {
                costa_pdtran(&m, &n, &alpha, abuf.data(), &one, &one, desca, &beta, cbuf.data(), &one,
                             &one, descc);
                Cblacs_gridexit(ctxt);
            }
            MPI_Barrier(MPI_COMM_WORLD);
        }
        if (sub != MPI_COMM_NULL) MPI_Comm_free(&sub);
    }
    int total = 0;
    MPI_Allreduce(&g_fail, &total, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (g_me == 0) std::printf(total ? "FAILED %d\n" : "ALL PASSED\n", total);
    MPI_Finalize();
    return total ? 1 : 0;
}
