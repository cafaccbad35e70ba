// ScaLAPACK-compatible entry points (include/costa/scalapack.h) over the MI355X tile path.
// Compiled twice: plain names (libcosta_amd_scalapack.so) and, with -DCOSTA_PREFIXED,
// costa_-prefixed names (libcosta_amd_prefixed_scalapack.so).
//
// Reference behaviour followed (eth-cscs/COSTA):
//   costa::pxgemr2d<T>     pxgemr2d/costa_pxgemr2d.cpp:14-171
//   costa::pxtran_op<T>    pxtran_op/costa_pxtran_op.cpp:15-175  (sub(A) is n x m: :68-69)
//   descriptor fields      scalapack.hpp:9-45; leading_dimension scalapack.cpp:37-39
//   ctxt -> MPI_Comm       scalapack.cpp:42-53 (Cblacs_get(ctxt, 10) + Cblacs2sys_handle)
//   communicator           comm_union(comm_a, comm_c) (scalapack.cpp:172-185, costa_pxgemr2d.cpp:60)
// Differences:
//   * The transform runs on the processes of the call's context (ictxt for p?gemr2d, the common
//     context for p?tran*), a communicator made once per context with MPI_Comm_create_group (only
//     those processes take part) and cached; the reference takes the union of A's and C's system
//     communicators -- the whole MPI_COMM_WORLD for ordinary grids -- and makes a new one on every
//     call (never freed).  ScaLAPACK defines ictxt as a context holding every process of A and C.
//   * Each matrix's process grid is read from ITS OWN descriptor context, and every grid cell is
//     mapped to its process's rank in that communicator (Cblacs_pnum, MPI_Group_translate_ranks);
//     the layouts are relabelled accordingly (grid_layout::reorder_ranks).  The reference builds
//     both p?gemr2d layouts with the grid of ictxt (costa_pxgemr2d.cpp:47,144,157) and assumes
//     grid rank = communicator rank, which mis-describes A or C whenever the grids differ.
//   * A process outside A's (or C's) context passes desc[CTXT] = -1 and owns nothing of it; the
//     grid shape, blocking and rank sources of that matrix come from the processes inside it
//     (one MPI_Allreduce over the communicator).
#include <mpi.h>

#include <costa/mpi.hpp>
#include <costa/scalapack.h>

#include <algorithm>
#include <cctype>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <stdexcept>
#include <utility>
#include <vector>

extern "C" {
// BLACS, resolved from the application's ScaLAPACK (reference blacs.hpp:6-35)
void Cblacs_gridinfo(int ictxt, int* nprow, int* npcol, int* myrow, int* mycol);
int Cblacs_pnum(int ictxt, int prow, int pcol);
void Cblacs_get(int ictxt, int what, int* val);
MPI_Comm Cblacs2sys_handle(int ictxt);
}

namespace {

[[noreturn]] void fatal(const char* where, const std::exception& e) {
    std::fprintf(stderr, "costa %s: %s\n", where, e.what());
    std::fflush(stderr);
    std::abort();
}

// the system communicator a BLACS context was made from: BLACS process numbers are its ranks
MPI_Comm sys_comm(int ctxt) {
    int sys = 0;
    Cblacs_get(ctxt, 10, &sys);
    return Cblacs2sys_handle(sys);
}

struct grid_info {
    int pm = 0, pn = 0, myr = -1, myc = -1;
    std::vector<int> pnum;  // BLACS process number of each grid cell, row-major
    bool member() const { return pm > 0 && myr >= 0; }
};

grid_info grid_of(int ctxt) {
    grid_info g;
    if (ctxt < 0) return g;  // this process is outside the context
    Cblacs_gridinfo(ctxt, &g.pm, &g.pn, &g.myr, &g.myc);
    if (g.pm < 1 || g.pn < 1 || g.myr < 0) return grid_info{};
    g.pnum.resize(size_t(g.pm) * size_t(g.pn));
    for (int r = 0; r < g.pm; ++r)
        for (int c = 0; c < g.pn; ++c) g.pnum[size_t(r) * g.pn + c] = Cblacs_pnum(ctxt, r, c);
    return g;
}

// The processes of `ctxt`'s grid as one communicator, rank k = grid cell k (row-major); made
// once per process set and kept (its RCCL communicator is cached on it, costa/transform.hpp
// comm_from_mpi).  The cache is keyed by the processes themselves -- their MPI_COMM_WORLD ranks
// in cell order -- not by the context handle: BLACS reuses handles after Cblacs_gridexit
// (possibly over another system communicator), and handles are local to each process.  Every
// process of a grid computes the same key, and it holds an entry for it exactly when it took part
// in the MPI_Comm_create_group that made one, so the members of a grid always agree on reusing
// or creating (a handle-keyed cache let one member reuse while another created, and hang).
// The cached communicators (and with them their RCCL communicators) are freed at the start of
// MPI_Finalize, through an attribute of MPI_COMM_SELF (MPI-3.1 §8.7.1).
struct comm_cache {
    std::map<std::vector<int>, MPI_Comm> by_procs;
};

comm_cache& cached_comms() {
    static comm_cache c;
    return c;
}

int free_cached_comms(MPI_Comm, int, void*, void*) {
    comm_cache& c = cached_comms();
    for (auto& kv : c.by_procs) MPI_Comm_free(&kv.second);
    c.by_procs.clear();
    return MPI_SUCCESS;
}

void free_at_finalize() {
    static bool done = false;
    if (done) return;
    int key = MPI_KEYVAL_INVALID;
    MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, free_cached_comms, &key, nullptr);
    MPI_Comm_set_attr(MPI_COMM_SELF, key, nullptr);
    done = true;
}

// The communicator of one call: the cached one, or -- when some grid process lies outside this
// process's MPI_COMM_WORLD (MPI_Comm_spawn / MPI_Comm_connect: its world rank translates to
// MPI_UNDEFINED, and two different grids could then share a key) -- one made for the call and
// freed after it.  Its RCCL communicator lives on it as an attribute, so it too is made and
// destroyed per call: such a call pays MPI_Comm_create_group, a unique-id broadcast and
// ncclCommInitRank every time.  Every member of such a grid sees
// an undefined rank (the members share no world), so all of them take the uncached way together.
struct call_comm {
    MPI_Comm comm = MPI_COMM_NULL;
    bool owned = false;
    call_comm() = default;
    call_comm(const call_comm&) = delete;
    call_comm& operator=(const call_comm&) = delete;
    ~call_comm() {
        if (owned && comm != MPI_COMM_NULL) MPI_Comm_free(&comm);
    }
};

void grid_comm(int ctxt, const grid_info& g, call_comm& cc) {
    comm_cache& cache = cached_comms();
    MPI_Comm sys = sys_comm(ctxt);
    MPI_Group all, grp, world;
    MPI_Comm_group(sys, &all);
    MPI_Group_incl(all, int(g.pnum.size()), g.pnum.data(), &grp);
    MPI_Group_free(&all);
    std::vector<int> cells(g.pnum.size()), procs(g.pnum.size(), MPI_UNDEFINED);
    for (size_t k = 0; k < cells.size(); ++k) cells[k] = int(k);
    MPI_Comm_group(MPI_COMM_WORLD, &world);
    MPI_Group_translate_ranks(grp, int(cells.size()), cells.data(), world, procs.data());
    MPI_Group_free(&world);
    const bool keyed = std::find(procs.begin(), procs.end(), MPI_UNDEFINED) == procs.end();
    if (keyed) {
        auto it = cache.by_procs.find(procs);
        if (it != cache.by_procs.end()) {
            MPI_Group_free(&grp);
            cc.comm = it->second;
            return;
        }
    }
    MPI_Comm out = MPI_COMM_NULL;
    MPI_Comm_create_group(sys, grp, 0x6c0d, &out);
    MPI_Group_free(&grp);
    if (out == MPI_COMM_NULL) throw std::runtime_error("could not make the context's communicator");
    cc.comm = out;
    if (!keyed) {
        cc.owned = true;
        return;
    }
    free_at_finalize();
    cache.by_procs.emplace(std::move(procs), out);
}

// One matrix's distribution as seen in `comm`: its grid, blocking and rank sources, and the
// rank in `comm` of every grid cell (row-major).
struct dist {
    int pm = 0, pn = 0, M = 0, N = 0, MB = 0, NB = 0, rsrc = 0, csrc = 0;
    int my_cell = -1;        // this process's grid cell, -1 outside the grid
    std::vector<int> rank;   // comm rank of each grid cell
};

// Collective over `comm`: the processes inside each matrix's context describe it, the others
// learn it from them.  A process that finds a bad grid still joins the reduction (its error
// flag is reduced with the descriptions), so every process of `comm` throws together instead of
// one aborting while the others wait in the collective.
std::vector<dist> distributions(MPI_Comm comm, const std::vector<const int*>& descs) {
    int P = 1;
    MPI_Comm_size(comm, &P);
    MPI_Group cg;
    MPI_Comm_group(comm, &cg);
    const size_t W = 8 + size_t(P);
    std::vector<int> buf(W * descs.size() + 1, -1);  // + the error flag (1: too large, 2: outside)
    std::vector<int> mine(descs.size(), -1);
    for (size_t d = 0; d < descs.size(); ++d) {
        const int* desc = descs[d];
        const grid_info g = grid_of(desc[1]);
        if (!g.member()) continue;
        const int cells = g.pm * g.pn;
        if (cells > P) {
            buf.back() = std::max(buf.back(), 1);
            continue;
        }
        int* b = &buf[W * d];
        b[0] = g.pm;
        b[1] = g.pn;
        for (int k = 0; k < 6; ++k) b[2 + k] = desc[2 + k];  // M N MB NB RSRC CSRC
        MPI_Group sg;
        MPI_Comm_group(sys_comm(desc[1]), &sg);
        MPI_Group_translate_ranks(sg, cells, g.pnum.data(), cg, b + 8);
        MPI_Group_free(&sg);
        for (int k = 0; k < cells; ++k)
            if (b[8 + k] == MPI_UNDEFINED || b[8 + k] < 0) buf.back() = std::max(buf.back(), 2);
        mine[d] = g.myr * g.pn + g.myc;
    }
    MPI_Group_free(&cg);
    MPI_Allreduce(MPI_IN_PLACE, buf.data(), int(buf.size()), MPI_INT, MPI_MAX, comm);
    if (buf.back() == 1) throw std::runtime_error("a matrix's grid is larger than the call's context");
    if (buf.back() == 2)
        throw std::runtime_error("a process of the matrix's grid is outside the call's context");
    std::vector<dist> out(descs.size());
    for (size_t d = 0; d < descs.size(); ++d) {
        const int* b = &buf[W * d];
        dist& x = out[d];
        x.pm = b[0], x.pn = b[1], x.M = b[2], x.N = b[3], x.MB = b[4], x.NB = b[5];
        x.rsrc = b[6], x.csrc = b[7];
        if (x.pm < 1 || x.pn < 1) throw std::runtime_error("no process holds the matrix's context");
        x.rank.assign(b + 8, b + 8 + x.pm * x.pn);
        x.my_cell = mine[d];
    }
    return out;
}

// block-cyclic layout of sub(X) in the call's communicator: built on the matrix's own grid
// (row-major cells), then relabelled cell -> comm rank
template <typename T>
costa::grid_layout<T> layout_of(const dist& x, int i, int j, int sub_m, int sub_n, T* ptr, int lld,
                                int P) {
    const int cells = x.pm * x.pn;
    auto L = costa::block_cyclic_layout<T>(x.M, x.N, x.MB, x.NB, i, j, sub_m, sub_n, x.pm, x.pn, 'R',
                                           x.rsrc, x.csrc, ptr, x.my_cell >= 0 ? lld : 1, 'C',
                                           x.my_cell >= 0 ? x.my_cell : cells);
    std::vector<int> perm(size_t(std::max(P, cells)));
    std::vector<char> used(perm.size(), 0);
    bool identity = true;
    for (int k = 0; k < cells; ++k) {
        perm[size_t(k)] = x.rank[size_t(k)];
        used[size_t(x.rank[size_t(k)])] = 1;
        identity = identity && x.rank[size_t(k)] == k;
    }
    for (size_t k = size_t(cells), r = 0; k < perm.size(); ++k) {  // the ranks outside the grid
        while (used[r]) ++r;
        perm[k] = int(r++);
    }
    if (!identity) L.reorder_ranks(perm);
    return L;
}

template <typename T>
void run(costa::grid_layout<T>& A, costa::grid_layout<T>& C, char op, T alpha, T beta, MPI_Comm comm) {
#ifdef COSTA_SCALAPACK_TEST_HOOK  // CPU tests (tests/scalapack/*.cpp): the layouts go to the test
    COSTA_SCALAPACK_TEST_HOOK(A, C, op, alpha, beta, comm);
#else
    costa::transform<T>(A, C, op, alpha, beta, costa::comm_from_mpi(comm));
#endif
}

template <typename T>
void pxgemr2d(int m, int n, const T* a, int ia, int ja, const int* desca, T* c, int ic, int jc,
              const int* descc, int ictxt) {
    if (m == 0 || n == 0) return;
    try {
        const grid_info gi = grid_of(ictxt);
        if (!gi.member()) return;  // not a process of the call's context: nothing to do
        call_comm cc;
        grid_comm(ictxt, gi, cc);
        MPI_Comm comm = cc.comm;
        int P = 1;
        MPI_Comm_size(comm, &P);
        const auto d = distributions(comm, {desca, descc});
        auto A = layout_of<T>(d[0], ia, ja, m, n, const_cast<T*>(a), desca[8], P);
        auto C = layout_of<T>(d[1], ic, jc, m, n, c, descc[8], P);
        run<T>(A, C, 'N', T(1), T(0), comm);  // the no-scale transform (transform.cpp:130-160)
    } catch (const std::exception& e) {
        fatal("p?gemr2d", e);
    }
}

template <typename T>
void pxtran(int m, int n, T alpha, const T* a, int ia, int ja, const int* desca, T beta, T* c,
            int ic, int jc, const int* descc, char op) {
    if (m == 0 || n == 0) return;
    try {
        if (desca[1] != descc[1])
            throw std::runtime_error("A and C must share one BLACS context");  // scalapack.cpp:18-23
        const grid_info g = grid_of(desca[1]);
        if (!g.member()) return;
        call_comm cc;
        grid_comm(desca[1], g, cc);
        MPI_Comm comm = cc.comm;
        int P = 1;
        MPI_Comm_size(comm, &P);
        const auto d = distributions(comm, {desca, descc});
        auto A = layout_of<T>(d[0], ia, ja, n, m, const_cast<T*>(a), desca[8], P);  // n x m
        auto C = layout_of<T>(d[1], ic, jc, m, n, c, descc[8], P);
        run<T>(A, C, op, alpha, beta, comm);
    } catch (const std::exception& e) {
        fatal("p?tran", e);
    }
}

using zf = std::complex<float>;
using zd = std::complex<double>;

}  // namespace

#ifdef COSTA_PREFIXED
#define NAME(x) costa_##x
#else
#define NAME(x) x
#endif

#define GEMR2D(fn, T, TI)                                                                       \
    void NAME(fn)(COSTA_GEMR2D_ARGS(TI)) {                                                      \
        pxgemr2d<T>(*m, *n, reinterpret_cast<const T*>(a), *ia, *ja, desca,                     \
                    reinterpret_cast<T*>(c), *ic, *jc, descc, *ictxt);                          \
    }                                                                                           \
    void NAME(fn##_)(COSTA_GEMR2D_ARGS(TI)) { NAME(fn)(m, n, a, ia, ja, desca, c, ic, jc, descc, ictxt); } \
    void NAME(fn##__)(COSTA_GEMR2D_ARGS(TI)) { NAME(fn)(m, n, a, ia, ja, desca, c, ic, jc, descc, ictxt); }

#define TRAN(fn, T, TI, OP)                                                                     \
    void NAME(fn)(COSTA_TRAN_ARGS(TI)) {                                                        \
        pxtran<T>(*m, *n, *reinterpret_cast<const T*>(alpha), reinterpret_cast<const T*>(a), *ia, \
                  *ja, desca, *reinterpret_cast<const T*>(beta), reinterpret_cast<T*>(c), *ic,  \
                  *jc, descc, OP);                                                              \
    }                                                                                           \
    void NAME(fn##_)(COSTA_TRAN_ARGS(TI)) { NAME(fn)(m, n, alpha, a, ia, ja, desca, beta, c, ic, jc, descc); } \
    void NAME(fn##__)(COSTA_TRAN_ARGS(TI)) { NAME(fn)(m, n, alpha, a, ia, ja, desca, beta, c, ic, jc, descc); }

extern "C" {
GEMR2D(psgemr2d, float, float)
GEMR2D(pdgemr2d, double, double)
GEMR2D(pcgemr2d, zf, float)
GEMR2D(pzgemr2d, zd, double)
TRAN(pstran, float, float, 'T')
TRAN(pdtran, double, double, 'T')
TRAN(pctranu, zf, float, 'T')
TRAN(pztranu, zd, double, 'T')
TRAN(pctranc, zf, float, 'C')
TRAN(pztranc, zd, double, 'C')

#ifdef COSTA_PREFIXED
GEMR2D(pigemr2d, int, int)
#else
void PSGEMR2D(COSTA_GEMR2D_ARGS(float)) { psgemr2d(m, n, a, ia, ja, desca, c, ic, jc, descc, ictxt); }
void PDGEMR2D(COSTA_GEMR2D_ARGS(double)) { pdgemr2d(m, n, a, ia, ja, desca, c, ic, jc, descc, ictxt); }
void PCGEMR2D(COSTA_GEMR2D_ARGS(float)) { pcgemr2d(m, n, a, ia, ja, desca, c, ic, jc, descc, ictxt); }
void PZGEMR2D(COSTA_GEMR2D_ARGS(double)) { pzgemr2d(m, n, a, ia, ja, desca, c, ic, jc, descc, ictxt); }
void PSTRAN(COSTA_TRAN_ARGS(float)) { pstran(m, n, alpha, a, ia, ja, desca, beta, c, ic, jc, descc); }
void PDTRAN(COSTA_TRAN_ARGS(double)) { pdtran(m, n, alpha, a, ia, ja, desca, beta, c, ic, jc, descc); }
void PCTRANU(COSTA_TRAN_ARGS(float)) { pctranu(m, n, alpha, a, ia, ja, desca, beta, c, ic, jc, descc); }
void PZTRANU(COSTA_TRAN_ARGS(double)) { pztranu(m, n, alpha, a, ia, ja, desca, beta, c, ic, jc, descc); }
void PCTRANC(COSTA_TRAN_ARGS(float)) { pctranc(m, n, alpha, a, ia, ja, desca, beta, c, ic, jc, descc); }
void PZTRANC(COSTA_TRAN_ARGS(double)) { pztranc(m, n, alpha, a, ia, ja, desca, beta, c, ic, jc, descc); }
#endif
}
