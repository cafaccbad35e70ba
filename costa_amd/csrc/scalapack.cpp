// ScaLAPACK-compatible entry points (include/costa/scalapack.h) over the MI355X tile path.
// Compiled twice: plain names (libcosta_amd_scalapack.so) and, with -DCOSTA_PREFIXED,
// costa_-prefixed names (libcosta_amd_prefixed_scalapack.so).
//
// Reference behaviour followed (eth-cscs/COSTA):
//   costa::pxgemr2d<T>     pxgemr2d/costa_pxgemr2d.cpp:14-171
//   costa::pxtran_op<T>    pxtran_op/costa_pxtran_op.cpp:15-175  (sub(A) is n x m: :68-69)
//   descriptor fields      scalapack.hpp:9-45; leading_dimension scalapack.cpp:37-39
//   rank grid ordering     scalapack.cpp:3-16 (probe of Cblacs_pcoord(ctxt, 1))
//   ctxt -> MPI_Comm       scalapack.cpp:42-53 (Cblacs_get(ctxt, 10) + Cblacs2sys_handle)
// Difference: each matrix's process grid is read from ITS OWN descriptor context; the
// reference builds both p?gemr2d layouts with the grid of `ictxt` (costa_pxgemr2d.cpp:47,144,
// 157), which mis-describes A or C whenever the two grids differ.
#include <mpi.h>

#include <costa/mpi.hpp>
#include <costa/scalapack.h>

#include <cctype>
#include <complex>
#include <cstdio>
#include <cstdlib>

extern "C" {
// BLACS, resolved from the application's ScaLAPACK (reference blacs.hpp:6-35)
void Cblacs_gridinfo(int ictxt, int* nprow, int* npcol, int* myrow, int* mycol);
void Cblacs_pcoord(int ictxt, int nodenum, int* prow, int* pcol);
void Cblacs_get(int ictxt, int what, int* val);
MPI_Comm Cblacs2sys_handle(int ictxt);
}

namespace {

[[noreturn]] void fatal(const char* where, const std::exception& e) {
    std::fprintf(stderr, "costa %s: %s\n", where, e.what());
    std::fflush(stderr);
    std::abort();
}

MPI_Comm comm_of(int ctxt) {
    int sys = 0;
    Cblacs_get(ctxt, 10, &sys);
    return Cblacs2sys_handle(sys);
}

// 'R' if rank 1 sits at (0, 1) of the grid, else 'C' (scalapack.cpp:3-16)
char grid_order(int ctxt, int P) {
    if (P <= 1) return 'C';
    int r = -1, c = -1;
    Cblacs_pcoord(ctxt, 1, &r, &c);
    return (r == 0 && c == 1) ? 'R' : 'C';
}

struct grid {
    int pm = 0, pn = 0;
    char order = 'C';
};

grid grid_of(int ctxt, MPI_Comm comm) {
    grid g;
    int myr, myc;
    Cblacs_gridinfo(ctxt, &g.pm, &g.pn, &myr, &myc);
    int P = 1;
    MPI_Comm_size(comm, &P);
    if (g.pm < 1 || g.pn < 1)
        throw std::runtime_error("this process is not part of the matrix's BLACS context");
    g.order = grid_order(ctxt, P);
    return g;
}

template <typename T>
costa::grid_layout<T> layout_of(const int* desc, int i, int j, int sub_m, int sub_n,
                                const grid& g, T* ptr, int rank) {
    return costa::block_cyclic_layout<T>(desc[2], desc[3], desc[4], desc[5], i, j, sub_m, sub_n,
                                         g.pm, g.pn, g.order, desc[6], desc[7], ptr, desc[8], 'C',
                                         rank);
}

template <typename T>
void pxgemr2d(int m, int n, const T* a, int ia, int ja, const int* desca, T* c, int ic, int jc,
              const int* descc, int ictxt) {
    if (m == 0 || n == 0) return;
    try {
        MPI_Comm comm = comm_of(ictxt);
        int rank = 0;
        MPI_Comm_rank(comm, &rank);
        const grid ga = grid_of(desca[1], comm), gc = grid_of(descc[1], comm);
        auto A = layout_of<T>(desca, ia, ja, m, n, ga, const_cast<T*>(a), rank);
        auto C = layout_of<T>(descc, ic, jc, m, n, gc, c, rank);
        costa::transform<T>(A, C, costa::comm_from_mpi(comm));
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
        MPI_Comm comm = comm_of(desca[1]);
        int rank = 0;
        MPI_Comm_rank(comm, &rank);
        const grid g = grid_of(desca[1], comm);
        auto A = layout_of<T>(desca, ia, ja, n, m, g, const_cast<T*>(a), rank);  // n x m
        auto C = layout_of<T>(descc, ic, jc, m, n, g, c, rank);
        costa::transform<T>(A, C, op, alpha, beta, costa::comm_from_mpi(comm));
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
