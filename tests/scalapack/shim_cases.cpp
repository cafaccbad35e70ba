// ScaLAPACK wrapper cases, one source built three ways (tests/test_scalapack_dropin.py):
//
//   -DSHIM_REF   linked with the REFERENCE's own wrappers and library, compiled from
//                /root/reference by oracle/Makefile (`make -C oracle scalapack`): writes every
//                process's local C after each case (`gen <dir>`); tests/golden/
//                make_scalapack_fixtures.py stores them as tests/golden/scalapack_np{1,4}.npz.
//                Reference entry points: prefixed_pxgemr2d.cpp (costa::pxgemr2d<T>,
//                costa_pxgemr2d.cpp:14-171), prefixed_pxtran{,u,c}.cpp (costa::pxtran_op<T>,
//                costa_pxtran_op.cpp:15-170).
//   (default)    linked with libcosta_amd_prefixed_scalapack.so: the shipped shims on the GPU
//                (one process: the 1-rank cases).
//   -DSHIM_HOOK  our shims (costa_amd/csrc/scalapack.cpp) compiled in with the test hook, which
//                hands the two layouts they build to a CPU executor: A gathered over the
//                processes, then the oracle (oracle/liboracle.so) applied to this process's
//                C blocks. 4 processes, no GPU: pins the shims' descriptor handling and grid
//                mapping at more than one process.
// `check <dir>` compares every process's local C, byte for byte (padding rows of lld included),
// with the files in <dir>; prints one line per case and "ALL PASSED" on success.
//
// Cases use Cblacs_gridinit grids over all processes (the reference builds both p?gemr2d layouts
// on ictxt's grid, costa_pxgemr2d.cpp:47,144,157, so A, C and ictxt share one context here).
#include <mpi.h>

#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#ifdef SHIM_HOOK
#include <costa/layout.hpp>
template <typename T>
void oracle_run(costa::grid_layout<T>& A, costa::grid_layout<T>& C, char op, T alpha, T beta, MPI_Comm comm);
#define COSTA_SCALAPACK_TEST_HOOK(A, C, op, alpha, beta, comm) oracle_run(A, C, op, alpha, beta, comm)
#include "../../costa_amd/csrc/scalapack.cpp"
#endif

extern "C" {
void Cblacs_pinfo(int*, int*);
void Cblacs_get(int, int, int*);
void Cblacs_gridinit(int*, char*, int, int);
void Cblacs_gridinfo(int, int*, int*, int*, int*);
void Cblacs_gridexit(int);
int numroc_(const int*, const int*, const int*, const int*, const int*);

#ifndef SHIM_HOOK  // the shims under test: the reference's or ours, same prefixed C ABI
#define GEMR2D(T) \
    const int*, const int*, const T*, const int*, const int*, const int*, T*, const int*, const int*, const int*, const int*
#define TRAN(T) \
    const int*, const int*, T*, const T*, const int*, const int*, const int*, const T*, T*, const int*, const int*, const int*
void costa_psgemr2d(GEMR2D(float));
void costa_pdgemr2d(GEMR2D(double));
void costa_pcgemr2d(GEMR2D(float));
void costa_pzgemr2d(GEMR2D(double));
void costa_pstran(TRAN(float));
void costa_pdtran(TRAN(double));
void costa_pctranu(TRAN(float));
void costa_pztranu(TRAN(double));
void costa_pctranc(TRAN(float));
void costa_pztranc(TRAN(double));
#endif
}

#ifdef SHIM_HOOK
extern "C" int oracle_transform(int t, char trans, const void* alpha, const void* beta, int a_nbr, int a_nbc,
                                const int* a_rs, const int* a_cs, const long long* a_tab, int a_cm,
                                void* const* a_bufs, int c_nbr, int c_nbc, const int* c_rs, const int* c_cs,
                                const long long* c_tab, int c_cm, void* const* c_bufs);
template <typename T> constexpr int oracle_type();
template <> constexpr int oracle_type<float>() { return 0; }
template <> constexpr int oracle_type<double>() { return 1; }
template <> constexpr int oracle_type<std::complex<float>>() { return 2; }
template <> constexpr int oracle_type<std::complex<double>>() { return 3; }
template <> constexpr int oracle_type<int>() { return 4; }  // costa_pigemr2d

// the CPU executor behind the hook: every process ORs its A blocks into a zeroed copy of the
// whole sub(A) (each element is held by exactly one process), then the oracle computes this
// process's C blocks from it
template <typename T>
void oracle_run(costa::grid_layout<T>& A, costa::grid_layout<T>& C, char op, T alpha, T beta, MPI_Comm comm) {
    const int ar = A.num_rows(), ac = A.num_cols();
    std::vector<T> g(size_t(ar) * size_t(ac));
    std::memset(static_cast<void*>(g.data()), 0, g.size() * sizeof(T));
    for (int b = 0; b < A.blocks.num_blocks(); ++b) {
        const auto& blk = A.blocks.get_block(b);
        for (int j = blk.cols_interval.start; j < blk.cols_interval.end; ++j)
            for (int i = blk.rows_interval.start; i < blk.rows_interval.end; ++i)
                g[size_t(j) * size_t(ar) + size_t(i)] =
                    blk.local_element(i - blk.rows_interval.start, j - blk.cols_interval.start);
    }
    MPI_Allreduce(MPI_IN_PLACE, g.data(), int(g.size() * sizeof(T)), MPI_BYTE, MPI_BOR, comm);
    const int a_rs[2] = {0, ar}, a_cs[2] = {0, ac};
    const long long a_tab[3] = {0, 0, ar};
    void* a_bufs[1] = {g.data()};
    const auto& cg = C.grid.grid();
    std::vector<long long> c_tab(size_t(cg.n_rows) * size_t(cg.n_cols) * 3, -1);
    std::vector<void*> c_bufs;
    for (int b = 0; b < C.blocks.num_blocks(); ++b) {
        const auto& blk = C.blocks.get_block(b);
        long long* e = &c_tab[(size_t(blk.coordinates.row) * size_t(cg.n_cols) + size_t(blk.coordinates.col)) * 3];
        e[0] = (long long)c_bufs.size();
        e[1] = 0;
        e[2] = blk.stride;
        c_bufs.push_back(blk.data);
    }
    const int rc = oracle_transform(oracle_type<T>(), op, &alpha, &beta, 1, 1, a_rs, a_cs, a_tab, 1, a_bufs,
                                    cg.n_rows, cg.n_cols, cg.rows_split.data(), cg.cols_split.data(),
                                    c_tab.data(), 1, c_bufs.data());
    if (rc != 0) {
        std::fprintf(stderr, "oracle_transform failed (%d)\n", rc);
        MPI_Abort(MPI_COMM_WORLD, 3);
    }
}
#endif

namespace {

struct mat {  // one distributed matrix of a case
    int M, N, MB, NB, rsrc, csrc, i, j, pad;  // i, j: 1-based start of the sub-matrix; pad: lld - lr
};

struct case_t {
    const char* name;
    char fn;  // 'G' p?gemr2d, 'T' p?tran, 'U' p?tranu, 'C' p?tranc
    char ty;  // 's' 'd' 'c' 'z'
    int m, n;  // sub(C) is m x n; sub(A) m x n for 'G', n x m otherwise
    mat a, c;
    double alpha[2], beta[2];
    bool c_nan;  // C starts as NaN (beta = 0 must not read it)
    int pm, pn;
    char order;  // Cblacs_gridinit order
};

// one-process cases and four-process cases (every grid covers all processes)
const std::vector<case_t>& cases(int np) {
    static const std::vector<case_t> one = {
        {"gemr2d_d", 'G', 'd', 150, 130, {170, 160, 16, 12, 0, 0, 11, 7, 3}, {165, 140, 20, 9, 0, 0, 3, 5, 0}, {1, 0}, {0, 0}, false, 1, 1, 'R'},
        {"gemr2d_s", 'G', 's', 97, 141, {120, 150, 32, 32, 0, 0, 1, 1, 0}, {100, 160, 7, 64, 0, 0, 4, 20, 5}, {1, 0}, {0, 0}, false, 1, 1, 'R'},
        {"gemr2d_c", 'G', 'c', 64, 80, {64, 90, 64, 16, 0, 0, 1, 11, 0}, {70, 80, 8, 8, 0, 0, 7, 1, 1}, {1, 0}, {0, 0}, false, 1, 1, 'R'},
        {"gemr2d_z", 'G', 'z', 75, 60, {80, 70, 13, 17, 0, 0, 6, 11, 2}, {75, 61, 25, 25, 0, 0, 1, 2, 0}, {1, 0}, {0, 0}, false, 1, 1, 'R'},
        {"tran_d", 'T', 'd', 150, 170, {200, 160, 32, 24, 0, 0, 7, 1, 0}, {160, 190, 20, 48, 0, 0, 2, 4, 1}, {0.75, 0}, {-1.5, 0}, false, 1, 1, 'R'},
        {"tran_d_copy_nanC", 'T', 'd', 128, 96, {100, 130, 16, 16, 0, 0, 3, 2, 0}, {130, 100, 32, 8, 0, 0, 1, 5, 0}, {1, 0}, {0, 0}, true, 1, 1, 'R'},
        {"tran_d_alpha_only", 'T', 'd', 60, 90, {90, 60, 8, 12, 0, 0, 1, 1, 0}, {60, 90, 12, 8, 0, 0, 1, 1, 0}, {2.5, 0}, {0, 0}, true, 1, 1, 'R'},
        {"tran_d_zero", 'T', 'd', 40, 50, {50, 40, 8, 8, 0, 0, 1, 1, 0}, {40, 50, 8, 8, 0, 0, 1, 1, 0}, {0, 0}, {0, 0}, false, 1, 1, 'R'},
        {"tran_s", 'T', 's', 111, 87, {90, 120, 16, 32, 0, 0, 2, 9, 4}, {120, 90, 24, 24, 0, 0, 5, 3, 0}, {-0.5, 0}, {2, 0}, false, 1, 1, 'R'},
        {"tranu_z", 'U', 'z', 70, 90, {90, 70, 16, 16, 0, 0, 1, 1, 0}, {70, 90, 24, 8, 0, 0, 1, 1, 0}, {0.75, -0.5}, {1.25, 0.25}, false, 1, 1, 'R'},
        {"tranc_z", 'C', 'z', 70, 90, {95, 72, 16, 16, 0, 0, 3, 2, 1}, {72, 95, 24, 8, 0, 0, 2, 4, 0}, {0.75, -0.5}, {1.25, 0.25}, false, 1, 1, 'R'},
        {"tranu_c", 'U', 'c', 50, 66, {66, 50, 10, 10, 0, 0, 1, 1, 0}, {50, 66, 9, 11, 0, 0, 1, 1, 0}, {1, 0}, {0, 0}, false, 1, 1, 'R'},
        {"tranc_c", 'C', 'c', 50, 66, {70, 55, 10, 10, 0, 0, 4, 3, 0}, {55, 70, 9, 11, 0, 0, 2, 3, 2}, {-1, 0.5}, {0.5, 0}, false, 1, 1, 'R'},
    };
    static const std::vector<case_t> four = {
        {"gemr2d_d_2x2R", 'G', 'd', 150, 130, {170, 160, 16, 12, 1, 1, 11, 7, 2}, {165, 140, 20, 9, 0, 1, 3, 5, 0}, {1, 0}, {0, 0}, false, 2, 2, 'R'},
        {"gemr2d_z_2x2C", 'G', 'z', 75, 60, {80, 70, 13, 17, 1, 0, 6, 11, 0}, {75, 61, 25, 25, 0, 0, 1, 2, 1}, {1, 0}, {0, 0}, false, 2, 2, 'C'},
        {"gemr2d_s_1x4R", 'G', 's', 97, 141, {120, 150, 32, 32, 0, 3, 1, 1, 0}, {100, 160, 7, 16, 0, 1, 4, 20, 3}, {1, 0}, {0, 0}, false, 1, 4, 'R'},
        {"gemr2d_c_4x1C", 'G', 'c', 64, 80, {64, 90, 8, 16, 2, 0, 1, 11, 0}, {70, 80, 8, 8, 3, 0, 7, 1, 0}, {1, 0}, {0, 0}, false, 4, 1, 'C'},
        {"tran_d_2x2R", 'T', 'd', 150, 170, {200, 160, 32, 24, 1, 0, 7, 1, 0}, {160, 190, 20, 48, 1, 1, 2, 4, 1}, {0.75, 0}, {-1.5, 0}, false, 2, 2, 'R'},
        {"tran_d_copy_nanC_2x2C", 'T', 'd', 128, 96, {100, 130, 16, 16, 0, 1, 3, 2, 0}, {130, 100, 32, 8, 1, 0, 1, 5, 0}, {1, 0}, {0, 0}, true, 2, 2, 'C'},
        {"tran_s_4x1C", 'T', 's', 111, 87, {90, 120, 16, 32, 3, 0, 2, 9, 0}, {120, 90, 24, 24, 1, 0, 5, 3, 2}, {-0.5, 0}, {2, 0}, false, 4, 1, 'C'},
        {"tranu_z_2x2C", 'U', 'z', 70, 90, {90, 70, 16, 16, 1, 1, 1, 1, 0}, {70, 90, 24, 8, 0, 1, 1, 1, 0}, {0.75, -0.5}, {1.25, 0.25}, false, 2, 2, 'C'},
        {"tranc_c_1x4R", 'C', 'c', 50, 66, {70, 55, 10, 10, 0, 2, 4, 3, 0}, {55, 70, 9, 11, 0, 3, 2, 3, 1}, {-1, 0.5}, {0.5, 0}, false, 1, 4, 'R'},
        {"tranc_z_2x2R", 'C', 'z', 70, 90, {95, 72, 16, 16, 0, 1, 3, 2, 1}, {72, 95, 24, 8, 1, 0, 2, 4, 0}, {0.75, -0.5}, {1.25, 0.25}, false, 2, 2, 'R'},
    };
    static const std::vector<case_t> none;
    return np == 1 ? one : np == 4 ? four : none;
}

// deterministic value of element (i, j) (global, 0-based) of stream s in [-1, 1)
double val(long i, long j, unsigned s) {
    uint32_t h = uint32_t(i + 7) * 2654435761u ^ uint32_t(j + 13) * 2246822519u ^ s * 3266489917u;
    h ^= h >> 15;
    h *= 2246822519u;
    h ^= h >> 13;
    return double(h % 2000001u) / 1000000.0 - 1.0;
}

int local_to_global(int l, int nb, int me, int src, int np) {
    return (l / nb * np + (me - src + np) % np) * nb + l % nb;
}

struct local_t {
    int lr, lc, lld;
};

local_t local_dims(const mat& x, int myr, int myc, int pm, int pn) {
    local_t d;
    d.lr = numroc_(&x.M, &x.MB, &myr, &x.rsrc, &pm);
    d.lc = numroc_(&x.N, &x.NB, &myc, &x.csrc, &pn);
    d.lld = (d.lr > 1 ? d.lr : 1) + x.pad;
    return d;
}

// fills a local array of element type T (complex: two reals per element)
template <typename R>
void fill(std::vector<R>& buf, int cplx, const mat& x, const local_t& d, int myr, int myc, int pm, int pn,
          unsigned stream, bool nan) {
    const int per = cplx ? 2 : 1;
    buf.assign(size_t(d.lld) * size_t(d.lc > 0 ? d.lc : 1) * per, R(0));
    for (int lj = 0; lj < d.lc; ++lj)
        for (int li = 0; li < d.lld; ++li) {
            const size_t k = (size_t(lj) * size_t(d.lld) + size_t(li)) * per;
            const bool in = li < d.lr;
            const long gi = in ? local_to_global(li, x.MB, myr, x.rsrc, pm) : -1 - li;
            const long gj = local_to_global(lj, x.NB, myc, x.csrc, pn);
            for (int p = 0; p < per; ++p)
                buf[k + size_t(p)] = nan ? R(std::nan("")) : R(val(gi, gj, stream + unsigned(p)));
        }
}

template <typename R>
void call(const case_t& k, const R* a, R* c, const int* desca, const int* descc, int ctxt) {
    R al[2] = {R(k.alpha[0]), R(k.alpha[1])}, be[2] = {R(k.beta[0]), R(k.beta[1])};
    const int m = k.m, n = k.n, ia = k.a.i, ja = k.a.j, ic = k.c.i, jc = k.c.j;
    constexpr bool dbl = sizeof(R) == 8;
#define PFX(x) costa_##x
    if (k.fn == 'G') {
        if (k.ty == 's' || k.ty == 'd') {
            if constexpr (dbl) PFX(pdgemr2d)(&m, &n, a, &ia, &ja, desca, c, &ic, &jc, descc, &ctxt);
            else PFX(psgemr2d)(&m, &n, a, &ia, &ja, desca, c, &ic, &jc, descc, &ctxt);
        } else {
            if constexpr (dbl) PFX(pzgemr2d)(&m, &n, a, &ia, &ja, desca, c, &ic, &jc, descc, &ctxt);
            else PFX(pcgemr2d)(&m, &n, a, &ia, &ja, desca, c, &ic, &jc, descc, &ctxt);
        }
    } else if (k.fn == 'T') {
        if constexpr (dbl) PFX(pdtran)(&m, &n, al, a, &ia, &ja, desca, be, c, &ic, &jc, descc);
        else PFX(pstran)(&m, &n, al, a, &ia, &ja, desca, be, c, &ic, &jc, descc);
    } else if (k.fn == 'U') {
        if constexpr (dbl) PFX(pztranu)(&m, &n, al, a, &ia, &ja, desca, be, c, &ic, &jc, descc);
        else PFX(pctranu)(&m, &n, al, a, &ia, &ja, desca, be, c, &ic, &jc, descc);
    } else {
        if constexpr (dbl) PFX(pztranc)(&m, &n, al, a, &ia, &ja, desca, be, c, &ic, &jc, descc);
        else PFX(pctranc)(&m, &n, al, a, &ia, &ja, desca, be, c, &ic, &jc, descc);
    }
#undef PFX
}

int g_me = 0, g_fail = 0;

template <typename R>
void run_case(const case_t& k, bool gen, const std::string& dir) {
    int ctxt = 0, pm = 0, pn = 0, myr = 0, myc = 0;
    char order[2] = {k.order, 0};
    Cblacs_get(-1, 0, &ctxt);
    Cblacs_gridinit(&ctxt, order, k.pm, k.pn);
    Cblacs_gridinfo(ctxt, &pm, &pn, &myr, &myc);
    const int cplx = k.ty == 'c' || k.ty == 'z';
    const local_t da = local_dims(k.a, myr, myc, pm, pn), dc = local_dims(k.c, myr, myc, pm, pn);
    std::vector<R> a, c;
    fill(a, cplx, k.a, da, myr, myc, pm, pn, 1, false);
    fill(c, cplx, k.c, dc, myr, myc, pm, pn, 3, k.c_nan);
    const int desca[9] = {1, ctxt, k.a.M, k.a.N, k.a.MB, k.a.NB, k.a.rsrc, k.a.csrc, da.lld};
    const int descc[9] = {1, ctxt, k.c.M, k.c.N, k.c.MB, k.c.NB, k.c.rsrc, k.c.csrc, dc.lld};
    call<R>(k, a.data(), c.data(), desca, descc, ctxt);
    const std::string path = dir + "/" + k.name + ".r" + std::to_string(g_me) + ".bin";
    const size_t bytes = c.size() * sizeof(R);
    if (gen) {
        FILE* f = std::fopen(path.c_str(), "wb");
        if (!f || std::fwrite(c.data(), 1, bytes, f) != bytes) {
            std::printf("rank %d: cannot write %s\n", g_me, path.c_str());
            g_fail++;
        }
        if (f) std::fclose(f);
    } else {
        std::vector<char> want(bytes + 1);
        FILE* f = std::fopen(path.c_str(), "rb");
        const size_t got = f ? std::fread(want.data(), 1, bytes + 1, f) : 0;
        if (f) std::fclose(f);
        const bool ok = got == bytes && std::memcmp(want.data(), c.data(), bytes) == 0;
        size_t first = 0;
        if (got == bytes && !ok)
            while (first < bytes && want[first] == reinterpret_cast<const char*>(c.data())[first]) ++first;
        int all = ok, all_ok = 0;
        MPI_Allreduce(&all, &all_ok, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
        if (!ok)
            std::printf("rank %d: %s differs (%zu bytes read, %zu expected, first difference at byte %zu)\n",
                        g_me, k.name, got, bytes, first);
        if (g_me == 0) std::printf("%-28s %s\n", k.name, all_ok ? "ok" : "FAIL");
        g_fail += !ok;
    }
    Cblacs_gridexit(ctxt);
}

}  // namespace

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int np = 0;
    Cblacs_pinfo(&g_me, &np);
    if (argc != 3 || (std::strcmp(argv[1], "gen") && std::strcmp(argv[1], "check")) || cases(np).empty()) {
        if (g_me == 0) std::printf("usage: mpiexec -n {1|4} %s gen|check <dir>\n", argv[0]);
        MPI_Finalize();
        return 2;
    }
    const bool gen = argv[1][0] == 'g';
    for (const case_t& k : cases(np)) {
        if (k.ty == 's' || k.ty == 'c') run_case<float>(k, gen, argv[2]);
        else run_case<double>(k, gen, argv[2]);
    }
    int total = 0;
    MPI_Allreduce(&g_fail, &total, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD);
    if (g_me == 0) std::printf(total ? "FAILED %d\n" : "ALL PASSED\n", total);
    MPI_Finalize();
    return total ? 1 : 0;
}
