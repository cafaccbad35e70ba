/*
 * TEST INFRASTRUCTURE ONLY — CPU restatement of COSTA's tile path, used as the parity
 * checker by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
 * Nothing in costa_amd/ links, loads or calls this file.
 *
 * Parity pin: checked against golden vectors produced by the reference itself
 * (oracle/_ref, compiled from /root/reference sources by oracle/Makefile; vectors in
 * tests/golden/, generator tests/golden/make_fixtures.py) and against the reference's own
 * unit-test known answers (tests/unit/test_utils.cpp).
 *
 * Restated from eth-cscs/COSTA (v2.3.2):
 *   oracle_copy_and_transform   src/costa/grid2grid/memory_utils.hpp:339-412
 *     copy (memcpy fast path + per-element branches)       memory_utils.hpp:20-51
 *     copy2D (row-major swaps dims; contiguous single copy) memory_utils.hpp:55-98
 *     transpose_col_major / transpose_row_major            memory_utils.hpp:101-291
 *     default_stride                                        memory_utils.hpp:330-337
 *   oracle_bc_table             block-cyclic geometry: scalapack_layout.cpp:152-285,
 *                               rank_from_grid scalapack_layout.cpp:40-56, numroc scalapack.cpp:56-94
 *   oracle_transform            the result of costa::transform (transform.cpp:162-200) stated
 *                               per element: C(i,j) = g(A(i,j) or A(j,i)) with g exactly the
 *                               branch copy_and_transform applies to the tile holding (i,j)
 *   oracle_transform_tiles      the reference's local (OpenMP) path: 256x256-blocked transpose
 *                               over tiles (communication_data.cpp:251-302 with
 *                               memory_utils.hpp:101-193), used as the timed CPU baseline
 *
 * Arithmetic: products and sums are separate roundings (build with -ffp-contract=off; the
 * reference's x86-64 build has no FMA), complex products as GCC's: (ac-bd, ad+bc) with the
 * C99 Annex G recovery of libgcc's __muldc3 / __mulsc3 when both parts are NaN (cmul_f/cmul_d).
 */
#include <math.h>
#include <stddef.h>
#include <stdlib.h>
#include <stdint.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

enum { OR_FLOAT = 0, OR_DOUBLE = 1, OR_CFLOAT = 2, OR_CDOUBLE = 3, OR_INT32 = 4 };

typedef struct { float re, im; } cf_t;
typedef struct { double re, im; } cd_t;

static size_t esize(int t) {
    switch (t) {
    case OR_FLOAT: return 4;
    case OR_DOUBLE: return 8;
    case OR_CFLOAT: return 8;
    case OR_CDOUBLE: return 16;
    case OR_INT32: return 4;
    }
    return 0;
}

/* ---------------------------------------------------------------- scalar rules */
/* kind: 0 memcpy, 1 zero, 2 alpha*x, 3 beta*y + alpha*x (memory_utils.hpp:29-48) */
static int kind_of(int t, const void* a, const void* b, int copy_mode, int conj) {
    int fast = 0, zero = 0, bzero = 0;
    switch (t) {
    case OR_FLOAT: {
        float x = *(const float*)a, y = *(const float*)b;
        fast = !(fabsf(x - 1.0f) > 0 || fabsf(y - 0.0f) > 0);
        zero = (x == 0.0f && y == 0.0f);
        bzero = (y == 0.0f);
        break;
    }
    case OR_DOUBLE: {
        double x = *(const double*)a, y = *(const double*)b;
        fast = !(fabs(x - 1.0) > 0 || fabs(y - 0.0) > 0);
        zero = (x == 0.0 && y == 0.0);
        bzero = (y == 0.0);
        break;
    }
    case OR_CFLOAT: {
        cf_t x = *(const cf_t*)a, y = *(const cf_t*)b;
        fast = !(hypotf(x.re - 1.0f, x.im) > 0 || hypotf(y.re, y.im) > 0);
        zero = (x.re == 0.0f && x.im == 0.0f && y.re == 0.0f && y.im == 0.0f);
        bzero = (y.re == 0.0f && y.im == 0.0f);
        break;
    }
    case OR_CDOUBLE: {
        cd_t x = *(const cd_t*)a, y = *(const cd_t*)b;
        fast = !(hypot(x.re - 1.0, x.im) > 0 || hypot(y.re, y.im) > 0);
        zero = (x.re == 0.0 && x.im == 0.0 && y.re == 0.0 && y.im == 0.0);
        bzero = (y.re == 0.0 && y.im == 0.0);
        break;
    }
    case OR_INT32: {
        int x = *(const int*)a, y = *(const int*)b;
        fast = !(abs(x - 1) > 0 || abs(y) > 0);
        zero = (x == 0 && y == 0);
        bzero = (y == 0);
        break;
    }
    }
    if (copy_mode && fast && !conj) return 0;
    if (zero) return 1;
    if (bzero) return 2;
    return 3;
}

/* Complex products as the reference's binary computes them.  std::complex<T>::operator* is
 * GCC's builtin complex multiply (C99 Annex G): the naive (ac - bd, ad + bc), and when BOTH parts
 * come out NaN a call to libgcc's __muldc3 / __mulsc3, which recovers infinities (third-party
 * code the reference links: GCC 11.4's libgcc, libgcc2.c; C99 G.5.1).  Restated here;
 * tests/test_oracle_golden.py pins this restatement to the compiler's own product over a grid of
 * special values, and tests/golden/specials_*.npz pin the whole path to the reference. */
#define ANNEX_G_MUL(NAME, R, INF, ISNAN, ISINF, COPYSIGN)                                     \
    static void NAME(R a, R b, R c, R d, R* re, R* im) {                                     \
        R ac = a * c, bd = b * d, ad = a * d, bc = b * c;                                    \
        R x = ac - bd, y = ad + bc;                                                          \
        if (ISNAN(x) && ISNAN(y)) {                                                          \
            int recalc = 0;                                                                  \
            if (ISINF(a) || ISINF(b)) { /* z infinite: box it, NaNs of w to 0 */             \
                a = COPYSIGN(ISINF(a) ? (R)1 : (R)0, a);                                     \
                b = COPYSIGN(ISINF(b) ? (R)1 : (R)0, b);                                     \
                if (ISNAN(c)) c = COPYSIGN((R)0, c);                                         \
                if (ISNAN(d)) d = COPYSIGN((R)0, d);                                         \
                recalc = 1;                                                                  \
            }                                                                                \
            if (ISINF(c) || ISINF(d)) { /* w infinite */                                     \
                c = COPYSIGN(ISINF(c) ? (R)1 : (R)0, c);                                     \
                d = COPYSIGN(ISINF(d) ? (R)1 : (R)0, d);                                     \
                if (ISNAN(a)) a = COPYSIGN((R)0, a);                                         \
                if (ISNAN(b)) b = COPYSIGN((R)0, b);                                         \
                recalc = 1;                                                                  \
            }                                                                                \
            if (!recalc && (ISINF(ac) || ISINF(bd) || ISINF(ad) || ISINF(bc))) {             \
                /* overflow: recover infinities, NaNs to 0 */                                \
                if (ISNAN(a)) a = COPYSIGN((R)0, a);                                         \
                if (ISNAN(b)) b = COPYSIGN((R)0, b);                                         \
                if (ISNAN(c)) c = COPYSIGN((R)0, c);                                         \
                if (ISNAN(d)) d = COPYSIGN((R)0, d);                                         \
                recalc = 1;                                                                  \
            }                                                                                \
            if (recalc) {                                                                    \
                R p = a * c, q = b * d, r = a * d, t = b * c;                                \
                x = INF * (p - q);                                                           \
                y = INF * (r + t);                                                           \
            }                                                                                \
        }                                                                                    \
        *re = x;                                                                             \
        *im = y;                                                                             \
    }
ANNEX_G_MUL(cmul_f, float, INFINITY, isnan, isinf, copysignf)
ANNEX_G_MUL(cmul_d, double, (double)INFINITY, isnan, isinf, copysign)

/* exported for tests/test_oracle_golden.py (the restatement against GCC's own product) */
void oracle_cmul(int t, const void* a, const void* b, void* out) {
    if (t == OR_CFLOAT) {
        const float* x = (const float*)a; const float* y = (const float*)b; float* o = (float*)out;
        cmul_f(x[0], x[1], y[0], y[1], &o[0], &o[1]);
    } else {
        const double* x = (const double*)a; const double* y = (const double*)b; double* o = (double*)out;
        cmul_d(x[0], x[1], y[0], y[1], &o[0], &o[1]);
    }
}

/* dst = g(src) for one element; `conj` applies only to complex types (block.hpp:13-25) */
static void apply1(int t, int kind, int conj, const void* a, const void* b, const void* src,
                   void* dst) {
    if (kind == 0) {
        memcpy(dst, src, esize(t));
        return;
    }
    switch (t) {
    case OR_FLOAT: {
        float x = *(const float*)src, al = *(const float*)a, be = *(const float*)b;
        float* d = (float*)dst;
        if (kind == 1) *d = 0.0f;
        else if (kind == 2) *d = al * x;
        else { float p = be * *d; float q = al * x; *d = p + q; }
        break;
    }
    case OR_DOUBLE: {
        double x = *(const double*)src, al = *(const double*)a, be = *(const double*)b;
        double* d = (double*)dst;
        if (kind == 1) *d = 0.0;
        else if (kind == 2) *d = al * x;
        else { double p = be * *d; double q = al * x; *d = p + q; }
        break;
    }
    case OR_INT32: {
        int x = *(const int*)src, al = *(const int*)a, be = *(const int*)b;
        int* d = (int*)dst;
        if (kind == 1) *d = 0;
        else if (kind == 2) *d = (int)((unsigned)al * (unsigned)x);
        else *d = (int)((unsigned)be * (unsigned)*d + (unsigned)al * (unsigned)x);
        break;
    }
    case OR_CFLOAT: {
        cf_t x = *(const cf_t*)src, al = *(const cf_t*)a, be = *(const cf_t*)b;
        cf_t* d = (cf_t*)dst;
        if (conj) x.im = -x.im;
        if (kind == 1) { d->re = 0.0f; d->im = 0.0f; break; }
        float pr, pi, qr, qi;
        cmul_f(al.re, al.im, x.re, x.im, &pr, &pi); /* alpha * el */
        if (kind == 2) { d->re = pr; d->im = pi; break; }
        cmul_f(be.re, be.im, d->re, d->im, &qr, &qi); /* beta * dst */
        d->re = qr + pr;
        d->im = qi + pi;
        break;
    }
    case OR_CDOUBLE: {
        cd_t x = *(const cd_t*)src, al = *(const cd_t*)a, be = *(const cd_t*)b;
        cd_t* d = (cd_t*)dst;
        if (conj) x.im = -x.im;
        if (kind == 1) { d->re = 0.0; d->im = 0.0; break; }
        double pr, pi, qr, qi;
        cmul_d(al.re, al.im, x.re, x.im, &pr, &pi); /* alpha * el */
        if (kind == 2) { d->re = pr; d->im = pi; break; }
        cmul_d(be.re, be.im, d->re, d->im, &qr, &qi); /* beta * dst */
        d->re = qr + pr;
        d->im = qi + pi;
        break;
    }
    }
}

/* ---------------------------------------------------------------- copy_and_transform */
void oracle_copy_and_transform(int t, int n_rows, int n_cols, const void* src, int src_stride,
                               int src_cm, void* dst, int dst_stride, int dst_cm, int transpose,
                               int conjugate, const void* alpha, const void* beta) {
    const size_t E = esize(t);
    const int cplx = (t == OR_CFLOAT || t == OR_CDOUBLE);
    const int conj = conjugate && cplx;
    const int will_t = (transpose && src_cm == dst_cm) || (!transpose && src_cm != dst_cm);
    if ((long long)n_rows * n_cols == 0) return;
    if (dst_stride == 0) {
        int r = will_t ? n_cols : n_rows, c = will_t ? n_rows : n_cols;
        dst_stride = dst_cm ? r : c;
    }
    if (src_stride == 0) src_stride = src_cm ? n_rows : n_cols;
    const char* s = (const char*)src;
    char* d = (char*)dst;
    /* F = contiguous extent of the source, S = strided extent */
    const int F = src_cm ? n_rows : n_cols, S = src_cm ? n_cols : n_rows;
    const int kind = kind_of(t, alpha, beta, !will_t, conj);
    if (!will_t) {
        /* copy2D: dst(f, s) at s*ldd + f */
        for (int j = 0; j < S; ++j)
            for (int i = 0; i < F; ++i)
                apply1(t, kind, conj, alpha, beta, s + ((size_t)j * src_stride + i) * E,
                       d + ((size_t)j * dst_stride + i) * E);
    } else {
        /* transpose: dst(s, f) at f*ldd + s */
        for (int j = 0; j < S; ++j)
            for (int i = 0; i < F; ++i)
                apply1(t, kind, conj, alpha, beta, s + ((size_t)j * src_stride + i) * E,
                       d + ((size_t)i * dst_stride + j) * E);
    }
}

/* ---------------------------------------------------------------- block-cyclic geometry */
static int numroc_(int n, int nb, int iproc, int isrc, int nprocs) {
    int dist = (nprocs + iproc - isrc) % nprocs, nblocks = n / nb;
    int len = (nblocks / nprocs) * nb, extra = nblocks % nprocs;
    if (dist < extra) len += nb;
    else if (dist == extra) len += n % nb;
    return len;
}
int oracle_numroc(int n, int nb, int iproc, int isrc, int nprocs) {
    return numroc_(n, nb, iproc, isrc, nprocs);
}

static int line_split_(int begin, int end, int nb, int* out) {
    int len = end - begin, rem = nb - begin % nb, k = 0;
    out[k++] = 0;
    if (rem >= len) { out[k++] = len; return k; }
    out[k++] = rem;
    for (int b = 0; b < (len - rem) / nb; ++b) { out[k] = out[k - 1] + nb; ++k; }
    if (out[k - 1] != len) out[k++] = len;
    return k;
}

/* Fills rows_split (<= sub_m/mb + 3 ints), cols_split, and tab[(i*nbc + j)*3 + {owner,
 * element offset in the owner's local buffer, ld}] for a ScaLAPACK layout whose ranks all
 * use the same `lld`.  Returns nbr*65536 + nbc. */
long long oracle_bc_table(int m, int n, int mb, int nb, int ia, int ja, int sub_m, int sub_n,
                          int pm, int pn, char order, int rsrc, int csrc, int lld, char data_ord,
                          int* rows_split, int* cols_split, long long* tab) {
    (void)m; (void)n;
    int i0 = ia - 1, j0 = ja - 1;
    int nr = line_split_(i0, i0 + sub_m, mb, rows_split) - 1;
    int nc = line_split_(j0, j0 + sub_n, nb, cols_split) - 1;
    int br = i0 / mb, bc = j0 / nb;
    int pr0 = (br % pm + rsrc) % pm, pc0 = (bc % pn + csrc) % pn;
    for (int i = 0; i < nr; ++i)
        for (int j = 0; j < nc; ++j) {
            int prow = (i % pm + pr0) % pm, pcol = (j % pn + pc0) % pn;
            int owner = (order == 'C' || order == 'c') ? pcol * pm + prow : prow * pn + pcol;
            long long lr = (long long)((br + i) / pm) * mb + (i0 + rows_split[i] - (long long)(br + i) * mb);
            long long lc = (long long)((bc + j) / pn) * nb + (j0 + cols_split[j] - (long long)(bc + j) * nb);
            long long off = (data_ord == 'R' || data_ord == 'r') ? lc + (long long)lld * lr
                                                                  : lr + (long long)lld * lc;
            long long* e = tab + ((long long)i * nc + j) * 3;
            e[0] = owner;
            e[1] = off;
            e[2] = lld;
        }
    return (long long)nr * 65536 + nc;
}

/* ---------------------------------------------------------------- global transform */
typedef struct {
    int nbr, nbc;
    const int* rs;         /* nbr+1 split ticks */
    const int* cs;         /* nbc+1 */
    const long long* tab;  /* per block: owner (-1: nobody holds it), element offset, ld */
    int col_major;
    void* const* bufs;     /* per rank */
} olayout;

static int find_cell(const int* split, int n, int x) {
    int lo = 0, hi = n; /* split[lo] <= x < split[hi] */
    while (hi - lo > 1) {
        int mid = (lo + hi) / 2;
        if (split[mid] <= x) lo = mid; else hi = mid;
    }
    return lo;
}

static char* elem_addr(const olayout* L, int gi, int gj, size_t E) {
    int i = find_cell(L->rs, L->nbr, gi), j = find_cell(L->cs, L->nbc, gj);
    const long long* e = L->tab + ((long long)i * L->nbc + j) * 3;
    if (e[0] < 0) return NULL;
    long long li = gi - L->rs[i], lj = gj - L->cs[j];
    long long off = e[1] + (L->col_major ? lj * e[2] + li : li * e[2] + lj);
    return (char*)L->bufs[e[0]] + off * (long long)E;
}

int oracle_transform(int t, char trans, const void* alpha, const void* beta,
                     int a_nbr, int a_nbc, const int* a_rs, const int* a_cs, const long long* a_tab,
                     int a_cm, void* const* a_bufs,
                     int c_nbr, int c_nbc, const int* c_rs, const int* c_cs, const long long* c_tab,
                     int c_cm, void* const* c_bufs) {
    const size_t E = esize(t);
    const int cplx = (t == OR_CFLOAT || t == OR_CDOUBLE);
    const int tr = (trans != 'N' && trans != 'n');
    const int conj = (trans == 'C' || trans == 'c') && cplx;
    /* ordering mismatch is itself a transpose (memory_utils.hpp:353-367) */
    const int will_t = (tr && a_cm == c_cm) || (!tr && a_cm != c_cm);
    const int kind = kind_of(t, alpha, beta, !will_t, conj);
    olayout A = {a_nbr, a_nbc, a_rs, a_cs, a_tab, a_cm, a_bufs};
    olayout C = {c_nbr, c_nbc, c_rs, c_cs, c_tab, c_cm, c_bufs};
    if (A.rs[A.nbr] != (tr ? C.cs[C.nbc] : C.rs[C.nbr])) return -1;
    if (A.cs[A.nbc] != (tr ? C.rs[C.nbr] : C.cs[C.nbc])) return -1;
    for (int i = 0; i < C.nbr; ++i)
        for (int j = 0; j < C.nbc; ++j) {
            if (C.tab[((long long)i * C.nbc + j) * 3] < 0) continue;
            for (int gj = C.cs[j]; gj < C.cs[j + 1]; ++gj)
                for (int gi = C.rs[i]; gi < C.rs[i + 1]; ++gi) {
                    char* d = elem_addr(&C, gi, gj, E);
                    const char* s = tr ? elem_addr(&A, gj, gi, E) : elem_addr(&A, gi, gj, E);
                    if (!s) return -2; /* source element held by nobody */
                    apply1(t, kind, conj, alpha, beta, s, d);
                }
        }
    return 0;
}

/* ---------------------------------------------------------------- CPU baseline
 * The reference's single-rank path for a list of local tile pairs: OpenMP over tiles, each
 * tile transposed in 256x256 sub-blocks (memory_utils.hpp:101-193; the nested omp region is
 * disabled inside the tile loop, :123-129) or copied column by column (:55-98).
 * tiles[k*6 + {src_off, src_ld, dst_off, dst_ld, F, S}] in elements; returns 0. */
int oracle_transform_tiles(int t, int will_transpose, int conj, const void* alpha,
                           const void* beta, const void* src, void* dst, const long long* tiles,
                           long long ntiles, int nthreads) {
    const size_t E = esize(t);
    const int kind = kind_of(t, alpha, beta, !will_transpose, conj);
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(static)
#endif
    for (long long k = 0; k < ntiles; ++k) {
        const long long* tl = tiles + k * 6;
        const char* s = (const char*)src + tl[0] * (long long)E;
        char* d = (char*)dst + tl[2] * (long long)E;
        const long long lds = tl[1], ldd = tl[3];
        const int F = (int)tl[4], S = (int)tl[5];
        if (!will_transpose) {
            for (int j = 0; j < S; ++j) {
                if (kind == 0) {
                    memcpy(d + j * ldd * (long long)E, s + j * lds * (long long)E, (size_t)F * E);
                    continue;
                }
                for (int i = 0; i < F; ++i)
                    apply1(t, kind, conj, alpha, beta, s + (j * lds + i) * (long long)E,
                           d + (j * ldd + i) * (long long)E);
            }
        } else {
            const int B = 256;
            for (int bj = 0; bj < S; bj += B)
                for (int bi = 0; bi < F; bi += B) {
                    int ei = bi + B < F ? bi + B : F, ej = bj + B < S ? bj + B : S;
                    for (int i = bi; i < ei; ++i)
                        for (int j = bj; j < ej; ++j)
                            apply1(t, kind, conj, alpha, beta, s + (j * lds + i) * (long long)E,
                                   d + ((long long)i * ldd + j) * (long long)E);
                }
        }
    }
    return 0;
}
