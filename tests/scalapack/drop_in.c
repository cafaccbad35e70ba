/* Drop-in check of the ScaLAPACK C ABI (libcosta_amd_prefixed_scalapack.so) through a real
 * BLACS (MKL BLACS over the image's MPICH), 1 MPI rank, GPU execution.
 *
 * For each case: block-cyclic A and C on a BLACS grid, submatrix offsets, then
 *   costa_pdgemr2d / costa_pzgemr2d  vs  MKL ScaLAPACK pdgemr2d_ / pzgemr2d_  (bit copies: equal)
 *   costa_pdtran, costa_pztranu, costa_pztranc, costa_pstran vs values computed here
 *     element by element with separate roundings (built with -ffp-contract=off)
 * Exit status 0 = every check passed.  Prints one line per case.
 */
#include <complex.h>
#include <math.h>
#include <mpi.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "costa/scalapack.h"

void Cblacs_pinfo(int*, int*);
void Cblacs_get(int, int, int*);
void Cblacs_gridinit(int*, char*, int, int);
void Cblacs_gridinfo(int, int*, int*, int*, int*);
void Cblacs_gridexit(int);
int numroc_(const int*, const int*, const int*, const int*, const int*);
void descinit_(int*, const int*, const int*, const int*, const int*, const int*, const int*,
               const int*, const int*, int*);
void pdgemr2d_(const int*, const int*, const double*, const int*, const int*, const int*, double*,
               const int*, const int*, const int*, const int*);

static int failures = 0;

typedef struct {
    int M, N, mb, nb, lld, lr, lc;
    int desc[9];
} dmat;

static void mkdesc(dmat* d, int M, int N, int mb, int nb, int ctxt, int myr, int myc, int pr,
                   int pc) {
    int z = 0, info = 0;
    d->M = M; d->N = N; d->mb = mb; d->nb = nb;
    d->lr = numroc_(&M, &mb, &myr, &z, &pr);
    d->lc = numroc_(&N, &nb, &myc, &z, &pc);
    d->lld = d->lr > 1 ? d->lr : 1;
    descinit_(d->desc, &M, &N, &mb, &nb, &z, &z, &ctxt, &d->lld, &info);
}

/* global (i, j) of local (li, lj) on a 1x1 grid is (li, lj) */
static double va(int i, int j) { return 0.5 + i * 1.25 - j * 0.75 + (i * 31 + j * 17) % 13; }

static void check(const char* name, int ok) {
    printf("%-44s %s\n", name, ok ? "ok" : "FAIL");
    if (!ok) failures++;
}

int main(int argc, char** argv) {
    MPI_Init(&argc, &argv);
    int me, np, ctxt, pr, pc, myr, myc;
    Cblacs_pinfo(&me, &np);
    Cblacs_get(-1, 0, &ctxt);
    Cblacs_gridinit(&ctxt, "R", 1, np);
    Cblacs_gridinfo(ctxt, &pr, &pc, &myr, &myc);

    /* ---- p?gemr2d: 300x200 sub-block at (5, 9) of A (37x41 blocks) -> (3, 2) of C (64x64) */
    {
        dmat A, C1, C2;
        mkdesc(&A, 320, 230, 37, 41, ctxt, myr, myc, pr, pc);
        mkdesc(&C1, 310, 260, 64, 64, ctxt, myr, myc, pr, pc);
        C2 = C1;
        double* a = malloc(sizeof(double) * A.lld * A.lc);
        double* c1 = malloc(sizeof(double) * C1.lld * C1.lc);
        double* c2 = malloc(sizeof(double) * C1.lld * C1.lc);
        for (int j = 0; j < A.lc; ++j)
            for (int i = 0; i < A.lr; ++i) a[i + (size_t)j * A.lld] = va(i, j);
        for (int k = 0; k < C1.lld * C1.lc; ++k) c1[k] = c2[k] = -1.0 - k;
        int m = 300, n = 200, ia = 5, ja = 9, ic = 3, jc = 2;
        costa_pdgemr2d(&m, &n, a, &ia, &ja, A.desc, c1, &ic, &jc, C1.desc, &ctxt);
        pdgemr2d_(&m, &n, a, &ia, &ja, A.desc, c2, &ic, &jc, C2.desc, &ctxt);
        check("pdgemr2d 300x200 (5,9)->(3,2) == MKL", !memcmp(c1, c2, sizeof(double) * C1.lld * C1.lc));
        int ok = 1;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < m; ++i)
                ok &= c1[(ic - 1 + i) + (size_t)(jc - 1 + j) * C1.lld] == a[(ia - 1 + i) + (size_t)(ja - 1 + j) * A.lld];
        check("pdgemr2d values", ok);
        /* m == 0 returns without touching C */
        int zero = 0;
        costa_pdgemr2d(&zero, &n, a, &ia, &ja, A.desc, c1, &ic, &jc, C1.desc, &ctxt);
        check("pdgemr2d m=0 no-op", !memcmp(c1, c2, sizeof(double) * C1.lld * C1.lc));
        free(a); free(c1); free(c2);
    }
    /* ---- pdtran: C(150x170 at (2,4)) = beta*C + alpha*A^T, A 170x150 at (7,1) */
    {
        dmat A, C;
        mkdesc(&A, 200, 160, 32, 24, ctxt, myr, myc, pr, pc);
        mkdesc(&C, 160, 190, 20, 48, ctxt, myr, myc, pr, pc);
        double* a = malloc(sizeof(double) * A.lld * A.lc);
        double* c = malloc(sizeof(double) * C.lld * C.lc);
        double* c0 = malloc(sizeof(double) * C.lld * C.lc);
        for (int j = 0; j < A.lc; ++j)
            for (int i = 0; i < A.lr; ++i) a[i + (size_t)j * A.lld] = va(i, j);
        for (int k = 0; k < C.lld * C.lc; ++k) c[k] = c0[k] = 0.25 * k - 3.0;
        int m = 150, n = 170, ia = 7, ja = 1, ic = 2, jc = 4;
        double alpha = 0.75, beta = -1.5;
        costa_pdtran(&m, &n, &alpha, a, &ia, &ja, A.desc, &beta, c, &ic, &jc, C.desc);
        int ok = 1;
        for (int k = 0; k < C.lld * C.lc; ++k) {
            int i = k % C.lld, j = k / C.lld;
            double want = c0[k];
            if (i >= ic - 1 && i < ic - 1 + m && j >= jc - 1 && j < jc - 1 + n) {
                double x = a[(ia - 1 + (j - jc + 1)) + (size_t)(ja - 1 + (i - ic + 1)) * A.lld];
                double p = beta * c0[k], q = alpha * x;
                want = p + q;
            }
            ok &= memcmp(&want, &c[k], sizeof(double)) == 0;
        }
        check("pdtran alpha=.75 beta=-1.5 (bit-exact)", ok);
        free(a); free(c); free(c0);
    }
    /* ---- pztranu / pztranc: complex<double>, alpha/beta complex */
    for (int conj = 0; conj < 2; ++conj) {
        dmat A, C;
        mkdesc(&A, 90, 70, 16, 16, ctxt, myr, myc, pr, pc);
        mkdesc(&C, 70, 90, 24, 8, ctxt, myr, myc, pr, pc);
        double* a = malloc(2 * sizeof(double) * A.lld * A.lc);
        double* c = malloc(2 * sizeof(double) * C.lld * C.lc);
        double* c0 = malloc(2 * sizeof(double) * C.lld * C.lc);
        for (int k = 0; k < A.lld * A.lc; ++k) { a[2 * k] = va(k, 1); a[2 * k + 1] = va(3, k) * 0.5; }
        for (int k = 0; k < C.lld * C.lc; ++k) { c[2 * k] = c0[2 * k] = 0.5 * k; c[2 * k + 1] = c0[2 * k + 1] = -0.25 * k; }
        int m = 70, n = 90, one = 1;
        double alpha[2] = {0.75, -0.5}, beta[2] = {1.25, 0.25};
        if (conj) costa_pztranc(&m, &n, alpha, a, &one, &one, A.desc, beta, c, &one, &one, C.desc);
        else costa_pztranu(&m, &n, alpha, a, &one, &one, A.desc, beta, c, &one, &one, C.desc);
        int ok = 1;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < m; ++i) {
                size_t kc = i + (size_t)j * C.lld, ka = j + (size_t)i * A.lld;
                double xr = a[2 * ka], xi = conj ? -a[2 * ka + 1] : a[2 * ka + 1];
                double yr = c0[2 * kc], yi = c0[2 * kc + 1];
                double pr_ = alpha[0] * xr - alpha[1] * xi, pi_ = alpha[0] * xi + alpha[1] * xr;
                double qr = beta[0] * yr - beta[1] * yi, qi = beta[0] * yi + beta[1] * yr;
                double wr = qr + pr_, wi = qi + pi_;
                ok &= !memcmp(&wr, &c[2 * kc], 8) && !memcmp(&wi, &c[2 * kc + 1], 8);
            }
        check(conj ? "pztranc complex alpha,beta (bit-exact)" : "pztranu complex alpha,beta (bit-exact)", ok);
        free(a); free(c); free(c0);
    }
    /* ---- pstran: float, alpha=1 beta=0 -> exact transpose */
    {
        dmat A, C;
        mkdesc(&A, 33, 47, 8, 5, ctxt, myr, myc, pr, pc);
        mkdesc(&C, 47, 33, 7, 9, ctxt, myr, myc, pr, pc);
        float* a = malloc(sizeof(float) * A.lld * A.lc);
        float* c = malloc(sizeof(float) * C.lld * C.lc);
        for (int k = 0; k < A.lld * A.lc; ++k) a[k] = (float)va(k, 2);
        for (int k = 0; k < C.lld * C.lc; ++k) c[k] = NAN;  /* beta = 0: C must not be read */
        int m = 47, n = 33, one = 1;
        float alpha = 1.f, beta = 0.f;
        costa_pstran(&m, &n, &alpha, a, &one, &one, A.desc, &beta, c, &one, &one, C.desc);
        int ok = 1;
        for (int j = 0; j < n; ++j)
            for (int i = 0; i < m; ++i) ok &= c[i + j * C.lld] == a[j + i * A.lld];
        check("pstran alpha=1 beta=0 over NaN C", ok);
        free(a); free(c);
    }
    Cblacs_gridexit(ctxt);
    MPI_Finalize();
    printf("%s\n", failures ? "FAILED" : "ALL PASSED");
    return failures ? 1 : 0;
}
