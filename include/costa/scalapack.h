/*
 * costa-mi355x — ScaLAPACK-compatible C ABI (drop-in for COSTA's costa_scalapack and
 * costa_prefixed_scalapack libraries).
 *
 *   libcosta_amd_scalapack.so           plain names: link it before ScaLAPACK to interpose
 *   libcosta_amd_prefixed_scalapack.so  the same functions with a costa_ prefix
 *
 * Reference declarations replaced (eth-cscs/COSTA):
 *   p{s,d,c,z}gemr2d[_,__,UPPER]          src/costa/pxgemr2d/pxgemr2d.h:7-160
 *   p{s,d}tran[_,__,UPPER]                src/costa/pxtran/pxtran.h:7-84       (op 'T')
 *   p{c,z}tranu[_,__,UPPER]               src/costa/pxtranu/pxtranu.h:7-86     (op 'T')
 *   p{c,z}tranc[_,__,UPPER]               src/costa/pxtranc/pxtranc.h:7-86     (op 'C')
 *   costa_p{s,d,c,z,i}gemr2d[_,__]        src/costa/pxgemr2d/prefixed_pxgemr2d.h
 *   costa_p{s,d}tran, costa_p{c,z}tranu, costa_p{c,z}tranc [_,__]   prefixed_pxtran*.h
 *
 * Semantics (ScaLAPACK):  p?gemr2d copies sub(A) (m x n at (ia, ja)) into sub(C) at (ic, jc);
 * p?tran* compute sub(C) = beta*sub(C) + alpha*op(sub(A)), sub(C) m x n, sub(A) n x m.
 * Descriptor fields: desc[1] context, [2..3] M, N, [4..5] MB, NB, [6..7] RSRC, CSRC, [8] LLD.
 * m == 0 or n == 0 returns immediately.  Errors are fatal (message + abort), as in the
 * reference.  Complex arguments are interleaved (re, im) float/double pairs.
 * The BLACS (Cblacs_*) and MPI symbols are resolved from the application's ScaLAPACK/MPI
 * (MPICH ABI: MPICH, Intel MPI, Cray MPICH).
 */
#ifndef COSTA_SCALAPACK_H
#define COSTA_SCALAPACK_H

#ifdef __cplusplus
extern "C" {
#endif

#define COSTA_GEMR2D_ARGS(T)                                                               \
    const int *m, const int *n, const T *a, const int *ia, const int *ja, const int *desca, \
        T *c, const int *ic, const int *jc, const int *descc, const int *ictxt
#define COSTA_TRAN_ARGS(T)                                                                  \
    const int *m, const int *n, T *alpha, const T *a, const int *ia, const int *ja,          \
        const int *desca, const T *beta, T *c, const int *ic, const int *jc, const int *descc

#define COSTA_DECL4(ret, name, args) \
    ret name(args);                  \
    ret name##_(args);               \
    ret name##__(args);

/* plain names (+ UPPER aliases below) */
COSTA_DECL4(void, psgemr2d, COSTA_GEMR2D_ARGS(float))
COSTA_DECL4(void, pdgemr2d, COSTA_GEMR2D_ARGS(double))
COSTA_DECL4(void, pcgemr2d, COSTA_GEMR2D_ARGS(float))
COSTA_DECL4(void, pzgemr2d, COSTA_GEMR2D_ARGS(double))
COSTA_DECL4(void, pstran, COSTA_TRAN_ARGS(float))
COSTA_DECL4(void, pdtran, COSTA_TRAN_ARGS(double))
COSTA_DECL4(void, pctranu, COSTA_TRAN_ARGS(float))
COSTA_DECL4(void, pztranu, COSTA_TRAN_ARGS(double))
COSTA_DECL4(void, pctranc, COSTA_TRAN_ARGS(float))
COSTA_DECL4(void, pztranc, COSTA_TRAN_ARGS(double))
void PSGEMR2D(COSTA_GEMR2D_ARGS(float));
void PDGEMR2D(COSTA_GEMR2D_ARGS(double));
void PCGEMR2D(COSTA_GEMR2D_ARGS(float));
void PZGEMR2D(COSTA_GEMR2D_ARGS(double));
void PSTRAN(COSTA_TRAN_ARGS(float));
void PDTRAN(COSTA_TRAN_ARGS(double));
void PCTRANU(COSTA_TRAN_ARGS(float));
void PZTRANU(COSTA_TRAN_ARGS(double));
void PCTRANC(COSTA_TRAN_ARGS(float));
void PZTRANC(COSTA_TRAN_ARGS(double));

/* costa_-prefixed names */
COSTA_DECL4(void, costa_psgemr2d, COSTA_GEMR2D_ARGS(float))
COSTA_DECL4(void, costa_pdgemr2d, COSTA_GEMR2D_ARGS(double))
COSTA_DECL4(void, costa_pcgemr2d, COSTA_GEMR2D_ARGS(float))
COSTA_DECL4(void, costa_pzgemr2d, COSTA_GEMR2D_ARGS(double))
COSTA_DECL4(void, costa_pigemr2d, COSTA_GEMR2D_ARGS(int))
COSTA_DECL4(void, costa_pstran, COSTA_TRAN_ARGS(float))
COSTA_DECL4(void, costa_pdtran, COSTA_TRAN_ARGS(double))
COSTA_DECL4(void, costa_pctranu, COSTA_TRAN_ARGS(float))
COSTA_DECL4(void, costa_pztranu, COSTA_TRAN_ARGS(double))
COSTA_DECL4(void, costa_pctranc, COSTA_TRAN_ARGS(float))
COSTA_DECL4(void, costa_pztranc, COSTA_TRAN_ARGS(double))

#ifdef __cplusplus
}
#endif
#endif /* COSTA_SCALAPACK_H */
