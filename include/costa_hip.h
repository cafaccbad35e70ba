/*
 * costa-mi355x — C ABI of the MI355X-native COSTA tile path (libcosta_amd.so).
 *
 * Plain pointers and sizes only; no C++ or torch types cross this boundary.
 * Every entry point returns a status code (COSTA_OK == 0); the message of the last
 * failure on the calling thread is available from costa_hip_last_error().
 * Exceptions never cross this boundary.
 *
 * Which reference interface each entry point replaces (paths under eth-cscs/COSTA):
 *
 *   costa_hip_block_cyclic_layout   costa::block_cyclic_layout<T>   src/costa/layout.hpp:70-86
 *   costa_hip_custom_layout         costa::custom_layout<T>         src/costa/layout.hpp:34-42
 *   costa_hip_transform             costa::transform<T>(A, C, trans, alpha, beta, comm)
 *                                                                  src/costa/grid2grid/transform.hpp:22-27
 *                                   (trans = 'N', alpha = 1, beta = 0 gives the no-scale
 *                                    overload transform.hpp:13-16)
 *   costa_hip_transform_batch       costa::transform<T>(vector<layout_ref>..., trans*, alpha*, beta*, comm)
 *                                   and costa::transformer<T>::transform()
 *                                                                  transform.hpp:38-43, transformer.hpp:8-62
 *   costa_hip_layout_reorder_ranks  grid_layout<T>::reorder_ranks   grid2grid/grid_layout.hpp:32-34
 *   costa_hip_copy_and_transform    costa::memory::copy_and_transform<T>
 *                                                                  src/costa/grid2grid/memory_utils.hpp:339-412
 *   costa_hip_execute_tiles         the pack / local / unpack loops
 *                                   communication_data.cpp:191-217 (copy_to_buffer),
 *                                   :219-244 (copy_from_buffer(idx)), :251-302 (copy_local_blocks)
 *   costa_hip_comm_*                the MPI_Comm argument of transform (one rank per GPU; the data
 *                                   exchange of exchange_async, transform.cpp:46-128, runs on RCCL)
 *   costa_hip_plan_export           utils::prepare_to_send / prepare_to_recv + communication_data
 *                                   ctor (utils.hpp:123-206, communication_data.cpp:103-164):
 *                                   the tile descriptor lists, host-only, for inspection and tests
 */
#ifndef COSTA_HIP_H
#define COSTA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define COSTA_OK 0
#define COSTA_ERR_ARG 1      /* invalid argument / inconsistent layouts */
#define COSTA_ERR_HIP 2      /* a HIP runtime call failed (e.g. no GPU) */
#define COSTA_ERR_NCCL 3     /* an RCCL call failed */
#define COSTA_ERR_INTERNAL 4 /* anything else (allocation failure, bug) */

/* ---- element types (the reference instantiates float, double, complex<float>,
 *      complex<double>: transform.cpp:284-376; int32 is the element type of the
 *      reference's own unit tests, tests/unit/test_utils.cpp) ---- */
typedef enum {
    COSTA_FLOAT = 0,
    COSTA_DOUBLE = 1,
    COSTA_CFLOAT = 2,  /* std::complex<float>, interleaved re/im */
    COSTA_CDOUBLE = 3, /* std::complex<double>, interleaved re/im */
    COSTA_INT32 = 4
} costa_dtype_t;

typedef struct costa_layout_s* costa_layout_t;
typedef struct costa_comm_s* costa_comm_t;

/* identical to costa::block_t (reference layout.hpp:14-19) */
typedef struct {
    void* data; /* first element of the block (host or device memory) */
    int ld;     /* leading dimension of the block */
    int row;    /* global block-row index */
    int col;    /* global block-column index */
} costa_block_t;

/* ---- tile descriptor: one "copy_and_transform" call in normalised form ----
 * The source tile has `nf` elements along its contiguous (fast) dimension and
 * `ns` along the strided one:  src element (f, s) lives at src + (s*lds + f)*sizeof(T).
 *   copy mode      : dst + (s*ldd + f)*sizeof(T)  = g(src(f, s))
 *   transpose mode : dst + (f*ldd + s)*sizeof(T)  = g(src(f, s))
 * g(x) = x (bit copy)                  scale kind COSTA_SCALE_BITCOPY (copy mode only)
 *      = 0                             COSTA_SCALE_ZERO   (alpha == beta == 0)
 *      = alpha*op(x)                   COSTA_SCALE_ALPHA  (beta == 0: C is not read)
 *      = beta*dst + alpha*op(x)        COSTA_SCALE_AXPBY
 * with op = conj when COSTA_TILE_CONJ is set.  Exactly the branches of
 * memory_utils.hpp:20-51 and 101-291.  `src`/`dst` are byte offsets added to the
 * launch's base pointers (absolute addresses when the base is NULL). */
#define COSTA_TILE_TRANSPOSE 0x1u
#define COSTA_TILE_CONJ 0x2u
#define COSTA_TILE_VEC_SRC 0x4u /* src tile columns may be read as 16-byte vectors: 16-byte aligned, or
                                  (4-byte elements, ops of at least one large sub-tile) dword aligned;
                                  the planner sets it for 16-byte alignment, the executor's work
                                  lists add the dword-aligned case */
#define COSTA_TILE_VEC_DST 0x8u /* dst tile rows/columns are 16-byte aligned */
#define COSTA_SCALE_SHIFT 4
#define COSTA_SCALE_MASK 0x30u
#define COSTA_SCALE_BITCOPY 0u
#define COSTA_SCALE_ZERO 1u
#define COSTA_SCALE_ALPHA 2u
#define COSTA_SCALE_AXPBY 3u
#define COSTA_SLOT_SHIFT 16 /* bits 16..31: index of the (alpha, beta) pair */

typedef struct {
    uint64_t src;
    uint64_t dst;
    int32_t nf;
    int32_t ns;
    int32_t lds;
    int32_t ldd;
    uint32_t flags;
    uint32_t order; /* locality hint: the executor may run ops in ascending `order` (ops are
                       independent, so any order gives the same result); the planner sets
                       the tile's rank in column-major order of its target coordinates, so
                       tiles sharing partially used cache lines run together.  0 = none. */
} costa_tile_op_t; /* 40 bytes */

/* ---- library ---- */
const char* costa_hip_last_error(void);
int costa_hip_version(void); /* major*10000 + minor*100 + patch */
int costa_hip_device_count(int* count); /* visible GPUs (COSTA_ERR_HIP without a GPU) */
/* the RCCL library the exchange runs on in this process (ncclGetVersion: major*10000 +
 * minor*100 + patch); which one the loader bound depends on what the process loaded first
 * (torch ships its own librccl under the same soname) */
int costa_hip_rccl_version(int* version);

/* ---- layouts (pointers may be host or device memory; never dereferenced
 *      until a transform runs) ---- */
int costa_hip_block_cyclic_layout(costa_dtype_t dtype, int m, int n, int block_m, int block_n,
                                  int i, int j, int sub_m, int sub_n, int p_m, int p_n,
                                  char rank_grid_ordering, int rsrc, int csrc, void* ptr, int lld,
                                  char data_ordering, int rank, costa_layout_t* out);
int costa_hip_custom_layout(costa_dtype_t dtype, int rowblocks, int colblocks, const int* rowsplit,
                            const int* colsplit, const int* owners, int nlocalblocks,
                            const costa_block_t* localblocks, char ordering, costa_layout_t* out);
void costa_hip_layout_destroy(costa_layout_t layout);
/* rank relabelling: owner(i, j) becomes reordering[owner(i, j)] (replaces any earlier one;
 * n = 0 restores the identity).  Replaces grid_layout<T>::reorder_ranks
 * (src/costa/grid2grid/grid_layout.hpp:32-34, grid2D.hpp:183-187, 219-221).  `reordering` must
 * be a permutation of 0..n-1 (COSTA_ERR_ARG otherwise) with n >= the layout's ranks.  A cell of
 * base owner o then belongs to rank reordering[o], so the process of rank r must hold the local
 * blocks of base rank o with reordering[o] == r (the inverse permutation at r).  The
 * permutations costa::optimal_reordering proposes (<costa/grid2grid/ranks_reordering.hpp>) swap
 * pairs of ranks, i.e. are their own inverse: then rank r holds the blocks of rank
 * reordering[r], as the reference's README puts it (README.md:343-362). */
int costa_hip_layout_reorder_ranks(costa_layout_t layout, const int* reordering, int n);
/* number of local blocks / the i-th block (global intervals, data pointer, ld) */
int costa_hip_layout_num_blocks(costa_layout_t layout);
int costa_hip_layout_block(costa_layout_t layout, int i, int* row_start, int* row_end,
                           int* col_start, int* col_end, void** data, int* ld);

/* ---- communicators: one process per GPU ----
 * costa_hip_comm_self: a single-rank communicator on `device` (no RCCL).
 * costa_hip_comm_create: rank `rank` of `nranks`; `id` is the 128-byte RCCL unique id made by
 * costa_hip_comm_unique_id on one rank and broadcast by the caller's control plane (MPI,
 * torch.distributed store, ...).  Collective over all ranks. */
int costa_hip_comm_self(int device, costa_comm_t* out);
int costa_hip_comm_unique_id(unsigned char id[128]);
int costa_hip_comm_create(const unsigned char id[128], int nranks, int rank, int device,
                          costa_comm_t* out);
int costa_hip_comm_rank(costa_comm_t comm);
int costa_hip_comm_size(costa_comm_t comm);
void costa_hip_comm_destroy(costa_comm_t comm);

/* ---- transforms: sub(C) = beta*sub(C) + alpha*op(sub(A)), op in {'N','T','C'} ----
 * alpha/beta point to ONE element of the layouts' dtype (complex: two reals).
 * Collective over `comm`; blocking (returns after C is complete). */
int costa_hip_transform(costa_layout_t A, costa_layout_t C, char trans, const void* alpha,
                        const void* beta, costa_comm_t comm);
/* several layout pairs in one exchange; trans/alpha/beta are arrays of n entries
 * (alpha/beta: n elements of the dtype). */
int costa_hip_transform_batch(int n, const costa_layout_t* A, const costa_layout_t* C,
                              const char* trans, const void* alpha, const void* beta,
                              costa_comm_t comm);

/* ---- stream-ordered variants (MI355X-native; no reference counterpart) ----
 * Enqueue the transform and return.  Layouts must be device-resident.  `stream` (a hipStream_t,
 * may be NULL) is joined at entry and made to wait for the result, so work queued on it after
 * this call sees sub(C) complete.  Transforms of one process run in call order.
 * costa_hip_synchronize waits for everything queued on the communicator's device. */
int costa_hip_transform_async(costa_layout_t A, costa_layout_t C, char trans, const void* alpha,
                              const void* beta, costa_comm_t comm, void* stream);
int costa_hip_transform_batch_async(int n, const costa_layout_t* A, const costa_layout_t* C,
                                    const char* trans, const void* alpha, const void* beta,
                                    costa_comm_t comm, void* stream);
int costa_hip_synchronize(costa_comm_t comm);

/* ---- direct tile entry points (device pointers) ---- */
int costa_hip_copy_and_transform(costa_dtype_t dtype, int n_rows, int n_cols, const void* src,
                                 int src_stride, int src_col_major, void* dst, int dst_stride,
                                 int dst_col_major, int transpose, int conjugate,
                                 const void* alpha, const void* beta);
/* runs `n` tile ops in ONE batched launch; `scalars` = n_slots (alpha, beta) pairs (host) */
int costa_hip_execute_tiles(costa_dtype_t dtype, const costa_tile_op_t* ops, int64_t n,
                            const void* src_base, void* dst_base, const void* scalars,
                            int n_slots, int device);

/* ---- plan inspection (host only, never touches a GPU) ----
 * Plans the transform for rank `rank` of `nranks` and copies the three descriptor
 * lists out.  Offsets of pack destinations / unpack sources are byte offsets into the
 * send / receive buffer; all other addresses are the layouts' own pointers.
 * Call once with NULL arrays to get the sizes in *info, then again with arrays of
 * at least those sizes. */
typedef struct {
    int64_t n_local;     /* local tile ops   (copy_local_blocks)           */
    int64_t n_pack;      /* pack tile ops    (copy_to_buffer)              */
    int64_t n_unpack;    /* unpack tile ops  (copy_from_buffer)            */
    int64_t send_elems;  /* elements in the send buffer                    */
    int64_t recv_elems;  /* elements in the receive buffer                 */
    int64_t local_elems; /* elements moved by local ops                    */
    int32_t n_ranks;     /* size of the counts/displacement arrays         */
    int32_t n_slots;     /* number of (alpha, beta) pairs                  */
} costa_plan_info_t;

int costa_hip_plan_export(int n, const costa_layout_t* A, const costa_layout_t* C,
                          const char* trans, const void* alpha, const void* beta, int rank,
                          int nranks, costa_plan_info_t* info, costa_tile_op_t* local_ops,
                          costa_tile_op_t* pack_ops, costa_tile_op_t* unpack_ops,
                          int64_t* send_counts, int64_t* send_displs, int64_t* recv_counts,
                          int64_t* recv_displs, void* scalars);

/* ---- measurement ----
 * With profiling on, every kernel launch and exchange is bracketed by HIP events on
 * the stream it runs on; the sums are read (and optionally reset) here. */
typedef struct {
    double pack_ms, local_ms, unpack_ms, exchange_ms, h2d_ms, d2h_ms;
    int64_t pack_launches, local_launches, unpack_launches;
    int64_t pack_bytes, local_bytes, unpack_bytes; /* algorithmic HBM bytes */
    int64_t transforms;
    int64_t plan_hits, plan_misses;
    int64_t host_groups; /* tile groups moved by the pipelined host staging */
    int64_t device_plans; /* plan-cache misses planned on the GPU (costa_hip_set_planner) */
    double plan_ms;       /* host wall time spent building plans (cache misses) */
    int64_t host_direct;  /* host-resident calls whose buffers were page-locked and in which some
                             tile groups moved by strided DMA between the caller's memory and
                             HBM (no host copies for those groups) */
    int64_t host_direct_groups; /* ... the tile groups that moved that way (PACK: a pack kernel
                                   from the DMA'd source rectangle; LOCAL / UNPACK: kernels
                                   writing the target rectangle's image, DMA'd back) */
    /* work items launched by the device-resident path, per kernel (r6): tile_kernel sub-tiles
       (the large, square, medium and 32 x 32 shapes), skew_kernel sub-tiles, cblock_kernel
       destination-block groups, tiny_kernel wavefront pieces */
    int64_t tile_items, skew_items, cblock_items, tiny_items;
    int64_t device_lists; /* work lists whose destination-block groups were built on the GPU
                             (costa_hip_set_list_builder) */
    int64_t fused_pieces; /* of tiny_items: wavefront pieces run as workgroups at the end of the
                             destination-block group launch (no tiny_kernel launch of their own) */
} costa_stats_t;
int costa_hip_set_profiling(int on);
int costa_hip_get_stats(costa_stats_t* out, int reset);
/* drop cached plans and device workspaces of this process */
int costa_hip_release_caches(void);

/* ---- host-resident layouts ----
 * How a transform whose layouts live in host memory reaches HBM (the reference's path starts
 * and ends in each rank's host buffers).  1 (default; env COSTA_HOST_STAGING): pipelined --
 * the tiles move in 64 MiB groups through pinned/device slot rings: host gather -> H2D ->
 * tile kernels -> D2H -> host scatter, both copy directions at once; with several ranks the
 * host gather writes the send package, the RCCL exchange follows, and the unpack kernels'
 * output comes back the same way.  When every host buffer of the call is page-locked
 * (hipHostMalloc, or registered by the caller with hipHostRegister) the pipeline skips the host
 * copies: each tile moves by strided DMA (hipMemcpy2DAsync) straight between the caller's memory
 * and the device slots, both directions at once.  0: mirror -- every byte range the layouts span is uploaded,
 * the kernels run on the mirror, the target ranges are copied back.  Mode 1 falls back to 0
 * for in-place layouts and target ranges shared by two batched jobs.  Results are identical. */
int costa_hip_set_host_staging(int mode);

/* Planner of plan-cache misses (the reference plans on the host at every call, utils.hpp:87-206,
 * communication_data.cpp:67-164).  1 (default): layout pairs of at least 4096 blocks are planned
 * on the GPU (100000 before the first GPU plan of the process, which loads the planner's kernels)
 * -- one thread per cell of the merged grid of the two layouts, a stable radix sort by
 * peer for the message order, scans for the package offsets; 0: always on the host; 2: on the GPU
 * wherever it applies.  The op lists are identical either way.  Layouts whose local blocks are
 * not exactly the rank's grid cells are planned on the host in every mode. */
int costa_hip_set_planner(int mode);
/* costa_hip_plan_export through the GPU planner of `device` (COSTA_ERR_ARG when it does not
 * apply to these layouts) */
int costa_hip_plan_export_device(int device, int n, const costa_layout_t* A, const costa_layout_t* C,
                                 const char* trans, const void* alpha, const void* beta, int rank,
                                 int nranks, costa_plan_info_t* info, costa_tile_op_t* local_ops,
                                 costa_tile_op_t* pack_ops, costa_tile_op_t* unpack_ops,
                                 int64_t* send_counts, int64_t* send_displs, int64_t* recv_counts,
                                 int64_t* recv_displs, void* scalars);

/* Builder of the executor's work lists on a plan-cache miss (after the planner): the
 * destination-block groups of the wavefront ops -- components of ops that tile a destination
 * range exactly, cut into column bands, in destination / XCD-slice order -- are 1 (default) built
 * on the GPU for lists of at least 16384 wavefront ops, 0 always on the host, 2 on the GPU wherever
 * they apply (env COSTA_LIST_BUILDER).  The lists are identical either way. */
int costa_hip_set_list_builder(int mode);
/* The executor's work lists of one tile-op list (diagnostics and tests; no kernel runs):
 * `kind` 0 local, 1 pack (destination = a dense package), 2 unpack; device < 0 builds them on the
 * host, device >= 0 with the destination-block groups on that GPU.  meta[12] receives n_large,
 * n_medium, n_skew, n_cblock, cblock_lds, cb_map, tiny_first, n_tiny, n_ordered, n_work, whether the
 * GPU built part of them, and the flags (bit 0 tr_shape, 1 sq, 2 full, 3 med_full, 4 med_sq,
 * 5 skew_wide).  `ordered` (cap_ordered ops) and `work` (cap_work entries) are filled when their
 * capacities suffice (NULL: sizes only). */
int costa_hip_work_export(int dtype, const costa_tile_op_t* ops, int64_t n_ops, int kind, int device,
                          costa_tile_op_t* ordered, int64_t cap_ordered, uint64_t* work,
                          int64_t cap_work, int64_t* meta);

#ifdef __cplusplus
}
#endif
#endif /* COSTA_HIP_H */
