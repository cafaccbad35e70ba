// Internal engine interface: type-erased layouts, the tile planner and the executor.
#pragma once

#include <costa/layout.hpp>
#include <costa_hip.h>

#include <array>
#include <cstdint>
#include <functional>
#include <memory>
#include <string>
#include <vector>

namespace costa {
namespace engine {

size_t dtype_size(costa_dtype_t t);
bool dtype_is_complex(costa_dtype_t t);

// One local block, element-type erased.  Intervals are in the layout's own (untransposed)
// global coordinates; `data` points at its first element.
struct eblock {
    interval rows, cols;
    char* data = nullptr;
    int ld = 0;
};

// A grid_layout<T> with the element type erased (owners row-major, like the reference's
// ranks[i][j]).  Plans are built from these.
struct elayout {
    costa_dtype_t dtype = COSTA_DOUBLE;
    std::vector<int> rows_split, cols_split;
    std::vector<int> owners;
    int n_ranks = 1;
    char ordering = 'C';
    std::vector<eblock> blocks;
    uint64_t hash = 0;   // content hash (plan-cache key); 0 = not computed yet
    uint64_t hash2 = 0;  // a second, independently seeded content hash (verified on a cache hit)

    int nbr() const { return int(rows_split.size()) - 1; }
    int nbc() const { return int(cols_split.size()) - 1; }
};

template <typename T>
costa_dtype_t dtype_of();

template <typename T>
elayout erase(const grid_layout<T>& L);

// content hash of a layout (splits, owners, ordering, every block's intervals/pointer/ld)
uint64_t layout_hash(const elayout& L);
// both content hashes (h1 == layout_hash(L)), stored in L.hash / L.hash2 by set_layout_hash
void layout_hashes(const elayout& L, uint64_t& h1, uint64_t& h2);
void set_layout_hash(elayout& L);

// scalars (alpha, beta) of one layout pair, stored as raw bytes of the dtype
struct scal {
    std::array<unsigned char, 16> alpha{};
    std::array<unsigned char, 16> beta{};
};

// one (A -> C) pair of a transform
struct job {
    const elayout* A = nullptr;
    const elayout* C = nullptr;
    char trans = 'N';
    scal s;
};

// The three tile-op lists of one rank plus the exchange geometry.  Addresses of pack
// destinations and unpack sources are byte offsets into the send / receive buffers.
struct plan {
    costa_dtype_t dtype = COSTA_DOUBLE;
    int rank = 0, n_ranks = 1;
    std::vector<costa_tile_op_t> local_ops, pack_ops, unpack_ops;
    std::vector<int64_t> send_counts, send_displs, recv_counts, recv_displs;  // elements
    int64_t send_elems = 0, recv_elems = 0, local_elems = 0;
    std::vector<scal> slots;
    // algorithmic HBM bytes of each list (read + write (+ read of C when beta != 0))
    int64_t local_bytes = 0, pack_bytes = 0, unpack_bytes = 0;
};

// per-job transform parameters, validated as the reference's transform does (plan.cpp)
struct job_params {
    bool transpose, conj, a_cm, c_cm;
    uint32_t kind_copy, kind_tr;  // scale kind of ops that copy / transpose
};
std::vector<job_params> check_jobs(const std::vector<job>& jobs, int n_ranks, costa_dtype_t& dtype);

// Build the plan of `rank` (of `n_ranks`) for a batch of jobs (host only).  `loopback` (test
// mode, see loopback_exchange()): 1 = the rank's own tiles all go through pack -> exchange with
// itself -> unpack instead of the local list; 2 = half of them (by a parity of their target
// coordinates, the same on both sides), the rest stays local.
std::unique_ptr<plan> make_plan(const std::vector<job>& jobs, int rank, int n_ranks,
                                int loopback = 0);

// The same plan built on the GPU (device_plan.hip, on `stream` of `device`): identical op lists,
// order and exchange geometry.  nullptr when it does not apply (local blocks that are not exactly
// the rank's grid cells, grids not starting at the same index, more than 2^32 merged cells).
std::unique_ptr<plan> make_plan_device(const std::vector<job>& jobs, int rank, int n_ranks,
                                       int loopback, int device, void* stream);
// planner of plan-cache misses (costa_hip_set_planner, COSTA_PLANNER): 0 host, 1 the GPU for
// layout pairs of at least 4096 blocks, 100000 before the first GPU plan of the process (default),
// 2 the GPU wherever it applies
int planner_mode();
void set_planner_mode(int mode);

// COSTA_LOOPBACK=1 or 2 (test only): a one-rank communicator gets a one-rank RCCL communicator
// and its transforms route tiles through PACK -> ncclSend/ncclRecv to itself -> UNPACK (all of
// them, or half with the rest on the concurrent LOCAL path), so the exchange machinery runs on
// a single GPU (two ranks cannot share one GPU under RCCL).  0 = off.
int loopback_exchange();

// A tuning override `name` from the environment, or nullptr.  Tuning overrides (work-list orders,
// wavefront budgets, shape choices, host-staging slots and threads) are read only when
// COSTA_TUNING=1: a user's environment cannot select shapes and orders that the GPU tests never
// run.  Behaviour switches (COSTA_LOOPBACK, COSTA_MAX_MSG_BYTES, COSTA_EXCHANGE_ROUNDS,
// COSTA_PLANNER, COSTA_HOST_STAGING) and the trace switches are read as documented.
const char* tuning_env(const char* name);

// largest single ncclSend/ncclRecv of the exchange (COSTA_MAX_MSG_BYTES, default 256 MiB)
size_t max_message_bytes();

// parts a peer's package (of at least 16 MiB) is exchanged in, each its own RCCL group, so that
// pack, exchange and unpack overlap (COSTA_EXCHANGE_ROUNDS, default 4; every rank must agree)
int exchange_rounds();

// normalise one copy_and_transform call (memory_utils.hpp:339-412) into a tile op
costa_tile_op_t make_tile_op(int n_rows, int n_cols, uint64_t src, int src_stride, bool src_cm,
                             uint64_t dst, int dst_stride, bool dst_cm, bool transpose, bool conj,
                             uint32_t scale_kind, uint32_t slot, size_t elem);

// scale kind of (alpha, beta) for `dtype` with the reference's branch rules
uint32_t scale_kind(costa_dtype_t dtype, const scal& s, bool copy_mode, bool conj);

// ---- executor (engine.cpp / tile_kernels.hip) ----
int device_count();
int rccl_version();  // ncclGetVersion of the RCCL this process loaded
struct comm;
struct comm* comm_self(int device);
struct comm* comm_create(const unsigned char* id, int nranks, int rank, int device);
void comm_unique_id(unsigned char* out);
int comm_rank(const struct comm* c);
int comm_size(const struct comm* c);
void comm_destroy(struct comm* c);

// blocking (default) or stream-ordered (async: device-resident layouts only; `user_stream`, a
// hipStream_t or null, is joined at entry and waits for the result)
void transform(const std::vector<job>& jobs, struct comm* c, void* user_stream = nullptr,
               bool async = false);
void synchronize(struct comm* c);  // wait for every queued transform of c's device
void resolve_pending();            // fold finished timing brackets into the statistics

void copy_and_transform(costa_dtype_t dtype, int n_rows, int n_cols, const void* src,
                        int src_stride, bool src_cm, void* dst, int dst_stride, bool dst_cm,
                        bool trans, bool conj, const void* alpha, const void* beta);

void execute_tiles(costa_dtype_t dtype, const costa_tile_op_t* ops, int64_t n,
                   const void* src_base, void* dst_base, const void* scalars, int n_slots,
                   int device);

// kernel launcher (tile_kernels.hip); `work` and `ops` are device arrays
// ops small enough for one wavefront each (tiny path): copy mode up to kTinyCopyBytes of
// data, transpose mode up to kTinyLdsBytes of staged tile (row pitch nf | 1); the defaults
// are smaller (tiny_copy_budget: one pass of the wavefront; kTinyLdsDefault staged)
constexpr int kTinyCopyBytes = 16384;
constexpr int kTinyLdsBytes = 8192;
// r11, cfg 5 'T' with the XCD remap and 32 bytes per lane per pass: 3.80 TB/s at 4 KiB
// against 3.0 at 8 KiB (profiles/r11/tiny_variants*.log)
constexpr int kTinyLdsDefault = 4096;
// staged bytes of one transposing wavefront op (kTinyLdsDefault);
// the launch gives each wavefront that much LDS
int64_t tiny_lds_budget();
// bytes a lane of the wavefront copy path moves per pass (tile_kernels.hip tiny_copy_bytes)
// (64 for every type since r11: 4-byte types at 128 gave cfg 5 'N' 3.77 against 4.15 TB/s once
// the XCD remap was on, profiles/r11/c5_budget.log; fewer VGPRs, more resident wavefronts)
constexpr int tiny_copy_lane_bytes(size_t) { return 64; }
// bytes of one copy-mode wavefront op / of one transposing wavefront op's staged tile (the
// budgets the host split cuts to)
int64_t tiny_copy_budget(int64_t elem_size, bool local_list = true);
// a large op that is not 16-byte aligned on both sides takes the wavefront path up to this many
// large sub-tiles of data (engine.cpp wave_knobs::policy)
constexpr int64_t kUnalignedWaveCap = 4;
constexpr int tiny_lds_bytes = kTinyLdsBytes;

struct launch_args {
    const costa_tile_op_t* ops;  // device, in build_work order: [sub-tiled ops | tiny ops]
    const uint64_t* work;   // per sub-tile: (op index << 32) | sub-tile index
    int64_t n_large;        // work items using the large sub-tile shape
    int64_t n_medium;       // then work[n_large, n_large + n_medium): the medium shape
    int64_t n_skew = 0;     // then n_skew items of the skew shape (unaligned destinations)
    int64_t n_cblock = 0;   // then n_cblock destination-block groups: index of the group's header op
    int64_t cblock_lds = 0; // LDS image of the largest group (elements)
    int cb_map = 0;         // cblock_map of the groups
    int64_t tiny_first;     // ops[tiny_first, tiny_first + n_tiny) run one per wavefront
    int64_t n_tiny;
    const char* src_base;
    char* dst_base;
    const void* scalars;    // device: n_slots x (alpha, beta) of the dtype
    bool any_transpose;     // false: copy-mode ops only, launch without the LDS tile
    bool any_axpby;         // false: no op reads its destination (beta == 0 everywhere)
    bool tr_shape;          // the work items are sub-tiles of the transposing lists' shape
    bool sq;                // ... of its square variant (work_split::sq)
    bool full;              // work_split::full
    bool med_full;          // work_split::med_full
    bool med_sq;            // work_split::med_sq
    bool skew_wide = false; // work_split::skew_wide
};
bool any_transpose(const std::vector<costa_tile_op_t>& ops);
bool any_axpby(const std::vector<costa_tile_op_t>& ops);
void launch_tiles(costa_dtype_t dtype, const launch_args& a, void* stream /* hipStream_t */);
// the wavefront pieces of a list with destination-block groups run as workgroups after the groups
// in the group kernel's launch (its tail) instead of a tiny_kernel launch (COSTA_FUSE_PIECES)
bool pieces_in_group_launch(int64_t n_cblock, int64_t n_tiny);
// destination columns taller than this are walked in panels of this many bytes of rows (engine.cpp
// build_work)
constexpr int64_t kPanelBytes = int64_t(128) << 10;
// destination-block groups (tile_kernels.hip cblock_kernel): threads per workgroup and 16-byte
// destination vectors per thread; a group holds at most kCblockThreads * kCblockChunks vectors
constexpr int kCblockThreads = 256;
constexpr int kCblockChunks = 4;
inline int64_t cblock_max_elems(int64_t E) { return int64_t(kCblockThreads) * kCblockChunks * (16 / E); }
// work-list position of workgroup b of a launch of nb destination-block groups of a transposing
// list (tile_kernels.hip cblock_kernel): the hardware deals workgroups round-robin over the 8
// XCDs; chunks of kCblockXcdChunk consecutive groups go to one XCD, the 8 XCDs on 8 adjacent
// chunks; the last partial round of chunks keeps the plain order.  A permutation of [0, nb)
// (tools/work_check.cpp xcd).  (constexpr: host and device.)
// r6: 16 (traffic of cfg 5 'T' 1.134x -> 1.050x of its algorithmic bytes; chunks of 4 / 8 / 12 /
// 16 in-run 0.600 / 0.602 / 0.605 / 0.605 ms, rocprofv3 590.7 / 591.4 / 589.5 / 595.5 us;
// profiles/r6m/, r6n/)
constexpr int64_t kCblockXcdChunk = 16;
constexpr int64_t cblock_xcd_order(int64_t b, int64_t nb, int64_t ch = kCblockXcdChunk) {
    return b / (8 * ch) * (8 * ch) + 8 * ch <= nb ? b / (8 * ch) * (8 * ch) + (b % 8) * ch + (b / 8) % ch : b;
}
// work-list position of workgroup b of nb when XCD x (= b mod 8) walks the x-th of 8 contiguous
// slices of the list, slice x holding nb / 8 items (one more for the first nb mod 8 slices).  A
// permutation of [0, nb); tiny_kernel's remap and the destination-block groups' XCD column bands
// (engine.cpp cblock_groups).  (constexpr: host and device.)
constexpr int64_t xcd_slice_order(int64_t b, int64_t nb) {
    return (b % 8) < nb % 8 ? (b % 8) * (nb / 8 + 1) + b / 8
                            : (nb % 8) * (nb / 8 + 1) + ((b % 8) - nb % 8) * (nb / 8) + b / 8;
}
// how a launch of destination-block groups maps workgroups onto the list (work_split::cb_map)
enum cblock_map { cb_round_robin = 0, cb_xcd_chunks = 1, cb_xcd_bands = 2 };
// sub-tile shapes (elements along the source's fast dim, along its slow dim) of a copy-only list
// or of a list with transposing ops: the large shape, the medium one (bf_m = bs_m = 0: none) and
// the large shape's square variant for lists whose large ops all fit it (bf_q = bs_q = 0: none),
// and the 32 x 32 shape the medium class takes when its ops all fit it (bf_s x bs_s)
struct shape_dims {
    int bf = 0, bs = 0, bf_m = 0, bs_m = 0, bf_q = 0, bs_q = 0, bf_s = 0, bs_s = 0;
    int cf = 0, cs = 0;  // the large class's dimensions (classification, merging): bf x bs for
                         // transposing lists, the r4 copy sub-tile for copy-only lists
    int bf_k = 0, bs_k = 0;  // the skew shape (transposes into unaligned destinations; 0: none)
    int bf_kw = 0, bs_kw = 0;  // its wide variant (sources off the 16-byte grid too; 4-byte types)
};
void tile_shapes(costa_dtype_t dtype, bool transposing_list, shape_dims* out);
// Execution order of an op list: `ordered` = [sub-tiled ops | tiny ops] (tiny ops sorted by the
// planner's locality hint, so wavefronts running at the same time share partially used cache
// lines),
// `work` = [large-shape sub-tiles | small-shape sub-tiles], indices into `ordered`.
struct work_split {
    int64_t n_large = 0, n_medium = 0, tiny_first = 0, n_tiny = 0;
    int64_t n_skew = 0;     // skew-shape work items, after the medium ones
    int64_t n_cblock = 0;   // destination-block groups, after the skew items (cblock_groups)
    int64_t cblock_lds = 0; // elements of the largest group's LDS image
    int cb_map = 0;         // cblock_map: how the groups' launch maps workgroups onto them
    bool tr_shape = false;  // sub-tiles cut with tile_shapes(dtype, true, ...)
    bool sq = false;        // ... the large ops with its square variant (bf_q x bs_q)
    bool full = false;      // every large op of a transposing list is aligned and a whole number
                            // of large sub-tiles (the launch may then take fewer threads)
    bool med_full = false;  // the same for the medium ops and the medium sub-tile
    bool med_sq = false;    // the medium class runs on 32 x 32 sub-tiles (bf_s x bs_s)
    bool skew_wide = false; // the skew items are sub-tiles of its wide variant (bf_kw x bs_kw)
    int64_t n_items() const { return n_large + n_medium + n_skew + n_cblock + n_tiny; }
};
// list_pack: the ops write the dense send package (their destinations are contiguous whatever
// their order), which changes the wavefront ops' order (wave_knobs::sort); local lists (both
// sides user matrices) cut copy ops finer than pack / unpack lists (tiny_copy_budget)
enum list_kind { list_local, list_pack, list_unpack };
// The part of a work list that build_work left on the GPU: the destination-block groups built by
// device_lists.hip.  `ordered` entries [at_ordered, at_ordered + n_ordered) and `work` entries
// [at_work, at_work + n_work) are d_ordered / d_work; the host vectors hold all the others, without
// a gap.  A caller that passes one (device, stream set) lets build_work build the groups there
// (list_builder_mode; `force`: wherever it applies).
struct device_section {
    int device = -1;
    void* stream = nullptr;  // hipStream_t
    bool force = false;
    std::shared_ptr<void> mem;  // owns d_ordered and d_work
    costa_tile_op_t* d_ordered = nullptr;
    uint64_t* d_work = nullptr;
    size_t at_ordered = 0, n_ordered = 0, at_work = 0, n_work = 0;
};
work_split build_work(costa_dtype_t dtype, const std::vector<costa_tile_op_t>& ops,
                      std::vector<costa_tile_op_t>& ordered, std::vector<uint64_t>& work,
                      list_kind kind = list_local, device_section* dev = nullptr);
// builder of the destination-block groups on a plan-cache miss (costa_hip_set_list_builder,
// COSTA_LIST_BUILDER): 0 the host, 1 the GPU for lists of at least kDeviceGroupsMin wavefront ops
// (default), 2 the GPU wherever it applies
constexpr size_t kDeviceGroupsMin = 16384;
int list_builder_mode();
void set_list_builder_mode(int mode);
// engine.cpp cblock_groups on the GPU (device_lists.hip): the same groups in the same order, the
// same bytes.  `wave`: the wavefront ops as indices into `ops`, in list order; base_at: the size of
// `ordered` so far (header indices count from there).  Fills sec's device part and `taken` (per
// wavefront op: it joined a group); -> the number of groups, or -1 when the GPU declines (keys
// wider than 64 bits) and the host builder must run.
int64_t cblock_groups_device(int64_t E, int64_t budget, uint32_t vec_bits, int bands_env,
                             const std::vector<costa_tile_op_t>& ops, const std::vector<uint32_t>& wave,
                             size_t base_at, device_section& sec, std::vector<char>& taken,
                             int64_t& lds, int& map);
// one list's work lists, built on the host (device < 0) or with the groups on GPU `device`, copied
// out whole (costa_hip_work_export); -> whether the GPU built part of them
bool work_export(costa_dtype_t dtype, const std::vector<costa_tile_op_t>& ops, list_kind kind,
                 int device, std::vector<costa_tile_op_t>& ordered, std::vector<uint64_t>& work,
                 work_split& w);
// launch arguments of one ordered op list
launch_args make_launch(const work_split& w, const void* d_ordered, const void* d_work,
                        const char* src_base, char* dst_base, const void* d_scalars, bool transpose,
                        bool axpby);

// ---- host-resident pipeline (host_pipe.cpp) ----
// Transforms whose layouts all live in host memory: pack, local and unpack ops in groups of
// dense packages moving through a pinned/device slot ring (H2D, kernels, the exchange and D2H
// overlap).
struct host_pipeline;
// false when a pack op's column exceeds a pipeline slot (the mirror scheme is used then)
bool host_pipeline_accepts(costa_dtype_t dtype, const std::vector<costa_tile_op_t>& pack_ops);
// pack_round / unpack_round: each op's exchange round (exchange_round_of_ops) of `rounds`
std::shared_ptr<host_pipeline> make_host_pipeline(costa_dtype_t dtype,
                                                  const std::vector<costa_tile_op_t>& pack_ops,
                                                  const std::vector<costa_tile_op_t>& local_ops,
                                                  const std::vector<costa_tile_op_t>& unpack_ops,
                                                  const std::vector<int>& pack_round,
                                                  const std::vector<int>& unpack_round, int rounds);
size_t host_pipeline_groups(const host_pipeline& hp);
// Blocking: returns when every target byte is back in host memory.  Tile kernels run on
// `compute_stream`; `exchange(stream, r)` (empty without one) is called once per round r, with
// `exchange_stream`, when round r's part of the send package is in `send_buf`; the unpack
// kernels of round r read `recv_buf` after it.
void run_host_pipeline(host_pipeline& hp, int device, void* compute_stream, void* exchange_stream,
                       char* send_buf, char* recv_buf,
                       const std::function<void(void*, int)>& exchange, const void* d_scalars);
// the exchange round of every pack op (by its first element) and unpack op (by its last)
void exchange_round_of_ops(const struct plan& p, int rounds, std::vector<int>& pack_round,
                           std::vector<int>& unpack_round);
void release_host_rings();
// host staging of host-resident layouts: 0 = mirror (every spanned range up, kernels, target
// ranges down), 1 = pipelined (default; falls back to the mirror where it does not apply)
int host_staging_mode();
void set_host_staging_mode(int mode);

// errors
struct error : std::runtime_error {
    int code;
    error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

// statistics
costa_stats_t& stats();
bool profiling();
void set_profiling(bool on);
void release_caches();

}  // namespace engine
}  // namespace costa
