// extern "C" boundary (include/costa_hip.h) and the C++ transform API
// (include/costa/transform.hpp).  No exception crosses the C boundary.
#include "engine.hpp"

#include <hip/hip_runtime.h>

#include <costa/transform.hpp>

#include <algorithm>
#include <cctype>
#include <complex>
#include <cstring>
#include <new>

struct costa_layout_s {
    costa::engine::elayout e;
    std::vector<int> base_owners;  // owners before a rank relabelling (empty: none applied)
};
struct costa_comm_s {
    costa::engine::comm* c = nullptr;
};

namespace {
thread_local std::string g_last_error;

template <typename F>
int guarded(F&& f) {
    try {
        f();
        return COSTA_OK;
    } catch (const costa::engine::error& e) {
        g_last_error = e.what();
        return e.code;
    } catch (const std::bad_alloc&) {
        g_last_error = "out of host memory";
        return COSTA_ERR_INTERNAL;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return COSTA_ERR_ARG;
    } catch (...) {
        g_last_error = "unknown error";
        return COSTA_ERR_INTERNAL;
    }
}

// Entry points that may switch the calling thread's HIP device (hipSetDevice to the
// communicator's or the call's device) put the caller's current device back on the way out:
// a process driving several GPUs keeps its own device selection across costa calls.
struct device_restore {
    int dev = -1;
    device_restore() {
        if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    }
    ~device_restore() {
        if (dev >= 0) (void)hipSetDevice(dev);
    }
};

template <typename F>
int gpu_guarded(F&& f) {
    device_restore keep;
    return guarded(std::forward<F>(f));
}

using costa::engine::dtype_size;
using costa::engine::elayout;
using costa::engine::job;
using costa::engine::scal;

template <typename F>
void with_type(costa_dtype_t t, F&& f) {
    switch (t) {
    case COSTA_FLOAT: f(float{}); return;
    case COSTA_DOUBLE: f(double{}); return;
    case COSTA_CFLOAT: f(std::complex<float>{}); return;
    case COSTA_CDOUBLE: f(std::complex<double>{}); return;
    case COSTA_INT32: f(int{}); return;
    }
    throw costa::engine::error(COSTA_ERR_ARG, "unknown dtype");
}

scal make_scal(costa_dtype_t t, const void* a, const void* b) {
    scal s;
    const size_t E = dtype_size(t);
    std::memcpy(s.alpha.data(), a, E);
    std::memcpy(s.beta.data(), b, E);
    return s;
}

void check_handles(int n, const costa_layout_t* A, const costa_layout_t* C) {
    if (n <= 0 || !A || !C) throw costa::engine::error(COSTA_ERR_ARG, "costa: empty batch");
    for (int i = 0; i < n; ++i)
        if (!A[i] || !C[i]) throw costa::engine::error(COSTA_ERR_ARG, "costa: null layout");
}

std::vector<job> make_jobs(int n, const costa_layout_t* A, const costa_layout_t* C,
                           const char* trans, const void* alpha, const void* beta) {
    check_handles(n, A, C);
    const costa_dtype_t t = A[0]->e.dtype;
    const size_t E = dtype_size(t);
    std::vector<job> jobs(static_cast<size_t>(n));
    for (int i = 0; i < n; ++i) {
        jobs[size_t(i)].A = &A[i]->e;
        jobs[size_t(i)].C = &C[i]->e;
        jobs[size_t(i)].trans = trans ? trans[i] : 'N';
        jobs[size_t(i)].s = make_scal(t, static_cast<const char*>(alpha) + size_t(i) * E,
                                      static_cast<const char*>(beta) + size_t(i) * E);
    }
    return jobs;
}
}  // namespace

namespace {
// one plan (from `make`) copied out as costa_hip_plan_export documents
template <typename F>
int export_plan(F make, int n, const costa_layout_t* A, const costa_layout_t* C, const char* trans,
                const void* alpha, const void* beta, int rank, int nranks, costa_plan_info_t* info,
                costa_tile_op_t* local_ops, costa_tile_op_t* pack_ops, costa_tile_op_t* unpack_ops,
                int64_t* send_counts, int64_t* send_displs, int64_t* recv_counts,
                int64_t* recv_displs, void* scalars) {
    return guarded([&] {
        if (!info || !alpha || !beta) throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        if (nranks < 1 || rank < 0 || rank >= nranks)
            throw costa::engine::error(COSTA_ERR_ARG, "bad rank/size");
        auto jobs = make_jobs(n, A, C, trans, alpha, beta);
        std::unique_ptr<costa::engine::plan> p = make(jobs);
        info->n_local = int64_t(p->local_ops.size());
        info->n_pack = int64_t(p->pack_ops.size());
        info->n_unpack = int64_t(p->unpack_ops.size());
        info->send_elems = p->send_elems;
        info->recv_elems = p->recv_elems;
        info->local_elems = p->local_elems;
        info->n_ranks = nranks;
        info->n_slots = int32_t(p->slots.size());
        auto cp = [](const auto& v, auto* dst) {
            if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(v[0]));
        };
        cp(p->local_ops, local_ops);
        cp(p->pack_ops, pack_ops);
        cp(p->unpack_ops, unpack_ops);
        cp(p->send_counts, send_counts);
        cp(p->send_displs, send_displs);
        cp(p->recv_counts, recv_counts);
        cp(p->recv_displs, recv_displs);
        if (scalars) {
            const size_t E = dtype_size(p->dtype);
            auto* out = static_cast<unsigned char*>(scalars);
            for (size_t t = 0; t < p->slots.size(); ++t) {
                std::memcpy(out + (2 * t) * E, p->slots[t].alpha.data(), E);
                std::memcpy(out + (2 * t + 1) * E, p->slots[t].beta.data(), E);
            }
        }
    });
}
}  // namespace

extern "C" {

const char* costa_hip_last_error(void) { return g_last_error.c_str(); }
int costa_hip_version(void) { return 100; }

int costa_hip_device_count(int* count) {
    return guarded([&] {
        if (!count) throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        *count = costa::engine::device_count();
    });
}

int costa_hip_rccl_version(int* version) {
    return guarded([&] {
        if (!version) throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        *version = costa::engine::rccl_version();
    });
}

int costa_hip_block_cyclic_layout(costa_dtype_t dtype, int m, int n, int block_m, int block_n,
                                  int i, int j, int sub_m, int sub_n, int p_m, int p_n,
                                  char rank_grid_ordering, int rsrc, int csrc, void* ptr, int lld,
                                  char data_ordering, int rank, costa_layout_t* out) {
    return guarded([&] {
        if (!out) throw costa::engine::error(COSTA_ERR_ARG, "null output handle");
        auto h = std::make_unique<costa_layout_s>();
        with_type(dtype, [&](auto z) {
            using T = decltype(z);
            auto L = costa::block_cyclic_layout<T>(m, n, block_m, block_n, i, j, sub_m, sub_n, p_m,
                                                   p_n, rank_grid_ordering, rsrc, csrc,
                                                   static_cast<T*>(ptr), lld, data_ordering, rank);
            h->e = costa::engine::erase(L);
            costa::engine::set_layout_hash(h->e);  // handles are immutable
        });
        *out = h.release();
    });
}

int costa_hip_custom_layout(costa_dtype_t dtype, int rowblocks, int colblocks, const int* rowsplit,
                            const int* colsplit, const int* owners, int nlocalblocks,
                            const costa_block_t* localblocks, char ordering, costa_layout_t* out) {
    static_assert(sizeof(costa_block_t) == sizeof(costa::block_t), "block_t layout");
    return guarded([&] {
        if (!out || !rowsplit || !colsplit || !owners || (nlocalblocks > 0 && !localblocks))
            throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        auto h = std::make_unique<costa_layout_s>();
        with_type(dtype, [&](auto z) {
            using T = decltype(z);
            auto L = costa::custom_layout<T>(rowblocks, colblocks, rowsplit, colsplit, owners,
                                             nlocalblocks,
                                             reinterpret_cast<const costa::block_t*>(localblocks),
                                             ordering);
            h->e = costa::engine::erase(L);
            costa::engine::set_layout_hash(h->e);  // handles are immutable
        });
        *out = h.release();
    });
}

void costa_hip_layout_destroy(costa_layout_t layout) { delete layout; }

int costa_hip_layout_reorder_ranks(costa_layout_t layout, const int* reordering, int n) {
    return guarded([&] {
        if (!layout || n < 0 || (n > 0 && !reordering))
            throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        auto& e = layout->e;
        if (layout->base_owners.empty()) layout->base_owners = e.owners;
        const std::vector<int>& base = layout->base_owners;
        int n_base = 0;
        for (int o : base) n_base = std::max(n_base, o + 1);
        // the reference replaces the relabelling (assigned_grid2D::reorder_ranks, grid2D.hpp:219-221)
        // and maps every owner through it (owner(), grid2D.hpp:183-187)
        if (n > 0 && n < n_base)
            throw costa::engine::error(COSTA_ERR_ARG, "costa: reordering shorter than the ranks");
        std::vector<char> seen(size_t(n), 0);
        for (int k = 0; k < n; ++k) {
            if (reordering[k] < 0 || reordering[k] >= n)
                throw costa::engine::error(COSTA_ERR_ARG, "costa: reordering out of range");
            if (seen[size_t(reordering[k])]++)
                throw costa::engine::error(COSTA_ERR_ARG, "costa: reordering is not a permutation");
        }
        std::vector<int> owners(base.size());
        for (size_t k = 0; k < base.size(); ++k) owners[k] = n > 0 ? reordering[base[k]] : base[k];
        e.owners = std::move(owners);
        e.n_ranks = std::max(e.n_ranks, n);
        costa::engine::set_layout_hash(e);  // a relabelled handle is a different layout
    });
}

int costa_hip_layout_num_blocks(costa_layout_t layout) {
    return layout ? int(layout->e.blocks.size()) : -1;
}

int costa_hip_layout_block(costa_layout_t layout, int i, int* row_start, int* row_end,
                           int* col_start, int* col_end, void** data, int* ld) {
    return guarded([&] {
        if (!layout || i < 0 || size_t(i) >= layout->e.blocks.size())
            throw costa::engine::error(COSTA_ERR_ARG, "block index out of range");
        const auto& b = layout->e.blocks[size_t(i)];
        if (row_start) *row_start = b.rows.start;
        if (row_end) *row_end = b.rows.end;
        if (col_start) *col_start = b.cols.start;
        if (col_end) *col_end = b.cols.end;
        if (data) *data = b.data;
        if (ld) *ld = b.ld;
    });
}

int costa_hip_comm_self(int device, costa_comm_t* out) {
    return gpu_guarded([&] {
        if (!out) throw costa::engine::error(COSTA_ERR_ARG, "null output handle");
        auto h = std::make_unique<costa_comm_s>();
        h->c = costa::engine::comm_self(device);
        *out = h.release();
    });
}

int costa_hip_comm_unique_id(unsigned char id[128]) {
    return guarded([&] { costa::engine::comm_unique_id(id); });
}

int costa_hip_comm_create(const unsigned char id[128], int nranks, int rank, int device,
                          costa_comm_t* out) {
    return gpu_guarded([&] {
        if (!out || !id) throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        auto h = std::make_unique<costa_comm_s>();
        h->c = costa::engine::comm_create(id, nranks, rank, device);
        *out = h.release();
    });
}

int costa_hip_comm_rank(costa_comm_t comm) { return comm ? costa::engine::comm_rank(comm->c) : -1; }
int costa_hip_comm_size(costa_comm_t comm) { return comm ? costa::engine::comm_size(comm->c) : -1; }
void costa_hip_comm_destroy(costa_comm_t comm) {
    if (!comm) return;
    costa::engine::comm_destroy(comm->c);
    delete comm;
}

int costa_hip_transform(costa_layout_t A, costa_layout_t C, char trans, const void* alpha,
                        const void* beta, costa_comm_t comm) {
    return costa_hip_transform_batch(1, &A, &C, &trans, alpha, beta, comm);
}

int costa_hip_transform_batch(int n, const costa_layout_t* A, const costa_layout_t* C,
                              const char* trans, const void* alpha, const void* beta,
                              costa_comm_t comm) {
    return gpu_guarded([&] {
        if (!comm || !alpha || !beta) throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        auto jobs = make_jobs(n, A, C, trans, alpha, beta);
        costa::engine::transform(jobs, comm->c);
    });
}

int costa_hip_transform_async(costa_layout_t A, costa_layout_t C, char trans, const void* alpha,
                              const void* beta, costa_comm_t comm, void* stream) {
    return costa_hip_transform_batch_async(1, &A, &C, &trans, alpha, beta, comm, stream);
}

int costa_hip_transform_batch_async(int n, const costa_layout_t* A, const costa_layout_t* C,
                                    const char* trans, const void* alpha, const void* beta,
                                    costa_comm_t comm, void* stream) {
    return gpu_guarded([&] {
        if (!comm || !alpha || !beta) throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        auto jobs = make_jobs(n, A, C, trans, alpha, beta);
        costa::engine::transform(jobs, comm->c, stream, true);
    });
}

int costa_hip_synchronize(costa_comm_t comm) {
    return gpu_guarded([&] {
        if (!comm) throw costa::engine::error(COSTA_ERR_ARG, "null communicator");
        costa::engine::synchronize(comm->c);
    });
}

int costa_hip_copy_and_transform(costa_dtype_t dtype, int n_rows, int n_cols, const void* src,
                                 int src_stride, int src_col_major, void* dst, int dst_stride,
                                 int dst_col_major, int transpose, int conjugate,
                                 const void* alpha, const void* beta) {
    return gpu_guarded([&] {
        if (!alpha || !beta) throw costa::engine::error(COSTA_ERR_ARG, "null scalar");
        costa::engine::copy_and_transform(dtype, n_rows, n_cols, src, src_stride, src_col_major != 0,
                                          dst, dst_stride, dst_col_major != 0, transpose != 0,
                                          conjugate != 0, alpha, beta);
    });
}

int costa_hip_execute_tiles(costa_dtype_t dtype, const costa_tile_op_t* ops, int64_t n,
                            const void* src_base, void* dst_base, const void* scalars,
                            int n_slots, int device) {
    return gpu_guarded([&] {
        if (n < 0 || (n > 0 && (!ops || !scalars)))
            throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        costa::engine::execute_tiles(dtype, ops, n, src_base, dst_base, scalars, n_slots, device);
    });
}

int costa_hip_plan_export(int n, const costa_layout_t* A, const costa_layout_t* C,
                          const char* trans, const void* alpha, const void* beta, int rank,
                          int nranks, costa_plan_info_t* info, costa_tile_op_t* local_ops,
                          costa_tile_op_t* pack_ops, costa_tile_op_t* unpack_ops,
                          int64_t* send_counts, int64_t* send_displs, int64_t* recv_counts,
                          int64_t* recv_displs, void* scalars) {
    return export_plan(
        [&](const std::vector<job>& jobs) { return costa::engine::make_plan(jobs, rank, nranks); },
        n, A, C, trans, alpha, beta, rank, nranks, info, local_ops, pack_ops, unpack_ops,
        send_counts, send_displs, recv_counts, recv_displs, scalars);
}

int costa_hip_plan_export_device(int device, int n, const costa_layout_t* A, const costa_layout_t* C,
                                 const char* trans, const void* alpha, const void* beta, int rank,
                                 int nranks, costa_plan_info_t* info, costa_tile_op_t* local_ops,
                                 costa_tile_op_t* pack_ops, costa_tile_op_t* unpack_ops,
                                 int64_t* send_counts, int64_t* send_displs, int64_t* recv_counts,
                                 int64_t* recv_displs, void* scalars) {
    device_restore keep;
    return export_plan(
        [&](const std::vector<job>& jobs) {
            auto p = costa::engine::make_plan_device(jobs, rank, nranks, 0, device, nullptr);
            if (!p)
                throw costa::engine::error(COSTA_ERR_ARG,
                                           "costa: the device planner does not apply to these "
                                           "layouts (local blocks are not exactly the rank's grid "
                                           "cells)");
            return p;
        },
        n, A, C, trans, alpha, beta, rank, nranks, info, local_ops, pack_ops, unpack_ops,
        send_counts, send_displs, recv_counts, recv_displs, scalars);
}

int costa_hip_set_planner(int mode) {
    return guarded([&] {
        if (mode < 0 || mode > 2) throw costa::engine::error(COSTA_ERR_ARG, "mode must be 0, 1 or 2");
        costa::engine::set_planner_mode(mode);
    });
}

int costa_hip_set_list_builder(int mode) {
    return guarded([&] {
        if (mode < 0 || mode > 2) throw costa::engine::error(COSTA_ERR_ARG, "mode must be 0, 1 or 2");
        costa::engine::set_list_builder_mode(mode);
    });
}

int costa_hip_work_export(int dtype, const costa_tile_op_t* ops, int64_t n_ops, int kind, int device,
                          costa_tile_op_t* ordered, int64_t cap_ordered, uint64_t* work,
                          int64_t cap_work, int64_t* meta) {
    auto body = [&] {
        if (!meta || (n_ops > 0 && !ops) || n_ops < 0) throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        if (dtype < COSTA_FLOAT || dtype > COSTA_INT32) throw costa::engine::error(COSTA_ERR_ARG, "bad dtype");
        if (kind < 0 || kind > 2) throw costa::engine::error(COSTA_ERR_ARG, "kind must be 0, 1 or 2");
        std::vector<costa_tile_op_t> in(ops, ops + n_ops), o;
        std::vector<uint64_t> w;
        costa::engine::work_split ws;
        const bool on_gpu = costa::engine::work_export(
            costa_dtype_t(dtype), in, costa::engine::list_kind(kind), device, o, w, ws);
        const int64_t m[12] = {ws.n_large, ws.n_medium, ws.n_skew, ws.n_cblock, ws.cblock_lds, ws.cb_map,
                               ws.tiny_first, ws.n_tiny, int64_t(o.size()), int64_t(w.size()), on_gpu,
                               int64_t(ws.tr_shape) | int64_t(ws.sq) << 1 | int64_t(ws.full) << 2 |
                                   int64_t(ws.med_full) << 3 | int64_t(ws.med_sq) << 4 |
                                   int64_t(ws.skew_wide) << 5};
        std::memcpy(meta, m, sizeof(m));
        if (ordered && cap_ordered >= int64_t(o.size()) && !o.empty())
            std::memcpy(ordered, o.data(), o.size() * sizeof(o[0]));
        if (work && cap_work >= int64_t(w.size()) && !w.empty()) std::memcpy(work, w.data(), w.size() * sizeof(w[0]));
    };
    return device >= 0 ? gpu_guarded(body) : guarded(body);  // (the host builder touches no GPU)
}

int costa_hip_set_profiling(int on) {
    costa::engine::set_profiling(on != 0);
    return COSTA_OK;
}

int costa_hip_get_stats(costa_stats_t* out, int reset) {
    return guarded([&] {
        if (!out) throw costa::engine::error(COSTA_ERR_ARG, "null argument");
        costa::engine::resolve_pending();  // timings of asynchronous transforms
        *out = costa::engine::stats();
        if (reset) costa::engine::stats() = costa_stats_t{};
    });
}

int costa_hip_set_host_staging(int mode) {
    return guarded([&] {
        if (mode != 0 && mode != 1) throw costa::engine::error(COSTA_ERR_ARG, "mode must be 0 or 1");
        costa::engine::set_host_staging_mode(mode);
    });
}

int costa_hip_release_caches(void) {
    return gpu_guarded([&] { costa::engine::release_caches(); });
}

}  // extern "C"

// ---------------------------------------------------------------- C++ API
namespace costa {
namespace {
void raise(int rc) {
    if (rc != COSTA_OK) throw hip_error(rc, g_last_error);
}
template <typename T>
engine::scal scal_of(T a, T b) {
    engine::scal s;
    std::memcpy(s.alpha.data(), &a, sizeof(T));
    std::memcpy(s.beta.data(), &b, sizeof(T));
    return s;
}
template <typename T>
void run(std::vector<layout_ref<T>>& from, std::vector<layout_ref<T>>& to, const char* trans,
         const T* alpha, const T* beta, costa_comm_t comm) {
    raise(gpu_guarded([&] {
        if (from.size() != to.size())
            throw engine::error(COSTA_ERR_ARG, "costa::transform: from/to sizes differ");
        if (!comm) throw engine::error(COSTA_ERR_ARG, "costa::transform: null communicator");
        std::vector<engine::elayout> es;
        es.reserve(2 * from.size());
        std::vector<engine::job> jobs(from.size());
        for (size_t i = 0; i < from.size(); ++i) {
            es.push_back(engine::erase(from[i].get()));
            jobs[i].A = &es.back();
            es.push_back(engine::erase(to[i].get()));
            jobs[i].C = &es.back();
            jobs[i].trans = trans ? trans[i] : 'N';
            jobs[i].s = alpha ? scal_of(alpha[i], beta[i]) : scal_of(T{1}, T{0});
        }
        engine::transform(jobs, comm->c);
    }));
}
}  // namespace

template <typename T>
void transform(grid_layout<T>& A, grid_layout<T>& C, costa_comm_t comm) {
    std::vector<layout_ref<T>> f{A}, t{C};
    run<T>(f, t, nullptr, nullptr, nullptr, comm);
}

template <typename T>
void transform(grid_layout<T>& A, grid_layout<T>& C, char trans, T alpha, T beta,
               costa_comm_t comm) {
    std::vector<layout_ref<T>> f{A}, t{C};
    run<T>(f, t, &trans, &alpha, &beta, comm);
}

template <typename T>
void transform(std::vector<layout_ref<T>>& from, std::vector<layout_ref<T>>& to,
               costa_comm_t comm) {
    run<T>(from, to, nullptr, nullptr, nullptr, comm);
}

template <typename T>
void transform(std::vector<layout_ref<T>>& from, std::vector<layout_ref<T>>& to, const char* trans,
               const T* alpha, const T* beta, costa_comm_t comm) {
    run<T>(from, to, trans, alpha, beta, comm);
}

#define COSTA_INSTANTIATE_TRANSFORM(T)                                                          \
    template void transform<T>(grid_layout<T>&, grid_layout<T>&, costa_comm_t);                 \
    template void transform<T>(grid_layout<T>&, grid_layout<T>&, char, T, T, costa_comm_t);     \
    template void transform<T>(std::vector<layout_ref<T>>&, std::vector<layout_ref<T>>&,        \
                               costa_comm_t);                                                   \
    template void transform<T>(std::vector<layout_ref<T>>&, std::vector<layout_ref<T>>&,        \
                               const char*, const T*, const T*, costa_comm_t);

COSTA_INSTANTIATE_TRANSFORM(float)
COSTA_INSTANTIATE_TRANSFORM(double)
COSTA_INSTANTIATE_TRANSFORM(std::complex<float>)
COSTA_INSTANTIATE_TRANSFORM(std::complex<double>)
COSTA_INSTANTIATE_TRANSFORM(int)

}  // namespace costa
