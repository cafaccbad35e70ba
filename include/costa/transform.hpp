// costa-mi355x — public C++ transform API (drop-in for COSTA's
// <costa/grid2grid/transform.hpp> and <costa/grid2grid/transformer.hpp>).
//
//   transform(A, C, comm)                        reference transform.hpp:13-16
//   transform(A, C, trans, alpha, beta, comm)    reference transform.hpp:22-27
//   transform(vector<layout_ref>..., comm)       reference transform.hpp:32-35
//   transform(vector<layout_ref>..., trans*, alpha*, beta*, comm)   transform.hpp:38-43
//   transformer<T>                               reference transformer.hpp:8-62
//
// The communicator is a costa_comm_t (one rank per GPU, data exchanged over RCCL).  With
// MPI available, <costa/mpi.hpp> adds the reference's exact MPI_Comm signatures on top.
#pragma once

#include <costa/grid2grid/comm_volume.hpp>
#include <costa/layout.hpp>
#include <costa_hip.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace costa {

// thrown by the C++ API when the C ABI reports an error
struct hip_error : std::runtime_error {
    int code;
    hip_error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

template <typename T>
void transform(grid_layout<T>& initial_layout, grid_layout<T>& final_layout, costa_comm_t comm);

template <typename T>
void transform(grid_layout<T>& initial_layout, grid_layout<T>& final_layout, char trans,
               T alpha, T beta, costa_comm_t comm);

template <typename T>
void transform(std::vector<layout_ref<T>>& initial_layouts,
               std::vector<layout_ref<T>>& final_layouts, costa_comm_t comm);

template <typename T>
void transform(std::vector<layout_ref<T>>& initial_layouts,
               std::vector<layout_ref<T>>& final_layouts, const char* trans, const T* alpha,
               const T* beta, costa_comm_t comm);

// Elements each rank pair exchanges when g_init is transformed into g_final with op `trans`
// (reference transform.hpp:44-48 / transform.cpp:9-44): every block of g_init (transposed view
// for 'T' / 'C') is intersected with the blocks of g_final; edge {a, b} (a <= b) adds the area
// owned by a in g_init and by b in g_final, relabelled owners included.  Host-only.
comm_volume communication_volume(assigned_grid2D& g_init, assigned_grid2D& g_final,
                                 char trans = 'N');

// batches several layout pairs into one exchange (reference transformer.hpp:8-62)
template <typename T>
struct transformer {
    std::vector<layout_ref<T>> from;
    std::vector<layout_ref<T>> to;
    std::vector<T> alpha;
    std::vector<T> beta;
    std::vector<char> transpose;
    costa_comm_t comm = nullptr;

    transformer() = default;
    explicit transformer(costa_comm_t c) : comm(c) {}

    void schedule(grid_layout<T>& f, grid_layout<T>& t) {
        from.push_back(f);
        to.push_back(t);
    }
    void schedule(grid_layout<T>& f, grid_layout<T>& t, char trans, T a, T b) {
        alpha.push_back(a);
        beta.push_back(b);
        transpose.push_back(trans);
        schedule(f, t);
    }
#ifdef MPI_VERSION
    // reference constructor: transformer(MPI_Comm) (transformer.hpp:24-27)
    explicit transformer(MPI_Comm c);
#endif

    void transform() {
        if (alpha.size() != beta.size() || alpha.size() != transpose.size())
            throw std::runtime_error("costa::transformer: inconsistent scheduling");
        if (!alpha.empty() && alpha.size() != from.size())
            throw std::runtime_error(
                "costa::transformer: mix of scaled and unscaled schedule() calls");
        if (!alpha.empty())
            costa::transform<T>(from, to, transpose.data(), alpha.data(), beta.data(), comm);
        else
            costa::transform<T>(from, to, comm);
        clear();
    }
    void clear() {
        from.clear();
        to.clear();
        alpha.clear();
        beta.clear();
        transpose.clear();
    }
};

#ifdef MPI_VERSION
// ---- MPI_Comm signatures of the reference (header-only: works with the application's MPI).
// Every MPI communicator gets ONE costa communicator (RCCL over the same ranks, one GPU per
// rank: node-local rank modulo the visible devices), cached as an MPI attribute and
// destroyed with the MPI communicator.  Collective over `comm` on first use.
namespace detail {
inline int mpi_comm_delete(MPI_Comm, int, void* attr, void*) {
    costa_hip_comm_destroy(static_cast<costa_comm_t>(attr));
    return MPI_SUCCESS;
}
inline int& mpi_keyval() {
    static int k = MPI_KEYVAL_INVALID;
    return k;
}
}  // namespace detail

inline costa_comm_t comm_from_mpi(MPI_Comm comm, int device = -1) {
    int& key = detail::mpi_keyval();
    if (key == MPI_KEYVAL_INVALID)
        MPI_Comm_create_keyval(MPI_COMM_NULL_COPY_FN, detail::mpi_comm_delete, &key, nullptr);
    void* val = nullptr;
    int flag = 0;
    MPI_Comm_get_attr(comm, key, &val, &flag);
    if (flag) return static_cast<costa_comm_t>(val);
    int rank = 0, size = 1;
    MPI_Comm_rank(comm, &rank);
    MPI_Comm_size(comm, &size);
    if (device < 0) {
        MPI_Comm node;
        MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
        int local = 0, ndev = 1;
        MPI_Comm_rank(node, &local);
        MPI_Comm_free(&node);
        if (costa_hip_device_count(&ndev) != COSTA_OK || ndev < 1)
            throw hip_error(COSTA_ERR_HIP, costa_hip_last_error());
        device = local % ndev;
    }
    unsigned char id[128] = {0};
    int rc = COSTA_OK;
    if (size > 1 && rank == 0) rc = costa_hip_comm_unique_id(id);
    if (size > 1) {
        MPI_Bcast(&rc, 1, MPI_INT, 0, comm);
        if (rc != COSTA_OK) throw hip_error(rc, "costa: RCCL unique id failed on rank 0");
        MPI_Bcast(id, 128, MPI_UNSIGNED_CHAR, 0, comm);
    }
    costa_comm_t c = nullptr;
    rc = costa_hip_comm_create(id, size, rank, device, &c);
    if (rc != COSTA_OK) throw hip_error(rc, costa_hip_last_error());
    MPI_Comm_set_attr(comm, key, c);
    return c;
}

template <typename T>
transformer<T>::transformer(MPI_Comm c) : comm(comm_from_mpi(c)) {}

// Rank-pair cost factors for comm_volume::apply_topology (reference utils.hpp:12,
// utils.cpp:30-88): 1 between nodes, 2 for ranks sharing a node (their volume counts half).
// Collective over `comm`.
inline std::vector<std::vector<int>> topology_cost(MPI_Comm comm) {
    int P = 1, rank = 0;
    MPI_Comm_size(comm, &P);
    MPI_Comm_rank(comm, &rank);
    MPI_Comm node;
    MPI_Comm_split_type(comm, MPI_COMM_TYPE_SHARED, rank, MPI_INFO_NULL, &node);
    int node_id = rank;  // a node is named by its smallest rank
    MPI_Allreduce(&rank, &node_id, 1, MPI_INT, MPI_MIN, node);
    MPI_Comm_free(&node);
    std::vector<int> node_of(size_t(P), 0);
    MPI_Allgather(&node_id, 1, MPI_INT, node_of.data(), 1, MPI_INT, comm);
    std::vector<std::vector<int>> cost(size_t(P), std::vector<int>(size_t(P), 1));
    for (int i = 0; i < P; ++i)
        for (int j = 0; j < P; ++j)
            if (node_of[size_t(i)] == node_of[size_t(j)]) cost[size_t(i)][size_t(j)] = 2;
    return cost;
}

template <typename T>
void transform(grid_layout<T>& A, grid_layout<T>& C, MPI_Comm comm) {
    transform<T>(A, C, comm_from_mpi(comm));
}
template <typename T>
void transform(grid_layout<T>& A, grid_layout<T>& C, char trans, T alpha, T beta, MPI_Comm comm) {
    transform<T>(A, C, trans, alpha, beta, comm_from_mpi(comm));
}
template <typename T>
void transform(std::vector<layout_ref<T>>& A, std::vector<layout_ref<T>>& C, MPI_Comm comm) {
    transform<T>(A, C, comm_from_mpi(comm));
}
template <typename T>
void transform(std::vector<layout_ref<T>>& A, std::vector<layout_ref<T>>& C, const char* trans,
               const T* alpha, const T* beta, MPI_Comm comm) {
    transform<T>(A, C, trans, alpha, beta, comm_from_mpi(comm));
}
#endif  // MPI_VERSION

}  // namespace costa
