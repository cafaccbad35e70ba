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

}  // namespace costa
