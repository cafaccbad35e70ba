// One tile of a transform as a costa_tile_op_t: the sub-tile address inside its block and the
// normalisation of copy_and_transform's dispatch.  Shared by the host planner (plan.cpp) and
// the device planner (device_plan.hip), so both emit bit-identical ops.
#pragma once

#include <cstdint>

#include "costa_hip.h"

#if defined(__HIPCC__)
#define COSTA_HD __host__ __device__
#else
#define COSTA_HD
#endif

namespace costa {
namespace engine {

// The stored-orientation sub-tile of a block for the target-coordinate rectangle
// [r0, r1) x [c0, c1) of a view that is transposed when `t` (block.cpp:72-111).
struct tile_side {
    uint64_t ptr;         // first element
    int ld;
    int n_rows, n_cols;   // stored orientation
};

COSTA_HD inline tile_side sub_tile(uint64_t data, int ld, int block_row0, int block_col0,
                                   bool row_major, bool t, int r0, int r1, int c0, int c1,
                                   uint64_t elem) {
    // back to the stored orientation of the block
    const int sr0 = t ? c0 : r0, sr1 = t ? c1 : r1;
    const int sc0 = t ? r0 : c0, sc1 = t ? r1 : c1;
    const int64_t dr = sr0 - block_row0, dc = sc0 - block_col0;
    const int64_t off = row_major ? dr * ld + dc : dc * ld + dr;
    return {data + uint64_t(off * int64_t(elem)), ld, sr1 - sr0, sc1 - sc0};
}

// copy_and_transform (memory_utils.hpp:339-412) as one op: an ordering mismatch is itself a
// transpose and cancels an explicit one (:353-367); stride 0 means the default stride
// (:330-337, 370-381); a transposing op never takes the memcpy branch.
COSTA_HD inline costa_tile_op_t tile_op(int n_rows, int n_cols, uint64_t src, int src_stride,
                                        bool src_cm, uint64_t dst, int dst_stride, bool dst_cm,
                                        bool transpose, bool conj, uint32_t kind, uint32_t slot,
                                        uint64_t elem) {
    const bool will_transpose = (transpose && src_cm == dst_cm) || (!transpose && src_cm != dst_cm);
    if (dst_stride == 0) {
        const int r = will_transpose ? n_cols : n_rows, c = will_transpose ? n_rows : n_cols;
        dst_stride = dst_cm ? r : c;
    }
    if (src_stride == 0) src_stride = src_cm ? n_rows : n_cols;
    costa_tile_op_t op{};
    op.src = src;
    op.dst = dst;
    op.nf = src_cm ? n_rows : n_cols;  // contiguous extent of the source
    op.ns = src_cm ? n_cols : n_rows;
    op.lds = src_stride;
    op.ldd = dst_stride;
    if (will_transpose && kind == COSTA_SCALE_BITCOPY) kind = COSTA_SCALE_ALPHA;  // never memcpy
    op.flags = (will_transpose ? COSTA_TILE_TRANSPOSE : 0u) | (conj ? COSTA_TILE_CONJ : 0u) |
               (kind << COSTA_SCALE_SHIFT) | (slot << COSTA_SLOT_SHIFT);
    if (src % 16 == 0 && (uint64_t(src_stride) * elem) % 16 == 0) op.flags |= COSTA_TILE_VEC_SRC;
    if (dst % 16 == 0 && (uint64_t(dst_stride) * elem) % 16 == 0) op.flags |= COSTA_TILE_VEC_DST;
    return op;
}

// algorithmic HBM bytes of one op: read + write (+ read of the target when beta != 0)
COSTA_HD inline int64_t op_alg_bytes(const costa_tile_op_t& op, uint64_t elem) {
    const uint32_t k = (op.flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
    const int64_t n = int64_t(op.nf) * op.ns;
    return int64_t(elem) * n * (1 + (k != COSTA_SCALE_ZERO) + (k == COSTA_SCALE_AXPBY));
}

}  // namespace engine
}  // namespace costa
