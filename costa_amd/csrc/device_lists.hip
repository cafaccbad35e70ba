// Destination-block groups built on the GPU (the work lists of a plan-cache miss,
// after the device planner).  engine.cpp cblock_groups restated as sorts, scans and
// one-thread-per-item kernels, so that cfg 5's 242 k wavefront tiles do not cost ~20 ms of host
// time (the reference builds its packages on the host at every call: utils.hpp:87-206,
// communication_data.cpp:251-302).  The same steps as the host builder:
//   candidates  one thread per op: the destination footprint [lo, hi) and leading dimension R of
//               the ops that may join a group (the host's filter), compacted in list order
//   order       one stable radix sort by (R, lo): the host's two stable LSD passes in one key
//   components  a max-scan of hi per R: a candidate starts a component when its lo lies past every
//               earlier footprint of its R (the host's sweep; singletons never group)
//   check       one thread per component: one transform, rows inside R, areas adding up to R x K;
//               then every op's four corners, sorted with the component in the key, must leave
//               exactly the range's own four corners with odd counts (the host's perfect-rectangle
//               test: the ops then tile the range exactly)
//   groups      column bands of at most `budget` elements: a scan of the band counts, one thread
//               per band for its op count and smallest locality hint
//   order       stable radix sorts by range offset, then (copy-only lists with hints) by the XCD
//               slice of each group's hint rank
//   emit        a scan of the groups' sizes; one thread per group writes [header, ops cut at the
//               band edges]
// Same groups, order and bytes as the host builder (tests/test_gpu_work_lists.py).  Keys that do not
// fit 64 bits (address spans past 2^50 elements and the like) decline to the host builder.
// Compiled as part of device_plan.hip (included at its end): one code object, the same rocPRIM
// instantiations (32-bit radix sort pairs, 32- and 64-bit scans) and one load for both.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/device/device_scan_by_key.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "engine.hpp"

namespace costa {
namespace engine {

#define DL_CHECK(x)                                                                    \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
            throw error(COSTA_ERR_HIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

namespace {

using u64 = unsigned long long;

// device-side totals, read back at the host's few synchronisation points
struct dl_totals {
    u64 lo_min, lo_max, hi_max;  // candidates' footprints
    u64 ncand, ncomp, ck_max;    // candidates, components, largest corner key of a checked one
    u64 ng, any_tr, hints_bad, lds, n_out;
    u64 n_ok, n_valid;  // components through the first check / both (trace)
    u64 n_bad, n_odd4;  // checked components with a stray odd corner / exactly four odd (trace)
};

constexpr int kThreads = 256;
unsigned dl_grid(int64_t n) { return unsigned(std::max<int64_t>(1, (n + kThreads - 1) / kThreads)); }

int bits_of(uint64_t x) {  // bits to hold x (at least 1)
    int b = 1;
    while (b < 64 && (x >> b) != 0) ++b;
    return b;
}

__device__ inline u64 wave_min(u64 v) {
    for (int o = 32; o > 0; o >>= 1) {
        const u64 w = __shfl_xor(v, o);
        v = w < v ? w : v;
    }
    return v;
}
__device__ inline u64 wave_max(u64 v) {
    for (int o = 32; o > 0; o >>= 1) {
        const u64 w = __shfl_xor(v, o);
        v = w > v ? w : v;
    }
    return v;
}

__device__ inline int64_t run_of(const costa_tile_op_t& op) {  // destination run (column height)
    return (op.flags & COSTA_TILE_TRANSPOSE) ? op.ns : op.nf;
}
__device__ inline int64_t runs_of(const costa_tile_op_t& op) {  // destination columns
    return (op.flags & COSTA_TILE_TRANSPOSE) ? op.nf : op.ns;
}

// candidates: footprint and leading dimension of every wavefront op that may join a group
__global__ void dl_candidates(const costa_tile_op_t* ops, const uint32_t* wave, int64_t nw, int64_t E,
                              int64_t budget, uint32_t* flag, uint64_t* lo, uint64_t* hi, int32_t* ldd,
                              dl_totals* t) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    u64 mn = ~0ull, mx = 0, hx = 0;
    if (i < nw) {
        const costa_tile_op_t op = ops[wave[i]];
        bool ok = op.nf > 0 && op.ns > 0 && op.ldd > 0 && op.dst % uint64_t(E) == 0;
        uint64_t l = 0, h = 0;
        if (ok) {
            const int64_t run = run_of(op), runs = runs_of(op);
            ok = run <= op.ldd && op.ldd <= budget;
            l = op.dst;
            h = op.dst + uint64_t(((runs - 1) * int64_t(op.ldd) + run) * E);
        }
        flag[i] = ok;
        lo[i] = l;
        hi[i] = h;
        ldd[i] = op.ldd;
        if (ok) mn = l, mx = l, hx = h;
    }
    mn = wave_min(mn);
    mx = wave_max(mx);
    hx = wave_max(hx);
    if ((threadIdx.x & 63) == 0 && hx != 0) {  // hi > 0 for every candidate
        atomicMin(&t->lo_min, mn);
        atomicMax(&t->lo_max, mx);
        atomicMax(&t->hi_max, hx);
    }
}

__global__ void dl_compact(const uint32_t* flag, const uint32_t* pos, int64_t nw, uint32_t* cand,
                           dl_totals* t) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= nw) return;
    if (flag[i]) cand[pos[i]] = uint32_t(i);
    if (i == nw - 1) t->ncand = pos[i] + flag[i];
}

// sort key (R, element offset of lo): R above the offset's sb bits
__global__ void dl_keys(const uint32_t* cand, int64_t nc, const uint64_t* lo, const int32_t* ldd,
                        uint64_t lo_min, int64_t E, int sb, uint64_t* key, uint32_t* val) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= nc) return;
    const uint32_t i = cand[k];
    key[k] = (uint64_t(uint32_t(ldd[i])) << sb) | ((lo[i] - lo_min) / uint64_t(E));
    val[k] = uint32_t(k);
}

// the candidates in (R, lo) order: wavefront position (s_i), op index (s_op), footprint
__global__ void dl_gather(const uint32_t* sval, const uint32_t* cand, const uint32_t* wave, int64_t nc,
                          const uint64_t* lo, const uint64_t* hi, const int32_t* ldd, uint32_t* s_i,
                          uint32_t* s_op, uint64_t* s_lo, uint64_t* s_hi, int32_t* s_ldd) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= nc) return;
    const uint32_t i = cand[sval[k]];
    s_i[k] = i;
    s_op[k] = wave[i];
    s_lo[k] = lo[i];
    s_hi[k] = hi[i];
    s_ldd[k] = ldd[i];
}

// a candidate starts a component at a new R or when it lies past every earlier footprint of its R
// pmax: the max-scan of (R, hi) -- its low hb bits are the largest hi (element offset) so far of
// the candidate's R
__global__ void dl_starts(const uint64_t* s_lo, const int32_t* s_ldd, const uint64_t* pmax, int64_t nc,
                          uint64_t lo_min, int64_t E, int hb, uint32_t* start) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= nc) return;
    start[k] = k == 0 || s_ldd[k] != s_ldd[k - 1] ||
               (s_lo[k] - lo_min) / uint64_t(E) > (pmax[k - 1] & ((uint64_t(1) << hb) - 1));
}

// the exclusive scan of the starts made inclusive: candidate k is in component cnum[k] - 1
__global__ void dl_inclusive(const uint32_t* start, int64_t nc, uint32_t* cnum) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k < nc) cnum[k] += start[k];
}

__global__ void dl_bounds(const uint32_t* start, const uint32_t* cnum, int64_t nc, uint32_t* comp_a,
                          uint32_t* comp_b, dl_totals* t) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= nc) return;
    const uint32_t c = cnum[k] - 1;
    if (start[k]) comp_a[c] = uint32_t(k);
    if (k + 1 == nc || start[k + 1]) comp_b[c] = uint32_t(k + 1);
    if (k + 1 == nc) t->ncomp = c + 1;
}

// per component: one transform, rows inside R, areas adding up to R x K
__global__ void dl_check(const costa_tile_op_t* ops, const uint32_t* s_op, const uint64_t* s_lo,
                         const int32_t* s_ldd, const uint32_t* comp_a, const uint32_t* comp_b, int64_t nc,
                         int64_t E, uint32_t vec_bits, int64_t* comp_K, uint32_t* comp_fl, uint32_t* comp_ok,
                         dl_totals* t) {
    const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    const int64_t ncomp = int64_t(t->ncomp);
    u64 ck = 0;
    if (c < ncomp) {
        const uint32_t a0 = comp_a[c], b = comp_b[c];
        uint32_t ok = 0;
        if (b - a0 >= 2) {
            const int64_t R = s_ldd[a0];
            const uint64_t base = s_lo[a0];
            const uint32_t fl = ops[s_op[a0]].flags & ~vec_bits;
            int64_t area = 0, K = 0;
            bool good = true;
            for (uint32_t k = a0; k < b && good; ++k) {
                const costa_tile_op_t op = ops[s_op[k]];
                const int64_t run = run_of(op), runs = runs_of(op);
                const int64_t e = int64_t(op.dst - base) / E;
                good = (op.flags & ~vec_bits) == fl && e % R + run <= R;
                area += run * runs;
                K = max(K, e / R + runs);
            }
            if (good && area == R * K && K <= INT32_MAX) {
                ok = 1;
                comp_K[c] = K;
                comp_fl[c] = fl;
                ck = u64(R) * u64(K + 1) + u64(K);
            }
        }
        comp_ok[c] = ok;
    }
    ck = wave_max(ck);
    if ((threadIdx.x & 63) == 0 && ck) atomicMax(&t->ck_max, ck);
    if (c < ncomp && comp_ok[c]) atomicAdd(&t->n_ok, 1ull);
}

// the four corners of every op of a checked component, the component above the corner's ck bits;
// ops of other components get a key past every real one
__global__ void dl_corners(const costa_tile_op_t* ops, const uint32_t* s_op, const uint64_t* s_lo,
                           const int32_t* s_ldd, const uint32_t* cnum, const uint32_t* comp_a,
                           const uint32_t* comp_ok, const int64_t* comp_K, int64_t nc, int64_t E, int ck,
                           uint64_t ncomp, uint64_t* keys) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= nc) return;
    const uint32_t c = cnum[k] - 1;
    uint64_t* out = keys + 4 * k;
    if (!comp_ok[c]) {
        out[0] = out[1] = out[2] = out[3] = ncomp << ck;
        return;
    }
    const uint64_t R = uint64_t(s_ldd[k]), base = s_lo[comp_a[c]], W = uint64_t(comp_K[c]) + 1;
    const costa_tile_op_t op = ops[s_op[k]];
    const uint64_t run = uint64_t(run_of(op)), runs = uint64_t(runs_of(op));
    const uint64_t e = (op.dst - base) / uint64_t(E), r0 = e % R, c0 = e / R;
    const uint64_t hc = uint64_t(c) << ck;
    out[0] = hc | (r0 * W + c0);
    out[1] = hc | (r0 * W + c0 + runs);
    out[2] = hc | ((r0 + run) * W + c0);
    out[3] = hc | ((r0 + run) * W + c0 + runs);
}

// runs of equal sorted corners: an odd count must be one of the range's four corners
__global__ void dl_parity(const uint64_t* sk, int64_t n, int ck, uint64_t ncomp, const int32_t* s_ldd,
                          const uint32_t* comp_a, const int64_t* comp_K, uint32_t* odd, uint32_t* bad) {
    const int64_t j = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (j >= n) return;
    const uint64_t key = sk[j];
    if (j > 0 && sk[j - 1] == key) return;
    const uint64_t c = key >> ck;
    if (c >= ncomp) return;
    int64_t m = 1;
    while (j + m < n && sk[j + m] == key) ++m;
    if (!(m & 1)) return;
    const uint64_t corner = key & ((uint64_t(1) << ck) - 1);
    const uint64_t R = uint64_t(s_ldd[comp_a[c]]), K = uint64_t(comp_K[c]), W = K + 1;
    if (corner == 0 || corner == K || corner == R * W || corner == R * W + K)
        atomicAdd(&odd[c], 1u);
    else
        atomicOr(&bad[c], 1u);
}

// groups (column bands) per component: none for components that failed a check
__global__ void dl_count(const uint32_t* comp_ok, const uint32_t* odd, const uint32_t* bad,
                         const int32_t* s_ldd, const uint32_t* comp_a, const int64_t* comp_K, int64_t budget,
                         int64_t nc, uint64_t* comp_ng, int64_t* comp_KB, dl_totals* t) {
    const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (c >= nc) return;
    if (c < int64_t(t->ncomp) && comp_ok[c]) {
        if (bad[c]) atomicAdd(&t->n_bad, 1ull);
        if (odd[c] == 4) atomicAdd(&t->n_odd4, 1ull);
    }
    if (c >= int64_t(t->ncomp) || !comp_ok[c] || bad[c] || odd[c] != 4) {
        comp_ng[c] = 0;
        return;
    }
    const int64_t R = s_ldd[comp_a[c]], K = comp_K[c];
    const int64_t KB = max(int64_t(1), budget / R);
    atomicAdd(&t->n_valid, 1ull);
    comp_KB[c] = KB;
    comp_ng[c] = uint64_t((K + KB - 1) / KB);
}

__global__ void dl_total(const uint64_t* comp_ng, const uint64_t* comp_gat, dl_totals* t) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const uint64_t n = t->ncomp;
    t->ng = n ? comp_gat[n - 1] + comp_ng[n - 1] : 0;
}

// each component's number at its first group; a max-scan fills the rest of its groups
__global__ void dl_seed(const uint64_t* comp_ng, const uint64_t* comp_gat, int64_t nc, uint64_t* g_comp,
                        const dl_totals* t) {
    const int64_t c = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (c >= nc || c >= int64_t(t->ncomp) || comp_ng[c] == 0) return;
    g_comp[comp_gat[c]] = uint64_t(c);
}

// per group: its range, its op count (an op cut at the band edges counts once per band), the
// smallest hint of its ops (0: one lacks a hint)
__global__ void dl_table(const costa_tile_op_t* ops, const uint32_t* s_op, const uint64_t* s_lo,
                         const int32_t* s_ldd, const uint32_t* comp_a, const uint32_t* comp_b,
                         const int64_t* comp_K, const int64_t* comp_KB, const uint32_t* comp_fl,
                         const uint64_t* comp_gat, const uint64_t* g_comp, int64_t ng, int64_t E,
                         uint64_t* g_dst, uint32_t* g_band, uint32_t* g_nops, uint32_t* g_hint, dl_totals* t) {
    const int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    u64 tr = 0, hb = 0, lds = 0;
    if (g < ng) {
        const uint32_t c = uint32_t(g_comp[g]);
        const uint32_t band = uint32_t(uint64_t(g) - comp_gat[c]);
        const uint32_t a0 = comp_a[c], b = comp_b[c];
        const int64_t R = s_ldd[a0], K = comp_K[c], KB = comp_KB[c];
        const uint64_t base = s_lo[a0];
        const int64_t cb0 = int64_t(band) * KB, cb1 = min(K, cb0 + KB);
        uint32_t n = 0, hint = UINT32_MAX;
        for (uint32_t k = a0; k < b; ++k) {
            const costa_tile_op_t op = ops[s_op[k]];
            const int64_t c0 = int64_t(op.dst - base) / E / R;
            if (max(cb0, c0) >= min(cb1, c0 + runs_of(op))) continue;
            ++n;
            hint = op.order ? min(hint, op.order) : 0u;
        }
        g_dst[g] = base + uint64_t(cb0 * R * E);
        g_band[g] = band;
        g_nops[g] = n;
        g_hint[g] = hint;
        tr = (comp_fl[c] & COSTA_TILE_TRANSPOSE) ? 1 : 0;
        hb = hint == 0 || hint == UINT32_MAX;
        lds = u64(R | 1) * u64(cb1 - cb0);
    }
    tr = wave_max(tr);
    hb = wave_max(hb);
    lds = wave_max(lds);
    if ((threadIdx.x & 63) == 0) {
        if (tr) atomicMax(&t->any_tr, tr);
        if (hb) atomicMax(&t->hints_bad, hb);
        if (lds) atomicMax(&t->lds, lds);
    }
}

__global__ void dl_taken(const uint32_t* cnum, const uint64_t* comp_ng, const uint32_t* s_i, int64_t nc,
                         uint8_t* taken) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= nc) return;
    if (comp_ng[cnum[k] - 1]) taken[s_i[k]] = 1;
}

__global__ void dl_dst_keys(const uint64_t* g_dst, int64_t ng, uint64_t lo_min, int64_t E, uint64_t* key,
                            uint32_t* iota) {
    const int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g >= ng) return;
    key[g] = (g_dst[g] - lo_min) / uint64_t(E);
    iota[g] = uint32_t(g);
}

__global__ void dl_iota(int64_t n, uint32_t* iota) {
    const int64_t g = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (g < n) iota[g] = uint32_t(g);
}

// the XCD slice of each group: slice x holds ranks [x (per + 1), ...) of the hint order, the first
// `rem` slices one more than the rest (xcd_slice_order's slices)
__global__ void dl_slices(const uint32_t* by, int64_t ng, uint32_t* band) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k >= ng) return;
    const int64_t per = ng / 8, rem = ng % 8;
    band[by[k]] = uint32_t(k < rem * (per + 1) ? k / (per + 1) : rem + (k - rem * (per + 1)) / per);
}

__global__ void dl_gather_u32(const uint32_t* src, const uint32_t* idx, int64_t n, uint32_t* dst) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k < n) dst[k] = src[idx[k]];
}

__global__ void dl_sizes(const uint32_t* order, const uint32_t* g_nops, int64_t ng, uint64_t* size) {
    const int64_t q = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (q < ng) size[q] = 1 + uint64_t(g_nops[order[q]]);
}

__global__ void dl_out_total(const uint64_t* at, const uint64_t* size, int64_t ng, dl_totals* t) {
    if (threadIdx.x == 0 && blockIdx.x == 0) t->n_out = at[ng - 1] + size[ng - 1];
}

// [header, ops...] per group in order, each op cut at its band's edges; the group's work entry
__global__ void dl_emit(const costa_tile_op_t* ops, const uint32_t* s_op, const uint64_t* s_lo,
                        const int32_t* s_ldd, const uint32_t* comp_a, const uint32_t* comp_b,
                        const int64_t* comp_K, const int64_t* comp_KB, const uint32_t* comp_fl,
                        const uint64_t* g_comp, const uint32_t* g_band, const uint32_t* g_nops,
                        const uint64_t* g_dst, const uint32_t* order, const uint64_t* at, int64_t ng,
                        int64_t E, uint64_t base_at, costa_tile_op_t* out_ops, uint64_t* out_work) {
    const int64_t q = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (q >= ng) return;
    const uint32_t g = order[q], c = uint32_t(g_comp[g]);
    const uint32_t a0 = comp_a[c], b = comp_b[c];
    const int64_t R = s_ldd[a0], K = comp_K[c], KB = comp_KB[c];
    const uint64_t base = s_lo[a0];
    const int64_t cb0 = int64_t(g_band[g]) * KB, cb1 = min(K, cb0 + KB);
    costa_tile_op_t* out = out_ops + at[q];
    out_work[q] = base_at + at[q];
    costa_tile_op_t h{};
    h.src = g_nops[g];
    h.dst = g_dst[g];
    h.nf = int32_t(R);
    h.ns = int32_t(cb1 - cb0);
    h.ldd = int32_t(R);
    h.flags = comp_fl[c];
    *out++ = h;
    for (uint32_t k = a0; k < b; ++k) {
        costa_tile_op_t op = ops[s_op[k]];
        const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
        const int64_t c0 = int64_t(op.dst - base) / E / R;
        const int64_t lo = max(cb0, c0), up = min(cb1, c0 + runs_of(op));
        if (lo >= up) continue;
        const int64_t d0 = lo - c0, dn = up - lo;  // destination columns of the op kept
        op.dst += uint64_t(d0 * R * E);
        if (tr) {
            op.src += uint64_t(d0 * E);
            op.nf = int32_t(dn);
        } else {
            op.src += uint64_t(d0 * int64_t(op.lds) * E);
            op.ns = int32_t(dn);
        }
        *out++ = op;
    }
}

// two stable passes of the planner's 32-bit radix sort make one stable sort of 64-bit keys (one
// rocPRIM instantiation for both, in one code object: device_plan.hip includes this file)
__global__ void dl_split_lo(const uint64_t* key, int64_t n, uint32_t* k32, uint32_t* iota) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i >= n) return;
    k32[i] = uint32_t(key[i]);
    iota[i] = uint32_t(i);
}
__global__ void dl_gather_hi(const uint64_t* key, const uint32_t* perm, int64_t n, uint32_t* k32) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) k32[i] = uint32_t(key[perm[i]] >> 32);
}
__global__ void dl_gather_u64(const uint64_t* src, const uint32_t* perm, int64_t n, uint64_t* dst) {
    const int64_t i = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[perm[i]];
}
// (R, hi) in one word: a max-scan of it is the max-scan of hi within each run of equal R
__global__ void dl_rhi(const int32_t* s_ldd, const uint64_t* s_hi, int64_t nc, uint64_t lo_min, int64_t E,
                       int hb, uint64_t* rhi) {
    const int64_t k = int64_t(blockIdx.x) * blockDim.x + threadIdx.x;
    if (k < nc) rhi[k] = (uint64_t(uint32_t(s_ldd[k])) << hb) | ((s_hi[k] - lo_min) / uint64_t(E));
}

// launched once before the first build: loads this file's code object (trace: its cost)
__global__ void dl_noop(uint32_t* p, int64_t n) {
    if (int64_t(threadIdx.x) < n) p[threadIdx.x] = 0;
}

// one device allocation carved into 256-byte aligned pieces
struct dl_mem {
    void* p = nullptr;
    size_t top = 0, cap = 0;
    dl_mem() = default;
    dl_mem(const dl_mem&) = delete;
    dl_mem& operator=(const dl_mem&) = delete;
    ~dl_mem() {
        if (p) (void)hipFree(p);
    }
    size_t take(size_t bytes) {
        const size_t o = top;
        top += (bytes + 255) & ~size_t(255);
        return o;
    }
    void alloc() {
        cap = std::max<size_t>(top, 256);
        DL_CHECK(hipMalloc(&p, cap));
    }
    template <typename T>
    T* at(size_t off) const {
        return reinterpret_cast<T*>(static_cast<char*>(p) + off);
    }
};

// rocPRIM scratch, grown when a call needs more
struct dl_scratch {
    void* p = nullptr;
    size_t n = 0;
    dl_scratch() = default;
    dl_scratch(const dl_scratch&) = delete;
    dl_scratch& operator=(const dl_scratch&) = delete;
    ~dl_scratch() {
        if (p) (void)hipFree(p);
    }
    void* ensure(size_t bytes) {
        if (bytes > n) {
            if (p) DL_CHECK(hipFree(p));
            p = nullptr;
            n = 0;
            DL_CHECK(hipMalloc(&p, std::max<size_t>(bytes, 256)));
            n = std::max<size_t>(bytes, 256);
        }
        return p;
    }
};

}  // namespace

int64_t cblock_groups_device(int64_t E, int64_t budget, uint32_t vec_bits, int bands_env,
                             const std::vector<costa_tile_op_t>& ops_h, const std::vector<uint32_t>& wave_h,
                             size_t base_at, device_section& sec, std::vector<char>& taken_h, int64_t& lds,
                             int& map) {
    // COSTA_PLAN_TRACE=1: the phases (stderr)
    static const bool trace = std::getenv("COSTA_PLAN_TRACE") != nullptr;
    auto now = [] {
        return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const double t0 = now();
    double lap[6] = {0, 0, 0, 0, 0, 0};
    lds = 0;
    map = cb_round_robin;
    taken_h.assign(wave_h.size(), 0);
    const int64_t nw = int64_t(wave_h.size());
    if (nw < 2) return 0;
    DL_CHECK(hipSetDevice(sec.device));
    hipStream_t s = static_cast<hipStream_t>(sec.stream);
    auto sync = [&] { DL_CHECK(hipStreamSynchronize(s)); };
    static bool loaded = false;
    if (trace && !loaded) {
        sync();
        const double w0 = now();
        hipLaunchKernelGGL(dl_noop, dim3(1), dim3(64), 0, s, static_cast<uint32_t*>(nullptr), int64_t(0));
        sync();
        std::fprintf(stderr, "[costa device groups] first launch of the process: %.2f ms\n", now() - w0);
    }
    loaded = true;

    // ---- candidates, their order, components, checks: arrays of nw (4 nw corners) ----
    const size_t N = size_t(nw);
    dl_mem m;
    const size_t o_ops = m.take(ops_h.size() * sizeof(costa_tile_op_t)), o_wave = m.take(N * 4);
    const size_t o_t = m.take(sizeof(dl_totals));
    const size_t o_flag = m.take(N * 4), o_pos = m.take(N * 4), o_cand = m.take(N * 4);
    const size_t o_lo = m.take(N * 8), o_hi = m.take(N * 8), o_ldd = m.take(N * 4);
    const size_t o_key = m.take(N * 8), o_sval = m.take(N * 4);
    const size_t o_si = m.take(N * 4), o_sop = m.take(N * 4), o_slo = m.take(N * 8), o_shi = m.take(N * 8);
    const size_t o_sldd = m.take(N * 4), o_rhi = m.take(N * 8), o_pmax = m.take(N * 8);
    const size_t o_start = m.take(N * 4), o_cnum = m.take(N * 4);
    const size_t o_ca = m.take(N * 4), o_cb = m.take(N * 4), o_cK = m.take(N * 8), o_cKB = m.take(N * 8);
    const size_t o_cfl = m.take(N * 4), o_cok = m.take(N * 4), o_odd = m.take(N * 4), o_bad = m.take(N * 4);
    const size_t o_cng = m.take(N * 8), o_cgat = m.take(N * 8);
    const size_t o_ck = m.take(4 * N * 8), o_sck = m.take(4 * N * 8), o_taken = m.take(N);
    const size_t o_ka = m.take(4 * N * 4), o_kb = m.take(4 * N * 4), o_va = m.take(4 * N * 4),
                 o_vb = m.take(4 * N * 4), o_perm = m.take(4 * N * 4);
    m.alloc();
    dl_scratch tmp;
    size_t q = 0;

    costa_tile_op_t* d_ops = m.at<costa_tile_op_t>(o_ops);
    uint32_t* d_wave = m.at<uint32_t>(o_wave);
    dl_totals* d_t = m.at<dl_totals>(o_t);
    uint32_t *flag = m.at<uint32_t>(o_flag), *pos = m.at<uint32_t>(o_pos), *cand = m.at<uint32_t>(o_cand);
    uint64_t *lo = m.at<uint64_t>(o_lo), *hi = m.at<uint64_t>(o_hi), *key = m.at<uint64_t>(o_key);
    int32_t* ldd = m.at<int32_t>(o_ldd);
    uint32_t *sval = m.at<uint32_t>(o_sval), *s_i = m.at<uint32_t>(o_si), *s_op = m.at<uint32_t>(o_sop);
    uint64_t *s_lo = m.at<uint64_t>(o_slo), *s_hi = m.at<uint64_t>(o_shi);
    uint64_t *rhi = m.at<uint64_t>(o_rhi), *pmax = m.at<uint64_t>(o_pmax);
    int32_t* s_ldd = m.at<int32_t>(o_sldd);
    uint32_t *start = m.at<uint32_t>(o_start), *cnum = m.at<uint32_t>(o_cnum);
    uint32_t *comp_a = m.at<uint32_t>(o_ca), *comp_b = m.at<uint32_t>(o_cb);
    int64_t *comp_K = m.at<int64_t>(o_cK), *comp_KB = m.at<int64_t>(o_cKB);
    uint32_t *comp_fl = m.at<uint32_t>(o_cfl), *comp_ok = m.at<uint32_t>(o_cok);
    uint32_t *odd = m.at<uint32_t>(o_odd), *bad = m.at<uint32_t>(o_bad);
    uint64_t *comp_ng = m.at<uint64_t>(o_cng), *comp_gat = m.at<uint64_t>(o_cgat);
    uint64_t *ckeys = m.at<uint64_t>(o_ck), *sckeys = m.at<uint64_t>(o_sck);
    uint8_t* taken = m.at<uint8_t>(o_taken);
    uint32_t *ka = m.at<uint32_t>(o_ka), *kb = m.at<uint32_t>(o_kb), *va = m.at<uint32_t>(o_va);
    uint32_t *vb = m.at<uint32_t>(o_vb), *perm = m.at<uint32_t>(o_perm);

    // the rocPRIM calls, with the template arguments device_plan.hip instantiates (one code object
    // holds both: the planner's first use loads this builder too), plus one max-scan
    auto scan_u32 = [&](uint32_t* in, uint32_t* out, size_t n) {  // exclusive, +
        DL_CHECK(rocprim::exclusive_scan(nullptr, q, in, out, uint32_t(0), n, rocprim::plus<uint32_t>(), s));
        DL_CHECK(rocprim::exclusive_scan(tmp.ensure(q), q, in, out, uint32_t(0), n, rocprim::plus<uint32_t>(), s));
    };
    auto scan_i64 = [&](uint64_t* in, uint64_t* out, size_t n) {  // exclusive, + (values < 2^63)
        int64_t *a = reinterpret_cast<int64_t*>(in), *b = reinterpret_cast<int64_t*>(out);
        DL_CHECK(rocprim::exclusive_scan(nullptr, q, a, b, int64_t(0), n, rocprim::plus<int64_t>(), s));
        DL_CHECK(rocprim::exclusive_scan(tmp.ensure(q), q, a, b, int64_t(0), n, rocprim::plus<int64_t>(), s));
    };
    auto max_u64 = [&](uint64_t* in, uint64_t* out, size_t n) {  // inclusive, max
        DL_CHECK(rocprim::inclusive_scan(nullptr, q, in, out, n, rocprim::maximum<uint64_t>(), s));
        DL_CHECK(rocprim::inclusive_scan(tmp.ensure(q), q, in, out, n, rocprim::maximum<uint64_t>(), s));
    };
    auto sort_u32 = [&](uint32_t* k, uint32_t* ks, uint32_t* v, uint32_t* vs, size_t n, int bits) {
        DL_CHECK(rocprim::radix_sort_pairs(nullptr, q, k, ks, v, vs, n, 0, bits, s));
        DL_CHECK(rocprim::radix_sort_pairs(tmp.ensure(q), q, k, ks, v, vs, n, 0, bits, s));
    };
    // stable order of n 64-bit keys (their low `bits`) -> p: LSD, two 32-bit passes
    auto sort_u64 = [&](const uint64_t* k, size_t n, int bits, uint32_t* p, uint32_t* k0, uint32_t* k1,
                        uint32_t* v0, uint32_t* v1) {
        hipLaunchKernelGGL(dl_split_lo, dim3(dl_grid(int64_t(n))), dim3(kThreads), 0, s, k, int64_t(n), k0, v0);
        DL_CHECK(hipGetLastError());
        if (bits <= 32) return sort_u32(k0, k1, v0, p, n, bits);
        sort_u32(k0, k1, v0, v1, n, 32);
        hipLaunchKernelGGL(dl_gather_hi, dim3(dl_grid(int64_t(n))), dim3(kThreads), 0, s, k, v1, int64_t(n), k0);
        DL_CHECK(hipGetLastError());
        sort_u32(k0, k1, v1, p, n, bits - 32);
    };

    dl_totals th{};
    th.lo_min = ~0ull;
    DL_CHECK(hipMemcpyAsync(d_ops, ops_h.data(), ops_h.size() * sizeof(costa_tile_op_t), hipMemcpyHostToDevice, s));
    DL_CHECK(hipMemcpyAsync(d_wave, wave_h.data(), N * 4, hipMemcpyHostToDevice, s));
    DL_CHECK(hipMemcpyAsync(d_t, &th, sizeof(th), hipMemcpyHostToDevice, s));
    DL_CHECK(hipMemsetAsync(odd, 0, N * 4, s));
    DL_CHECK(hipMemsetAsync(bad, 0, N * 4, s));
    DL_CHECK(hipMemsetAsync(taken, 0, N, s));
    hipLaunchKernelGGL(dl_candidates, dim3(dl_grid(nw)), dim3(kThreads), 0, s, d_ops, d_wave, nw, E, budget, flag,
                       lo, hi, ldd, d_t);
    DL_CHECK(hipGetLastError());
    scan_u32(flag, pos, N);
    hipLaunchKernelGGL(dl_compact, dim3(dl_grid(nw)), dim3(kThreads), 0, s, flag, pos, nw, cand, d_t);
    DL_CHECK(hipGetLastError());
    DL_CHECK(hipMemcpyAsync(&th, d_t, sizeof(th), hipMemcpyDeviceToHost, s));
    sync();
    lap[0] = now() - t0;
    const int64_t nc = int64_t(th.ncand);
    if (nc < 2) return 0;
    const uint64_t lo_min = th.lo_min;
    const int sb = bits_of((th.lo_max - lo_min) / uint64_t(E)), lb = bits_of(uint64_t(budget));
    const int hb = bits_of((th.hi_max - lo_min) / uint64_t(E));
    if (sb + lb > 64 || hb + lb > 64) return -1;
    const size_t NC = size_t(nc);

    // (R, lo) order, components
    hipLaunchKernelGGL(dl_keys, dim3(dl_grid(nc)), dim3(kThreads), 0, s, cand, nc, lo, ldd, lo_min, E, sb, key, va);
    DL_CHECK(hipGetLastError());
    sort_u64(key, NC, sb + lb, sval, ka, kb, va, vb);
    hipLaunchKernelGGL(dl_gather, dim3(dl_grid(nc)), dim3(kThreads), 0, s, sval, cand, d_wave, nc, lo, hi, ldd, s_i,
                       s_op, s_lo, s_hi, s_ldd);
    hipLaunchKernelGGL(dl_rhi, dim3(dl_grid(nc)), dim3(kThreads), 0, s, s_ldd, s_hi, nc, lo_min, E, hb, rhi);
    DL_CHECK(hipGetLastError());
    max_u64(rhi, pmax, NC);
    hipLaunchKernelGGL(dl_starts, dim3(dl_grid(nc)), dim3(kThreads), 0, s, s_lo, s_ldd, pmax, nc, lo_min, E, hb,
                       start);
    DL_CHECK(hipGetLastError());
    scan_u32(start, cnum, NC);
    hipLaunchKernelGGL(dl_inclusive, dim3(dl_grid(nc)), dim3(kThreads), 0, s, start, nc, cnum);
    hipLaunchKernelGGL(dl_bounds, dim3(dl_grid(nc)), dim3(kThreads), 0, s, start, cnum, nc, comp_a, comp_b, d_t);
    hipLaunchKernelGGL(dl_check, dim3(dl_grid(nc)), dim3(kThreads), 0, s, d_ops, s_op, s_lo, s_ldd, comp_a, comp_b, nc,
                       E, vec_bits, comp_K, comp_fl, comp_ok, d_t);
    DL_CHECK(hipGetLastError());
    DL_CHECK(hipMemcpyAsync(&th, d_t, sizeof(th), hipMemcpyDeviceToHost, s));
    sync();
    lap[1] = now() - t0;
    const uint64_t ncomp = th.ncomp;
    if (th.ck_max == 0) return 0;  // no component passed
    const int ck = bits_of(th.ck_max), cb = bits_of(ncomp);
    if (ck + cb > 64) return -1;

    // perfect-rectangle test, group counts
    hipLaunchKernelGGL(dl_corners, dim3(dl_grid(nc)), dim3(kThreads), 0, s, d_ops, s_op, s_lo, s_ldd, cnum, comp_a,
                       comp_ok, comp_K, nc, E, ck, ncomp, ckeys);
    DL_CHECK(hipGetLastError());
    sort_u64(ckeys, 4 * NC, ck + cb, perm, ka, kb, va, vb);
    hipLaunchKernelGGL(dl_gather_u64, dim3(dl_grid(4 * nc)), dim3(kThreads), 0, s, ckeys, perm, 4 * nc, sckeys);
    hipLaunchKernelGGL(dl_parity, dim3(dl_grid(4 * nc)), dim3(kThreads), 0, s, sckeys, 4 * nc, ck, ncomp, s_ldd,
                       comp_a, comp_K, odd, bad);
    hipLaunchKernelGGL(dl_count, dim3(dl_grid(nc)), dim3(kThreads), 0, s, comp_ok, odd, bad, s_ldd, comp_a, comp_K,
                       budget, nc, comp_ng, comp_KB, d_t);
    DL_CHECK(hipGetLastError());
    scan_i64(comp_ng, comp_gat, NC);
    hipLaunchKernelGGL(dl_total, dim3(1), dim3(64), 0, s, comp_ng, comp_gat, d_t);
    DL_CHECK(hipGetLastError());
    DL_CHECK(hipMemcpyAsync(&th, d_t, sizeof(th), hipMemcpyDeviceToHost, s));
    sync();
    lap[2] = now() - t0;
    const int64_t ng = int64_t(th.ng);
    if (ng == 0) return 0;
    if (ng > int64_t(UINT32_MAX)) return -1;
    const size_t G = size_t(ng);

    // ---- the group table, the order ----
    dl_mem mg;
    const size_t o_gc = mg.take(G * 8), o_gc2 = mg.take(G * 8), o_gd = mg.take(G * 8), o_gb = mg.take(G * 4);
    const size_t o_gn = mg.take(G * 4), o_gh = mg.take(G * 4), o_gk = mg.take(G * 8);
    const size_t o_io = mg.take(G * 4), o_o1 = mg.take(G * 4), o_by = mg.take(G * 4), o_sh = mg.take(G * 4);
    const size_t o_bd = mg.take(G * 4), o_bk = mg.take(G * 4), o_sbk = mg.take(G * 4), o_ord = mg.take(G * 4);
    const size_t o_sz = mg.take(G * 8), o_at = mg.take(G * 8);
    const size_t o_gka = mg.take(G * 4), o_gkb = mg.take(G * 4), o_gva = mg.take(G * 4), o_gvb = mg.take(G * 4);
    mg.alloc();
    uint64_t *g_comp0 = mg.at<uint64_t>(o_gc), *g_comp = mg.at<uint64_t>(o_gc2), *g_dst = mg.at<uint64_t>(o_gd);
    uint32_t *g_band = mg.at<uint32_t>(o_gb), *g_nops = mg.at<uint32_t>(o_gn), *g_hint = mg.at<uint32_t>(o_gh);
    uint64_t* gkey = mg.at<uint64_t>(o_gk);
    uint32_t *iota = mg.at<uint32_t>(o_io), *order1 = mg.at<uint32_t>(o_o1), *by = mg.at<uint32_t>(o_by);
    uint32_t *shint = mg.at<uint32_t>(o_sh), *slice = mg.at<uint32_t>(o_bd), *bkey = mg.at<uint32_t>(o_bk);
    uint32_t *sbkey = mg.at<uint32_t>(o_sbk), *order = mg.at<uint32_t>(o_ord);
    uint64_t *gsize = mg.at<uint64_t>(o_sz), *gat = mg.at<uint64_t>(o_at);
    uint32_t *gka = mg.at<uint32_t>(o_gka), *gkb = mg.at<uint32_t>(o_gkb), *gva = mg.at<uint32_t>(o_gva);
    uint32_t* gvb = mg.at<uint32_t>(o_gvb);

    DL_CHECK(hipMemsetAsync(g_comp0, 0, G * 8, s));
    hipLaunchKernelGGL(dl_seed, dim3(dl_grid(nc)), dim3(kThreads), 0, s, comp_ng, comp_gat, nc, g_comp0, d_t);
    DL_CHECK(hipGetLastError());
    max_u64(g_comp0, g_comp, G);
    hipLaunchKernelGGL(dl_table, dim3(dl_grid(ng)), dim3(kThreads), 0, s, d_ops, s_op, s_lo, s_ldd, comp_a, comp_b,
                       comp_K, comp_KB, comp_fl, comp_gat, g_comp, ng, E, g_dst, g_band, g_nops, g_hint, d_t);
    hipLaunchKernelGGL(dl_taken, dim3(dl_grid(nc)), dim3(kThreads), 0, s, cnum, comp_ng, s_i, nc, taken);
    hipLaunchKernelGGL(dl_dst_keys, dim3(dl_grid(ng)), dim3(kThreads), 0, s, g_dst, ng, lo_min, E, gkey, iota);
    DL_CHECK(hipGetLastError());
    sort_u64(gkey, G, hb, order1, gka, gkb, gva, gvb);
    DL_CHECK(hipMemcpyAsync(&th, d_t, sizeof(th), hipMemcpyDeviceToHost, s));
    sync();
    lap[3] = now() - t0;
    const bool any_tr = th.any_tr != 0, hints = th.hints_bad == 0;
    lds = int64_t(th.lds);
    map = any_tr ? cb_xcd_chunks : cb_round_robin;
    const bool bands = bands_env == 1 || (bands_env == -1 && !any_tr);
    const uint32_t* final_order = order1;
    if (bands && ng >= 16 && hints) {
        // stable by hint, the slices of that order; then stable by slice over the range order
        hipLaunchKernelGGL(dl_iota, dim3(dl_grid(ng)), dim3(kThreads), 0, s, ng, iota);
        DL_CHECK(hipGetLastError());
        sort_u32(g_hint, shint, iota, by, G, 32);
        hipLaunchKernelGGL(dl_slices, dim3(dl_grid(ng)), dim3(kThreads), 0, s, by, ng, slice);
        hipLaunchKernelGGL(dl_gather_u32, dim3(dl_grid(ng)), dim3(kThreads), 0, s, slice, order1, ng, bkey);
        DL_CHECK(hipGetLastError());
        sort_u32(bkey, sbkey, order1, order, G, 3);
        final_order = order;
        map = cb_xcd_bands;
    }

    // ---- emission ----
    hipLaunchKernelGGL(dl_sizes, dim3(dl_grid(ng)), dim3(kThreads), 0, s, final_order, g_nops, ng, gsize);
    DL_CHECK(hipGetLastError());
    scan_i64(gsize, gat, G);
    hipLaunchKernelGGL(dl_out_total, dim3(1), dim3(64), 0, s, gat, gsize, ng, d_t);
    DL_CHECK(hipGetLastError());
    DL_CHECK(hipMemcpyAsync(&th, d_t, sizeof(th), hipMemcpyDeviceToHost, s));
    sync();
    lap[4] = now() - t0;
    const size_t n_out = size_t(th.n_out);
    void* out = nullptr;
    const size_t out_ops_bytes = (n_out * sizeof(costa_tile_op_t) + 255) & ~size_t(255);
    DL_CHECK(hipMalloc(&out, out_ops_bytes + G * 8));
    sec.mem = std::shared_ptr<void>(out, [](void* p) { (void)hipFree(p); });
    sec.d_ordered = static_cast<costa_tile_op_t*>(out);
    sec.d_work = reinterpret_cast<uint64_t*>(static_cast<char*>(out) + out_ops_bytes);
    hipLaunchKernelGGL(dl_emit, dim3(dl_grid(ng)), dim3(kThreads), 0, s, d_ops, s_op, s_lo, s_ldd, comp_a, comp_b,
                       comp_K, comp_KB, comp_fl, g_comp, g_band, g_nops, g_dst, final_order, gat, ng, E,
                       uint64_t(base_at), sec.d_ordered, sec.d_work);
    DL_CHECK(hipGetLastError());
    DL_CHECK(hipMemcpyAsync(taken_h.data(), taken, N, hipMemcpyDeviceToHost, s));
    sync();
    sec.at_ordered = base_at;
    sec.n_ordered = n_out;
    sec.n_work = G;
    if (trace) {
        lap[5] = now() - t0;
        std::fprintf(stderr,
                     "[costa device groups] %lld candidates, %llu components (%llu / %llu checked, %llu stray, %llu four), %lld groups: upload + candidates "
                     "%.2f ms, order + components + check %.2f, corners + counts %.2f, group table + order "
                     "%.2f, slices + sizes %.2f, emit %.2f\n",
                     (long long)nc, (unsigned long long)ncomp, th.n_ok, th.n_valid, th.n_bad, th.n_odd4, (long long)ng, lap[0], lap[1] - lap[0],
                     lap[2] - lap[1], lap[3] - lap[2], lap[4] - lap[3], lap[5] - lap[4]);
    }
    return ng;
}

}  // namespace engine
}  // namespace costa
