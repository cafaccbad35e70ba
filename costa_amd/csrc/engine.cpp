// Executor: device workspaces, plan cache, host staging, and the exchange.
//
// One transform = the reference's exchange_async (grid2grid/transform.cpp:46-128) re-laid
// for one GPU per rank:
//   main stream : [H2D of host-resident data] -> PACK kernel -> RCCL send/recv (all peers,
//                 one group) -> UNPACK kernel -> [D2H]
//   aux stream  : LOCAL kernel, overlapping pack + exchange (the reference overlaps its
//                 local copy with the MPI messages in flight, transform.cpp:96-101)
// Plans are cached by layout content (the reference re-plans every call).
#include <exception>
#include <thread>
#include "engine.hpp"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <numeric>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <mutex>
#include <unordered_map>

namespace costa {
namespace engine {

#define HIP_CHECK(x)                                                                   \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
            throw error(COSTA_ERR_HIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)
#define NCCL_CHECK(x)                                                                   \
    do {                                                                                \
        ncclResult_t r_ = (x);                                                          \
        if (r_ != ncclSuccess)                                                          \
            throw error(COSTA_ERR_NCCL, std::string(#x " failed: ") + ncclGetErrorString(r_)); \
    } while (0)

// ---------------------------------------------------------------- statistics
namespace {
costa_stats_t g_stats{};
bool g_profiling = false;
std::recursive_mutex g_mutex;  // transforms of one process are serialised (the reference's
                               // per-type workspace singleton is not re-entrant either)
}  // namespace
costa_stats_t& stats() { return g_stats; }
bool profiling() { return g_profiling; }
void set_profiling(bool on) { g_profiling = on; }

// ---------------------------------------------------------------- device memory
struct dbuf {
    void* p = nullptr;
    size_t n = 0;
    dbuf() = default;
    dbuf(const dbuf&) = delete;
    dbuf& operator=(const dbuf&) = delete;
    ~dbuf() {
        if (p) (void)hipFree(p);
    }
    void reserve(size_t bytes) {
        if (bytes <= n) return;
        if (p) HIP_CHECK(hipFree(p));
        p = nullptr;
        n = 0;
        // round up to 2 MiB so growing workspaces do not reallocate every call
        size_t want = (bytes + (size_t(2) << 20) - 1) & ~((size_t(2) << 20) - 1);
        HIP_CHECK(hipMalloc(&p, want));
        n = want;
    }
    template <typename X>
    void upload(const std::vector<X>& v, hipStream_t s) {
        if (v.empty()) return;
        reserve(v.size() * sizeof(X));
        HIP_CHECK(hipMemcpyAsync(p, v.data(), v.size() * sizeof(X), hipMemcpyHostToDevice, s));
    }
};

// ---------------------------------------------------------------- per-device context
struct device_ctx {
    struct timed {
        int phase;
        hipEvent_t a, b;
    };
    int device = 0;
    hipStream_t main = nullptr, aux = nullptr, xch = nullptr;  // xch: the RCCL exchange rounds
    hipEvent_t ev_ready = nullptr, ev_local = nullptr, ev_user = nullptr, ev_done = nullptr;
    std::vector<hipEvent_t> ev_packed, ev_moved;  // per exchange round
    void round_events(size_t n) {
        while (ev_packed.size() < n) {
            hipEvent_t a, b;
            HIP_CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
            HIP_CHECK(hipEventCreateWithFlags(&b, hipEventDisableTiming));
            ev_packed.push_back(a);
            ev_moved.push_back(b);
        }
    }
    std::vector<hipEvent_t> free_events;  // timing events ready for reuse
    std::deque<timed> pending;            // recorded phase brackets not yet read
    dbuf send, recv;
    explicit device_ctx(int dev) : device(dev) {
        HIP_CHECK(hipSetDevice(dev));
        // blocking streams: they order after work on the legacy default stream
        HIP_CHECK(hipStreamCreate(&main));
        HIP_CHECK(hipStreamCreate(&aux));
        HIP_CHECK(hipStreamCreate(&xch));
        for (hipEvent_t* e : {&ev_ready, &ev_local, &ev_user, &ev_done})
            HIP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    }
    ~device_ctx() {
        (void)hipSetDevice(device);
        (void)hipStreamSynchronize(main);
        (void)hipStreamSynchronize(aux);
        (void)hipStreamSynchronize(xch);
        for (auto e : ev_packed) (void)hipEventDestroy(e);
        for (auto e : ev_moved) (void)hipEventDestroy(e);
        for (auto& t : pending) {
            (void)hipEventDestroy(t.a);
            (void)hipEventDestroy(t.b);
        }
        for (auto e : free_events) (void)hipEventDestroy(e);
        for (hipEvent_t e : {ev_ready, ev_local, ev_user, ev_done}) (void)hipEventDestroy(e);
        (void)hipStreamDestroy(main);
        (void)hipStreamDestroy(aux);
        (void)hipStreamDestroy(xch);
    }
    hipEvent_t take_event();
    void resolve(size_t max_n = size_t(-1));  // read finished brackets into the statistics
};

namespace {
std::map<int, std::unique_ptr<device_ctx>>& ctx_map() {
    static std::map<int, std::unique_ptr<device_ctx>> m;
    return m;
}
device_ctx& ctx(int device) {
    auto& m = ctx_map();
    auto it = m.find(device);
    if (it == m.end()) it = m.emplace(device, std::make_unique<device_ctx>(device)).first;
    HIP_CHECK(hipSetDevice(device));
    return *it->second;
}
}  // namespace

// ---------------------------------------------------------------- communicator
struct comm {
    int rank = 0, size = 1, device = 0;
    ncclComm_t nccl = nullptr;
    ~comm() {
        if (nccl) (void)ncclCommDestroy(nccl);
    }
};

int device_count() {
    int n = 0;
    HIP_CHECK(hipGetDeviceCount(&n));
    return n;
}

int rccl_version() {
    int v = 0;
    NCCL_CHECK(ncclGetVersion(&v));
    return v;
}

namespace {
comm* new_comm(int device) {
    const int n = device_count();
    if (device < 0 || device >= n) throw error(COSTA_ERR_ARG, "costa: device index out of range");
    auto* c = new comm;
    c->device = device;
    return c;
}

void init_nccl(comm* c, const ncclUniqueId& uid, int nranks, int rank, const char* what) {
    HIP_CHECK(hipSetDevice(c->device));
    ncclResult_t r = ncclCommInitRank(&c->nccl, nranks, uid, rank);
    if (r != ncclSuccess) {
        delete c;
        throw error(COSTA_ERR_NCCL, std::string(what) + ": " + ncclGetErrorString(r));
    }
}
}  // namespace

comm* comm_self(int device) {
    comm* c = new_comm(device);
    if (loopback_exchange()) {  // test mode: a real one-rank RCCL communicator
        ncclUniqueId uid;
        NCCL_CHECK(ncclGetUniqueId(&uid));
        init_nccl(c, uid, 1, 0, "loopback ncclCommInitRank");
    }
    return c;
}

comm* comm_create(const unsigned char* id, int nranks, int rank, int device) {
    if (nranks < 1 || rank < 0 || rank >= nranks) throw error(COSTA_ERR_ARG, "costa: bad rank/size");
    if (nranks == 1) return comm_self(device);
    comm* c = new_comm(device);
    c->rank = rank;
    c->size = nranks;
    ncclUniqueId uid;
    std::memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
    init_nccl(c, uid, nranks, rank, "ncclCommInitRank");
    return c;
}

const char* tuning_env(const char* name) {
    static const bool on = [] {
        const char* s = std::getenv("COSTA_TUNING");
        return s && std::atoi(s) == 1;
    }();
    return on ? std::getenv(name) : nullptr;
}

int loopback_exchange() {
    static const int mode = [] {
        const char* s = std::getenv("COSTA_LOOPBACK");
        const int m = s ? std::atoi(s) : 0;
        return m == 1 || m == 2 ? m : 0;
    }();
    return mode;
}

// Largest ncclSend / ncclRecv: 256 MiB by default (override COSTA_MAX_MSG_BYTES), never more
// than kMaxMessageCap.  A single self send/recv above 2^30 bytes delivered only its first half
// (the failure starts where twice the byte count passes INT32_MAX, and the lost
// part is exactly the second of two halves); the last size measured intact was 2^30 - 233472
// bytes, so the cap stays 1 MiB below 2^30 (exactly 2^30 is already on the failing side of
// 2 * count > INT32_MAX).  tests/test_gpu_rccl_system.py moves a package in pieces of the cap.
constexpr size_t kMaxMessageCap = (size_t(1) << 30) - (size_t(1) << 20);
size_t max_message_bytes() {
    static const size_t v = [] {
        const char* s = std::getenv("COSTA_MAX_MSG_BYTES");  // tuning override
        const long long x = s ? std::atoll(s) : 0;
        const size_t want = x > 0 ? size_t(x) : (size_t(1) << 28);
        return std::min(want, kMaxMessageCap);
    }();
    return v;
}

// Exchange rounds: a peer's package of at least kRoundMinBytes moves in exchange_rounds() equal
// parts, each its own RCCL group on the exchange stream, so that packing part r+1, moving part
// r and unpacking part r-1 overlap.  Both sides of a pair derive the parts from the pair's
// element count alone, so they agree on every message.
constexpr size_t kRoundMinBytes = size_t(16) << 20;
int exchange_rounds() {
    static const int v = [] {
        const char* s = std::getenv("COSTA_EXCHANGE_ROUNDS");  // tuning / reproduction override
        const int x = s ? std::atoi(s) : 4;
        return std::max(1, std::min(16, x));
    }();
    return v;
}

namespace {
int parts_of(int64_t n, size_t E, int R) { return size_t(n) * E >= kRoundMinBytes ? R : 1; }
// element range [lo, hi) of round r of a package of n elements (empty past its parts)
void round_range(int64_t n, size_t E, int R, int r, int64_t& lo, int64_t& hi) {
    const int parts = parts_of(n, E, R);
    if (r >= parts) {
        lo = hi = n;
        return;
    }
    lo = n * r / parts;
    hi = n * (r + 1) / parts;
}
// round holding element o (0 <= o < n) of a package of n elements
int round_of(int64_t o, int64_t n, size_t E, int R) {
    const int parts = parts_of(n, E, R);
    int r = int(o * parts / n);
    while (r > 0 && o < n * r / parts) --r;
    while (r + 1 < parts && o >= n * (r + 1) / parts) ++r;
    return r;
}
// the peer whose package holds element o of a buffer laid out by displs / counts
size_t peer_of(const std::vector<int64_t>& displs, int64_t o) {
    const auto it = std::upper_bound(displs.begin(), displs.end(), o);
    return size_t(it - displs.begin()) - 1;
}
}  // namespace

void exchange_round_of_ops(const plan& p, int rounds, std::vector<int>& pack_round,
                           std::vector<int>& unpack_round) {
    const size_t E = dtype_size(p.dtype);
    pack_round.clear();
    unpack_round.clear();
    for (const auto& op : p.pack_ops) {
        const int64_t o = int64_t(op.dst / E);
        const size_t q = peer_of(p.send_displs, o);
        pack_round.push_back(round_of(o - p.send_displs[q], p.send_counts[q], E, rounds));
    }
    for (const auto& op : p.unpack_ops) {
        const int64_t first = int64_t(op.src / E);
        const int64_t last = first + int64_t(op.nf) * op.ns - 1;
        const size_t q = peer_of(p.recv_displs, first);
        unpack_round.push_back(round_of(last - p.recv_displs[q], p.recv_counts[q], E, rounds));
    }
}

int comm_rank(const comm* c) { return c->rank; }
int comm_size(const comm* c) { return c->size; }
void comm_destroy(comm* c) { delete c; }

void comm_unique_id(unsigned char* out) {
    ncclUniqueId uid;
    NCCL_CHECK(ncclGetUniqueId(&uid));
    std::memcpy(out, uid.internal, NCCL_UNIQUE_ID_BYTES);
}

// ---------------------------------------------------------------- work lists
bool any_transpose(const std::vector<costa_tile_op_t>& ops) {
    for (const auto& op : ops)
        if (op.flags & COSTA_TILE_TRANSPOSE) return true;
    return false;
}

bool any_axpby(const std::vector<costa_tile_op_t>& ops) {
    for (const auto& op : ops)
        if (((op.flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT) == COSTA_SCALE_AXPBY) return true;
    return false;
}

// Work classes.  An op goes to the large shape (a 1024-thread workgroup per sub-tile) when it
// holds at least half a large sub-tile of data; every other op runs on the wavefront path
// (tiny_kernel): ops over a wavefront's budget are first cut, here on the host, into
// rectangular sub-ops within it (a sub-rectangle of a tile op is a tile op).  Budgets: copy
// mode one wavefront pass of data (tiny_copy_budget), transpose mode tiny_lds_budget() of staged
// tile (row pitch nf | 1).
// Copy mode: a part of one wavefront pass (64 lanes x tiny_copy_lane_bytes), an op the wavefront
// moves in one round trip, cut finer for more wavefronts in flight.  Local lists: half (2 KiB);
// r3 with the XCD column bands, cfg 5 'N' 0.434-0.436 ms at 2 KiB against 0.446-0.447 at 3 KiB,
// 0.438 at 2.5, 0.449-0.451 at 1.5, 0.466 at 4, 0.517 at 1 (profiles/r3b/README.md §copy_budget).  Pack
// and unpack lists (one side the dense package): three quarters (3 KiB); through the loopback
// exchange pack 'N' 0.587-0.590 ms against 0.607-0.608 at 2 KiB, unpack 0.592-0.597 against
// 0.607-0.608 (profiles/r3b/README.md §copy_budget; r11: 3 KiB best for every list,
// profiles/r11/c5_budget_uc64.log).
// (COSTA_TINY_COPY: another budget in bytes up to kTinyCopyBytes, tuning runs only)
int64_t tiny_copy_budget(int64_t E, bool local) {
    static const int64_t env = [] {
        const char* s = tuning_env("COSTA_TINY_COPY");
        const int64_t v = s ? std::atoll(s) : 0;
        return v >= 256 && v <= kTinyCopyBytes ? v : int64_t(0);
    }();
    return env ? env : (local ? 32 : 48) * int64_t(tiny_copy_lane_bytes(size_t(E)));
}

// Transpose mode: the staged tile, kTinyLdsDefault bytes of LDS per wavefront
// (COSTA_TINY_LDS: another budget up to kTinyLdsBytes, tuning runs only)
int64_t tiny_lds_budget() {
    static const int64_t b = [] {
        const char* s = tuning_env("COSTA_TINY_LDS");
        const int64_t v = s ? std::atoll(s) : 0;
        return v >= 256 && v <= kTinyLdsBytes ? v : int64_t(kTinyLdsDefault);
    }();
    return b;
}

static bool is_tiny(const costa_tile_op_t& op, int64_t E, bool local) {
    if (op.flags & COSTA_TILE_TRANSPOSE) return int64_t(op.nf | 1) * op.ns * E <= tiny_lds_budget();
    return int64_t(op.nf) * op.ns * E <= tiny_copy_budget(E, local);
}

static uint32_t vec_flags(uint64_t src, int64_t lds, uint64_t dst, int64_t ldd, int64_t E) {
    uint32_t f = 0;
    if (src % 16 == 0 && (lds * E) % 16 == 0) f |= COSTA_TILE_VEC_SRC;
    if (dst % 16 == 0 && (ldd * E) % 16 == 0) f |= COSTA_TILE_VEC_DST;
    return f;
}

// cut `op` into near-equal rectangles that each fit the wavefront budget: the grid of pieces
// (nfc x nsc pieces of cf x cs elements at most), then the pieces themselves
namespace {
struct wave_grid {
    int64_t nfc = 1, nsc = 1;
};
wave_grid wave_pieces(const costa_tile_op_t& op, int64_t E, bool local) {
    wave_grid g;
    if (is_tiny(op, E, local)) return g;
    const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
    const int64_t budget = (tr ? tiny_lds_budget() : tiny_copy_budget(E, local)) / E;  // elements
    const int64_t nf = op.nf, ns = op.ns;
    // transpose: pieces at most 16 elements wide along f (the source's contiguous dimension),
    // as tall along s as the budget allows: the destination runs (which a beta != 0 op both reads
    // and writes) stay long.  cfg 5 'T' 0.726 ms with near-square pieces (32 wide), 0.716 with 16,
    // 0.728 with 12, 0.758 with 8, 0.754 cut along s first; fp64 / c64 / c128 pack and unpack
    // lists equal at 16 (profiles/r3b/README.md §side).  Copy: whole columns when one fits, else tall pieces
    static const int64_t side_env = [] {  // COSTA_TR_SIDE (tuning): the cut's side along f
        const char* v = tuning_env("COSTA_TR_SIDE");
        return v ? std::max<int64_t>(1, std::atoll(v)) : int64_t(0);
    }();
    const int64_t sq_side = std::max<int64_t>(1, int64_t(std::sqrt(double(budget))));
    const int64_t side = tr ? (side_env ? side_env : std::min<int64_t>(16, sq_side)) : budget;
    g.nfc = (nf + side - 1) / side;
    const int64_t cf = (nf + g.nfc - 1) / g.nfc;
    const int64_t cs_max = std::max<int64_t>(1, budget / (tr ? (cf | 1) : cf));
    g.nsc = (ns + cs_max - 1) / cs_max;
    return g;
}
// writes the g.nfc * g.nsc pieces of `op` at `out`
void emit_pieces(const costa_tile_op_t& op, int64_t E, const wave_grid& g, bool local, costa_tile_op_t* out) {
    if (g.nfc == 1 && g.nsc == 1) {
        *out = op;
        return;
    }
    const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
    const int64_t nf = op.nf, ns = op.ns;
    const uint32_t keep = op.flags & ~uint32_t(COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST);
    for (int64_t i = 0; i < g.nfc; ++i) {
        const int64_t f0 = i * nf / g.nfc, f1 = (i + 1) * nf / g.nfc;
        for (int64_t j = 0; j < g.nsc; ++j) {
            const int64_t s0 = j * ns / g.nsc, s1 = (j + 1) * ns / g.nsc;
            costa_tile_op_t sub = op;
            sub.src = op.src + uint64_t((s0 * op.lds + f0) * E);
            sub.dst = op.dst + uint64_t((tr ? f0 * op.ldd + s0 : s0 * op.ldd + f0) * E);
            sub.nf = int32_t(f1 - f0);
            sub.ns = int32_t(s1 - s0);
            sub.flags = keep | vec_flags(sub.src, op.lds, sub.dst, op.ldd, E);
            if (!is_tiny(sub, E, local)) throw error(COSTA_ERR_INTERNAL, "costa: wave split over budget");
            *out++ = sub;
        }
    }
}

// XCD column bands (wave_knobs::xcd_bands): the tiny kernel gives XCD x the x-th eighth of
// the list; destination order alone makes that eighth a run of whole target block-rows, so an A
// cache line shared by the tiles above and below a block-row boundary is fetched again one
// block-row of the XCD's traffic later (~11 MB for cfg 5: past its 4 MB L2).  Here the list is
// first split into eight bands of target columns (by the planner's column-major hint, equal piece
// counts), each band in destination order: every XCD walks all block-rows of its own columns, and
// the two tiles sharing the line run ~1/8 of a block-row apart on the same XCD.
void xcd_bands(const std::vector<const costa_tile_op_t*>& ops, int64_t E, int k, bool local,
               std::vector<uint32_t>& perm) {
    const uint64_t nb = 8 * uint64_t(k);  // bands: XCD x walks bands k x .. k x + k - 1 in turn
    const size_t n = perm.size();
    std::vector<uint64_t> pieces(n);
    uint64_t total = 0;
    for (size_t i = 0; i < n; ++i) {
        const wave_grid g = wave_pieces(*ops[i], E, local);
        pieces[i] = uint64_t(g.nfc * g.nsc);
        total += pieces[i];
    }
    std::vector<uint32_t> by_hint(n);
    for (size_t i = 0; i < n; ++i) by_hint[i] = uint32_t(i);
    std::stable_sort(by_hint.begin(), by_hint.end(),
                     [&](uint32_t x, uint32_t y) { return ops[x]->order < ops[y]->order; });
    std::vector<uint32_t> band(n);
    uint64_t cum = 0;
    for (const uint32_t i : by_hint) {
        band[i] = uint32_t(std::min<uint64_t>(nb - 1, cum * nb / std::max<uint64_t>(total, 1)));
        cum += pieces[i];
    }
    std::stable_sort(perm.begin(), perm.end(), [&](uint32_t x, uint32_t y) { return band[x] < band[y]; });
}

// (key, item) pairs whose items ascend in list order, sorted by key with equal keys in item
// order -- what std::sort of the pairs gives -- by a stable LSD radix sort of 16-bit digits over
// the keys' span (cfg 4's 262 k sub-tiles: a comparison sort cost ~7 ms of a plan-cache miss)
void sort_pairs_by_key(std::vector<std::pair<uint64_t, uint64_t>>& kv) {
    const size_t n = kv.size();
    if (n < 2) return;
    uint64_t lo = ~uint64_t(0), hi = 0;
    for (const auto& p : kv) lo = std::min(lo, p.first), hi = std::max(hi, p.first);
    std::vector<std::pair<uint64_t, uint64_t>> tmp(n);
    std::vector<uint32_t> at((size_t(1) << 16) + 1);
    const uint64_t span = hi - lo;
    for (int sh = 0; sh == 0 || (sh < 64 && (span >> sh) != 0); sh += 16) {
        std::fill(at.begin(), at.end(), 0u);
        for (const auto& p : kv) ++at[(((p.first - lo) >> sh) & 0xFFFFu) + 1];
        for (size_t d = 1; d < at.size(); ++d) at[d] += at[d - 1];
        for (const auto& p : kv) tmp[at[((p.first - lo) >> sh) & 0xFFFFu]++] = p;
        kv.swap(tmp);
    }
}

// Merges ops that continue each other: the op whose source starts where op a's source ends along
// s (a.src + a.ns * lds) and whose destination continues a's the same way (one destination
// stride further for copies, ns elements further for transposes), with the same extent along f,
// strides and flags (16-byte alignment flags aside: the merged op keeps a's, which describe its
// start and strides), joins a (then the same along f).  Same elements, same transform: only the
// op boundaries move.  Order hint: a's (the tile the merged op starts at).  `root` (optional): for every input op, the
// input op it ended up merged into (itself when it survives).
void merge_adjacent(std::vector<costa_tile_op_t>& v, int64_t E, std::vector<uint32_t>* root = nullptr) {
    std::vector<uint32_t> id(v.size());  // input index of each op of v
    for (size_t i = 0; i < v.size(); ++i) id[i] = uint32_t(i);
    if (root) {
        root->resize(v.size());
        for (size_t i = 0; i < v.size(); ++i) (*root)[i] = uint32_t(i);
    }
    if (v.size() < 2) return;
    for (int pass = 0; pass < 2; ++pass) {  // 0: along s, 1: along f
        // the ops in source order (a radix sort of (src, index)), and an open-addressing table
        // src -> the first op of that source address (std::unordered_map and std::sort cost cfg 3 /
        // cfg 4's 65 k-op lists ~5 ms of a plan-cache miss)
        std::vector<std::pair<uint64_t, uint64_t>> kv(v.size());
        for (size_t i = 0; i < v.size(); ++i) kv[i] = {v[i].src, i};
        sort_pairs_by_key(kv);
        std::vector<uint32_t> idx(v.size());
        for (size_t k = 0; k < v.size(); ++k) idx[k] = uint32_t(kv[k].second);
        int tb = 4;
        while ((size_t(1) << tb) < 2 * v.size()) ++tb;
        const size_t tmask = (size_t(1) << tb) - 1;
        std::vector<std::pair<uint64_t, uint32_t>> table(tmask + 1, {~uint64_t(0), 0u});
        auto slot_of = [&](uint64_t a) { return size_t((a * 0x9E3779B97F4A7C15ull) >> (64 - tb)); };
        for (size_t i = 0; i < v.size(); ++i) {  // ascending index: the first op of a src stays
            size_t h = slot_of(v[i].src);
            while (table[h].first != ~uint64_t(0) && table[h].first != v[i].src) h = (h + 1) & tmask;
            if (table[h].first == ~uint64_t(0)) table[h] = {v[i].src, uint32_t(i)};
        }
        auto find_src = [&](uint64_t a) -> int64_t {  // the first op at source address a, or -1
            for (size_t h = slot_of(a);; h = (h + 1) & tmask) {
                if (table[h].first == a) return int64_t(table[h].second);
                if (table[h].first == ~uint64_t(0)) return -1;
            }
        };
        std::vector<char> gone(v.size(), 0);
        for (const uint32_t i : idx) {
            if (gone[i]) continue;
            costa_tile_op_t& a = v[i];
            const bool tr = a.flags & COSTA_TILE_TRANSPOSE;
            for (;;) {
                const int64_t n = pass == 0 ? a.ns : a.nf;
                const uint64_t next_src = a.src + uint64_t(pass == 0 ? n * a.lds * E : n * E);
                const uint64_t next_dst =
                    a.dst + uint64_t(pass == 0 ? (tr ? n : n * a.ldd) * E : (tr ? n * a.ldd : n) * E);
                const int64_t nx = find_src(next_src);
                if (nx < 0 || gone[nx] || uint32_t(nx) == i) break;
                const costa_tile_op_t& b = v[size_t(nx)];
                const uint32_t vec = COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST;
                const bool same = b.dst == next_dst && (b.flags & ~vec) == (a.flags & ~vec) && b.lds == a.lds &&
                                  b.ldd == a.ldd && (pass == 0 ? b.nf == a.nf : b.ns == a.ns);
                const int64_t total = n + (pass == 0 ? b.ns : b.nf);
                if (!same || total > (int64_t(1) << 30)) break;
                (pass == 0 ? a.ns : a.nf) = int32_t(total);
                if (!a.order) a.order = b.order;  // the merged op keeps the hint of its first tile
                gone[nx] = 1;
                if (root) (*root)[id[nx]] = id[i];
            }
        }
        size_t o = 0;
        for (size_t i = 0; i < v.size(); ++i)
            if (!gone[i]) {
                id[o] = id[i];
                v[o++] = v[i];
            }
        v.resize(o);
        id.resize(o);
    }
    if (root)  // path compression: pass 1 merged pass-0 survivors
        for (size_t i = 0; i < root->size(); ++i) {
            uint32_t r = (*root)[i];
            while ((*root)[r] != r) r = (*root)[r];
            (*root)[i] = r;
        }
}

// Ops of a list merged (merge_adjacent), keeping a merged op only when it fills the large
// shape's sub-tiles at least half along each dimension (bf x bs): a strip of one block's width
// (nf = 24 of a 64-wide sub-tile, say, a package's tiles continuing along s) would run the large
// shape a third full, slower than its tiles on the wavefront path (loopback unpack fp64 24^2
// beta != 0: 1.571 against 1.412 ms); its tiles stay apart instead.
std::vector<costa_tile_op_t> merge_filled(const std::vector<costa_tile_op_t>& cand, int64_t E, int bf, int bs) {
    std::vector<costa_tile_op_t> v = cand;
    std::vector<uint32_t> root;
    merge_adjacent(v, E, &root);
    if (v.size() == cand.size()) return v;
    std::vector<costa_tile_op_t> out;
    out.reserve(cand.size());
    std::vector<char> keep(cand.size(), 0);  // per root: the merged op is kept
    std::vector<uint32_t> count(cand.size(), 0);
    for (size_t i = 0; i < cand.size(); ++i) ++count[root[i]];
    // v holds the surviving ops in input order, i.e. in the order of their roots
    size_t k = 0;
    for (size_t i = 0; i < cand.size(); ++i) {
        if (root[i] != i) continue;
        const costa_tile_op_t& m = v[k++];
        keep[i] = count[i] == 1 || (2 * int64_t(m.nf) >= bf && 2 * int64_t(m.ns) >= bs);
        if (keep[i]) out.push_back(m);
    }
    for (size_t i = 0; i < cand.size(); ++i)
        if (!keep[root[i]]) out.push_back(cand[i]);
    return out;
}

// Only ops with equal strides can continue each other: block-cyclic layouts have one stride per
// local matrix, while a custom layout whose blocks are separate buffers has one per block (cfg 5:
// hundreds), whose tiles practically never continue across blocks.  Lists with more than 16
// distinct source strides skip the merge (cfg 5's 245 k ops: the merge pass cost 2x build_work).
bool few_strides(const std::vector<costa_tile_op_t>& ops) {
    int32_t seen[16];
    int k = 0;
    for (const auto& o : ops) {
        bool found = false;
        for (int i = 0; i < k && !found; ++i) found = seen[i] == o.lds;
        if (found) continue;
        if (k == 16) return false;
        seen[k++] = o.lds;
    }
    return true;
}

// runs fn(begin, end) over [0, n) on up to 8 host threads (one when n < min_items)
template <typename F>
void host_parallel(size_t n, F fn, size_t min_items = 32768) {
    const size_t hw = std::max(1u, std::thread::hardware_concurrency());
    const size_t T = n < min_items ? 1 : std::min<size_t>(8, hw);
    if (T == 1) return fn(size_t(0), n);
    std::vector<std::thread> th;
    std::vector<std::exception_ptr> err(T);
    for (size_t t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            try {
                fn(n * t / T, n * (t + 1) / T);
            } catch (...) {
                err[t] = std::current_exception();
            }
        });
    for (auto& x : th) x.join();
    for (auto& e : err)
        if (e) std::rethrow_exception(e);
}
}  // namespace

namespace {
// Destination-block groups (r5, tile_kernels.hip cblock_kernel).  Among the ops bound for the
// wavefront path, those whose destination footprints (same leading dimension R) overlap or touch
// form components; a component whose ops tile R x K elements exactly -- whole columns of a
// buffer whose leading dimension is R: a custom layout's own block buffer (cfg 5), or several of
// them back to back -- is one contiguous destination range, written by one workgroup in 16-byte
// vectors instead of one element a lane per wavefront piece.  Components above the workgroup's
// budget (cblock_max_elems) are cut into column bands, their ops cut at the band edges (a
// sub-rectangle of a tile op is a tile op).  Ops of a component must share one transform (flags
// apart from the vector bits).  Emitted into `ordered` as [header, ops...] per group (header: src
// = number of ops, dst = the range, nf = R, ns = K, flags = the transform); `work` gets the
// header indices in destination order; the grouped ops leave `wave_ops`.  COSTA_CBLOCK=0
// (tuning): off.
// the destination-block groups apply to this list (cblock_groups' own conditions, apart from the
// list's length)
bool cblock_enabled(costa_dtype_t dtype, list_kind kind) {
    static const int on = [] {
        const char* s = tuning_env("COSTA_CBLOCK");
        return s ? std::atoi(s) : 1;
    }();
    const bool real = dtype == COSTA_FLOAT || dtype == COSTA_DOUBLE || dtype == COSTA_INT32;
    return on && real && kind != list_pack;
}

int64_t cblock_groups(costa_dtype_t dtype, std::vector<const costa_tile_op_t*>& wave_ops, list_kind kind,
                      std::vector<costa_tile_op_t>& ordered, std::vector<uint64_t>& work, int64_t& lds,
                      int& map, const std::vector<costa_tile_op_t>& ops, device_section* dev) {
    static const int on = [] {
        const char* s = tuning_env("COSTA_CBLOCK");
        return s ? std::atoi(s) : 1;
    }();
    // COSTA_CB_BANDS (tuning): 1 XCD column bands for every list, 0 never, -1 (default) as below
    static const int bands_env = [] {
        const char* s = tuning_env("COSTA_CB_BANDS");
        return s ? std::atoi(s) : -1;
    }();
    lds = 0;
    map = cb_round_robin;
    // COSTA_PLAN_TRACE=1: the phases of the group builder (stderr)
    static const bool trace = std::getenv("COSTA_PLAN_TRACE") != nullptr;
    const auto t0 = std::chrono::steady_clock::now();
    double lap_ms[7] = {0, 0, 0, 0, 0, 0, 0};  // candidates, sort, components, check, groups, order, emit
    auto lap = [&](int k) {
        if (trace) lap_ms[k] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    };
    // real types (complex elements are on the large shapes wherever it matters: cfg 4)
    const bool real = dtype == COSTA_FLOAT || dtype == COSTA_DOUBLE || dtype == COSTA_INT32;
    if (!on || !real || kind == list_pack || wave_ops.size() < 2) return 0;
    const int64_t E = int64_t(dtype_size(dtype));
    const uint32_t vec_bits = COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST;
    // a range of n elements starting off the 16-byte grid spans up to n + V - 1 elements of
    // whole vectors: the workgroup's kCblockChunks vectors a thread must cover that
    const int64_t budget = cblock_max_elems(E) - (16 / E - 1);
    // on the GPU (device_lists.hip) for long lists: the same groups, order and bytes
    const int lb_mode = list_builder_mode();
    if (dev && dev->device >= 0 && (dev->force || lb_mode == 2 || (lb_mode == 1 && wave_ops.size() >= kDeviceGroupsMin))) {
        std::vector<uint32_t> wave(wave_ops.size());
        for (size_t i = 0; i < wave_ops.size(); ++i) wave[i] = uint32_t(wave_ops[i] - ops.data());
        std::vector<char> taken;
        const int64_t ng = cblock_groups_device(E, budget, vec_bits, bands_env, ops, wave, ordered.size(), *dev,
                                                taken, lds, map);
        if (ng >= 0) {
            if (ng > 0) {
                dev->at_work = work.size();
                size_t o = 0;
                for (size_t i = 0; i < wave_ops.size(); ++i)
                    if (!taken[i]) wave_ops[o++] = wave_ops[i];
                wave_ops.resize(o);
                g_stats.device_lists++;
            }
            if (trace)
                std::fprintf(stderr, "[costa groups] %lld groups built on the GPU in %.2f ms\n", (long long)ng,
                             std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
            return ng;
        }
    }
    struct cand {
        uint64_t lo, hi;
        int32_t ldd;
        uint32_t i;
    };
    std::vector<cand> cs;
    cs.reserve(wave_ops.size());
    for (uint32_t i = 0; i < wave_ops.size(); ++i) {
        const costa_tile_op_t& op = *wave_ops[i];
        if (op.nf <= 0 || op.ns <= 0 || op.ldd <= 0 || op.dst % uint64_t(E) != 0) continue;
        const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
        const int64_t run = tr ? op.ns : op.nf, runs = tr ? op.nf : op.ns;
        if (run > op.ldd || op.ldd > budget) continue;
        cs.push_back({op.dst, op.dst + uint64_t(((runs - 1) * int64_t(op.ldd) + run) * E), op.ldd, i});
    }
    if (cs.size() < 2) return 0;
    lap(0);
    // order by (ldd, lo): stable LSD radix sorts, lo (element offsets from the lowest) first, then
    // ldd (<= budget); a comparison sort of cfg 5's 245 k candidates cost ~10 ms of a plan miss
    {
        uint64_t lo_min = ~uint64_t(0), lo_max = 0;
        for (const auto& c : cs) lo_min = std::min(lo_min, c.lo), lo_max = std::max(lo_max, c.lo);
        std::vector<cand> tmp(cs.size());
        constexpr int B = 16;  // 2 passes for cfg 5's 1 GiB arena, 1 for the leading dimensions
        std::vector<uint32_t> at((size_t(1) << B) + 1);
        auto pass = [&](auto digit) {
            std::fill(at.begin(), at.end(), 0u);
            for (const auto& c : cs) ++at[digit(c) + 1];
            for (size_t d = 1; d < at.size(); ++d) at[d] += at[d - 1];
            for (const auto& c : cs) tmp[at[digit(c)]++] = c;
            cs.swap(tmp);
        };
        const uint64_t span = (lo_max - lo_min) / uint64_t(E);
        for (int sh = 0; sh == 0 || (sh < 64 && (span >> sh) != 0); sh += B)
            pass([&](const cand& c) { return size_t(((c.lo - lo_min) / uint64_t(E) >> sh) & ((1u << B) - 1)); });
        for (int sh = 0; sh == 0 || (sh < 31 && (uint64_t(budget) >> sh) != 0); sh += B)
            pass([&](const cand& c) { return size_t((uint32_t(c.ldd) >> sh) & ((1u << B) - 1)); });
    }
    lap(1);
    // components: runs of candidates (one leading dimension) whose footprints overlap or touch
    struct comp {
        size_t a, b;
    };
    std::vector<comp> comps;
    for (size_t a = 0; a < cs.size();) {
        size_t b = a + 1;
        uint64_t hi = cs[a].hi;
        while (b < cs.size() && cs[b].ldd == cs[a].ldd && cs[b].lo <= hi) hi = std::max(hi, cs[b].hi), ++b;
        if (b - a >= 2) comps.push_back({a, b});
        a = b;
    }
    lap(2);
    // per component (host threads): does it tile its R x K range exactly, and how many groups
    // (column bands of at most `budget` elements) it makes
    struct cinfo {
        int64_t K = 0, KB = 0;
        uint64_t n_groups = 0;
        uint32_t fl = 0;
    };
    std::vector<cinfo> ci(comps.size());
    // (gathering the candidates' ops into sorted order first made the passes below no faster on
    // the box: tiling check + group table + emission 16.5 against 12.4 ms, profiles/r6g/)
    auto op_of = [&](size_t k) -> const costa_tile_op_t& { return *wave_ops[cs[k].i]; };
    host_parallel(comps.size(), [&](size_t x0, size_t x1) {
        std::vector<uint64_t> corner;
        for (size_t x = x0; x < x1; ++x) {
            const size_t a0 = comps[x].a, b = comps[x].b;
            const int64_t R = cs[a0].ldd;
            const uint64_t base = cs[a0].lo;
            const uint32_t fl = op_of(a0).flags & ~vec_bits;
            int64_t area = 0, K = 0;
            bool ok = true;
            for (size_t k = a0; k < b && ok; ++k) {
                const costa_tile_op_t& op = op_of(k);
                const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
                const int64_t run = tr ? op.ns : op.nf, runs = tr ? op.nf : op.ns;
                const int64_t e = int64_t(op.dst - base) / E;
                ok = (op.flags & ~vec_bits) == fl && e % R + run <= R;
                area += run * runs;
                K = std::max(K, e / R + runs);
            }
            if (!ok || area != R * K || K > INT32_MAX) continue;
            // ... and tile it exactly: with the areas adding up to R x K, the ops tile the range
            // iff every corner point occurs an even number of times, the range's own four corners
            // apart, which occur once ("perfect rectangle").  Overlapping ops whose areas happen to
            // add up would leave elements no op writes, and the group kernel would store its
            // uninitialised LDS there (costa_hip_execute_tiles takes caller ops).
            corner.clear();
            const uint64_t W = uint64_t(K) + 1;
            for (size_t k = a0; k < b; ++k) {
                const costa_tile_op_t& op = op_of(k);
                const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
                const uint64_t run = uint64_t(tr ? op.ns : op.nf), runs = uint64_t(tr ? op.nf : op.ns);
                const uint64_t e = (op.dst - base) / uint64_t(E), r0 = e % uint64_t(R), c0 = e / uint64_t(R);
                for (const uint64_t r : {r0, r0 + run})
                    for (const uint64_t c : {c0, c0 + runs}) corner.push_back(r * W + c);
            }
            std::sort(corner.begin(), corner.end());
            const uint64_t ur = uint64_t(R), uk = uint64_t(K), want[4] = {0, uk, ur * W, ur * W + uk};
            int n_odd = 0;
            for (size_t k = 0; k < corner.size() && ok;) {
                size_t m = k;
                while (m < corner.size() && corner[m] == corner[k]) ++m;
                if ((m - k) & 1) ok = n_odd < 4 && corner[k] == want[n_odd++];
                k = m;
            }
            if (!ok || n_odd != 4) continue;
            const int64_t KB = std::max<int64_t>(1, budget / R);
            ci[x] = {K, KB, uint64_t((K + KB - 1) / KB), fl};
        }
    }, 4096);
    lap(3);
    std::vector<uint64_t> g_at(comps.size() + 1, 0);
    for (size_t x = 0; x < comps.size(); ++x) g_at[x + 1] = g_at[x] + ci[x].n_groups;
    const size_t ng = size_t(g_at.back());
    if (ng == 0) return 0;
    // per group (host threads): its range, its op count (an op cut at the band edges counts once
    // per band), the smallest locality hint of its ops (0: one lacks a hint)
    struct group {
        uint64_t dst;
        uint32_t comp, band, n_ops, hint;
    };
    std::vector<group> gs(ng);
    std::vector<char> taken(wave_ops.size(), 0);
    auto band_cols = [&](size_t x, uint32_t band, int64_t& cb0, int64_t& cb1) {
        cb0 = int64_t(band) * ci[x].KB;
        cb1 = std::min(ci[x].K, cb0 + ci[x].KB);
    };
    host_parallel(comps.size(), [&](size_t x0, size_t x1) {
        for (size_t x = x0; x < x1; ++x) {
            if (ci[x].n_groups == 0) continue;
            const size_t a0 = comps[x].a, b = comps[x].b;
            const int64_t R = cs[a0].ldd;
            const uint64_t base = cs[a0].lo;
            for (uint32_t band = 0; band < ci[x].n_groups; ++band) {
                int64_t cb0, cb1;
                band_cols(x, band, cb0, cb1);
                group& g = gs[size_t(g_at[x]) + band];
                g = {base + uint64_t(cb0 * R * E), uint32_t(x), band, 0, UINT32_MAX};
                for (size_t k = a0; k < b; ++k) {
                    const costa_tile_op_t& op = op_of(k);
                    const int64_t c0 = int64_t(op.dst - base) / E / R;
                    const int64_t runs = (op.flags & COSTA_TILE_TRANSPOSE) ? op.nf : op.ns;
                    if (std::max(cb0, c0) >= std::min(cb1, c0 + runs)) continue;
                    ++g.n_ops;
                    g.hint = op.order ? std::min(g.hint, op.order) : 0;
                }
            }
        }
    }, 4096);
    // (one thread: the grouped ops are scattered over the list, and threads marking them shared
    // cache lines)
    for (size_t x = 0; x < comps.size(); ++x)
        if (ci[x].n_groups)
            for (size_t k = comps[x].a; k < comps[x].b; ++k) taken[cs[k].i] = 1;
    lap(4);
    // destination order: a stable radix sort of the groups by range offset
    std::vector<uint32_t> order(ng);
    {
        uint64_t lo = ~uint64_t(0), hi = 0;
        for (const auto& g : gs) lo = std::min(lo, g.dst), hi = std::max(hi, g.dst);
        std::vector<uint32_t> tmp(ng);
        for (size_t g = 0; g < ng; ++g) order[g] = uint32_t(g);
        constexpr int B = 16;
        std::vector<uint32_t> at((size_t(1) << B) + 1);
        const uint64_t span = (hi - lo) / uint64_t(E);
        for (int sh = 0; sh == 0 || (sh < 64 && (span >> sh) != 0); sh += B) {
            auto digit = [&](uint32_t g) { return size_t(((gs[g].dst - lo) / uint64_t(E) >> sh) & ((1u << B) - 1)); };
            std::fill(at.begin(), at.end(), 0u);
            for (const uint32_t g : order) ++at[digit(g) + 1];
            for (size_t d = 1; d < at.size(); ++d) at[d] += at[d - 1];
            for (const uint32_t g : order) tmp[at[digit(g)]++] = g;
            order.swap(tmp);
        }
    }
    bool any_tr = false;
    for (const auto& g : gs) any_tr = any_tr || (ci[g.comp].fl & COSTA_TILE_TRANSPOSE);
    map = any_tr ? cb_xcd_chunks : cb_round_robin;
    bool hints = true;
    for (const auto& g : gs) hints = hints && g.hint != 0 && g.hint != UINT32_MAX;
    // XCD column bands for copy-only lists (r6, COSTA_CB_BANDS=0 / 1 (tuning): never / always):
    // the groups in the planner's column-major order of their first target tile are cut into 8
    // slices of the kernel's sizes (xcd_slice_order), slice x -- one band of target columns --
    // walked by XCD x in destination order.  A source block split by a target block-row boundary
    // is then read by two groups of one XCD about 1/8 of a block-row of its traffic apart, while
    // the line they share is still in its L2: cfg 5 'N' reads 1.46x -> 1.03x their bytes, and
    // with the 16-byte chunk loads of copy groups 0.436 -> 0.427 ms (each alone: +1 %, +1 %;
    // profiles/r6c/, r6d/).  Transposing lists keep the 4-group XCD chunks ('T' 0.600 against
    // 0.619 ms with bands).
    const bool bands = bands_env == 1 || (bands_env == -1 && !any_tr);
    if (bands && ng >= 16 && hints) {
        // (stable counting sorts: by hint, 2 x 16-bit digits; then the slices, 8 buckets)
        const size_t per = ng / 8, rem = ng % 8;
        std::vector<uint32_t> by(ng), tmp(ng), at16((size_t(1) << 16) + 1);
        for (size_t i = 0; i < ng; ++i) by[i] = uint32_t(i);
        for (int sh = 0; sh < 32; sh += 16) {
            std::fill(at16.begin(), at16.end(), 0u);
            for (const uint32_t g : by) ++at16[((gs[g].hint >> sh) & 0xFFFFu) + 1];
            for (size_t d = 1; d < at16.size(); ++d) at16[d] += at16[d - 1];
            for (const uint32_t g : by) tmp[at16[(gs[g].hint >> sh) & 0xFFFFu]++] = g;
            by.swap(tmp);
        }
        std::vector<uint8_t> band(ng);
        for (size_t k = 0; k < ng; ++k)
            band[by[k]] = uint8_t(k < rem * (per + 1) ? k / (per + 1) : rem + (k - rem * (per + 1)) / per);
        uint32_t at8[9] = {0};
        for (const uint32_t g : order) ++at8[band[g] + 1];
        for (int d = 1; d < 9; ++d) at8[d] += at8[d - 1];
        for (const uint32_t g : order) tmp[at8[band[g]]++] = g;
        order.swap(tmp);
        map = cb_xcd_bands;
    }
    lap(5);
    // [header, ops...] per group in that order, each op cut at its band's edges (a sub-rectangle
    // of a tile op is a tile op), written straight into their places (host threads)
    const size_t base_at = ordered.size();
    std::vector<uint64_t> at(ng + 1, 0);
    for (size_t q = 0; q < ng; ++q) at[q + 1] = at[q] + 1 + gs[order[q]].n_ops;
    size_t rest = 0;  // the remaining wavefront ops' pieces follow: room for most of them
    for (size_t i = 0; i < wave_ops.size(); ++i) rest += !taken[i];
    ordered.reserve(base_at + size_t(at[ng]) + 4 * rest + 1024);
    ordered.resize(base_at + size_t(at[ng]));
    work.reserve(work.size() + ng);
    for (size_t q = 0; q < ng; ++q) {
        work.push_back(uint64_t(base_at + at[q]));
        const group& g = gs[order[q]];
        int64_t cb0, cb1;
        band_cols(g.comp, g.band, cb0, cb1);
        lds = std::max(lds, int64_t(cs[comps[g.comp].a].ldd | 1) * (cb1 - cb0));
    }
    host_parallel(ng, [&](size_t q0, size_t q1) {
        for (size_t q = q0; q < q1; ++q) {
            const group& g = gs[order[q]];
            const size_t x = g.comp, a0 = comps[x].a, b = comps[x].b;
            const int64_t R = cs[a0].ldd;
            const uint64_t base = cs[a0].lo;
            int64_t cb0, cb1;
            band_cols(x, g.band, cb0, cb1);
            costa_tile_op_t* out = &ordered[base_at + size_t(at[q])];
            costa_tile_op_t h{};
            h.src = g.n_ops;
            h.dst = g.dst;
            h.nf = int32_t(R);
            h.ns = int32_t(cb1 - cb0);
            h.ldd = int32_t(R);
            h.flags = ci[x].fl;
            *out++ = h;
            for (size_t k = a0; k < b; ++k) {
                costa_tile_op_t op = op_of(k);
                const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
                const int64_t c0 = int64_t(op.dst - base) / E / R;
                const int64_t runs = tr ? op.nf : op.ns;
                const int64_t lo = std::max(cb0, c0), up = std::min(cb1, c0 + runs);
                if (lo >= up) continue;
                const int64_t d0 = lo - c0, dn = up - lo;  // destination columns of the op kept
                op.dst += uint64_t(d0 * R * E);
                if (tr) {  // destination columns = source f
                    op.src += uint64_t(d0 * E);
                    op.nf = int32_t(dn);
                } else {  // destination columns = source s
                    op.src += uint64_t(d0 * int64_t(op.lds) * E);
                    op.ns = int32_t(dn);
                }
                *out++ = op;
            }
        }
    }, 4096);
    size_t o = 0;
    for (size_t i = 0; i < wave_ops.size(); ++i)
        if (!taken[i]) wave_ops[o++] = wave_ops[i];
    wave_ops.resize(o);
    if (trace) {
        lap(6);
        std::fprintf(stderr,
                     "[costa groups] %zu candidates, %zu components, %zu groups: candidates %.2f ms, sort %.2f, "
                     "components %.2f, tiling check %.2f, group table %.2f, order %.2f, emit %.2f\n",
                     cs.size(), comps.size(), ng, lap_ms[0], lap_ms[1] - lap_ms[0], lap_ms[2] - lap_ms[1],
                     lap_ms[3] - lap_ms[2], lap_ms[4] - lap_ms[3], lap_ms[5] - lap_ms[4], lap_ms[6] - lap_ms[5]);
    }
    return int64_t(ng);
}

struct wave_knobs {  // defaults, overridable for tuning runs
    int policy = 2;  // COSTA_WAVE_POLICY 1: every op below the large threshold takes the wave
                     // path; 2: also large ops that are not 16-byte aligned on both sides, up to
                     // kUnalignedWaveCap large sub-tiles of data (r11: cfg 5 geometry with
                     // doubled edges 3.41 -> 4.14 TB/s 'N', 3.47 -> 3.88 'T', the rest
                     // unchanged; profiles/r11/c5_align_policy*.log).  Bigger unaligned ops stay
                     // on the large shape (its guarded path): cut into wavefront pieces, a
                     // 16384^2 fp32 op would become ~350 k pieces of host and device list.
    int skew_xcd = -1;   // COSTA_SKEW_XCD=F (tuning): F skew sub-tiles continuing each other's
                         // source rows on one XCD (one L2) at the same time; -1 (default):
                         // kSkewWideGroup for lists on the wide skew variant, else none
    int panel_rows = 0;  // COSTA_PANEL_ROWS (tuning): rows per destination panel of the
                         // destination-ordered sub-tiles; 0: 128 KiB of rows (default), -1: none
    int large_sort = 3;  // COSTA_LARGE_SORT 1: large ops in the order of the planner's locality
                         // hint (column-major target order: consecutive ops continue down the
                         // same target columns, so the write stream is sequential in aggregate);
                         // 0: list order (the reference's message order: target row-major, every
                         // op a new target column at the same in-column offset, which camps on
                         // HBM channels; tools/copy_ceiling.hip "pat ... ord-1" 6.27 against 5.64
                         // TB/s, "segcamp" 4.4-4.9 against 6.4); 2: 1, then the sub-tiles by
                         // the address of their first destination element (one sub-tile-wide
                         // band of target columns at a time, instead of an op's 2-4 sub-tiles
                         // side by side); 3 (default): 2 for lists whose shaped ops all transpose
                         // 4- or 8-byte elements (fp64 / c64 'T' 16384^2: 0.710 against 0.747 ms
                         // with 256^2 blocks, 0.709 against 0.797 with 512^2; fp32 with its
                         // 128 x 128 sub-tiles 0.366 against 0.396 with 256^2, 0.366 against
                         // 0.454 with 512^2), else 1 (c128 with 128^2 blocks: 2.87 against 2.27
                         // ms; copy lists untested under 2; profiles/r2/order/)
    int copy_granule = 1;  // copy ops into destinations off the 64-byte grid cut at each column's
                           // granules (granule_split; r6: fp64 16384^2 'N' ldc + 1 / + 2 / + 3
                           // 0.89 / 0.79 / 0.93 -> 0.76 / 0.76 / 0.74 ms, fp32 + 1 0.51 -> 0.41,
                           // int32 + 3 0.51 -> 0.41, 16-byte aligned fp32 + 4 level; profiles/r6b/);
                           // COSTA_COPY_GRANULE=0 (tuning): off
    int force_sq = 0;   // COSTA_FORCE_SQ=1 (tuning): transposing lists of fp64 / c64 / c128 take the
                        // square sub-tile whatever their ops' size
    int merge = 2;      // COSTA_MERGE=0: ops that continue each other are not merged, 1: only
                        // ops below half a large sub-tile (r3); 2 (default): every op (tuning; the
                        // skew list always merges)
    int xcd_bands = 1;  // COSTA_XCD_BANDS=k: destination-ordered wavefront lists in 8 k column
                        // bands, k per XCD (xcd_bands); 0: off.  cfg 5 'N' 0.476 -> 0.446 ms with
                        // k = 1 (2 / 4 / 16: 0.464 / 0.475 / 0.490), 'T' equal; through the
                        // loopback exchange unpack 'N' 0.609 -> 0.592, 'T' 1.016 -> 0.960
                        // (profiles/r3b/README.md §bands)
    int sort = 5;    // COSTA_TINY_SORT 0: list order, 1: by source, 2: by destination address,
                     // 3: by the planner's locality hint (costa_tile_op_t::order), 4: 3 for
                     // copy-only lists, 2 for lists that transpose (cfg 5 'T' 3.88 against
                     // 3.79 TB/s, 'N' equal; profiles/r11/c5_env.log), else as 2; 5 (default):
                     // pack lists by source address (their destinations, the dense package,
                     // are contiguous per op in any order), every other list by destination
                     // address.  cfg 5 under 5 against 4 on one lease (tools/c5_sort_probe.py,
                     // profiles/r2c/c5_sort.log): local 'N' 0.497 / 0.499-0.502 ms, 'T' equal;
                     // with every tile through the exchange (COSTA_LOOPBACK=1) 'N' pack 0.557-0.561
                     // / 0.596-0.600, unpack 0.556-0.558 / 0.606-0.610, 'T' pack 0.725-0.729 /
                     // 0.751-0.761, unpack equal
};
// f-neighbour skew sub-tiles grouped per XCD on the wide variant (fp32 16384^2 'T', both sides
// lld 16385: 0.453 / 0.440 / 0.428 / 0.419-0.424 ms with groups of 1 / 2 / 4 / 8; profiles/r3b/README.md §skew)
constexpr int64_t kSkewWideGroup = 8;
const wave_knobs& knobs() {
    static wave_knobs k = [] {
        wave_knobs x;
        if (const char* s = tuning_env("COSTA_WAVE_POLICY")) x.policy = std::atoi(s) == 1 ? 1 : 2;
        if (const char* s = tuning_env("COSTA_TINY_SORT")) x.sort = std::max(0, std::min(5, std::atoi(s)));
        if (const char* s = tuning_env("COSTA_LARGE_SORT")) x.large_sort = std::max(0, std::min(3, std::atoi(s)));
        if (const char* s = tuning_env("COSTA_PANEL_ROWS")) x.panel_rows = std::max(-1, std::atoi(s));
        if (const char* s = tuning_env("COSTA_SKEW_XCD")) x.skew_xcd = std::max(-1, std::atoi(s));
        if (const char* s = tuning_env("COSTA_XCD_BANDS")) x.xcd_bands = std::atoi(s);
        if (const char* s = tuning_env("COSTA_MERGE")) x.merge = std::atoi(s);
        if (const char* s = tuning_env("COSTA_FORCE_SQ")) x.force_sq = std::atoi(s);
        if (const char* s = tuning_env("COSTA_COPY_GRANULE")) x.copy_granule = std::atoi(s);
        return x;
    }();
    return k;
}
}  // namespace

// Copies into destinations off the 64-byte grid (a ScaLAPACK lld that is not a multiple of 64
// bytes, or a sub-matrix offset): the large copy shape writes each destination column in 1 KiB
// segments from the op's first row, so every segment boundary inside a column is a 64-byte
// granule shared by two workgroups, which HBM services as a read-modify-write.  Cut
// instead at each column's own granules: the op's columns are split by their residue modulo the
// period p after which a column starts at the same granule offset again (p * ldd * E = 0 mod 64),
// so each part has one offset eps for every column; its first G - eps rows (G = 64 / E elements:
// the head of each column's first granule) become an op of their own (the wavefront path), and
// the rest starts every column on a granule boundary, its segments whole granules.  Sub-rectangles
// of a copy op are copy ops: the same elements, the same transform; only the op boundaries move.
// Ops below `min_elems` (the wavefront path anyway) and transposing ops (the skew shape, §3b) stay
// as they are.  -> true when `out` holds a split list
bool granule_split(const std::vector<costa_tile_op_t>& ops, int64_t E, int64_t min_elems,
                   std::vector<costa_tile_op_t>& out) {
    const int64_t G = 64 / E;
    auto split_it = [&](const costa_tile_op_t& op) {
        if (G <= 1 || (op.flags & COSTA_TILE_TRANSPOSE) || op.dst % uint64_t(E) != 0) return false;
        if (int64_t(op.nf) * op.ns < min_elems || op.nf < 2 * G) return false;
        if (int64_t(std::max(op.lds, op.ldd)) * 64 > INT32_MAX) return false;  // p * ld must fit
        return op.dst % 64 != 0 || (uint64_t(op.ldd) * uint64_t(E)) % 64 != 0;
    };
    bool any = false;
    for (const auto& op : ops) any = any || split_it(op);
    if (!any) return false;
    out.clear();
    out.reserve(ops.size() + 64);
    const uint32_t vec_bits = COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST;
    for (const auto& op : ops) {
        if (!split_it(op)) {
            out.push_back(op);
            continue;
        }
        const uint64_t row_bytes = uint64_t(op.ldd) * uint64_t(E);
        const int64_t p = 64 / int64_t(std::gcd(row_bytes % 64 == 0 ? uint64_t(64) : row_bytes % 64, uint64_t(64)));
        // 4-byte sources are read as 16-byte vectors at dword alignment (build_work: mis)
        const uint32_t keep_vs = E == 4 ? (op.flags & COSTA_TILE_VEC_SRC) : 0u;
        for (int64_t r = 0; r < std::min<int64_t>(p, op.ns); ++r) {
            costa_tile_op_t part = op;
            part.src = op.src + uint64_t(r * int64_t(op.lds) * E);
            part.dst = op.dst + uint64_t(r * int64_t(op.ldd) * E);
            part.ns = int32_t((op.ns - r + p - 1) / p);
            part.lds = int32_t(int64_t(op.lds) * p);
            part.ldd = int32_t(int64_t(op.ldd) * p);
            const int64_t eps = int64_t(part.dst % 64) / E;
            const int64_t h = eps > 0 ? std::min<int64_t>(op.nf, G - eps) : 0;
            if (h > 0) {  // the head of each column's first granule
                costa_tile_op_t head = part;
                head.nf = int32_t(h);
                head.flags = (op.flags & ~vec_bits) | vec_flags(head.src, head.lds, head.dst, head.ldd, E) | keep_vs;
                out.push_back(head);
            }
            if (h < op.nf) {
                costa_tile_op_t body = part;
                body.src += uint64_t(h * E);
                body.dst += uint64_t(h * E);
                body.nf = int32_t(op.nf - h);
                body.flags = (op.flags & ~vec_bits) | vec_flags(body.src, body.lds, body.dst, body.ldd, E) | keep_vs;
                out.push_back(body);
            }
        }
    }
    return true;
}

work_split build_work(costa_dtype_t dtype, const std::vector<costa_tile_op_t>& ops_in,
                      std::vector<costa_tile_op_t>& ordered, std::vector<uint64_t>& work,
                      list_kind kind, device_section* dev) {
    const bool pack_list = kind == list_pack, local = kind == list_local;
    // Sources off the 16-byte grid: 4-byte elements are read as 16-byte vectors anyway (dword
    // alignment suffices for global_load_dwordx4): fp32 16384^2 'T' with lld 16386 0.405 against
    // 0.499 ms element by element; 8-byte elements stay element-wise (0.794 against 0.755 ms);
    // misaligned 16-byte stores lost for both (tools/unaligned_mis.sh, profiles/r3/).
    // COSTA_MISALIGNED_VEC (tuning): bit 0 destinations, bit 1 sources, for every element size.
    static const int mis_env = [] {
        const char* s = tuning_env("COSTA_MISALIGNED_VEC");
        return s ? std::atoi(s) : -1;
    }();
    // (by default only for ops of at least one large sub-tile: smaller ones keep their class)
    const int mis = mis_env >= 0 ? mis_env : dtype_size(dtype) == 4 ? 2 : 0;
    // tiles of one local matrix that continue each other in source and destination become one op
    // (a 16384^2 'T' with 24^2 blocks on one rank: one op on the large shape instead of 466 k
    // wavefront tiles)
    const wave_knobs& kn0 = knobs();
    // COSTA_PLAN_TRACE=1: where build_work spends its time (stderr; get_plan traces the whole miss)
    static const bool trace = std::getenv("COSTA_PLAN_TRACE") != nullptr;
    const auto bw0 = std::chrono::steady_clock::now();
    double bw_t[4] = {0, 0, 0, 0};  // classify + shaped lists, groups, wavefront order, pieces
    double sub_t[3] = {0, 0, 0};    // ... of the first: merge, vector flags + granule cut, classify
    auto lap = [&](int k) {
        if (!trace) return;
        const double t = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - bw0).count();
        bw_t[k] = t;
    };
    auto mark = [&](int k) {
        if (trace) sub_t[k] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - bw0).count();
    };
    std::vector<costa_tile_op_t> ops_merged;
    const std::vector<costa_tile_op_t>* ops_src = &ops_in;
    if (kn0.merge && ops_in.size() > 1 && few_strides(ops_in)) {
        shape_dims sh0;
        tile_shapes(dtype, any_transpose(ops_in), &sh0);
        // every op is a candidate, large ones included (r4): blocks that do not fill the
        // sub-tiles then run as whole merged ops (16384^2 'T' on one rank: c128 80^2 / 96^2
        // 2.919 / 2.554 -> 2.101 / 2.103 ms, fp64 96^2 0.800 -> 0.699, 100^2 0.947 -> 0.700, 80^2
        // beta != 0 1.212 -> 1.030; filled sizes unchanged; profiles/r4s/).  COSTA_MERGE=1
        // (tuning): small ops only, as in r3
        const int64_t half_large = kn0.merge == 1 ? int64_t(sh0.cf) * sh0.cs / 2 : INT64_MAX;
        std::vector<costa_tile_op_t> cand;  // the ops that may merge (the rest: ops_merged as they are)
        for (const auto& op : ops_in)
            (int64_t(op.nf) * op.ns < half_large ? cand : ops_merged).push_back(op);
        const size_t n_cand0 = cand.size();
        cand = merge_filled(cand, int64_t(dtype_size(dtype)), sh0.cf, sh0.cs);
        if (cand.size() < n_cand0) {
            ops_merged.insert(ops_merged.end(), cand.begin(), cand.end());
            ops_src = &ops_merged;
        }
    }
    mark(0);
    std::vector<costa_tile_op_t> ops_mis;
    bool mis_any = false;  // (the list is copied only when some op gains a flag: cfg 5's 245 k
                           // small ops gain none, and the copy cost a plan-cache miss ~2 ms)
    if (mis) {
        const uint64_t E = dtype_size(dtype);
        shape_dims shm;
        tile_shapes(dtype, any_transpose(ops_in), &shm);
        const int64_t min_elems = mis_env >= 0 ? 0 : int64_t(shm.cf) * shm.cs;
        auto gain = [&](const costa_tile_op_t& op) {
            uint32_t f = 0;
            if (int64_t(op.nf) * op.ns < min_elems) return f;
            if ((mis & 1) && op.dst % 4 == 0 && (uint64_t(op.ldd) * E) % 4 == 0) f |= COSTA_TILE_VEC_DST;
            if ((mis & 2) && op.src % 4 == 0 && (uint64_t(op.lds) * E) % 4 == 0) f |= COSTA_TILE_VEC_SRC;
            return f & ~op.flags;
        };
        for (const auto& op : *ops_src) mis_any = mis_any || gain(op) != 0;
        if (mis_any) {
            ops_mis = *ops_src;
            for (auto& op : ops_mis) op.flags |= gain(op);
        }
    }
    const std::vector<costa_tile_op_t>* ops_pre = mis_any ? &ops_mis : ops_src;
    std::vector<costa_tile_op_t> ops_gran;
    if (kn0.copy_granule) {
        shape_dims shg;
        tile_shapes(dtype, any_transpose(ops_in), &shg);
        if (granule_split(*ops_pre, int64_t(dtype_size(dtype)), int64_t(shg.cf) * shg.cs / 2, ops_gran))
            ops_pre = &ops_gran;
    }
    const std::vector<costa_tile_op_t>& ops = *ops_pre;
    mark(1);
    const bool tr_shape = any_transpose(ops);
    shape_dims sh;
    tile_shapes(dtype, tr_shape, &sh);
    const int64_t E = int64_t(dtype_size(dtype));
    const wave_knobs& kn = knobs();
    ordered.clear();
    work.clear();
    std::vector<const costa_tile_op_t*> wave_ops;  // ops for the wavefront path, in list order
    wave_ops.reserve(ops.size());
    const uint32_t vec_both = COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST;
    const int64_t sub_elems = int64_t(sh.cf) * sh.cs;                // one large class unit
    const int64_t med_elems = int64_t(sh.bf_m) * sh.bs_m;            // one medium sub-tile (0: none)
    // classify: wavefront path, the medium shape (aligned ops of at least half its sub-tile, in
    // lists that transpose) or the large shape
    // (a medium launch of fewer than kMinMediumOps ops costs more than it saves: it runs ahead of
    // the wavefront kernel, not beside it; cfg 5 'T' with its 969 medium ops 0.802 against 0.791
    // ms without, profiles/r2/shapes/ab_medium_cfg5T.log)
    constexpr size_t kMinMediumOps = 4096;
    std::vector<uint8_t> cls(ops.size(), 3);  // 0 large, 1 medium, 2 wavefront, 3 empty
    auto is_large = [&](const costa_tile_op_t& op, int64_t lo) {
        const int64_t elems = int64_t(op.nf) * op.ns;
        const bool aligned = (op.flags & vec_both) == vec_both;
        bool large = 2 * elems >= lo;
        if (kn.policy == 2 && !aligned && elems <= kUnalignedWaveCap * sub_elems) large = false;
        return large && !is_tiny(op, E, local);
    };
    // A transposing list whose large ops all fit the square variant of the large shape (bf_q x
    // bs_q) runs them on it: one sub-tile per op instead of a half-filled large one (fp64 / c64 /
    // c128 64^2 blocks).  Without a medium tier (complex types) the large class then starts at
    // half a square sub-tile.
    const int64_t q_elems = int64_t(sh.bf_q) * sh.bs_q;
    const int64_t q_lo = med_elems > 0 ? sub_elems : q_elems;
    bool sq = q_elems > 0;
    size_t n_cand = 0;
    for (size_t li = 0; sq && li < ops.size(); ++li) {
        const costa_tile_op_t& op = ops[li];
        if (op.nf <= 0 || op.ns <= 0 || !is_large(op, q_lo)) continue;
        ++n_cand;
        // c128 (r4): also lists whose large ops are aligned whole multiples of the square
        // sub-tile, which then run in destination-address order (below): BASELINE cfg 4's 128^2
        // blocks 16384^2 2.288 -> 2.119-2.134 ms, 32768^2 9.32 -> 9.05-9.10 ms; the 64 x 128
        // shape in that order 2.346 / 9.51, the square shape in hint order 2.237 / 9.52
        // (profiles/r4e/, r4f/)
        const bool whole_q = E == 16 && (op.flags & vec_both) == vec_both && op.nf % sh.bf_q == 0 &&
                             op.ns % sh.bs_q == 0;
        sq = kn.force_sq || (op.nf <= sh.bf_q && op.ns <= sh.bs_q) || whole_q;
    }
    sq = sq && n_cand > 0;
    const int64_t large_lo = sq ? q_lo : sub_elems;
    size_t n_med = 0;
    for (size_t li = 0; li < ops.size(); ++li) {
        const costa_tile_op_t& op = ops[li];
        if (op.nf <= 0 || op.ns <= 0) continue;
        const int64_t elems = int64_t(op.nf) * op.ns;
        const bool aligned = (op.flags & vec_both) == vec_both;
        if (is_large(op, large_lo))
            cls[li] = 0;
        else if (med_elems > 0 && aligned && 2 * elems >= med_elems && (op.flags & COSTA_TILE_TRANSPOSE))
            cls[li] = 1, ++n_med;
        else
            cls[li] = 2;
    }
    // the medium class on 32 x 32 sub-tiles (nb = 32 blocks): in a transposing list whose
    // aligned transposing ops outside the large class that hold at least half a 32 x 32 sub-tile
    // all fit one, and are at least kMinMediumOps many
    bool med_sq = tr_shape && sh.bf_s > 0;
    size_t n_msq = 0, n_exact = 0;
    const int64_t s_elems = int64_t(sh.bf_s) * sh.bs_s;
    for (size_t li = 0; med_sq && li < ops.size(); ++li) {
        const costa_tile_op_t& op = ops[li];
        if (cls[li] == 0 || cls[li] == 3 || (op.flags & vec_both) != vec_both || !(op.flags & COSTA_TILE_TRANSPOSE))
            continue;
        if (2 * int64_t(op.nf) * op.ns < s_elems) continue;
        if (op.nf > sh.bf_s || op.ns > sh.bs_s) med_sq = false;
        ++n_msq;
        n_exact += op.nf == sh.bf_s && op.ns == sh.bs_s;
    }
    // ... and at least 9 in 10 of them fill a sub-tile exactly (partly filled 32 x 32 sub-tiles lost
    // to the wavefront path: fp32 24^2 blocks 1.105 against 0.688 ms, c64 28^2 1.43 against 1.14;
    // profiles/r2e/s32/partial.log)
    med_sq = med_sq && n_msq >= kMinMediumOps && n_exact * 10 >= n_msq * 9;
    if (med_sq) {
        n_med = n_msq;
        for (size_t li = 0; li < ops.size(); ++li) {
            const costa_tile_op_t& op = ops[li];
            if (cls[li] == 0 || cls[li] == 3) continue;
            const bool m = (op.flags & vec_both) == vec_both && (op.flags & COSTA_TILE_TRANSPOSE) &&
                           2 * int64_t(op.nf) * op.ns >= s_elems;
            cls[li] = m ? 1 : 2;
        }
    }
    // transposes whose destination columns are off the 16-byte grid (an odd ScaLAPACK lld) go to
    // the skew shape (tile_kernels.hip skew_kernel): the cut between its sub-tiles follows the
    // 64-byte granules of each destination column, so no granule is shared by two workgroups
    // (measured: a copy whose 128-byte lines are split between workgroups at 16-byte granularity
    // 0.808 against 0.672 ms, at 64-byte granularity 0.702; tools/partial_line_probe.hip).  Every
    // element is written once: ops that read C (beta != 0) go there too.
    const int64_t k_elems = int64_t(sh.bf_k) * sh.bs_k;
    static const bool skew_on = [] {  // COSTA_SKEW=0: off (tuning)
        const char* s = tuning_env("COSTA_SKEW");
        return !s || std::atoi(s) != 0;
    }();
    // r4: also destinations on the 16-byte grid whose columns start off the 64-byte one (lld not
    // a multiple of 8 fp64 / 16 fp32 elements): the large shape's column segments then share
    // their edge granules with the neighbouring sub-tiles.  fp64 16384^2 'T' lld + 2 / + 4
    // 1.046 / 1.015 -> 0.855 / 0.837 ms, beta != 0 1.444 -> 1.244; fp32 lld + 4 / + 8 / + 24
    // 0.687 / 0.620 / 0.595 -> 0.466 / 0.482 / 0.466; aligned and 64-byte-aligned ld unchanged
    // (profiles/r4l/)
    // (r6) ...except transposes into a destination range a destination-block group may write: a
    // custom layout's own block buffer (leading dimension within a group's budget) is written by
    // its group in whole 16-byte vectors whatever its alignment, so such ops stay on the wavefront
    // path, where cblock_groups finds them; left out, their block's other ops fail the exactness
    // test too (cfg 5 'T': 45 skew ops broke 334 groups into 2 672 wavefront pieces)
    const bool groups_on = cblock_enabled(dtype, kind);
    const int64_t group_budget = cblock_max_elems(E) - (16 / E - 1);
    for (size_t li = 0; skew_on && k_elems > 0 && li < ops.size(); ++li) {
        const costa_tile_op_t& op = ops[li];
        if (cls[li] == 3 || !(op.flags & COSTA_TILE_TRANSPOSE)) continue;
        const bool off_granule = op.dst % 64 != 0 || (uint64_t(op.ldd) * uint64_t(E)) % 64 != 0;
        if ((op.flags & COSTA_TILE_VEC_DST) && !off_granule) continue;
        if (op.dst % uint64_t(E) != 0 || 2 * int64_t(op.nf) * op.ns < k_elems)
            continue;
        if (cls[li] == 1) --n_med;
        if (groups_on && op.ns <= op.ldd && op.ldd <= group_budget) {
            cls[li] = 2;
            continue;
        }
        cls[li] = 4;
    }
    mark(2);
    std::vector<uint32_t> shaped[3];  // [0] large, [1] medium, [2] skew
    std::vector<costa_tile_op_t> skew_ops;
    for (size_t li = 0; li < ops.size(); ++li) {
        const int c = cls[li] == 1 && n_med < kMinMediumOps ? 2 : cls[li];
        if (c < 2) shaped[c].push_back(uint32_t(li));
        else if (c == 2) wave_ops.push_back(&ops[li]);
        else if (c == 4) skew_ops.push_back(ops[li]);
    }
    // skew ops that continue each other in source and destination (the tiles of one local
    // matrix) become one op: a tile edge inside a destination column would otherwise be a
    // partial granule shared by two workgroups again
    merge_adjacent(skew_ops, E);
    for (size_t i = 0; i < skew_ops.size(); ++i) shaped[2].push_back(uint32_t(i));
    // 4-byte types reading sources off the 16-byte grid too: the wide skew variant, its
    // f-neighbours (which share the misaligned source runs' partial lines) grouped on one XCD
    bool skew_wide = false;
    for (const auto& op : skew_ops)
        skew_wide = skew_wide || (E == 4 && (op.src % 16 != 0 || (uint64_t(op.lds) * uint64_t(E)) % 16 != 0));
    const int64_t skew_group = kn.skew_xcd >= 0 ? kn.skew_xcd : skew_wide ? kSkewWideGroup : 0;
    // each shape's ops in hint order when every one carries a hint; lists whose shaped ops all
    // transpose 8-byte elements then take the sub-tiles in destination-address order (wave_knobs)
    int64_t n_work[3] = {0, 0, 0};
    for (int c = 0; c < 3; ++c) {
        const int bf = c == 2 ? (skew_wide ? sh.bf_kw : sh.bf_k) : c ? (med_sq ? sh.bf_s : sh.bf_m) : sq ? sh.bf_q : sh.bf;
        const int bs = c == 2 ? (skew_wide ? sh.bs_kw : sh.bs_k) : c ? (med_sq ? sh.bs_s : sh.bs_m) : sq ? sh.bs_q : sh.bs;
        const std::vector<uint32_t>& sel = shaped[c];
        const std::vector<costa_tile_op_t>& src_ops = c == 2 ? skew_ops : ops;
        std::vector<uint32_t> sperm(sel.size());
        for (size_t i = 0; i < sel.size(); ++i) sperm[i] = uint32_t(i);
        if (kn.large_sort >= 1 && !sel.empty()) {
            bool hints = true;
            for (uint32_t li : sel) hints = hints && src_ops[li].order != 0;
            if (hints)
                std::stable_sort(sperm.begin(), sperm.end(), [&](uint32_t x, uint32_t y) {
                    return src_ops[sel[x]].order < src_ops[sel[y]].order;
                });
        }
        const size_t op0 = ordered.size(), w0 = work.size();
        for (const uint32_t k : sperm) {
            const costa_tile_op_t& op = src_ops[sel[k]];
            const uint64_t i = ordered.size();
            if (i > 0xFFFFFFFFull) throw error(COSTA_ERR_ARG, "costa: too many tiles in one list");
            ordered.push_back(op);
            const uint64_t n = uint64_t((op.nf + bf - 1) / bf) * uint64_t((op.ns + bs - 1) / bs);
            if (n > 0xFFFFFFFFull) throw error(COSTA_ERR_ARG, "costa: tile too large");
            for (uint64_t q = 0; q < n; ++q) work.push_back((i << 32) | q);
        }
        bool by_address = kn.large_sort == 2;
        if (kn.large_sort == 3) {
            by_address = (E == 4 || E == 8 || (E == 16 && c == 0 && sq)) && ordered.size() > op0;
            for (size_t i = op0; i < ordered.size(); ++i)
                by_address = by_address && (ordered[i].flags & COSTA_TILE_TRANSPOSE);
        }
        if (by_address && work.size() - w0 > 1) {
            // sub-tiles by the address of their first destination element (stable)
            std::vector<std::pair<uint64_t, uint64_t>> key(work.size() - w0);
            for (size_t x = 0; x < key.size(); ++x) {
                const uint64_t wx = work[w0 + x];
                const costa_tile_op_t& op = ordered[size_t(wx >> 32)];
                const uint64_t q = wx & 0xFFFFFFFFull, nbf = uint64_t((op.nf + bf - 1) / bf);
                const int64_t f0 = int64_t(q % nbf) * bf, s0 = int64_t(q / nbf) * bs;
                const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
                key[x] = {op.dst + uint64_t((tr ? f0 * op.ldd + s0 : s0 * op.ldd + f0) * E), wx};
            }
            // Destination columns taller than 128 KiB are walked in panels of 128 KiB of rows, each
            // panel band by band (r4): the sub-tiles in flight then cover 4 adjacent bands of a
            // panel instead of one band's full height, and read 4 KiB of each source column
            // instead of 1 KiB.  c128 'T' 32768^2 (512 KiB columns) 9.06-9.07 -> 8.66 ms; fp64
            // 32768^2 4.35 -> 4.27; 64 / 32 KiB panels lost (profiles/r4p/, r4q/).  Lists of
            // one destination stride only (the panel is cut from row / column positions).
            int64_t panel = kn.panel_rows;
            const int64_t ld0 = ordered[size_t(key[0].second >> 32)].ldd;
            bool one_ld = true;
            for (size_t i = op0; i < ordered.size() && one_ld; ++i) one_ld = ordered[i].ldd == ld0;
            // (c64, on its 128 x 128 sub-tiles, ran 1 % slower with them: 4.36 against 4.31 ms)
            if (panel == 0)
                panel = ld0 * E > kPanelBytes && dtype != COSTA_CFLOAT ? kPanelBytes / E : -1;
            // key = panel (16 bits) | column (24) | row in the panel (24): a panel of 2^24 rows or
            // more, a column index or a panel index past its field keeps the plain address order
            if (panel >= (int64_t(1) << 24)) panel = -1;
            if (panel > 0 && one_ld) {
                uint64_t lo = ~uint64_t(0), hi = 0;
                for (const auto& k : key) {
                    lo = std::min(lo, k.first);
                    hi = std::max(hi, k.first);
                }
                const uint64_t ld = uint64_t(ld0), last = (hi - lo) / uint64_t(E);
                const bool fits = last / ld < (uint64_t(1) << 24) && ld / uint64_t(panel) < (uint64_t(1) << 16);
                if (fits) {
                    for (auto& k : key) {
                        const uint64_t e = (k.first - lo) / uint64_t(E);
                        const uint64_t row = e % ld, col = e / ld;
                        k.first = ((row / uint64_t(panel)) << 48) | (col << 24) | (row % uint64_t(panel));
                    }
                }
            }
            sort_pairs_by_key(key);
            for (size_t x = 0; x < key.size(); ++x) work[w0 + x] = key[x].second;
        }
        if (c == 2 && skew_group > 1 && work.size() - w0 > 1) {
            // runs of F f-neighbours at one destination position, then run r of every 8 runs
            // spread to positions r, r + 8, ...: dispatch goes round-robin over the 8 XCDs
            const int64_t F = skew_group;
            std::vector<std::pair<uint64_t, uint64_t>> key(work.size() - w0);
            for (size_t x = 0; x < key.size(); ++x) {
                const uint64_t wx = work[w0 + x];
                const costa_tile_op_t& op = ordered[size_t(wx >> 32)];
                const uint64_t q = wx & 0xFFFFFFFFull, nbf = uint64_t((op.nf + bf - 1) / bf);
                const int64_t f0 = int64_t(q % nbf) * bf, s0 = int64_t(q / nbf) * bs;
                const int64_t fp = f0 / (bf * F) * (bf * F);
                key[x] = {((op.dst + uint64_t((fp * op.ldd + s0) * E)) << 6) | uint64_t((f0 - fp) / bf), wx};
            }
            std::sort(key.begin(), key.end());
            const size_t n = key.size(), blk = size_t(8 * F);
            for (size_t b = 0; b < n; b += blk) {
                const size_t m = std::min(blk, n - b);
                for (size_t x = 0; x < m; ++x) {
                    const size_t run = x / size_t(F), in = x % size_t(F);
                    const size_t to = m == blk ? in * 8 + run : x;
                    work[w0 + b + to] = key[b + x].second;
                }
            }
        }
        n_work[c] = int64_t(work.size() - w0);
    }
    lap(0);
    // destination-block groups out of the wavefront ops (after the skew items in `work`)
    int64_t cblock_lds = 0;
    int cb_map = cb_round_robin;
    const int64_t n_cblock = cblock_groups(dtype, wave_ops, kind, ordered, work, cblock_lds, cb_map, ops, dev);
    const size_t n_dev = dev ? dev->n_ordered : 0;  // the groups' entries left on the GPU
    lap(1);
    // ops are independent (disjoint destinations), so any order is valid; neighbours in
    // memory run at the same time and share the partially used cache lines at their edges.
    // The wavefront ops are ordered first, then cut into their pieces straight into the ordered
    // list (pieces of one op stay together, in f-major order).
    const size_t nw = wave_ops.size();
    uint32_t top = 0;  // largest hint (0: none of the ops carries one)
    bool tr = false;
    for (const auto* o : wave_ops) {
        top = std::max(top, o->order);
        tr = tr || (o->flags & COSTA_TILE_TRANSPOSE);
    }
    const int mode = kn.sort == 5   ? (pack_list ? 1 : 2)
                     : kn.sort == 4 ? (tr || top == 0 ? 2 : 3)
                     : kn.sort == 3 && top == 0 ? 2 : kn.sort;
    std::vector<uint32_t> perm(nw);
    if (mode == 3 && size_t(top) <= 4 * nw + 1024) {
        // the planner's hints are ranks within the list: a stable counting sort
        std::vector<uint32_t> at(size_t(top) + 2, 0);
        for (const auto* o : wave_ops) ++at[size_t(o->order) + 1];
        for (size_t k = 1; k < at.size(); ++k) at[k] += at[k - 1];
        for (size_t i = 0; i < nw; ++i) perm[at[wave_ops[i]->order]++] = uint32_t(i);
    } else if (mode == 2 && nw > 0) {
        // by destination address: a stable LSD radix sort of the element offsets from the lowest
        // destination (14-bit digits, only as many passes as the span needs)
        uint64_t lo = ~uint64_t(0), hi = 0;
        for (const auto* o : wave_ops) {
            lo = std::min(lo, o->dst);
            hi = std::max(hi, o->dst);
        }
        std::vector<uint64_t> key(nw), key2(nw);
        std::vector<uint32_t> idx2(nw);
        for (size_t i = 0; i < nw; ++i) {
            key[i] = (wave_ops[i]->dst - lo) / uint64_t(E);
            perm[i] = uint32_t(i);
        }
        const uint64_t span = (hi - lo) / uint64_t(E);
        constexpr int B = 14;
        std::vector<uint32_t> at((1 << B) + 1);
        for (int shift = 0; shift == 0 || (shift < 64 && (span >> shift) != 0); shift += B) {
            std::fill(at.begin(), at.end(), 0u);
            for (size_t i = 0; i < nw; ++i) ++at[((key[i] >> shift) & ((1 << B) - 1)) + 1];
            for (int d = 1; d <= (1 << B); ++d) at[d] += at[d - 1];
            for (size_t i = 0; i < nw; ++i) {
                const uint32_t p = at[(key[i] >> shift) & ((1 << B) - 1)]++;
                key2[p] = key[i];
                idx2[p] = perm[i];
            }
            key.swap(key2);
            perm.swap(idx2);
        }
    } else if (mode >= 1 && mode <= 3) {  // sort (key, index) pairs: stable
        std::vector<std::pair<uint64_t, uint32_t>> key(nw);
        for (size_t i = 0; i < nw; ++i) {
            const costa_tile_op_t& o = *wave_ops[i];
            key[i] = {mode == 1 ? o.src : mode == 2 ? o.dst : o.order, uint32_t(i)};
        }
        std::sort(key.begin(), key.end());
        for (size_t i = 0; i < nw; ++i) perm[i] = key[i].second;
    } else {
        for (size_t i = 0; i < nw; ++i) perm[i] = uint32_t(i);
    }
    if (kn.xcd_bands && mode == 2 && top > 0 && nw > 1) xcd_bands(wave_ops, E, kn.xcd_bands, local, perm);
    lap(2);
    // pieces: count per op, scan, fill (host threads for long lists)
    std::vector<wave_grid> grid(nw);
    std::vector<size_t> at_piece(nw + 1, 0);
    host_parallel(nw, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i) grid[i] = wave_pieces(*wave_ops[perm[i]], E, local);
    });
    for (size_t i = 0; i < nw; ++i)
        at_piece[i + 1] = at_piece[i] + size_t(grid[i].nfc * grid[i].nsc);
    work_split w;
    w.tr_shape = tr_shape;
    w.sq = sq;
    w.full = tr_shape && !sq && !shaped[0].empty();
    for (const uint32_t li : shaped[0]) {
        const costa_tile_op_t& op = ops[li];
        w.full = w.full && (op.flags & vec_both) == vec_both && op.nf % sh.bf == 0 && op.ns % sh.bs == 0;
    }
    w.med_sq = med_sq && !shaped[1].empty();
    w.med_full = !shaped[1].empty() && n_work[1] > 0 && !w.med_sq;
    for (const uint32_t li : shaped[1])
        w.med_full = w.med_full && ops[li].nf % sh.bf_m == 0 && ops[li].ns % sh.bs_m == 0;
    w.n_large = n_work[0];
    w.n_medium = n_work[1];
    w.n_skew = n_work[2];
    w.skew_wide = skew_wide && n_work[2] > 0;
    w.n_cblock = n_cblock;
    w.cblock_lds = cblock_lds;
    w.cb_map = cb_map;

    w.tiny_first = int64_t(ordered.size() + n_dev);
    w.n_tiny = int64_t(at_piece[nw]);
    const size_t base = ordered.size();
    ordered.resize(base + at_piece[nw]);
    host_parallel(nw, [&](size_t b, size_t e) {
        for (size_t i = b; i < e; ++i)
            emit_pieces(*wave_ops[perm[i]], E, grid[i], local, &ordered[base + at_piece[i]]);
    });
    if (trace) {
        lap(3);
        std::fprintf(stderr,
                     "[costa build_work] %zu ops (%s list): classify + shaped %.2f ms (merge %.2f, flags + "
                     "granules %.2f, classify %.2f, work items %.2f), groups %.2f (%lld), "
                     "wavefront order %.2f, pieces %.2f (%lld)\n",
                     ops_in.size(), pack_list ? "pack" : local ? "local" : "unpack", bw_t[0], sub_t[0],
                     sub_t[1] - sub_t[0], sub_t[2] - sub_t[1], bw_t[0] - sub_t[2], bw_t[1] - bw_t[0],
                     (long long)n_cblock, bw_t[2] - bw_t[1], bw_t[3] - bw_t[2], (long long)w.n_tiny);
    }
    return w;
}

launch_args make_launch(const work_split& w, const void* d_ordered, const void* d_work,
                        const char* src_base, char* dst_base, const void* d_scalars, bool transpose,
                        bool axpby) {
    launch_args a;
    a.ops = static_cast<const costa_tile_op_t*>(d_ordered);
    a.work = static_cast<const uint64_t*>(d_work);
    a.n_large = w.n_large;
    a.n_medium = w.n_medium;
    a.n_skew = w.n_skew;
    a.n_cblock = w.n_cblock;
    a.cblock_lds = w.cblock_lds;
    a.cb_map = w.cb_map;
    a.tiny_first = w.tiny_first;
    a.n_tiny = w.n_tiny;
    a.src_base = src_base;
    a.dst_base = dst_base;
    a.scalars = d_scalars;
    a.any_transpose = transpose;
    a.any_axpby = axpby;
    a.tr_shape = w.tr_shape;
    a.sq = w.sq;
    a.full = w.full;
    a.med_full = w.med_full;
    a.med_sq = w.med_sq;
    a.skew_wide = w.skew_wide;
    return a;
}

// ---------------------------------------------------------------- residency / staging
namespace {

// Byte ranges of host memory touched by a layout's blocks, merged; used to stage
// host-resident matrices through HBM (the path starts and ends in host memory).
struct hrange {
    uintptr_t lo, hi;
    size_t dev_off;
};

size_t block_extent_bytes(const eblock& b, char ordering, size_t E) {
    const int64_t nr = b.rows.length(), nc = b.cols.length();
    if (nr == 0 || nc == 0) return 0;
    const int64_t fast = ordering == 'R' ? nc : nr, slow = ordering == 'R' ? nr : nc;
    return size_t((slow - 1) * int64_t(b.ld) + fast) * E;
}

bool is_device_ptr(const void* p) {
    hipPointerAttribute_t a;
    hipError_t e = hipPointerGetAttributes(&a, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

// true if every block is in device memory; false if every block is host memory
bool layout_on_device(const elayout& L) {
    if (L.blocks.empty()) return true;
    bool first = is_device_ptr(L.blocks.front().data);
    // check block pointers that leave the current device allocation
    uintptr_t lo = 0, hi = 0;
    for (const auto& b : L.blocks) {
        uintptr_t p = reinterpret_cast<uintptr_t>(b.data);
        if (first && p >= lo && p < hi) continue;
        bool d = is_device_ptr(b.data);
        if (d != first)
            throw error(COSTA_ERR_ARG, "costa: a layout mixes host and device blocks");
        if (d) {
            hipDeviceptr_t base = nullptr;
            size_t sz = 0;
            if (hipMemGetAddressRange(&base, &sz, const_cast<char*>(b.data)) == hipSuccess) {
                lo = reinterpret_cast<uintptr_t>(base);
                hi = lo + sz;
            } else {
                (void)hipGetLastError();
            }
        }
    }
    return first;
}

}  // namespace

// ---------------------------------------------------------------- host staging mode
namespace {
int g_host_mode = -1;
}
int host_staging_mode() {
    if (g_host_mode < 0) {
        const char* s = std::getenv("COSTA_HOST_STAGING");
        g_host_mode = s ? (std::atoi(s) != 0) : 1;
    }
    return g_host_mode;
}
void set_host_staging_mode(int mode) {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    g_host_mode = mode != 0;
}

// ---------------------------------------------------------------- plan cache
namespace {

struct hasher {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    uint64_t h2 = 0x2545F4914F6CDD1Dull;  // second lane: other seed, other multiplier
    void mix(uint64_t v) {
        v ^= v >> 33;
        v *= 0xff51afd7ed558ccdull;
        v ^= v >> 33;
        h = (h ^ v) * 0xc4ceb9fe1a85ec53ull + 0x165667b19e3779f9ull;
        h ^= h >> 29;
        h2 = (h2 + v) * 0x9fb21c651e98df25ull;
        h2 ^= h2 >> 31;
    }
    void mix_vec(const std::vector<int>& v) {
        mix(v.size());
        for (int x : v) mix(uint64_t(uint32_t(x)));
    }
    void mix_layout(const elayout& L) {
        mix(uint64_t(L.dtype));
        mix(uint64_t(uint8_t(L.ordering)));
        mix(uint64_t(L.n_ranks));
        mix_vec(L.rows_split);
        mix_vec(L.cols_split);
        mix_vec(L.owners);
        mix(L.blocks.size());
        for (const auto& b : L.blocks) {
            mix(uint64_t(uint32_t(b.rows.start)) | (uint64_t(uint32_t(b.rows.end)) << 32));
            mix(uint64_t(uint32_t(b.cols.start)) | (uint64_t(uint32_t(b.cols.end)) << 32));
            mix(reinterpret_cast<uintptr_t>(b.data));
            mix(uint64_t(uint32_t(b.ld)));
        }
    }
};

}  // namespace

uint64_t layout_hash(const elayout& L) {
    hasher h;
    h.mix_layout(L);
    return h.h | 1;  // never 0 (0 = "not computed")
}

void layout_hashes(const elayout& L, uint64_t& h1, uint64_t& h2) {
    hasher h;
    h.mix_layout(L);
    h1 = h.h | 1;
    h2 = h.h2;
}

void set_layout_hash(elayout& L) { layout_hashes(L, L.hash, L.hash2); }

namespace {

struct cached_plan {
    std::unique_ptr<plan> p;
    int device = 0;
    // staging of host-resident layouts (empty when everything is in HBM)
    bool staged = false;
    std::vector<hrange> h2d_ranges, d2h_ranges;  // uploaded / copied back
    dbuf stage;
    // device copies of the op lists and work lists
    dbuf d_local, w_local, d_scal;
    work_split l_local;                     // how the work list splits over the kernel shapes
    bool tr_local = true, ax_local = true;  // any op of the list transposes / reads C
    struct xround {  // one exchange round: its pack ops (by their first element) and unpack
                     // ops (by their last element)
        dbuf d_pack, w_pack, d_unpack, w_unpack;
        work_split l_pack, l_unpack;
        bool tr_unpack = false, ax_unpack = false;
    };
    std::vector<std::unique_ptr<xround>> rounds;
    std::vector<unsigned char> scal_host;
    std::shared_ptr<host_pipeline> pipe;  // host-resident single-rank calls (host_pipe.cpp)
};

constexpr size_t kMaxPlans = 16;
// A plan is found by a 64-bit hash and then verified against its full key: the second content
// hash of every layout plus cheap identity fields (sizes, first / last block pointer and ld).
// A hit on the hash alone would replay another layout pair's raw device addresses.
struct keyed_plan {
    uint64_t h = 0;
    std::vector<uint64_t> key;
    std::unique_ptr<cached_plan> plan;
};
std::list<keyed_plan> g_plans;  // MRU first

void key_layout(std::vector<uint64_t>& k, const elayout& L) {
    uint64_t h1 = L.hash, h2 = L.hash2;
    if (!h1) layout_hashes(L, h1, h2);  // C++-API layouts are hashed per call
    k.push_back(h1);
    k.push_back(h2);
    k.push_back(uint64_t(L.dtype) | uint64_t(uint8_t(L.ordering)) << 8 |
                uint64_t(uint32_t(L.n_ranks)) << 32);
    k.push_back(uint64_t(uint32_t(L.nbr())) | uint64_t(uint32_t(L.nbc())) << 32);
    k.push_back(L.blocks.size());
    if (!L.blocks.empty())
        for (const eblock* b : {&L.blocks.front(), &L.blocks.back()}) {
            k.push_back(reinterpret_cast<uintptr_t>(b->data));
            k.push_back(uint64_t(uint32_t(b->ld)) | uint64_t(uint32_t(b->rows.start)) << 32);
        }
}

// remap every block pointer of `L` that lies in a staged range to its device address
elayout remap(const elayout& L, const std::vector<hrange>& ranges, char* dev) {
    elayout out = L;
    for (auto& b : out.blocks) {
        uintptr_t p = reinterpret_cast<uintptr_t>(b.data);
        auto it = std::upper_bound(ranges.begin(), ranges.end(), p,
                                   [](uintptr_t v, const hrange& r) { return v < r.lo; });
        if (it == ranges.begin()) throw error(COSTA_ERR_INTERNAL, "costa: staging map miss");
        --it;
        b.data = dev + it->dev_off + (p - it->lo);
    }
    return out;
}

std::vector<hrange> collect_ranges(const std::vector<const elayout*>& Ls) {
    std::vector<hrange> r;
    for (const elayout* L : Ls) {
        const size_t E = dtype_size(L->dtype);
        for (const auto& b : L->blocks) {
            size_t ext = block_extent_bytes(b, L->ordering, E);
            if (!ext) continue;
            uintptr_t lo = reinterpret_cast<uintptr_t>(b.data);
            r.push_back({lo, lo + ext, 0});
        }
    }
    std::sort(r.begin(), r.end(), [](const hrange& x, const hrange& y) { return x.lo < y.lo; });
    std::vector<hrange> m;
    for (const auto& x : r) {
        if (!m.empty() && x.lo <= m.back().hi)
            m.back().hi = std::max(m.back().hi, x.hi);
        else
            m.push_back(x);
    }
    return m;
}

}  // namespace

// ---------------------------------------------------------------- planner choice
namespace {
int g_planner = -1;                         // costa_hip_set_planner / COSTA_PLANNER
constexpr size_t kDevicePlanBlocks = 4096;  // smaller layout pairs plan on the host
// The first GPU plan of a process loads the planner's kernels (about 15 ms on MI355X); before
// that, only layout pairs whose host planning costs as much go to the GPU.
constexpr size_t kColdDevicePlanBlocks = 100000;
bool g_device_planner_warm = false;
}  // namespace

int planner_mode() {
    if (g_planner < 0) {
        const char* s = std::getenv("COSTA_PLANNER");
        g_planner = s ? std::max(0, std::min(2, std::atoi(s))) : 1;
    }
    return g_planner;
}

void set_planner_mode(int mode) {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    g_planner = mode;
}

namespace {
int g_list_builder = -1;  // costa_hip_set_list_builder / COSTA_LIST_BUILDER
}  // namespace

int list_builder_mode() {
    if (g_list_builder < 0) {
        const char* s = std::getenv("COSTA_LIST_BUILDER");
        g_list_builder = s ? std::max(0, std::min(2, std::atoi(s))) : 1;
    }
    return g_list_builder;
}

void set_list_builder_mode(int mode) {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    g_list_builder = mode;
}

namespace {
// a work list into device memory: the host entries around the section the GPU built
template <typename X>
void upload_list(dbuf& d, const std::vector<X>& h, const X* sec, size_t at, size_t n, hipStream_t s) {
    if (!sec || n == 0) return d.upload(h, s);
    const size_t total = h.size() + n;
    d.reserve(total * sizeof(X));
    X* p = static_cast<X*>(d.p);
    if (at) HIP_CHECK(hipMemcpyAsync(p, h.data(), at * sizeof(X), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(p + at, sec, n * sizeof(X), hipMemcpyDeviceToDevice, s));
    if (h.size() > at)
        HIP_CHECK(hipMemcpyAsync(p + at + n, h.data() + at, (h.size() - at) * sizeof(X), hipMemcpyHostToDevice, s));
}
}  // namespace

bool work_export(costa_dtype_t dtype, const std::vector<costa_tile_op_t>& ops, list_kind kind, int device,
                 std::vector<costa_tile_op_t>& ordered, std::vector<uint64_t>& work, work_split& w) {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    if (device < 0) {
        w = build_work(dtype, ops, ordered, work, kind);
        return false;
    }
    device_ctx& dc = ctx(device);
    device_section sec;
    sec.device = device;
    sec.stream = dc.main;
    sec.force = true;
    w = build_work(dtype, ops, ordered, work, kind, &sec);
    if (!sec.n_ordered) return false;
    std::vector<costa_tile_op_t> o(sec.n_ordered);
    std::vector<uint64_t> k(sec.n_work);
    HIP_CHECK(hipMemcpyAsync(o.data(), sec.d_ordered, o.size() * sizeof(o[0]), hipMemcpyDeviceToHost, dc.main));
    HIP_CHECK(hipMemcpyAsync(k.data(), sec.d_work, k.size() * sizeof(k[0]), hipMemcpyDeviceToHost, dc.main));
    HIP_CHECK(hipStreamSynchronize(dc.main));
    ordered.insert(ordered.begin() + std::ptrdiff_t(sec.at_ordered), o.begin(), o.end());
    work.insert(work.begin() + std::ptrdiff_t(sec.at_work), k.begin(), k.end());
    return true;
}

namespace {
// the plan of a cache miss, built on the GPU when the planner mode asks for it and the layouts
// allow it (make_plan_device), else on the host; both give the same plan
std::unique_ptr<plan> plan_jobs(const std::vector<job>& jobs, comm* c, hipStream_t s) {
    const int lb = c->size == 1 && c->nccl ? loopback_exchange() : 0;
    const int mode = planner_mode();
    size_t blocks = 0;
    for (const job& j : jobs) blocks += j.A->blocks.size() + j.C->blocks.size();
    const size_t need = g_device_planner_warm ? kDevicePlanBlocks : kColdDevicePlanBlocks;
    if (mode == 2 || (mode == 1 && blocks >= need)) {
        if (auto p = make_plan_device(jobs, c->rank, c->size, lb, c->device, s)) {
            g_stats.device_plans++;
            g_device_planner_warm = true;
            return p;
        }
    }
    return make_plan(jobs, c->rank, c->size, lb);
}

cached_plan* get_plan(const std::vector<job>& jobs, comm* c, device_ctx& dc) {
    std::vector<uint64_t> key;
    key.reserve(4 + jobs.size() * 30);
    key.push_back(uint64_t(uint32_t(c->rank)) | uint64_t(uint32_t(c->size)) << 32);
    key.push_back(uint64_t(uint32_t(c->device)) | uint64_t(uint32_t(host_staging_mode())) << 32);
    key.push_back(jobs.size());
    for (const auto& j : jobs) {
        key_layout(key, *j.A);  // handles cache their hashes
        key_layout(key, *j.C);
        uint64_t w = uint64_t(uint8_t(std::toupper(static_cast<unsigned char>(j.trans))));
        // the scale kinds (not the values) are baked into the ops
        for (bool cm : {true, false})
            w = w << 8 | scale_kind(j.A->dtype, j.s, cm, std::toupper(j.trans) == 'C');
        key.push_back(w);
    }
    hasher h;
    for (uint64_t w : key) h.mix(w);
    for (auto it = g_plans.begin(); it != g_plans.end(); ++it) {
        if (it->h == h.h && it->key == key) {
            g_plans.splice(g_plans.begin(), g_plans, it);
            g_stats.plan_hits++;
            return g_plans.front().plan.get();
        }
    }
    g_stats.plan_misses++;
    // COSTA_PLAN_TRACE=1: where a plan-cache miss spends its host time (stderr)
    static const bool trace = std::getenv("COSTA_PLAN_TRACE") != nullptr;
    auto now = [] {
        return std::chrono::duration<double, std::milli>(
                   std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const double t0 = now();
    double t_resid = 0, t_plan = 0, t_work = 0;

    auto cp = std::make_unique<cached_plan>();
    cp->device = c->device;
    // residency: all device, or stage the host-resident layouts
    bool all_dev = true;
    std::vector<const elayout*> host_layouts;
    std::vector<bool> on_dev;
    for (const auto& j : jobs)
        for (const elayout* L : {j.A, j.C}) {
            bool d = layout_on_device(*L);
            on_dev.push_back(d);
            all_dev = all_dev && d;
        }
    std::vector<elayout> remapped;
    std::vector<job> pj = jobs;
    std::vector<hrange> staged_ranges;
    std::vector<uint8_t> range_flags;
    if (!all_dev) {
        cp->staged = true;
        std::vector<const elayout*> As, Cs;
        size_t k = 0;
        for (const auto& j : jobs) {
            if (!on_dev[k++]) As.push_back(j.A);
            if (!on_dev[k++]) Cs.push_back(j.C);
        }
        std::vector<const elayout*> all = As;
        all.insert(all.end(), Cs.begin(), Cs.end());
        auto ranges = collect_ranges(all);
        size_t off = 0;
        for (auto& r : ranges) {
            r.dev_off = off;
            off += ((r.hi - r.lo) + 255) & ~size_t(255);
        }
        // per merged range: holds A data (bit 0), C data (bit 1), C blocks of more than one
        // job (bit 2); C ranges are copied back, A ranges and C ranges the kernels do not
        // overwrite completely are uploaded (decided once the ops are known, below)
        range_flags.assign(ranges.size(), 0);
        std::vector<int> c_job(ranges.size(), -1);
        auto range_of = [&](uintptr_t p) {
            auto it = std::upper_bound(ranges.begin(), ranges.end(), p,
                                       [](uintptr_t v, const hrange& r) { return v < r.lo; });
            return size_t(it - ranges.begin()) - 1;
        };
        k = 0;
        for (size_t t = 0; t < jobs.size(); ++t) {
            const bool a_host = !on_dev[k++], c_host = !on_dev[k++];
            for (int side = 0; side < 2; ++side) {
                if (!(side == 0 ? a_host : c_host)) continue;
                const elayout* L = side == 0 ? jobs[t].A : jobs[t].C;
                const size_t E = dtype_size(L->dtype);
                for (const auto& b : L->blocks) {
                    if (!block_extent_bytes(b, L->ordering, E)) continue;
                    const size_t i = range_of(reinterpret_cast<uintptr_t>(b.data));
                    if (side == 0) {
                        range_flags[i] |= 1;
                    } else {
                        range_flags[i] |= 2;
                        if (c_job[i] >= 0 && c_job[i] != int(t)) range_flags[i] |= 4;
                        c_job[i] = int(t);
                    }
                }
            }
        }
        // Pipelined staging (host_pipe.cpp) when every layout is host-resident, no range holds
        // both source and target data (in-place) and no target range is shared by two jobs
        // (their updates would have to be applied in order).
        bool pipe_ok = host_staging_mode() == 1 &&
                       std::none_of(on_dev.begin(), on_dev.end(), [](bool d) { return d; });
        for (uint8_t f : range_flags)
            if ((f & 3) == 3 || (f & 4)) pipe_ok = false;
        if (pipe_ok) {
            const double tp = now();
            auto hplan = plan_jobs(jobs, c, dc.main);  // host addresses
            g_stats.plan_ms += now() - tp;
            if (host_pipeline_accepts(hplan->dtype, hplan->pack_ops)) {
                cp->staged = false;
                cp->p = std::move(hplan);
                const int R = c->nccl ? exchange_rounds() : 1;
                std::vector<int> pr, ur;
                exchange_round_of_ops(*cp->p, R, pr, ur);
                cp->pipe = make_host_pipeline(cp->p->dtype, cp->p->pack_ops, cp->p->local_ops,
                                              cp->p->unpack_ops, pr, ur, R);
                g_plans.push_front({h.h, std::move(key), std::move(cp)});
                while (g_plans.size() > kMaxPlans) g_plans.pop_back();
                return g_plans.front().plan.get();
            }
        }
        cp->stage.reserve(std::max<size_t>(off, 256));
        staged_ranges = ranges;
        remapped.reserve(jobs.size() * 2);
        k = 0;
        for (auto& j : pj) {
            if (!on_dev[k++]) {
                remapped.push_back(remap(*j.A, ranges, static_cast<char*>(cp->stage.p)));
                j.A = &remapped.back();
            }
            if (!on_dev[k++]) {
                remapped.push_back(remap(*j.C, ranges, static_cast<char*>(cp->stage.p)));
                j.C = &remapped.back();
            }
        }
    }
    t_resid = now() - t0;
    cp->p = plan_jobs(pj, c, dc.main);
    const plan& p = *cp->p;
    t_plan = now() - t0 - t_resid;
    g_stats.plan_ms += t_plan;
    if (cp->staged) {
        // A C-only range needs no upload when the kernels overwrite every byte of it: one job's
        // C blocks only, no op reading C (beta = 0), and the ops' writes (disjoint: each C
        // element is written once per job) add up to the whole range.
        const size_t E = dtype_size(p.dtype);
        const uintptr_t base = reinterpret_cast<uintptr_t>(cp->stage.p);
        std::vector<size_t> written(staged_ranges.size(), 0);
        std::vector<bool> reads_c(staged_ranges.size(), false);
        auto account = [&](const std::vector<costa_tile_op_t>& ops) {
            for (const auto& op : ops) {
                if (op.dst < base) continue;  // device-resident destination
                const size_t off = size_t(op.dst - base);
                auto it = std::upper_bound(staged_ranges.begin(), staged_ranges.end(), off,
                                           [](size_t v, const hrange& r) { return v < r.dev_off; });
                if (it == staged_ranges.begin()) continue;
                const size_t i = size_t(it - staged_ranges.begin()) - 1;
                if (off >= staged_ranges[i].dev_off + (staged_ranges[i].hi - staged_ranges[i].lo))
                    continue;
                written[i] += size_t(op.nf) * size_t(op.ns) * E;
                if (((op.flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT) == COSTA_SCALE_AXPBY)
                    reads_c[i] = true;
            }
        };
        account(p.local_ops);
        account(p.unpack_ops);
        for (size_t i = 0; i < staged_ranges.size(); ++i) {
            const hrange& r = staged_ranges[i];
            const uint8_t f = range_flags[i];
            const bool overwritten = f == 2 && !reads_c[i] && written[i] == r.hi - r.lo;
            if ((f & 1) || ((f & 2) && !overwritten)) cp->h2d_ranges.push_back(r);
            if (f & 2) cp->d2h_ranges.push_back(r);
        }
    }
    cp->tr_local = any_transpose(p.local_ops);
    cp->ax_local = any_axpby(p.local_ops);
    std::vector<costa_tile_op_t> ord_l;
    std::vector<uint64_t> w_l;
    // the destination-block groups of long lists are built on the GPU and stay there (sec_*)
    auto section = [&] {
        device_section d;
        d.device = c->device;
        d.stream = dc.main;
        return d;
    };
    device_section sec_l = section();
    cp->l_local = build_work(p.dtype, p.local_ops, ord_l, w_l, list_local, &sec_l);
    // exchange rounds: pack ops go to the round of their first element (every element a round
    // sends is packed by then), unpack ops to the round of their last (every element they read
    // has arrived)
    const int R = c->nccl ? exchange_rounds() : 1;
    std::vector<std::vector<costa_tile_op_t>> pk(static_cast<size_t>(R)), up(static_cast<size_t>(R));
    {
        std::vector<int> pr, ur;
        exchange_round_of_ops(p, R, pr, ur);
        for (size_t i = 0; i < p.pack_ops.size(); ++i) pk[size_t(pr[i])].push_back(p.pack_ops[i]);
        for (size_t i = 0; i < p.unpack_ops.size(); ++i) up[size_t(ur[i])].push_back(p.unpack_ops[i]);
    }
    std::vector<std::vector<costa_tile_op_t>> ord_p(static_cast<size_t>(R)), ord_u(static_cast<size_t>(R));
    std::vector<std::vector<uint64_t>> w_p(static_cast<size_t>(R)), w_u(static_cast<size_t>(R));
    std::vector<device_section> sec_u(static_cast<size_t>(R), section());
    for (int r = 0; r < R; ++r) {
        auto x = std::make_unique<cached_plan::xround>();
        x->tr_unpack = any_transpose(up[size_t(r)]);
        x->ax_unpack = any_axpby(up[size_t(r)]);
        x->l_pack = build_work(p.dtype, pk[size_t(r)], ord_p[size_t(r)], w_p[size_t(r)], list_pack);
        x->l_unpack = build_work(p.dtype, up[size_t(r)], ord_u[size_t(r)], w_u[size_t(r)], list_unpack,
                                 &sec_u[size_t(r)]);
        cp->rounds.push_back(std::move(x));
    }
    t_work = now() - t0 - t_resid - t_plan;
    upload_list(cp->d_local, ord_l, sec_l.d_ordered, sec_l.at_ordered, sec_l.n_ordered, dc.main);
    upload_list(cp->w_local, w_l, sec_l.d_work, sec_l.at_work, sec_l.n_work, dc.main);
    for (int r = 0; r < R; ++r) {
        auto& x = *cp->rounds[size_t(r)];
        const device_section& su = sec_u[size_t(r)];
        x.d_pack.upload(ord_p[size_t(r)], dc.main);
        x.w_pack.upload(w_p[size_t(r)], dc.main);
        upload_list(x.d_unpack, ord_u[size_t(r)], su.d_ordered, su.at_ordered, su.n_ordered, dc.main);
        upload_list(x.w_unpack, w_u[size_t(r)], su.d_work, su.at_work, su.n_work, dc.main);
    }
    HIP_CHECK(hipStreamSynchronize(dc.main));  // host vectors above are temporaries
    if (trace)
        std::fprintf(stderr,
                     "[costa plan] %zu local / %zu pack / %zu unpack ops: residency %.2f ms, "
                     "planning %.2f, work lists %.2f, upload %.2f, total %.2f\n",
                     p.local_ops.size(), p.pack_ops.size(), p.unpack_ops.size(), t_resid, t_plan,
                     t_work, now() - t0 - t_resid - t_plan - t_work, now() - t0);

    g_plans.push_front({h.h, std::move(key), std::move(cp)});
    while (g_plans.size() > kMaxPlans) g_plans.pop_back();
    return g_plans.front().plan.get();
}

void upload_scalars(cached_plan& cp, const std::vector<job>& jobs, hipStream_t s) {
    const size_t E = dtype_size(cp.p->dtype);
    std::vector<unsigned char> host(jobs.size() * 2 * E);
    for (size_t t = 0; t < jobs.size(); ++t) {
        std::memcpy(&host[(2 * t) * E], jobs[t].s.alpha.data(), E);
        std::memcpy(&host[(2 * t + 1) * E], jobs[t].s.beta.data(), E);
    }
    if (host != cp.scal_host || !cp.d_scal.p) {
        // stream-ordered behind earlier (possibly asynchronous) transforms that still read the
        // old values; pageable source -> the runtime stages it before returning
        cp.d_scal.reserve(host.size());
        cp.scal_host = host;
        HIP_CHECK(hipMemcpyAsync(cp.d_scal.p, cp.scal_host.data(), host.size(),
                                 hipMemcpyHostToDevice, s));
    }
}

}  // namespace

void release_caches() {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    g_plans.clear();
    release_host_rings();
    ctx_map().clear();
}

// ---------------------------------------------------------------- transform
// Phases are bracketed by pooled event pairs on the stream they run on; the pairs are
// resolved (elapsed time added to the statistics) at the next synchronisation point, so
// asynchronous transforms are timed too.
namespace {
enum phase { PH_LOCAL, PH_PACK, PH_EXCHANGE, PH_UNPACK, PH_H2D, PH_D2H };

struct phase_timer {
    device_ctx& dc;
    bool on;
    int ph = 0;
    hipEvent_t a = nullptr;
    hipStream_t s = nullptr;
    phase_timer(device_ctx& d, bool prof) : dc(d), on(prof) {}
    void start(int p, hipStream_t st) {
        if (!on) return;
        ph = p;
        s = st;
        a = dc.take_event();
        HIP_CHECK(hipEventRecord(a, s));
    }
    void stop() {
        if (!on || !a) return;
        hipEvent_t b = dc.take_event();
        HIP_CHECK(hipEventRecord(b, s));
        dc.pending.push_back({ph, a, b});
        a = nullptr;
        if (dc.pending.size() > 1024) dc.resolve(64);
    }
};
}  // namespace

void device_ctx::resolve(size_t max_n) {
    size_t n = 0;
    while (!pending.empty() && n < max_n) {
        timed t = pending.front();
        pending.pop_front();
        float ms = 0.f;
        HIP_CHECK(hipEventSynchronize(t.b));
        HIP_CHECK(hipEventElapsedTime(&ms, t.a, t.b));
        double* acc[] = {&g_stats.local_ms, &g_stats.pack_ms, &g_stats.exchange_ms,
                         &g_stats.unpack_ms, &g_stats.h2d_ms, &g_stats.d2h_ms};
        *acc[t.phase] += ms;
        free_events.push_back(t.a);
        free_events.push_back(t.b);
        ++n;
    }
}

hipEvent_t device_ctx::take_event() {
    if (free_events.empty()) {
        hipEvent_t e;
        HIP_CHECK(hipEventCreate(&e));
        return e;
    }
    hipEvent_t e = free_events.back();
    free_events.pop_back();
    return e;
}

void resolve_pending() {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    for (auto& kv : ctx_map()) {
        HIP_CHECK(hipSetDevice(kv.first));
        kv.second->resolve();
    }
}

void synchronize(comm* c) {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    if (!c) throw error(COSTA_ERR_ARG, "costa: null communicator");
    device_ctx& dc = ctx(c->device);
    HIP_CHECK(hipStreamSynchronize(dc.main));
    HIP_CHECK(hipStreamSynchronize(dc.aux));
    HIP_CHECK(hipStreamSynchronize(dc.xch));
    dc.resolve();
}

namespace {
// The exchange: one RCCL group of ncclSend / ncclRecv, one pair per peer, at the reference's
// displacements (communication_data.cpp:152-154).  Each peer's package moves as pieces of at
// most max_message_bytes(): RCCL was measured to lose the second half of a single >1 GiB self
// send/recv (tools/loopback_probe.py); pieces to one peer match in issue order on both sides.
// Round `round` of `rounds` (exchange_rounds(); rounds = 1: everything at once).
void issue_exchange(comm* c, const plan& p, char* sb, char* rb, hipStream_t s, int round = 0,
                    int rounds = 1) {
    const size_t E = dtype_size(p.dtype);
    const size_t piece = max_message_bytes();
    NCCL_CHECK(ncclGroupStart());
    for (int q = 0; q < c->size; ++q) {
        int64_t slo, shi, rlo, rhi;
        round_range(p.send_counts[size_t(q)], E, rounds, round, slo, shi);
        round_range(p.recv_counts[size_t(q)], E, rounds, round, rlo, rhi);
        const size_t sbytes = size_t(shi - slo) * E, rbytes = size_t(rhi - rlo) * E;
        char* sp = sb + size_t(p.send_displs[size_t(q)] + slo) * E;
        char* rp = rb + size_t(p.recv_displs[size_t(q)] + rlo) * E;
        for (size_t o = 0; o < sbytes; o += piece)
            NCCL_CHECK(ncclSend(sp + o, std::min(piece, sbytes - o), ncclUint8, q, c->nccl, s));
        for (size_t o = 0; o < rbytes; o += piece)
            NCCL_CHECK(ncclRecv(rp + o, std::min(piece, rbytes - o), ncclUint8, q, c->nccl, s));
    }
    NCCL_CHECK(ncclGroupEnd());
}
}  // namespace

void transform(const std::vector<job>& jobs, comm* c, void* user_stream, bool async) {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    if (!c) throw error(COSTA_ERR_ARG, "costa: null communicator");
    device_ctx& dc = ctx(c->device);
    cached_plan& cp = *get_plan(jobs, c, dc);
    const plan& p = *cp.p;
    const size_t E = dtype_size(p.dtype);
    if (async && (cp.staged || cp.pipe))
        throw error(COSTA_ERR_ARG,
                    "costa: asynchronous transforms need device-resident layouts (host data is "
                    "staged synchronously)");
    hipStream_t user = static_cast<hipStream_t>(user_stream);
    // everything runs on the context's streams, in call order (they own the workspaces);
    // a caller stream is joined at entry and made to wait for the result at exit
    if (user) {
        HIP_CHECK(hipEventRecord(dc.ev_user, user));
        HIP_CHECK(hipStreamWaitEvent(dc.main, dc.ev_user, 0));
    }
    upload_scalars(cp, jobs, dc.main);
    if (cp.pipe) {  // host-resident: pipelined gather -> H2D -> [exchange] -> kernels -> D2H
        const bool xchg = c->nccl != nullptr && (p.send_elems > 0 || p.recv_elems > 0);
        char *sb = nullptr, *rb = nullptr;
        std::function<void(void*, int)> fn;
        if (xchg) {
            dc.send.reserve(size_t(p.send_elems) * E + 256);
            dc.recv.reserve(size_t(p.recv_elems) * E + 256);
            sb = static_cast<char*>(dc.send.p);
            rb = static_cast<char*>(dc.recv.p);
            const int R = exchange_rounds();
            fn = [&, R](void* s, int r) {
                issue_exchange(c, p, sb, rb, static_cast<hipStream_t>(s), r, R);
            };
        }
        // tile kernels on the aux stream, behind the scalars uploaded on main; the exchange on main
        HIP_CHECK(hipEventRecord(dc.ev_ready, dc.main));
        HIP_CHECK(hipStreamWaitEvent(dc.aux, dc.ev_ready, 0));
        run_host_pipeline(*cp.pipe, c->device, dc.aux, dc.main, sb, rb, fn, cp.d_scal.p);
        g_stats.transforms++;
        return;
    }
    phase_timer tm(dc, g_profiling);

    // H2D of host-resident data
    if (cp.staged) {
        tm.start(PH_H2D, dc.main);
        for (const auto& r : cp.h2d_ranges)
            HIP_CHECK(hipMemcpyAsync(static_cast<char*>(cp.stage.p) + r.dev_off,
                                     reinterpret_cast<void*>(r.lo), r.hi - r.lo,
                                     hipMemcpyHostToDevice, dc.main));
        tm.stop();
    }

    const bool exchange = c->nccl != nullptr && (p.send_elems > 0 || p.recv_elems > 0);
    // LOCAL on the aux stream when there is an exchange to overlap, else on main
    hipStream_t ls = exchange ? dc.aux : dc.main;
    if (exchange) {
        HIP_CHECK(hipEventRecord(dc.ev_ready, dc.main));
        HIP_CHECK(hipStreamWaitEvent(dc.aux, dc.ev_ready, 0));
    }
    if (cp.l_local.n_items()) {
        tm.start(PH_LOCAL, ls);
        launch_tiles(p.dtype,
                     make_launch(cp.l_local, cp.d_local.p, cp.w_local.p, nullptr, nullptr,
                                 cp.d_scal.p, cp.tr_local, cp.ax_local),
                     ls);
        tm.stop();
    }

    if (exchange) {
        dc.send.reserve(size_t(p.send_elems) * E + 256);
        dc.recv.reserve(size_t(p.recv_elems) * E + 256);
        char* sb = static_cast<char*>(dc.send.p);
        char* rb = static_cast<char*>(dc.recv.p);
        // main: pack round r -> the exchange stream moves round r -> aux (after LOCAL): unpack
        // round r; so packing r+1, moving r and unpacking r-1 overlap
        const int R = int(cp.rounds.size());
        dc.round_events(size_t(R));
        for (int r = 0; r < R; ++r) {
            const auto& x = *cp.rounds[size_t(r)];
            if (x.l_pack.n_items()) {
                tm.start(PH_PACK, dc.main);
                launch_tiles(p.dtype,
                             make_launch(x.l_pack, x.d_pack.p, x.w_pack.p, nullptr, sb, cp.d_scal.p,
                                         false, false),
                             dc.main);
                tm.stop();
            }
            HIP_CHECK(hipEventRecord(dc.ev_packed[size_t(r)], dc.main));
            HIP_CHECK(hipStreamWaitEvent(dc.xch, dc.ev_packed[size_t(r)], 0));
            tm.start(PH_EXCHANGE, dc.xch);
            issue_exchange(c, p, sb, rb, dc.xch, r, R);
            tm.stop();
            HIP_CHECK(hipEventRecord(dc.ev_moved[size_t(r)], dc.xch));
        }
        for (int r = 0; r < R; ++r) {
            const auto& x = *cp.rounds[size_t(r)];
            if (!x.l_unpack.n_items()) continue;
            HIP_CHECK(hipStreamWaitEvent(dc.aux, dc.ev_moved[size_t(r)], 0));
            tm.start(PH_UNPACK, dc.aux);
            launch_tiles(p.dtype,
                         make_launch(x.l_unpack, x.d_unpack.p, x.w_unpack.p, rb, nullptr,
                                     cp.d_scal.p, x.tr_unpack, x.ax_unpack),
                         dc.aux);
            tm.stop();
        }
        // the call ends on main once LOCAL, every unpack and every round of the exchange are done
        HIP_CHECK(hipEventRecord(dc.ev_local, dc.aux));
        HIP_CHECK(hipStreamWaitEvent(dc.main, dc.ev_local, 0));
        HIP_CHECK(hipStreamWaitEvent(dc.main, dc.ev_moved[size_t(R - 1)], 0));
    }

    // D2H of the target data
    if (cp.staged) {
        tm.start(PH_D2H, dc.main);
        for (const auto& r : cp.d2h_ranges)
            HIP_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(r.lo),
                                     static_cast<char*>(cp.stage.p) + r.dev_off, r.hi - r.lo,
                                     hipMemcpyDeviceToHost, dc.main));
        tm.stop();
    }

    g_stats.transforms++;
    auto count_items = [&](const work_split& w) {
        g_stats.tile_items += w.n_large + w.n_medium;
        g_stats.skew_items += w.n_skew;
        g_stats.cblock_items += w.n_cblock;
        g_stats.tiny_items += w.n_tiny;
        if (!dtype_is_complex(p.dtype) && pieces_in_group_launch(w.n_cblock, w.n_tiny))
            g_stats.fused_pieces += w.n_tiny;
    };
    if (cp.l_local.n_items()) {
        g_stats.local_launches++;
        g_stats.local_bytes += p.local_bytes;
        count_items(cp.l_local);
    }
    if (exchange) {
        for (const auto& x : cp.rounds) {
            g_stats.pack_launches += x->l_pack.n_items() ? 1 : 0;
            g_stats.unpack_launches += x->l_unpack.n_items() ? 1 : 0;
            count_items(x->l_pack);
            count_items(x->l_unpack);
        }
        g_stats.pack_bytes += p.pack_bytes;
        g_stats.unpack_bytes += p.unpack_bytes;
    }

    if (async) {
        if (user) {  // (no marker without a caller stream: each one widened the gap between calls)
            HIP_CHECK(hipEventRecord(dc.ev_done, dc.main));
            HIP_CHECK(hipStreamWaitEvent(user, dc.ev_done, 0));
        }
        return;
    }
    HIP_CHECK(hipStreamSynchronize(dc.main));
    dc.resolve();
}


// ---------------------------------------------------------------- direct tile calls
void execute_tiles(costa_dtype_t dtype, const costa_tile_op_t* ops, int64_t n,
                   const void* src_base, void* dst_base, const void* scalars, int n_slots,
                   int device) {
    std::lock_guard<std::recursive_mutex> lk(g_mutex);
    device_ctx& dc = ctx(device);
    std::vector<costa_tile_op_t> v(ops, ops + n);
    for (const auto& op : v)
        if ((op.flags >> COSTA_SLOT_SHIFT) >= uint32_t(std::max(n_slots, 0)))
            throw error(COSTA_ERR_ARG, "costa_hip_execute_tiles: scalar slot out of range");
    std::vector<costa_tile_op_t> ord;
    std::vector<uint64_t> w;
    const work_split nl = build_work(dtype, v, ord, w);
    dbuf d_ops, d_work, d_scal;
    d_ops.upload(ord, dc.main);
    d_work.upload(w, dc.main);
    const size_t E = dtype_size(dtype);
    std::vector<unsigned char> sc(static_cast<const unsigned char*>(scalars),
                                  static_cast<const unsigned char*>(scalars) + size_t(n_slots) * 2 * E);
    d_scal.upload(sc, dc.main);
    launch_tiles(dtype,
                 make_launch(nl, d_ops.p, d_work.p, static_cast<const char*>(src_base),
                             static_cast<char*>(dst_base), d_scal.p, any_transpose(v),
                             any_axpby(v)),
                 dc.main);
    HIP_CHECK(hipStreamSynchronize(dc.main));
}

void copy_and_transform(costa_dtype_t dtype, int n_rows, int n_cols, const void* src,
                        int src_stride, bool src_cm, void* dst, int dst_stride, bool dst_cm,
                        bool trans, bool conj, const void* alpha, const void* beta) {
    if (n_rows < 0 || n_cols < 0 || src_stride < 0 || dst_stride < 0)
        throw error(COSTA_ERR_ARG, "costa_hip_copy_and_transform: negative size or stride");
    if (size_t(n_rows) * size_t(n_cols) == 0) return;  // memory_utils.hpp:72-74
    const size_t E = dtype_size(dtype);
    scal s;
    std::memcpy(s.alpha.data(), alpha, E);
    std::memcpy(s.beta.data(), beta, E);
    const bool cj = conj && dtype_is_complex(dtype);
    const bool wt = (trans && src_cm == dst_cm) || (!trans && src_cm != dst_cm);
    costa_tile_op_t op = make_tile_op(n_rows, n_cols, reinterpret_cast<uintptr_t>(src), src_stride,
                                      src_cm, reinterpret_cast<uintptr_t>(dst), dst_stride, dst_cm,
                                      trans, cj, scale_kind(dtype, s, !wt, cj), 0, E);
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    std::vector<unsigned char> sc(2 * E);
    std::memcpy(sc.data(), alpha, E);
    std::memcpy(sc.data() + E, beta, E);
    execute_tiles(dtype, &op, 1, nullptr, nullptr, sc.data(), 1, dev);
}

}  // namespace engine
}  // namespace costa
