// Host-resident transforms as a pipeline over PCIe.
//
// The reference's path starts and ends in host memory (each rank's local matrix buffer).  The
// mirror scheme of engine.cpp uploads every byte range a layout spans, runs the kernels, and
// copies the target ranges back: one direction at a time, so a call costs H2D + D2H.  Here the
// tile ops are cut into groups of at most kSlot bytes of source and target data, and each group
// moves through a ring of slots:
//
//   host threads : gather the group's source tiles (and, for beta != 0, its old target tiles)
//                  densely into a pinned slot                         [the reference's PACK
//                  format, communication_data.cpp:191-217: stored shape, dense]
//   copy stream 1: pinned slot -> device slot (H2D)
//   compute      : the tile kernels, rewritten to read the dense source package and write a
//                  dense target package (copy_and_transform of every tile, on the GPU)
//   copy stream 2: device target package -> pinned slot (D2H)
//   host threads : scatter the target package into the caller's C
//
// so H2D of group g+1, the kernels of group g and D2H of group g-1 overlap: the two copy
// directions run at the same time (PCIe is full duplex only from pinned memory: 56 GB/s for
// H2D and D2H together from pageable memory, 97 GB/s from pinned, tools/pcie_probe.hip,
// profiles/r07/pcie_probe.log).  Device memory needed: the ring, not a mirror of A and C.
// Only C bytes the ops write are ever stored to the caller's memory.  The host threads move
// bytes only (strided memcpy); every element's transform runs in the tile kernels.
//
// With an exchange (several ranks, the ScaLAPACK situation) the groups come in three kinds, in
// this order (the reference's exchange_async, transform.cpp:46-128):
//   PACK   the host gather IS the pack (a bit copy into the dense package): it goes straight
//          into the device send buffer; after a round's last pack group its RCCL group starts
//   LOCAL  as above, on the compute stream, overlapping the exchange
//   UNPACK the unpack kernels read the receive buffer once their round has arrived and write
//          dense target packages, copied back and scattered like LOCAL ones
// in the order PACK(0) | LOCAL, PACK(1) | UNPACK(0), ..., UNPACK(R-1) over the exchange rounds
// (engine.cpp exchange_rounds(); "|": alternating group by group), so the uploads of one round
// and the downloads of the previous one share the ring.
#include <emmintrin.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <mutex>
#include <thread>

#include "engine.hpp"

namespace costa {
namespace engine {

#define HP_CHECK(x)                                                                    \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess)                                                          \
            throw error(COSTA_ERR_HIP, std::string(#x " failed: ") + hipGetErrorString(e_)); \
    } while (0)

namespace {

// source (and target) bytes per group; COSTA_HOST_SLOT_MIB overrides (tuning, COSTA_TUNING=1)
const size_t kSlot = [] {
    const char* s = tuning_env("COSTA_HOST_SLOT_MIB");
    const long v = s ? std::atol(s) : 64;
    return size_t(std::max(1L, std::min(1024L, v))) << 20;
}();
constexpr int kRing = 4;                      // slots in flight
constexpr int kLag = 3;                       // scatter of group g runs at step g + kLag
static_assert(kLag < kRing, "a pinned target slot is scattered before its reuse");
constexpr size_t kItemBytes = size_t(256) << 10;  // host copy work item
constexpr size_t kAlign = 256;
constexpr int kMaxRounds = 16;                // exchange rounds (engine.cpp exchange_rounds())

size_t align_up(size_t x) { return (x + kAlign - 1) & ~(kAlign - 1); }

// Copy n bytes, storing whole 16-byte blocks of the destination with streaming (non-temporal)
// stores: neither the pinned packages nor the caller's C are read again by this host, and a
// streaming store skips the read-for-ownership of the line.  The caller fences.
inline void copy_nt(char* dst, const char* src, size_t n) {
    if (n < 256) {
        std::memcpy(dst, src, n);
        return;
    }
    const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
    std::memcpy(dst, src, head);
    dst += head;
    src += head;
    n -= head;
    const size_t body = n & ~size_t(63);
    for (size_t i = 0; i < body; i += 64) {
        const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
        const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
        const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
        const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
        _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
    std::memcpy(dst + body, src + body, n - body);
}

// ---------------------------------------------------------------- host thread pool
class pool {
  public:
    explicit pool(int n) {
        for (int i = 0; i < n - 1; ++i) th_.emplace_back([this] { loop(); });
    }
    ~pool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    // run f(0..n-1) on the workers and the calling thread; returns when all are done
    void run(size_t n, const std::function<void(size_t)>& f) {
        if (n == 0) return;
        if (th_.empty() || n == 1) {
            for (size_t i = 0; i < n; ++i) f(i);
            return;
        }
        {
            std::lock_guard<std::mutex> lk(m_);
            fn_ = &f;
            n_ = n;
            next_.store(0);
            busy_ = th_.size();
            ++gen_;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(m_);
        done_.wait(lk, [this] { return busy_ == 0; });
        fn_ = nullptr;
    }

  private:
    void work() {
        for (size_t i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
            }
            work();
            std::lock_guard<std::mutex> lk(m_);
            if (--busy_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    size_t busy_ = 0;
    uint64_t gen_ = 0;
    bool stop_ = false;
};

int host_threads() {
    if (const char* s = tuning_env("COSTA_HOST_THREADS")) return std::max(1, std::atoi(s));
    const int hw = int(std::thread::hardware_concurrency());
    return std::max(1, std::min(16, hw));
}

pool& thread_pool() {  // never destroyed: its threads outlive static destruction at exit
    static pool* p = new pool(host_threads());
    return *p;
}

// ---------------------------------------------------------------- per-device ring
struct ring {
    int device = 0;
    size_t slot = 0;          // bytes of one package; at most kSlot, sized to the largest group
    hipStream_t up = nullptr, down = nullptr;
    hipStream_t pk = nullptr;  // direct PACK groups' pack kernels (not behind earlier exchange
                               // rounds on the exchange stream: ADVICE r5)
    char* pin_in = nullptr;   // kRing x 2*slot: [source package | old target package]
    char* pin_out = nullptr;  // kRing x slot: target package
    char* dev = nullptr;      // kRing x 2*slot: [source package | target package]
    hipEvent_t up_done[kRing]{}, kern_done[kRing]{}, down_done[kRing]{};
    hipEvent_t packed[kMaxRounds]{}, moved[kMaxRounds]{};  // per exchange round: its part of
                                                             // the send buffer uploaded / moved
    hipEvent_t packed_k[kMaxRounds]{};  // ... and packed by the direct groups' kernels (on pk)
    ring(int d, size_t slot_bytes) : device(d), slot(slot_bytes) {
        HP_CHECK(hipStreamCreateWithFlags(&up, hipStreamNonBlocking));
        HP_CHECK(hipStreamCreateWithFlags(&down, hipStreamNonBlocking));
        HP_CHECK(hipStreamCreateWithFlags(&pk, hipStreamNonBlocking));
        HP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&pin_in), kRing * 2 * slot, hipHostMallocDefault));
        HP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&pin_out), kRing * slot, hipHostMallocDefault));
        HP_CHECK(hipMalloc(reinterpret_cast<void**>(&dev), kRing * 2 * slot));
        for (int k = 0; k < kRing; ++k)
            for (hipEvent_t* e : {&up_done[k], &kern_done[k], &down_done[k]})
                HP_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
        for (int r = 0; r < kMaxRounds; ++r) {
            HP_CHECK(hipEventCreateWithFlags(&packed[r], hipEventDisableTiming));
            HP_CHECK(hipEventCreateWithFlags(&packed_k[r], hipEventDisableTiming));
            HP_CHECK(hipEventCreateWithFlags(&moved[r], hipEventDisableTiming));
        }
    }
    ~ring() {
        (void)hipSetDevice(device);
        (void)hipStreamSynchronize(up);
        (void)hipStreamSynchronize(down);
        (void)hipStreamSynchronize(pk);
        for (int k = 0; k < kRing; ++k)
            for (hipEvent_t e : {up_done[k], kern_done[k], down_done[k]}) (void)hipEventDestroy(e);
        for (int r = 0; r < kMaxRounds; ++r) {
            (void)hipEventDestroy(packed[r]);
            (void)hipEventDestroy(packed_k[r]);
            (void)hipEventDestroy(moved[r]);
        }
        (void)hipFree(dev);
        (void)hipHostFree(pin_in);
        (void)hipHostFree(pin_out);
        (void)hipStreamDestroy(up);
        (void)hipStreamDestroy(down);
        (void)hipStreamDestroy(pk);
    }
};

std::map<int, std::unique_ptr<ring>>& rings() {  // freed by release_caches(), not at exit
    static auto* m = new std::map<int, std::unique_ptr<ring>>;
    return *m;
}

// the device's ring, reallocated when a pipeline needs larger slots than it has: a small
// host-resident call pins a few MiB, not kRing x 3 x kSlot
ring& ring_of(int device, size_t slot_bytes) {
    auto& m = rings();
    auto it = m.find(device);
    if (it != m.end() && it->second->slot < slot_bytes) {
        m.erase(it);  // the destructor waits for the ring's copy streams
        it = m.end();
    }
    if (it == m.end()) it = m.emplace(device, std::make_unique<ring>(device, slot_bytes)).first;
    return *it->second;
}

}  // namespace

void release_host_rings() { rings().clear(); }

// ---------------------------------------------------------------- the pipeline of one plan
struct host_pipeline {
    enum kind_t { PACK, LOCAL, UNPACK };
    struct rect {         // h rows of w elements at a stride of pitch elements from host address base
        uintptr_t base = 0;
        int64_t w = 0, h = 0, pitch = 0;
    };
    struct hop {          // one op (or piece of one) with its host addresses
        costa_tile_op_t op;
        uint64_t in_off, out_off;  // offsets in the group's source / target packages
    };
    struct item {         // host copy work item: rows [lo, hi) of op `k`'s slow dimension
        uint32_t k;
        int32_t lo, hi;
    };
    struct group {
        kind_t kind = LOCAL;
        int round = 0;                // PACK / UNPACK: its exchange round
        size_t first = 0, count = 0;  // hops
        size_t in_bytes = 0, out_bytes = 0;
        uint64_t send_off = 0;        // PACK: the group's byte range starts here in the send buffer
        bool reads_old = false;
        std::vector<item> gather, scatter;  // scatter items double as old-target gathers
        work_split split;
        size_t ord_first = 0, work_first = 0;
        bool any_tr = false;
        int64_t alg_bytes = 0;
        // direct mode (page-locked caller memory): the group's host footprints -- the source of
        // a PACK group, the target of an UNPACK group, both of a LOCAL one -- as rectangles of
        // the caller's arrays, each moved by one strided DMA into / out of a dense device image,
        // and the op list that reads / writes those images (build_direct)
        bool direct = false;
        rect src_rect, dst_rect;
        work_split split_d;
        size_t ord_first_d = 0, work_first_d = 0;
        bool any_tr_d = false;
    };
    costa_dtype_t dtype = COSTA_DOUBLE;
    size_t E = 8;
    std::vector<hop> hops;
    // execution order (make_host_pipeline): PACK(0) | LOCAL, PACK(r) | UNPACK(r-1) for
    // r = 1..R-1, UNPACK(R-1), "|" alternating group by group
    std::vector<group> groups;
    int rounds = 1;
    size_t slot_bytes = 0;            // ring slot the largest package needs (<= kSlot)
    int rounds_before = 0;           // exchange rounds issued before the first group
    std::vector<int> rounds_after;    // ... issued once group t is enqueued (cumulative)
    void* d_ops = nullptr;   // every group's ordered device ops (package offsets)
    void* d_work = nullptr;
    // direct mode, built on the first call that finds the caller's memory page-locked
    bool direct_built = false;
    size_t n_direct = 0;      // groups whose footprints are rectangles
    void* d_ops_d = nullptr;  // ... and their device ops (image offsets)
    void* d_work_d = nullptr;
    // the caller's host byte ranges the ops read or write (merged): when all of them are
    // page-locked the pipeline moves tiles by strided DMA instead of host copies
    std::vector<std::pair<uintptr_t, uintptr_t>> host_ranges;
    ~host_pipeline() {
        for (void* p : {d_ops, d_work, d_ops_d, d_work_d})
            if (p) (void)hipFree(p);
    }
};

namespace {

// contiguous run length and count of the target side of an op (copy: columns of nf elements;
// transpose: rows of ns elements)
inline void target_shape(const costa_tile_op_t& op, int64_t& run, int64_t& runs) {
    const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
    run = tr ? op.ns : op.nf;
    runs = tr ? op.nf : op.ns;
}

void add_items(std::vector<host_pipeline::item>& v, uint32_t k, int64_t run_bytes, int64_t runs) {
    const int64_t per = std::max<int64_t>(1, int64_t(kItemBytes) / std::max<int64_t>(1, run_bytes));
    for (int64_t lo = 0; lo < runs; lo += per)
        v.push_back({k, int32_t(lo), int32_t(std::min(runs, lo + per))});
}

// cut an op into pieces of at most one slot (a sub-rectangle of a tile op is a tile op); pack
// ops are cut into whole columns only, so that every piece stays one contiguous range of the
// dense send package
void cut(const costa_tile_op_t& op, size_t E, bool whole_columns, std::vector<costa_tile_op_t>& out) {
    if (op.nf <= 0 || op.ns <= 0) return;
    if (align_up(size_t(op.nf) * size_t(op.ns) * E) <= kSlot) {
        out.push_back(op);
        return;
    }
    const int64_t cap = int64_t((kSlot - kAlign) / E);  // elements per piece
    const bool tr = op.flags & COSTA_TILE_TRANSPOSE;
    const int64_t cf = std::min<int64_t>(op.nf, cap);
    if (whole_columns && cf < op.nf) throw error(COSTA_ERR_INTERNAL, "costa: pack column over a slot");
    const int64_t cs = std::max<int64_t>(1, cap / cf);
    for (int64_t f0 = 0; f0 < op.nf; f0 += cf)
        for (int64_t s0 = 0; s0 < op.ns; s0 += cs) {
            costa_tile_op_t p = op;
            p.nf = int32_t(std::min<int64_t>(cf, op.nf - f0));
            p.ns = int32_t(std::min<int64_t>(cs, op.ns - s0));
            p.src = op.src + uint64_t((s0 * op.lds + f0) * int64_t(E));
            p.dst = op.dst + uint64_t((tr ? f0 * op.ldd + s0 : s0 * op.ldd + f0) * int64_t(E));
            out.push_back(p);
        }
}

}  // namespace

// The union of footprints (h rows of w elements at address a, stride pitch; one per hop) as one
// rectangle of the caller's array: every footprint must share the pitch and lie on the same 2D
// grid as the first, and together they must tile their bounding box exactly (the ops of a
// transform are disjoint, so equal areas suffice).  Returns false otherwise.
struct foot {
    uintptr_t a;
    int64_t w, h, pitch;
};
bool rectangle_of(const std::vector<foot>& f, size_t E, host_pipeline::rect& r,
                  std::vector<std::pair<int64_t, int64_t>>& xy) {
    if (f.empty()) return false;
    const int64_t P = f[0].pitch;
    int64_t x0 = INT64_MAX, x1 = INT64_MIN, y0 = INT64_MAX, y1 = INT64_MIN, area = 0;
    xy.clear();
    for (const auto& q : f) {
        if (q.pitch != P || P <= 0 || q.w > P) return false;
        const int64_t d = int64_t(q.a) - int64_t(f[0].a);
        if (d % int64_t(E)) return false;
        const int64_t e = d / int64_t(E);
        const int64_t y = e >= 0 ? e / P : -((-e + P - 1) / P), x = e - y * P;
        if (x + q.w > P) return false;
        xy.push_back({x, y});
        x0 = std::min(x0, x), x1 = std::max(x1, x + q.w);
        y0 = std::min(y0, y), y1 = std::max(y1, y + q.h);
        area += q.w * q.h;
    }
    if (area != (x1 - x0) * (y1 - y0)) return false;
    r.base = uintptr_t(int64_t(f[0].a) + (y0 * P + x0) * int64_t(E));
    r.w = x1 - x0, r.h = y1 - y0, r.pitch = P;
    for (auto& p : xy) p = {p.first - x0, p.second - y0};  // position inside the rectangle
    return true;
}

bool host_pipeline_accepts(costa_dtype_t dtype, const std::vector<costa_tile_op_t>& pack_ops) {
    const size_t E = dtype_size(dtype);
    for (const auto& op : pack_ops)
        if (size_t(op.nf) * E > kSlot - kAlign) return false;
    return true;
}

std::shared_ptr<host_pipeline> make_host_pipeline(costa_dtype_t dtype,
                                                  const std::vector<costa_tile_op_t>& pack_ops,
                                                  const std::vector<costa_tile_op_t>& local_ops,
                                                  const std::vector<costa_tile_op_t>& unpack_ops,
                                                  const std::vector<int>& pack_round,
                                                  const std::vector<int>& unpack_round, int rounds) {
    using hpl = host_pipeline;
    if (rounds < 1 || rounds > kMaxRounds) throw error(COSTA_ERR_ARG, "costa: exchange rounds out of range");
    auto hp = std::make_shared<hpl>();
    hp->dtype = dtype;
    hp->rounds = rounds;
    const size_t E = dtype_size(dtype);
    hp->E = E;

    // Segments: PACK(r), LOCAL, UNPACK(r); groups in list order inside a segment (the planner's
    // key order: for block-cyclic layouts a local group is a band of target rows read from a
    // band of source columns; pack groups are contiguous ranges of the send package).
    std::vector<std::pair<hpl::kind_t, int>> segs{{hpl::LOCAL, 0}};
    for (int r = 0; r < rounds; ++r) {
        segs.push_back({hpl::PACK, r});
        segs.push_back({hpl::UNPACK, r});
    }
    std::map<std::pair<int, int>, std::vector<hpl::group>> built;
    std::vector<hpl::group>* dest = nullptr;
    hpl::group g;
    auto close = [&] {
        const hpl::kind_t k = g.kind;
        const int rd = g.round;
        if (g.count) dest->push_back(std::move(g));
        g = hpl::group{};
        g.kind = k;
        g.round = rd;
        g.first = hp->hops.size();
    };
    for (const auto& sg : segs) {
        dest = &built[{int(sg.first), sg.second}];
        const hpl::kind_t kind = sg.first;
        const auto& ops = kind == hpl::PACK ? pack_ops : kind == hpl::LOCAL ? local_ops : unpack_ops;
        const auto* rd = kind == hpl::PACK ? &pack_round : kind == hpl::UNPACK ? &unpack_round : nullptr;
        std::vector<costa_tile_op_t> pieces;
        for (size_t i = 0; i < ops.size(); ++i)
            if (!rd || (*rd)[i] == sg.second) cut(ops[i], E, kind == hpl::PACK, pieces);
        close();
        g.kind = kind;
        g.round = sg.second;
        // LOCAL: pieces come in target row-band order (the planner's key order); a band is a run
        // of pieces whose targets cover the same rows of one array.  A group takes whole bands
        // while they fit, so that its footprints stay rectangles of the caller's arrays (direct
        // mode, below); a band larger than a slot is cut piece by piece as before.
        std::vector<size_t> band_end(pieces.size(), 0);
        if (kind == hpl::LOCAL) {
            size_t b0 = 0;
            auto xrange = [&](const costa_tile_op_t& q, int64_t& x, int64_t& w) {
                int64_t run, runs;
                target_shape(q, run, runs);
                const int64_t e = (int64_t(q.dst) - int64_t(pieces[b0].dst)) / int64_t(E);
                const int64_t P = std::max<int64_t>(1, q.ldd);
                x = ((e % P) + P) % P;
                w = run;
            };
            for (size_t i = 0; i <= pieces.size(); ++i) {
                bool same = false;
                if (i < pieces.size() && i > b0) {
                    int64_t x, w, xb, wb;
                    xrange(pieces[i], x, w);
                    xrange(pieces[b0], xb, wb);
                    same = pieces[i].ldd == pieces[b0].ldd && x == xb && w == wb;
                }
                if (i == pieces.size() || (i > b0 && !same)) {
                    for (size_t j = b0; j < i; ++j) band_end[j] = i;
                    b0 = i;
                }
            }
        }
        for (size_t pi = 0; pi < pieces.size(); ++pi) {
            const auto& p = pieces[pi];
            if (kind == hpl::LOCAL && g.count && (pi == 0 || band_end[pi - 1] == pi)) {
                size_t bin = 0;  // a band starts here: close the group if the whole band won't fit
                for (size_t j = pi; j < band_end[pi]; ++j)
                    bin += align_up(size_t(pieces[j].nf) * size_t(pieces[j].ns) * E);
                if (bin <= kSlot && (g.in_bytes + bin > kSlot || g.out_bytes + bin > kSlot)) close();
            }
            const size_t bytes = size_t(p.nf) * size_t(p.ns) * E;
            if (kind == hpl::PACK) {  // dense; a group is one contiguous range of the package
                if (g.count && (g.in_bytes + bytes > kSlot || p.dst != g.send_off + g.in_bytes)) close();
                if (!g.count) g.send_off = p.dst;
                hp->hops.push_back({p, p.dst - g.send_off, 0});
                g.in_bytes += bytes;
            } else {
                const size_t ab = align_up(bytes);
                const size_t in = kind == hpl::LOCAL ? ab : 0;
                if (g.count && (g.in_bytes + in > kSlot || g.out_bytes + ab > kSlot)) close();
                hp->hops.push_back({p, g.in_bytes, g.out_bytes});
                g.in_bytes += in;
                g.out_bytes += ab;
            }
            ++g.count;
        }
        close();
    }
    // Execution order: PACK(0) alternating with LOCAL, then PACK(r) alternating with UNPACK(r-1)
    // for r = 1..R-1, then UNPACK(R-1): uploads and downloads alternate through the ring, so
    // both copy directions stay busy (PCIe duplex)
    auto interleave = [&](std::vector<hpl::group>& a, std::vector<hpl::group>& b) {
        for (size_t i = 0; i < std::max(a.size(), b.size()); ++i) {
            if (i < a.size()) hp->groups.push_back(std::move(a[i]));
            if (i < b.size()) hp->groups.push_back(std::move(b[i]));
        }
    };
    interleave(built[{int(hpl::PACK), 0}], built[{int(hpl::LOCAL), 0}]);
    for (int r = 1; r < rounds; ++r)
        interleave(built[{int(hpl::PACK), r}], built[{int(hpl::UNPACK), r - 1}]);
    std::vector<hpl::group> none;
    interleave(built[{int(hpl::UNPACK), rounds - 1}], none);
    // ring slot: the largest package, in 2 MiB steps
    for (const auto& gr : hp->groups)
        hp->slot_bytes = std::max(hp->slot_bytes, std::max(gr.in_bytes, gr.out_bytes));
    const size_t step = size_t(2) << 20;
    hp->slot_bytes = std::min(kSlot, std::max(step, (hp->slot_bytes + step - 1) / step * step));
    // round r of the exchange is issued once every pack group of rounds <= r is enqueued
    std::vector<int> last_pack(size_t(rounds), -1);
    for (size_t t = 0; t < hp->groups.size(); ++t)
        if (hp->groups[t].kind == hpl::PACK) last_pack[size_t(hp->groups[t].round)] = int(t);
    hp->rounds_after.assign(hp->groups.size(), 0);
    int upto = -1;
    for (int r = 0; r < rounds; ++r) {
        upto = std::max(upto, last_pack[size_t(r)]);
        if (upto < 0)
            hp->rounds_before = r + 1;
        else
            for (size_t t = size_t(upto); t < hp->groups.size(); ++t) hp->rounds_after[t] = r + 1;
    }

    // device op lists (LOCAL / UNPACK): every op writes the dense target package (ldd = the
    // contiguous run of the target); LOCAL ops read the dense source package (lds = nf),
    // UNPACK ops keep their receive-buffer offsets.  Bases are added at launch.
    std::vector<costa_tile_op_t> all_ord;
    std::vector<uint64_t> all_work;
    for (auto& gr : hp->groups) {
        for (size_t i = gr.first; i < gr.first + gr.count; ++i) {
            const uint32_t k = uint32_t(i);
            const auto& h = hp->hops[i];
            if (gr.kind != hpl::UNPACK) add_items(gr.gather, k, int64_t(h.op.nf) * int64_t(E), h.op.ns);
            if (gr.kind == hpl::PACK) continue;
            int64_t run, runs;
            target_shape(h.op, run, runs);
            add_items(gr.scatter, k, run * int64_t(E), runs);
        }
        if (gr.kind == hpl::PACK) continue;
        std::vector<costa_tile_op_t> dev_ops;
        dev_ops.reserve(gr.count);
        for (size_t i = gr.first; i < gr.first + gr.count; ++i) {
            const auto& h = hp->hops[i];
            costa_tile_op_t d = h.op;
            int64_t run, runs;
            target_shape(d, run, runs);
            if (gr.kind == hpl::LOCAL) {
                d.src = h.in_off;
                d.lds = d.nf;
            }
            d.dst = h.out_off;
            d.ldd = int32_t(run);
            d.flags &= ~uint32_t(COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST);
            if (d.src % 16 == 0 && (int64_t(d.lds) * int64_t(E)) % 16 == 0) d.flags |= COSTA_TILE_VEC_SRC;
            if ((int64_t(d.ldd) * int64_t(E)) % 16 == 0) d.flags |= COSTA_TILE_VEC_DST;
            dev_ops.push_back(d);
            const uint32_t kind = (d.flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT;
            if (kind == COSTA_SCALE_AXPBY) gr.reads_old = true;
            const int64_t n = int64_t(d.nf) * d.ns;
            gr.alg_bytes += int64_t(E) * n * (1 + (kind != COSTA_SCALE_ZERO) + (kind == COSTA_SCALE_AXPBY));
        }
        gr.any_tr = any_transpose(dev_ops);
        std::vector<costa_tile_op_t> ord;
        std::vector<uint64_t> work;
        gr.split = build_work(dtype, dev_ops, ord, work);
        gr.ord_first = all_ord.size();
        gr.work_first = all_work.size();
        all_ord.insert(all_ord.end(), ord.begin(), ord.end());
        all_work.insert(all_work.end(), work.begin(), work.end());
    }
    {  // host footprints: sources of PACK / LOCAL hops, targets of LOCAL / UNPACK hops
        auto& r = hp->host_ranges;
        for (const auto& gr : hp->groups)
            for (size_t i = gr.first; i < gr.first + gr.count; ++i) {
                const auto& op = hp->hops[i].op;
                if (gr.kind != hpl::UNPACK)
                    r.push_back({uintptr_t(op.src),
                                 uintptr_t(op.src + ((uint64_t(op.ns) - 1) * uint64_t(op.lds) + uint64_t(op.nf)) * E)});
                if (gr.kind != hpl::PACK) {
                    int64_t run, runs;
                    target_shape(op, run, runs);
                    r.push_back({uintptr_t(op.dst),
                                 uintptr_t(op.dst + ((uint64_t(runs) - 1) * uint64_t(op.ldd) + uint64_t(run)) * E)});
                }
            }
        // merged where they overlap, not where they only touch: footprints lie inside their own
        // arrays, so every merged range stays inside one allocation and its two ends tell whether
        // that allocation is page-locked (a pageable array between two page-locked ones stays a
        // range of its own)
        std::sort(r.begin(), r.end());
        size_t o = 0;
        for (size_t i = 0; i < r.size(); ++i) {
            if (o && r[i].first < r[o - 1].second)
                r[o - 1].second = std::max(r[o - 1].second, r[i].second);
            else
                r[o++] = r[i];
        }
        r.resize(o);
    }
    if (!all_ord.empty()) {
        HP_CHECK(hipMalloc(&hp->d_ops, all_ord.size() * sizeof(costa_tile_op_t)));
        HP_CHECK(hipMemcpy(hp->d_ops, all_ord.data(), all_ord.size() * sizeof(costa_tile_op_t),
                           hipMemcpyHostToDevice));
    }
    if (!all_work.empty()) {
        HP_CHECK(hipMalloc(&hp->d_work, all_work.size() * sizeof(uint64_t)));
        HP_CHECK(hipMemcpy(hp->d_work, all_work.data(), all_work.size() * sizeof(uint64_t),
                           hipMemcpyHostToDevice));
    }
    return hp;
}

size_t host_pipeline_groups(const host_pipeline& hp) { return hp.groups.size(); }

namespace {
// Direct mode of a pipeline, built once, on its first call from page-locked memory (calls from
// pageable memory never pay for it).  A group goes direct when the footprints it moves are
// rectangles of the caller's arrays (rectangle_of): the source of a PACK group, the target of
// an UNPACK group, both of a LOCAL group; its ops are rewritten against the dense device images
// of those rectangles:
//   PACK    image -> the send buffer at the package offsets (a pack kernel replaces the host
//           gather; the reference's PACK, communication_data.cpp:191-217)
//   LOCAL   source image -> target image
//   UNPACK  the receive buffer -> target image (communication_data.cpp:219-244)
// Other groups keep the host gather / scatter through the pinned slots, in the same call.
void build_direct(host_pipeline& hp) {
    using hpl = host_pipeline;
    hp.direct_built = true;
    const size_t E = hp.E;
    std::vector<costa_tile_op_t> all_ord;
    std::vector<uint64_t> all_work;
    for (auto& gr : hp.groups) {
        std::vector<foot> fs, ft;
        for (size_t i = gr.first; i < gr.first + gr.count; ++i) {
            const auto& op = hp.hops[i].op;
            int64_t run, runs;
            target_shape(op, run, runs);
            if (gr.kind != hpl::UNPACK) fs.push_back({uintptr_t(op.src), op.nf, op.ns, op.lds});
            if (gr.kind != hpl::PACK) ft.push_back({uintptr_t(op.dst), run, runs, op.ldd});
        }
        std::vector<std::pair<int64_t, int64_t>> ps, pt;
        if ((gr.kind != hpl::UNPACK && !rectangle_of(fs, E, gr.src_rect, ps)) ||
            (gr.kind != hpl::PACK && !rectangle_of(ft, E, gr.dst_rect, pt)))
            continue;
        // an image must fit its device slot half
        const size_t S = hp.slot_bytes;
        if (size_t(gr.src_rect.w * gr.src_rect.h) * E > S || size_t(gr.dst_rect.w * gr.dst_rect.h) * E > S)
            continue;
        std::vector<costa_tile_op_t> dev_ops;
        for (size_t i = gr.first; i < gr.first + gr.count; ++i) {
            const size_t j = i - gr.first;
            costa_tile_op_t d = hp.hops[i].op;
            if (gr.kind != hpl::UNPACK) {
                d.src = uint64_t((ps[j].second * gr.src_rect.w + ps[j].first) * int64_t(E));
                d.lds = int32_t(gr.src_rect.w);
            }
            if (gr.kind != hpl::PACK) {
                d.dst = uint64_t((pt[j].second * gr.dst_rect.w + pt[j].first) * int64_t(E));
                d.ldd = int32_t(gr.dst_rect.w);
            }
            d.flags &= ~uint32_t(COSTA_TILE_VEC_SRC | COSTA_TILE_VEC_DST);
            if (d.src % 16 == 0 && (int64_t(d.lds) * int64_t(E)) % 16 == 0) d.flags |= COSTA_TILE_VEC_SRC;
            if (d.dst % 16 == 0 && (int64_t(d.ldd) * int64_t(E)) % 16 == 0) d.flags |= COSTA_TILE_VEC_DST;
            dev_ops.push_back(d);
        }
        if (gr.kind == hpl::PACK) {
            gr.alg_bytes = 0;
            for (const auto& d : dev_ops) gr.alg_bytes += 2 * int64_t(E) * int64_t(d.nf) * d.ns;
        }
        gr.any_tr_d = any_transpose(dev_ops);
        std::vector<costa_tile_op_t> ord;
        std::vector<uint64_t> work;
        gr.split_d = build_work(hp.dtype, dev_ops, ord, work,
                                gr.kind == hpl::PACK ? list_pack : gr.kind == hpl::UNPACK ? list_unpack : list_local);
        gr.ord_first_d = all_ord.size();
        gr.work_first_d = all_work.size();
        all_ord.insert(all_ord.end(), ord.begin(), ord.end());
        all_work.insert(all_work.end(), work.begin(), work.end());
        gr.direct = true;
        ++hp.n_direct;
    }
    if (!all_ord.empty()) {
        HP_CHECK(hipMalloc(&hp.d_ops_d, all_ord.size() * sizeof(costa_tile_op_t)));
        HP_CHECK(hipMemcpy(hp.d_ops_d, all_ord.data(), all_ord.size() * sizeof(costa_tile_op_t),
                           hipMemcpyHostToDevice));
    }
    if (!all_work.empty()) {
        HP_CHECK(hipMalloc(&hp.d_work_d, all_work.size() * sizeof(uint64_t)));
        HP_CHECK(hipMemcpy(hp.d_work_d, all_work.data(), all_work.size() * sizeof(uint64_t),
                           hipMemcpyHostToDevice));
    }
}
}  // namespace

namespace {
// every byte range page-locked host memory (hipHostMalloc / hipHostRegister), checked at both
// ends of each range (a range is one layout's footprint inside one caller array)
bool all_pinned(const std::vector<std::pair<uintptr_t, uintptr_t>>& ranges) {
    if (ranges.empty()) return false;
    for (const auto& r : ranges)
        for (uintptr_t p : {r.first, r.second - 1}) {
            hipPointerAttribute_t a{};
            if (hipPointerGetAttributes(&a, reinterpret_cast<void*>(p)) != hipSuccess) {
                (void)hipGetLastError();  // pageable memory: an error the runtime keeps otherwise
                return false;
            }
            if (a.type != hipMemoryTypeHost) return false;
        }
    return true;
}
}  // namespace

void run_host_pipeline(host_pipeline& hp, int device, void* compute_stream, void* exchange_stream,
                       char* send_buf, char* recv_buf,
                       const std::function<void(void*, int)>& exchange, const void* d_scalars) {
    using hpl = host_pipeline;
    ring& R = ring_of(device, hp.slot_bytes);
    const size_t S = R.slot;
    hipStream_t comp = static_cast<hipStream_t>(compute_stream);
    hipStream_t xs = static_cast<hipStream_t>(exchange_stream);
    pool& P = thread_pool();
    const size_t E = hp.E;
    const size_t G = hp.groups.size();
    const bool prof = profiling();
    // page-locked caller memory: tiles move by strided DMA between the caller's arrays and the
    // device slots (no host gather / scatter, no pinned slots); the host only issues, stream
    // events order everything.  pinned H2D + D2H of 1-16 KiB rows at once: 94-97 GB/s
    // (tools/pcie_probe.hip, profiles/r4h/)
    const bool pinned = all_pinned(hp.host_ranges);
    if (pinned && !hp.direct_built) build_direct(hp);
    const bool direct = pinned && hp.n_direct > 0;
    auto is_direct = [&](const hpl::group* x) { return direct && x && x->direct; };
    size_t n_direct_run = 0;
    // timing brackets (profiling only): per group kernel, the exchange, and the spans of both
    // copy streams
    std::vector<hipEvent_t> evs;
    auto ev = [&](hipStream_t s) {
        hipEvent_t e;
        HP_CHECK(hipEventCreate(&e));
        evs.push_back(e);
        HP_CHECK(hipEventRecord(e, s));
        return e;
    };
    struct kbracket {
        hipEvent_t a, b;
        bool unpack;
    };
    std::vector<kbracket> kern_t, pack_t;
    hipEvent_t up0 = nullptr, up1 = nullptr, dn0 = nullptr, dn1 = nullptr, x0 = nullptr, x1 = nullptr;
    // every slot starts free: the ring's events are recorded on idle streams
    for (int k = 0; k < kRing; ++k) {
        HP_CHECK(hipEventRecord(R.up_done[k], R.up));
        HP_CHECK(hipEventRecord(R.down_done[k], R.down));
    }
    // exchange round r starts once its part of the send package is in HBM (after the last pack
    // group of rounds <= r); LOCAL groups and the pack groups of later rounds overlap it
    int issued = 0;
    auto issue_rounds = [&](int upto) {
        for (; issued < upto && exchange; ++issued) {
            HP_CHECK(hipEventRecord(R.packed[issued], R.up));
            HP_CHECK(hipStreamWaitEvent(xs, R.packed[issued], 0));
            HP_CHECK(hipEventRecord(R.packed_k[issued], R.pk));  // direct groups' pack kernels
            HP_CHECK(hipStreamWaitEvent(xs, R.packed_k[issued], 0));
            if (prof && !x0) x0 = ev(xs);
            exchange(xs, issued);
            if (prof) x1 = ev(xs);
            HP_CHECK(hipEventRecord(R.moved[issued], xs));
        }
    };
    issue_rounds(hp.rounds_before);

    // Host copy work of one step: the source gather of group t (plus its old target values
    // when an op reads C) and the target scatter of group t - kLag, in one parallel pass.
    auto host_step = [&](const hpl::group* g, char* pin, const hpl::group* o, const char* pout,
                         pool& Pool) {
        const size_t ng = g ? g->gather.size() : 0;
        const size_t nold = g && g->reads_old ? g->scatter.size() : 0;
        const size_t ns = o ? o->scatter.size() : 0;
        Pool.run(ng + nold + ns, [&](size_t i) {
            if (i < ng) {  // source tile columns -> dense package
                const auto& it = g->gather[i];
                const auto& h = hp.hops[it.k];
                const size_t run = size_t(h.op.nf) * E;
                const char* src = reinterpret_cast<const char*>(h.op.src);
                char* dst = pin + h.in_off;
                for (int64_t s = it.lo; s < it.hi; ++s)
                    copy_nt(dst + size_t(s) * run, src + size_t(s) * size_t(h.op.lds) * E, run);
            } else if (i < ng + nold) {  // old target values, for beta != 0 ops only
                const auto& it = g->scatter[i - ng];
                const auto& h = hp.hops[it.k];
                if (((h.op.flags & COSTA_SCALE_MASK) >> COSTA_SCALE_SHIFT) != COSTA_SCALE_AXPBY)
                    return;
                int64_t run, runs;
                target_shape(h.op, run, runs);
                const size_t rb = size_t(run) * E;
                const char* src = reinterpret_cast<const char*>(h.op.dst);
                char* dst = pin + S + h.out_off;
                for (int64_t r = it.lo; r < it.hi; ++r)
                    copy_nt(dst + size_t(r) * rb, src + size_t(r) * size_t(h.op.ldd) * E, rb);
            } else {  // dense target package -> the caller's C
                const auto& it = o->scatter[i - ng - nold];
                const auto& h = hp.hops[it.k];
                int64_t run, runs;
                target_shape(h.op, run, runs);
                const size_t rb = size_t(run) * E;
                char* dst = reinterpret_cast<char*>(h.op.dst);
                const char* src = pout + h.out_off;
                for (int64_t r = it.lo; r < it.hi; ++r)
                    copy_nt(dst + size_t(r) * size_t(h.op.ldd) * E, src + size_t(r) * rb, rb);
            }
            _mm_sfence();  // streaming stores globally visible before the DMA / the caller
        });
    };

    // direct mode: one strided DMA per rectangle between the caller's array and the device image
    auto move_rect = [&](const hpl::rect& r, char* image, bool up) {
        const size_t w = size_t(r.w) * E, pitch = size_t(r.pitch) * E;
        void* host = reinterpret_cast<void*>(r.base);
        if (up)
            HP_CHECK(hipMemcpy2DAsync(image, w, host, pitch, w, size_t(r.h), hipMemcpyHostToDevice, R.up));
        else
            HP_CHECK(hipMemcpy2DAsync(host, pitch, image, w, w, size_t(r.h), hipMemcpyDeviceToHost, R.down));
    };

    // COSTA_HOST_PIPE_TRACE=1: host-side time split (copies / waits / issue) on stderr
    static const bool trace = std::getenv("COSTA_HOST_PIPE_TRACE") != nullptr;
    double t_copy = 0, t_wait_up = 0, t_wait_down = 0, t_issue = 0;
    auto now = [] {
        return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
    };
    const double t_begin = now();

    // group t's copies and kernels (this thread only issues; stream events order them); its
    // host gather is done, and the pinned target slot's previous group (t - kRing) scattered
    auto issue = [&](size_t t) {
        const double t3 = now();
        const int k = int(t % kRing);
        const hpl::group* g = &hp.groups[t];
        const bool gd = is_direct(g);
        char* pin = R.pin_in + size_t(k) * 2 * S;
        char* dev = R.dev + size_t(k) * 2 * S;
        n_direct_run += gd;
        if (g->kind == hpl::PACK && gd) {
            // direct: the source rectangle up into the device slot, then the pack kernel into the
            // send buffer on the ring's pack stream; its round's RCCL group waits for that stream
            // (issue_rounds).  On the exchange stream itself the kernel -- and with it the slot's
            // next user, every later upload -- queued behind the earlier rounds' exchange
            HP_CHECK(hipStreamWaitEvent(R.up, R.down_done[k], 0));  // the slot's previous user
            if (prof && !up0) up0 = ev(R.up);
            move_rect(g->src_rect, dev, true);
            HP_CHECK(hipEventRecord(R.up_done[k], R.up));
            if (prof) up1 = ev(R.up);
            HP_CHECK(hipStreamWaitEvent(R.pk, R.up_done[k], 0));
            hipEvent_t k0 = prof ? ev(R.pk) : nullptr;
            launch_tiles(hp.dtype,
                         make_launch(g->split_d, static_cast<const costa_tile_op_t*>(hp.d_ops_d) + g->ord_first_d,
                                     static_cast<const uint64_t*>(hp.d_work_d) + g->work_first_d, dev, send_buf,
                                     d_scalars, g->any_tr_d, false),
                         R.pk);
            if (prof) pack_t.push_back({k0, ev(R.pk), false});
            HP_CHECK(hipEventRecord(R.down_done[k], R.pk));  // the device slot is free again
            issue_rounds(hp.rounds_after[t]);
            t_issue += now() - t3;
            return;
        }
        if (g->kind == hpl::PACK) {  // the host gather is the pack: upload into the send buffer
            if (prof && !up0) up0 = ev(R.up);
            HP_CHECK(hipMemcpyAsync(send_buf + g->send_off, pin, g->in_bytes, hipMemcpyHostToDevice,
                                    R.up));
            HP_CHECK(hipEventRecord(R.up_done[k], R.up));
            if (prof) up1 = ev(R.up);
            issue_rounds(hp.rounds_after[t]);
            t_issue += now() - t3;
            return;
        }
        const bool unpack = g->kind == hpl::UNPACK;
        if (unpack && (!exchange || issued <= g->round))
            throw error(COSTA_ERR_INTERNAL, "costa: unpack group before its exchange round");
        // the device slot is free once its previous target package has been copied out
        HP_CHECK(hipStreamWaitEvent(R.up, R.down_done[k], 0));
        if (g->in_bytes || g->reads_old) {
            if (prof && !up0) up0 = ev(R.up);
            if (gd) {
                if (g->in_bytes) move_rect(g->src_rect, dev, true);
                if (g->reads_old) move_rect(g->dst_rect, dev + S, true);
            } else {
                if (g->in_bytes) HP_CHECK(hipMemcpyAsync(dev, pin, g->in_bytes, hipMemcpyHostToDevice, R.up));
                if (g->reads_old)
                    HP_CHECK(hipMemcpyAsync(dev + S, pin + S, g->out_bytes, hipMemcpyHostToDevice,
                                            R.up));
            }
            if (prof) up1 = ev(R.up);
        }
        HP_CHECK(hipEventRecord(R.up_done[k], R.up));
        HP_CHECK(hipStreamWaitEvent(comp, R.up_done[k], 0));
        if (unpack) HP_CHECK(hipStreamWaitEvent(comp, R.moved[g->round], 0));
        hipEvent_t k0 = prof ? ev(comp) : nullptr;
        if (gd)
            launch_tiles(hp.dtype,
                         make_launch(g->split_d, static_cast<const costa_tile_op_t*>(hp.d_ops_d) + g->ord_first_d,
                                     static_cast<const uint64_t*>(hp.d_work_d) + g->work_first_d,
                                     unpack ? recv_buf : dev, dev + S, d_scalars, g->any_tr_d, g->reads_old),
                         comp);
        else
            launch_tiles(hp.dtype,
                         make_launch(g->split, static_cast<const costa_tile_op_t*>(hp.d_ops) + g->ord_first,
                                     static_cast<const uint64_t*>(hp.d_work) + g->work_first,
                                     unpack ? recv_buf : dev, dev + S, d_scalars, g->any_tr,
                                     g->reads_old),
                         comp);
        if (prof) kern_t.push_back({k0, ev(comp), unpack});
        HP_CHECK(hipEventRecord(R.kern_done[k], comp));
        HP_CHECK(hipStreamWaitEvent(R.down, R.kern_done[k], 0));
        if (prof && !dn0) dn0 = ev(R.down);
        if (gd)
            move_rect(g->dst_rect, dev + S, false);
        else
            HP_CHECK(hipMemcpyAsync(R.pin_out + size_t(k) * S, dev + S, g->out_bytes,
                                    hipMemcpyDeviceToHost, R.down));
        HP_CHECK(hipEventRecord(R.down_done[k], R.down));
        if (prof) dn1 = ev(R.down);
        issue_rounds(hp.rounds_after[t]);
        t_issue += now() - t3;
    };

    // one pass per step t: the gather of group t and the scatter of group t - kLag together, on
    // every host thread (r5: gathers and scatters on two halves of the threads, each at its own
    // pace, ran 56-58 against 83 GB/s -- the gather on 8 threads became the bound;
    // profiles/r5d/)
    for (size_t t = 0; t < G + kLag; ++t) {
        const int k = int(t % kRing);
        const hpl::group* g = t < G ? &hp.groups[t] : nullptr;
        const hpl::group* o = t >= size_t(kLag) ? &hp.groups[t - kLag] : nullptr;
        if (o && o->kind == hpl::PACK) o = nullptr;  // nothing comes back from a pack group
        if (is_direct(o)) o = nullptr;               // ... nor to the host threads from a direct one
        const hpl::group* gh = is_direct(g) ? nullptr : g;  // group t's host gather
        const int ko = int((t + kRing - kLag) % kRing);     // slot of group t - kLag
        double t0 = now();
        // the pinned source slot is free once its previous upload has landed
        if (gh) HP_CHECK(hipEventSynchronize(R.up_done[k]));
        double t1 = now();
        // group t - kLag's target package has landed in its pinned slot
        if (o) HP_CHECK(hipEventSynchronize(R.down_done[ko]));
        double t2 = now();
        if (gh || o) host_step(gh, R.pin_in + size_t(k) * 2 * S, o, R.pin_out + size_t(ko) * S, P);
        t_wait_up += t1 - t0;
        t_wait_down += t2 - t1;
        t_copy += now() - t2;
        if (g) issue(t);  // (the target slot of group t - kRing was scattered at step t - 1)
    }
    issue_rounds(hp.rounds);  // a rank with nothing to upload still takes part in the exchange
    if (trace)
        std::fprintf(stderr,
                     "[costa host pipe] groups %zu, %d exchange round(s), slot %zu MiB threads %d%s: "
                     "total %.2f ms, copies %.2f, wait-up %.2f, wait-down %.2f, issue %.2f\n",
                     G, exchange ? hp.rounds : 0, S >> 20, host_threads(),
                     direct ? (n_direct_run == G ? " (direct DMA)" : " (direct DMA: some groups)") : "",
                     (now() - t_begin) * 1e3, t_copy * 1e3, t_wait_up * 1e3, t_wait_down * 1e3, t_issue * 1e3);
    HP_CHECK(hipStreamSynchronize(R.up));
    HP_CHECK(hipStreamSynchronize(R.pk));
    HP_CHECK(hipStreamSynchronize(xs));
    HP_CHECK(hipStreamSynchronize(comp));
    HP_CHECK(hipStreamSynchronize(R.down));

    auto& st = stats();
    for (const auto& gr : hp.groups) {
        if (gr.kind == hpl::LOCAL) {
            st.local_bytes += gr.alg_bytes;
            st.local_launches++;
        } else if (gr.kind == hpl::UNPACK) {
            st.unpack_bytes += gr.alg_bytes;
            st.unpack_launches++;
        }
    }
    st.host_groups += int64_t(G);
    if (n_direct_run) st.host_direct++;
    st.host_direct_groups += int64_t(n_direct_run);
    if (direct)
        for (const auto& gr : hp.groups)
            if (gr.kind == hpl::PACK && gr.direct) {
                st.pack_bytes += gr.alg_bytes;
                st.pack_launches++;
            }
    if (prof) {
        float ms = 0.f;
        for (auto& x : kern_t) {
            HP_CHECK(hipEventElapsedTime(&ms, x.a, x.b));
            (x.unpack ? st.unpack_ms : st.local_ms) += ms;
        }
        for (auto& x : pack_t) {
            HP_CHECK(hipEventElapsedTime(&ms, x.a, x.b));
            st.pack_ms += ms;
        }
        if (up0 && up1 && hipEventElapsedTime(&ms, up0, up1) == hipSuccess) st.h2d_ms += ms;
        if (dn0 && dn1 && hipEventElapsedTime(&ms, dn0, dn1) == hipSuccess) st.d2h_ms += ms;
        if (x0 && x1 && hipEventElapsedTime(&ms, x0, x1) == hipSuccess) st.exchange_ms += ms;
    }
    for (hipEvent_t e : evs) (void)hipEventDestroy(e);
}

}  // namespace engine
}  // namespace costa
