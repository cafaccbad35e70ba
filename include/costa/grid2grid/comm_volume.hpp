// costa-mi355x: communication volume between ranks (drop-in for the reference's
// <costa/grid2grid/comm_volume.hpp>, src/costa/grid2grid/comm_volume.hpp:7-160).
//
// An undirected graph over ranks: volume[{a, b}] (a <= b) = elements that move between ranks a
// and b in a transformation (a == b: elements that stay local).  Built by
// costa::communication_volume (<costa/transform.hpp>), consumed by costa::optimal_reordering
// (<costa/grid2grid/ranks_reordering.hpp>).  Host-only; no GPU involved.
#pragma once

#include <algorithm>
#include <cstddef>
#include <functional>
#include <ostream>
#include <unordered_map>
#include <vector>

namespace costa {

struct edge_t {
    int src = 0;
    int dest = 0;

    edge_t() = default;
    edge_t(int s, int d) : src(s), dest(d) {}

    edge_t sorted() const { return {std::min(src, dest), std::max(src, dest)}; }
    bool operator==(const edge_t& o) const { return src == o.src && dest == o.dest; }
};

}  // namespace costa

namespace std {
template <>
struct hash<costa::edge_t> {
    size_t operator()(const costa::edge_t& e) const noexcept {
        const size_t a = std::hash<int>()(e.src), b = std::hash<int>()(e.dest);
        return a ^ (b + 0x9e3779b97f4a7c15ull + (a << 6) + (a >> 2));
    }
};
}  // namespace std

namespace costa {

struct weighted_edge_t {
    edge_t e;
    int w = 0;

    weighted_edge_t() = default;
    weighted_edge_t(int src, int dest, int weight) : e{src, dest}, w(weight) {}

    int weight() const { return w; }
    int src() const { return e.src; }
    int dest() const { return e.dest; }
    const edge_t& edge() const { return e; }
    bool operator==(const weighted_edge_t& o) const { return e == o.e && w == o.w; }
    bool operator<(const weighted_edge_t& o) const { return w < o.w; }
};

struct comm_volume {
    using volume_t = std::unordered_map<edge_t, size_t>;
    volume_t volume;

    comm_volume() = default;
    explicit comm_volume(volume_t&& v) : volume(std::move(v)) {}

    comm_volume& operator+=(const comm_volume& other) {
        for (const auto& kv : other.volume) volume[kv.first.sorted()] += kv.second;
        return *this;
    }
    comm_volume operator+(const comm_volume& other) const {
        comm_volume r;
        for (const auto& kv : volume) r.volume[kv.first.sorted()] += kv.second;
        for (const auto& kv : other.volume) r.volume[kv.first.sorted()] += kv.second;
        return r;
    }
    // divide every edge's volume by the cost factor of its rank pair (e.g. topology_cost)
    void apply_topology(const std::vector<std::vector<int>>& topology) {
        for (auto& kv : volume) kv.second /= size_t(topology[size_t(kv.first.src)][size_t(kv.first.dest)]);
    }
    // elements that change rank (local edges a == b excluded)
    size_t total_volume() const {
        size_t sum = 0;
        for (const auto& kv : volume)
            if (kv.first.src != kv.first.dest) sum += kv.second;
        return sum;
    }
    friend std::ostream& operator<<(std::ostream& os, const comm_volume& cv) {
        os << "Communication volume consists of the following:\n";
        for (const auto& kv : cv.volume) os << kv.first.src << "->" << kv.first.dest << ": " << kv.second << "\n";
        return os;
    }
};

}  // namespace costa
