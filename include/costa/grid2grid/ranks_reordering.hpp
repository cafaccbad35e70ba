// costa-mi355x: rank relabelling (drop-in for the reference's
// <costa/grid2grid/ranks_reordering.hpp>, src/costa/grid2grid/ranks_reordering.hpp:7).
#pragma once

#include <costa/grid2grid/comm_volume.hpp>

#include <vector>

namespace costa {

// A permutation of the ranks 0..n_ranks-1 that keeps as much data local as the greedy
// matching of the reference finds (ranks_reordering.cpp:4-61): every rank pair {a, b} is worth
// volume(a, b) - volume(a, a) - volume(b, b) (what swapping a and b keeps local beyond what
// already stays); pairs are taken by decreasing worth (ties by rank ids), each rank at most
// once, and a taken pair swaps its two ranks.  `reordered` tells whether the result differs
// from the identity.  Apply it with grid_layout::reorder_ranks / assigned_grid2D::reorder_ranks
// on the target layouts.
std::vector<int> optimal_reordering(comm_volume& comm_volume, int n_ranks, bool& reordered);

}  // namespace costa
