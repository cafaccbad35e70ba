// Compatibility header: same path as the reference's <costa/grid2grid/grid_layout.hpp>.
#pragma once
#include <costa/layout.hpp>
