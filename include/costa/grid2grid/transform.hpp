// Compatibility header: same path as the reference's <costa/grid2grid/transform.hpp>.
#pragma once
#include <costa/mpi.hpp>
