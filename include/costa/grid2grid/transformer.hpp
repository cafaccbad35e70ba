// Compatibility header: same path as the reference's <costa/grid2grid/transformer.hpp>.
#pragma once
#include <costa/mpi.hpp>
