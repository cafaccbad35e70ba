// costa-mi355x: the reference's MPI_Comm API.  Include this (or the grid2grid/ compatibility
// headers) to get transform(..., MPI_Comm) and transformer<T>(MPI_Comm).
#pragma once
#include <mpi.h>

#include <costa/layout.hpp>
#include <costa/transform.hpp>
