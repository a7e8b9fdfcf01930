// 3-D Cartesian domain decomposition, MPI-free.
//
// Reproduces the reference's MPI_Dims_create(P,3) + MPI_Cart_create(periods={1,0,0},
// reorder=false) + Cart_coords + Cart_shift semantics (mpi_new.cpp:409-433):
//  * dims balanced and non-increasing (2 -> 2x1x1, 4 -> 2x2x1, 8 -> 2x2x2);
//  * row-major rank order, coords[2] fastest;
//  * local extents X = (N+1)/dims[0], remainder added to the last rank,
//    global offset x0 = coords[0]*((N+1)/dims[0]);
//  * neighbours: x periodic (always present), y/z absent (-1) at the global faces.
// Local storage is padded by one ghost layer: owned nodes are local 1..X, global
// index of local i is x0 + i - 1.
#pragma once

#include <array>
#include <string>

#include "common.hpp"

namespace wave3d {

struct Topology {
    int nprocs = 1, rank = 0;
    int N = 0;
    int dims[3] = {1, 1, 1};
    int coords[3] = {0, 0, 0};
    int ext[3] = {0, 0, 0};  // X, Y, Z (owned nodes per axis)
    int off[3] = {0, 0, 0};  // x0, y0, z0 (global index of local index 1)
    int nbr[3][2] = {{-1, -1}, {-1, -1}, {-1, -1}};  // [axis][0 = minus, 1 = plus]

    static void dims_create(int nprocs, int dims[3]);  // honours non-zero presets
    static Topology make(int N, int nprocs, int rank, const int* dims_override = nullptr);

    int rank_of(int c0, int c1, int c2) const { return (c0 * dims[1] + c1) * dims[2] + c2; }
    bool first(int a) const { return coords[a] == 0; }
    bool last(int a) const { return coords[a] == dims[a] - 1; }
    int X() const { return ext[0]; }
    int Y() const { return ext[1]; }
    int Z() const { return ext[2]; }

    // Nodes updated by the stencil for layers >= 1, in local indices: every owned x
    // (the periodic planes x=0 and x=N are stencil points, mpi_new.cpp:170-176) and the
    // global interior 1..N-1 in y and z (faces are Dirichlet, mpi_new.cpp:160-169).
    Box compute_box() const;
    // Nodes whose error enters the per-layer maxima (layers >= 1): global 1..N-1 in
    // every axis (mpi_new.cpp:331-337).
    Box error_box() const;
    // All owned nodes (layer 0 / initial condition, mpi_new.cpp:274-286).
    Box owned_box() const;

    // Local plane index that is sent towards the minus / plus x neighbour. On the periodic
    // axis the duplicated global plane is skipped (mpi_new.cpp:186-187).
    int x_send_minus() const { return first(0) ? 2 : 1; }
    int x_send_plus() const { return last(0) ? ext[0] - 1 : ext[0]; }

    std::string describe() const;
};

}  // namespace wave3d
