#include "halo.hpp"

namespace wave3d {

HaloPlan make_halo_plan(const Topology& t, i64 x_plane, int row, bool self_msg) {
    HaloPlan p;
    const i64 X = t.ext[0], Y = t.ext[1];
    const i64 count[3] = {x_plane, X * row, X * (Y + 2)};
    p.self_x = t.nbr[0][0] == t.rank && !self_msg;
    for (int a = 0; a < 3; ++a) {
        if (a == 0 && p.self_x) continue;
        // travelling +a: send from the plus face to nbr[a][1] (tag 2a+1)
        if (t.nbr[a][1] >= 0) p.sends.push_back({a, 1, t.nbr[a][1], 2 * a + 1, count[a]});
        // travelling -a: send from the minus face to nbr[a][0] (tag 2a+2)
        if (t.nbr[a][0] >= 0) p.sends.push_back({a, 0, t.nbr[a][0], 2 * a + 2, count[a]});
        // receive the +a traveller from the minus neighbour into the minus ghost
        if (t.nbr[a][0] >= 0) p.recvs.push_back({a, 0, t.nbr[a][0], 2 * a + 1, count[a]});
        // receive the -a traveller from the plus neighbour into the plus ghost
        if (t.nbr[a][1] >= 0) p.recvs.push_back({a, 1, t.nbr[a][1], 2 * a + 2, count[a]});
    }
    return p;
}

}  // namespace wave3d
