"""Cartesian decomposition (SURVEY C16/P1, Appendix A 'Decomposition')."""
import pytest


@pytest.mark.parametrize("P,dims", [(1, [1, 1, 1]), (2, [2, 1, 1]), (3, [3, 1, 1]), (4, [2, 2, 1]),
                                    (6, [3, 2, 1]), (8, [2, 2, 2]), (12, [3, 2, 2]),
                                    (16, [4, 2, 2]), (18, [3, 3, 2]), (24, [4, 3, 2]),
                                    (27, [3, 3, 3]), (32, [4, 4, 2]), (64, [4, 4, 4])])
def test_dims_create_matches_mpi(C, P, dims):
    assert C.dims_create(P, [0, 0, 0]) == dims


def test_dims_create_presets(C):
    assert C.dims_create(8, [1, 0, 0]) == [1, 4, 2]
    assert C.dims_create(8, [0, 0, 4]) == [2, 1, 4]
    with pytest.raises(Exception):
        C.dims_create(8, [3, 0, 0])


def test_extents_offsets_remainder(C):
    # N=32 -> 33 nodes over 2 ranks: 16 + 17 (remainder on the last rank)
    t0 = C.topology(32, 2, 0, [0, 0, 0])
    t1 = C.topology(32, 2, 1, [0, 0, 0])
    assert t0["ext"] == [16, 33, 33] and t0["off"] == [0, 0, 0]
    assert t1["ext"] == [17, 33, 33] and t1["off"] == [16, 0, 0]
    # every global node owned exactly once
    for P in (2, 3, 4, 8, 12):
        seen = set()
        for r in range(P):
            t = C.topology(20, P, r, [0, 0, 0])
            for a in range(3):
                assert t["ext"][a] >= 1
            cells = {(t["off"][0] + i, t["off"][1] + j, t["off"][2] + k)
                     for i in range(t["ext"][0]) for j in range(t["ext"][1]) for k in range(t["ext"][2])}
            assert not (cells & seen)
            seen |= cells
        assert len(seen) == 21 ** 3


def test_rank_order_and_neighbours(C):
    # reorder=false, row-major with coords[2] fastest
    P = 8
    for r in range(P):
        t = C.topology(32, P, r, [0, 0, 0])
        c = t["coords"]
        assert r == (c[0] * 2 + c[1]) * 2 + c[2]
        # x periodic: both neighbours always exist
        assert t["nbr"][0][0] >= 0 and t["nbr"][0][1] >= 0
        # y/z: none at the global faces
        assert (t["nbr"][1][0] < 0) == (c[1] == 0)
        assert (t["nbr"][2][1] < 0) == (c[2] == 1)


def test_boxes(C):
    t = C.topology(32, 1, 0, [0, 0, 0])
    # local index = global + 1; periodic planes x=0,N are stencil points
    assert t["compute_box"] == [1, 33, 2, 32, 2, 32]
    assert t["error_box"] == [2, 32, 2, 32, 2, 32]
    assert t["owned_box"] == [1, 33, 1, 33, 1, 33]
    assert t["self_x"] and t["sends"] == [] and t["recvs"] == []


def test_halo_plan_symmetric(C):
    """Every send has exactly one matching receive (peer, tag, size) — the property the
    tag-less RCCL transport relies on, in canonical per-peer FIFO order."""
    for P in (2, 3, 4, 6, 8, 12):
        tops = [C.topology(40, P, r, [0, 0, 0]) for r in range(P)]
        for r, t in enumerate(tops):
            for (axis, side, peer, tag, count) in t["sends"]:
                match = [m for m in tops[peer]["recvs"] if m[2] == r and m[3] == tag]
                assert len(match) == 1 and match[0][4] == count
            # FIFO order per peer: sends to a peer and that peer's receives from us agree
            for peer in {m[2] for m in t["sends"]}:
                s_tags = [m[3] for m in t["sends"] if m[2] == peer]
                r_tags = [m[3] for m in tops[peer]["recvs"] if m[2] == r]
                assert s_tags == r_tags
