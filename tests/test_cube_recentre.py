"""laserMapping's cube recentring (laserMapping.cpp:325-507) on the oracle: teacher-forced sequences
(tests/recentre_seq.py) drive the vehicle across the +-x, +-y (375 m) and +-z (125 m) thresholds while
the 21 x 21 x 11 grid holds map points, one frame moving the centre twice. After every frame each stored
point, re-bucketed directly from its coordinates with the current centre (cube_index,
laserMapping.cpp:314-323), must sit in the cube the shifts left it in. CPU test; the device's map is
compared with this one in tests/test_gpu_parity.py::test_mapping_cube_recentring."""
import numpy as np
import pytest

import oracle_binding as ob
import recentre_seq
from lvo_amd_loader import abi


@pytest.mark.parametrize("axis", recentre_seq.AXES)
def test_oracle_recentring_matches_direct_rebucketing(axis):
    along = "xyz".index(axis[1])
    o = ob.Oracle(abi.default_params(64))
    prev = o.cube_check()["cen"]
    assert prev == (10, 10, 5)
    moves, held = [], []
    for corner, surf, q, t in recentre_seq.sequence(axis):
        before = o.cube_check()["points"]
        o.set_mapping_input(corner, surf, q, t)
        m = o.mapping()
        chk = o.cube_check()
        assert chk["misplaced"] == 0, (axis, chk)
        assert chk["points"] == m["map_total_points"]
        d = np.array(chk["cen"]) - np.array(prev)
        assert all(d[i] == 0 for i in range(3) if i != along), (axis, prev, chk["cen"])
        moves.append(int(d[along]))
        held.append(before)
        prev = chk["cen"]
    # travel towards + moves the centre index down (the cubes shift towards 0), towards - up
    sign = -1 if axis[0] == "+" else 1
    assert all(mv * sign >= 0 for mv in moves), moves
    assert sum(abs(mv) for mv in moves) >= 3, moves
    assert max(abs(mv) for mv in moves) >= 2, moves               # one frame shifts twice
    assert any(abs(mv) > 0 and h > 0 for mv, h in zip(moves, held)), (moves, held)   # shifts a non-empty grid
