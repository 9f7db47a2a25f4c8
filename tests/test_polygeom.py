"""Post-selection geometry in libsbo against the oracle's
pure-Python restatement of polydist (src/libraries/polygeom_lib.cpp:401-474),
bg::correct and bg::within, plus hand-derived cases.

Parity is unpinned against the reference itself: it needs Boost (absent) and
its tests hold no polygon fixtures; the hand-derived cases below pin the
quirks SURVEY.md Appendix A lists (nearest vertex, first minimum, empty ring)."""
import numpy as np
import pytest

from oracle import oracle as O
from safe_bayesian_optimization_amd import node as ND


def _ring(pts, close=True):
    p = [tuple(map(float, q)) for q in pts]
    if close:
        p.append(p[0])
    return np.array([q[0] for q in p]), np.array([q[1] for q in p])


SQUARE = [(0, 0), (4, 0), (4, 4), (0, 4)]  # counter-clockwise


def test_nearest_vertex_quirk():
    # a point beside the middle of the bottom edge: the true projection is
    # (2, 0) at distance 1, polydist returns the nearest vertex (0, 0)
    rx, ry = _ring(SQUARE)
    px, py, d = ND.polydist(rx, ry, 2.0, -1.0)
    assert (px, py) == (0.0, 0.0)
    assert d == np.sqrt(5.0)
    assert (px, py, d) == O.polydist(rx, ry, 2.0, -1.0)


def test_first_minimum_wins():
    # equidistant to (4, 0) and (4, 4): the first in ring order wins
    rx, ry = _ring(SQUARE)
    px, py, d = ND.polydist(rx, ry, 5.0, 2.0)
    assert (px, py) == (4.0, 0.0)
    assert (px, py, d) == O.polydist(rx, ry, 5.0, 2.0)


def test_empty_ring():
    px, py, d, st = ND.polydist(np.zeros(0), np.zeros(0), 1.0, 1.0, status=True)
    assert st == 5 and (px, py, d) == (0.0, 0.0, 1e8)   # SBO_E_EMPTY, reference's intended output
    assert O.polydist(np.zeros(0), np.zeros(0), 1.0, 1.0) is None


def test_repeated_vertex_zero_edge():
    # a zero-length edge takes diff_norm = 1 (:444-446)
    rx, ry = _ring([(0, 0), (0, 0), (3, 0), (3, 3)])
    for p in [(0.5, -0.5), (-1.0, 0.0), (3.2, 1.4), (1.0, 1.0)]:
        assert ND.polydist(rx, ry, *p) == O.polydist(rx, ry, *p)


def test_correct_closes_and_reverses():
    cw = [(0, 0), (0, 4), (4, 4), (4, 0)]
    rx, ry = _ring(cw, close=False)
    cx, cy = ND.polygon_correct(rx, ry)
    ox, oy = O.polygon_correct(rx, ry)
    assert np.array_equal(cx, ox) and np.array_equal(cy, oy)
    assert cx.size == 5 and (cx[0], cy[0]) == (cx[-1], cy[-1])
    assert O.ring_area2(cx, cy) > 0
    # already counter-clockwise and closed: unchanged
    rx, ry = _ring(SQUARE)
    cx, cy = ND.polygon_correct(rx, ry)
    assert np.array_equal(cx, rx) and np.array_equal(cy, ry)


def test_within_interior_boundary_outside():
    rx, ry = _ring(SQUARE)
    assert ND.point_within(rx, ry, 2.0, 2.0) == 1
    assert ND.point_within(rx, ry, 4.0, 2.0) == 0      # on an edge
    assert ND.point_within(rx, ry, 0.0, 0.0) == 0      # on a vertex
    assert ND.point_within(rx, ry, 5.0, 2.0) == 0
    cw = _ring(SQUARE[::-1])
    assert ND.point_within(*cw, 2.0, 2.0) == 1         # either orientation


@pytest.mark.parametrize("seed", range(25))
def test_random_rings_match_oracle(seed):
    rng = np.random.default_rng(7000 + seed)
    n = int(rng.integers(3, 40))
    ang = np.sort(rng.uniform(0, 2 * np.pi, n))
    if seed % 2:
        ang = ang[::-1]                                    # clockwise input
    r = rng.uniform(0.5, 3.0, n)
    pts = np.stack([r * np.cos(ang) + rng.normal(), r * np.sin(ang) + rng.normal()], 1)
    if seed % 5 == 0:
        pts[1] = pts[0]                                    # repeated vertex
    rx, ry = _ring(pts, close=bool(seed % 3))
    cx, cy = ND.polygon_correct(rx, ry)
    ox, oy = O.polygon_correct(rx, ry)
    assert np.array_equal(cx, ox) and np.array_equal(cy, oy)
    for q in rng.uniform(-5, 5, size=(20, 2)):
        assert ND.polydist(cx, cy, *q) == O.polydist(cx, cy, *q)
        assert ND.point_within(cx, cy, *q) == O.point_within(cx, cy, *q)


def test_project_subgoal_paths():
    rx, ry = _ring(SQUARE[::-1])                          # the node's polygon is clockwise
    Dx = np.array([0.0, 9.0, 5.0])
    Dy = np.array([0.0, 9.0, 1.0])
    # goal inside: the goal itself (:657-666)
    assert ND.project_subgoal(rx, ry, (1.0, 1.0), 2, Dx, Dy) == (1, 1.0, 1.0, 0.0)
    # goal outside: frontier point (5, 1) projected onto the corrected ring
    code, x, y, d = ND.project_subgoal(rx, ry, (10.0, 10.0), 2, Dx, Dy)
    cx, cy = O.polygon_correct(rx, ry)
    assert (code, x, y, d) == (0,) + O.polydist(cx, cy, 5.0, 1.0)
    # no subgoal (:670)
    assert ND.project_subgoal(rx, ry, (10.0, 10.0), -1, Dx, Dy)[0] == -1
