"""Device frontier: sbo_frontier / sbo_subgoal with device
pointers -- GPU raster, owner map and image, host border follow -- must
return exactly what the host restatement and the oracle return
(src/safe_bayesian_optimization_node.cpp:418-550): same indices, same order,
duplicates included, same subgoal."""
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402
from safe_bayesian_optimization_amd import node as ND  # noqa: E402
from safe_bayesian_optimization_amd.gp import Context  # noqa: E402


@pytest.fixture(scope="module")
def ctx():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = Context(0)
    yield c
    c.close()


def _dev(a, dt):
    return torch.as_tensor(np.ascontiguousarray(a, dt), device="cuda:0")


def _grid(w, h, x0, x1, y0, y1):
    gx = np.linspace(x0, x1, w)
    gy = np.linspace(y0, y1, h)
    QY, QX = np.meshgrid(gy, gx, indexing="ij")
    return QX.reshape(-1), QY.reshape(-1)


def _field(rng, h, w, sigma=2.0):
    from scipy.ndimage import gaussian_filter
    return gaussian_filter(rng.normal(size=(h, w)), sigma).reshape(-1)


def _both(ctx, Dx, Dy, s, w, h):
    fd = ctx.frontier(_dev(Dx, np.float64), _dev(Dy, np.float64), _dev(s, np.uint8), w, h)
    fh = ND.find_safety_contour_indices(Dx, Dy, s, w, h)
    return fd, fh


@pytest.mark.parametrize("seed", range(10))
def test_device_frontier_and_subgoal_match_host(ctx, seed):
    rng = np.random.default_rng(300 + seed)
    w, h = (int(v) for v in rng.integers(5, 90, size=2))
    Dx, Dy = _grid(w, h, rng.uniform(-3, 1), rng.uniform(2, 9), rng.uniform(-2, 1), rng.uniform(2, 7))
    mu = _field(rng, h, w) * 5
    sd = rng.uniform(0.01, 1.0, size=Dx.size)
    lo, hi, s = O.compute_sets(mu, sd, 2.0, float(np.percentile(mu, 30 + seed)))
    fd, fh = _both(ctx, Dx, Dy, s, w, h)
    assert np.array_equal(fd, fh)
    assert np.array_equal(fd, O.find_safety_contour_indices(Dx, Dy, s, w, h))
    d = {k: _dev(v, np.float64) for k, v in (("Dx", Dx), ("Dy", Dy), ("lo", lo), ("hi", hi))}
    for g in rng.uniform(-2, 8, size=(3, 2)):
        got = ctx.subgoal(d["Dx"], d["Dy"], d["lo"], d["hi"], _dev(s, np.uint8), w, h, *g)
        assert got == ND.next_subgoal(Dx, Dy, lo, hi, s, w, h, *g) == O.next_subgoal(Dx, Dy, lo, hi, s, w, h, *g)


@pytest.mark.parametrize("seed", range(4))
def test_scattered_points_last_writer_wins(ctx, seed):
    """More points than pixels, unordered, several per pixel: the device's
    atomicMax owner must equal the host's sequential last writer, pixel by
    pixel, through the frontier indices (and points at max x/y are dropped)."""
    rng = np.random.default_rng(500 + seed)
    w, h = (int(v) for v in rng.integers(8, 50, size=2))
    m = int(w * h * rng.uniform(1.5, 4.0))
    Dx = rng.uniform(-4.0, 7.0, size=m)
    Dy = rng.uniform(-1.0, 9.0, size=m)
    Dx[::17] = np.floor(Dx[::17])                  # exact integers: boundary pixels and dropped maxima
    s = (rng.uniform(size=m) < 0.6).astype(np.uint8)
    fd, fh = _both(ctx, Dx, Dy, s, w, h)
    assert np.array_equal(fd, fh)


def test_fixture_images_through_the_raster(ctx, contour_cases):
    """The hand-derived contour fixtures, rasterised from coordinates that map
    one point per pixel: the device frontier is the fixture's contour pixels
    mapped to grid indices, in the fixture's order."""
    for case in contour_cases:
        img = np.array(case["mask"], np.uint8)
        h, w = img.shape
        # point 0 = (0, 0) and the last point = (w, h) (unsafe sentinels) pin the
        # int-truncated bounds to [0, w] x [0, h]; point 1 + y*w + x sits at the
        # centre of pixel (x, y) and, written after point 0, owns it; (w, h)
        # maps past the image and is dropped
        cx, cy = _grid(w, h, 0.5, w - 0.5, 0.5, h - 0.5)
        Dx = np.concatenate([[0.0], cx, [float(w)]])
        Dy = np.concatenate([[0.0], cy, [float(h)]])
        s = np.concatenate([[0], (img.reshape(-1) > 0).astype(np.uint8), [0]]).astype(np.uint8)
        fd, fh = _both(ctx, Dx, Dy, s, w, h)
        assert np.array_equal(fd, fh), case["name"]
        want = [1 + int(y) * w + int(x) for c in case["contours"] for x, y in c]
        assert fd.tolist() == want, case["name"]


def test_edges(ctx):
    e = np.zeros(0)
    assert ctx.frontier(_dev(e, np.float64), _dev(e, np.float64), _dev(np.zeros(0), np.uint8), 4, 4).size == 0
    Dx, Dy = _grid(20, 10, 0.0, 5.0, 0.0, 3.0)
    none = np.zeros(Dx.size, np.uint8)
    fd, fh = _both(ctx, Dx, Dy, none, 20, 10)
    assert fd.size == 0 and fh.size == 0
    z = _dev(np.zeros(Dx.size), np.float64)
    assert ctx.subgoal(_dev(Dx, np.float64), _dev(Dy, np.float64), z, z, _dev(none, np.uint8), 20, 10) == -1
    allsafe = np.ones(Dx.size, np.uint8)
    fd, fh = _both(ctx, Dx, Dy, allsafe, 20, 10)
    assert np.array_equal(fd, fh) and fd.size > 0
    # degenerate bounds (max_x == min_x after truncation) drop every point
    Dx2 = np.full(Dx.size, 0.5)
    fd, fh = _both(ctx, Dx2, Dy, allsafe, 20, 10)
    assert fd.size == 0 and fh.size == 0
    # host arrays take the host path and give the same answer
    assert np.array_equal(ctx.frontier(Dx, Dy, allsafe, 20, 10), ND.find_safety_contour_indices(Dx, Dy, allsafe, 20, 10))


def test_c4_scale_frontier(ctx):
    """A 1000 x 1000 grid (C4's M) with a smooth safe set: identical to the
    host path; both timed (printed)."""
    rng = np.random.default_rng(7)
    w = h = 1000
    Dx, Dy = _grid(w, h, 0.0, 18.0, 0.0, 18.0)
    mu = _field(rng, h, w, 12.0)
    s = (mu > np.percentile(mu, 40)).astype(np.uint8)
    lo = mu - 0.1
    hi = mu + 0.1 + rng.uniform(0, 0.01, size=mu.size)
    d = [_dev(v, np.float64) for v in (Dx, Dy, lo, hi)] + [_dev(s, np.uint8)]
    ctx.subgoal(*d, w, h, 9.0, 9.0)  # warm
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    gd = ctx.subgoal(*d, w, h, 9.0, 9.0)
    t1 = time.perf_counter()
    gh = ND.next_subgoal(Dx, Dy, lo, hi, s, w, h, 9.0, 9.0)
    t2 = time.perf_counter()
    fd, fh = _both(ctx, Dx, Dy, s, w, h)
    print(f"C4 frontier {fd.size} pts; subgoal device {1e3 * (t1 - t0):.2f} ms, host {1e3 * (t2 - t1):.2f} ms")
    assert np.array_equal(fd, fh) and gd == gh >= 0


@pytest.mark.parametrize("w,h,sigma", [(1000, 1000, 12.0), (1000, 1000, 3.0), (300, 120, 4.0)])
def test_device_frontier_topology(ctx, w, h, sigma):
    """The device raster + border follow at C4 size (and the mapper's own
    300 x 120 grid, config/lpsc.yaml:38) against the scipy.ndimage topology
    of tests/frontier_props.py -- no border follower in the check: the
    frontier's pixels are exactly the outer borders of the external safe
    components, with at most #contours - 1 breaks in 8-adjacency."""
    from tests.frontier_props import check_flat_frontier
    from scipy.ndimage import gaussian_filter
    rng = np.random.default_rng(int(sigma * 10) + w)
    img = (gaussian_filter(rng.normal(size=(h, w)), sigma) > 0).astype(np.uint8)
    cx, cy = _grid(w, h, 0.5, w - 0.5, 0.5, h - 0.5)
    Dx = np.concatenate([[0.0], cx, [float(w)]])
    Dy = np.concatenate([[0.0], cy, [float(h)]])
    s = np.concatenate([[0], img.reshape(-1), [0]]).astype(np.uint8)
    fd = ctx.frontier(_dev(Dx, np.float64), _dev(Dy, np.float64), _dev(s, np.uint8), w, h)
    pix = np.stack([(fd - 1) % w, (fd - 1) // w], axis=1)
    exp = check_flat_frontier(img, pix)
    print(f"{w}x{h} sigma {sigma}: {len(exp)} external components, frontier {fd.size} px")
