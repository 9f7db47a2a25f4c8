"""Synthetic terrain workloads for the planning-tick hot path.

The reference's only data fixture, ``data/terrain.csv``, is a missing blob
(/root/reference/.MISSING_LARGE_BLOBS:1).  Its format and the way the sim
samples it are defined by ``src/turtlesim_spatial_publisher.py``:

* ``np.loadtxt(terrain_file, delimiter=',', skiprows=1)`` -- one header row,
  then an R x C numeric matrix (:56-57);
* terrain coordinates are centred, +-C/2 by +-R/2, and pose coordinates are
  terrain coordinates / ``scale_factor`` = 10 (:68-74);
* ``get_terrain_value`` maps a pose to (row, col) with ``int(...*(C-1))``,
  clamps, and min-max normalises the value to [0, 10] (:77-100);
* 30 initial points uniformly within radius 1 of the start pose (:111-149),
  then one measurement per second at the robot pose (:151-183).

All randomness is a counter-based SplitMix64 so the same inputs can be
regenerated anywhere (tests, bench, the GPU box) without shipping them.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

_GAMMA = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(seed: int, n: int, offset: int = 0) -> np.ndarray:
    """Counter-based SplitMix64: element i is the (offset+i+1)-th output of a
    SplitMix64 stream started at ``seed``."""
    with np.errstate(over="ignore"):
        ctr = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + ctr * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed: int, n: int, offset: int = 0) -> np.ndarray:
    """U[0, 1) doubles from the top 53 bits."""
    return (splitmix64(seed, n, offset) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def normal(seed: int, n: int, offset: int = 0) -> np.ndarray:
    """Standard normals by Box-Muller on two interleaved uniform streams."""
    u = uniform(seed, 2 * n, 2 * offset)
    u1 = np.maximum(u[0::2], 1e-300)
    u2 = u[1::2]
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)


@dataclass
class Hyper:
    """GP hyper-parameters, defaults from /root/reference/config/lpsc.yaml:35-37.

    ``noise_level`` is treated as a noise *variance* (sklearn WhiteKernel
    naming); ``sigma_f`` is the signal standard deviation, so sf2 = sigma_f^2.
    """
    length_scale: float = 0.4
    sigma_f: float = 1.0
    noise_level: float = 0.1
    prior_mean: float = 0.0

    @property
    def sf2(self) -> float:
        return self.sigma_f * self.sigma_f

    @property
    def sn2(self) -> float:
        return self.noise_level


@dataclass
class Workload:
    name: str
    x: np.ndarray        # training x (f64)
    y: np.ndarray        # training y
    obs: np.ndarray      # observations
    qx: np.ndarray       # query grid x (row-major over the grid)
    qy: np.ndarray
    width: int           # n_width_cells
    height: int          # n_height_cells
    hyper: Hyper
    f_min: float
    beta: float = 2.0    # config/safe_bayesian_optimization.yaml:4
    side: float | None = None   # the square the observation field is defined on (more_points)
    seed: int = 0


def smooth_field(px, py, side: float, ell: float, seed: int, bumps: int = 32):
    """Sum of ``bumps`` Gaussian bumps, widths U[2l, 4l], amplitudes U[-1, 1]."""
    u = uniform(seed ^ 0x5EED, 4 * bumps)
    cx = u[0::4] * side
    cy = u[1::4] * side
    w = (2.0 + 2.0 * u[2::4]) * ell
    a = 2.0 * u[3::4] - 1.0
    f = np.zeros_like(np.asarray(px, np.float64))
    for b in range(bumps):
        f += a[b] * np.exp(-((px - cx[b]) ** 2 + (py - cy[b]) ** 2) / (2.0 * w[b] ** 2))
    return f


def synthetic(n: int, grid_w: int, grid_h: int | None = None, seed: int = 0,
              hyper: Hyper | None = None, name: str | None = None) -> Workload:
    """C2-C5 style workload: N points uniform over a square of
    side l*sqrt(N/8) (about 8 points per l^2, cond(K) ~ 1e3), observations =
    smooth field + N(0, sn2), a grid_w x grid_h query grid over the square,
    f_min = 40th percentile of the observations (S covers ~60% of cells)."""
    hyper = hyper or Hyper()
    grid_h = grid_h or grid_w
    side = hyper.length_scale * math.sqrt(n / 8.0)
    u = uniform(seed, 2 * n)
    x = u[0::2] * side
    y = u[1::2] * side
    obs = smooth_field(x, y, side, hyper.length_scale, seed) + math.sqrt(hyper.sn2) * normal(seed + 1, n)
    gx = np.linspace(0.0, side, grid_w)
    gy = np.linspace(0.0, side, grid_h)
    QY, QX = np.meshgrid(gy, gx, indexing="ij")
    f_min = float(np.percentile(obs, 40.0))
    return Workload(name or f"synthetic_n{n}_g{grid_w}x{grid_h}", x, y, obs, QX.reshape(-1), QY.reshape(-1),
                    grid_w, grid_h, hyper, f_min, side=side, seed=seed)


def synthetic_box(n: int, grid_w: int, grid_h: int, x_range=(0.0, 1.0), y_range=(0.0, 2.5), seed: int = 0,
                  hyper: Hyper | None = None, name: str | None = None) -> Workload:
    """The stress variant of SURVEY.md 8(d): N points uniform over the mapping
    node's own box (config/lpsc.yaml:32-33, x_range [0, 1], y_range [0, 2.5]),
    the same smooth field + N(0, sn2) observations, a grid_w x grid_h query
    grid over the box.  With l = 0.4 the box is only 2.5 x 6.25 length scales,
    so at large N almost no K* tile is negligible (the skip-free regime) and
    K is ill-conditioned (cond ~1e4-1e5)."""
    hyper = hyper or Hyper()
    (x0, x1), (y0, y1) = x_range, y_range
    u = uniform(seed, 2 * n)
    x = x0 + u[0::2] * (x1 - x0)
    y = y0 + u[1::2] * (y1 - y0)
    side = max(x1 - x0, y1 - y0)
    obs = smooth_field(x - x0, y - y0, side, hyper.length_scale, seed) + math.sqrt(hyper.sn2) * normal(seed + 1, n)
    gx = np.linspace(x0, x1, grid_w)
    gy = np.linspace(y0, y1, grid_h)
    QY, QX = np.meshgrid(gy, gx, indexing="ij")
    f_min = float(np.percentile(obs, 40.0))
    return Workload(name or f"lpsc_box_n{n}_g{grid_w}x{grid_h}", x, y, obs, QX.reshape(-1), QY.reshape(-1),
                    grid_w, grid_h, hyper, f_min, seed=seed)


def clustered(n: int, grid_w: int, grid_h: int | None = None, seed: int = 0, clusters: int = 64,
              spread: float = 0.15, hyper: Hyper | None = None, name: str | None = None) -> Workload:
    """``synthetic``'s square and bounding box (corner points pinned), but the
    N points in ``clusters`` tight Gaussian clusters of s.d. ``spread`` (ADVICE
    r5: the same box area as C4-like data -- what SBO_OPT_INV_OZ_ADAPT takes
    for "the same data" -- at another density, so conditioning differs);
    observations = smooth field + N(0, sn2)."""
    hyper = hyper or Hyper()
    grid_h = grid_h or grid_w
    side = hyper.length_scale * math.sqrt(n / 8.0)
    u = uniform(seed ^ 0xC1, 2 * clusters + n)
    cx, cy = u[0:2 * clusters:2] * side, u[1:2 * clusters:2] * side
    k = np.minimum((u[2 * clusters:] * clusters).astype(np.int64), clusters - 1)
    x = np.clip(cx[k] + spread * normal(seed + 2, n), 0.0, side)
    y = np.clip(cy[k] + spread * normal(seed + 3, n), 0.0, side)
    x[0], y[0], x[-1], y[-1] = 0.0, 0.0, side, side
    obs = smooth_field(x, y, side, hyper.length_scale, seed) + math.sqrt(hyper.sn2) * normal(seed + 1, n)
    gx = np.linspace(0.0, side, grid_w)
    gy = np.linspace(0.0, side, grid_h)
    QY, QX = np.meshgrid(gy, gx, indexing="ij")
    f_min = float(np.percentile(obs, 40.0))
    return Workload(name or f"clustered_n{n}_g{grid_w}x{grid_h}", x, y, obs, QX.reshape(-1), QY.reshape(-1),
                    grid_w, grid_h, hyper, f_min, side=side, seed=seed)


def robot_path(n: int, side: float, seed: int = 0, v_max: float = 0.3, w_max: float = 1.0):
    """Training locations shaped like the publisher's stream: 30 points
    uniform within radius 1 of the start pose (turtlesim_spatial_publisher.py
    :111-149), then one sample per second at the robot pose (:43, :151-183).

    The robot follows waypoints the way reactive_navigation drives it: heading
    turned toward the waypoint at <= ``w_max`` rad/s, speed
    min(v_max, leg speed, distance) (config/reactive_planner.yaml:9-12: gains
    1.0, 0.3 m/s, 1 rad/s), and it waits a few ticks at every waypoint (the
    planner replans on each new sample, :552-566).  Leg speeds are U[0.02,
    v_max]: slow legs lay dense lines of points (one per 0.02 units, l/20),
    fast ones sparse ones, dwells exact duplicates -- clustered, path-shaped
    data on a domain of side ``side`` that the path covers only in part."""
    u = uniform(seed ^ 0xBA7, 8 * n + 64)
    ang = 2.0 * math.pi * u[0:60:2]
    dist = u[1:60:2]
    c = side / 2.0
    x = np.empty(n)
    y = np.empty(n)
    k0 = min(30, n)
    x[:k0] = np.clip(c + dist[:k0] * np.cos(ang[:k0]), 0.1, side - 0.1)
    y[:k0] = np.clip(c + dist[:k0] * np.sin(ang[:k0]), 0.1, side - 0.1)
    px, py, th = c, c, 0.0
    wx = wy = c
    leg_v = v_max
    dwell = 0
    j = 64
    for i in range(k0, n):
        if dwell > 0:
            dwell -= 1
        else:
            dx, dy = wx - px, wy - py
            d = math.hypot(dx, dy)
            if d < 0.05:
                # a new waypoint 2-10 units away, inside the domain; dwell 0-8 ticks
                a = 2.0 * math.pi * u[j]
                r = 2.0 + 8.0 * u[j + 1]
                wx = min(max(px + r * math.cos(a), 0.5), side - 0.5)
                wy = min(max(py + r * math.sin(a), 0.5), side - 0.5)
                leg_v = 0.02 + (v_max - 0.02) * u[j + 2]
                dwell = int(9 * u[j + 3])
                j += 4
            else:
                err = math.atan2(dy, dx) - th
                err = (err + math.pi) % (2.0 * math.pi) - math.pi
                th += max(-w_max, min(w_max, err))
                v = min(leg_v, d) * max(0.0, math.cos(err))
                px = min(max(px + v * math.cos(th), 0.1), side - 0.1)
                py = min(max(py + v * math.sin(th), 0.1), side - 0.1)
        x[i], y[i] = px, py
    return x, y


def path_workload(n: int, grid_w: int = 1000, grid_h: int | None = None, side: float | None = None, seed: int = 0,
                  hyper: Hyper | None = None, name: str | None = None) -> Workload:
    """Path-clustered workload: ``robot_path`` training
    locations on a square of side 150 l (60 units at l = 0.4) by default,
    observations = smooth field + N(0, sn2), a grid_w x grid_h query grid over
    the data bounds, f_min = 40th percentile of the observations."""
    hyper = hyper or Hyper()
    grid_h = grid_h or grid_w
    side = side or 150.0 * hyper.length_scale
    x, y = robot_path(n, side, seed)
    obs = smooth_field(x, y, side, hyper.length_scale, seed) + math.sqrt(hyper.sn2) * normal(seed + 1, n)
    gx = np.linspace(x.min(), x.max(), grid_w)
    gy = np.linspace(y.min(), y.max(), grid_h)
    QY, QX = np.meshgrid(gy, gx, indexing="ij")
    f_min = float(np.percentile(obs, 40.0))
    return Workload(name or f"path_n{n}_g{grid_w}x{grid_h}", x, y, obs, QX.reshape(-1), QY.reshape(-1),
                    grid_w, grid_h, hyper, f_min, side=side, seed=seed)


def more_points(wl: Workload, k: int, seed: int = 99):
    """k further measurements for a synthetic workload (the node's trigger:
    one new point per spatial_data_size change, node.cpp:552-566): locations
    uniform over the training points' bounding box, observations from the
    workload's own field + N(0, sn2).  Returns (x, y, obs) as f64 arrays."""
    if wl.side is None:
        raise ValueError("more_points: workload without a field square (synthetic / path_workload only)")
    u = uniform(seed ^ 0xADD, 2 * k)
    x = wl.x.min() + u[0::2] * (wl.x.max() - wl.x.min())
    y = wl.y.min() + u[1::2] * (wl.y.max() - wl.y.min())
    h = wl.hyper
    obs = smooth_field(x, y, wl.side, h.length_scale, wl.seed) + math.sqrt(h.sn2) * normal(seed + 7, k)
    return x, y, obs


def make_terrain_csv(rows: int = 48, cols: int = 64, seed: int = 7) -> np.ndarray:
    """Stand-in for the missing data/terrain.csv: a smooth stiffness-like field
    in [700, 1100] (config/lpsc.yaml:5 stiffness_range)."""
    r = np.arange(rows, dtype=np.float64)
    c = np.arange(cols, dtype=np.float64)
    R, Cc = np.meshgrid(r, c, indexing="ij")
    f = smooth_field(Cc, R, float(max(rows, cols)), max(rows, cols) / 16.0, seed, bumps=12)
    f = (f - f.min()) / (f.max() - f.min())
    return 700.0 + 400.0 * f


def write_terrain_csv(path: str, data: np.ndarray) -> None:
    np.savetxt(path, data, delimiter=",", header="terrain", comments="", fmt="%.6f")


def load_terrain_csv(path: str) -> np.ndarray:
    return np.loadtxt(path, delimiter=",", skiprows=1)


def terrain_value(terrain: np.ndarray, px, py, scale_factor: float = 10.0):
    """``get_terrain_value`` (turtlesim_spatial_publisher.py:77-100), vectorised."""
    rows, cols = terrain.shape
    x_min, x_max = -cols / 2.0, cols / 2.0
    y_min, y_max = -rows / 2.0, rows / 2.0
    tx = np.asarray(px, np.float64) * scale_factor
    ty = np.asarray(py, np.float64) * scale_factor
    col = ((tx - x_min) / (x_max - x_min) * (cols - 1)).astype(np.int64)
    row = ((ty - y_min) / (y_max - y_min) * (rows - 1)).astype(np.int64)
    col = np.clip(col, 0, cols - 1)
    row = np.clip(row, 0, rows - 1)
    v = terrain[row, col]
    return (v - terrain.min()) / (terrain.max() - terrain.min()) * 10.0


def c1_workload(terrain: np.ndarray, n_total: int = 200, grid: int = 100, seed: int = 1,
                f_min: float | None = None) -> Workload:
    """C1: ~200 measurements on the terrain stand-in and a grid x grid query map.

    30 initial points within radius 1 of the start pose (clamped 0.1 inside the
    terrain bounds, publisher :116-134), then the robot drives a lissajous path
    and publishes one measurement per tick (:151-183)."""
    rows, cols = terrain.shape
    sf = 10.0
    xmin, xmax = -cols / 2.0 / sf + 0.1, cols / 2.0 / sf - 0.1
    ymin, ymax = -rows / 2.0 / sf + 0.1, rows / 2.0 / sf - 0.1
    u = uniform(seed, 60)
    ang = 2.0 * math.pi * u[0::2]
    dist = u[1::2]
    sx, sy = 0.0, 0.0
    ix = np.clip(sx + dist * np.cos(ang), xmin, xmax)
    iy = np.clip(sy + dist * np.sin(ang), ymin, ymax)
    t = np.arange(n_total - 30, dtype=np.float64)
    px = np.clip(0.8 * (xmax - 0.1) * np.sin(0.031 * t), xmin, xmax)
    py = np.clip(0.8 * (ymax - 0.1) * np.sin(0.047 * t + 0.5), ymin, ymax)
    x = np.concatenate([ix, px])
    y = np.concatenate([iy, py])
    obs = terrain_value(terrain, x, y, sf)
    gx = np.linspace(-cols / 2.0 / sf, cols / 2.0 / sf, grid)
    gy = np.linspace(-rows / 2.0 / sf, rows / 2.0 / sf, grid)
    QY, QX = np.meshgrid(gy, gx, indexing="ij")
    hyper = Hyper()
    if f_min is None:
        f_min = float(np.percentile(obs, 40.0))
    return Workload("C1", x, y, obs, QX.reshape(-1), QY.reshape(-1), grid, grid, hyper, f_min)


CONFIGS = {
    # name: (N, grid_w, grid_h)   -- BASELINE.json configs[1..4]
    "C2": (2048, 256, 256),
    "C3": (8192, 1024, 1024),
    "C4": (16384, 1000, 1000),
}
