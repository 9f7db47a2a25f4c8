"""Host-side mirror of the reference node's hot-path API.

``OptimizerCore`` keeps the member state and method names of
``OptimizerNode`` (/root/reference/src/safe_bayesian_optimization_node.cpp):

    D_, mu_, std_, Q_, S_                      :129-134
    beta_, f_min_                              :136-137, params :48-58
    terrain_width_cells_, terrain_height_cells_ :167-168
    current_goal_ (defaults to (0, 0))         :171, :1324-1327
    process_terrain_map(response)              :625-647 (unpack + ComputeSets)
    ComputeSets / ComputeConfidenceIntervals / UpdateSafeSet   :399-416
    FindSafetyContourIndices                   :418-497
    GetNextSubgoal                             :499-550

ComputeSets runs on the GPU (libsbo ``sbo_compute_sets_f64`` on the node's
f64 ``mu_``/``std_``, IEEE double, no FMA); the frontier and the subgoal
selection run in libsbo's host code, as do the post-selection geometry the
node applies to the subgoal (``bg::within`` goal short-circuit, ring
``bg::correct``, ``polydist`` projection: ``ProjectSubgoal``, :649-723).  The
ROS transport and the construction of the eroded safe-set hull (CGAL alpha
shapes, Boost buffer, :725-1200) are out of scope.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N
from .gp import Context, TerrainMapResponse, _ptr


class OptimizerCore:
    def __init__(self, beta: float = 2.0, f_min: float = 0.0, device: int = 0, ctx: Context | None = None):
        # node.cpp:48-58 defaults: opt.beta 2.0, opt.f_min 0.0
        self.beta_ = float(beta)
        self.f_min_ = float(f_min)
        self.ctx = ctx
        self._device = device
        self.D_ = np.zeros((0, 2), np.float64)
        self.mu_ = np.zeros(0, np.float64)    # Eigen::VectorXd (:129-130)
        self.std_ = np.zeros(0, np.float64)
        self.Q_ = np.zeros((0, 2), np.float64)
        self.S_ = np.zeros(0, np.uint8)
        self.terrain_width_cells_ = 0
        self.terrain_height_cells_ = 0
        self.current_goal_ = (0.0, 0.0)
        self._lib = N.lib()

    # ---------------------------------------------------------- callbacks
    def goal_point_callback(self, x: float, y: float) -> None:
        self.current_goal_ = (float(x), float(y))

    def process_terrain_map(self, response: TerrainMapResponse) -> None:
        """Unpack the service response (:631-644) and ComputeSets() (:647)."""
        if not response.success:
            raise RuntimeError(f"Terrain map request failed: {response.message}")
        self.terrain_width_cells_ = int(response.n_width_cells)
        self.terrain_height_cells_ = int(response.n_height_cells)
        m = len(response.x_coords)
        D = np.empty((m, 2), np.float64)
        D[:, 0] = np.asarray(response.x_coords, np.float64)
        D[:, 1] = np.asarray(response.y_coords, np.float64)
        self.D_ = D
        self.mu_ = np.ascontiguousarray(response.values, np.float64)          # :641-643, widened as Eigen does
        self.std_ = np.ascontiguousarray(response.uncertainties, np.float64)
        self.ComputeSets()

    # ---------------------------------------------------------- acquisition
    def ComputeSets(self) -> None:
        """ComputeConfidenceIntervals() then UpdateSafeSet() (:399-407), fused
        into one device pass."""
        m = self.mu_.size
        lo = np.empty(m, np.float64)
        hi = np.empty(m, np.float64)
        s = np.empty(m, np.uint8)
        if m:
            ctx = self._context()
            ctx.check(self._lib.sbo_compute_sets_f64(ctx.handle, _ptr(self.mu_), _ptr(self.std_), m, self.beta_,
                                                     self.f_min_, _ptr(lo), _ptr(hi), _ptr(s), 0))
        self.Q_ = np.stack([lo, hi], axis=1)
        self.S_ = s

    def ComputeConfidenceIntervals(self) -> None:
        self.ComputeSets()

    def UpdateSafeSet(self) -> None:
        """S_ = Q_.col(0) > f_min_ (:409) -- recomputed from the current Q_."""
        self.S_ = (self.Q_[:, 0] > self.f_min_).astype(np.uint8)

    # -------------------------------------------------------------- frontier
    def FindSafetyContourIndices(self) -> np.ndarray:
        m = self.D_.shape[0]
        if m == 0 or self.S_.size == 0:
            return np.zeros(0, np.int32)  # "D_ or S_ is empty" (:419-422)
        Dx = np.ascontiguousarray(self.D_[:, 0])
        Dy = np.ascontiguousarray(self.D_[:, 1])
        cap = 8 * max(1, self.terrain_width_cells_) * max(1, self.terrain_height_cells_) + 16
        out = np.empty(cap, np.int32)
        cnt = ctypes.c_int64(0)
        st = self._lib.sbo_find_safety_contour_indices(_ptr(Dx), _ptr(Dy), _ptr(np.ascontiguousarray(self.S_)), m,
                                                       self.terrain_width_cells_, self.terrain_height_cells_,
                                                       _ptr(out), cap, ctypes.byref(cnt))
        N.check(st)
        return out[:cnt.value].copy()

    def GetNextSubgoal(self) -> int:
        m = self.D_.shape[0]
        if m == 0:
            return -1
        Dx = np.ascontiguousarray(self.D_[:, 0])
        Dy = np.ascontiguousarray(self.D_[:, 1])
        lo = np.ascontiguousarray(self.Q_[:, 0])
        hi = np.ascontiguousarray(self.Q_[:, 1])
        return int(self._lib.sbo_next_subgoal(_ptr(Dx), _ptr(Dy), _ptr(lo), _ptr(hi),
                                              _ptr(np.ascontiguousarray(self.S_)), m, self.terrain_width_cells_,
                                              self.terrain_height_cells_, self.current_goal_[0],
                                              self.current_goal_[1]))

    def _context(self) -> Context:
        if self.ctx is None:
            self.ctx = Context(self._device)
        return self.ctx


def find_contours_external(img: np.ndarray):
    """libsbo's restatement of cv::findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    pcap = 8 * w * h + 16
    ccap = w * h + 1
    pts = np.empty(2 * pcap, np.int32)
    st = np.empty(ccap + 1, np.int64)
    nc = N.lib().sbo_find_contours_external(_ptr(img), w, h, _ptr(pts), pcap, _ptr(st), ccap)
    if nc < 0:
        raise RuntimeError("contour capacity exceeded")
    pts = pts.reshape(-1, 2)
    return [pts[st[c]:st[c + 1]].copy() for c in range(nc)]


def find_safety_contour_indices(Dx, Dy, safe, width: int, height: int) -> np.ndarray:
    Dx = np.ascontiguousarray(Dx, np.float64)
    Dy = np.ascontiguousarray(Dy, np.float64)
    safe = np.ascontiguousarray(safe, np.uint8)
    cap = 8 * max(1, width) * max(1, height) + 16
    out = np.empty(cap, np.int32)
    cnt = ctypes.c_int64(0)
    N.check(N.lib().sbo_find_safety_contour_indices(_ptr(Dx), _ptr(Dy), _ptr(safe), Dx.size, int(width),
                                                    int(height), _ptr(out), cap, ctypes.byref(cnt)))
    return out[:cnt.value].copy()


def next_subgoal(Dx, Dy, lo, hi, safe, width: int, height: int, gx: float = 0.0, gy: float = 0.0) -> int:
    c = lambda a, dt: np.ascontiguousarray(a, dt)  # noqa: E731
    Dx, Dy, lo, hi = (c(a, np.float64) for a in (Dx, Dy, lo, hi))
    safe = c(safe, np.uint8)
    return int(N.lib().sbo_next_subgoal(_ptr(Dx), _ptr(Dy), _ptr(lo), _ptr(hi), _ptr(safe), Dx.size, int(width),
                                        int(height), float(gx), float(gy)))


# ---- post-selection geometry (csrc/polygeom.cpp) ----------
def _f64(a):
    return np.ascontiguousarray(a, np.float64)


def polygon_correct(rx, ry):
    """bg::correct of the node's ring copy (:676-682): returns the closed,
    counter-clockwise ring as new arrays."""
    n = len(rx)
    cx = np.zeros(n + 1, np.float64)
    cy = np.zeros(n + 1, np.float64)
    cx[:n] = rx
    cy[:n] = ry
    out = ctypes.c_int64(0)
    N.check(N.lib().sbo_polygon_correct(_ptr(cx), _ptr(cy), n, n + 1, ctypes.byref(out)))
    return cx[:out.value].copy(), cy[:out.value].copy()


def polydist(rx, ry, px: float, py: float, status: bool = False):
    """polydist (src/libraries/polygeom_lib.cpp:401-474) -> (x, y, dist);
    with status=True the sbo_status is appended instead of raised."""
    rx, ry = _f64(rx), _f64(ry)
    ox, oy, od = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    st = N.lib().sbo_polydist(_ptr(rx), _ptr(ry), rx.size, float(px), float(py), ctypes.byref(ox),
                              ctypes.byref(oy), ctypes.byref(od))
    if status:
        return ox.value, oy.value, od.value, int(st)
    N.check(st)
    return ox.value, oy.value, od.value


def point_within(rx, ry, px: float, py: float) -> int:
    """bg::within(point, polygon) (:657): 1 strictly inside, else 0."""
    rx, ry = _f64(rx), _f64(ry)
    return int(N.lib().sbo_point_within(_ptr(rx), _ptr(ry), rx.size, float(px), float(py)))


def project_subgoal(rx, ry, goal, subgoal_index: int, Dx, Dy):
    """The node's subgoal step after GetNextSubgoal (:651-704) ->
    (code, x, y, dist): code 1 = goal used, 0 = projected frontier point, -1 = none."""
    rx, ry, Dx, Dy = _f64(rx), _f64(ry), _f64(Dx), _f64(Dy)
    ox, oy, od = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
    code = N.lib().sbo_project_subgoal(_ptr(rx), _ptr(ry), rx.size, float(goal[0]), float(goal[1]),
                                       int(subgoal_index), _ptr(Dx), _ptr(Dy), Dx.size, ctypes.byref(ox),
                                       ctypes.byref(oy), ctypes.byref(od))
    return int(code), ox.value, oy.value, od.value
