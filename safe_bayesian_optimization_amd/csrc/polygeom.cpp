// polygeom.cpp -- host side of the node's post-selection geometry (SURVEY.md
// §8(f)4; no device: O(vertices) per tick, run once on the chosen subgoal).
//
//   goal short-circuit   src/safe_bayesian_optimization_node.cpp:651-666  (bg::within)
//   ring copy + correct  src/safe_bayesian_optimization_node.cpp:675-682  (bg::correct)
//   subgoal projection   src/safe_bayesian_optimization_node.cpp:688-704  -> polydist
//   polydist             src/libraries/polygeom_lib.cpp:401-474
//
// Rings are passed as Boost stores them: x[] and y[] of the exterior ring,
// closing point included (polygon<point, false, true> is counter-clockwise
// and closed, include/polygeom_lib.h:60).
//
// polydist quirk kept on purpose: the reference sets
// VertexListRolled[j] = VertexList[j] (polygeom_lib.cpp:439-440), so the
// candidate point of edge i is (1-w)*V[i] + w*V[i] -- vertex i up to the
// rounding of that blend -- and the "projection" is the nearest vertex.  The
// blend, the edge weights w and the distances are evaluated exactly as the
// reference writes them (no FMA: the library is built with
// -ffp-contract=off; pow(d, 2) is d*d, which GCC folds it to) so ties and
// roundings match.  Boost's own algorithms (correct, within) are third-party
// code absent from the tree (Boost version unpinned); they are restated from
// their documented behaviour.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

// bg::distance(point, point), cartesian pythagoras: sqrt(dx^2 + dy^2).
inline double pyth(double ax, double ay, double bx, double by) {
    const double dx = ax - bx, dy = ay - by;
    return std::sqrt(dx * dx + dy * dy);
}

// Twice the signed area of a closed ring; > 0 counter-clockwise.
double ring_area2(const double *x, const double *y, int64_t n) {
    double s = 0.0;
    for (int64_t i = 0; i + 1 < n; ++i) s += x[i] * y[i + 1] - x[i + 1] * y[i];
    return s;
}

// Side of p w.r.t. the directed segment a->b (> 0: left).
inline double side(double ax, double ay, double bx, double by, double px, double py) {
    return (bx - ax) * (py - ay) - (by - ay) * (px - ax);
}

}  // namespace
}  // namespace sbo

extern "C" {

SBO_API sbo_status sbo_polygon_correct(double *rx, double *ry, int64_t n, int64_t cap, int64_t *n_out) {
    if (!n_out || n < 0) return SBO_E_INVAL;
    *n_out = n;
    if (n == 0) return SBO_OK;
    if (!rx || !ry) return SBO_E_INVAL;
    if (n > 2 && (rx[0] != rx[n - 1] || ry[0] != ry[n - 1])) {  // close an open ring
        if (n + 1 > cap) return SBO_E_INVAL;
        rx[n] = rx[0];
        ry[n] = ry[0];
        ++n;
    }
    if (sbo::ring_area2(rx, ry, n) < 0.0) {  // clockwise -> reverse (counter-clockwise type)
        std::reverse(rx, rx + n);
        std::reverse(ry, ry + n);
    }
    *n_out = n;
    return SBO_OK;
}

SBO_API sbo_status sbo_polydist(const double *rx, const double *ry, int64_t n, double px, double py, double *proj_x,
                                double *proj_y, double *dist) {
    if (!proj_x || !proj_y || !dist || n < 0) return SBO_E_INVAL;
    if (n <= 1) {  // (:420-423), then the reference pops an empty vector: reported, not reproduced
        *dist = 100000000.0;
        *proj_x = 0.0;
        *proj_y = 0.0;
        return SBO_E_EMPTY;
    }
    if (!rx || !ry) return SBO_E_INVAL;
    const int64_t nv = n - 1;  // closing point dropped (:431)
    // dxy[j] = V[j] - V[j-1] (wrapping), |dxy[j]| with 0 -> 1   (:438-447)
    std::vector<double> dx(nv), dy(nv), dn(nv);
    for (int64_t i = 0; i < nv; ++i) {
        const int64_t j = (i + 1) % nv;
        dx[j] = rx[j] - rx[i];
        dy[j] = ry[j] - ry[i];
        const double d = sbo::pyth(dx[j], dy[j], 0.0, 0.0);
        dn[j] = d == 0.0 ? 1.0 : d;
    }
    double bd = 0.0, bx = 0.0, by = 0.0;
    for (int64_t i = 0; i < nv; ++i) {  // (:453-468); std::min_element keeps the first minimum
        const double n2 = dn[i] * dn[i];
        const double wt = (px - rx[i]) * (dx[i] / n2) + (py - ry[i]) * (dy[i] / n2);
        const double w = std::max(std::min(wt, 1.0), 0.0);
        const double cx = (1 - w) * rx[i] + w * rx[i];  // VertexListRolled[i] == VertexList[i]
        const double cy = (1 - w) * ry[i] + w * ry[i];
        const double d = sbo::pyth(px, py, cx, cy);
        if (i == 0 || d < bd) {
            bd = d;
            bx = cx;
            by = cy;
        }
    }
    *dist = bd;
    *proj_x = bx;
    *proj_y = by;
    return SBO_OK;
}

SBO_API int sbo_point_within(const double *rx, const double *ry, int64_t n, double px, double py) {
    if (!rx || !ry || n < 3) return 0;
    int wn = 0;
    for (int64_t i = 0; i < n; ++i) {
        const int64_t j = (i + 1) % n;
        const double ax = rx[i], ay = ry[i], bx = rx[j], by = ry[j];
        if (ax == bx && ay == by) continue;
        const double s = sbo::side(ax, ay, bx, by, px, py);
        if (s == 0.0 && std::min(ax, bx) <= px && px <= std::max(ax, bx) && std::min(ay, by) <= py &&
            py <= std::max(ay, by))
            return 0;  // on the boundary: not within
        if (ay <= py) {
            if (by > py && s > 0.0) ++wn;
        } else if (by <= py && s < 0.0) {
            --wn;
        }
    }
    return wn != 0;
}

SBO_API int sbo_project_subgoal(const double *rx, const double *ry, int64_t n, double goal_x, double goal_y,
                                int64_t subgoal_index, const double *Dx, const double *Dy, int64_t m, double *out_x,
                                double *out_y, double *out_dist) {
    if (!out_x || !out_y || !out_dist || n < 0) return -1;
    if (sbo_point_within(rx, ry, n, goal_x, goal_y)) {  // (:657-666)
        *out_x = goal_x;
        *out_y = goal_y;
        *out_dist = 0.0;
        return 1;
    }
    if (subgoal_index < 0 || subgoal_index >= m || !Dx || !Dy || !rx || !ry) return -1;  // (:670)
    std::vector<double> cx(rx, rx + n), cy(ry, ry + n);
    cx.push_back(0.0);
    cy.push_back(0.0);
    int64_t nc = n;
    if (sbo_polygon_correct(cx.data(), cy.data(), n, n + 1, &nc) != SBO_OK) return -1;  // (:676-682)
    if (sbo_polydist(cx.data(), cy.data(), nc, Dx[subgoal_index], Dy[subgoal_index], out_x, out_y, out_dist) !=
        SBO_OK)
        return -1;
    return 0;
}

}  // extern "C"
