// sbo_node.hpp -- C++ host mirror of the reference node's hot-path API over
// the libsbo C ABI (include/sbo.h).  Header only; link with -lsbo.
//
// Mirrors OptimizerNode in
// /root/reference/src/safe_bayesian_optimization_node.cpp:
//   state   D_ (:132, here SoA Dx_/Dy_ = the two Eigen columns), mu_, std_ (:129-130),
//           Q_ (:134, here Qlo_/Qhi_), S_ (:133), beta_, f_min_ (:136-137),
//           terrain_width_cells_, terrain_height_cells_ (:167-168), current goal (:171)
//   process_terrain_map (:625-647)   ComputeSets / ComputeConfidenceIntervals / UpdateSafeSet (:399-416)
//   FindSafetyContourIndices (:418-497)   GetNextSubgoal (:499-550)
// and the mapper side of the GetTerrainMapWithUncertainty service
// (response fields :606-644) as TerrainMapper.
//
// Error behaviour follows the node: failures return false / -1 and leave a
// message in last_error() (the node logs a warning and returns); only the
// constructors throw, as the node's constructor does for bad parameters
// (:61-66).
#pragma once

#include <algorithm>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "sbo.h"

namespace sbo {

// GetTerrainMapWithUncertainty::Response, in the order the node reads it.
struct TerrainMap {
    bool success = false;
    std::string message;
    int n_width_cells = 0;
    int n_height_cells = 0;
    std::vector<double> x_coords, y_coords;
    std::vector<float> values;         // mu
    std::vector<float> uncertainties;  // sigma
};

class Context {
public:
    explicit Context(int device = 0) {
        if (sbo_create(device, &ctx_) != SBO_OK) throw std::runtime_error("sbo_create failed");
    }
    ~Context() { sbo_destroy(ctx_); }
    Context(const Context &) = delete;
    Context &operator=(const Context &) = delete;
    sbo_ctx *get() const { return ctx_; }
    std::string last_error() const { return sbo_last_error(ctx_); }

    // FindSafetyContourIndices / GetNextSubgoal on device-resident grid data
    // (e.g. the tick's own lo/hi/S outputs): GPU raster, host border follow.
    std::vector<int32_t> frontier_device(const double *Dx, const double *Dy, const uint8_t *safe, int64_t m,
                                         int width, int height) const {
        int64_t count = 0;
        std::vector<int32_t> out((size_t)8 * (size_t)std::max(width, 1) * (size_t)std::max(height, 1) + 16);
        if (sbo_frontier(ctx_, Dx, Dy, safe, m, width, height, out.data(), (int64_t)out.size(), &count,
                         SBO_DEVICE_PTRS) != SBO_OK)
            throw std::runtime_error("sbo_frontier: " + last_error());
        out.resize((size_t)count);
        return out;
    }
    int64_t subgoal_device(const double *Dx, const double *Dy, const double *lo, const double *hi,
                           const uint8_t *safe, int64_t m, int width, int height, double gx, double gy) const {
        int64_t idx = -1;
        if (sbo_subgoal(ctx_, Dx, Dy, lo, hi, safe, m, width, height, gx, gy, &idx, SBO_DEVICE_PTRS) != SBO_OK)
            throw std::runtime_error("sbo_subgoal: " + last_error());
        return idx;
    }

private:
    sbo_ctx *ctx_ = nullptr;
};

// The GP mapper (external terrain_mapping_node in the reference).
class TerrainMapper {
public:
    explicit TerrainMapper(Context &ctx, sbo_hyper hyper = sbo_hyper{0.4, 1.0, 0.1, 0.0}) : ctx_(ctx), hyper_(hyper) {}

    bool fit(const std::vector<float> &x, const std::vector<float> &y, const std::vector<float> &obs) {
        if (x.size() != y.size() || x.size() != obs.size()) return fail("fit: size mismatch");
        return ok(sbo_fit(ctx_.get(), x.data(), y.data(), obs.data(), (int64_t)x.size(), hyper_, 0));
    }
    bool append(const std::vector<float> &x, const std::vector<float> &y, const std::vector<float> &obs) {
        if (x.size() != y.size() || x.size() != obs.size()) return fail("append: size mismatch");
        return ok(sbo_append(ctx_.get(), x.data(), y.data(), obs.data(), (int64_t)x.size(), 0));
    }
    // Serve a map over the given grid (row-major, width x height).
    TerrainMap grid(const std::vector<double> &gx, const std::vector<double> &gy, int width, int height) {
        TerrainMap r;
        const size_t m = gx.size();
        if (m != gy.size() || m != (size_t)width * (size_t)height) {
            r.message = "grid: size mismatch";
            return r;
        }
        std::vector<float> qx(gx.begin(), gx.end()), qy(gy.begin(), gy.end());
        r.values.resize(m);
        r.uncertainties.resize(m);
        const sbo_status st = sbo_predict(ctx_.get(), qx.data(), qy.data(), (int64_t)m, r.values.data(),
                                          r.uncertainties.data(), 0);
        if (st != SBO_OK) {
            r.message = ctx_.last_error();
            return r;
        }
        r.success = true;
        r.message = "ok";
        r.n_width_cells = width;
        r.n_height_cells = height;
        r.x_coords = gx;
        r.y_coords = gy;
        return r;
    }
    const std::string &last_error() const { return err_; }

private:
    bool ok(sbo_status s) {
        if (s == SBO_OK) return true;
        err_ = std::string(sbo_status_string(s)) + ": " + ctx_.last_error();
        return false;
    }
    bool fail(const char *m) {
        err_ = m;
        return false;
    }
    Context &ctx_;
    sbo_hyper hyper_;
    std::string err_;
};

// The node side: ComputeSets on the device, frontier + subgoal on the host.
class OptimizerCore {
public:
    OptimizerCore(Context &ctx, double beta = 2.0, double f_min = 0.0) : ctx_(ctx), beta_(beta), f_min_(f_min) {}

    void goal_point_callback(double x, double y) { goal_ = {x, y}; }

    // :625-647 -- unpack the response, then ComputeSets().
    bool process_terrain_map(const TerrainMap &r) {
        if (!r.success) {
            err_ = "Terrain map request failed: " + r.message;
            return false;
        }
        terrain_width_cells_ = r.n_width_cells;
        terrain_height_cells_ = r.n_height_cells;
        Dx_ = r.x_coords;
        Dy_ = r.y_coords;
        mu_.assign(r.values.begin(), r.values.end());               // :641-643: widened into VectorXd
        std_.assign(r.uncertainties.begin(), r.uncertainties.end());
        return ComputeSets();
    }

    // :399-416 -- c = beta*std; Q(:,0) = mu - c; Q(:,1) = mu + c; S = Q(:,0) > f_min
    bool ComputeSets() {
        const size_t m = mu_.size();
        Qlo_.assign(m, 0.0);
        Qhi_.assign(m, 0.0);
        S_.assign(m, 0);
        if (m == 0) return true;
        const sbo_status st = sbo_compute_sets_f64(ctx_.get(), mu_.data(), std_.data(), (int64_t)m, beta_, f_min_,
                                               Qlo_.data(), Qhi_.data(), S_.data(), 0);
        if (st != SBO_OK) {
            err_ = ctx_.last_error();
            return false;
        }
        return true;
    }

    std::vector<int> FindSafetyContourIndices() const {
        const int64_t m = (int64_t)Dx_.size();
        if (m == 0 || S_.empty()) return {};
        std::vector<int32_t> out((size_t)8 * std::max(1, terrain_width_cells_) * std::max(1, terrain_height_cells_) + 16);
        int64_t cnt = 0;
        if (sbo_find_safety_contour_indices(Dx_.data(), Dy_.data(), S_.data(), m, terrain_width_cells_,
                                            terrain_height_cells_, out.data(), (int64_t)out.size(), &cnt) != SBO_OK)
            return {};
        return std::vector<int>(out.begin(), out.begin() + cnt);
    }

    int GetNextSubgoal() const {
        return (int)sbo_next_subgoal(Dx_.data(), Dy_.data(), Qlo_.data(), Qhi_.data(), S_.data(), (int64_t)Dx_.size(),
                                     terrain_width_cells_, terrain_height_cells_, goal_.first, goal_.second);
    }

    // The node's subgoal step (:651-704): the goal when it lies inside the
    // eroded safe ring, else the frontier subgoal projected by polydist onto
    // it.  ring_x/ring_y: the polygon's outer() (closing point included).
    // Returns 1 (goal), 0 (projected) or -1 (no subgoal); *xy, *dist out.
    int ProjectSubgoal(const std::vector<double> &ring_x, const std::vector<double> &ring_y, double *x, double *y,
                       double *dist) const {
        const int64_t n = (int64_t)ring_x.size();
        if (sbo_point_within(ring_x.data(), ring_y.data(), n, goal_.first, goal_.second)) {  // no frontier needed
            *x = goal_.first;
            *y = goal_.second;
            *dist = 0.0;
            return 1;
        }
        return sbo_project_subgoal(ring_x.data(), ring_y.data(), (int64_t)ring_x.size(), goal_.first, goal_.second,
                                   GetNextSubgoal(), Dx_.data(), Dy_.data(), (int64_t)Dx_.size(), x, y, dist);
    }

    const std::vector<double> &Qlo() const { return Qlo_; }
    const std::vector<double> &Qhi() const { return Qhi_; }
    const std::vector<uint8_t> &S() const { return S_; }
    const std::string &last_error() const { return err_; }

private:
    Context &ctx_;
    double beta_, f_min_;
    std::vector<double> Dx_, Dy_, Qlo_, Qhi_;
    std::vector<double> mu_, std_;   // Eigen::VectorXd mu_, std_ (:129-130)
    std::vector<uint8_t> S_;
    int terrain_width_cells_ = 0, terrain_height_cells_ = 0;
    std::pair<double, double> goal_{0.0, 0.0};
    std::string err_;
};

}  // namespace sbo
