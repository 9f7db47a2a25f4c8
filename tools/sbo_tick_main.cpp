// sbo_tick_main.cpp -- one ROS-free planning tick driven
// from C++ through include/sbo_node.hpp:
//   measurements -> TerrainMapper::fit -> TerrainMapper::grid (service
//   response) -> OptimizerCore::process_terrain_map (ComputeSets on the
//   device) -> GetNextSubgoal (host frontier), plus the fused device tick
//   (sbo_tick) whose grid argmax is cross-checked against the node path.
// The workload is terrain.synthetic() restated (counter-based SplitMix64),
// so Python and C++ build the same inputs.
//
//   sbo_tick_main N GRID_W GRID_H [SEED] [GOAL_X GOAL_Y]
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sbo_node.hpp"

namespace {

uint64_t splitmix(uint64_t seed, uint64_t ctr) {
    uint64_t z = seed + ctr * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
double uniform(uint64_t seed, uint64_t i) { return (double)(splitmix(seed, i + 1) >> 11) * (1.0 / 9007199254740992.0); }
double normal(uint64_t seed, uint64_t i) {
    const double u1 = std::max(uniform(seed, 2 * i), 1e-300), u2 = uniform(seed, 2 * i + 1);
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
}
double field(double px, double py, double side, double ell, uint64_t seed) {
    const uint64_t s = seed ^ 0x5EED;
    double f = 0.0;
    for (int b = 0; b < 32; ++b) {
        const double cx = uniform(s, 4 * b) * side, cy = uniform(s, 4 * b + 1) * side;
        const double w = (2.0 + 2.0 * uniform(s, 4 * b + 2)) * ell, a = 2.0 * uniform(s, 4 * b + 3) - 1.0;
        f += a * std::exp(-((px - cx) * (px - cx) + (py - cy) * (py - cy)) / (2.0 * w * w));
    }
    return f;
}

}  // namespace

int main(int argc, char **argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s N GRID_W GRID_H [SEED] [GOAL_X GOAL_Y]\n", argv[0]);
        return 2;
    }
    const int64_t n = std::atoll(argv[1]);
    const int gw = std::atoi(argv[2]), gh = std::atoi(argv[3]);
    const uint64_t seed = argc > 4 ? std::strtoull(argv[4], nullptr, 10) : 0;
    const double goal_x = argc > 6 ? std::atof(argv[5]) : 0.0, goal_y = argc > 6 ? std::atof(argv[6]) : 0.0;
    const sbo_hyper h{0.4, 1.0, 0.1, 0.0};
    const double side = h.length_scale * std::sqrt(n / 8.0);

    std::vector<float> x(n), y(n), obs(n);
    std::vector<double> o64(n);
    for (int64_t i = 0; i < n; ++i) {
        const double xi = uniform(seed, 2 * i) * side, yi = uniform(seed, 2 * i + 1) * side;
        x[i] = (float)xi;
        y[i] = (float)yi;
        o64[i] = field(xi, yi, side, h.length_scale, seed) + std::sqrt(h.noise_level) * normal(seed + 1, i);
        obs[i] = (float)o64[i];
    }
    std::vector<double> sorted(o64);
    std::sort(sorted.begin(), sorted.end());
    const double pos = 0.4 * (double)(n - 1);
    const int64_t lo_i = (int64_t)pos;
    const double f_min = sorted[lo_i] + (pos - lo_i) * (sorted[std::min<int64_t>(lo_i + 1, n - 1)] - sorted[lo_i]);

    std::vector<double> gx((size_t)gw * gh), gy((size_t)gw * gh);
    for (int r = 0; r < gh; ++r)
        for (int c = 0; c < gw; ++c) {
            gx[(size_t)r * gw + c] = gw > 1 ? side * c / (gw - 1) : 0.0;
            gy[(size_t)r * gw + c] = gh > 1 ? side * r / (gh - 1) : 0.0;
        }

    sbo::Context ctx(0);
    sbo::TerrainMapper mapper(ctx, h);
    auto t0 = std::chrono::steady_clock::now();
    if (!mapper.fit(x, y, obs)) {
        std::fprintf(stderr, "fit failed: %s\n", mapper.last_error().c_str());
        return 1;
    }
    auto t1 = std::chrono::steady_clock::now();
    const sbo::TerrainMap map = mapper.grid(gx, gy, gw, gh);
    if (!map.success) {
        std::fprintf(stderr, "grid failed: %s\n", map.message.c_str());
        return 1;
    }
    auto t2 = std::chrono::steady_clock::now();
    sbo::OptimizerCore node(ctx, 2.0, f_min);
    node.goal_point_callback(goal_x, goal_y);
    if (!node.process_terrain_map(map)) {
        std::fprintf(stderr, "process_terrain_map failed: %s\n", node.last_error().c_str());
        return 1;
    }
    const int subgoal = node.GetNextSubgoal();
    const size_t frontier = node.FindSafetyContourIndices().size();
    auto t3 = std::chrono::steady_clock::now();

    // fused device tick on the same grid: its argmax must be the node's width argmax over S
    std::vector<float> qx(gx.begin(), gx.end()), qy(gy.begin(), gy.end());
    sbo_key key{0.0, -1};
    if (sbo_tick(ctx.get(), qx.data(), qy.data(), (int64_t)qx.size(), 2.0, f_min, SBO_SCORE_WIDTH, 0, nullptr,
                 nullptr, nullptr, nullptr, nullptr, &key, 0) != SBO_OK) {
        std::fprintf(stderr, "tick failed: %s\n", ctx.last_error().c_str());
        return 1;
    }
    int64_t best = -1;
    double bw = 0.0;
    for (size_t i = 0; i < node.S().size(); ++i)
        if (node.S()[i]) {
            const double w = node.Qhi()[i] - node.Qlo()[i];
            if (best < 0 || w > bw) { best = (int64_t)i; bw = w; }
        }
    const auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    size_t nsafe = 0;
    for (uint8_t s : node.S()) nsafe += s;
    std::printf("{\"n\": %lld, \"m\": %zu, \"f_min\": %.17g, \"safe\": %zu, \"frontier\": %zu, \"subgoal\": %d, "
                "\"tick_argmax\": %lld, \"tick_score\": %.17g, \"node_argmax\": %lld, \"fit_ms\": %.3f, "
                "\"map_ms\": %.3f, \"node_ms\": %.3f}\n",
                (long long)n, gx.size(), f_min, nsafe, frontier, subgoal, (long long)key.idx, key.score,
                (long long)best, ms(t0, t1), ms(t1, t2), ms(t2, t3));
    return key.idx == best ? 0 : 3;
}
