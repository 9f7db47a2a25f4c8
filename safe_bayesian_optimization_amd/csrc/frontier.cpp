// frontier.cpp -- host side of the node's subgoal selection (no device).
//
//   FindSafetyContourIndices  src/safe_bayesian_optimization_node.cpp:418-497
//   GetNextSubgoal            src/safe_bayesian_optimization_node.cpp:499-550
//
// cv::findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE) is a third-party call
// (OpenCV, version unpinned, CMakeLists.txt:28) that is absent from the
// reference tree; BorderFollower restates OpenCV 4.5.x's Suzuki-Abe border
// following: the image is zero padded by one pixel, scanned in raster order,
// an outer border starts at a 0 -> 1 transition whose last marked border
// pixel on the row is not a left/inner border pixel (so components inside a
// hole are skipped), borders are followed counter-clockwise from the first
// clockwise neighbour, right-bound pixels are marked -126 and the rest 2,
// every traversed pixel is emitted (1-px structures emit duplicates) and the
// contour list comes back in reverse discovery order.
//
// The node's O(M) unordered_map<int, unordered_map<int,int>> (:468-475) is
// a dense width x height owner array here: same last-writer-wins semantics,
// one pass, no hashing.
#include <algorithm>
#include <climits>
#include <cmath>
#include <cstdint>
#include <utility>
#include <vector>

#include "sbo_internal.hpp"

namespace sbo {
namespace {

struct Pt {
    int32_t x, y;
};

class BorderFollower {
public:
    BorderFollower(const uint8_t *img, int w, int h) : w_(w), h_(h), W_((int64_t)w + 2) {
        pad_.assign((size_t)(W_ * (h + 2)), 0);
        for (int y = 0; y < h; ++y) {
            signed char *dst = &pad_[(size_t)((y + 1) * W_ + 1)];
            const uint8_t *src = img + (int64_t)y * w;
            for (int x = 0; x < w; ++x) dst[x] = src[x] ? 1 : 0;
        }
        for (int s = 0; s < 8; ++s) step_[s] = kDx[s] + kDy[s] * W_;
    }

    // Discovery-ordered contours; caller reverses.
    void run(std::vector<Pt> &pts, std::vector<int64_t> &starts) {
        for (int64_t y = 1; y <= h_; ++y) {
            signed char *row = &pad_[(size_t)(y * W_)];
            int prev = 0;
            int64_t last_border = 0;  // column of the last marked border pixel on this row
            for (int64_t x = 1; x <= w_; ++x) {
                const int p = row[x];
                if (p == prev) continue;
                const bool outer_start = prev == 0 && p == 1 && !(row[last_border] > 0);
                if (outer_start) {
                    starts.push_back((int64_t)pts.size());
                    last_border = x;
                    follow(y * W_ + x, (int32_t)(x - 1), (int32_t)(y - 1), pts);
                    prev = row[x];
                    continue;
                }
                prev = p;
                if (p & ~1) last_border = x;
            }
        }
    }

private:
    static constexpr int kDx[8] = {1, 1, 0, -1, -1, -1, 0, 1};
    static constexpr int kDy[8] = {0, -1, -1, -1, 0, 1, 1, 1};

    void follow(int64_t start, int32_t x, int32_t y, std::vector<Pt> &pts) {
        signed char *im = pad_.data();
        // clockwise search for the first neighbour, starting after the left one
        int dir = 4;
        int64_t first = start;
        do {
            dir = (dir + 7) & 7;
            first = start + step_[dir];
        } while (im[first] == 0 && dir != 4);
        if (dir == 4) {  // isolated pixel
            im[start] = -126;
            pts.push_back({x, y});
            return;
        }
        int64_t cur = start;
        for (;;) {
            const int from = dir;  // direction of the previous border pixel, as seen from cur
            int t = dir;
            int64_t next = cur;
            while (t < 15) {       // counter-clockwise, starting after `from`
                ++t;
                next = cur + step_[t & 7];
                if (im[next] != 0) break;
            }
            dir = t & 7;
            if ((unsigned)(dir - 1) < (unsigned)from)
                im[cur] = -126;    // the right neighbour was examined and is background
            else if (im[cur] == 1)
                im[cur] = 2;
            pts.push_back({x, y});
            x += kDx[dir];
            y += kDy[dir];
            if (next == start && cur == first) break;
            cur = next;
            dir = (dir + 4) & 7;
        }
    }

    int w_, h_;
    int64_t W_;
    int64_t step_[8];
    std::vector<signed char> pad_;
};

constexpr int BorderFollower::kDx[8];
constexpr int BorderFollower::kDy[8];

// static_cast<int>(double) as the node's x86-64 build executes it
// (cvttsd2si): NaN and out-of-range values become INT_MIN.
int trunc_to_int(double v) {
    if (!(v > -2147483649.0 && v < 2147483648.0)) return INT_MIN;
    return static_cast<int>(v);
}

void contours_external(const uint8_t *img, int w, int h, std::vector<Pt> &pts, std::vector<int64_t> &starts) {
    std::vector<Pt> dpts;
    std::vector<int64_t> dstarts;
    BorderFollower(img, w, h).run(dpts, dstarts);
    dstarts.push_back((int64_t)dpts.size());
    const int64_t nc = (int64_t)dstarts.size() - 1;
    pts.clear();
    starts.clear();
    pts.reserve(dpts.size());
    for (int64_t c = nc - 1; c >= 0; --c) {
        starts.push_back((int64_t)pts.size());
        pts.insert(pts.end(), dpts.begin() + dstarts[c], dpts.begin() + dstarts[c + 1]);
    }
    starts.push_back((int64_t)pts.size());
}

}  // namespace

// Frontier pixels (y * width + x) in the node's order: contours in reverse
// discovery order, every traversed pixel (duplicates kept).
void trace_external_pixels(const uint8_t *img, int w, int h, std::vector<int32_t> &pix) {
    std::vector<Pt> pts;
    std::vector<int64_t> starts;
    contours_external(img, w, h, pts, starts);
    pix.clear();
    pix.reserve(pts.size());
    for (const Pt &p : pts) pix.push_back(p.y * w + p.x);
}

// GetNextSubgoal's selection (:508-550) over the frontier F with its
// gathered coordinates and bounds: sort by distance to the goal (stable on
// the frontier position), keep the nearest max(1, F/4), strict-> argmax of
// hi - lo from -1.  Returns the position in F, or -1.
int64_t select_subgoal(size_t nf, const double *fx, const double *fy, const double *flo, const double *fhi,
                       double goal_x, double goal_y) {
    if (nf == 0) return -1;  // "No frontier points found" (:503-506)
    std::vector<double> width(nf);
    std::vector<std::pair<double, size_t>> order(nf);
    for (size_t i = 0; i < nf; ++i) {
        width[i] = fhi[i] - flo[i];                     // Q(idx,1) - Q(idx,0) (:516)
        const double dx = fx[i] - goal_x, dy = fy[i] - goal_y;
        order[i] = {std::sqrt(dx * dx + dy * dy), i};  // rowwise().norm() (:522-523)
    }
    std::sort(order.begin(), order.end());              // distance, then frontier position (:526-530)
    const size_t top = std::max<size_t>(1, nf / 4);     // (:533)
    double best_w = -1.0;
    int64_t best = -1;
    for (size_t t = 0; t < top; ++t) {                  // strict > from -1.0 (:536-547)
        const size_t fi = order[t].second;
        if (width[fi] > best_w) {
            best_w = width[fi];
            best = (int64_t)fi;
        }
    }
    return best;
}

namespace {

// FindSafetyContourIndices (:418-497).
void frontier_indices(const double *Dx, const double *Dy, const uint8_t *safe, int64_t m, int width, int height,
                      std::vector<int32_t> &out) {
    out.clear();
    if (m <= 0 || width <= 0 || height <= 0) return;
    const auto mmx = std::minmax_element(Dx, Dx + m);
    const auto mmy = std::minmax_element(Dy, Dy + m);
    // int-truncated bounds (:431-434)
    const int min_x = trunc_to_int(*mmx.first), max_x = trunc_to_int(*mmx.second);
    const int min_y = trunc_to_int(*mmy.first), max_y = trunc_to_int(*mmy.second);
    const double span_x = (double)(max_x - min_x), span_y = (double)(max_y - min_y);
    const size_t npx = (size_t)width * (size_t)height;
    std::vector<uint8_t> img(npx, 0);
    std::vector<int32_t> owner(npx, -1);
    for (int64_t i = 0; i < m; ++i) {
        // scale by width / height (not width-1): D == max maps past the image and is dropped (:450-453)
        const int x = trunc_to_int((Dx[i] - min_x) / span_x * width);
        const int y = trunc_to_int((Dy[i] - min_y) / span_y * height);
        if (x >= 0 && x < width && y >= 0 && y < height) {
            const size_t k = (size_t)y * width + x;
            img[k] = safe[i] ? 255 : 0;  // later points overwrite earlier ones (:454)
            owner[k] = (int32_t)i;       // coord_to_index[x][y] = i (:473)
        }
    }
    std::vector<Pt> pts;
    std::vector<int64_t> starts;
    contours_external(img.data(), width, height, pts, starts);
    out.reserve(pts.size());
    for (const Pt &p : pts) {
        const int32_t idx = owner[(size_t)p.y * width + p.x];
        if (idx >= 0) out.push_back(idx);  // pixels without a grid point are skipped (:484-490)
    }
}

}  // namespace
}  // namespace sbo

extern "C" {

SBO_API int64_t sbo_find_contours_external(const uint8_t *img, int width, int height, int32_t *pts, int64_t pts_cap,
                                           int64_t *start, int64_t contours_cap) {
    if (!img || width <= 0 || height <= 0) return 0;
    std::vector<sbo::Pt> p;
    std::vector<int64_t> s;
    sbo::contours_external(img, width, height, p, s);
    const int64_t nc = (int64_t)s.size() - 1;
    if (nc > contours_cap || (int64_t)p.size() > pts_cap || !pts || !start) return -1;
    for (size_t k = 0; k < p.size(); ++k) {
        pts[2 * k] = p[k].x;
        pts[2 * k + 1] = p[k].y;
    }
    for (int64_t c = 0; c <= nc; ++c) start[c] = s[(size_t)c];
    return nc;
}

SBO_API sbo_status sbo_find_safety_contour_indices(const double *Dx, const double *Dy, const uint8_t *safe, int64_t m,
                                                   int width_cells, int height_cells, int32_t *out, int64_t out_cap,
                                                   int64_t *count) {
    if (!count) return SBO_E_INVAL;
    *count = 0;
    if (m < 0) return SBO_E_INVAL;
    if (m == 0) return SBO_OK;  // "D_ or S_ is empty" (:419-422)
    if (!Dx || !Dy || !safe) return SBO_E_INVAL;
    std::vector<int32_t> f;
    sbo::frontier_indices(Dx, Dy, safe, m, width_cells, height_cells, f);
    *count = (int64_t)f.size();
    if ((int64_t)f.size() > out_cap || (!out && !f.empty())) return SBO_E_INVAL;
    std::copy(f.begin(), f.end(), out);
    return SBO_OK;
}

SBO_API int64_t sbo_next_subgoal(const double *Dx, const double *Dy, const double *lo, const double *hi,
                                 const uint8_t *safe, int64_t m, int width_cells, int height_cells, double goal_x,
                                 double goal_y) {
    if (m <= 0 || !Dx || !Dy || !lo || !hi || !safe) return -1;
    std::vector<int32_t> F;
    sbo::frontier_indices(Dx, Dy, safe, m, width_cells, height_cells, F);
    const size_t nf = F.size();
    std::vector<double> fx(nf), fy(nf), flo(nf), fhi(nf);
    for (size_t i = 0; i < nf; ++i) {
        fx[i] = Dx[F[i]];
        fy[i] = Dy[F[i]];
        flo[i] = lo[F[i]];
        fhi[i] = hi[F[i]];
    }
    const int64_t b = sbo::select_subgoal(nf, fx.data(), fy.data(), flo.data(), fhi.data(), goal_x, goal_y);
    return b >= 0 ? F[(size_t)b] : -1;
}

}  // extern "C"
