// Greedy non-maximum suppression on the host for the MTCNN box logic (face_detector.py).
// facenet-pytorch's detect_face runs torchvision's batched_nms / its own batched_nms_numpy: greedy, in a given
// score order, a box is dropped when a KEPT box earlier in that order overlaps it above the threshold.  The
// numpy restatement compared every kept box with every remaining one (O(kept x n)); with PNet's 10^5 windows per
// 1080p pyramid level that is seconds to minutes.
//
// Here the kept boxes are bucketed by size class: a box whose extent (plus the 'Min' mode's extra pixel and a
// one-pixel margin) is at most 2^g goes to the uniform grid of class g, whose cells are 2^g wide, as a linked list
// per cell keyed by the cell of its (x1, y1) corner.  A candidate is compared only with the kept boxes of the
// cells whose corners can lie within reach: for class g, corners in [c.x1 - 2^g - 2, c.x2 + 2] (and the same in
// y), every other kept box is disjoint from it and has overlap 0, which never suppresses.  The cross-scale NMS
// of detect_face mixes 12-pixel and frame-sized boxes; one grid sized for the largest box (the round-4 version)
// put all small boxes in a few cells and fell back to O(kept x n) (12 s per 1080p frame).  The overlap arithmetic
// is the numpy code's, in float32 and in the same operation order (this file is built with -ffp-contract=off), so
// the kept set is the same: degenerate boxes (non-positive extent or area, non-finite coordinates: 'Min' mode's
// 0 / 0 = NaN suppresses regardless of distance) are compared with every kept box instead.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <unordered_map>
#include <vector>

#include "frhip.h"

namespace {

struct Box {
    float x1, y1, x2, y2, area;
};

// IoU mode (torchvision.ops.nms): drop when ov > thresh (NaN keeps the candidate); 'Min' mode (nms_numpy): keep
// when ov <= thresh (NaN drops it)
inline bool suppressed(const Box& k, const Box& c, float t, bool min_mode) {
    const float xx1 = k.x1 > c.x1 ? k.x1 : c.x1, yy1 = k.y1 > c.y1 ? k.y1 : c.y1;
    const float xx2 = k.x2 < c.x2 ? k.x2 : c.x2, yy2 = k.y2 < c.y2 ? k.y2 : c.y2;
    float ov;
    if (!min_mode) {
        const float iw = xx2 - xx1, ih = yy2 - yy1;
        const float inter = (iw > 0.f ? iw : 0.f) * (ih > 0.f ? ih : 0.f);
        ov = inter / ((k.area + c.area) - inter);
    } else {
        const float iw = xx2 - xx1 + 1.f, ih = yy2 - yy1 + 1.f;
        const float inter = (iw > 0.f ? iw : 0.f) * (ih > 0.f ? ih : 0.f);
        ov = inter / (k.area < c.area ? k.area : c.area);
    }
    return min_mode ? !(ov <= t) : ov > t;
}

constexpr int NCLASS = 40;
constexpr double MARGIN = 2.0;           // 'Min' mode counts one more pixel per side; one more for rounding
constexpr int64_t DENSE_MAX = 1 << 24;   // cells of a dense class grid; larger extents hash their cells
// ... and only while the grid is not mostly empty: batched_nms offsets image i by i x (frame + 1), so a batch of B
// frames spreads its boxes along a diagonal and a dense grid would grow as B^2; a class grid stays dense
// while it has at most DENSE_FILL cells per box of the class (or DENSE_MIN cells in all)
constexpr int64_t DENSE_MIN = 1 << 16, DENSE_FILL = 16;

// The kept boxes of one grid cell, contiguous (a cell holds a handful: one or two cache lines per lookup).
typedef std::vector<Box> Cell;

template <bool MIN_MODE>
bool cell_hits(const Cell& k, const Box& c, float t) {
    for (const Box& q : k)
        if (suppressed(q, c, t, MIN_MODE)) return true;
    return false;
}

// One size class: cells of the class's largest extent (+ margin) over [ox, ..) x [oy, ..); each used cell owns a
// Cell of kept boxes keyed by the cell of the box's (x1, y1) corner
struct ClassGrid {
    bool used = false, dense = true;
    int64_t count = 0;                               // boxes of the class
    double cs = 1.0, ext = 0.0;
    float amin = INFINITY, amax = 0.f;               // area range of the class
    float wmax = 0.f, hmax = 0.f;                    // largest width / height (IoU mode: x2 - x1, y2 - y1)
    int64_t nx = 0, ny = 0;
    std::vector<int32_t> slot;                       // dense: [ny][nx] -> index into cells, -1 = empty
    std::unordered_map<uint64_t, int32_t> hslot;     // sparse
    std::vector<Cell> cells;
    int64_t cell_of(double v, double o) const { return (int64_t)std::floor((v - o) / cs); }
    static uint64_t key(int64_t cx, int64_t cy) { return ((uint64_t)(uint32_t)cx << 32) | (uint64_t)(uint32_t)cy; }
    const Cell* get(int64_t cx, int64_t cy) const {
        if (dense) {
            if (cx < 0 || cy < 0 || cx >= nx || cy >= ny) return nullptr;
            const int32_t s = slot[(size_t)(cy * nx + cx)];
            return s < 0 ? nullptr : &cells[(size_t)s];
        }
        auto it = hslot.find(key(cx, cy));
        return it == hslot.end() ? nullptr : &cells[(size_t)it->second];
    }
    void push(int64_t cx, int64_t cy, const Box& q) {
        int32_t s;
        if (dense) {
            int32_t& r = slot[(size_t)(cy * nx + cx)];
            if (r < 0) { r = (int32_t)cells.size(); cells.emplace_back(); }
            s = r;
        } else {
            auto it = hslot.find(key(cx, cy));
            if (it == hslot.end()) { s = (int32_t)cells.size(); cells.emplace_back(); hslot[key(cx, cy)] = s; }
            else s = it->second;
        }
        cells[(size_t)s].push_back(q);
    }
};

template <bool MIN_MODE>
int nms_run(const float* boxes, int64_t n, const int64_t* order, float thresh, int64_t* keep, int64_t* n_keep) {
    std::vector<Box> b((size_t)n);
    std::vector<signed char> cls((size_t)n);  // size class, -1 = degenerate
    std::vector<ClassGrid> grid(NCLASS);
    double mx = INFINITY, my = INFINITY, Mx = -INFINITY, My = -INFINITY;
    for (int64_t i = 0; i < n; ++i) {
        Box& q = b[(size_t)i];
        q.x1 = boxes[4 * i]; q.y1 = boxes[4 * i + 1]; q.x2 = boxes[4 * i + 2]; q.y2 = boxes[4 * i + 3];
        const float w = MIN_MODE ? q.x2 - q.x1 + 1.f : q.x2 - q.x1, h = MIN_MODE ? q.y2 - q.y1 + 1.f : q.y2 - q.y1;
        q.area = w * h;
        const bool d = !(q.x2 - q.x1 >= 0.f) || !(q.y2 - q.y1 >= 0.f) || !(q.area > 0.f) || !std::isfinite(q.x1) ||
                       !std::isfinite(q.y1) || !std::isfinite(q.x2) || !std::isfinite(q.y2);
        if (d) { cls[(size_t)i] = -1; continue; }
        const double e = std::fmax((double)q.x2 - q.x1, (double)q.y2 - q.y1) + MARGIN;
        int g = 0;
        while (g < NCLASS - 1 && std::ldexp(1.0, g) < e) ++g;
        cls[(size_t)i] = (signed char)g;
        grid[(size_t)g].used = true;
        grid[(size_t)g].count++;
        grid[(size_t)g].ext = std::fmax(grid[(size_t)g].ext, e);
        grid[(size_t)g].amin = std::fmin(grid[(size_t)g].amin, q.area);
        grid[(size_t)g].amax = std::fmax(grid[(size_t)g].amax, q.area);
        grid[(size_t)g].wmax = std::fmax(grid[(size_t)g].wmax, q.x2 - q.x1);
        grid[(size_t)g].hmax = std::fmax(grid[(size_t)g].hmax, q.y2 - q.y1);
        mx = std::fmin(mx, q.x1); my = std::fmin(my, q.y1);
        Mx = std::fmax(Mx, q.x2); My = std::fmax(My, q.y2);
    }
    const double ox = mx - 2 * MARGIN, oy = my - 2 * MARGIN;  // every corner in reach of a candidate is >= ox
    std::vector<int> used;
    for (int g = 0; g < NCLASS; ++g) {
        ClassGrid& G = grid[(size_t)g];
        if (!G.used) continue;
        used.push_back(g);
        // IoU mode: only corners within (1 - t) x the larger extent can suppress (reach(), below), so the cells
        // shrink with the threshold; 'Min' mode: a box anywhere inside a larger one can, cells of the extent
        G.cs = MIN_MODE ? G.ext : std::fmax(G.ext * (1.0 - 2.0 * (double)thresh / (1.0 + (double)thresh)), 2.0);
        G.nx = (int64_t)std::floor((Mx + 2 * MARGIN - ox) / G.cs) + 1;
        G.ny = (int64_t)std::floor((My + 2 * MARGIN - oy) / G.cs) + 1;
        G.dense = G.nx > 0 && G.ny > 0 && G.nx <= DENSE_MAX / G.ny &&
                  G.nx * G.ny <= std::max(DENSE_MIN, DENSE_FILL * G.count);
        if (G.dense) G.slot.assign((size_t)(G.nx * G.ny), -1);
    }
    std::vector<int64_t> kept_degen, kept_all;
    for (int64_t oi = 0; oi < n; ++oi) {
        const int64_t i = order[oi];
        if (i < 0 || i >= n) return FR_ERR_ARG;
        const Box& c = b[(size_t)i];
        bool drop = false;
        for (int64_t k : kept_degen)
            if (suppressed(b[(size_t)k], c, thresh, MIN_MODE)) { drop = true; break; }
        if (!drop) {
            if (cls[(size_t)i] < 0) {
                for (int64_t k : kept_all)
                    if (suppressed(b[(size_t)k], c, thresh, MIN_MODE)) { drop = true; break; }
            } else {
                // 'Min' mode: a kept box of class g overlapping c (with the margin) has its corner in
                // [c.x1 - ext_g, c.x2 + MARGIN] x [c.y1 - ext_g, c.y2 + MARGIN].  IoU mode: IoU > t needs
                // I > t (A_k + A_c) / (1 + t), and I <= W_ov min(h_k, h_c), so the overlap width W_ov exceeds
                // t (A_k + A_c) / ((1 + t) min(h_k, h_c)); with W_ov <= w_c - (k.x1 - c.x1) (k right of c) or
                // w_k - (c.x1 - k.x1) (left of it), |k.x1 - c.x1| < max(w_c, w_k) - that (the same in y), taken
                // over the class's extremes (largest w / h, smallest area); also min(A_k, A_c) > t max(A_k, A_c).
                // Exact-arithmetic bounds, with MARGIN pixels and a 1 % area slack against float32 rounding
                for (int g : used) {
                    const ClassGrid& G = grid[(size_t)g];
                    int64_t x0, x1, y0, y1;
                    if (MIN_MODE) {
                        x0 = G.cell_of((double)c.x1 - G.ext, ox); x1 = G.cell_of((double)c.x2 + MARGIN, ox);
                        y0 = G.cell_of((double)c.y1 - G.ext, oy); y1 = G.cell_of((double)c.y2 + MARGIN, oy);
                    } else {
                        const double t = thresh > 0.f ? 0.99 * thresh : 0.0;
                        if (t > 0.0 && ((double)G.amax < t * c.area || (double)G.amin * t > (double)c.area)) continue;
                        const double tt = (double)thresh / (1.0 + (double)thresh), asum = (double)G.amin + c.area;
                        const double wc = (double)c.x2 - c.x1, hc = (double)c.y2 - c.y1;
                        const double hmin = std::fmin(hc, (double)G.hmax), wmin = std::fmin(wc, (double)G.wmax);
                        const double rx = std::fmax(wc, (double)G.wmax) - (hmin > 0.0 ? tt * asum / hmin : 0.0) + MARGIN;
                        const double ry = std::fmax(hc, (double)G.hmax) - (wmin > 0.0 ? tt * asum / wmin : 0.0) + MARGIN;
                        if (rx < 0.0 || ry < 0.0) continue;
                        x0 = G.cell_of((double)c.x1 - rx, ox); x1 = G.cell_of((double)c.x1 + rx, ox);
                        y0 = G.cell_of((double)c.y1 - ry, oy); y1 = G.cell_of((double)c.y1 + ry, oy);
                    }
                    for (int64_t cy = y0; cy <= y1 && !drop; ++cy)
                        for (int64_t cx = x0; cx <= x1 && !drop; ++cx)
                            if (const Cell* k = G.get(cx, cy)) drop = cell_hits<MIN_MODE>(*k, c, thresh);
                    if (drop) break;
                }
            }
        }
        if (drop) continue;
        keep[(*n_keep)++] = i;
        kept_all.push_back(i);
        if (cls[(size_t)i] < 0) kept_degen.push_back(i);
        else {
            ClassGrid& G = grid[(size_t)cls[(size_t)i]];
            G.push(G.cell_of(c.x1, ox), G.cell_of(c.y1, oy), c);
        }
    }
    return FR_OK;
}

}  // namespace

extern "C" int fr_nms_host(const float* boxes, int64_t n, const int64_t* order, float thresh, int min_mode,
                           int64_t* keep, int64_t* n_keep) {
    if (!boxes || !order || !keep || !n_keep || n < 0) return FR_ERR_ARG;
    *n_keep = 0;
    if (n == 0) return FR_OK;
    return min_mode ? nms_run<true>(boxes, n, order, thresh, keep, n_keep)
                    : nms_run<false>(boxes, n, order, thresh, keep, n_keep);
}
