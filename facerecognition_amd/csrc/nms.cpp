// Greedy non-maximum suppression on the host for the MTCNN box logic (face_detector.py).
// facenet-pytorch's detect_face runs torchvision's batched_nms / its own batched_nms_numpy: greedy, in a given
// score order, a box is dropped when a KEPT box earlier in that order overlaps it above the threshold.  The
// numpy restatement compared every kept box with every remaining one (O(kept x n)); with PNet's 10^5 windows per
// 1080p pyramid level that is seconds to minutes.  Here the kept boxes are bucketed in a uniform grid of cells
// no smaller than the largest box, so a candidate is compared only with the kept boxes of the 3 x 3 cells around
// its corner -- the only ones whose overlap can be non-zero.  The overlap arithmetic is the numpy code's, in
// float32 and in the same operation order (this file is built with -ffp-contract=off), so the kept set is the
// same: degenerate boxes (non-positive extent or area, where 'Min' mode's 0 / 0 = NaN suppresses regardless of
// distance) are compared with every kept box instead.
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

}  // namespace

extern "C" int fr_nms_host(const float* boxes, int64_t n, const int64_t* order, float thresh, int min_mode,
                           int64_t* keep, int64_t* n_keep) {
    if (!boxes || !order || !keep || !n_keep || n < 0) return FR_ERR_ARG;
    *n_keep = 0;
    if (n == 0) return FR_OK;
    std::vector<Box> b((size_t)n);
    std::vector<char> degen((size_t)n);
    float cell = 0.f, mx = INFINITY, my = INFINITY;
    for (int64_t i = 0; i < n; ++i) {
        Box& q = b[(size_t)i];
        q.x1 = boxes[4 * i]; q.y1 = boxes[4 * i + 1]; q.x2 = boxes[4 * i + 2]; q.y2 = boxes[4 * i + 3];
        const float w = min_mode ? q.x2 - q.x1 + 1.f : q.x2 - q.x1, h = min_mode ? q.y2 - q.y1 + 1.f : q.y2 - q.y1;
        q.area = w * h;
        const bool d = !(q.x2 - q.x1 >= 0.f) || !(q.y2 - q.y1 >= 0.f) || !(q.area > 0.f) || !std::isfinite(q.x1) ||
                       !std::isfinite(q.y1) || !std::isfinite(q.x2) || !std::isfinite(q.y2);
        degen[(size_t)i] = d;
        if (!d) {
            cell = std::fmax(cell, std::fmax(q.x2 - q.x1, q.y2 - q.y1));
            mx = std::fmin(mx, q.x1);
            my = std::fmin(my, q.y1);
        }
    }
    const double C = (double)cell + 2.0;  // min mode counts one pixel more per side
    auto key = [&](int64_t cx, int64_t cy) { return (cx << 32) ^ (cy & 0xffffffffLL); };
    std::unordered_map<int64_t, std::vector<int64_t>> grid;
    std::vector<int64_t> kept_degen, kept_all;
    for (int64_t oi = 0; oi < n; ++oi) {
        const int64_t i = order[oi];
        if (i < 0 || i >= n) return FR_ERR_ARG;
        const Box& c = b[(size_t)i];
        bool drop = false;
        for (int64_t k : kept_degen)
            if (suppressed(b[(size_t)k], c, thresh, min_mode)) { drop = true; break; }
        if (!drop) {
            if (degen[(size_t)i]) {
                for (int64_t k : kept_all)
                    if (suppressed(b[(size_t)k], c, thresh, min_mode)) { drop = true; break; }
            } else {
                const int64_t cx = (int64_t)std::floor(((double)c.x1 - mx) / C), cy = (int64_t)std::floor(((double)c.y1 - my) / C);
                for (int64_t dx = -1; dx <= 1 && !drop; ++dx)
                    for (int64_t dy = -1; dy <= 1 && !drop; ++dy) {
                        auto it = grid.find(key(cx + dx, cy + dy));
                        if (it == grid.end()) continue;
                        for (int64_t k : it->second)
                            if (suppressed(b[(size_t)k], c, thresh, min_mode)) { drop = true; break; }
                    }
            }
        }
        if (drop) continue;
        keep[(*n_keep)++] = i;
        kept_all.push_back(i);
        if (degen[(size_t)i]) kept_degen.push_back(i);
        else {
            const int64_t cx = (int64_t)std::floor(((double)c.x1 - mx) / C), cy = (int64_t)std::floor(((double)c.y1 - my) / C);
            grid[key(cx, cy)].push_back(i);
        }
    }
    return FR_OK;
}
