// Device-side crop preparation, the steps before the embedding path:
//   * fr_resize_u8: the Resize((S, S)) of get_transform / get_facenet_transform
//     (inference/extract_embeddings.py:170-185): PIL Image.resize(..., BILINEAR) on RGB u8, i.e. Pillow's
//     separable two-pass resampler (libImaging/Resample.c): triangle filter with support 1 x the scale
//     factor when downscaling (antialiased), coefficients computed in double and normalised to 22-bit
//     fixed point, horizontal pass first into a u8 intermediate over the rows the vertical pass needs,
//     then the vertical pass; every output = clip8((2^21 + sum(pixel * coef)) >> 22).  The coefficient
//     tables are built on the host with Pillow's double arithmetic (resize_tables below).
//   * fr_warp_affine_u8: the 5-point alignment warp of align_face (extract_embeddings.py:216-242,
//     recognition_engine.py:169-204): cv2.warpAffine(image, M, (112, 112), borderValue=0), INTER_LINEAR,
//     BORDER_CONSTANT, restated from OpenCV's fixed-point path (imgwarp.cpp): M inverted in double,
//     source coordinates on a 1/32-pixel grid (AB_BITS 10, INTER_BITS 5, cvRound = round half to even),
//     bilinear weights (32 - t) * (32 - u) * 32 ... summing to 2^15, out = (sum + 2^14) >> 15; corners
//     outside the image read 0.
// Both are byte work (u8 in, u8 out): HBM-bound one-thread-per-output-pixel kernels, 3 channels each.
#include "kernels.h"

#include <cmath>
#include <mutex>
#include <tuple>
#include <map>
#include <vector>

namespace fr {
namespace {

constexpr int PB = 22;  // Pillow PRECISION_BITS (32 - 8 - 2)

__device__ __forceinline__ uint8_t clip8(int v) {
    v >>= PB;  // arithmetic shift: floor, as Pillow's clip8 lookup
    return (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
}

// horizontal pass: tmp[b][r][x][c] for source rows r0 .. r0 + rows - 1
__global__ __launch_bounds__(256) void resize_h_kernel(const uint8_t* __restrict__ in, int B, int H, int W,
                                                       int r0, int rows, int OW, const int32_t* __restrict__ bounds,
                                                       const int32_t* __restrict__ kk, int ks,
                                                       uint8_t* __restrict__ tmp) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t total = (size_t)B * rows * OW;
    if (i >= total) return;
    const int x = (int)(i % OW);
    const size_t br = i / OW;
    const int r = (int)(br % rows), b = (int)(br / rows);
    const int xmin = bounds[2 * x], xn = bounds[2 * x + 1];
    const int32_t* k = kk + (size_t)x * ks;
    const uint8_t* src = in + (((size_t)b * H + r0 + r) * W + xmin) * 3;
    int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
    for (int t = 0; t < xn; ++t) {
        const int w = k[t];
        s0 += src[3 * t] * w;
        s1 += src[3 * t + 1] * w;
        s2 += src[3 * t + 2] * w;
    }
    uint8_t* d = tmp + i * 3;
    d[0] = clip8(s0);
    d[1] = clip8(s1);
    d[2] = clip8(s2);
}

// vertical pass: out[b][y][x][c] from src [b][rows][OW][3] (rows relative to the first used row)
__global__ __launch_bounds__(256) void resize_v_kernel(const uint8_t* __restrict__ src, int B, int rows, int OW, int OH,
                                                       const int32_t* __restrict__ bounds,
                                                       const int32_t* __restrict__ kk, int ks,
                                                       uint8_t* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t total = (size_t)B * OH * OW;
    if (i >= total) return;
    const int x = (int)(i % OW);
    const size_t by = i / OW;
    const int y = (int)(by % OH), b = (int)(by / OH);
    const int ymin = bounds[2 * y], yn = bounds[2 * y + 1];
    const int32_t* k = kk + (size_t)y * ks;
    const uint8_t* s = src + (((size_t)b * rows + ymin) * OW + x) * 3;
    const size_t rs = (size_t)OW * 3;
    int s0 = 1 << (PB - 1), s1 = s0, s2 = s0;
    for (int t = 0; t < yn; ++t) {
        const int w = k[t];
        s0 += s[t * rs] * w;
        s1 += s[t * rs + 1] * w;
        s2 += s[t * rs + 2] * w;
    }
    uint8_t* d = out + i * 3;
    d[0] = clip8(s0);
    d[1] = clip8(s1);
    d[2] = clip8(s2);
}

// cv2.warpAffine, INTER_LINEAR, BORDER_CONSTANT(0); M: forward 2x3 matrices [B][6] (double)
__global__ __launch_bounds__(256) void warp_affine_kernel(const uint8_t* __restrict__ in, int B, int H, int W,
                                                          const double* __restrict__ Mf, uint8_t* __restrict__ out,
                                                          int OH, int OW) {
#pragma clang fp contract(off)
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    const size_t total = (size_t)B * OH * OW;
    if (i >= total) return;
    const int x = (int)(i % OW);
    const size_t by = i / OW;
    const int y = (int)(by % OH), b = (int)(by / OH);
    const double* m = Mf + (size_t)b * 6;
    // inverse map (imgwarp.cpp: warpAffine without WARP_INVERSE_MAP)
    double M0 = m[0], M1 = m[1], M2 = m[2], M3 = m[3], M4 = m[4], M5 = m[5];
    double D = M0 * M4 - M1 * M3;
    D = D != 0. ? 1. / D : 0.;
    const double A11 = M4 * D, A22 = M0 * D;
    M0 = A11;
    M1 *= -D;
    M3 *= -D;
    M4 = A22;
    const double b1 = -M0 * M2 - M1 * M5;
    const double b2 = -M3 * M2 - M4 * M5;
    M2 = b1;
    M5 = b2;
    constexpr int AB_BITS = 10, AB_SCALE = 1 << AB_BITS, INTER_BITS = 5, TAB = 1 << INTER_BITS;
    constexpr int round_delta = AB_SCALE / TAB / 2;
    const int X0 = __double2int_rn((M1 * y + M2) * AB_SCALE) + round_delta;
    const int Y0 = __double2int_rn((M4 * y + M5) * AB_SCALE) + round_delta;
    const int adelta = __double2int_rn(M0 * x * AB_SCALE);
    const int bdelta = __double2int_rn(M3 * x * AB_SCALE);
    const int X = (X0 + adelta) >> (AB_BITS - INTER_BITS);
    const int Y = (Y0 + bdelta) >> (AB_BITS - INTER_BITS);
    const int sx = X >> INTER_BITS, sy = Y >> INTER_BITS;
    const int tx = X & (TAB - 1), ty = Y & (TAB - 1);
    // initInterTab2D(INTER_LINEAR, fixpt): products of (1 - t/32, t/32) x 2^15, exact integers
    const int w0 = (TAB - ty) * (TAB - tx) * 32, w1 = (TAB - ty) * tx * 32, w2 = ty * (TAB - tx) * 32, w3 = ty * tx * 32;
    uint8_t* d = out + i * 3;
    if (sx >= W || sx + 1 < 0 || sy >= H || sy + 1 < 0) {
        d[0] = d[1] = d[2] = 0;
        return;
    }
    const uint8_t* img = in + (size_t)b * H * W * 3;
    const bool x0ok = sx >= 0 && sx < W, x1ok = sx + 1 >= 0 && sx + 1 < W;
    const bool y0ok = sy >= 0 && sy < H, y1ok = sy + 1 >= 0 && sy + 1 < H;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const int v0 = (x0ok && y0ok) ? img[((size_t)sy * W + sx) * 3 + c] : 0;
        const int v1 = (x1ok && y0ok) ? img[((size_t)sy * W + sx + 1) * 3 + c] : 0;
        const int v2 = (x0ok && y1ok) ? img[((size_t)(sy + 1) * W + sx) * 3 + c] : 0;
        const int v3 = (x1ok && y1ok) ? img[((size_t)(sy + 1) * W + sx + 1) * 3 + c] : 0;
        const int v = (v0 * w0 + v1 * w1 + v2 * w2 + v3 * w3 + (1 << 14)) >> 15;
        d[c] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
    }
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc (Resample.c) for one axis, in double as Pillow
// (box = [0, in_size]); returns ksize and fills bounds [out][2] = (xmin, xn), kk [out][ksize].
int pillow_coeffs(int in_size, int out_size, std::vector<int32_t>& bounds, std::vector<int32_t>& kk) {
    const double in0 = 0.0, in1 = (double)(float)in_size;
    double scale = (in1 - in0) / out_size, filterscale = scale;
    if (filterscale < 1.0) filterscale = 1.0;
    const double support = 1.0 * filterscale;  // BILINEAR filter support 1.0
    const int ksize = (int)std::ceil(support) * 2 + 1;
    bounds.assign((size_t)out_size * 2, 0);
    kk.assign((size_t)out_size * ksize, 0);
    std::vector<double> k(ksize);
    for (int xx = 0; xx < out_size; ++xx) {
        const double center = in0 + (xx + 0.5) * scale;
        double ww = 0.0;
        const double ss = 1.0 / filterscale;
        int xmin = (int)(center - support + 0.5);
        if (xmin < 0) xmin = 0;
        int xmax = (int)(center + support + 0.5);
        if (xmax > in_size) xmax = in_size;
        xmax -= xmin;
        for (int x = 0; x < xmax; ++x) {
            double t = (x + xmin - center + 0.5) * ss;
            if (t < 0.0) t = -t;
            const double w = t < 1.0 ? 1.0 - t : 0.0;
            k[x] = w;
            ww += w;
        }
        for (int x = 0; x < xmax; ++x)
            if (ww != 0.0) k[x] /= ww;
        for (int x = 0; x < ksize; ++x) {
            const double v = x < xmax ? k[x] : 0.0;
            kk[(size_t)xx * ksize + x] = v < 0 ? (int32_t)(-0.5 + v * (1 << PB)) : (int32_t)(0.5 + v * (1 << PB));
        }
        bounds[2 * xx] = xmin;
        bounds[2 * xx + 1] = xmax;
    }
    return ksize;
}

struct ResizeTables {
    int32_t *bh = nullptr, *kh = nullptr, *bv = nullptr, *kv = nullptr;
    int ksh = 0, ksv = 0, row0 = 0, rows = 0;
};

std::mutex g_rt_mu;
std::map<std::tuple<int, int, int, int, int>, ResizeTables> g_rt;  // (device, H, W, OH, OW)

hipError_t upload(int32_t** d, const std::vector<int32_t>& v) {
    hipError_t e = hipMalloc((void**)d, std::max<size_t>(v.size(), 1) * sizeof(int32_t));
    if (e != hipSuccess) return e;
    return hipMemcpy(*d, v.data(), v.size() * sizeof(int32_t), hipMemcpyHostToDevice);
}

// device tables for one (H, W) -> (OH, OW) resize, built once per process and device
hipError_t resize_tables(int H, int W, int OH, int OW, ResizeTables* out) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lk(g_rt_mu);
    auto key = std::make_tuple(dev, H, W, OH, OW);
    auto it = g_rt.find(key);
    if (it != g_rt.end()) {
        *out = it->second;
        return hipSuccess;
    }
    std::vector<int32_t> bh, kh, bv, kv;
    ResizeTables t;
    t.ksh = pillow_coeffs(W, OW, bh, kh);
    t.ksv = pillow_coeffs(H, OH, bv, kv);
    // the horizontal pass covers only the source rows the vertical pass reads (Pillow: ybox_first/last)
    t.row0 = bv[0];
    t.rows = bv[2 * (OH - 1)] + bv[2 * (OH - 1) + 1] - t.row0;
    for (int y = 0; y < OH; ++y) bv[2 * y] -= t.row0;
    if ((e = upload(&t.bh, bh)) != hipSuccess || (e = upload(&t.kh, kh)) != hipSuccess ||
        (e = upload(&t.bv, bv)) != hipSuccess || (e = upload(&t.kv, kv)) != hipSuccess)
        return e;
    g_rt[key] = t;
    *out = t;
    return hipSuccess;
}

}  // namespace

size_t resize_u8_workspace(int B, int H, int W, int OH, int OW) {
    (void)OH;
    // the horizontal pass's u8 intermediate covers at most all H source rows
    return W == OW ? 0 : (size_t)B * H * OW * 3;
}

hipError_t launch_resize_u8(const uint8_t* in, int B, int H, int W, uint8_t* out, int OH, int OW, void* ws,
                            hipStream_t s) {
    ResizeTables t;
    hipError_t e = resize_tables(H, W, OH, OW, &t);
    if (e != hipSuccess) return e;
    const uint8_t* src = in;
    int rows = H;
    if (W != OW) {  // Pillow: need_horizontal (a square S x S output of a square input resizes both axes)
        const size_t n = (size_t)B * t.rows * OW;
        hipLaunchKernelGGL(resize_h_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, B, H, W, t.row0,
                           t.rows, OW, t.bh, t.kh, t.ksh, (uint8_t*)ws);
        src = (const uint8_t*)ws;
        rows = t.rows;
    } else {
        // no horizontal pass: the vertical bounds are relative to row0 of the unshifted input
        src = in + (size_t)t.row0 * W * 3;
        rows = H;
    }
    if (H != OH) {
        const size_t n = (size_t)B * OH * OW;
        hipLaunchKernelGGL(resize_v_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, B, rows, OW, OH,
                           t.bv, t.kv, t.ksv, out);
    } else {
        // no vertical pass: the horizontal result is the output
        const size_t n = (size_t)B * t.rows * OW * 3;
        if (W != OW) return hipMemcpyAsync(out, ws, n, hipMemcpyDeviceToDevice, s);
        return hipMemcpyAsync(out, in, (size_t)B * H * W * 3, hipMemcpyDeviceToDevice, s);
    }
    return hipGetLastError();
}

hipError_t launch_warp_affine_u8(const uint8_t* in, int B, int H, int W, const double* M, uint8_t* out, int OH, int OW,
                                 hipStream_t s) {
    const size_t n = (size_t)B * OH * OW;
    hipLaunchKernelGGL(warp_affine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, in, B, H, W, M, out, OH,
                       OW);
    return hipGetLastError();
}

}  // namespace fr
