// MTCNN P/R/O-net building blocks on the device: the face detector that runs
// before the embedding path (preprocessing/face_detector.py:78-97, 144-210 -> facenet-pytorch MTCNN,
// restated in oracle/mtcnn.py).  The nets are tiny (3x3 / 2x2 convs of 3..128 channels, ~10^6 MAC per
// 12x12 window), so these kernels are f32 CUDA-core work, not MFMA: f32 keeps the face probabilities
// within float rounding of the fp32 reference, so the threshold decisions (0.6 / 0.7 / 0.7) and the
// NMS orders match it.  Layout NHWC f32 throughout.
//   * area_resample_kernel: F.interpolate(mode='area') (= adaptive average pooling) of u8 RGB image
//     regions -- whole images for the PNet pyramid, box crops for RNet (24x24) / ONet (48x48) -- with
//     the (x - 127.5) * 0.0078125 normalisation; window sums of u8 values are exact in f32 and the
//     division is torch's sum / kh / kw, so the result is bit-identical to the CPU reference;
//   * conv_kernel: valid 3x3 / 2x2 / 1x1 conv, stride 1, bias + PReLU; a thread per output pixel and
//     output-channel block, weights through the scalar cache;
//   * maxpool_ceil_kernel: MaxPool2d(k, 2, ceil_mode=True);
//   * dense_kernel: Linear (+ PReLU); weights pre-permuted on the host to the NHWC flatten order;
//   * head_kernel: the classification / regression heads: softmax of the first two outputs, the rest raw.
#include "kernels.h"

namespace fr {
namespace {

__global__ __launch_bounds__(256) void area_resample_kernel(const uint8_t* __restrict__ img, int H, int W,
                                                            const int32_t* __restrict__ reg, int n, int oh, int ow,
                                                            float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)n * oh * ow) return;
    const int k = (int)(i / ((int64_t)oh * ow)), p = (int)(i - (int64_t)k * oh * ow);
    const int oy = p / ow, ox = p - oy * ow;
    const int32_t* r = reg + 5 * k;  // image, y0, x0, h, w
    const int im = r[0], y0 = r[1], x0 = r[2], h = r[3], w = r[4];
    const int ys = oy * h / oh, ye = ((oy + 1) * h + oh - 1) / oh;
    const int xs = ox * w / ow, xe = ((ox + 1) * w + ow - 1) / ow;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int y = ys; y < ye; ++y) {
        const uint8_t* row = img + (((size_t)im * H + y0 + y) * W + x0) * 3;
        for (int x = xs; x < xe; ++x) {
            s0 += (float)row[3 * x];
            s1 += (float)row[3 * x + 1];
            s2 += (float)row[3 * x + 2];
        }
    }
    const float kh = (float)(ye - ys), kw = (float)(xe - xs);
    float* o = out + (size_t)i * 3;
    o[0] = (s0 / kh / kw - 127.5f) * 0.0078125f;
    o[1] = (s1 / kh / kw - 127.5f) * 0.0078125f;
    o[2] = (s2 / kh / kw - 127.5f) * 0.0078125f;
}

// One thread per output pixel and CB output channels (blockIdx.y), accumulators in registers: the weights of
// a (tap, input channel) step are the same for every lane of the workgroup, so they come through the scalar
// cache (s_load, 4 input channels per load when Cin % 4 == 0) and each input value loaded feeds CB FMAs (the
// one-thread-per-output kernel loaded an input and a weight per FMA).  Each output still sums its taps in the
// same (r, s, c) order with fmaf.  Weights [Cout][kh][kw][Cin].
template <int CB, bool V4>
__global__ __launch_bounds__(256) void conv_kernel(const float* __restrict__ x, int B, int H, int W, int Cin,
                                                   const float* __restrict__ wt, const float* __restrict__ bias,
                                                   const float* __restrict__ slope, int Cout, int kh, int kw,
                                                   float* __restrict__ y) {
    const int Ho = H - kh + 1, Wo = W - kw + 1;
    const int64_t pix = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int co0 = blockIdx.y * CB;
    const bool live = pix < (int64_t)B * Ho * Wo;
    const int64_t pc = live ? pix : 0;  // dead lanes compute pixel 0 and store nothing (uniform loops)
    const int ox = (int)(pc % Wo), oy = (int)((pc / Wo) % Ho), b = (int)(pc / ((int64_t)Wo * Ho));
    const int KK = kh * kw * Cin;
    float acc[CB];
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[j] = 0.f;
    for (int r = 0; r < kh; ++r)
        for (int s = 0; s < kw; ++s) {
            const float* xp = x + (((size_t)b * H + oy + r) * W + ox + s) * Cin;
            const float* wp = wt + (size_t)co0 * KK + (r * kw + s) * Cin;
            if (V4) {
                for (int c = 0; c < Cin; c += 4) {
                    const float4 xv = *(const float4*)(xp + c);
#pragma unroll
                    for (int j = 0; j < CB; ++j) {
                        const float4 wv = *(const float4*)(wp + (size_t)j * KK + c);  // wave-uniform: scalar load
                        acc[j] = fmaf(xv.x, wv.x, acc[j]);
                        acc[j] = fmaf(xv.y, wv.y, acc[j]);
                        acc[j] = fmaf(xv.z, wv.z, acc[j]);
                        acc[j] = fmaf(xv.w, wv.w, acc[j]);
                    }
                }
            } else {
                for (int c = 0; c < Cin; ++c) {
                    const float xv = xp[c];
#pragma unroll
                    for (int j = 0; j < CB; ++j) acc[j] = fmaf(xv, wp[(size_t)j * KK + c], acc[j]);
                }
            }
        }
    if (!live) return;
    float* yp = y + (size_t)pix * Cout + co0;
#pragma unroll
    for (int j = 0; j < CB; ++j) {
        float v = acc[j] + (bias ? bias[co0 + j] : 0.f);
        if (slope) v = v >= 0.f ? v : v * slope[co0 + j];
        yp[j] = v;
    }
}

__global__ __launch_bounds__(256) void maxpool_ceil_kernel(const float* __restrict__ x, int B, int H, int W, int C,
                                                           int k, int s, int Ho, int Wo, float* __restrict__ y) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= (int64_t)B * Ho * Wo * C) return;
    const int c = (int)(i % C);
    const int64_t pix = i / C;
    const int ox = (int)(pix % Wo), oy = (int)((pix / Wo) % Ho), b = (int)(pix / ((int64_t)Wo * Ho));
    float m = -INFINITY;
    for (int r = 0; r < k; ++r) {
        const int iy = oy * s + r;
        if (iy >= H) break;
        for (int q = 0; q < k; ++q) {
            const int ix = ox * s + q;
            if (ix >= W) break;
            m = fmaxf(m, x[(((size_t)b * H + iy) * W + ix) * C + c]);
        }
    }
    y[i] = m;
}

// out[b][n] = x[b] . w[n] + bias[n] (PReLU when slope): one wave per (b, n), lanes over K
__global__ __launch_bounds__(256) void dense_kernel(const float* __restrict__ x, int B, int K, const float* __restrict__ wt,
                                                    const float* __restrict__ bias, const float* __restrict__ slope,
                                                    int N, float* __restrict__ y) {
    const int64_t wv = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
    const int lane = threadIdx.x & 63;
    if (wv >= (int64_t)B * N) return;
    const int n = (int)(wv % N), b = (int)(wv / N);
    float acc = 0.f;
    for (int k = lane; k < K; k += 64) acc = fmaf(x[(size_t)b * K + k], wt[(size_t)n * K + k], acc);
    for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (lane == 0) {
        float v = acc + (bias ? bias[n] : 0.f);
        if (slope) v = v >= 0.f ? v : v * slope[n];
        y[(size_t)b * N + n] = v;
    }
}

// heads of M rows of C features: out[m][j] = x[m] . w[j] + b[j]; columns 0, 1 -> softmax (torch's
// exp(v - max) / sum); the rest raw (box regression, landmarks)
__global__ __launch_bounds__(256) void head_kernel(const float* __restrict__ x, int64_t M, int C,
                                                   const float* __restrict__ wt, const float* __restrict__ bias, int NO,
                                                   float* __restrict__ out) {
    const int64_t m = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (m >= M) return;
    const float* xp = x + (size_t)m * C;
    float* o = out + (size_t)m * NO;
    for (int j = 0; j < NO; ++j) {
        float acc = 0.f;
        for (int c = 0; c < C; ++c) acc = fmaf(xp[c], wt[(size_t)j * C + c], acc);
        o[j] = acc + bias[j];
    }
    const float mx = fmaxf(o[0], o[1]);
    const float e0 = expf(o[0] - mx), e1 = expf(o[1] - mx);
    const float sum = e0 + e1;
    o[0] = e0 / sum;
    o[1] = e1 / sum;
}

inline unsigned blocks(int64_t n, int per) { return (unsigned)((n + per - 1) / per); }

}  // namespace

// MaxPool2d(k, s, ceil_mode=True, padding 0) output size (a last window must start inside the input)
int pool_ceil_out(int H, int k, int s) {
    int o = (H - k + s - 1) / s + 1;
    if ((o - 1) * s >= H) --o;
    return o < 1 ? 1 : o;
}

hipError_t launch_area_resample(const uint8_t* img, int H, int W, const int32_t* regions, int n, int oh, int ow,
                                float* out, hipStream_t s) {
    hipLaunchKernelGGL(area_resample_kernel, dim3(blocks((int64_t)n * oh * ow, 256)), dim3(256), 0, s, img, H, W,
                       regions, n, oh, ow, out);
    return hipGetLastError();
}

template <int CB>
static hipError_t conv_cb(const float* x, int B, int H, int W, int Cin, const float* w, const float* bias,
                          const float* slope, int Cout, int kh, int kw, float* y, hipStream_t s) {
    const dim3 grid(blocks((int64_t)B * (H - kh + 1) * (W - kw + 1), 256), Cout / CB);
    auto k = Cin % 4 == 0 ? conv_kernel<CB, true> : conv_kernel<CB, false>;
    hipLaunchKernelGGL(k, grid, dim3(256), 0, s, x, B, H, W, Cin, w, bias, slope, Cout, kh, kw, y);
    return hipGetLastError();
}

// CB output channels per thread: the largest of 16, 8, 5, 4, 2, 1 dividing Cout (PNet conv1's 10 -> 5)
hipError_t launch_mtcnn_conv(const float* x, int B, int H, int W, int Cin, const float* w, const float* bias,
                             const float* slope, int Cout, int kh, int kw, float* y, hipStream_t s) {
    if (Cout % 16 == 0) return conv_cb<16>(x, B, H, W, Cin, w, bias, slope, Cout, kh, kw, y, s);
    if (Cout % 8 == 0) return conv_cb<8>(x, B, H, W, Cin, w, bias, slope, Cout, kh, kw, y, s);
    if (Cout % 5 == 0) return conv_cb<5>(x, B, H, W, Cin, w, bias, slope, Cout, kh, kw, y, s);
    if (Cout % 4 == 0) return conv_cb<4>(x, B, H, W, Cin, w, bias, slope, Cout, kh, kw, y, s);
    if (Cout % 2 == 0) return conv_cb<2>(x, B, H, W, Cin, w, bias, slope, Cout, kh, kw, y, s);
    return conv_cb<1>(x, B, H, W, Cin, w, bias, slope, Cout, kh, kw, y, s);
}

hipError_t launch_mtcnn_maxpool(const float* x, int B, int H, int W, int C, int k, int st, int Ho, int Wo, float* y,
                                hipStream_t s) {
    hipLaunchKernelGGL(maxpool_ceil_kernel, dim3(blocks((int64_t)B * Ho * Wo * C, 256)), dim3(256), 0, s, x, B, H,
                       W, C, k, st, Ho, Wo, y);
    return hipGetLastError();
}

hipError_t launch_mtcnn_dense(const float* x, int B, int K, const float* w, const float* bias, const float* slope,
                              int N, float* y, hipStream_t s) {
    hipLaunchKernelGGL(dense_kernel, dim3(blocks((int64_t)B * N * 64, 256)), dim3(256), 0, s, x, B, K, w, bias, slope,
                       N, y);
    return hipGetLastError();
}

hipError_t launch_mtcnn_head(const float* x, int64_t M, int C, const float* w, const float* bias, int NO, float* out,
                             hipStream_t s) {
    hipLaunchKernelGGL(head_kernel, dim3(blocks(M, 256)), dim3(256), 0, s, x, M, C, w, bias, NO, out);
    return hipGetLastError();
}

}  // namespace fr
