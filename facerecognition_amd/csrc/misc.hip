// Memory-bound helper kernels of the embedding path (gfx950):
//  * preprocess   — get_transform()/get_facenet_transform() ToTensor+Normalize(0.5,0.5)
//                   (inference/extract_embeddings.py:170-185) fused with the HWC→NHWC8 bf16 pack
//  * maxpool      — ResNet-50 stem maxpool 3x3 s2 p1 (models/arcface/arcface_model.py:122),
//                   InceptionResnetV1 MaxPool2d(3, 2) (maxpool_3a, Mixed_6a/7a branches)
//  * avgpool      — adaptive avgpool to 1x1 (arcface_model.py:129-130; IRV1 avgpool_1a)
//  * head finalize— split-K reduction of the folded BN1d·Linear·BN1d head + F.normalize
//                   (arcface_model.py:192-196, extract_embeddings.py:381/434)
//  * segment mean — per-identity mean + renorm (extract_embeddings.py:755-760, :555-592)
#include "kernels.h"

#include <algorithm>
#include "../../include/frhip.h"

namespace fr {
namespace {

// x = (u/255 - 0.5)/0.5 = (2u - 255)/255: store q = 2u - 255 (an integer in [-255, 255], exact
// in bf16 and f16) twice; the stem weights carry 1/255 as a hi/lo pair (engine.cpp make_convw).
template <bool F16>
__global__ __launch_bounds__(256) void preprocess_u8_kernel(const uint8_t* __restrict__ in, int npix,
                                                            bf16_t* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= npix) return;
    const uint8_t* q = in + 3 * (size_t)i;
    float f[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int c = 0; c < 3; ++c) f[c] = f[c + 3] = 2.0f * (float)q[c] - 255.0f;
    *(uint4*)(out + 8 * (size_t)i) = Num<F16>::pack8(f);
}

// Already-normalized f32 NCHW (get_transform() output): q = 255 * x, rounded once.
template <bool F16>
__global__ __launch_bounds__(256) void preprocess_f32_kernel(const float* __restrict__ in, int B, int HW,
                                                             bf16_t* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= B * HW) return;
    const int b = i / HW, p = i - b * HW;
    const float* q = in + (size_t)b * 3 * HW + p;
    const float a = 255.0f * q[0], c = 255.0f * q[HW], d = 255.0f * q[2 * (size_t)HW];
    float f[8] = {a, c, d, a, c, d, 0, 0};
    *(uint4*)(out + 8 * (size_t)i) = Num<F16>::pack8(f);
}

template <bool F16>
__global__ __launch_bounds__(256) void maxpool_kernel(const bf16_t* __restrict__ x, int B, int H, int W, int Cx,
                                                      int x_off, int C, int k, int stride, int pad,
                                                      bf16_t* __restrict__ y, int Cy, int y_off, int Ho, int Wo) {
    const int G = C / 8;
    const size_t total = (size_t)B * Ho * Wo * G;
    for (size_t it = blockIdx.x * 256ull + threadIdx.x; it < total; it += (size_t)gridDim.x * 256) {
        const int g = (int)(it % G);
        const size_t pix = it / G;
        const int ow = (int)(pix % Wo);
        const int oh = (int)((pix / Wo) % Ho);
        const int b = (int)(pix / ((size_t)Wo * Ho));
        float m[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
        for (int r = 0; r < k; ++r) {
            const int ih = oh * stride - pad + r;
            if ((unsigned)ih >= (unsigned)H) continue;
            for (int s = 0; s < k; ++s) {
                const int iw = ow * stride - pad + s;
                if ((unsigned)iw >= (unsigned)W) continue;
                const uint4 v = *(const uint4*)(x + ((size_t)(b * H + ih) * W + iw) * Cx + x_off + g * 8);
                float f[8];
                Num<F16>::unpack8(v, f);
#pragma unroll
                for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], f[e]);
            }
        }
        *(uint4*)(y + pix * Cy + y_off + g * 8) = Num<F16>::pack8(m);
    }
}

// k = 3 (IRV1's and ResNet-50's pools): the nine 16-B loads of a window issued together (clamped addresses,
// out-of-image taps masked to -inf afterwards) instead of one dependent load per loop trip; same values
template <bool F16, bool YB = false>  // YB: f16 input, bf16 output (the end of an f16 plan section)
__global__ __launch_bounds__(256) void maxpool3_kernel(const bf16_t* __restrict__ x, int B, int H, int W, int Cx,
                                                       int x_off, int C, int stride, int pad,
                                                       bf16_t* __restrict__ y, int Cy, int y_off, int Ho, int Wo) {
    const int G = C / 8;
    const size_t total = (size_t)B * Ho * Wo * G;
    for (size_t it = blockIdx.x * 256ull + threadIdx.x; it < total; it += (size_t)gridDim.x * 256) {
        const int g = (int)(it % G);
        const size_t pix = it / G;
        const int ow = (int)(pix % Wo);
        const int oh = (int)((pix / Wo) % Ho);
        const int b = (int)(pix / ((size_t)Wo * Ho));
        uint4 v[9];
        unsigned ok = 0;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int ih = oh * stride - pad + t / 3, iw = ow * stride - pad + t % 3;
            const bool in = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            ok |= in ? 1u << t : 0u;
            const int ch = in ? ih : 0, cw = in ? iw : 0;
            v[t] = *(const uint4*)(x + ((size_t)(b * H + ch) * W + cw) * Cx + x_off + g * 8);
        }
        float m[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            if (!(ok >> t & 1u)) continue;
            float f[8];
            Num<F16>::unpack8(v[t], f);
#pragma unroll
            for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], f[e]);
        }
        *(uint4*)(y + pix * Cy + y_off + g * 8) = YB ? Num<false>::pack8(m) : Num<F16>::pack8(m);
    }
}

template <bool F16>
__global__ __launch_bounds__(256) void avgpool_kernel(const bf16_t* __restrict__ x, int B, int HW, int C,
                                                      bf16_t* __restrict__ y) {
    const int G = C / 8;
    const int it = blockIdx.x * 256 + threadIdx.x;
    if (it >= B * G) return;
    const int b = it / G, g = it - b * G;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const bf16_t* base = x + (size_t)b * HW * C + g * 8;
    for (int p = 0; p < HW; ++p) {
        float f[8];
        Num<F16>::unpack8(*(const uint4*)(base + (size_t)p * C), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += f[e];
    }
    const float inv = 1.0f / (float)HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    *(uint4*)(y + (size_t)b * C + g * 8) = Num<F16>::pack8(acc);
}

__device__ __forceinline__ float block_sum_256(float v, float* red) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

// One block per row: out[b][n] = sum_s partial[s][b][n] + bias[n]; optional L2 normalize.  N % 4 == 0 and
// N <= 1024 (the launcher checks): a thread owns 4 consecutive columns, float4 loads, the split loop
// unrolled so its loads are in flight together.
__global__ __launch_bounds__(256) void head_finalize_kernel(const float* __restrict__ partial, int split, int B,
                                                            int N, int Npad, const float* __restrict__ bias,
                                                            int normalize, float* __restrict__ out) {
    __shared__ float red[4];
    const int b = blockIdx.x, n = 4 * threadIdx.x;
    const bool own = n < N;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (own) {
        if (bias) v = *(const float4*)(bias + n);
        const float* src = partial + (size_t)b * Npad + n;
        const size_t stride = (size_t)B * Npad;
        int s = 0;
        for (; s + 4 <= split; s += 4) {
            float4 q[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) q[u] = *(const float4*)(src + (s + u) * stride);
#pragma unroll
            for (int u = 0; u < 4; ++u) { v.x += q[u].x; v.y += q[u].y; v.z += q[u].z; v.w += q[u].w; }
        }
        for (; s < split; ++s) {
            const float4 q = *(const float4*)(src + s * stride);
            v.x += q.x; v.y += q.y; v.z += q.z; v.w += q.w;
        }
    }
    if (normalize) {
        const float tot = block_sum_256(own ? v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w : 0.f, red);
        const float inv = 1.0f / fmaxf(sqrtf(tot), 1e-12f);
        v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
    }
    if (own) *(float4*)(out + (size_t)b * N + n) = v;
}

// Head GEMV for small batches (bs = 1 is the reference's online path, recognition_engine.py:328-381): the
// 25088 -> 512 head as split-K partials [S][B][Npad] for head_finalize_kernel, like the implicit-GEMM head, but
// with no 128-row MFMA tile of which one row is real.  Grid (Npad / 16, S): each wave owns 4 output rows over
// the block's K chunk, lanes stride K by 8 elements (one 16-B load of each weight row and of each input row
// per step), f32 FMAs, a wave reduction per (row, probe).  The weight matrix (25.7 MB) is read once in total.
template <bool F16, int NB>
__global__ __launch_bounds__(256) void head_gemv_kernel(const bf16_t* __restrict__ x, int B, int K,
                                                        const bf16_t* __restrict__ w, int Kpad, int N, int Npad,
                                                        int kchunk, float* __restrict__ partial) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n0 = blockIdx.x * 16 + wave * 4, s = blockIdx.y;
    const int k0 = s * kchunk, k1 = min(K, k0 + kchunk);
    float acc[4][NB];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[j][b] = 0.f;
    for (int k = k0 + 8 * lane; k < k1; k += 512) {
        float xf[NB][8];
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            const uint4 v = b < B ? *(const uint4*)(x + (size_t)b * K + k) : make_uint4(0u, 0u, 0u, 0u);
            Num<F16>::unpack8(v, xf[b]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float wf[8];
            Num<F16>::unpack8(*(const uint4*)(w + (size_t)(n0 + j) * Kpad + k), wf);
#pragma unroll
            for (int b = 0; b < NB; ++b)
#pragma unroll
                for (int e = 0; e < 8; ++e) acc[j][b] = fmaf(wf[e], xf[b][e], acc[j][b]);
        }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int b = 0; b < NB; ++b) {
            float v = acc[j][b];
#pragma unroll
            for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
            if (lane == 0 && b < B) partial[((size_t)s * B + b) * Npad + n0 + j] = v;
        }
}

__global__ __launch_bounds__(256) void l2norm_rows_kernel(float* __restrict__ x, int D) {
    __shared__ float red[4];
    float* row = x + (size_t)blockIdx.x * D;
    float ss = 0.f;
    for (int n = threadIdx.x; n < D; n += 256) ss += row[n] * row[n];
    const float tot = block_sum_256(ss, red);
    const float inv = 1.0f / fmaxf(sqrtf(tot), 1e-12f);
    for (int n = threadIdx.x; n < D; n += 256) row[n] *= inv;
}

// np.mean over a segment (row order, f32) then / (np.linalg.norm + 1e-8).
__global__ __launch_bounds__(256) void segment_mean_kernel(const float* __restrict__ E, int D,
                                                           const int32_t* __restrict__ seg, float* __restrict__ out) {
    __shared__ float red[4];
    const int s = blockIdx.x;
    const int r0 = seg[s], r1 = seg[s + 1];
    const float cnt = (float)(r1 - r0);
    float ss = 0.f;
    for (int d = threadIdx.x; d < D; d += 256) {
        float acc = 0.f;
        for (int r = r0; r < r1; ++r) acc += E[(size_t)r * D + d];
        const float m = r1 > r0 ? acc / cnt : 0.f;
        out[(size_t)s * D + d] = m;
        ss += m * m;
    }
    const float tot = block_sum_256(ss, red);
    const float inv = 1.0f / (sqrtf(tot) + 1e-8f);
    for (int d = threadIdx.x; d < D; d += 256) out[(size_t)s * D + d] *= inv;
}

// cosine_similarity (recognition_engine.py:41-63): a row with |norm-1| >= 1e-3 is divided
// by its norm so the match kernel's dot product equals dot/(|a||b|); zero rows stay zero.
__global__ __launch_bounds__(256) void gallery_prepare_kernel(float* __restrict__ G, int D) {
    __shared__ float red[4];
    float* row = G + (size_t)blockIdx.x * D;
    float ss = 0.f;
    for (int d = threadIdx.x; d < D; d += 256) ss += row[d] * row[d];
    const float nrm = sqrtf(block_sum_256(ss, red));
    if (nrm == 0.f || fabsf(nrm - 1.0f) < 1e-3f) return;
    const float inv = 1.0f / nrm;
    for (int d = threadIdx.x; d < D; d += 256) row[d] *= inv;
}

// FaceNetModel.projection + F.normalize (facenet_model.py:32-35): out[b] = W x[b] + bias (f32), then
// out[b] / max(||out[b]||, 1e-12) when normalize.  x rows are the already L2-normalized IRV1 outputs.
__global__ __launch_bounds__(256) void proj_l2_kernel(const float* x, int K, const float* W, const float* bias, int N,
                                                      int normalize, float* out) {
    __shared__ float xs[1024];
    __shared__ float red[8];
    const int b = blockIdx.x;
    for (int k = threadIdx.x; k < K; k += 256) xs[k] = x[(size_t)b * K + k];
    __syncthreads();
    float ss = 0.f;
    for (int n = threadIdx.x; n < N; n += 256) {
        const float* w = W + (size_t)n * K;
        float acc = 0.f;
        for (int k = 0; k < K; ++k) acc = fmaf(w[k], xs[k], acc);
        acc += bias ? bias[n] : 0.f;
        out[(size_t)b * N + n] = acc;
        ss += acc * acc;
    }
    if (!normalize) return;
    const float inv = 1.0f / fmaxf(sqrtf(block_sum_256(ss, red)), 1e-12f);
    __syncthreads();
    for (int n = threadIdx.x; n < N; n += 256) out[(size_t)b * N + n] *= inv;
}

// max |x| of a bf16/f16 NHWC tensor into `slots` partial maxima (atomicMax on the non-negative f32 bit
// pattern, vector-memory atomics): the amax an fp8 consumer's activation scale needs when its producer is a
// kernel without an amax epilogue (an LDS-resident stage, engine.cpp forward)
template <bool F16>
__global__ __launch_bounds__(256) void amax_kernel(const bf16_t* __restrict__ x, size_t n8, float* __restrict__ amax,
                                                   int slots) {
    float m = 0.f;
    for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n8; i += (size_t)gridDim.x * 256) {
        float f[8];
        Num<F16>::unpack8(*(const uint4*)(x + 8 * i), f);
#pragma unroll
        for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(f[e]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    if ((threadIdx.x & 63) == 0) atomicMax((unsigned int*)amax + (blockIdx.x % slots), __float_as_uint(m));
}

}  // namespace

hipError_t launch_amax(const bf16_t* x, size_t n, int f16, float* amax, int slots, hipStream_t s) {
    if (n % 8 || slots < 1) return hipErrorInvalidValue;
    const size_t n8 = n / 8;
    int blocks = (int)std::min<size_t>((n8 + 255) / 256, 1024);
    if (blocks < 1) blocks = 1;
    if (f16) hipLaunchKernelGGL(amax_kernel<true>, dim3(blocks), dim3(256), 0, s, x, n8, amax, slots);
    else hipLaunchKernelGGL(amax_kernel<false>, dim3(blocks), dim3(256), 0, s, x, n8, amax, slots);
    return hipGetLastError();
}

hipError_t launch_proj_l2(const float* x, int B, int K, const float* W, const float* bias, int N, int normalize,
                          float* out, hipStream_t s) {
    if (K > 1024) return hipErrorInvalidValue;
    hipLaunchKernelGGL(proj_l2_kernel, dim3(B), dim3(256), 0, s, x, K, W, bias, N, normalize, out);
    return hipGetLastError();
}

hipError_t launch_preprocess(const void* in, int in_fmt, int B, int H, int W, bf16_t* out, int f16, hipStream_t s) {
    const int npix = B * H * W;
    const int blocks = (npix + 255) / 256;
    if (in_fmt == FR_IN_U8_NHWC) {
        if (f16) hipLaunchKernelGGL(preprocess_u8_kernel<true>, dim3(blocks), dim3(256), 0, s, (const uint8_t*)in, npix, out);
        else hipLaunchKernelGGL(preprocess_u8_kernel<false>, dim3(blocks), dim3(256), 0, s, (const uint8_t*)in, npix, out);
    } else {
        if (f16) hipLaunchKernelGGL(preprocess_f32_kernel<true>, dim3(blocks), dim3(256), 0, s, (const float*)in, B, H * W, out);
        else hipLaunchKernelGGL(preprocess_f32_kernel<false>, dim3(blocks), dim3(256), 0, s, (const float*)in, B, H * W, out);
    }
    return hipGetLastError();
}

hipError_t launch_maxpool(const bf16_t* x, int B, int H, int W, int Cx, int x_off, int C, int k, int stride,
                          int pad, bf16_t* y, int Cy, int y_off, int Ho, int Wo, int f16, hipStream_t s, int y_bf16) {
    const size_t total = (size_t)B * Ho * Wo * (C / 8);
    int blocks = (int)((total + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    if (y_bf16) {  // f16 -> bf16: 3x3 only
        if (!f16 || k != 3) return hipErrorInvalidValue;
        hipLaunchKernelGGL((maxpool3_kernel<true, true>), dim3(blocks), dim3(256), 0, s, x, B, H, W, Cx, x_off, C, stride,
                           pad, y, Cy, y_off, Ho, Wo);
        return hipGetLastError();
    }
    if (k == 3) {
        if (f16)
            hipLaunchKernelGGL(maxpool3_kernel<true>, dim3(blocks), dim3(256), 0, s, x, B, H, W, Cx, x_off, C, stride, pad,
                               y, Cy, y_off, Ho, Wo);
        else
            hipLaunchKernelGGL(maxpool3_kernel<false>, dim3(blocks), dim3(256), 0, s, x, B, H, W, Cx, x_off, C, stride, pad,
                               y, Cy, y_off, Ho, Wo);
        return hipGetLastError();
    }
    if (f16)
        hipLaunchKernelGGL(maxpool_kernel<true>, dim3(blocks), dim3(256), 0, s, x, B, H, W, Cx, x_off, C, k, stride,
                           pad, y, Cy, y_off, Ho, Wo);
    else
        hipLaunchKernelGGL(maxpool_kernel<false>, dim3(blocks), dim3(256), 0, s, x, B, H, W, Cx, x_off, C, k, stride,
                           pad, y, Cy, y_off, Ho, Wo);
    return hipGetLastError();
}

hipError_t launch_avgpool(const bf16_t* x, int B, int H, int W, int C, bf16_t* y, int f16, hipStream_t s) {
    const int total = B * (C / 8);
    if (f16)
        hipLaunchKernelGGL(avgpool_kernel<true>, dim3((total + 255) / 256), dim3(256), 0, s, x, B, H * W, C, y);
    else
        hipLaunchKernelGGL(avgpool_kernel<false>, dim3((total + 255) / 256), dim3(256), 0, s, x, B, H * W, C, y);
    return hipGetLastError();
}

hipError_t launch_head_finalize(const float* partial, int split, int B, int N, int Npad, const float* bias,
                                int normalize, float* out, hipStream_t s) {
    if (N % 4 || N > 1024 || Npad % 4) return hipErrorInvalidValue;
    hipLaunchKernelGGL(head_finalize_kernel, dim3(B), dim3(256), 0, s, partial, split, B, N, Npad, bias, normalize,
                       out);
    return hipGetLastError();
}

// S split-K partials of the head for B <= 8 probes (head_gemv_kernel); head_finalize_kernel sums them
bool head_gemv_supported(int B, int K, int Kpad, int Npad) { return B >= 1 && B <= 8 && K % 8 == 0 && Kpad >= K && Npad % 16 == 0; }

hipError_t launch_head_gemv(const bf16_t* x, int B, int K, const bf16_t* w, int Kpad, int N, int Npad, int S, int f16,
                            float* partial, hipStream_t s) {
    if (!head_gemv_supported(B, K, Kpad, Npad) || S < 1) return hipErrorInvalidValue;
    const int kchunk = (K + 8 * S - 1) / (8 * S) * 8;
    void (*k)(const bf16_t*, int, int, const bf16_t*, int, int, int, int, float*) =
        B == 1   ? (f16 ? head_gemv_kernel<true, 1> : head_gemv_kernel<false, 1>)
        : B == 2 ? (f16 ? head_gemv_kernel<true, 2> : head_gemv_kernel<false, 2>)
        : B <= 4 ? (f16 ? head_gemv_kernel<true, 4> : head_gemv_kernel<false, 4>)
                 : (f16 ? head_gemv_kernel<true, 8> : head_gemv_kernel<false, 8>);
    hipLaunchKernelGGL(k, dim3(Npad / 16, S), dim3(256), 0, s, x, B, K, w, Kpad, N, Npad, kchunk, partial);
    return hipGetLastError();
}

hipError_t launch_l2norm_rows(float* x, int B, int D, hipStream_t s) {
    hipLaunchKernelGGL(l2norm_rows_kernel, dim3(B), dim3(256), 0, s, x, D);
    return hipGetLastError();
}

hipError_t launch_segment_mean_normalize(const float* E, int D, const int32_t* seg_start, int n_seg, float* out,
                                         hipStream_t s) {
    hipLaunchKernelGGL(segment_mean_kernel, dim3(n_seg), dim3(256), 0, s, E, D, seg_start, out);
    return hipGetLastError();
}

hipError_t launch_gallery_prepare(float* G, int64_t N, int D, hipStream_t s) {
    // one block per row; chunk the grid to stay within grid.x limits
    const int64_t chunk = 1 << 30;
    for (int64_t r0 = 0; r0 < N; r0 += chunk) {
        const int64_t n = (N - r0) < chunk ? (N - r0) : chunk;
        hipLaunchKernelGGL(gallery_prepare_kernel, dim3((unsigned)n), dim3(256), 0, s, G + r0 * D, D);
    }
    return hipGetLastError();
}

}  // namespace fr
