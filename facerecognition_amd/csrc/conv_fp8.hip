// FP8 implicit-GEMM convolution for CDNA4 (gfx950): BASELINE config 5 ("ArcFace fp8 weights, CDNA4
// fp8 MFMA").  Same GEMM view, DMA staging and fused epilogue as conv_igemm.hip, but each K-step is
// 128 deep and runs on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, 2x the bf16
// MFMA rate):
//   * weights: OCP e4m3 [Npad][Kpad8] (Kpad8 % 128 == 0), per-output-channel f32 scale sw[n]
//     (host quantization, weights.py -> engine make_convw), applied in the epilogue;
//   * activations stay bf16 in HBM and LDS (the residual stream keeps bf16 precision); each MFMA
//     operand is converted in registers with v_cvt_scalef32_pk_fp8_bf16 (x / 2^e) and the MFMA's
//     e8m0 B-scale multiplies 2^e back, so no product leaves the fp8 range.  e is the per-tensor
//     power of two with amax(x) / 2^e <= 448, from the producer epilogue's atomic amax (dynamic
//     per-tensor scaling; the hardware converter does not saturate: > ~464 would become NaN).
// The epilogue optionally records amax(|y|) of what it stores (atomicMax on the f32 bit pattern) for
// the next conv.  Requirements: Cin % 64 == 0 (every IResNet100 conv but the bf16 stem).
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int KS = 128;                // K per step
constexpr uint32_t OOB = 0x80000000u;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) int i32x8_t;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
typedef __attribute__((ext_vector_type(2))) short i16x2_t;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// power-of-two activation scale exponent: amax / 2^e <= 448
__device__ __forceinline__ int act_exp(const float* amax, int slots) {
    float a = 448.f;
    if (amax) {
        a = 0.f;
        for (int i = 0; i < slots; ++i) a = fmaxf(a, amax[i]);
    }
    if (!(a > 0.f)) return 0;
    int e = (int)ceilf(log2f(a / 448.f));
    return e < -60 ? -60 : (e > 60 ? 60 : e);
}

// 8 bf16 (one uint4) -> 8 e4m3 bytes (two dwords), x / 2^e
__device__ __forceinline__ uint2 cvt8(const uint4& v, float scale) {
    i16x2_t o0 = {0, 0}, o1 = {0, 0};
    o0 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o0, __builtin_bit_cast(bf16x2_t, v.x), scale, false);
    o0 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o0, __builtin_bit_cast(bf16x2_t, v.y), scale, true);
    o1 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o1, __builtin_bit_cast(bf16x2_t, v.z), scale, false);
    o1 = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o1, __builtin_bit_cast(bf16x2_t, v.w), scale, true);
    return make_uint2(__builtin_bit_cast(uint32_t, o0), __builtin_bit_cast(uint32_t, o1));
}

__device__ __forceinline__ void atomic_amax(float* dst, float v) {
    atomicMax((unsigned int*)dst, __float_as_uint(v));  // v >= 0: the f32 bit order is the value order
}

// blocks per CU that the two LDS stages allow (2 x (2*BM + BN) x 128 B)
template <int BM, int BN>
struct Fp8Occ {
    static constexpr int value = 2 * (2 * BM + BN) * 128 <= 80 * 1024 ? 2 : 1;
};

template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(64 * WM * WN, (Fp8Occ<BM, BN>::value)) void conv_fp8_kernel(ConvArgs p, int tiles_n) {
    constexpr int NW = WM * WN, NT = 64 * NW;
    static_assert(NW == 4, "4 waves");
    constexpr int TWM = BM / WM, TWN = BN / WN;
    constexpr int FM = TWM / 16, FN = TWN / 16;
    constexpr int NA = BM / (8 * NW), NB = BN / (8 * NW);
    constexpr int SUB_A = BM * 128;                  // one 64-channel bf16 sub-tile
    constexpr int STAGE = 2 * SUB_A + BN * 128;      // [A0][A1][W]
    constexpr int EPI_LD = BN + 4;
    constexpr int LDS_BYTES = 2 * STAGE > BM * EPI_LD * 4 ? 2 * STAGE : BM * EPI_LD * 4;
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int tm = lid / tiles_n, tn = lid - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int nkt = p.Kpad / KS;

    const int lrow = lane >> 3;
    const int cl = (lane & 7) ^ ((4 * wave + (lane >> 4)) & 7);
    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * p.H * p.W * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const uint32_t w_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.Npad * p.Kpad);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w8, 0, w_bytes, 0x00020000);

    const int HoWo = p.Ho * p.Wo;
    int a_ih[NA], a_iw[NA];
    uint32_t a_base[NA];
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int m = m0 + 8 * (wave + NW * i) + lrow;
        if (m < p.M) {
            const int b = m / HoWo, r = m - b * HoWo;
            const int oh = r / p.Wo, ow = r - oh * p.Wo;
            a_ih[i] = oh * p.sh - p.ph;
            a_iw[i] = ow * p.sw - p.pw;
            a_base[i] = (uint32_t)((((b * p.H + a_ih[i]) * p.W + a_iw[i]) * p.Cx + p.x_off + 8 * cl) * 2);
        } else {
            a_ih[i] = -(1 << 28);
            a_iw[i] = 0;
            a_base[i] = 0;
        }
    }
    uint32_t b_base[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) b_base[j] = (uint32_t)((n0 + 8 * (wave + NW * j) + lrow) * p.Kpad + 16 * cl);

    // one 64-channel activation chunk q (k = 64q .. 64q+63: tap rs = 64q / Cin, channels c0 = 64q % Cin)
    auto issue_a = [&](int q, char* dst) {
        const int k0 = q * 64;
        const int rs = k0 / p.Cin, c0 = k0 - rs * p.Cin;
        const int r = rs / p.Kw, s = rs - r * p.Kw;
        const bool kin = k0 < p.K;
        const int soff = ((r * p.W + s) * p.Cx + c0) * 2;
#pragma unroll
        for (int i = 0; i < NA; ++i) {
            const int ih = a_ih[i] + r, iw = a_iw[i] + s;
            const bool ok = kin && (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
            dma16(xr, dst + (wave + NW * i) * 1024, ok ? a_base[i] + (uint32_t)soff : OOB);
        }
    };
    auto issue = [&](int kt, int buf) {
        char* st = smem + buf * STAGE;
        issue_a(2 * kt, st);
        issue_a(2 * kt + 1, st + SUB_A);
#pragma unroll
        for (int j = 0; j < NB; ++j) dma16(wr, st + 2 * SUB_A + (wave + NW * j) * 1024, b_base[j] + (uint32_t)(kt * KS));
    };

    const int ex = act_exp(p.x_amax, max(p.amax_slots, 1));
    const float xs = __builtin_bit_cast(float, (uint32_t)(127 + ex) << 23);  // 2^ex
    const int scale_b = 127 + ex;

    f32x4_t acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    const int g = lane >> 4;
    auto compute = [&](int buf) {
        const char* st = smem + buf * STAGE;
        i32x8_t wf[FN], af[FM];
#pragma unroll
        for (int i = 0; i < FN; ++i) {  // weights: 32 k-bytes per lane = 16-B chunks 2g, 2g+1
            const int row = wn * TWN + i * 16 + (lane & 15);
            const uint4 lo = *(const uint4*)(st + 2 * SUB_A + row * 128 + swz(row, 2 * g) * 16);
            const uint4 hi = *(const uint4*)(st + 2 * SUB_A + row * 128 + swz(row, 2 * g + 1) * 16);
            wf[i] = (i32x8_t){(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
        }
#pragma unroll
        for (int j = 0; j < FM; ++j) {  // activations: k = 32g .. 32g+31 -> sub-tile g>>1, chunks 4(g&1)..+3
            const int row = wm * TWM + j * 16 + (lane & 15);
            const char* sa = st + (g >> 1) * SUB_A + row * 128;
            uint2 q[4];
#pragma unroll
            for (int c = 0; c < 4; ++c) q[c] = cvt8(*(const uint4*)(sa + swz(row, 4 * (g & 1) + c) * 16), xs);
            af[j] = (i32x8_t){(int)q[0].x, (int)q[0].y, (int)q[1].x, (int)q[1].y, (int)q[2].x, (int)q[2].y, (int)q[3].x,
                              (int)q[3].y};
        }
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wf[i], af[j], acc[i][j], 0, 0, 0, 127, 0,
                                                                             scale_b);
    };

    if (nkt > 0) {
        issue(0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    int buf = 0;
    for (int kt = 0; kt < nkt; ++kt) {
        if (kt + 1 < nkt) issue(kt + 1, buf ^ 1);
        compute(buf);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        buf ^= 1;
    }

    // epilogue: accumulators -> LDS f32 tile -> 8-channel groups (fixed channel group per thread)
    float* sE = (float*)smem;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int ml = wm * TWM + j * 16 + (lane & 15);
            const int nl = wn * TWN + i * 16 + 4 * (lane >> 4);
            *(f32x4_t*)(sE + ml * EPI_LD + nl) = acc[i][j];
        }
    __syncthreads();
    constexpr int G = BN / 8, RS = NT / G, ITER = BM / RS;
    static_assert(NT % G == 0 && BM % RS == 0, "epilogue mapping");
    const int gg = tid % G, ml0 = tid / G;
    const int n = n0 + gg * 8;
    const bool nv = n < p.Cout;
    const int nn = nv ? n : 0;
    float ws8[8], b8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sl8[8], as8[8], ab8[8];
    {
        const float4 w0 = *(const float4*)(p.wscale + nn), w1 = *(const float4*)(p.wscale + nn + 4);
        ws8[0] = w0.x; ws8[1] = w0.y; ws8[2] = w0.z; ws8[3] = w0.w; ws8[4] = w1.x; ws8[5] = w1.y; ws8[6] = w1.z; ws8[7] = w1.w;
    }
    if (p.bias && !p.bias9) {
        const float4 c0 = *(const float4*)(p.bias + nn), c1 = *(const float4*)(p.bias + nn + 4);
        b8[0] = c0.x; b8[1] = c0.y; b8[2] = c0.z; b8[3] = c0.w; b8[4] = c1.x; b8[5] = c1.y; b8[6] = c1.z; b8[7] = c1.w;
    }
    if (p.act == 2) {
        const float4 s0 = *(const float4*)(p.slope + nn), s1 = *(const float4*)(p.slope + nn + 4);
        sl8[0] = s0.x; sl8[1] = s0.y; sl8[2] = s0.z; sl8[3] = s0.w; sl8[4] = s1.x; sl8[5] = s1.y; sl8[6] = s1.z; sl8[7] = s1.w;
    }
    if (p.y2) {
        const float4 a0 = *(const float4*)(p.aff_s + nn), a1 = *(const float4*)(p.aff_s + nn + 4);
        const float4 c0 = *(const float4*)(p.aff_b + nn), c1 = *(const float4*)(p.aff_b + nn + 4);
        as8[0] = a0.x; as8[1] = a0.y; as8[2] = a0.z; as8[3] = a0.w; as8[4] = a1.x; as8[5] = a1.y; as8[6] = a1.z; as8[7] = a1.w;
        ab8[0] = c0.x; ab8[1] = c0.y; ab8[2] = c0.z; ab8[3] = c0.w; ab8[4] = c1.x; ab8[5] = c1.y; ab8[6] = c1.z; ab8[7] = c1.w;
    }
    float amax = 0.f;
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int ml = ml0 + it * RS, m = m0 + ml;
        if (m >= p.M || !nv) continue;
        const float4 v0 = *(const float4*)(sE + ml * EPI_LD + gg * 8);
        const float4 v1 = *(const float4*)(sE + ml * EPI_LD + gg * 8 + 4);
        float v[8] = {v0.x * ws8[0] + b8[0], v0.y * ws8[1] + b8[1], v0.z * ws8[2] + b8[2], v0.w * ws8[3] + b8[3],
                      v1.x * ws8[4] + b8[4], v1.y * ws8[5] + b8[5], v1.z * ws8[6] + b8[6], v1.w * ws8[7] + b8[7]};
        if (p.bias9) {
            const int r = m % HoWo;
            const float* bb = p.bias9 + (size_t)border_class(r / p.Wo, r % p.Wo, p.Ho, p.Wo) * p.Npad + nn;
            const float4 c0 = *(const float4*)bb, c1 = *(const float4*)(bb + 4);
            v[0] += c0.x; v[1] += c0.y; v[2] += c0.z; v[3] += c0.w; v[4] += c1.x; v[5] += c1.y; v[6] += c1.z; v[7] += c1.w;
        }
        if (p.res) {
            float f[8];
            unpack8_bf16(*(const uint4*)(p.res + (size_t)m * p.Cres + p.res_off + n), f);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += f[e];
        }
        if (p.act == 1) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        } else if (p.act == 2) {
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * sl8[e];
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
        *(uint4*)(p.y + (size_t)m * p.Cy + p.y_off + n) = pack8_bf16(v);
        if (p.y2) {
            float u[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) u[e] = v[e] * as8[e] + ab8[e];
            *(uint4*)(p.y2 + (size_t)m * p.Cy2 + p.y2_off + n) = pack8_bf16(u);
        }
    }
    if (p.y_amax) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
        if (lane == 0) atomic_amax(p.y_amax + blockIdx.x % max(p.amax_slots, 1), amax);
    }
}

template <int BM, int BN, int WM, int WN>
hipError_t launch_fp8_variant(const ConvArgs& a, hipStream_t s) {
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.Cout + BN - 1) / BN;
    dim3 grid(tiles_m * tiles_n), block(64 * WM * WN);
    auto k = conv_fp8_kernel<BM, BN, WM, WN>;
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, block, 0, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a, tiles_n);
    else
        hipLaunchKernelGGL(k, grid, block, 0, s, a, tiles_n);
    return hipGetLastError();
}

}  // namespace

// Tile choice: the bf16 planner's shape classes (N <= 64 -> 128x64, else 64x128 or 128x128 by size).
int conv_fp8_tile(int M, int Cout) {
    if (Cout <= 64) return TILE_128x64;
    const long t128 = (long)((M + 127) / 128) * ((Cout + 127) / 128);
    return t128 >= 512 ? TILE_128x128 : TILE_64x128;
}

hipError_t launch_conv_fp8(const ConvArgs& a, hipStream_t s) {
    if (a.Cin % 64 != 0 || a.Kpad % KS != 0 || !a.w8 || !a.wscale || a.x2) return hipErrorInvalidValue;
    switch (a.tile) {
        // 4 x 1 waves: each wave converts only its own activation fragments (2 x 2 converted every
        // fragment twice; the bf16 -> e4m3 conversion costs as much issue time as the fp8 MFMAs)
        case TILE_128x64: return launch_fp8_variant<128, 64, 4, 1>(a, s);
        case TILE_64x128: return launch_fp8_variant<64, 128, 4, 1>(a, s);
        default: return launch_fp8_variant<128, 128, 4, 1>(a, s);
    }
}

}  // namespace fr
