// FP8 LDS-resident stage (BASELINE config 5: "ArcFace fp8 weights (CDNA4 fp8 MFMA)"): the stride-1
// IBasicBlocks of IResNet100 layer3 that the fp8 plan puts in e4m3 (tools/fp8_plan.py: the least
// sensitive tail, layer3.16 .. layer3.29), one workgroup per image as conv_stage.hip, on
// v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 x e4m3, twice the bf16 rate).
//   * LDS holds the residual stream x in bf16 (X: [32 planes of 8 channels][196 pixels][16 B], 98 KiB)
//     and the current conv's input in e4m3 (Q: [16 planes of 16 channels][14 rows x 16 positions][16 B],
//     56 KiB, columns 0 / 15 the zero halo, rows -1 / 14 read as the zero slot at position 0 as in the
//     bf16 stage): the identity never passes through fp8.
//   * activations: one power-of-two scale 2^e per image and conv input (the smallest with amax / 2^e <=
//     448, e4m3's largest normal), from a workgroup max-reduction in the producing epilogue; weights:
//     e4m3 with a per-output-channel f32 scale (weights.quantize_fp8).  The MFMA's own e8m0 scales stay
//     1; the epilogue applies sw[n] 2^e and the accumulator seeds (bias, or x + bias) are divided by it.
//   * K-step = one tap x 128 input channels (18 per conv; 36 of the bf16 stage's 32-channel steps would be
//     72): 28 MFMAs per wave per step (8 waves = 2 pixel halves x 4 channel groups of 64, as the bf16
//     stage), weights from L2 into a 2-slot register ring one step ahead (32 KiB per step; a step is
//     ~2x a bf16 step's MFMA time), patch fragments through a 3-deep register ring two fragments ahead.
// Numerics = the fake-quant model of tools/fp8_plan.py / tests/test_gpu_fp8.py: conv(q(x), q(w)) in f32;
// a block output is rounded to bf16 first (the residual stream), and the next conv1 quantizes that value,
// as the per-conv path (conv_fp8.hip reading the bf16 tensor) does.
#include "kernels.h"

#include <hip/hip_ext.h>

#include <type_traits>

namespace fr {
namespace {

constexpr int SW = 14, SWP = 16, SC = 256, SPIX = SW * SW;
constexpr int QPOS = SW * SWP;                  // 224 stored positions per Q plane
constexpr int QPLANE_B = QPOS * 16;             // 3584
constexpr int Q_B = (SC / 16) * QPLANE_B;       // 57344
constexpr int XPLANE_B = SPIX * 16;             // 3136
constexpr int X_B = (SC / 8) * XPLANE_B;        // 100352
constexpr int RED = Q_B + X_B;                  // 8 wave maxima
constexpr int LDS8 = RED + 64;                  // 157760
constexpr int KST = 2 * 9;                      // K-steps per conv: 2 halves of 128 channels x 9 taps
constexpr int WSTEP_B = 4 * SC * 32;            // 32768: [4 groups][256 rows][32 B]
constexpr int NW = 8, FN = 4, FM = 7, NPW = 64;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((ext_vector_type(8))) int i32x8_t;

__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// smallest e with amax / 2^e <= 448 (0 for an all-zero input), clamped to the e8m0 range we use
__device__ __forceinline__ int act_exp(float a) {
    if (!(a > 0.f)) return 0;
    const int e = (int)ceilf(log2f(a / 448.f));
    return e < -100 ? -100 : (e > 100 ? 100 : e);
}
__device__ __forceinline__ float pow2(int e) { return ldexpf(1.f, e); }

// 4 f32 -> 4 e4m3 bytes (one dword), v / 2^e (v_cvt_scalef32_pk_fp8_f32 divides by its scale operand)
__device__ __forceinline__ uint32_t cvt4(float a, float b, float c, float d, float s) {
    typedef short i16x2 __attribute__((ext_vector_type(2)));
    i16x2 o = {0, 0};
    o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, a, b, s, false);
    o = __builtin_amdgcn_cvt_scalef32_pk_fp8_f32(o, c, d, s, true);
    return __builtin_bit_cast(uint32_t, o);
}

__device__ __forceinline__ float wave_max(float v) {
    for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
}

// block max of every wave's `v` (after a barrier every lane holds it); the RED slots are reused per call
__device__ __forceinline__ float block_max(char* smem, float v, int wave, int lane) {
    v = wave_max(v);
    if (lane == 0) ((float*)(smem + RED))[wave] = v;
    __syncthreads();
    const float4 a = *(const float4*)(smem + RED), b = *(const float4*)(smem + RED + 16);
    const float m = fmaxf(fmaxf(fmaxf(a.x, a.y), fmaxf(a.z, a.w)), fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w)));
    return m;
}

__global__ __launch_bounds__(64 * NW, 1) void stage8_kernel(StageArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [Q][X][RED]
    char* const Q = smem;
    char* const X = smem + Q_B;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const int b = blockIdx.x;
    const int nconv = 2 * p.nblk;
    const int total = nconv * KST;
    const uint8_t* w8 = (const uint8_t*)p.w;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)w8, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)total * WSTEP_B), 0x00020000);
    const size_t img = (size_t)b * SPIX * SC;

    // ---- X <- the stage input (bf16 NHWC): 6272 16-B slots, plane-major; Q <- zeros (the halo)
    {
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)p.x, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * SPIX * SC * 2), 0x00020000);
        for (int u = 0; u < (X_B / 1024 + NW - 1) / NW; ++u) {
            const int piece = wave + NW * u;
            if (piece < X_B / 1024) {
                const int q = piece * 64 + lane, plane = q / SPIX, pix = q - plane * SPIX;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(X + piece * 1024), 16,
                                                         (uint32_t)(((img + (size_t)pix * SC) + plane * 8) * 2), 0, 0, 0);
            }
        }
        for (int c = opaque_tid(); c < Q_B / 16; c += 64 * NW) *(uint4*)(Q + c * 16) = make_uint4(0, 0, 0, 0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // quantize X into Q with the input's scale (8 channels of one pixel per slot)
    auto quantize_x = [&](float s) {
        for (int c = opaque_tid(); c < X_B / 16; c += 64 * NW) {
            const int plane = c / SPIX, pix = c - plane * SPIX, r = pix / SW, col = pix - r * SW;
            float f[8];
            unpack8_bf16(*(const uint4*)(X + c * 16), f);
            const uint2 q = make_uint2(cvt4(f[0], f[1], f[2], f[3], s), cvt4(f[4], f[5], f[6], f[7], s));
            *(uint2*)(Q + (plane >> 1) * QPLANE_B + (r * SWP + col + 1) * 16 + (plane & 1) * 8) = q;
        }
    };
    int e_in;
    {
        float m = 0.f;
        for (int c = opaque_tid(); c < X_B / 16; c += 64 * NW) {
            float f[8];
            unpack8_bf16(*(const uint4*)(X + c * 16), f);
#pragma unroll
            for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(f[e]));
        }
        e_in = act_exp(block_max(smem, m, wave, lane));
        quantize_x(pow2(e_in));
        __syncthreads();
    }

    // ---- operands.  A (weights): lane row n = 64 wn + 16 i + (lane & 15), k-group g = lane >> 4: 32 B at
    // (g * 256 + n) * 32 of the step image.  B (Q): position 16 (7 wm + j) + (lane & 15) of row r, planes
    // 8 h + 2 g, + 1 (channels 128 h + 32 g .. + 31)
    const uint32_t wvo = (uint32_t)(((lane >> 4) * SC + wn * NPW + (lane & 15)) * 32);
    const int bbase = 2 * (lane >> 4) * QPLANE_B + ((wm * 7) * SWP + (lane & 15)) * 16;
    const int zoff = 2 * (lane >> 4) * QPLANE_B;  // position 0 (a zero halo slot) of the lane's planes
    f32x4_t acc[FN][FM];
    i32x8_t wq[2][FN];
    auto wload = [&](i32x8_t (&w)[FN], int g) {
        const uint32_t so = (uint32_t)(g < total ? g : total - 1) * WSTEP_B;
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const uint4 lo = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, wvo + i * 512, so, 0));
            const uint4 hi = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wr, wvo + i * 512 + 16, so, 0));
            w[i] = (i32x8_t){(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
        }
    };
    // B fragment j of K-step (h, tap); rows -1 / 14 (wave-uniform: j = 0 of wm 0 at dh = 0, j = 6 of wm 1 at
    // dh = 2) read the zero slot
    auto bread = [&](int h, int tap, int j) {
        const int dh = tap / 3, dw = tap % 3;
        const char* a = Q + 8 * h * QPLANE_B + bbase + (j * SWP + (dh - 1) * SWP + dw) * 16;
        if ((j == 0 && dh == 0 && wm == 0) || (j == 6 && dh == 2 && wm == 1)) a = Q + 8 * h * QPLANE_B + zoff;
        const uint4 lo = *(const uint4*)a, hi = *(const uint4*)(a + QPLANE_B);
        return (i32x8_t){(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
    };

    // per-channel epilogue constants of conv cv: 4 channels n .. n + 3 of fragment i
    auto chan = [&](int i, int ln) { return wn * NPW + 16 * i + 4 * (ln >> 4); };
    auto cls_row = [&](int j, int ln) {  // border class of the lane's pixel in fragment j (row 7 wm + j)
        const int r = wm * 7 + j, cc = ln & 15;
        return (r == 0 ? 0 : (r == SW - 1 ? 6 : 3)) + (cc == 0 ? 0 : (cc == SW - 1 ? 2 : 1));
    };
    // conv1's seed: bias[class] / (sw[n] 2^e)
    auto seed_bias = [&](int cv, float s2e) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const int n = chan(i, ln);
            const float4 sw = *(const float4*)(p.wscale + (size_t)cv * SC + n);
            const float4 inv = make_float4(1.f / (sw.x * s2e), 1.f / (sw.y * s2e), 1.f / (sw.z * s2e), 1.f / (sw.w * s2e));
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const float4 bb = *(const float4*)(p.ep + ((size_t)cv * 9 + cls_row(j, ln)) * SC + n);
                acc[i][j] = (f32x4_t){bb.x * inv.x, bb.y * inv.y, bb.z * inv.z, bb.w * inv.w};
            }
        }
    };
    seed_bias(0, pow2(e_in));

    auto run_conv = [&](int cv, auto second_tag) {
        constexpr bool second = decltype(second_tag)::value;
        const int g0 = cv * KST;
        wload(wq[0], g0);
        i32x8_t bq[3];
        bq[0] = bread(0, 0, 0);
        bq[1] = bread(0, 0, 1);
#pragma unroll 1
        for (int s2 = 0; s2 < KST; s2 += 2) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int s = s2 + u, h = s / 9, tap = s % 9;
                const int sn = s + 1, hn = sn / 9, tapn = sn % 9;  // next step (sn == KST: unused reads)
                asm volatile("" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                wload(wq[u ^ 1], g0 + sn);
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    // fragment f = 7 s + j lives in bq[f % 3]; prefetch f + 2
                    const int f = 7 * u + j;  // 14 fragments per 2 steps; 14 % 3 != 0, so index by f mod 3
                    const int jn = j + 2;
                    const i32x8_t nb = jn < FM ? bread(h, tap, jn) : bread(sn < KST ? hn : 0, sn < KST ? tapn : 0, jn - FM);
                    const i32x8_t cur = bq[f % 3];
#pragma unroll
                    for (int i = 0; i < FN; ++i)
                        acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(wq[u][i], cur, acc[i][j], 0, 0, 0,
                                                                                     127, 0, 127);
                    bq[(f + 2) % 3] = nb;
                }
            }
            // the 3-slot fragment ring advanced by 14 (== 2 mod 3) per iteration: rotate it back
            const i32x8_t t0 = bq[0], t1 = bq[1], t2 = bq[2];
            bq[0] = t2;
            bq[1] = t0;
            bq[2] = t1;
        }
        // ---- epilogue.  v = acc * sw[n] 2^e_in (the seed was pre-divided, so v = bias + conv, or x + bias + conv)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave is past its Q reads
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const float s_in = pow2(e_in);
        float m = 0.f;
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const int n = chan(i, ln);
            const float4 sw = *(const float4*)(p.wscale + (size_t)cv * SC + n);
            const float4 sc = make_float4(sw.x * s_in, sw.y * s_in, sw.z * s_in, sw.w * s_in);
            float4 s1 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!second) {
                const float4 sl = *(const float4*)(p.slope + (size_t)cv * SC + n);
                s1 = make_float4(sl.x - 1.f, sl.y - 1.f, sl.z - 1.f, sl.w - 1.f);
            }
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                float v0 = acc[i][j][0] * sc.x, v1 = acc[i][j][1] * sc.y, v2 = acc[i][j][2] * sc.z, v3 = acc[i][j][3] * sc.w;
                if (!second) {
                    v0 = fmaf(s1.x, min0_raw(v0), v0);
                    v1 = fmaf(s1.y, min0_raw(v1), v1);
                    v2 = fmaf(s1.z, min0_raw(v2), v2);
                    v3 = fmaf(s1.w, min0_raw(v3), v3);
                } else {  // the block output is the bf16 residual; the next conv quantizes that same value
                    const uint32_t a01 = pack2_bf16(v0, v1), a23 = pack2_bf16(v2, v3);
                    v0 = __uint_as_float(a01 << 16);
                    v1 = __uint_as_float(a01 & 0xffff0000u);
                    v2 = __uint_as_float(a23 << 16);
                    v3 = __uint_as_float(a23 & 0xffff0000u);
                }
                acc[i][j] = (f32x4_t){v0, v1, v2, v3};
                if ((ln & 15) < SW) m = fmaxf(m, fmaxf(fmaxf(fabsf(v0), fabsf(v1)), fmaxf(fabsf(v2), fabsf(v3))));
            }
        }
        const int e_out = act_exp(block_max(smem, m, wave, ln));
        const float s_out = pow2(e_out);
        const int cc = ln & 15;
        const bool real = cc < SW;
        // conv1: t -> Q (e4m3 / 2^e_out); conv2's seed = (x + b2[class]) / (sw2[n] 2^e_out), x from X
        // conv2: x' -> X (bf16) and Q (e4m3 / 2^e_out); the next conv1's seed = b1'[class] / (sw1'[n] 2^e_out)
        const int cn = cv + 1 < nconv ? cv + 1 : cv;
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const int n = chan(i, ln);
            const float4 swn = *(const float4*)(p.wscale + (size_t)cn * SC + n);
            const float4 inv = make_float4(1.f / (swn.x * s_out), 1.f / (swn.y * s_out), 1.f / (swn.z * s_out),
                                           1.f / (swn.w * s_out));
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int r = wm * 7 + j, pix = r * SW + cc;
                const f32x4_t v = acc[i][j];
                // Q: lanes of columns 14 / 15 write zeros into the halo slots they cover
                const uint32_t q = real ? cvt4(v[0], v[1], v[2], v[3], s_out) : 0u;
                if (r < SW - 1 || cc < 15)  // row 13's column 15 would be past the plane (the next row's halo)
                    *(uint32_t*)(Q + (n >> 4) * QPLANE_B + (r * SWP + cc + 1) * 16 + (n & 15)) = q;
                char* const xs = X + (n >> 3) * XPLANE_B + (real ? pix : 0) * 16 + (n & 7) * 2;
                const float4 bb = *(const float4*)(p.ep + ((size_t)cn * 9 + cls_row(j, ln)) * SC + n);
                if (!second) {
                    float f[8];
                    unpack8_bf16(make_uint4(((const uint2*)xs)->x, ((const uint2*)xs)->y, 0u, 0u), f);
                    acc[i][j] = (f32x4_t){(f[0] + bb.x) * inv.x, (f[1] + bb.y) * inv.y, (f[2] + bb.z) * inv.z,
                                          (f[3] + bb.w) * inv.w};
                } else {
                    if (real) *(uint2*)xs = make_uint2(pack2_bf16(v[0], v[1]), pack2_bf16(v[2], v[3]));
                    acc[i][j] = (f32x4_t){bb.x * inv.x, bb.y * inv.y, bb.z * inv.z, bb.w * inv.w};
                }
            }
        }
        e_in = e_out;
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // Q / X complete
        bf16_t* const yo = second ? (cv == nconv - 1 ? p.y : (p.dbg_x ? p.dbg_x[cv >> 1] : nullptr)) : nullptr;
        if (yo) {  // the block output, NHWC, from X (the stage output once; with FR_OPT_KEEP_INTERMEDIATES every block)
            for (int c = opaque_tid(); c < X_B / 16; c += 64 * NW) {
                const int plane = c / SPIX, pix = c - plane * SPIX;
                *(uint4*)(yo + img + (size_t)pix * SC + plane * 8) = *(const uint4*)(X + c * 16);
            }
            __builtin_amdgcn_s_waitcnt(0);  // drained here, not by a compiler vmcnt(0) at every K-loop head
        }
    };
#pragma unroll 1
    for (int blk = 0; blk < p.nblk; ++blk) {
        run_conv(2 * blk, std::false_type{});
        run_conv(2 * blk + 1, std::true_type{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

size_t stage8_weight_bytes(int nconv) { return (size_t)nconv * KST * WSTEP_B; }

// One conv's e4m3 rows [C][Kpad8] (K order (kh, kw, c)) -> the fp8 stage's 18 K-step images:
// step s = h * 9 + tap: [4 groups g][256 rows n][32 B] = channels 128 h + 32 g .. + 31 at tap.
void stage8_pack_weights(const uint8_t* rows, int Kpad8, uint8_t* out) {
    for (int h = 0; h < 2; ++h)
        for (int tap = 0; tap < 9; ++tap) {
            uint8_t* s = out + (size_t)(h * 9 + tap) * WSTEP_B;
            for (int g = 0; g < 4; ++g)
                for (int n = 0; n < SC; ++n)
                    for (int e = 0; e < 32; ++e)
                        s[(g * SC + n) * 32 + e] = rows[(size_t)n * Kpad8 + tap * SC + 128 * h + 32 * g + e];
        }
}

hipError_t launch_stage8(const StageArgs& a, hipStream_t s) {
    if (a.B <= 0 || !a.w || !a.wscale || !a.ep || !a.slope || a.f16) return hipErrorInvalidValue;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)stage8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS8);
        attr = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(stage8_kernel, dim3(a.B), dim3(64 * NW), LDS8, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(stage8_kernel, dim3(a.B), dim3(64 * NW), LDS8, s, a);
    return hipGetLastError();
}

}  // namespace fr
