// Small-M implicit GEMM (CDNA4 / gfx950): the convs of small batches (bs = 1 is the reference's online path,
// recognition_engine.py:328-381 -> extract_embedding_single), where M = B*Ho*Wo is a few hundred pixels.  The
// LDS-resident stages put one image on one CU (layer3 at bs = 1: 1.7 ms on one CU) and the implicit-GEMM tiles
// leave most CUs idle while one block walks a long K; split-K needs a second (epilogue) launch per conv.
// Here one WAVE computes a 16-pixel x 64-channel output tile over the whole K with no LDS and no barrier: every
// K-step (32 deep) it loads its 4 weight fragments (16 B per lane, the [Npad][Kpad] rows) and its pixel fragment
// (16 B per lane: the im2col gather, zero by out-of-range buffer offsets at the padding) straight from global
// memory into registers, PF steps ahead, and issues 4 v_mfma_f32_16x16x32.  A 3x3 256->256 conv of one 14x14
// image is 13 x 4 = 52 waves, ~2-3 us.  The K-concatenated 1x1 projection (a transition block's downsample,
// ConvArgs::x2) continues the K loop.  Per output the 32-deep MFMA chain runs over k in order and the epilogue
// is conv_igemm's (acc + bias, + the border-class bias, + residual, activation), so the result equals
// conv_igemm tile 0 bit for bit: an autotuner candidate (FR_TILE_SMALL) that changes nothing numerically.
// KS = 4 / 8 / 16 (the candidate's split): KS waves share one tile, each over a contiguous K chunk, and sum their
// partials through LDS in wave order before the epilogue (deterministic, but the f32 summation order of a
// split-K plan): at bs = 1 a 3x3 256->256 conv has 52 tiles, and one wave walking K = 2304 alone waits on
// 72 steps of weight loads.
// NF = 4 / 2 / 1: 16-channel fragments per tile (64 / 32 / 16 output channels).  A narrower tile spreads a small
// conv over more CUs: at bs = 1 layer3's 52 tiles of 64 channels used 52 of 256 CUs, each pulling its whole 64 x K
// weight slab and 16 x K patch through one CU's L2 port (~290 KB, 2+ us); 16-channel tiles are 208 workgroups of
// ~150 KB each.  The narrower tiles keep PF = 8 steps of loads in flight (their ring is smaller).  KS = 1 with
// NF = 2 / 1 (one wave per 16 px x 32 / 16 ch) is also a candidate at large M: the N = 32 / 96 convs of FaceNet's
// Block35 at bs = 256 fill half of an implicit-GEMM tile's 64 or 128 columns.
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr uint32_t OOB = 0x80000000u;

template <bool F16, int KS, int NFR>
__global__ __launch_bounds__(KS == 1 ? 256 : 64 * KS) void conv_small_kernel(ConvArgs p, int n_mf, int n_units) {
    constexpr int PF = NFR == 4 ? 4 : 8;  // K-steps of loads in flight
    typedef Num<F16> T;
    typedef typename T::frag frag;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int unit = KS == 1 ? blockIdx.x * 4 + wv : blockIdx.x;  // KS > 1: one tile per workgroup
    if (unit >= n_units) return;
    const int mf = unit % n_mf, ng = unit / n_mf;  // pixel fragment, 64-channel group
    const int n0 = ng * 16 * NFR;
    const int g = lane >> 4;                       // k-group: k = 32 s + 8 g .. + 7
    const int m = 16 * mf + (lane & 15);           // the lane's pixel (B operand row)
    const bool mv = m < p.M;
    const int HoWo = p.Ho * p.Wo;
    const int mb = mv ? m / HoWo : 0, mr = mv ? m - mb * HoWo : 0, oh = mr / p.Wo, ow = mr - oh * p.Wo;
    const int ih0 = oh * p.sh - p.ph, iw0 = ow * p.sw - p.pw;

    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * p.H * p.W * p.Cx * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.x2 ? p.x2 : p.x), 0,
        (uint32_t)min((size_t)0x7fffffff, p.x2 ? (size_t)p.B * p.H2 * p.W2 * p.Cx2 * 2 : (size_t)0), 0x00020000);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.w, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)p.Npad * p.Kpad * 2), 0x00020000);
    const int K1 = p.x2 ? p.K1 : p.K;          // the conv's own K; the projection K-steps follow
    const int nks_all = p.Kpad / 32;
    // this wave's K chunk [s_beg, s_end) (all of K for KS = 1)
    const int s_beg = KS == 1 ? 0 : nks_all * wv / KS, s_end = KS == 1 ? nks_all : nks_all * (wv + 1) / KS;
    const int nks = s_end - s_beg;
    const uint32_t wbase = (uint32_t)(((n0 + (lane & 15)) * p.Kpad + 8 * g) * 2);
    const uint32_t x2base = (mv && p.x2)
                                ? (uint32_t)((((mb * p.H2 + oh * p.st2) * p.W2 + ow * p.st2) * p.Cx2 + p.x2_off + 8 * g) * 2)
                                : OOB;
    // the lane's pixel at tap (0, 0) and the mask of the taps inside the image (0 past M), so a K-step costs a
    // scalar tap offset plus a bit test (a 32-deep step lies inside one tap: Cin % 32 == 0)
    const uint32_t xbase = (uint32_t)((((mb * p.H + ih0) * p.W + iw0) * p.Cx + p.x_off + 8 * g) * 2);
    uint32_t vmask = 0;
    for (int r = 0; r < p.Kh; ++r)
        for (int t = 0; t < p.Kw; ++t)
            if (mv && (unsigned)(ih0 + r) < (unsigned)p.H && (unsigned)(iw0 + t) < (unsigned)p.W) vmask |= 1u << (r * p.Kw + t);

    // Operand ring of PF K-steps: the steady-state loop issues the loads of step s + PF right after the MFMAs of
    // step s, unconditionally (steps past the end read zeros by out-of-range offsets), so the loop body has no
    // branch around a load and the compiler waits for exactly the loads each step consumes.
    frag wa[PF][NFR], xb[PF];
    // the next main-conv K-step as (kernel row, kernel column, channel), wave-uniform
    int lc = (32 * s_beg) % p.Cin, lt = (32 * s_beg) / p.Cin, lr = lt / p.Kw;
    lt -= lr * p.Kw;
    auto load_step = [&](int si, int slot) {  // si: the step's index inside the chunk
        const int s = s_beg + si;
        const int k0 = 32 * s;
        const bool proj = k0 >= K1;  // projection K-steps (or the zero padding past K)
        uint32_t xo;
        if (!proj) {
            const int tap = lr * p.Kw + lt;
            const int soff = ((lr * p.W + lt) * p.Cx + lc) * 2;
            xo = ((vmask >> tap) & 1u) ? xbase + (uint32_t)soff : OOB;
            lc += 32;
            if (lc == p.Cin) {
                lc = 0;
                if (++lt == p.Kw) { lt = 0; ++lr; }
            }
        } else {
            const int c = k0 - K1;
            xo = (s < s_end && p.x2 && c < p.C2) ? x2base + (uint32_t)(c * 2) : OOB;
        }
        if (s >= s_end) xo = OOB;
        xb[slot] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(proj ? x2r : xr, xo, 0, 0));
        const uint32_t so = s < s_end ? (uint32_t)(s * 64) : OOB;
#pragma unroll
        for (int i = 0; i < NFR; ++i)
            wa[slot][i] = __builtin_bit_cast(
                frag, __builtin_amdgcn_raw_buffer_load_b128(wr, wbase + (uint32_t)(i * 16 * p.Kpad * 2), so, 0));
    };
    f32x4_t acc[NFR];
#pragma unroll
    for (int i = 0; i < NFR; ++i) acc[i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    auto mfmas = [&](int q) {
#pragma unroll
        for (int i = 0; i < NFR; ++i) acc[i] = T::mfma(wa[q][i], xb[q], acc[i]);
    };
    // the epilogue's global operands (bias, residual), loaded before the K loop: issued after the output stores
    // they could alias, each would be a full memory round trip per fragment
    float4 bz[NFR], b9z[NFR], sz[NFR];
    uint2 rz[NFR];
    const int bcls = border_class(oh, ow, p.Ho, p.Wo);
#pragma unroll
    for (int i = 0; i < NFR; ++i) {
        const int n = n0 + 16 * i + 4 * g;
        const bool nv = n < p.Cout && (KS == 1 || i == wv);  // KS > 1: wave i runs fragment i's epilogue
        const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
        bz[i] = (p.bias && !p.bias9 && nv) ? *(const float4*)(p.bias + n) : z;
        b9z[i] = (p.bias9 && nv) ? *(const float4*)(p.bias9 + (size_t)bcls * p.Npad + n) : z;
        sz[i] = (p.act == 2 && nv) ? *(const float4*)(p.slope + n) : z;
        rz[i] = (p.res && mv && nv) ? *(const uint2*)(p.res + (size_t)m * p.Cres + p.res_off + n) : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int q = 0; q < PF; ++q) load_step(q, q);
    int s0 = 0;
    for (; s0 + PF <= nks; s0 += PF) {
#pragma unroll
        for (int q = 0; q < PF; ++q) {
            mfmas(q);
            load_step(s0 + q + PF, q);
        }
    }
#pragma unroll
    for (int q = 0; q < PF - 1; ++q)
        if (s0 + q < nks) mfmas(q);
    if (KS > 1) {  // partials through LDS, summed in wave order by wave i for fragment i
        __shared__ f32x4_t part[KS > 1 ? KS : 1][NFR][64];
#pragma unroll
        for (int i = 0; i < NFR; ++i) part[wv][i][lane] = acc[i];
        __syncthreads();
        if (wv >= NFR) return;
#pragma unroll
        for (int i = 0; i < NFR; ++i)
            if (i == wv) {
                f32x4_t t = part[0][i][lane];
#pragma unroll
                for (int k = 1; k < KS; ++k) t += part[k][i][lane];
                acc[i] = t;
            }
    }
    if (!mv) return;
    // epilogue (conv_igemm's arithmetic): lane holds channels n .. n + 3 of fragment i of pixel m
#pragma unroll
    for (int i = 0; i < NFR; ++i) {
        const int n = n0 + 16 * i + 4 * g;
        if (n >= p.Cout || (KS > 1 && i != wv)) continue;
        float v[4] = {acc[i][0] + bz[i].x, acc[i][1] + bz[i].y, acc[i][2] + bz[i].z, acc[i][3] + bz[i].w};
        if (p.bias9) {
            v[0] += b9z[i].x; v[1] += b9z[i].y; v[2] += b9z[i].z; v[3] += b9z[i].w;
        }
        if (p.res) {
            float f[8];
            T::unpack8(make_uint4(rz[i].x, rz[i].y, 0u, 0u), f);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += f[e];
        }
        if (p.act == 1) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
        } else if (p.act == 2) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * (&sz[i].x)[e];
        }
        float o8[8] = {v[0], v[1], v[2], v[3], 0.f, 0.f, 0.f, 0.f};
        const uint4 pk = F16 && p.y_bf16 ? Num<false>::pack8(o8) : T::pack8(o8);
        *(uint2*)(p.y + (size_t)m * p.Cy + p.y_off + n) = make_uint2(pk.x, pk.y);
    }
}

}  // namespace

bool small_supported(const ConvArgs& a, int nf) {
    const bool kcat = a.x2 != nullptr;
    return a.B > 0 && a.M > 0 && a.Cin % 32 == 0 && a.Kh * a.Kw <= 32 && a.Cout % (16 * nf) == 0 && a.Npad >= a.Cout &&
           a.Kpad % 32 == 0 &&
           a.Cx % 8 == 0 && a.x_off % 8 == 0 && a.Cy % 4 == 0 && a.y_off % 4 == 0 && !a.y2 && !a.partial && !a.w8 &&
           !a.y_amax && (!a.res || (a.Cres % 4 == 0 && a.res_off % 4 == 0)) &&
           (kcat ? (a.C2 % 32 == 0 && a.Cx2 % 8 == 0 && a.x2_off % 8 == 0 && a.K1 == a.Kh * a.Kw * a.Cin &&
                    a.K1 + a.C2 <= a.Kpad && a.K == a.K1 + a.C2)
                 : a.K == a.Kh * a.Kw * a.Cin) &&
           (!a.y_bf16 || (a.f16 && !a.res)) &&
           // buffer records and offsets are 31-bit: past 2 GiB an operand would read zeros, silently
           (size_t)a.B * a.H * a.W * a.Cx * 2 <= 0x7fffffffull && (size_t)a.Npad * a.Kpad * 2 <= 0x7fffffffull &&
           (size_t)a.M * a.Cy * 2 <= 0x7fffffffull && (!a.res || (size_t)a.M * a.Cres * 2 <= 0x7fffffffull) &&
           (!kcat || (size_t)a.B * a.H2 * a.W2 * a.Cx2 * 2 <= 0x7fffffffull);
}

// split = KS | NF << 8 (NF field 0: the 64-channel tile)
hipError_t launch_conv_small(const ConvArgs& a, int split, hipStream_t s) {
    const int ks = split & 0xff, nf = (split >> 8) ? (split >> 8) : 4;
    if (!small_supported(a, nf) || !small_split_ok(split)) return hipErrorInvalidValue;
    const int n_mf = (a.M + 15) / 16, n_units = n_mf * (a.Cout / (16 * nf));
    const dim3 grid((unsigned)(ks == 1 ? (n_units + 3) / 4 : n_units)), block(ks == 1 ? 256 : 64 * ks);
    void (*k)(ConvArgs, int, int) = nullptr;
#define FR_SMALL_K(KS, NF) \
    if (ks == KS && nf == NF) k = a.f16 ? conv_small_kernel<true, KS, NF> : conv_small_kernel<false, KS, NF>;
    FR_SMALL_K(1, 4) FR_SMALL_K(4, 4) FR_SMALL_K(8, 4) FR_SMALL_K(1, 2) FR_SMALL_K(4, 2) FR_SMALL_K(8, 2)
    FR_SMALL_K(1, 1) FR_SMALL_K(4, 1) FR_SMALL_K(8, 1) FR_SMALL_K(16, 1)
#undef FR_SMALL_K
    if (!k) return hipErrorInvalidValue;
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, block, 0, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a, n_mf, n_units);
    else
        hipLaunchKernelGGL(k, grid, block, 0, s, a, n_mf, n_units);
    return hipGetLastError();
}

bool small_split_ok(int split) {
    const int ks = split & 0xff, nf = split >> 8;
    switch (nf) {
        case 0: return ks == 1 || ks == 4 || ks == 8;
        case 2: return ks == 1 || ks == 4 || ks == 8;
        case 1: return ks == 1 || ks == 4 || ks == 8 || ks == 16;
        default: return false;
    }
}

}  // namespace fr
