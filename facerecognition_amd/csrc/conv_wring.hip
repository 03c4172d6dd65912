// Implicit-GEMM convolution with the weights streamed from L2 straight into registers (CDNA4 / gfx950):
// the wide IResNet100 convs the LDS-resident stages do not cover -- layer4 (7x7, 512 channels: 6 convs,
// the block-0 one with its downsample K-concatenated), layer3.0 (28x28 -> 256 and the stride-2
// transition), layer4.0.conv1.  Same GEMM view as conv_igemm.hip (M = B*Ho*Wo pixels, N = Cout,
// K = (kh, kw, c) with c fastest, then the K-concatenated 1x1 projection), same fused epilogue.
//
// Why a second kernel: at these shapes the 4-wave 64x64-per-wave igemm tiles read both operands through
// LDS (16 fragment reads per 32 MFMAs) and refill both by LDS-DMA every 64-deep K-step behind a
// vmcnt(0) barrier, and M x N is small (layer4: 12544 x 512), so 128x128 tiles leave 136 of 256 CUs
// with two blocks and 120 with one.  Here:
//   * a block = 112 pixels (7 fragments; layer4: two whole 7x7 images) x 256 output channels, 8 waves,
//     one per 32 channels: 14 v_mfma_f32_16x16x32 per wave per 32-deep K-substep, 56 accumulators;
//     layer4 is 128 x 2 = 256 blocks, one per CU;
//   * operand A (weights, pre-packed per substep as [4 groups of 8 ch][Npad rows][16 B], wring_pack_weights)
//     goes from L2 into a 4-slot register ring, 3 substeps ahead: no LDS, no barrier for the weights; the
//     block index runs over pixels fastest, so an XCD's blocks share one 256-channel weight half (L2);
//   * operand B (the im2col gather) goes global -> LDS by LDS-DMA into a 4-stage ring of 64-channel
//     K-steps (128-B rows XOR-swizzled by the source offset, as in conv_igemm.hip; 128 rows per stage so
//     every wave issues exactly two 1-KiB pieces; rows 112..127 are zero-filled), three stages ahead,
//     one barrier per stage behind a counted vmcnt wait (the younger weight loads stay in flight);
//   * epilogue through an f32 LDS tile (bias or border-class bias, residual, ReLU/PReLU, coalesced
//     8-channel stores), as conv_igemm.hip.
#include "kernels.h"

#include <hip/hip_ext.h>

#include <cstdlib>

namespace fr {
namespace {

constexpr int FM = 7;                       // pixel fragments
constexpr int BM = 16 * FM;                 // 112 pixels per block
constexpr int SROWS = 128;                  // LDS rows per stage (112 used)
constexpr int NST = 4;                      // LDS stages
// KSS = 32-deep substeps per LDS stage (2: 128-B rows, 16 KiB stages; 4: 256-B rows, 32 KiB stages, half
// the barriers, needs Cin % 128 == 0); NW = waves = output channels / 32 (8: 256 channels, one block per
// CU; 4: 128 channels, two blocks per CU)
#ifndef FR_WRING_DEPTH
#define FR_WRING_DEPTH 4  // weight register ring: substeps in flight + 1 (4: 3 ahead; 8: 7 ahead), divides 16
#endif
static_assert(16 % FR_WRING_DEPTH == 0, "ring slots must be compile-time within a 16-substep iteration");

template <int KSS, int NW>
struct WGeo {
    static constexpr int BN = 32 * NW, EPI_LD = BN + 4, EPI_B = BM * EPI_LD * 4;
    static constexpr int CH = 32 * KSS, ROWB = 2 * CH, NCH = ROWB / 16, RPP = 1024 / ROWB;
    static constexpr int STAGE_B = SROWS * ROWB;
    static constexpr int PPW = SROWS * ROWB / 1024 / NW;  // DMA pieces per wave per stage
    static constexpr int P = PPW + 2 * KSS;               // VMEM ops per stage (DMA + weight loads)
    static constexpr int LDS = EPI_B > NST * STAGE_B ? EPI_B : NST * STAGE_B;
    // vmcnt when stage t's last substep waits for DMA(t + 1): VMEM ops younger than it (the prologue
    // issues DMA0..3 then W0..2; stage t issues its KSS weight loads (2 ops each) and, after the
    // boundary, DMA(t + 4)): t = 0 / 1 / >= 2
    static constexpr int WP = 2 * (FR_WRING_DEPTH - 1);  // VMEM ops of the prologue's weight loads
    static constexpr int Yb0 = 2 * PPW + 2 * KSS + WP, Yb1 = 2 * PPW + 4 * KSS + WP, Yb = 2 * PPW + 6 * KSS;
    static_assert(Yb0 <= 63 && Yb1 <= 63 && Yb <= 63, "vmcnt field");
    __device__ static int swz(int row) { return KSS == 2 ? (row >> 1) & 7 : row & 15; }
};

template <int N>
__device__ __forceinline__ void wait_vm() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
constexpr uint32_t OOB = 0x80000000u;


typedef __attribute__((address_space(3))) void lds_void;


__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, 0, 0, 0);
}

template <bool F16, int KSS, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void conv_wring_kernel(ConvArgs p, int tiles_m) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    typedef WGeo<KSS, NW> Gm;
    constexpr int CH = Gm::CH, ROWB = Gm::ROWB, NCH = Gm::NCH, RPP = Gm::RPP, STAGE_B = Gm::STAGE_B;
    constexpr int BN = Gm::BN, EPI_LD = Gm::EPI_LD, PPW = Gm::PPW;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int tn = lid / tiles_m, tm = lid - tn * tiles_m;  // pixels fastest: an XCD keeps one weight half
    const int m0 = tm * BM, n0 = tn * BN;
    const int nks = p.Kpad / 32;  // 32-deep substeps (a multiple of KSS, host-checked)

    // ---- operand B: piece q = wave + NW i (i < PPW) of a stage holds rows RPP q .. RPP q + RPP - 1; the
    // lane's row and its source chunk (the logical chunk stored at its linear destination position)
    const int lrow = lane / NCH;
    const int cl = (lane % NCH) ^ Gm::swz(RPP * wave + lrow);  // the same for every i
    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * p.H * p.W * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.x2 ? p.x2 : p.x), 0,
        (uint32_t)min((size_t)0x7fffffff, p.x2 ? (size_t)p.B * p.H2 * p.W2 * p.Cx2 * 2 : (size_t)0), 0x00020000);
    const int HoWo = p.Ho * p.Wo;
    int a_ih[PPW], a_iw[PPW];
    uint32_t a_base[PPW], a_base2[PPW];
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
        const int row = RPP * (wave + NW * i) + lrow, m = m0 + row;
        if (row < BM && m < p.M) {
            const int b = m / HoWo, r = m - b * HoWo, oh = r / p.Wo, ow = r - oh * p.Wo;
            a_ih[i] = oh * p.sh - p.ph;
            a_iw[i] = ow * p.sw - p.pw;
            a_base[i] = (uint32_t)((((b * p.H + a_ih[i]) * p.W + a_iw[i]) * p.Cx + p.x_off + 8 * cl) * 2);
            a_base2[i] = p.x2 ? (uint32_t)((((b * p.H2 + oh * p.st2) * p.W2 + ow * p.st2) * p.Cx2 + p.x2_off + 8 * cl) * 2)
                              : OOB;
        } else {
            a_ih[i] = -(1 << 28);
            a_iw[i] = 0;
            a_base[i] = 0;
            a_base2[i] = OOB;
        }
    }
    const int K1 = p.x2 ? p.K1 : p.Kpad;
    int r_cur = 0, s_cur = 0, c_cur = 0, k_cur = 0;  // the next stage to issue: tap (r, s), channel base
    // a stage's DMA in two halves: prep (offsets of the next stage, VALU; may run before a barrier) and
    // fire (the LDS-DMA issue into `slot`)
    uint32_t d_off[PPW];
    bool d_x2 = false;
    auto prep = [&]() {
        // branch-free (x or the projection input x2 by selects): a branch around the DMAs made the
        // compiler's counted waits for the weight registers conservative
        d_x2 = k_cur >= K1;  // projection K-steps: x2 at the output's stride-st2 position
        const uint32_t c2 = (uint32_t)((k_cur - K1) * 2);
        const int soff = ((r_cur * p.W + s_cur) * p.Cx + c_cur) * 2;
#pragma unroll
        for (int i = 0; i < PPW; ++i) {
            const int ih = a_ih[i] + r_cur, iw = a_iw[i] + s_cur;
            const bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
            const uint32_t o1 = ok ? a_base[i] + (uint32_t)soff : OOB;
            const uint32_t o2 = a_base2[i] == OOB ? OOB : a_base2[i] + c2;
            d_off[i] = d_x2 ? o2 : o1;
        }
        k_cur += CH;
        c_cur += CH;
        if (c_cur == p.Cin) {
            c_cur = 0;
            if (++s_cur == p.Kw) { s_cur = 0; ++r_cur; }
        }
    };
    auto fire = [&](int slot) {
        const char* dst = smem + slot * STAGE_B;
        const __amdgpu_buffer_rsrc_t rs = d_x2 ? x2r : xr;
#pragma unroll
        for (int i = 0; i < PPW; ++i) dma16(rs, dst + (wave + NW * i) * 1024, d_off[i]);
    };
    auto issue = [&](int slot) {
        prep();
        fire(slot);
    };

    // ---- operand A: packed weights, lane (n = 16 i + (lane & 15) of the wave's 32, group lane >> 4)
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.wimg, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)p.Kpad * p.Npad * 2), 0x00020000);
    const uint32_t wvo = (uint32_t)(((lane >> 4) * p.Npad + n0 + 32 * wave + (lane & 15)) * 16);
    const uint32_t wstep = (uint32_t)(64 * p.Npad);  // bytes per substep image
    constexpr int WD = FR_WRING_DEPTH;
    frag wq[WD][2];
    auto wload = [&](frag (&w)[2], int s) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
            w[i] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(wr, wvo + i * 256,
                                                                                  (uint32_t)s * wstep, 0));
    };

    // B fragment j, substep kk of a stage: row 16 j + (lane & 15), logical chunk 4 kk + (lane >> 4)
    int boff[KSS];
#pragma unroll
    for (int kk = 0; kk < KSS; ++kk)
        boff[kk] = (lane & 15) * ROWB + ((4 * kk + (lane >> 4)) ^ Gm::swz(lane & 15)) * 16;
    frag bq[2][FM];
    auto bread = [&](frag (&b)[FM], int slot, int kk) {
        const char* a = smem + slot * STAGE_B + boff[kk];
#pragma unroll
        for (int j = 0; j < FM; ++j) b[j] = *(const frag*)(a + j * 16 * ROWB);
    };

    f32x4_t acc[2][FM];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    // ---- prologue: stages 0..3 into the four slots, weight substeps 0..2 (vmcnt order: DMA0 .. DMA3
    // (PPW ops each), W0 W1 W2 (2 each)); stage 0 landed, its first B fragments read
    issue(0);
    issue(1);
    issue(2);
    issue(3);
#pragma unroll
    for (int q = 0; q < WD - 1; ++q) wload(wq[q], q);
    wait_vm<3 * PPW + Gm::WP>();
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    bread(bq[0], 0, 0);

    auto mfmas = [&](int slot_w, frag (&b)[FM]) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(wq[slot_w][i], b[j], acc[i][j]);
    };
    // Stage t's LAST substep opens with the stage boundary: every wave's DMA of stage t + 1 landed (counted
    // vmcnt + barrier), every wave is past its reads of stage t (all issued one substep earlier and drained
    // by the lgkmcnt(0) before the barrier), so stage t's slot is refilled with stage t + 4 and stage
    // t + 1's first B fragments are read while the last substep's MFMAs run: the barrier and the cold
    // fragment read of a stage overlap MFMAs instead of preceding them.  Every stage issues all of its
    // VMEM ops unconditionally (past the end the DMAs re-fill slots nobody reads again: zeros, or in-bounds
    // bytes of x2, and the weight loads repeat the last substep); a branch around them made the compiler's
    // own waits for the weight registers drain everything.  VMEM ops younger than DMA(t + 1) at that wait:
    // WGeo::Yb(t) (the prologue's order makes t = 0, 1 differ).
    // 16 substeps per loop iteration: at the loop head the compiler cannot track the register ring
    // carried around the back edge, so the head should come rarely; a partial last iteration breaks out.
#pragma unroll 1
    for (int s4 = 0; s4 < nks; s4 += 16) {
#pragma unroll
        for (int u = 0; u < 16 / KSS; ++u) {
            const int t = s4 / KSS + u;
            if (u > 0 && KSS * t >= nks) break;
            const int slot = t & (NST - 1), nslot = (t + 1) & (NST - 1);
#pragma unroll
            for (int kk = 0; kk < KSS; ++kk) {
                const int s = t * KSS + kk, w = (u * KSS + kk) % WD;  // s4 % 16 == 0: compile-time ring slots
                __builtin_amdgcn_sched_barrier(0);
                wload(wq[(w + WD - 1) % WD], s + WD - 1 < nks ? s + WD - 1 : nks - 1);
                if (kk + 1 < KSS) {
                    bread(bq[(kk + 1) & 1], slot, kk + 1);
                    mfmas(w, bq[kk & 1]);
#pragma unroll
                    for (int q = 0; q < FM; ++q) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                } else {
                    prep();  // stage t + 4's offsets while the previous substep's MFMAs run
                    if (t >= 2) wait_vm<Gm::Yb>();
                    else if (t == 1) wait_vm<Gm::Yb1>();
                    else wait_vm<Gm::Yb0>();
                    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                    fire(slot);  // stage t + 4 into stage t's slot
                    bread(bq[(kk + 1) & 1], nslot, 0);
                    mfmas(w, bq[kk & 1]);
#pragma unroll
                    for (int q = 0; q < FM; ++q) {
                        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                    }
                }
            }
        }
    }

    // ---- epilogue: accumulators -> f32 LDS tile [BM][EPI_LD] -> coalesced 8-channel groups
    constexpr int G = BN / 8, RS = 64 * NW / G, ITER = BM / RS;  // 32 groups, 16 rows per pass, 7 passes
    static_assert(RS * G == 64 * NW && ITER * RS == BM, "epilogue mapping");
    const int g = tid % G, ml0 = tid / G, n = n0 + g * 8;
    uint4 rr[ITER];
    if (p.res) {
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const int m = m0 + ml0 + it * RS;
            rr[it] = *(const uint4*)(p.res + (size_t)(m < p.M ? m : 0) * p.Cres + p.res_off + n);
        }
    }
    // every wave is past its B reads, and the trailing DMAs into the stage slots (which the f32 tile
    // overlays) have landed
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    float* sE = (float*)smem;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j)
            *(f32x4_t*)(sE + (16 * j + (lane & 15)) * EPI_LD + 32 * wave + 16 * i + 4 * (lane >> 4)) = acc[i][j];
    __syncthreads();
    float bias8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sl8[8];
    if (p.bias && !p.bias9) {
        const float4 b0 = *(const float4*)(p.bias + n), b1 = *(const float4*)(p.bias + n + 4);
        bias8[0] = b0.x; bias8[1] = b0.y; bias8[2] = b0.z; bias8[3] = b0.w;
        bias8[4] = b1.x; bias8[5] = b1.y; bias8[6] = b1.z; bias8[7] = b1.w;
    }
    if (p.act == 2) {
        const float4 s0 = *(const float4*)(p.slope + n), s1 = *(const float4*)(p.slope + n + 4);
        sl8[0] = s0.x; sl8[1] = s0.y; sl8[2] = s0.z; sl8[3] = s0.w;
        sl8[4] = s1.x; sl8[5] = s1.y; sl8[6] = s1.z; sl8[7] = s1.w;
    }
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int ml = ml0 + it * RS, m = m0 + ml;
        if (m >= p.M) continue;
        const float4 v0 = *(const float4*)(sE + ml * EPI_LD + g * 8);
        const float4 v1 = *(const float4*)(sE + ml * EPI_LD + g * 8 + 4);
        float v[8] = {v0.x + bias8[0], v0.y + bias8[1], v0.z + bias8[2], v0.w + bias8[3],
                      v1.x + bias8[4], v1.y + bias8[5], v1.z + bias8[6], v1.w + bias8[7]};
        if (p.bias9) {  // border-class bias (bias8 is zero then)
            const int r = m % HoWo;
            const float* bb = p.bias9 + (size_t)border_class(r / p.Wo, r % p.Wo, p.Ho, p.Wo) * p.Npad + n;
            const float4 b0 = *(const float4*)bb, b1 = *(const float4*)(bb + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
        }
        if (p.res) {
            float f[8];
            T::unpack8(rr[it], f);
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
        *(uint4*)(p.y + (size_t)m * p.Cy + p.y_off + n) = F16 && p.y_bf16 ? Num<false>::pack8(v) : T::pack8(v);
    }
}

// out[s][g][n][e] = w[n][32 s + 8 g + e]: one 32-deep substep image per s
__global__ __launch_bounds__(256) void wring_pack_kernel(const bf16_t* __restrict__ w, int Kpad, int Npad,
                                                         bf16_t* __restrict__ out) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x, total = (size_t)(Kpad / 32) * 4 * Npad;
    if (i >= total) return;
    const int n = (int)(i % Npad), g = (int)((i / Npad) % 4), s = (int)(i / ((size_t)4 * Npad));
    *(uint4*)(out + i * 8) = *(const uint4*)(w + (size_t)n * Kpad + 32 * s + 8 * g);
}

}  // namespace

// waves per block for a conv: 8 (256-channel blocks) when Cout % 256 == 0, else 4 (128-channel blocks)
static int wring_nw(const ConvArgs& a) { return a.Cout % 256 == 0 ? 8 : 4; }

bool wring_supported(const ConvArgs& a) {
    const bool kcat = a.x2 != nullptr;
    const int bn = 32 * wring_nw(a);
    return a.B > 0 && a.Cin % 64 == 0 && a.Cout % 128 == 0 && a.Cout % bn == 0 && a.Npad % bn == 0 &&
           a.Npad >= a.Cout && a.Kpad % 64 == 0 && a.Kpad / 64 >= 3 &&
           (kcat ? (a.C2 % 64 == 0 && a.K1 == a.Kh * a.Kw * a.Cin && a.K1 + a.C2 == a.Kpad) : a.K == a.Kpad) &&
           a.K == a.Kh * a.Kw * a.Cin + (kcat ? a.C2 : 0) && a.Cx % 8 == 0 && a.x_off % 8 == 0 &&
           a.Cy % 8 == 0 && a.y_off % 8 == 0 && !a.y2 && !a.partial && !a.w8 && !a.y_amax &&
           (!a.y_bf16 || (a.f16 && !a.res)) && (!a.res || (a.Cres % 8 == 0 && a.res_off % 8 == 0));
}

size_t wring_packed_elems(int Kpad, int Npad) { return (size_t)Kpad * Npad; }

hipError_t wring_pack_weights(const bf16_t* w, int Kpad, int Npad, bf16_t* out, hipStream_t s) {
    const size_t total = (size_t)(Kpad / 32) * 4 * Npad;
    hipLaunchKernelGGL(wring_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, w, Kpad, Npad, out);
    return hipGetLastError();
}

template <int KSS, int NW>
hipError_t launch_kss(const ConvArgs& a, hipStream_t s) {
    typedef WGeo<KSS, NW> Gm;
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = a.Cout / Gm::BN;
    auto k = a.f16 ? conv_wring_kernel<true, KSS, NW> : conv_wring_kernel<false, KSS, NW>;
    const int lds = Gm::LDS;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr[a.f16 ? 1 : 0] = true;
    }
    const dim3 grid((unsigned)(tiles_m * tiles_n));
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, dim3(64 * NW), lds, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a, tiles_m);
    else
        hipLaunchKernelGGL(k, grid, dim3(64 * NW), lds, s, a, tiles_m);
    return hipGetLastError();
}

// 128-channel stages where the channel counts allow (FR_AB wring_kss=2 forces 64-channel stages)
static bool use_kss4(const ConvArgs& a) {
    static const int force = [] { return ab_int("wring_kss", 0); }();
    const bool ok = a.Cin % 128 == 0 && (!a.x2 || a.C2 % 128 == 0) && a.Kpad % 128 == 0 && a.Kpad / 128 >= 3;
    return ok && force != 2;
}


hipError_t launch_conv_wring(const ConvArgs& a, hipStream_t s) {
    if (!wring_supported(a) || !a.wimg) return hipErrorInvalidValue;
    if (wring_nw(a) == 4) return launch_kss<2, 4>(a, s);  // 128-channel blocks: two per CU (64 KiB stages)
    return use_kss4(a) ? launch_kss<4, 8>(a, s) : launch_kss<2, 8>(a, s);
}

}  // namespace fr
