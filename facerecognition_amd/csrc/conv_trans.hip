// Fused IResNet100 transition block layer1.0 (insightface IBasicBlock with stride 2):
//   t = PReLU(conv3x3_s1(bn1(x)) + b1)            112x112x64 -> 112x112x64   (236.8 GFLOP at bs = 256)
//   y = conv3x3_s2(t) + downsample1x1_s2(x) + b2  -> 56x56x64                 ( 65.8 GFLOP)
// bn1 is folded into conv1 as a border-class bias (ep1 [9][64]), bn2 / bn3 / the downsample BN into the
// weights and b2 (weights.fold_state_dict; the downsample rows K-concatenated after conv2's 576).
//
// As two launches (conv_rows 112^2, then the implicit-GEMM transition) the 411 MB t tensor goes to HBM
// and back and x is read twice; both kernels are bounded by that traffic and by their short K (576):
// 0.43 ms at bs = 256.  Here one workgroup (4 waves, one per SIMD) owns one image and walks down it in
// 57 phases, keeping only a few rows of x and t in LDS:
//   * x ring: 6 rows x 114 positions (zero halo columns) x 64 channels, 128-B positions with their 16-B
//     chunks XOR-swizzled by the position (conflict-free fragment reads for every tap shift); phase s
//     reads x rows 2s-1 .. 2s+2 while the LDS-DMA fills rows 2s+3, 2s+4 for the next phase;
//   * t ring: 5 rows x 113 positions, each row stored de-interleaved (even columns at 0..55, odd columns
//     -1, 1, .., 111 at 56..112), so the stride-2 conv reads 16 consecutive positions per fragment like a
//     stride-1 conv; phase s writes t rows 2s, 2s+1 while conv2 reads rows 2s-3 .. 2s-1;
//   * phase s: conv1 of t rows 2s, 2s+1 (wave = t row x 32 channels: 7 x 2 fragments, 18 K-steps), the
//     downsample of output row s (2 K-steps, its sums seeded with b2 become conv2's seeds next phase) and
//     conv2 of output row s-1 (wave = 16 channels x 4 fragments of 16 output columns, 18 K-steps; 8 of
//     the 64 columns are padding), one barrier per phase;
//   * ALL weights live in registers for the whole kernel (conv1: 36 A fragments = 144 VGPRs per wave,
//     conv2 + downsample: 20 = 80 VGPRs): nothing but the x rows and the y rows crosses the memory
//     hierarchy in the phase loop.
// HBM per image: x read once (1.6 MB) + y written once (0.4 MB); MFMA per image 2 x 1.18 GFLOP.
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int TW = 112;                   // x / t width and height
constexpr int OW = 56;                    // y width and height
constexpr int TCH = 64;                   // channels of x, t, y
constexpr int XPOS = TW + 2;              // x row: 0 = left halo, 1..112 = columns, 113 = right halo
constexpr int XROW_B = XPOS * 128;        // 14592
constexpr int XSLOTS = 6;
constexpr int XQ = XPOS * 8;              // 16-B slots per x row (912)
constexpr int XPIECES = (XQ + 63) / 64;   // 1-KiB DMA pieces per row (15, the last 16 lanes)
constexpr int TPOS = 113;                 // t row: even columns 0..55, odd columns (-1, 1, .., 111) 56..112
constexpr int TROW_B = TPOS * 128;        // 14464
constexpr int TSLOTS = 5;
constexpr int T_OFF = 0;
constexpr int X_OFF = TSLOTS * TROW_B;    // 72320
constexpr int TAB = X_OFF + XSLOTS * XROW_B;  // 159872: ep1 [9][64] (rows TROWF apart), slope1 [64], b2 [64] (f32)
constexpr int TROWF = TCH + 8;             // ep1 row stride in floats: 2 bank slots of padding (the rows of a
                                           // fragment's border classes fall on different banks)
constexpr int TAB_B = (9 * TROWF + 2 * TCH) * 4;
constexpr int TRANS_LDS = 163840;         // the whole LDS (padding-lane fragment reads stay inside it)
static_assert(TAB + TAB_B <= TRANS_LDS, "lds");
constexpr int NPH = OW + 1;               // phases
constexpr int KS1 = 18, KS2 = 20;         // K-steps: conv1 (9 taps x 2 channel halves), conv2 + downsample
constexpr uint32_t OOB = 0x80000000u;

// 16-byte LDS-DMA (buffer_load_dwordx4 ... lds; lane l lands at lds_addr + 16 l) from inline asm: the
// compiler then does not see the LDS write, and its waitcnt pass does not put a vmcnt(0) (the whole DMA)
// in front of the phase's fragment reads, none of which reads the slots in flight.  The kernel's own waits
// cover the DMA (m0 is reserved to the compiler, hence the pragma; nothing else here uses m0).
typedef int v4i32 __attribute__((ext_vector_type(4)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(const v4i32& rsrc, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
                 : "memory", "m0");
}
#pragma clang diagnostic pop

// acc += w * b with the weight fragment in AGPRs (the whole weight set stays in the accumulator half of the
// register file for the kernel; hipcc only offers MFMA operands from VGPRs and would copy every fragment
// through v_accvgpr_read).  Not volatile: the scheduler may interleave it like the builtin.  hipcc does not pad
// inline asm, so: a VALU-written accumulator seed needs 2 wait states before its first MFMA (the FIRST form),
// and the MFMA result needs 8 before a VALU reads it (mfma_drain() ahead of such reads).
template <bool F16, bool FIRST = false>
__device__ __forceinline__ void mfma_aw(f32x4_t& acc, const typename Num<F16>::frag& w, const typename Num<F16>::frag& b) {
    if (F16) {
        if (FIRST) asm("s_nop 1\n\tv_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(b));
        else asm("v_mfma_f32_16x16x32_f16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(b));
    } else {
        if (FIRST) asm("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(b));
        else asm("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "a"(w), "v"(b));
    }
}
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 7" ::: "memory"); }


template <bool F16>
__global__ __launch_bounds__(256, 1) void trans_kernel(TransArgs p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x;
    if (b >= p.B) return;
    const int r1 = wave >> 1;  // conv1: t row 2s + r1
    const int np = wave & 1;   // conv1: output channels 32 np .. 32 np + 31 (n-fragments 2 np, 2 np + 1)
    const int l15 = lane & 15, lg = lane >> 4;

    // ---- weights into registers (K-step images [ks][4 groups][64 rows][16 B])
    frag w1[KS1][2], w2[KS2];
#pragma unroll
    for (int ks = 0; ks < KS1; ++ks)
#pragma unroll
        for (int i = 0; i < 2; ++i)
            w1[ks][i] = *(const frag*)(p.w1 + ((size_t)(ks * 4 + lg) * 64 + 16 * (2 * np + i) + l15) * 8);
#pragma unroll
    for (int ks = 0; ks < KS2; ++ks) w2[ks] = *(const frag*)(p.w2 + ((size_t)(ks * 4 + lg) * 64 + 16 * wave + l15) * 8);

    // ---- epilogue tables into LDS; t ring: the zero row -1 (slot 0) and the zero column -1 of every slot
    {
        float* tab = (float*)(smem + TAB);
        for (int i = threadIdx.x; i < 9 * TCH; i += 256) tab[(i / TCH) * TROWF + i % TCH] = p.ep1[i];
        for (int i = threadIdx.x; i < TCH; i += 256) {
            tab[9 * TROWF + i] = p.slope1[i];
            tab[9 * TROWF + TCH + i] = p.b2[i];
        }
        for (int i = threadIdx.x; i < TROW_B / 16; i += 256) *(uint4*)(smem + T_OFF + i * 16) = make_uint4(0, 0, 0, 0);
        if (threadIdx.x < (TSLOTS - 1) * 8) {
            const int sl = 1 + threadIdx.x / 8, c = threadIdx.x % 8;
            *(uint4*)(smem + T_OFF + sl * TROW_B + 56 * 128 + c * 16) = make_uint4(0, 0, 0, 0);
        }
    }

    // ---- x row DMA: row `row` into its slot (row + 1) % 6; rows outside the image read as zeros
    // (the resource spans this image only: 32-bit offsets at any batch size)
    const uint32_t x_bytes = (uint32_t)(TW * TW * TCH * 2);
    const uint64_t xp = (uint64_t)(p.x + (size_t)b * TW * TW * TCH);
    const v4i32 xr = {(int)(uint32_t)xp, (int)((xp >> 32) & 0xffff), (int)x_bytes, 0x00020000};
    // per piece u (pieces wave + 4 u): the lane's source offset within a row (or OOB for halo columns)
    uint32_t colpart[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int q = (wave + 4 * u) * 64 + lane, pos = q >> 3, ch = q & 7, col = pos - 1;
        const int g = ch ^ (pos & 7);
        colpart[u] = (unsigned)col < (unsigned)TW ? (uint32_t)((col * TCH + g * 8) * 2) : OOB;
    }
    auto dma_row = [&](int row) {
        const int slot = (row + 1) % XSLOTS;
        const bool rin = (unsigned)row < (unsigned)TW;
        const uint32_t rbase = (uint32_t)((rin ? row : 0) * TW * TCH * 2);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int piece = wave + 4 * u;
            if (piece < XPIECES && piece * 64 + lane < XQ) {
                const uint32_t off = rin && colpart[u] != OOB ? rbase + colpart[u] : OOB;
                dma16(xr, (uint32_t)(uintptr_t)(smem + X_OFF + slot * XROW_B + piece * 1024), off);
            }
        }
    };
    for (int row = -1; row <= 2; ++row) dma_row(row);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- per-lane fragment offsets
    // conv1 B: t column 16 j + l15 at tap column dw reads x position 16 j + l15 + dw
    int xo[3];
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
        const int pos = l15 + dw;
        xo[dw] = pos * 128 + ((lg ^ (pos & 7)) * 16);
    }
    // conv2 B: output column 16 j + l15 (= c) at tap column dw reads t column 2c + dw - 1: position
    // 56 + c (dw 0), c (dw 1), 57 + c (dw 2)
    int to2[3];
#pragma unroll
    for (int dw = 0; dw < 3; ++dw) {
        const int pos = l15 + (dw == 0 ? 56 : (dw == 1 ? 0 : 57));
        to2[dw] = pos * 128 + ((lg ^ (pos & 7)) * 16);
    }
    // downsample B: x column 2c at position 2c + 1
    int xd;
    {
        const int pos = 2 * l15 + 1;
        xd = pos * 128 + ((lg ^ (pos & 7)) * 16);
    }
    // conv1 epilogue: t column p = 16 j + l15 -> position pe = p/2 (even) or 56 + (p+1)/2 (odd) = 8 j + pel
    int te[2];
    {
        const int pel = (l15 & 1) ? 56 + ((l15 + 1) >> 1) : (l15 >> 1);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int n = 16 * (2 * np + i) + 4 * lg;
            te[i] = pel * 128 + ((((n >> 3) ^ (pel & 7))) * 16) + ((n >> 2) & 1) * 8;
        }
    }
    const float* tab = (const float*)(smem + TAB);
    float4 s1m[2];  // conv1 PReLU: slope - 1
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const float4 sl = *(const float4*)(tab + 9 * TROWF + 16 * (2 * np + i) + 4 * lg);
        s1m[i] = make_float4(sl.x - 1.f, sl.y - 1.f, sl.z - 1.f, sl.w - 1.f);
    }
    const int n2 = 16 * wave + 4 * lg;  // conv2: the lane's 4 output channels
    const float4 b2v = *(const float4*)(tab + 9 * TROWF + TCH + n2);

    f32x4_t acc1[2][7], acc2[4], accd[4];
    bf16_t* const yb = p.y + (size_t)b * OW * OW * TCH;
    // one x-row DMA piece (u: 0..3 of row 2s + 3, 4..7 of row 2s + 4), spread over loop A's first K-steps
    auto dma_piece = [&](int s, int u) {
        const int row = 2 * s + 3 + (u >> 2), piece = wave + 4 * (u & 3);
        if (row <= TW && piece < XPIECES && piece * 64 + lane < XQ) {
            const bool rin = row < TW;
            const uint32_t off = rin && colpart[u & 3] != OOB
                                     ? (uint32_t)(row * TW * TCH * 2) + colpart[u & 3]
                                     : OOB;
            dma16(xr, (uint32_t)(uintptr_t)(smem + X_OFF + ((row + 1) % XSLOTS) * XROW_B + piece * 1024), off);
        }
    };
    // conv1 epilogue of tile (i, j): PReLU -> bf16 -> the t row's slot
    auto epi1 = [&](char* tb, int i, int j) {
        float v[8];
        v[0] = fmaf(s1m[i].x, min0_raw(acc1[i][j][0]), acc1[i][j][0]);
        v[1] = fmaf(s1m[i].y, min0_raw(acc1[i][j][1]), acc1[i][j][1]);
        v[2] = fmaf(s1m[i].z, min0_raw(acc1[i][j][2]), acc1[i][j][2]);
        v[3] = fmaf(s1m[i].w, min0_raw(acc1[i][j][3]), acc1[i][j][3]);
        v[4] = v[5] = v[6] = v[7] = 0.f;
        const uint4 pk = T::pack8(v);
        *(uint2*)(tb + 1024 * j + te[i]) = make_uint2(pk.x, pk.y);
    };

    // Phase s: conv1 of t rows 2s, 2s+1 (s = 56: rows 112, 113, discarded), the downsample of output row s and
    // conv2 of output row s - 1 (s = 0: of row 0 from the zero / not yet written t slots, discarded).  Two
    // K loops: A = conv1 fragments 0..3 (+ the downsample's 2 K-steps, + the next rows' DMA pieces);
    // B = conv1 fragments 4..6 + conv2, with the epilogue of fragments 0..3 interleaved; then the epilogue
    // of fragments 4..6 and conv2's stores.  Every phase runs the same instruction stream.
#pragma unroll 1
    for (int s = 0; s < NPH; ++s) {
        const int tr = 2 * s + r1;  // this wave's t row
        const int o = s > 0 ? s - 1 : 0;  // conv2's output row
        // seeds: conv1 = bias of the border class, downsample = b2 (conv2 then starts from the downsample)
        {
            const int rc = tr == 0 ? 0 : (tr == TW - 1 ? 2 : 1);
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                const int cc = (j == 0 && l15 == 0) ? 0 : ((j == 6 && l15 == 15) ? 2 : 1);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const float4 bb = *(const float4*)(tab + (3 * rc + cc) * TROWF + 16 * (2 * np + i) + 4 * lg);
                    acc1[i][j] = (f32x4_t){bb.x, bb.y, bb.z, bb.w};
                }
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) accd[j] = (f32x4_t){b2v.x, b2v.y, b2v.z, b2v.w};
        }
        // x row of tap row dh for this wave's t row: tr + dh - 1 -> slot (tr + dh) % 6
        int xb[3];
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) xb[dh] = X_OFF + ((tr + dh) % XSLOTS) * XROW_B;
        int tb2[3];  // conv2: t row 2o + dh - 1 -> slot (2o + dh) % 5
#pragma unroll
        for (int dh = 0; dh < 3; ++dh) tb2[dh] = T_OFF + ((2 * o + dh) % TSLOTS) * TROW_B;
        const int xdb = X_OFF + ((2 * s + 1) % XSLOTS) * XROW_B;  // downsample: x row 2s

        // ---- loop A: conv1 fragments 0..3, the downsample at K-steps 0 / 1, DMA pieces at K-steps 0..7
        {
            frag ba[2][4], bd[2][4];
            auto rdA = [&](int ks, int buf) {
                const int tap = ks >> 1, cg = ks & 1, dh = tap / 3, dw = tap % 3;
#pragma unroll
                for (int j = 0; j < 4; ++j) ba[buf][j] = *(const frag*)(smem + xb[dh] + 2048 * j + (xo[dw] ^ (cg << 6)));
            };
            auto rdD = [&](int cg) {
#pragma unroll
                for (int j = 0; j < 4; ++j) bd[cg][j] = *(const frag*)(smem + xdb + 4096 * j + (xd ^ (cg << 6)));
            };
            rdA(0, 0);
            rdD(0);
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) {
                __builtin_amdgcn_sched_barrier(0);
                if (ks + 1 < KS1) rdA(ks + 1, (ks + 1) & 1);
                if (ks == 0) rdD(1);
                if (ks < 8) dma_piece(s, ks);
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (ks == 0) mfma_aw<F16, true>(acc1[i][j], w1[ks][i], ba[ks & 1][j]);
                        else mfma_aw<F16>(acc1[i][j], w1[ks][i], ba[ks & 1][j]);
                    }
                if (ks < 2) {
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        if (ks == 0) mfma_aw<F16, true>(accd[j], w2[KS1 + ks], bd[ks][j]);
                        else mfma_aw<F16>(accd[j], w2[KS1 + ks], bd[ks][j]);
                    }
                }
            }
        }
        // ---- loop B: conv1 fragments 4..6 + conv2 of output row o; the epilogue of fragments 0..3 rides along
        char* const tb = smem + T_OFF + ((tr + 1) % TSLOTS) * TROW_B;  // this wave's t row slot
        {
            frag bb[2][3], bt[2][4];
            auto rdB = [&](int ks, int buf) {
                const int tap = ks >> 1, cg = ks & 1, dh = tap / 3, dw = tap % 3;
#pragma unroll
                for (int j = 0; j < 3; ++j)
                    bb[buf][j] = *(const frag*)(smem + xb[dh] + 2048 * (4 + j) + (xo[dw] ^ (cg << 6)));
#pragma unroll
                for (int j = 0; j < 4; ++j) bt[buf][j] = *(const frag*)(smem + tb2[dh] + 2048 * j + (to2[dw] ^ (cg << 6)));
            };
            rdB(0, 0);
#pragma unroll
            for (int ks = 0; ks < KS1; ++ks) {
                __builtin_amdgcn_sched_barrier(0);
                if (ks + 1 < KS1) rdB(ks + 1, (ks + 1) & 1);
#pragma unroll
                for (int j = 0; j < 3; ++j)
#pragma unroll
                    for (int i = 0; i < 2; ++i) {
                        if (ks == 0) mfma_aw<F16, true>(acc1[i][4 + j], w1[ks][i], bb[ks & 1][j]);
                        else mfma_aw<F16>(acc1[i][4 + j], w1[ks][i], bb[ks & 1][j]);
                    }
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (ks == 0) mfma_aw<F16, true>(acc2[j], w2[ks], bt[ks & 1][j]);
                    else mfma_aw<F16>(acc2[j], w2[ks], bt[ks & 1][j]);
                }
                if (ks >= 1 && ks <= 8) epi1(tb, (ks - 1) & 1, (ks - 1) >> 1);
            }
        }
        // ---- tail: epilogue of fragments 4..6, conv2's output row, the downsample sums become conv2's seeds
        mfma_drain();  // the last MFMAs' results are read by VALU below
#pragma unroll
        for (int j = 4; j < 7; ++j)
#pragma unroll
            for (int i = 0; i < 2; ++i) epi1(tb, i, j);
        if (s > 0) {
            bf16_t* const yr = yb + (size_t)o * OW * TCH + n2;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int c = 16 * j + l15;
                float v[8] = {acc2[j][0], acc2[j][1], acc2[j][2], acc2[j][3], 0.f, 0.f, 0.f, 0.f};
                const uint4 pk = T::pack8(v);
                if (c < OW) *(uint2*)(yr + (size_t)c * TCH) = make_uint2(pk.x, pk.y);
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc2[j] = accd[j];
        // the next phase's x rows landed (the y stores may stay in flight), every t write is done
        if (s > 0) asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// out[ks][g][n][e] = w[n][32 ks + 8 g + e]  (n < 64)
__global__ __launch_bounds__(256) void trans_pack_kernel(const bf16_t* __restrict__ w, int Kpad, int KS,
                                                         bf16_t* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x, total = KS * 4 * 64;
    if (i >= total) return;
    const int n = i % 64, g = (i / 64) % 4, ks = i / 256;
    *(uint4*)(out + (size_t)i * 8) = *(const uint4*)(w + (size_t)n * Kpad + 32 * ks + 8 * g);
}

}  // namespace

bool trans_supported(int B, int H, int W, int Cin, int Cmid, int Cout, int K1, int K2) {
    return B > 0 && H == TW && W == TW && Cin == TCH && Cmid == TCH && Cout == TCH && K1 == 32 * KS1 &&
           K2 == 32 * KS2;
}

size_t trans_packed_elems(int K) { return (size_t)(K / 32) * 4 * 64 * 8; }

hipError_t trans_pack_weights(const bf16_t* w, int Kpad, int K, bf16_t* out, hipStream_t s) {
    const int KS = K / 32, total = KS * 4 * 64;
    hipLaunchKernelGGL(trans_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, s, w, Kpad, KS, out);
    return hipGetLastError();
}

hipError_t launch_trans(const TransArgs& a, hipStream_t s) {
    if (!trans_supported(a.B, TW, TW, TCH, TCH, TCH, 32 * KS1, 32 * KS2) || !a.x || !a.y || !a.w1 || !a.w2 || !a.ep1 ||
        !a.slope1 || !a.b2)
        return hipErrorInvalidValue;
    auto k = a.f16 ? trans_kernel<true> : trans_kernel<false>;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, TRANS_LDS);
        attr[a.f16 ? 1 : 0] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(256), TRANS_LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(256), TRANS_LDS, s, a);
    return hipGetLastError();
}

}  // namespace fr
