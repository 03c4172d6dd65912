// FaceNet InceptionResnetV1 stem at 160x160 (facenet_model.py:12-16 -> facenet_pytorch conv2d_1a, conv2d_2a,
// conv2d_2b, maxpool_3a) as ONE launch:
//   1a  3x3/s2 valid  8 -> 32   160 -> 79  (the 8-channel prepared input [q0 q1 q2 q0 q1 q2 0 0], weights hi/lo
//                                           split: misc.hip preprocess, weights.fold_state_dict)
//   2a  3x3/s1 valid 32 -> 32    79 -> 77
//   2b  3x3/s1 pad 1 32 -> 64    77 -> 77
//   maxpool 3x3/s2   64          77 -> 38
//   3b  1x1          64 -> 80    38 -> 38  (round 6)
// each conv + folded BN + ReLU.  With u8 crops (the product input) the kernel also does the input preparation
// (misc.hip preprocess_u8: q = 2u - 255, exact in f16) on the rows it loads, so nothing but the crops (76.8 KB per
// face) is read.  As four launches the 1a / 2a / 2b tensors (0.4 / 0.38 / 0.76 MB per face) went
// to HBM and back and every conv paid its few-K-step prologue: 0.35 ms at bs = 256 for 87 GFLOP
// (profiles/r05_irv1_layer_profile.txt).  Here one workgroup (4 waves, one per SIMD) owns one image and walks
// down it in 43 phases; only row rings live in LDS:
//   * IN  9 rows of the prepared input, 160 positions x 16 B, each row de-interleaved (even positions at 0..79,
//         odd at 80..159: the stride-2 taps read 16 consecutive positions); phase s LDS-DMAs rows 4s+5 .. 4s+8;
//   * A1  6 rows of 1a, A2 6 rows of 2a (+ one zero row: 2b's padding rows), B2 5 rows of 2b; each row is
//         plane-major ([C/8 planes][80 positions][16 B]: a fragment's 16 lanes read 256 contiguous bytes) and
//         A2 keeps zero halo positions 0 and 78 (2b's padding columns);
//   * PL  2 pooled rows (maxpool output, [8 planes][48 positions][16 B]), the 1x1 conv2d_3b's B operand;
//   * phase s: 1a rows 2s, 2s+1; 2a rows 2s-4, 2s-3; 2b rows 2s-7, 2s-6; maxpool row s-5; 3b row s-6 -- each reads
//     only rows finished in earlier phases, so one barrier per phase; wave w takes row (w >> 1) of each pair: 1a / 2a
//     n-fragment (w & 1) (16 of 32 channels), 2b n-fragments 2 (w & 1) .. +1 (32 of 64), five 16-column
//     fragments (80 columns: 1-3 discarded);
//   * all weights (1a 3 + 2a 9 + 2b 18 fragments per wave) stay in registers; bias + ReLU seeds / epilogues;
//     outputs rounded to the storage format exactly where the per-conv path rounds them (1a, 2a, 2b; the max
//     of rounded values is exact), so only the f32 summation order differs.
// Bounds: per face 2 x (79^2 x 32 x 72 + 77^2 x 32 x 288 + 77^2 x 64 x 288 + 38^2 x 80 x 64) = 0.371 GFLOP (K of
// 1a as stored, 72); HBM: the u8 crop once (76.8 KB; the prepared input, 409.6 KB, for f32 input) + the conv2d_3b
// output once (231 KB).
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int IW = 160, W1 = 79, W2 = 77, WP = 38;
constexpr int RPOS = 80;                       // positions per plane row (A1 / A2 / B2)
constexpr int PL = RPOS * 16;                  // 1280 B per plane row
constexpr int IN_ROW = IW * 16;                // 2560
constexpr int IN_OFF = 0, IN_SLOTS = 9;
constexpr int A1_OFF = IN_OFF + IN_SLOTS * IN_ROW;   // 23040
constexpr int A1_ROW = 4 * PL, A1_SLOTS = 6;          // 5120
constexpr int A2_OFF = A1_OFF + A1_SLOTS * A1_ROW;    // 53760
constexpr int A2_ROW = 4 * PL, A2_SLOTS = 6;          // + the zero row (slot 6)
constexpr int B2_OFF = A2_OFF + (A2_SLOTS + 1) * A2_ROW;  // 89600
constexpr int B2_ROW = 8 * PL, B2_SLOTS = 5;          // 10240
constexpr int PO_OFF = B2_OFF + B2_SLOTS * B2_ROW;   // 140800: pooled rows
constexpr int PO_PL = 48 * 16, PO_ROW = 8 * PO_PL;    // 768 B per plane (38 + 10 discarded positions)
constexpr int STEM_END = PO_OFF + 2 * PO_ROW;         // 153088
constexpr int STEM_LDS = STEM_END + 2048;             // discarded columns' taps read up to 2 positions past a row
constexpr int NPH = 44;                               // phases: maxpool row s - 5, 3b row s - 6 (s = 6 .. 43)
constexpr int C3B = 80;                               // conv2d_3b output channels
constexpr uint32_t OOB = 0x80000000u;
static_assert(STEM_LDS <= 163840, "lds");

typedef int v4i32 __attribute__((ext_vector_type(4)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// 16-byte LDS-DMA (lane l lands at lds_addr + 16 l), invisible to the compiler's waitcnt pass (conv_trans.hip):
// the phase-end vmcnt(0) covers it
__device__ __forceinline__ void dma16(const v4i32& rsrc, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
                 : "memory", "m0");
}
#pragma clang diagnostic pop

template <bool F16>
__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
    if (F16) return make_uint2(pack2_f16(a, b), pack2_f16(c, d));
    return make_uint2(pack2_bf16(a, b), pack2_bf16(c, d));
}

__device__ __forceinline__ int fresh_lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

template <bool F16, bool U8>
__global__ __launch_bounds__(256, 1) void stem160_kernel(Stem160Args p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x;
    if (b >= p.B) return;
    const int lane = threadIdx.x & 63, l15 = lane & 15, lg = lane >> 4;
    const int hr = wave >> 1, nh = wave & 1;  // the wave's row of each pair, its n-fragment half

    // ---- weights into registers: lane (lg, l15) of fragment (n-frag f, K-step s) = rows[16 f + l15][32 s + 8 lg ..]
    frag w1[3], w2[9], w3[9][2];
#pragma unroll
    for (int s = 0; s < 3; ++s) w1[s] = *(const frag*)(p.w1 + (size_t)(16 * nh + l15) * p.kp1 + 32 * s + 8 * lg);
#pragma unroll
    for (int s = 0; s < 9; ++s) w2[s] = *(const frag*)(p.w2 + (size_t)(16 * nh + l15) * p.kp2 + 32 * s + 8 * lg);
#pragma unroll
    for (int s = 0; s < 9; ++s)
#pragma unroll
        for (int i = 0; i < 2; ++i)
            w3[s][i] = *(const frag*)(p.w3 + (size_t)(16 * (2 * nh + i) + l15) * p.kp3 + 32 * s + 8 * lg);
    const float4 bb1 = *(const float4*)(p.b1 + 16 * nh + 4 * lg);
    const float4 bb2 = *(const float4*)(p.b2 + 16 * nh + 4 * lg);
    float4 bb3[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) bb3[i] = *(const float4*)(p.b3 + 16 * (2 * nh + i) + 4 * lg);
    // conv2d_3b: n-fragments wave and (wave 0) 4; K 64 = 2 steps
    const int n4[2] = {wave, wave == 0 ? 4 : -1};
    frag w4[2][2];
    float4 bb4[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int nf = n4[i] < 0 ? 0 : n4[i];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) w4[i][ks] = *(const frag*)(p.w4 + (size_t)(16 * nf + l15) * p.kp4 + 32 * ks + 8 * lg);
        bb4[i] = *(const float4*)(p.b4 + 16 * nf + 4 * lg);
    }

    // ---- input rows: DMA of row `row` (3 pieces: slots 0-63, 64-127, 128-159) into its ring slot; out of the
    // image: zeros (OOB offsets)
    const uint32_t in_bytes = (uint32_t)(IW * IW * 16);
    const uint64_t xp = (uint64_t)(p.x + (size_t)b * IW * IW * 8);
    const v4i32 xr = {(int)(uint32_t)xp, (int)((xp >> 32) & 0xffff), (int)in_bytes, 0x00020000};
    auto dma_piece = [&](int row, int piece) {  // piece 0..2 of the row
        const int ln = fresh_lane();
        const int q = 64 * piece + ln;  // de-interleaved slot
        if (q < IW) {
            const int pos = q < 80 ? 2 * q : 2 * (q - 80) + 1;
            const uint32_t off = row < IW ? (uint32_t)((row * IW + pos) * 16) : OOB;
            dma16(xr, (uint32_t)(uintptr_t)(smem + IN_OFF + (row % IN_SLOTS) * IN_ROW + piece * 1024), off);
        }
    };
    // u8 crops: thread t < 40 k converts positions 4 (t % 40) .. + 3 of row (first + t / 40) into the prepared
    // 8-channel form [q0 q1 q2 q0 q1 q2 0 0], q = 2u - 255 (exact in f16 / bf16), and stores them de-interleaved
    const uint8_t* ub = p.u8 + (size_t)b * IW * IW * 3;
    auto u8_load = [&](int row, uint32_t (&v)[3]) {
        const int t = threadIdx.x % 40;
        v[0] = v[1] = v[2] = 0;
        if ((unsigned)row < (unsigned)IW) {
            const uint32_t* src = (const uint32_t*)(ub + (size_t)row * IW * 3 + 12 * t);
            v[0] = src[0]; v[1] = src[1]; v[2] = src[2];
        }
    };
    auto u8_store = [&](int row, const uint32_t (&v)[3]) {
        const int t = threadIdx.x % 40;
        char* dst = smem + IN_OFF + (row % IN_SLOTS) * IN_ROW;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            float q[8];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int byte = 3 * e + c;
                const uint32_t u = (v[byte >> 2] >> (8 * (byte & 3))) & 0xffu;
                q[c] = q[c + 3] = 2.0f * (float)u - 255.0f;
            }
            q[6] = q[7] = 0.f;
            const int pos = 4 * t + e, slot = (pos & 1) ? 80 + (pos >> 1) : (pos >> 1);
            *(uint4*)(dst + slot * 16) = T::pack8(q);
        }
    };
    // prologue: rows 0..4, zero A2 (halo positions and the zero row)
    if (U8) {
        if (threadIdx.x < 200) {
            uint32_t v[3];
            u8_load(threadIdx.x / 40, v);
            u8_store(threadIdx.x / 40, v);
        }
    } else {
        for (int u = wave; u < 15; u += 4) dma_piece(u / 3, u % 3);
    }
    for (int i = threadIdx.x; i < (A2_SLOTS + 1) * A2_ROW / 16; i += 256)
        *(uint4*)(smem + A2_OFF + i * 16) = make_uint4(0, 0, 0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    bf16_t* const yb = p.y + (size_t)b * WP * WP * C3B;
    f32x4_t acc[2][5];

#pragma unroll 1
    for (int s = 0; s < NPH; ++s) {
        // next phase's input rows 4s+5 .. 4s+8: 12 DMA pieces, 3 per wave; u8: loaded now, stored at the phase end
        uint32_t uv[3];
        if (U8) {
            if (threadIdx.x < 160) u8_load(4 * s + 5 + threadIdx.x / 40, uv);
        } else {
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const int u = wave + 4 * k;
                dma_piece(4 * s + 5 + u / 3, u % 3);
            }
        }
        const int ln = fresh_lane(), c15 = ln & 15, g = ln >> 4;
        // ---- 1a: row i1 = 2s + hr, K = 3 steps of 4 taps x 8 channels (tap 8 repeated for the zero-weight pad)
        {
            const int i1 = 2 * s + hr;
#pragma unroll
            for (int f = 0; f < 5; ++f) acc[0][f] = (f32x4_t){bb1.x, bb1.y, bb1.z, bb1.w};
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) {
                const int tap = min(4 * ks + g, 8), kh = tap / 3, kw = tap - 3 * kh;
                const int row = (2 * i1 + kh) % IN_SLOTS;
                const int q0 = kw == 0 ? c15 : (kw == 1 ? 80 + c15 : c15 + 1);
                const char* src = smem + IN_OFF + row * IN_ROW + q0 * 16;
                frag bq[5];
#pragma unroll
                for (int f = 0; f < 5; ++f) bq[f] = *(const frag*)(src + f * 256);
#pragma unroll
                for (int f = 0; f < 5; ++f) acc[0][f] = T::mfma(w1[ks], bq[f], acc[0][f]);
            }
            char* dst = smem + A1_OFF + (i1 % A1_SLOTS) * A1_ROW + (2 * nh + (g >> 1)) * PL + (g & 1) * 8 + c15 * 16;
#pragma unroll
            for (int f = 0; f < 5; ++f)
                if (16 * f + c15 < W1)
                    *(uint2*)(dst + f * 256) = pack4<F16>(relu_bits(acc[0][f][0]), relu_bits(acc[0][f][1]),
                                                          relu_bits(acc[0][f][2]), relu_bits(acc[0][f][3]));
        }
        // ---- 2a: row i2 = 2s - 4 + hr from 1a rows i2 .. i2 + 2 (valid conv); 9 K-steps = taps x 32 channels
        {
            const int i2 = 2 * s - 4 + hr;
#pragma unroll
            for (int f = 0; f < 5; ++f) acc[0][f] = (f32x4_t){bb2.x, bb2.y, bb2.z, bb2.w};
            frag bq[2][5];
            auto rd = [&](int t, frag (&q)[5]) {
                const int kh = t / 3, kw = t % 3;
                const char* src = smem + A1_OFF + (((i2 + kh) % A1_SLOTS + A1_SLOTS) % A1_SLOTS) * A1_ROW + g * PL +
                                  (c15 + kw) * 16;
#pragma unroll
                for (int f = 0; f < 5; ++f) q[f] = *(const frag*)(src + f * 256);
            };
            rd(0, bq[0]);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                if (t + 1 < 9) rd(t + 1, bq[(t + 1) & 1]);
#pragma unroll
                for (int f = 0; f < 5; ++f) acc[0][f] = T::mfma(w2[t], bq[t & 1][f], acc[0][f]);
            }
            if ((unsigned)i2 < (unsigned)W2) {  // rows outside the image stay unwritten: 2b reads the zero row there
                char* dst = smem + A2_OFF + (i2 % A2_SLOTS) * A2_ROW + (2 * nh + (g >> 1)) * PL + (g & 1) * 8 +
                            (1 + c15) * 16;
#pragma unroll
                for (int f = 0; f < 5; ++f)
                    if (16 * f + c15 < W2)
                        *(uint2*)(dst + f * 256) = pack4<F16>(relu_bits(acc[0][f][0]), relu_bits(acc[0][f][1]),
                                                              relu_bits(acc[0][f][2]), relu_bits(acc[0][f][3]));
            }
        }
        // ---- 2b: row i3 = 2s - 7 + hr from 2a rows i3 - 1 .. i3 + 1 (padding rows: the zero row; padding
        // columns: halo positions 0 / 78); 2 n-fragments
        {
            const int i3 = 2 * s - 7 + hr;
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int f = 0; f < 5; ++f) acc[i][f] = (f32x4_t){bb3[i].x, bb3[i].y, bb3[i].z, bb3[i].w};
            frag bq[2][5];
            auto rd = [&](int t, frag (&q)[5]) {
                const int kh = t / 3, kw = t % 3, r = i3 + kh - 1;
                const int slot = (unsigned)r < (unsigned)W2 ? r % A2_SLOTS : A2_SLOTS;
                const char* src = smem + A2_OFF + slot * A2_ROW + g * PL + (c15 + kw) * 16;
#pragma unroll
                for (int f = 0; f < 5; ++f) q[f] = *(const frag*)(src + f * 256);
            };
            rd(0, bq[0]);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                if (t + 1 < 9) rd(t + 1, bq[(t + 1) & 1]);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int f = 0; f < 5; ++f) acc[i][f] = T::mfma(w3[t][i], bq[t & 1][f], acc[i][f]);
            }
            if ((unsigned)i3 < (unsigned)W2) {
                char* dst = smem + B2_OFF + (i3 % B2_SLOTS) * B2_ROW + (g & 1) * 8 + c15 * 16;
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int f = 0; f < 5; ++f)
                        if (16 * f + c15 < W2)
                            *(uint2*)(dst + (2 * (2 * nh + i) + (g >> 1)) * PL + f * 256) =
                                pack4<F16>(relu_bits(acc[i][f][0]), relu_bits(acc[i][f][1]), relu_bits(acc[i][f][2]),
                                           relu_bits(acc[i][f][3]));
            }
        }
        // ---- 3b: row r3 = s - 6 of the pooled rows (1x1 64 -> 80), straight to global memory
        {
            const int r3 = s - 6;
            if (r3 >= 0) {
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int f = 0; f < 3; ++f) acc[i][f] = (f32x4_t){bb4[i].x, bb4[i].y, bb4[i].z, bb4[i].w};
                const char* src = smem + PO_OFF + (r3 & 1) * PO_ROW + g * PO_PL + c15 * 16;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks) {
                    frag bq[3];
#pragma unroll
                    for (int f = 0; f < 3; ++f) bq[f] = *(const frag*)(src + 4 * ks * PO_PL + f * 256);
#pragma unroll
                    for (int i = 0; i < 2; ++i)
                        if (n4[i] >= 0)
#pragma unroll
                            for (int f = 0; f < 3; ++f) acc[i][f] = T::mfma(w4[i][ks], bq[f], acc[i][f]);
                }
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    if (n4[i] >= 0)
#pragma unroll
                        for (int f = 0; f < 3; ++f) {
                            const int px = 16 * f + c15;
                            if (px < WP)
                                *(uint2*)(yb + ((size_t)r3 * WP + px) * C3B + 16 * n4[i] + 4 * g) =
                                    pack4<F16>(relu_bits(acc[i][f][0]), relu_bits(acc[i][f][1]), relu_bits(acc[i][f][2]),
                                               relu_bits(acc[i][f][3]));
                        }
            }
        }
        // ---- maxpool row r = s - 5 from 2b rows 2r .. 2r + 2 (written in earlier phases): 38 x 8 planes, into the
        // pooled ring (3b reads it next phase)
        {
            const int r = s - 5;
            if (r >= 0 && r < WP) {
                for (int it = threadIdx.x; it < WP * 8; it += 256) {
                    // lanes walk the output columns of one plane: their 16-B reads are 32 B apart (2-way bank sharing);
                    // walking the planes of one column put 8 lanes on the same banks
                    const int pl = it / WP, oc = it - pl * WP;
                    float m[8];
#pragma unroll
                    for (int e = 0; e < 8; ++e) m[e] = -INFINITY;
#pragma unroll
                    for (int kh = 0; kh < 3; ++kh) {
                        const char* src = smem + B2_OFF + ((2 * r + kh) % B2_SLOTS) * B2_ROW + pl * PL + 2 * oc * 16;
#pragma unroll
                        for (int kw = 0; kw < 3; ++kw) {
                            float f[8];
                            T::unpack8(*(const uint4*)(src + kw * 16), f);
#pragma unroll
                            for (int e = 0; e < 8; ++e) m[e] = fmaxf(m[e], f[e]);
                        }
                    }
                    *(uint4*)(smem + PO_OFF + (r & 1) * PO_ROW + pl * PO_PL + oc * 16) = T::pack8(m);
                }
            }
        }
        if (U8 && threadIdx.x < 160) u8_store(4 * s + 5 + threadIdx.x / 40, uv);
        // the next phase's input rows landed, every ring write of this phase is visible
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

}  // namespace

bool stem160_supported(int H, int W, int Cin, int K1, int K2, int K3, int K4, int C1, int C2, int C3, int C4) {
    return H == IW && W == IW && Cin == 8 && K1 == 72 && K2 == 288 && K3 == 288 && K4 == 64 && C1 == 32 && C2 == 32 &&
           C3 == 64 && C4 == C3B;
}

hipError_t launch_stem160(const Stem160Args& a, hipStream_t s) {
    if (a.B <= 0 || (!a.x && !a.u8) || !a.y || !a.w1 || !a.w2 || !a.w3 || !a.w4 || !a.b1 || !a.b2 || !a.b3 || !a.b4 ||
        a.kp1 < 96 || a.kp2 < 288 || a.kp3 < 288 || a.kp4 < 64)
        return hipErrorInvalidValue;
    const bool u8 = a.u8 != nullptr;
    auto k = a.f16 ? (u8 ? stem160_kernel<true, true> : stem160_kernel<true, false>)
                   : (u8 ? stem160_kernel<false, true> : stem160_kernel<false, false>);
    static bool attr[4] = {false, false, false, false};
    const int ai = (a.f16 ? 2 : 0) + (u8 ? 1 : 0);
    if (!attr[ai]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, STEM_LDS);
        attr[ai] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(256), STEM_LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(256), STEM_LDS, s, a);
    return hipGetLastError();
}

}  // namespace fr
