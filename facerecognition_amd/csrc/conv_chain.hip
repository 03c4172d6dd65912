// FaceNet InceptionResnetV1 repeat_2 -- ten Block17 at 8x8x896 (facenet_model.py:12-16 -> facenet_pytorch
// Block17: x0 = branch0(x), x1 = branch1(x) = 7x1(1x7(1x1(x))), y = relu(conv2d(cat(x0, x1)) * 0.1 + x)) -- as
// ONE launch.  As per-conv launches the 40 convs of the ten blocks are 3.8-7.5 GFLOP each at bs = 256: every
// launch pays a ramp, a few K-steps of exposed latency and a tail, and together they ran at ~330 TFLOP/s
// (0.68 ms, profiles/r05_irv1_layer_profile.txt).  A block of image b reads nothing but image b's block input,
// so here one workgroup owns one image for all ten blocks:
//   * LDS: x (the block input / residual stream, 112 planes of 8 channels x 64 pixels x 16 B = 112 KiB, read as
//     the MFMA B operand: a fragment's 16 lanes read 16 consecutive pixels of one plane, 256 contiguous bytes,
//     conflict-free), two 128-channel branch buffers R1 / R2 (16 KiB each), four 16-B zero slots (the 1x7 / 7x1
//     taps outside the image) and the per-block bias tables, double-buffered;
//   * per block, five passes over one 8x8 image (M = 64 pixels = 4 fragments), each ending in one barrier:
//       A  t1 = relu(W_b1.0 x + b)        x  -> R1   K 896 (28 K-steps), N 128
//       B  t  = relu(W_1x7 * t1 + b)      R1 -> R2   K 7 x 128
//       C  b1 = relu(W_7x1 * t + b)       R2 -> R1   K 7 x 128
//       D  b0 = relu(W_b0 x + b)          x  -> R2   K 896
//       E  x  = relu(W' [b0 | b1] + b' + x)  R2|R1 -> x in place   K 256 (8 K-steps), N 896   (W', b' carry the
//          block's 0.1 scale, weights.fold_state_dict)
//   * 8 waves, 2 per SIMD: in A-D wave w computes output channels 16w..16w+15 (one n-fragment) for all four
//     pixel fragments; in E channels 112w..112w+111 (7 n-fragments).  Every weight fragment is loaded by ONE
//     wave per CU, straight from L2 into a register ring 14 fragments deep: the weights are pre-packed per wave
//     in the order the wave consumes them ([wave][block][168 fragments][64 lanes][16 B]), so the whole chain is
//     one linear stream per wave and the ring runs ahead across pass and block boundaries;
//   * biases: the next block's table is LDS-DMA'd during this block (inline asm, hidden from the compiler's
//     waitcnt pass; every later weight-load wait covers it, the pass barriers publish it);
//   * the same rounding points as the per-conv path (t1, t, b1, b0 and every block output rounded to the
//     storage format); only the f32 summation order differs (E accumulates onto bias + x).
// Bounds: per image and block 2 x 64 x 688,128 = 88.1 MFLOP against 1.38 MB of weights (every
// CU streams every weight byte: 64 FLOP per weight byte at M = 64, so the L2 -> CU weight stream, not the MFMA
// pipe, is the expected limit); HBM: x read once and y written once per image (115 KB each).
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int NPIX = 64;                 // 8 x 8
constexpr int CX = 896;                  // block channels
constexpr int PLB = NPIX * 16;           // bytes per plane of 8 channels
constexpr int X_OFF = 0;                 // 112 planes
constexpr int R1_OFF = (CX / 8) * PLB;   // 114688: t1, then b1
constexpr int R2_OFF = R1_OFF + 16 * PLB;  // 131072: t, then b0
// zero slots ZBASE + 4096 k (k = 0..3, the K-step's 32-channel group: an out-of-image tap's address is ZBASE and
// the group's plane offset 4096 k rides in the instruction's offset field); the bias tables fill the gaps
constexpr int ZBASE = 151536;
__device__ __forceinline__ constexpr int pb_off(int slot) { return slot ? 159744 : 147456; }  // A-D biases, 2 KiB
__device__ __forceinline__ constexpr int qb_off(int slot) { return slot ? 155648 : 151552; }  // E biases, 3.5 KiB
constexpr int CHAIN17_LDS = 163840;
static_assert(R2_OFF + 16 * PLB == 147456, "layout");
static_assert(147456 + 2048 <= ZBASE && 151552 + 3584 <= ZBASE + 4096 && 155648 + 3584 <= ZBASE + 8192 &&
                  159744 + 2048 <= ZBASE + 12288 && ZBASE + 12288 + 16 == CHAIN17_LDS,
              "bias tables must sit between the zero slots");
constexpr int NWV = 8;
constexpr int KSA = 28, KSE = 8, NFE = 7;         // K-steps of A-D / of E, E's n-fragments per wave
constexpr int FRAGS = 4 * KSA + KSE * NFE;        // 168 weight fragments per wave and block
constexpr int RING = 14;                           // register ring (fragments); divides 28 and 56
constexpr int BIAS_BLK = 4 * 128 + CX;            // 1408 floats per block: A | B | C | D (128 each) | E (896)
static_assert(KSA % RING == 0 && (KSE * NFE) % RING == 0 && FRAGS % RING == 0, "ring slots must be compile-time");

typedef int v4i32 __attribute__((ext_vector_type(4)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// 16-byte LDS-DMA (lane l lands at lds_addr + 16 l), invisible to the compiler's waitcnt pass (conv_trans.hip)
__device__ __forceinline__ void dma16(const v4i32& rsrc, uint32_t lds_addr, uint32_t voff, uint32_t soff) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "s"(soff)
                 : "memory", "m0");
}
#pragma clang diagnostic pop

// The lane id recomputed where used (v_mbcnt in volatile asm, never hoisted or kept live across the block loop):
// the loop-invariant per-lane addresses of all five passes would otherwise stay live for the whole kernel and
// push the E pass into scratch spills, whose reloads wait for the entire weight ring (conv_stage.hip fresh_lane)
__device__ __forceinline__ int fresh_lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool F16>
__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
    if (F16) return make_uint2(pack2_f16(a, b), pack2_f16(c, d));
    return make_uint2(pack2_bf16(a, b), pack2_bf16(c, d));
}

template <bool F16>
__global__ __launch_bounds__(64 * NWV, 1) void chain17_kernel(Chain17Args p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x;
    if (b >= p.B) return;

    // ---- bias tables: block `blk` into slot `slot` (waves 0-1: the A-D part, 2-5: the E part)
    const uint64_t bp = (uint64_t)p.bias;
    const v4i32 br = {(int)(uint32_t)bp, (int)((bp >> 32) & 0xffff), (int)(p.nblk * BIAS_BLK * 4), 0x00020000};
    auto issue_bias = [&](int blk, int slot) {
        const uint32_t so = (uint32_t)(blk * BIAS_BLK * 4);
        const int lane = fresh_lane();
        if (wave < 2) {
            dma16(br, (uint32_t)(uintptr_t)(smem + pb_off(slot) + wave * 1024), (uint32_t)(wave * 1024 + lane * 16), so);
        } else if (wave < 5 || (wave == 5 && lane < 32)) {
            const int q = wave - 2;  // 1-KiB piece of the E part
            dma16(br, (uint32_t)(uintptr_t)(smem + qb_off(slot) + q * 1024), (uint32_t)(2048 + q * 1024 + lane * 16), so);
        }
    };

    // ---- x -> LDS: 64 lanes = 4 planes x 16 pixels (64-B runs of a pixel in global, conflict-free 128-B runs in LDS)
    const bf16_t* xb = p.x + (size_t)b * NPIX * CX;
    for (int c = threadIdx.x; c < NPIX * CX / 8; c += 64 * NWV) {
        const int q = c >> 6, l = c & 63, pl = 4 * (q % 28) + (l >> 4), px = 16 * (q / 28) + (l & 15);
        *(uint4*)(smem + X_OFF + pl * PLB + px * 16) = *(const uint4*)(xb + (size_t)px * CX + pl * 8);
    }
    if (threadIdx.x < 4) *(uint4*)(smem + ZBASE + threadIdx.x * 4096) = make_uint4(0, 0, 0, 0);
    issue_bias(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- the wave's weight stream
    const uint32_t w_bytes = (uint32_t)((size_t)NWV * p.nblk * FRAGS * 1024);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, w_bytes, 0x00020000);
    frag wq[RING];
    auto wload = [&](int slot, int g) {  // fragment g of this wave's stream (past the end: zeros, never used)
        wq[slot] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(wr, (uint32_t)(fresh_lane() * 16), (uint32_t)g * 1024u, 0));
    };
    const int gw = wave * p.nblk * FRAGS;
#pragma unroll
    for (int q = 0; q < RING; ++q) wload(q, gw + q);

    f32x4_t acc[NFE][4];
    frag bq[2][4];

    // A / D (KIND 0 / 3): 1x1 over x; B (1): 1x7 over R1; C (2): 7x1 over R2.  One n-fragment (channels 16 wave ..)
    auto pass_n = [&](auto kind_tag, int g0, int slot) {
        constexpr int KIND = decltype(kind_tag)::value;
        const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
        // per-lane B-fragment base: plane lg of the K-step's 32-channel group, pixel 16 j + l15 (j: offset 256 j)
        const int pbase = lg * PLB + l15 * 16;
        const int c8 = l15 & 7, r8 = l15 >> 3;  // column / row-in-fragment of the lane's pixel
        {
            const float4 bs = *(const float4*)(smem + pb_off(slot) + (KIND * 128 + 16 * wave + 4 * lg) * 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[0][j] = (f32x4_t){bs.x, bs.y, bs.z, bs.w};
        }
        int at[KIND == 1 || KIND == 2 ? 7 : 1][4];  // tap-shifted addresses (ZBASE outside the image)
        if (KIND == 1 || KIND == 2) {
#pragma unroll
            for (int t = 0; t < 7; ++t)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (KIND == 1) {
                        const int a = R1_OFF + pbase + 256 * j + (t - 3) * 16;
                        at[t][j] = (unsigned)(c8 + t - 3) < 8u ? a : ZBASE;
                    } else {
                        const int a = R2_OFF + pbase + 256 * j + (t - 3) * 128;
                        at[t][j] = (unsigned)(2 * j + r8 + t - 3) < 8u ? a : ZBASE;
                    }
                }
        }
        auto rd = [&](int s, frag (&q)[4]) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (KIND == 1 || KIND == 2) q[j] = *(const frag*)(smem + at[s >> 2][j] + (s & 3) * 4096);
                else q[j] = *(const frag*)(smem + X_OFF + pbase + 256 * j + s * 4096);
            }
        };
        rd(0, bq[0]);
#pragma unroll
        for (int s = 0; s < KSA; ++s) {
            __builtin_amdgcn_sched_barrier(0);  // keep each step's loads in that step (the scheduler sinks them)
            if (s + 1 < KSA) rd(s + 1, bq[(s + 1) & 1]);
            const frag w = wq[s % RING];
            wload(s % RING, g0 + s + RING);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[0][j] = T::mfma(w, bq[s & 1][j], acc[0][j]);
        }
        // epilogue: ReLU -> storage format -> the destination buffer (A, C -> R1; B, D -> R2).  No pass writes what
        // it reads, and the previous reader of the destination finished before the last pass barrier
        char* const dst = smem + (KIND == 0 || KIND == 2 ? R1_OFF : R2_OFF) + (2 * wave + (lg >> 1)) * PLB + (lg & 1) * 8 +
                          l15 * 16;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            *(uint2*)(dst + 256 * j) = pack4<F16>(relu_bits(acc[0][j][0]), relu_bits(acc[0][j][1]),
                                                  relu_bits(acc[0][j][2]), relu_bits(acc[0][j][3]));
        lds_barrier();
    };

    // E: x = relu(W' [b0 | b1] + b' + x); 7 n-fragments (channels 112 wave ..), K-steps 0-3 over R2 (b0), 4-7 over R1
    auto pass_e = [&](int g0, int slot) {
        const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
        const int pbase = lg * PLB + l15 * 16;
#pragma unroll
        for (int i = 0; i < NFE; ++i) {
            const int n = NFE * wave + i;
            const float4 bs = *(const float4*)(smem + qb_off(slot) + (16 * n + 4 * lg) * 4);
            const char* xs = smem + X_OFF + (2 * n + (lg >> 1)) * PLB + (lg & 1) * 8 + l15 * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint2 xv = *(const uint2*)(xs + 256 * j);
                float f[8];
                T::unpack8(make_uint4(xv.x, xv.y, 0, 0), f);
                acc[i][j] = (f32x4_t){bs.x + f[0], bs.y + f[1], bs.z + f[2], bs.w + f[3]};
            }
        }
        auto rd = [&](int s, frag (&q)[4]) {
#pragma unroll
            for (int j = 0; j < 4; ++j)
                q[j] = *(const frag*)(smem + (s < 4 ? R2_OFF : R1_OFF) + pbase + 256 * j + (s & 3) * 4096);
        };
        rd(0, bq[0]);
#pragma unroll
        for (int s = 0; s < KSE; ++s) {
            __builtin_amdgcn_sched_barrier(0);
            if (s + 1 < KSE) rd(s + 1, bq[(s + 1) & 1]);
#pragma unroll
            for (int i = 0; i < NFE; ++i) {
                const int f = NFE * s + i;
                const frag w = wq[f % RING];
                wload(f % RING, g0 + f + RING);
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = T::mfma(w, bq[s & 1][j], acc[i][j]);
            }
        }
        // in place: each lane overwrites exactly the x values it seeded from; no wave reads x in this pass
#pragma unroll
        for (int i = 0; i < NFE; ++i) {
            const int n = NFE * wave + i;
            char* const xd = smem + X_OFF + (2 * n + (lg >> 1)) * PLB + (lg & 1) * 8 + l15 * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                *(uint2*)(xd + 256 * j) = pack4<F16>(relu_bits(acc[i][j][0]), relu_bits(acc[i][j][1]),
                                                     relu_bits(acc[i][j][2]), relu_bits(acc[i][j][3]));
        }
        lds_barrier();
    };

#pragma unroll 1
    for (int blk = 0; blk < p.nblk; ++blk) {
        const int slot = blk & 1;
        if (blk + 1 < p.nblk) issue_bias(blk + 1, slot ^ 1);
        const int g0 = gw + blk * FRAGS;
        pass_n(std::integral_constant<int, 0>{}, g0, slot);
        pass_n(std::integral_constant<int, 1>{}, g0 + KSA, slot);
        pass_n(std::integral_constant<int, 2>{}, g0 + 2 * KSA, slot);
        pass_n(std::integral_constant<int, 3>{}, g0 + 3 * KSA, slot);
        pass_e(g0 + 4 * KSA, slot);
    }

    // ---- x -> y (NHWC), the same 4-plane x 16-pixel lane map as the load
    bf16_t* yb = p.y + (size_t)b * NPIX * CX;
    for (int c = threadIdx.x; c < NPIX * CX / 8; c += 64 * NWV) {
        const int q = c >> 6, l = c & 63, pl = 4 * (q % 28) + (l >> 4), px = 16 * (q / 28) + (l & 15);
        *(uint4*)(yb + (size_t)px * CX + pl * 8) = *(const uint4*)(smem + X_OFF + pl * PLB + px * 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

bool chain17_supported(int H, int W, int C, int nblk) { return H == 8 && W == 8 && C == CX && nblk >= 1; }

// + RING fragments: the last wave's ring prefetches that far past its stream (the buffer offset is not range-checked)
size_t chain17_weight_elems(int nblk) { return ((size_t)NWV * nblk * FRAGS + RING) * 512; }

size_t chain17_bias_floats(int nblk) { return (size_t)nblk * BIAS_BLK; }

// One block's member convs ([Npad][Kpad] rows, K order (kh, kw, c)) into the per-wave streams:
// fragment = 16 output rows x 32 K, lane (g, r) holds rows[row0 + r][k0 + 8 g .. + 7].
void chain17_pack_block(const bf16_t* rA, int kpA, const bf16_t* r17, int kp17, const bf16_t* r71, int kp71,
                        const bf16_t* rE, int kpE, int blk, int nblk, bf16_t* out) {
    auto frag = [](bf16_t* dst, const bf16_t* rows, int kp, int row0, int k0) {
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) dst[l * 8 + e] = rows[(size_t)(row0 + (l & 15)) * kp + k0 + 8 * (l >> 4) + e];
    };
    for (int w = 0; w < NWV; ++w) {
        bf16_t* o = out + (size_t)(w * nblk + blk) * FRAGS * 512;
        int f = 0;
        for (int s = 0; s < KSA; ++s) frag(o + (size_t)(f++) * 512, rA, kpA, 16 * w, 32 * s);        // A: branch1.0
        for (int s = 0; s < KSA; ++s) frag(o + (size_t)(f++) * 512, r17, kp17, 16 * w, 32 * s);      // B: 1x7
        for (int s = 0; s < KSA; ++s) frag(o + (size_t)(f++) * 512, r71, kp71, 16 * w, 32 * s);      // C: 7x1
        for (int s = 0; s < KSA; ++s) frag(o + (size_t)(f++) * 512, rA, kpA, 128 + 16 * w, 32 * s);  // D: branch0
        for (int s = 0; s < KSE; ++s)
            for (int i = 0; i < NFE; ++i) frag(o + (size_t)(f++) * 512, rE, kpE, 16 * (NFE * w + i), 32 * s);  // E
    }
}

hipError_t launch_chain17(const Chain17Args& a, hipStream_t s) {
    if (a.B <= 0 || a.nblk <= 0 || !a.x || !a.y || !a.w || !a.bias) return hipErrorInvalidValue;
    auto k = a.f16 ? chain17_kernel<true> : chain17_kernel<false>;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, CHAIN17_LDS);
        attr[a.f16 ? 1 : 0] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), CHAIN17_LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), CHAIN17_LDS, s, a);
    return hipGetLastError();
}

}  // namespace fr
