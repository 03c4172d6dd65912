// ResNet-50 ArcFace layer3.1 .. layer3.5 -- five torchvision Bottlenecks at 7x7x1024 (arcface_model.py:118-132:
// the torchvision resnet50 backbone; y = relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1(x)))))))) + x)) -- as ONE
// launch.  As per-conv launches the 15 convs run at 300-540 TFLOP/s (profiles/r06_r50_layer_profile.txt: 22 + 28 +
// 17 us per block at bs = 256), each paying a ramp and a store / reload of its activation.  A block of image b reads
// nothing but image b's block input, so here one workgroup owns one image for all five blocks (the scheme of
// conv_chain.hip's IRV1 repeat_2):
//   * LDS: x (the block input / residual stream: 128 planes of 8 channels x 49 pixels x 16 B = 100,352 B, read as
//     the MFMA B operand: a fragment's 16 lanes read 16 consecutive pixels of one plane), t1 (conv1's output, 32
//     planes of 50 positions: position 49 stays zero, the 3x3 taps outside the image read it), t2 (conv2's output,
//     32 planes x 50) and the per-block bias tables, double-buffered: 163,840 B.  The pixel fragments are 16
//     pixels: 4 fragments cover 64 slots, of which 49 are the image; lanes of the 15 slots past it read whatever
//     follows the plane (their MFMA columns are never stored: every epilogue store is masked to pixel < 49);
//   * per block, three passes, each ending in one barrier:
//       1  t1 = relu(W1 x + b1)            x  -> t1   K 1024 (32 K-steps), N 256: wave w channels 32w .. 32w+31
//       2  t2 = relu(W2 * t1 + b2)         t1 -> t2   K 9 x 256 (72 K-steps), N 256: the same channels
//       3  x  = relu(W3 t2 + b3 + x)       t2 -> x in place   K 256 (8 K-steps), N 1024: channels 128w .. 128w+127,
//          as two halves of 4 n-fragments (64 accumulators each, so the 256-VGPR budget holds the weight ring)
//   * 8 waves, 2 per SIMD.  Every weight fragment is loaded by ONE wave per CU, straight from L2 into a 16-deep
//     register ring; the weights are pre-packed per wave in consumption order ([wave][block][272 fragments][64
//     lanes][16 B]), so the chain is one linear stream per wave and the ring runs ahead across passes and blocks;
//   * the same rounding points as the per-conv path (t1, t2 and every block output rounded to the storage
//     format); only the f32 summation order differs (pass 3 accumulates onto bias + x).
// Bounds: per image and block 2 x 49 x 1,114,112 = 109 MFLOP (142 with the 64-slot fragments)
// against 2.23 MB of weights: the L2 -> CU weight stream (571 MB per block at bs = 256), not the MFMA pipe, is the
// expected limit; HBM: x read once and y written once per image (100 KB each).
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int NPIX = 49;                     // 7 x 7
constexpr int CX = 1024;                     // block channels
constexpr int CP = 256;                      // bottleneck channels
constexpr int XPL = NPIX * 16;               // 784: x plane bytes
constexpr int TPL = (NPIX + 1) * 16;         // 800: t1 / t2 plane bytes (t1's position 49 = zero)
constexpr int X_OFF = 0;
constexpr int T1_OFF = X_OFF + (CX / 8) * XPL;     // 100352
constexpr int T2_OFF = T1_OFF + (CP / 8) * TPL;    // 125952
constexpr int BIAS_OFF = T2_OFF + (CP / 8) * TPL;  // 151552
constexpr int BIAS_BLK = 2 * CP + CX;              // 1536 floats per block: b1 | b2 | b3
constexpr int BIAS_B = BIAS_BLK * 4;               // 6144: six 1-KiB DMA pieces
constexpr int R50C_LDS = BIAS_OFF + 2 * BIAS_B;    // 163840
// A K-step's four lane groups read four planes in one ds_read_b128, whose lane groups of one LDS cycle pair lane
// group 0 with 1 and 2 with 3: their planes must lie a multiple of 256 B apart, or a 16-B slot of one meets the
// other's (2-way conflicts on every fragment read at the natural 8-channel order).  So a K-step's 32 input channels
// are four planes spread out -- x: s + 32 lg (32 x 784 = 98 x 256), t1 / t2: s + 8 lg (8 x 800 = 25 x 256) -- and
// the weight streams are packed in the same K order (chain_r50_pack_block).
static_assert((32 * XPL) % 256 == 0 && (8 * TPL) % 256 == 0, "conflict-free plane spread");
static_assert(R50C_LDS <= 163840, "lds");
constexpr int NWV = 8;
constexpr int KS1 = CX / 32, KS2 = 9 * CP / 32, KS3 = CP / 32;  // 32, 72, 8
constexpr int NF12 = 2, NF3 = 4;                                  // n-fragments per wave: passes 1-2 / each pass-3 half
constexpr int FRAGS = KS1 * NF12 + KS2 * NF12 + 2 * KS3 * NF3;   // 272 weight fragments per wave and block
constexpr int RING = 16;                                          // register ring (fragments)
static_assert((KS1 * NF12) % RING == 0 && (KS2 * NF12) % RING == 0 && (KS3 * NF3) % RING == 0, "compile-time ring slots");

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

// the lane id recomputed where used (never hoisted or kept live across the block loop: conv_chain.hip)
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
__global__ __launch_bounds__(64 * NWV, 1) void chain_r50_kernel(Chain17Args p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x;
    if (b >= p.B) return;

    // ---- bias tables: block `blk` into slot `slot` (waves 0-5, one 1-KiB piece each)
    const uint64_t bp = (uint64_t)p.bias;
    const v4i32 br = {(int)(uint32_t)bp, (int)((bp >> 32) & 0xffff), (int)(p.nblk * BIAS_B), 0x00020000};
    auto issue_bias = [&](int blk, int slot) {
        if (wave < BIAS_B / 1024)
            dma16(br, (uint32_t)(uintptr_t)(smem + BIAS_OFF + slot * BIAS_B + wave * 1024),
                  (uint32_t)(wave * 1024 + fresh_lane() * 16), (uint32_t)(blk * BIAS_B));
    };

    // ---- x -> LDS planes: thread c = (pixel, plane): a pixel's 128 16-B pieces are contiguous in global
    const bf16_t* xb = p.x + (size_t)b * NPIX * CX;
    for (int c = threadIdx.x; c < NPIX * CX / 8; c += 64 * NWV) {
        const int px = c >> 7, pl = c & 127;
        *(uint4*)(smem + X_OFF + pl * XPL + px * 16) = *(const uint4*)(xb + (size_t)c * 8);
    }
    if (threadIdx.x < CP / 8) *(uint4*)(smem + T1_OFF + threadIdx.x * TPL + NPIX * 16) = make_uint4(0, 0, 0, 0);
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

    f32x4_t acc[NF3][4];
    frag bq[2][4];

    // passes 1 (KIND 0: 1x1 over x) and 2 (KIND 1: 3x3 over t1): n-fragments 2 wave, 2 wave + 1
    auto pass12 = [&](auto kind_tag, int g0, int slot) {
        constexpr int KIND = decltype(kind_tag)::value;
        constexpr int KS = KIND == 0 ? KS1 : KS2;
        const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
#pragma unroll
        for (int i = 0; i < NF12; ++i) {
            const float4 bs = *(const float4*)(smem + BIAS_OFF + slot * BIAS_B + (KIND * CP + 16 * (NF12 * wave + i) + 4 * lg) * 4);
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){bs.x, bs.y, bs.z, bs.w};
        }
        // B fragment j of K-step s: KIND 0 -> x plane s + 32 lg, pixel 16 j + l15; KIND 1 -> tap s / 8 (kh, kw), t1
        // plane s % 8 + 8 lg at the tap-shifted pixel (position 49, zero, outside the image or past it)
        int at[4];
        auto taps = [&](int t) {
            const int kh = t / 3 - 1, kw = t % 3 - 1;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int px = 16 * j + l15, r = px / 7, c = px - 7 * (px / 7);
                const bool ok = px < NPIX && (unsigned)(r + kh) < 7u && (unsigned)(c + kw) < 7u;
                at[j] = T1_OFF + 8 * lg * TPL + (ok ? px + 7 * kh + kw : NPIX) * 16;
            }
        };
        auto rd = [&](int s, frag (&q)[4]) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (KIND == 1) q[j] = *(const frag*)(smem + at[j] + (s & 7) * TPL);
                else q[j] = *(const frag*)(smem + X_OFF + (s + 32 * lg) * XPL + (16 * j + l15) * 16);
            }
        };
        if (KIND == 1) taps(0);
        rd(0, bq[0]);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            __builtin_amdgcn_sched_barrier(0);  // keep each step's loads in that step (the scheduler sinks them)
            if (s + 1 < KS) {
                if (KIND == 1 && (s + 1) % 8 == 0) taps((s + 1) / 8);
                rd(s + 1, bq[(s + 1) & 1]);
            }
#pragma unroll
            for (int i = 0; i < NF12; ++i) {
                const int f = NF12 * s + i;
                const frag w = wq[f % RING];
                wload(f % RING, g0 + f + RING);
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = T::mfma(w, bq[s & 1][j], acc[i][j]);
            }
        }
        // epilogue: ReLU -> storage format -> t1 (pass 1) / t2 (pass 2), pixels < 49 only.  Neither pass writes
        // what it reads, and the previous reader of the destination finished before the last pass barrier
#pragma unroll
        for (int i = 0; i < NF12; ++i) {
            const int n = NF12 * wave + i;
            char* const dst = smem + (KIND == 0 ? T1_OFF : T2_OFF) + (2 * n + (lg >> 1)) * TPL + (lg & 1) * 8 + l15 * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (16 * j + l15 < NPIX)
                    *(uint2*)(dst + 256 * j) = pack4<F16>(relu_bits(acc[i][j][0]), relu_bits(acc[i][j][1]),
                                                          relu_bits(acc[i][j][2]), relu_bits(acc[i][j][3]));
        }
        lds_barrier();
    };

    // pass 3, half h: x = relu(W3 t2 + b3 + x) for n-fragments 8 wave + 4 h .. +3.  Each lane seeds from and
    // overwrites exactly its own x values; no wave reads another's channels in this pass (the barrier comes after
    // the second half)
    auto pass3 = [&](int h, int g0, int slot) {
        const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
#pragma unroll
        for (int i = 0; i < NF3; ++i) {
            const int n = 2 * NF3 * wave + NF3 * h + i;
            const float4 bs = *(const float4*)(smem + BIAS_OFF + slot * BIAS_B + (2 * CP + 16 * n + 4 * lg) * 4);
            const char* xs = smem + X_OFF + (2 * n + (lg >> 1)) * XPL + (lg & 1) * 8 + l15 * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint2 xv = *(const uint2*)(xs + 256 * j);  // (past pixel 48: another plane's bytes, never stored)
                float f[8];
                T::unpack8(make_uint4(xv.x, xv.y, 0, 0), f);
                acc[i][j] = (f32x4_t){bs.x + f[0], bs.y + f[1], bs.z + f[2], bs.w + f[3]};
            }
        }
        auto rd = [&](int s, frag (&q)[4]) {
#pragma unroll
            for (int j = 0; j < 4; ++j) q[j] = *(const frag*)(smem + T2_OFF + (s + 8 * lg) * TPL + (16 * j + l15) * 16);
        };
        rd(0, bq[0]);
#pragma unroll
        for (int s = 0; s < KS3; ++s) {
            __builtin_amdgcn_sched_barrier(0);
            if (s + 1 < KS3) rd(s + 1, bq[(s + 1) & 1]);
#pragma unroll
            for (int i = 0; i < NF3; ++i) {
                const int f = NF3 * s + i;
                const frag w = wq[f % RING];
                wload(f % RING, g0 + f + RING);
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = T::mfma(w, bq[s & 1][j], acc[i][j]);
            }
        }
#pragma unroll
        for (int i = 0; i < NF3; ++i) {
            const int n = 2 * NF3 * wave + NF3 * h + i;
            char* const xd = smem + X_OFF + (2 * n + (lg >> 1)) * XPL + (lg & 1) * 8 + l15 * 16;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (16 * j + l15 < NPIX)
                    *(uint2*)(xd + 256 * j) = pack4<F16>(relu_bits(acc[i][j][0]), relu_bits(acc[i][j][1]),
                                                         relu_bits(acc[i][j][2]), relu_bits(acc[i][j][3]));
        }
    };

#pragma unroll 1
    for (int blk = 0; blk < p.nblk; ++blk) {
        const int slot = blk & 1;
        if (blk + 1 < p.nblk) issue_bias(blk + 1, slot ^ 1);
        const int g0 = gw + blk * FRAGS;
        pass12(std::integral_constant<int, 0>{}, g0, slot);
        pass12(std::integral_constant<int, 1>{}, g0 + KS1 * NF12, slot);
        pass3(0, g0 + (KS1 + KS2) * NF12, slot);
        pass3(1, g0 + (KS1 + KS2) * NF12 + KS3 * NF3, slot);
        lds_barrier();
    }

    // ---- x -> y (NHWC), the load's thread map
    bf16_t* yb = p.y + (size_t)b * NPIX * CX;
    for (int c = threadIdx.x; c < NPIX * CX / 8; c += 64 * NWV) {
        const int px = c >> 7, pl = c & 127;
        *(uint4*)(yb + (size_t)c * 8) = *(const uint4*)(smem + X_OFF + pl * XPL + px * 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace

bool chain_r50_supported(int H, int W, int C, int nblk) { return H == 7 && W == 7 && C == CX && nblk >= 1; }

// + RING fragments: the last wave's ring prefetches that far past its stream (the buffer offset is not range-checked)
size_t chain_r50_weight_elems(int nblk) { return ((size_t)NWV * nblk * FRAGS + RING) * 512; }

size_t chain_r50_bias_floats(int nblk) { return (size_t)nblk * BIAS_BLK; }

// One block's member convs ([Npad][Kpad] rows, K order (kh, kw, c)) into the per-wave streams: fragment = 16
// output rows x 32 K, lane (g, r) holds rows[row0 + r][kb(g) .. + 7], kb(g) = the first input channel of the plane
// lane group g reads in that K-step (the kernel's spread plane order)
void chain_r50_pack_block(const bf16_t* r1, int kp1, const bf16_t* r2, int kp2, const bf16_t* r3, int kp3, int blk,
                          int nblk, bf16_t* out) {
    auto frag = [](bf16_t* dst, const bf16_t* rows, int kp, int row0, auto kb) {
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) dst[l * 8 + e] = rows[(size_t)(row0 + (l & 15)) * kp + kb(l >> 4) + e];
    };
    for (int w = 0; w < NWV; ++w) {
        bf16_t* o = out + (size_t)(w * nblk + blk) * FRAGS * 512;
        int f = 0;
        for (int s = 0; s < KS1; ++s)  // conv1: x plane s + 32 g
            for (int i = 0; i < NF12; ++i)
                frag(o + (size_t)(f++) * 512, r1, kp1, 16 * (NF12 * w + i), [&](int g) { return 8 * (s + 32 * g); });
        for (int s = 0; s < KS2; ++s)  // conv2: tap s / 8, t1 plane s % 8 + 8 g
            for (int i = 0; i < NF12; ++i)
                frag(o + (size_t)(f++) * 512, r2, kp2, 16 * (NF12 * w + i),
                     [&](int g) { return CP * (s / 8) + 8 * (s % 8 + 8 * g); });
        for (int h = 0; h < 2; ++h)  // conv3: t2 plane s + 8 g
            for (int s = 0; s < KS3; ++s)
                for (int i = 0; i < NF3; ++i)
                    frag(o + (size_t)(f++) * 512, r3, kp3, 16 * (2 * NF3 * w + NF3 * h + i), [&](int g) { return 8 * (s + 8 * g); });
    }
}

hipError_t launch_chain_r50(const Chain17Args& a, hipStream_t s) {
    if (a.B <= 0 || a.nblk <= 0 || !a.x || !a.y || !a.w || !a.bias) return hipErrorInvalidValue;
    auto k = a.f16 ? chain_r50_kernel<true> : chain_r50_kernel<false>;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, R50C_LDS);
        attr[a.f16 ? 1 : 0] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), R50C_LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), R50C_LDS, s, a);
    return hipGetLastError();
}

}  // namespace fr
