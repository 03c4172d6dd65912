// FaceNet InceptionResnetV1 repeat_1 -- five Block35 at 17x17x256 (facenet_model.py:12-16 -> facenet_pytorch
// Block35: x0 = 1x1(x), x1 = 3x3(1x1(x)), x2 = 3x3(3x3(1x1(x))), y = relu(conv2d(cat(x0, x1, x2)) * 0.17 + x)) --
// as ONE launch.  Per conv the blocks are 25 launches of 1.4-3.6 GFLOP with 32- and 96-channel outputs: each pays a
// ramp and a tail around a few K-steps, and the 32-channel 3x3 convs fill a quarter of every MFMA tile row they
// could use (0.38 ms at bs = 256 for 57 GFLOP, profiles/r05_irv1_layer_profile.txt).  Here one workgroup owns one
// image for all five blocks; the 32-channel branch tensors live in LDS, the 256-channel block input / output goes
// through global memory (148 KB per image does not fit beside them):
//   P1  [t1 | t2 | b0] = relu(W [b1.0 | b2.0 | b0] x + b)   K 256 (8 K-steps, x fragments from global memory two
//       K-steps ahead in registers), N 96
//   P2  b1 = relu(3x3(t1) + b), t = relu(3x3(t2) + b)         K 9 taps x 32, two convs side by side
//   P3  b2 = relu(3x3(t) + b)                                  K 9 x 32
//   P4  y = relu(W' [b0 | b1 | b2] + b' + x)                   K 96, N 256 in two halves (W', b' carry the 0.17)
// * LDS tensors are plane-major ([4 planes of 8 channels][positions][16 B]: a fragment's 16 lanes read 16 positions
//   of one plane); the 3x3 inputs t1 / t2 / t are stored zero-padded (19 x 19 positions),
//   so every tap is a uniform shift of the lane's position; b2 reuses t1's buffer;
// * 8 waves: px-group (w & 3) = five 16-pixel fragments (20 fragments: 289 pixels + 31 discarded), and the upper
//   bit picks the n-fragments: P1 3 of 6, P2 the conv, P3 one of 2, P4 4 of 8 per half; weight fragments come
//   straight from global memory (L1 / L2: 150 KB per block), ahead of their pass;
// * the block outputs between blocks are stored plane-major in global memory ([32 planes][289 pixels][16 B]:
//   coalesced 16-B staging / stores); the chain input (conv2d_4b) and output (repeat_1.4, read by mixed_6a) are NHWC;
// * the same rounding points as the per-conv path (t1, t2, b0, b1, t, b2 and every block output in the storage
//   format); only the f32 summation order differs (P4 accumulates onto bias + x).
// Bounds: per image and block 2 x 289 x (256 x 96 + 3 x 288 x 32 + 96 x 256) = 44.4 MFLOP; global traffic per image
// and block: x read twice (staging, residual) and y written once (148 KB each), L2 / Infinity-Cache served.
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int SW = 17, NPX = SW * SW;      // 289
constexpr int PW = SW + 2;                 // padded width 19
constexpr int PPL = 5888;                  // padded plane: 19 x 19 = 361 positions (+ 7) x 16 B
constexpr int UPL = 5120;                  // unpadded plane: 320 pixel slots x 16 B
constexpr int TP_B = 4 * PPL;              // 25600: a padded 32-channel tensor
constexpr int TU_B = 4 * UPL;              // 20480: an unpadded one
constexpr int T1_OFF = 0;                  // t1, then b2
constexpr int T2_OFF = T1_OFF + TP_B;
constexpr int T_OFF = T2_OFF + TP_B;
constexpr int B0_OFF = T_OFF + TP_B;       // 76800
constexpr int B1_OFF = B0_OFF + TU_B;
constexpr int C35_LDS = B1_OFF + TU_B;     // 117760
static_assert(C35_LDS <= 163840, "lds");
static_assert(PW * PW <= PPL / 16 && PPL % 256 == 0, "padded plane");
constexpr int NWV = 8;

// per-block packed weights: W1 [96][256] | W21 [32][288] | W22 [32][288] | W3 [32][288] | W4 [256][96]
constexpr int W1_E = 96 * 256, W2_E = 32 * 288, W4_E = 256 * 96;
constexpr int W21_O = W1_E, W22_O = W21_O + W2_E, W3_O = W22_O + W2_E, W4_O = W3_O + W2_E;
constexpr int WBLK = W4_O + W4_E;          // 76,800 elements per block
// per-block biases: 96 | 32 | 32 | 32 | 256
constexpr int BB2A = 96, BB2B = 128, BB3 = 160, BB4 = 192, BBLK = 448;

__device__ __forceinline__ int fresh_lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

template <bool F16>
__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
    if (F16) return make_uint2(pack2_f16(a, b), pack2_f16(c, d));
    return make_uint2(pack2_bf16(a, b), pack2_bf16(c, d));
}

// padded position of pixel p (the discarded pixels >= 289 take pixel 0's: their taps stay inside the plane)
__device__ __forceinline__ int ppos(int p) {
    const int r = p / SW, c = p - r * SW;
    return p < NPX ? (r + 1) * PW + c + 1 : PW + 1;
}

template <bool F16>
__global__ __launch_bounds__(64 * NWV, 1) void chain35_kernel(Chain35Args p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int b = blockIdx.x;
    if (b >= p.B) return;
    const int pg = wave & 3, hi = wave >> 2;

    // the padded tensors' halos and guards stay zero (epilogues write interior positions only)
    for (int i = threadIdx.x; i < 3 * TP_B / 16; i += 64 * NWV) *(uint4*)(smem + T1_OFF + i * 16) = make_uint4(0, 0, 0, 0);
    __syncthreads();

    f32x4_t acc[5][5];
    const size_t img = (size_t)b * NPX * 256;

#pragma unroll 1
    for (int blk = 0; blk < p.nblk; ++blk) {
        const bf16_t* xin = p.io[blk];
        bf16_t* yout = (bf16_t*)p.io[blk + 1];
        const bool in_planar = blk > 0, out_planar = blk + 1 < p.nblk;
        const bf16_t* W = p.w + (size_t)blk * WBLK;
        const float* BI = p.bias + (size_t)blk * BBLK;
        // 3x3 over a padded 32-channel tensor: NF n-fragments (weights wt, loaded a pass ahead), the wave's five pixel
        // fragments
        auto conv3 = [&](auto nf_tag, int src_off, const frag (&wt)[9][2]) {
            constexpr int NF = decltype(nf_tag)::value;
            const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
            int pos[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) pos[j] = src_off + lg * PPL + ppos(16 * (5 * pg + j) + l15) * 16;
            frag bq[2][5];
            auto rd = [&](int t, frag (&q)[5]) {
                const int sh = ((t / 3 - 1) * PW + (t % 3 - 1)) * 16;
#pragma unroll
                for (int j = 0; j < 5; ++j) q[j] = *(const frag*)(smem + pos[j] + sh);
            };
            rd(0, bq[0]);
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                __builtin_amdgcn_sched_barrier(0);
                if (t + 1 < 9) rd(t + 1, bq[(t + 1) & 1]);
#pragma unroll
                for (int i = 0; i < NF; ++i)
#pragma unroll
                    for (int j = 0; j < 5; ++j) acc[i][j] = T::mfma(wt[t][i], bq[t & 1][j], acc[i][j]);
            }
        };
        auto relu_store = [&](int NF, int dst_off, bool padded, int n0) {
            const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
            for (int i = 0; i < NF; ++i) {
                const int pl = 2 * (n0 + i) + (lg >> 1);
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int px = 16 * (5 * pg + j) + l15;
                    if (px < NPX) {
                        const int a = dst_off + (padded ? pl * PPL + ppos(px) * 16 : pl * UPL + px * 16) + (lg & 1) * 8;
                        *(uint2*)(smem + a) = pack4<F16>(relu_bits(acc[i][j][0]), relu_bits(acc[i][j][1]),
                                                         relu_bits(acc[i][j][2]), relu_bits(acc[i][j][3]));
                    }
                }
            }
        };
        // 3x3 weights of NF n-fragments (n0 ..) of a [32][288] image: lane (lg, l15) of (tap t, i) = row 16 (n0 + i) + l15,
        // K 32 t + 8 lg
        auto load3 = [&](frag (&wt)[9][2], const bf16_t* wc, int n0, int NF) {
            const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
            const bf16_t* wl = wc + (size_t)(16 * n0 + l15) * 288 + 8 * lg;
#pragma unroll
            for (int t = 0; t < 9; ++t)
                for (int i = 0; i < NF; ++i) wt[t][i] = *(const frag*)(wl + (size_t)16 * 288 * i + 32 * t);
        };
        // P4 half h: the weights of its 4 n-fragments and the residual x at the lane's channels / pixels
        frag w4[3][4];
        uint2 rx[4][5];
        auto load4 = [&](int h) {
            const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
            const int n0 = 8 * h + 4 * hi;
            const bf16_t* wl = W + W4_O + (size_t)(16 * n0 + l15) * 96 + 8 * lg;
#pragma unroll
            for (int s = 0; s < 3; ++s)
#pragma unroll
                for (int i = 0; i < 4; ++i) w4[s][i] = *(const frag*)(wl + (size_t)16 * 96 * i + 32 * s);
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = 16 * (n0 + i) + 4 * lg;
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int px = min(16 * (5 * pg + j) + l15, NPX - 1);
                    const size_t o = in_planar ? (size_t)((n >> 3) * NPX + px) * 8 + (n & 7) : (size_t)px * 256 + n;
                    rx[i][j] = *(const uint2*)(xin + img + o);
                }
            }
        };

        frag wt[9][2];

        // ---------------- P1: [t1 | t2 | b0] = relu(W1 x + b), n-fragments 3 hi .. 3 hi + 2.  The x fragments come
        // straight from global memory (16 pixels of one 8-channel plane: 256 contiguous bytes in the plane-major
        // layout) two K-steps ahead in registers, like the weights; no LDS staging and no barrier in the K loop
        {
            const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
            float4 bs[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) bs[i] = *(const float4*)(BI + 16 * (3 * hi + i) + 4 * lg);
            const bf16_t* wl = W + (size_t)(16 * 3 * hi + l15) * 256 + 8 * lg;  // row 16 nf + l15, K 32 s + 8 lg
            // element offset of the lane's x fragment j at K-step 0 (plane lg); + 4 planes per K-step
            int xo[5];
#pragma unroll
            for (int j = 0; j < 5; ++j) {
                const int px = min(16 * (5 * pg + j) + l15, NPX - 1);  // discarded pixels re-read pixel 288
                xo[j] = in_planar ? (lg * NPX + px) * 8 : px * 256 + lg * 8;
            }
            const int xstep = in_planar ? 4 * NPX * 8 : 32;
            const bf16_t* xi = xin + img;
            frag wq[3][3], xq[3][5];
            auto ld = [&](int s, int slot) {
#pragma unroll
                for (int i = 0; i < 3; ++i) wq[slot][i] = *(const frag*)(wl + (size_t)16 * 256 * i + 32 * s);
#pragma unroll
                for (int j = 0; j < 5; ++j) xq[slot][j] = *(const frag*)(xi + xo[j] + s * xstep);
            };
            ld(0, 0);
            ld(1, 1);
#pragma unroll
            for (int i = 0; i < 3; ++i)
#pragma unroll
                for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t){bs[i].x, bs[i].y, bs[i].z, bs[i].w};
#pragma unroll
            for (int s = 0; s < 8; ++s) {
                __builtin_amdgcn_sched_barrier(0);
                if (s + 2 < 8) ld(s + 2, (s + 2) % 3);
#pragma unroll
                for (int i = 0; i < 3; ++i)
#pragma unroll
                    for (int j = 0; j < 5; ++j) acc[i][j] = T::mfma(wq[s % 3][i], xq[s % 3][j], acc[i][j]);
            }
            load3(wt, W + (hi ? W22_O : W21_O), 0, 2);  // P2's weights, in flight during this epilogue and barrier
            // epilogue: n-fragment 3 hi + i -> t1 (0, 1: padded), t2 (2, 3: padded), b0 (4, 5)
#pragma unroll
            for (int i = 0; i < 3; ++i) {
                const int nf = 3 * hi + i;
                const int tsel = nf >> 1, pl = 2 * (nf & 1) + (lg >> 1);
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int px = 16 * (5 * pg + j) + l15;
                    if (px < NPX) {
                        const int a = tsel == 2 ? B0_OFF + pl * UPL + px * 16 : (tsel == 0 ? T1_OFF : T2_OFF) + pl * PPL + ppos(px) * 16;
                        *(uint2*)(smem + a + (lg & 1) * 8) = pack4<F16>(relu_bits(acc[i][j][0]), relu_bits(acc[i][j][1]),
                                                                        relu_bits(acc[i][j][2]), relu_bits(acc[i][j][3]));
                    }
                }
            }
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }

        // ---------------- P2: b1 = relu(3x3 t1), t = relu(3x3 t2) -- waves 0-3 the first, 4-7 the second
        {
            const int ln = fresh_lane(), lg = ln >> 4;
            const float* bb = BI + (hi ? BB2B : BB2A);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const float4 v = *(const float4*)(bb + 16 * i + 4 * lg);
#pragma unroll
                for (int j = 0; j < 5; ++j) acc[i][j] = (f32x4_t){v.x, v.y, v.z, v.w};
            }
            conv3(std::integral_constant<int, 2>{}, hi ? T2_OFF : T1_OFF, wt);
            load3(wt, W + W3_O, hi, 1);  // P3's weights, in flight during this epilogue and barrier
            if (hi) relu_store(2, T_OFF, true, 0);
            else relu_store(2, B1_OFF, false, 0);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        // ---------------- P3: b2 = relu(3x3 t) into t1's buffer; n-fragment hi
        {
            const int ln = fresh_lane(), lg = ln >> 4;
            const float4 v = *(const float4*)(BI + BB3 + 16 * hi + 4 * lg);
#pragma unroll
            for (int j = 0; j < 5; ++j) acc[0][j] = (f32x4_t){v.x, v.y, v.z, v.w};
            conv3(std::integral_constant<int, 1>{}, T_OFF, wt);
            load4(0);
            relu_store(1, T1_OFF, true, hi);
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        // ---------------- P4: y = relu(W4 [b0 | b1 | b2] + b + x), two halves of 128 channels, 4 n-fragments per wave
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int ln = fresh_lane(), l15 = ln & 15, lg = ln >> 4;
            const int n0 = 8 * h + 4 * hi;
            // seeds: bias + the residual x at the lane's 4 channels of each of its pixels
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const float4 v = *(const float4*)(BI + BB4 + 16 * (n0 + i) + 4 * lg);
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    float f[8];
                    T::unpack8(make_uint4(rx[i][j].x, rx[i][j].y, 0, 0), f);
                    acc[i][j] = (f32x4_t){v.x + f[0], v.y + f[1], v.z + f[2], v.w + f[3]};
                }
            }
#pragma unroll
            for (int s = 0; s < 3; ++s) {
                frag bq[5];
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int px = 16 * (5 * pg + j) + l15;
                    const int a = s == 0 ? B0_OFF + lg * UPL + px * 16
                                         : (s == 1 ? B1_OFF + lg * UPL + px * 16 : T1_OFF + lg * PPL + ppos(px) * 16);
                    bq[j] = *(const frag*)(smem + a);
                }
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 5; ++j) acc[i][j] = T::mfma(w4[s][i], bq[j], acc[i][j]);
            }
            if (h == 0) load4(1);  // the second half's weights and residual, in flight during these stores
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = 16 * (n0 + i) + 4 * lg;
#pragma unroll
                for (int j = 0; j < 5; ++j) {
                    const int px = 16 * (5 * pg + j) + l15;
                    if (px < NPX) {
                        const size_t o = out_planar ? (size_t)((n >> 3) * NPX + px) * 8 + (n & 7) : (size_t)px * 256 + n;
                        *(uint2*)(yout + img + o) = pack4<F16>(relu_bits(acc[i][j][0]), relu_bits(acc[i][j][1]),
                                                               relu_bits(acc[i][j][2]), relu_bits(acc[i][j][3]));
                    }
                }
            }
        }
        // the block output is complete in global memory before any wave stages it as the next block's input
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
}

}  // namespace

bool chain35_supported(int H, int W, int C, int nblk) { return H == SW && W == SW && C == 256 && nblk >= 1 && nblk <= 8; }
size_t chain35_weight_elems(int nblk) { return (size_t)nblk * WBLK; }
size_t chain35_bias_floats(int nblk) { return (size_t)nblk * BBLK; }

// One block's member convs ([Npad][Kpad] rows, K order (kh, kw, c)) into the compact per-block image
void chain35_pack_block(const bf16_t* r1, int kp1, const bf16_t* r21, int kp21, const bf16_t* r22, int kp22,
                        const bf16_t* r3, int kp3, const bf16_t* r4, int kp4, int blk, bf16_t* out) {
    bf16_t* o = out + (size_t)blk * WBLK;
    auto copy = [](bf16_t* dst, const bf16_t* rows, int kp, int n, int k) {
        for (int r = 0; r < n; ++r)
            for (int c = 0; c < k; ++c) dst[(size_t)r * k + c] = rows[(size_t)r * kp + c];
    };
    copy(o, r1, kp1, 96, 256);
    copy(o + W21_O, r21, kp21, 32, 288);
    copy(o + W22_O, r22, kp22, 32, 288);
    copy(o + W3_O, r3, kp3, 32, 288);
    copy(o + W4_O, r4, kp4, 256, 96);
}

// per-block bias table: [P1 96 | branch1.1 32 | branch2.1 32 | branch2.2 32 | conv2d 256]
void chain35_pack_bias(const float* b1, const float* b21, const float* b22, const float* b3, const float* b4, int blk,
                       float* out) {
    float* o = out + (size_t)blk * BBLK;
    for (int i = 0; i < 96; ++i) o[i] = b1[i];
    for (int i = 0; i < 32; ++i) o[BB2A + i] = b21[i];
    for (int i = 0; i < 32; ++i) o[BB2B + i] = b22[i];
    for (int i = 0; i < 32; ++i) o[BB3 + i] = b3[i];
    for (int i = 0; i < 256; ++i) o[BB4 + i] = b4[i];
}

hipError_t launch_chain35(const Chain35Args& a, hipStream_t s) {
    if (a.B <= 0 || a.nblk <= 0 || a.nblk > 8 || !a.w || !a.bias) return hipErrorInvalidValue;
    for (int i = 0; i <= a.nblk; ++i)
        if (!a.io[i]) return hipErrorInvalidValue;
    auto k = a.f16 ? chain35_kernel<true> : chain35_kernel<false>;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, C35_LDS);
        attr[a.f16 ? 1 : 0] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), C35_LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), C35_LDS, s, a);
    return hipGetLastError();
}

}  // namespace fr
