// ResNet-50 ArcFace layer1.1 and layer1.2 -- torchvision Bottlenecks at 28x28x256 (arcface_model.py:118-132; y =
// relu_bits(bn3(conv3(relu_bits(bn2(conv2(relu_bits(bn1(conv1(x)))))))) + x), conv1 1x1 256 -> 64, conv2 3x3 64 -> 64, conv3 1x1
// 64 -> 256) -- one launch per block.  As per-conv launches each block is ~111 us at bs = 256
// (profiles/r06_r50_layer_profile.txt: 31 + 35 + 47 us): conv1 reads and conv3 writes the 103 MB 256-channel tensors and
// conv3 reads the residual again, and the 64-channel intermediates make two more HBM round trips.  Here one workgroup
// owns one image and walks down it row by row, so only the block input (read once) and output (written once) touch
// HBM:
//   * software-pipelined rows, ONE barrier per phase: phase r runs conv1 of x row r + 2 (into a 4-row ring of t1 rows
//     with zero halo columns; a zero row stands in for the rows outside the image), conv2 of row r (t1 rows r - 1 ..
//     r + 1, into a 2-row t2 ring) and conv3 of row r - 1 onto bias + the residual x row r - 1 (into a 2-row NHWC
//     staging ring) -- three independent accumulator chains per wave, interleaved K-step by K-step -- after the
//     coalesced 16-B stores of row r - 2 from the staging ring;
//   * x rows arrive by LDS-DMA into a 6-row ring two phases ahead (inline asm, hidden from the compiler's waitcnt
//     pass; counted vmcnt waits per phase; past the image a dummy row keeps the count fixed);
//   * ALL weights live in registers for the whole kernel (34 fragments = 136 VGPRs per wave: wave w computes pixel
//     fragment w >> 2 of the row -- 28 pixels in two 16-pixel fragments -- and output channels 16 (w & 3) .. of
//     conv1 / conv2, 64 (w & 3) .. of conv3);
//   * x rows are stored plane-major ([32 planes of 8 channels][28 pixels][16 B]); conv1's K-step s reads planes
//     s + 8 lg (lane group lg), 8 planes = 3584 B apart, a multiple of 256 B, so the lane groups that share an LDS
//     cycle never meet (the weights are packed in that K order); t1 / t2 planes are 512 B;
//   * the same rounding points as the per-conv path (t1, t2 and the block output in the storage format); only the f32
//     summation order differs (conv3 accumulates onto bias + x).
// Bounds: per image 2 x 784 x 69,632 = 109 MFLOP against 802 KB of HBM traffic (x + y): at bs = 256
// 206 MB per launch, the HBM stream, not the MFMA pipe (28 GFLOP), is the expected limit.
#include "kernels.h"

#include <hip/hip_ext.h>

#include <type_traits>

namespace fr {
namespace {

constexpr int IW = 28;                     // image width / height
constexpr int CX = 256, CP = 64;           // block output / bottleneck channels
constexpr int TPL = 32 * 16;               // 512: t1 / t2 plane bytes (32 positions)
constexpr int TROW = (CP / 8) * TPL;       // 4096
constexpr int YROW = IW * CX * 2;          // 14336: one output row
constexpr int XR = 6;                      // x ring rows (7, three phases ahead, measured slower)
constexpr int NWV = 8;
constexpr int YPIECES = YROW / 16;         // 896 16-B pieces per output row

// DS = false: layer1.1 / 1.2 (x = the 256-channel block input, the residual added onto conv3); DS = true: layer1.0
// (x = the 64-channel maxpool output; conv3's K is [t2 64 | x 64], the downsample K-concatenated as in the per-conv
// plan, no residual add)
template <bool DS>
struct Geo {
    static constexpr int CIN = DS ? 64 : 256;
    static constexpr int XPL = DS ? 512 : IW * 16;        // x plane bytes: 448, or 512 with 4 pad positions (DS)
    static constexpr int XROW = (CIN / 8) * XPL;          // 14336 / 4096
    static constexpr int KS1 = CIN / 32;                  // conv1 K-steps: 8 / 2
    static constexpr int KS3 = DS ? 4 : 2;                // conv3 K-steps
    static constexpr int NFR = KS1 + 18 + 4 * KS3;        // weight fragments per wave: 34 / 36
    static constexpr int NDMA = XROW / 1024;              // DMA instructions per x row: 14 / 4
    static constexpr int X_OFF = 0;
    static constexpr int T1_OFF = X_OFF + XR * XROW;      // t1 rows (slots 0-3) + the zero row (slot 4)
    static constexpr int T2_OFF = T1_OFF + 5 * TROW;      // 2 t2 rows
    static constexpr int Y_OFF = T2_OFF + 2 * TROW;       // 2 output rows, NHWC, 16-B chunks XOR-swizzled by the pixel
    static constexpr int LDS = Y_OFF + 2 * YROW;          // 143360 / 67584
    // conv1's K-step s reads x plane s + 8 lg (8 planes = 3584 B apart) or, on 512-B planes, 4 s + lg
    __device__ static int plane1(int s, int lg) { return DS ? 4 * s + lg : s + 8 * lg; }
    static int kb1(int s, int g) { return 8 * (DS ? 4 * s + g : s + 8 * g); }
    static_assert((8 * (IW * 16)) % 256 == 0 && TPL % 256 == 0 && (DS ? XPL % 256 == 0 : true), "conflict-free planes");
    static_assert(XROW % 1024 == 0 && LDS <= 160 * 1024, "DMA split / LDS");
};

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

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool F16>
__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
    if (F16) return make_uint2(pack2_f16(a, b), pack2_f16(c, d));
    return make_uint2(pack2_bf16(a, b), pack2_bf16(c, d));
}

// Phase r waits for x row r + 2 (issued in phase r - 2, rows 0 / 1 before the loop).  VMEM ops per phase, in issue
// order: D DMA instructions (the row r + 4; waves 0-5: two of the 14, 6-7: one), then S stores of row r - 2 when
// r >= 2 (waves 0-5: two 16-B pieces per thread, 6-7: one).  Younger than row r + 2's DMA: phases -2 .. 2 -> the
// next DMA only; 3 -> + phase 2's stores; >= 4 -> + phases r - 2 and r - 1's stores.
template <int D, int S>
__device__ __forceinline__ void wait_row(int r) {
    if (r >= 4) wait_vm<D + 2 * S>();
    else if (r == 3) wait_vm<D + S>();
    else wait_vm<D>();
}

template <bool F16, bool DS>
__global__ __launch_bounds__(64 * NWV, 1) void bneck28_kernel(Chain17Args p) {
    typedef Geo<DS> G;
    constexpr int XPL = G::XPL, XROW = G::XROW, KS1 = G::KS1, KS3 = G::KS3, NFR = G::NFR;
    constexpr int X_OFF = G::X_OFF, T1_OFF = G::T1_OFF, T2_OFF = G::T2_OFF, Y_OFF = G::Y_OFF;
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, l15 = lane & 15, lg = lane >> 4;
    const int b = blockIdx.x;
    if (b >= p.B) return;
    const int P = wave >> 2, q = wave & 3;  // pixel fragment, channel quarter
    const int px = 16 * P + l15;            // the lane's pixel (>= 28: a discarded MFMA column)
    const bool pv = px < IW;

    // t1 (all slots: halos, the zero row) starts zero; epilogues write interior positions only
    for (int i = threadIdx.x; i < 5 * TROW / 16; i += 64 * NWV) *(uint4*)(smem + T1_OFF + i * 16) = make_uint4(0, 0, 0, 0);

    // ---- weights (this wave's 34 / 36 fragments) and biases, into registers once (issued before the first x rows:
    // the first row wait covers them)
    const frag* wp = (const frag*)p.w + (size_t)q * NFR * 64 + lane;
    frag w1[KS1], w2[18], w3[KS3][4];
#pragma unroll
    for (int s = 0; s < KS1; ++s) w1[s] = wp[64 * s];
#pragma unroll
    for (int s = 0; s < 18; ++s) w2[s] = wp[64 * (KS1 + s)];
#pragma unroll
    for (int s = 0; s < KS3; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) w3[s][i] = wp[64 * (KS1 + 18 + 4 * s + i)];
    const float4 b1 = *(const float4*)(p.bias + 16 * q + 4 * lg), b2 = *(const float4*)(p.bias + 64 + 16 * q + 4 * lg);
    float4 b3[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b3[i] = *(const float4*)(p.bias + 128 + 16 * (4 * q + i) + 4 * lg);

    // ---- x row DMA, instruction k = the row's LDS bytes 1024 k ..: 256 channels -- k = 0..13, pieces 64 k .. + 63
    // (piece = plane * 28 + pixel), wave w issues k = w and k = w + 8 (< 14); 64 channels -- k = 0..3, planes 2 k and
    // 2 k + 1 at 32 positions (positions 28-31 repeat pixel 27), waves 0-3 one each
    constexpr int CIN = G::CIN;
    const uint64_t xp = (uint64_t)p.x;
    const v4i32 xr = {(int)(uint32_t)xp, (int)((xp >> 32) & 0xffff), (int)((size_t)p.B * IW * IW * CIN * 2), 0x00020000};
    auto piece_src = [&](int k) {
        if (DS) {
            const int pl = 2 * k + (lane >> 5), x = min(lane & 31, IW - 1);
            return (uint32_t)(x * CIN * 2 + pl * 16);
        }
        const int pc = 64 * k + lane, pl = pc / IW, x = pc - pl * IW;
        return (uint32_t)(x * CIN * 2 + pl * 16);
    };
    const uint32_t src0 = piece_src(DS ? (wave & 3) : wave), src1 = piece_src(wave + 8 < 14 ? wave + 8 : wave);
    auto dma_row = [&](int row) {  // rows past the image re-read the last one (a dummy keeping the VMEM count fixed)
        const int rr = row < IW ? row : IW - 1;
        const uint32_t so = (uint32_t)(((size_t)b * IW + rr) * IW * CIN * 2);
        char* const dst = smem + X_OFF + (row % XR) * XROW;
        if (DS) {
            if (wave < 4) dma16(xr, (uint32_t)(uintptr_t)(dst + 1024 * wave), src0, so);
            return;
        }
        dma16(xr, (uint32_t)(uintptr_t)(dst + 1024 * wave), src0, so);
        if (wave + 8 < 14) dma16(xr, (uint32_t)(uintptr_t)(dst + 1024 * (wave + 8)), src1, so);
    };
    dma_row(0);
    dma_row(1);

    const uint32_t ysw = (uint32_t)(px & 31);  // the staging rows' chunk swizzle of the lane's pixel
    auto store_row = [&](int row) {  // staging slot row % 2 -> y row: 896 16-B pieces; thread t stores t and t + 512
        bf16_t* yr = p.y + ((size_t)b * IW + row) * IW * CX;
        const char* st = smem + Y_OFF + (row & 1) * YROW;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = threadIdx.x + 512 * u;
            if (k < YPIECES) {
                const int x = k >> 5, c = k & 31;
                *(uint4*)(yr + (size_t)k * 8) = *(const uint4*)(st + x * 512 + ((c ^ (x & 31)) << 4));
            }
        }
    };
    auto t1_slot = [](int row) { return (unsigned)row < (unsigned)IW ? row & 3 : 4; };

    // one phase: conv1 of row r + 2 (C1), conv2 of row r (C2), conv3 of row r - 1 (C3)
    auto phase = [&](auto c1_tag, auto c2_tag, auto c3_tag, int r) {
        constexpr bool C1 = decltype(c1_tag)::value, C2 = decltype(c2_tag)::value, C3 = decltype(c3_tag)::value;
        if (DS) {  // (waves 4-7 issue no DMA)
            if (wave < 4) wait_row<1, 2>(r);
        } else if (wave < 6) {
            wait_row<2, 2>(r);
        } else {
            wait_row<1, 1>(r);
        }
        lds_barrier();  // x row r + 2 landed; t1 row r + 1, t2 row r - 1 and staging row r - 2 complete; the slots
                        // written below were last read in phase r - 1
        dma_row(r + 4);  // into the slot of row r - 2 (last read by phase r - 1's conv3)

        const int a = r + 2, c = r - 1;
        const char* xs1 = smem + X_OFF + (C1 ? a % XR : 0) * XROW + px * 16;  // (+ plane * XPL)
        const char* ts[3];
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) ts[kh] = smem + T1_OFF + t1_slot(r + kh - 1) * TROW + lg * TPL + px * 16;
        const char* t2s = smem + T2_OFF + (C3 ? c & 1 : 0) * TROW + lg * TPL + px * 16;
        const char* xs3 = smem + X_OFF + (C3 ? c % XR : 0) * XROW + lg * XPL + px * 16;  // (DS: conv3's x K-steps)

        f32x4_t a1 = (f32x4_t){b1.x, b1.y, b1.z, b1.w}, a2 = (f32x4_t){b2.x, b2.y, b2.z, b2.w}, a3[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) a3[i] = (f32x4_t){b3[i].x, b3[i].y, b3[i].z, b3[i].w};
        if (C3 && !DS) {
            const char* xs = smem + X_OFF + (c % XR) * XROW + px * 16 + (lg & 1) * 8;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint2 xv = *(const uint2*)(xs + (2 * (4 * q + i) + (lg >> 1)) * XPL);  // (px >= 28: never stored)
                float f[8];
                T::unpack8(make_uint4(xv.x, xv.y, 0, 0), f);
                a3[i] += (f32x4_t){f[0], f[1], f[2], f[3]};
            }
        }
        // K-step k: conv2 step k (tap k / 2, channel half k % 2), conv1 step k (< KS1), conv3 step k (< KS3: t2, then
        // DS: x)
        auto rd = [&](int k, frag& f1, frag& f2, frag& f3) {
            if (C2) {
                const int t = k >> 1, kh = t / 3, kw = t - 3 * kh;
                f2 = *(const frag*)(ts[kh] + 4 * (k & 1) * TPL + kw * 16);
            }
            if (C1 && k < KS1) f1 = *(const frag*)(xs1 + G::plane1(k, lg) * XPL);
            if (C3 && k < KS3) f3 = *(const frag*)(k < 2 ? t2s + 4 * k * TPL : xs3 + 4 * (k - 2) * XPL);
        };
        // fragments read PD steps ahead; row r - 2's stores issue once the MFMAs run (step 1)
        constexpr int PD = 2, NB = PD + 1;
        frag f1[NB], f2[NB], f3[NB];
        constexpr int KS = C2 ? 18 : (C1 && KS1 > KS3) || !C3 ? KS1 : KS3;
#pragma unroll
        for (int k = 0; k < PD; ++k) rd(k, f1[k], f2[k], f3[k]);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            __builtin_amdgcn_sched_barrier(0);  // keep each step's loads in that step
            if (k + PD < KS) rd(k + PD, f1[(k + PD) % NB], f2[(k + PD) % NB], f3[(k + PD) % NB]);
            if (k == 1 && r >= 2) store_row(r - 2);
            if (C3 && k < KS3) {
#pragma unroll
                for (int i = 0; i < 4; ++i) a3[i] = T::mfma(w3[k][i], f3[k % NB], a3[i]);
            }
            if (C1 && k < KS1) a1 = T::mfma(w1[k], f1[k % NB], a1);
            if (C2) a2 = T::mfma(w2[k], f2[k % NB], a2);
        }
        __builtin_amdgcn_sched_barrier(0);
        // epilogues (pixels < 28): t1 row a (position px + 1), t2 row r, staging row c
        if (pv) {
            if (C1)
                *(uint2*)(smem + T1_OFF + (a & 3) * TROW + (2 * q + (lg >> 1)) * TPL + (px + 1) * 16 + (lg & 1) * 8) =
                    pack4<F16>(relu_bits(a1[0]), relu_bits(a1[1]), relu_bits(a1[2]), relu_bits(a1[3]));
            if (C2)
                *(uint2*)(smem + T2_OFF + (r & 1) * TROW + (2 * q + (lg >> 1)) * TPL + px * 16 + (lg & 1) * 8) =
                    pack4<F16>(relu_bits(a2[0]), relu_bits(a2[1]), relu_bits(a2[2]), relu_bits(a2[3]));
            if (C3) {
                char* const st = smem + Y_OFF + (c & 1) * YROW + px * 512;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t ch = 16 * (4 * q + i) + 4 * lg;  // 4 channels: chunk ch / 8, half (ch & 4)
                    *(uint2*)(st + (((ch >> 3) ^ ysw) << 4) + (ch & 4) * 2) =
                        pack4<F16>(relu_bits(a3[i][0]), relu_bits(a3[i][1]), relu_bits(a3[i][2]), relu_bits(a3[i][3]));
                }
            }
        }
    };
    typedef std::true_type Y;
    typedef std::false_type N;
    phase(Y{}, N{}, N{}, -2);
    phase(Y{}, N{}, N{}, -1);
    phase(Y{}, Y{}, N{}, 0);
#pragma unroll 1
    for (int r = 1; r <= IW - 3; ++r) phase(Y{}, Y{}, Y{}, r);
    phase(N{}, Y{}, Y{}, IW - 2);
    phase(N{}, Y{}, Y{}, IW - 1);
    phase(N{}, N{}, Y{}, IW);
    lds_barrier();  // staging row 27 complete
    store_row(IW - 1);
    wait_vm<0>();  // (the dummy DMA rows too) -- nothing in flight when the workgroup ends
}

}  // namespace

bool bneck28_supported(int H, int W, int C, int P) { return H == IW && W == IW && C == CX && P == CP; }

size_t bneck28_block_elems(bool ds) { return (size_t)4 * (ds ? Geo<true>::NFR : Geo<false>::NFR) * 512; }

// One block's member convs ([Npad][Kpad] rows, K order (kh, kw, c); ds: conv3's rows [t2 64 | x 64]) into its
// per-quarter register images [quarter q][34 / 36 fragments][64 lanes][8]; fragment = 16 output rows x 32 K, lane
// (g, r) holds rows[row0 + r][kb(g) .. + 7] (conv1, 256 channels: x planes s + 8 g, the kernel's spread order)
void bneck28_pack_block(const bf16_t* r1, int kp1, const bf16_t* r2, int kp2, const bf16_t* r3, int kp3, bool ds,
                        bf16_t* out) {
    auto frag = [](bf16_t* dst, const bf16_t* rows, int kp, int row0, auto kb) {
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) dst[l * 8 + e] = rows[(size_t)(row0 + (l & 15)) * kp + kb(l >> 4) + e];
    };
    const int ks1 = ds ? Geo<true>::KS1 : Geo<false>::KS1, ks3 = ds ? Geo<true>::KS3 : Geo<false>::KS3;
    const int nfr = ds ? Geo<true>::NFR : Geo<false>::NFR;
    for (int q = 0; q < 4; ++q) {
        bf16_t* o = out + (size_t)q * nfr * 512;
        int f = 0;
        for (int s = 0; s < ks1; ++s)
            frag(o + (size_t)(f++) * 512, r1, kp1, 16 * q, [&](int g) { return ds ? Geo<true>::kb1(s, g) : Geo<false>::kb1(s, g); });
        for (int s = 0; s < 18; ++s) frag(o + (size_t)(f++) * 512, r2, kp2, 16 * q, [&](int g) { return 32 * s + 8 * g; });
        for (int s = 0; s < ks3; ++s)
            for (int i = 0; i < 4; ++i)
                frag(o + (size_t)(f++) * 512, r3, kp3, 16 * (4 * q + i), [&](int g) { return 32 * s + 8 * g; });
    }
}

// a.w / a.bias: this block's images and its [conv1 64 | conv2 64 | conv3 256] biases
hipError_t launch_bneck28(const Chain17Args& a, bool ds, hipStream_t s) {
    if (a.B <= 0 || !a.x || !a.y || !a.w || !a.bias) return hipErrorInvalidValue;
    if ((size_t)a.B * IW * IW * (ds ? Geo<true>::CIN : Geo<false>::CIN) * 2 >= 0x80000000ull)
        return hipErrorInvalidValue;  // the x DMA's buffer offsets are 31-bit
    auto k = ds ? (a.f16 ? bneck28_kernel<true, true> : bneck28_kernel<false, true>)
                : (a.f16 ? bneck28_kernel<true, false> : bneck28_kernel<false, false>);
    const int lds = ds ? Geo<true>::LDS : Geo<false>::LDS;
    static bool attr[4] = {false, false, false, false};
    const int ai = (ds ? 2 : 0) + (a.f16 ? 1 : 0);
    if (!attr[ai]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr[ai] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), lds, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), lds, s, a);
    return hipGetLastError();
}

}  // namespace fr
