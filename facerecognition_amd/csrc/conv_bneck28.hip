// ResNet-50 ArcFace layer1.1 and layer1.2 -- torchvision Bottlenecks at 28x28x256 (arcface_model.py:118-132; y =
// relu(bn3(conv3(relu(bn2(conv2(relu(bn1(conv1(x)))))))) + x), conv1 1x1 256 -> 64, conv2 3x3 64 -> 64, conv3 1x1
// 64 -> 256) -- one launch per block.  As per-conv launches each block is ~111 us at bs = 256
// (profiles/r06_r50_layer_profile.txt: 31 + 35 + 47 us): conv1 reads and conv3 writes the 103 MB 256-channel tensors and
// conv3 reads the residual again, and the 64-channel intermediates make two more HBM round trips.  Here one workgroup
// owns one image and walks down it row by row, so only the block input (read once) and output (written once) touch
// HBM:
//   * phase r: conv1 of x row r + 1 into a 3-row ring of t1 rows (zero halo columns; a zero row stands in for the
//     rows outside the image), conv2 of output row r from t1 rows r - 1 .. r + 1, conv3 of row r onto bias + the
//     residual x row r into an LDS staging row, then the row's coalesced 16-B stores; four barriers per phase;
//   * x rows arrive by LDS-DMA into a 4-row ring three phases ahead (inline asm, hidden from the compiler's waitcnt
//     pass; counted vmcnt waits per phase: every phase issues the same VMEM ops, past the image a dummy row);
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

namespace fr {
namespace {

constexpr int IW = 28;                     // image width / height
constexpr int CX = 256, CP = 64;           // block / bottleneck channels
constexpr int XPL = IW * 16;               // 448: x plane bytes (one row)
constexpr int XROW = (CX / 8) * XPL;       // 14336: one x row
constexpr int TPL = 32 * 16;               // 512: t1 / t2 plane bytes (32 positions)
constexpr int TROW = (CP / 8) * TPL;       // 4096
constexpr int X_OFF = 0;                   // 4 x rows
constexpr int T1_OFF = X_OFF + 4 * XROW;   // 57344: t1 rows (slots 0-2) + the zero row (slot 3)
constexpr int T2_OFF = T1_OFF + 4 * TROW;  // 73728
constexpr int Y_OFF = T2_OFF + TROW;       // 77824: the output row, NHWC, 16-B chunks XOR-swizzled by the pixel
constexpr int BN28_LDS = Y_OFF + XROW;     // 92160
constexpr int NWV = 8;
constexpr int NFR = 8 + 18 + 8;            // weight fragments per wave: conv1 8 K-steps, conv2 18, conv3 2 x 4
constexpr int XPIECES = XROW / 16;         // 896 16-B pieces per row = 14 DMA instructions
static_assert((8 * XPL) % 256 == 0 && TPL % 256 == 0, "conflict-free planes");
static_assert(XPIECES == 14 * 64, "DMA split");

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

// VMEM ops a wave issues per phase: D DMA instructions (waves 0-5: two of the 14, 6-7: one) and S row stores
// (waves 0-5: two 16-B pieces per thread, 6-7: one)
template <int D, int S>
struct Waits {
    static constexpr int OPS = D + S;
    __device__ static void before_row0() { wait_vm<3 * D>(); }                   // rows 1-3 may stay in flight
    __device__ static void before(int r) {                                      // phase r needs x row r + 1
        if (r >= 3) wait_vm<S + 2 * OPS>();
        else if (r == 2) wait_vm<2 * OPS>();
        else if (r == 1) wait_vm<D + OPS>();
        else wait_vm<2 * D>();
    }
};

template <bool F16>
__global__ __launch_bounds__(64 * NWV, 1) void bneck28_kernel(Chain17Args p) {
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
    for (int i = threadIdx.x; i < 4 * TROW / 16; i += 64 * NWV) *(uint4*)(smem + T1_OFF + i * 16) = make_uint4(0, 0, 0, 0);

    // ---- weights (this wave's 34 fragments) and biases, into registers once
    const frag* wp = (const frag*)p.w + (size_t)(blockIdx.y * 4 + q) * NFR * 64 + lane;
    frag w1[8], w2[18], w3[2][4];
#pragma unroll
    for (int s = 0; s < 8; ++s) w1[s] = wp[64 * s];
#pragma unroll
    for (int s = 0; s < 18; ++s) w2[s] = wp[64 * (8 + s)];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) w3[s][i] = wp[64 * (26 + 4 * s + i)];
    const float* bb = p.bias + (size_t)blockIdx.y * 384;
    const float4 b1 = *(const float4*)(bb + 16 * q + 4 * lg), b2 = *(const float4*)(bb + 64 + 16 * q + 4 * lg);
    float4 b3[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b3[i] = *(const float4*)(bb + 128 + 16 * (4 * q + i) + 4 * lg);
    // (issued before the first x rows: the row-0 wait below covers them)


    // ---- x row DMA: instruction k (0..13) = pieces 64 k .. 64 k + 63 (piece = plane * 28 + pixel); wave w issues k = w
    // and k = w + 8 (< 14)
    const uint64_t xp = (uint64_t)p.x;
    const v4i32 xr = {(int)(uint32_t)xp, (int)((xp >> 32) & 0xffff), (int)min((size_t)0x7fffffff, (size_t)p.B * IW * IW * CX * 2),
                      0x00020000};
    auto piece_src = [&](int k) {
        const int pc = 64 * k + lane, pl = pc / IW, x = pc - pl * IW;
        return (uint32_t)(x * CX * 2 + pl * 16);
    };
    const uint32_t src0 = piece_src(wave), src1 = piece_src(wave + 8 < 14 ? wave + 8 : wave);
    auto dma_row = [&](int row) {  // rows past the image re-read the last one (a dummy keeping the VMEM count fixed)
        const int rr = row < IW ? row : IW - 1;
        const uint32_t so = (uint32_t)(((size_t)b * IW + rr) * IW * CX * 2);
        char* const dst = smem + X_OFF + (row & 3) * XROW;
        dma16(xr, (uint32_t)(uintptr_t)(dst + 1024 * wave), src0, so);
        if (wave + 8 < 14) dma16(xr, (uint32_t)(uintptr_t)(dst + 1024 * (wave + 8)), src1, so);
    };
#pragma unroll
    for (int r = 0; r < 4; ++r) dma_row(r);


    // conv1 of x row `row` (< 28) into t1 slot row % 3
    auto conv1 = [&](int row) {
        f32x4_t acc = (f32x4_t){b1.x, b1.y, b1.z, b1.w};
        const char* xs = smem + X_OFF + (row & 3) * XROW + px * 16;
#pragma unroll
        for (int s = 0; s < 8; ++s) acc = T::mfma(w1[s], *(const frag*)(xs + (s + 8 * lg) * XPL), acc);
        if (pv)
            *(uint2*)(smem + T1_OFF + (row % 3) * TROW + (2 * q + (lg >> 1)) * TPL + (px + 1) * 16 + (lg & 1) * 8) =
                pack4<F16>(fmaxf(acc[0], 0.f), fmaxf(acc[1], 0.f), fmaxf(acc[2], 0.f), fmaxf(acc[3], 0.f));
    };
    const uint32_t ysw = (uint32_t)(px & 31);  // the staging row's chunk swizzle of the lane's pixel

    Waits<2, 2> wa;
    Waits<1, 1> wb;
    if (wave < 6) wa.before_row0(); else wb.before_row0();
    lds_barrier();  // row 0 landed everywhere; t1 zeroed
    conv1(0);

#pragma unroll 1
    for (int r = 0; r < IW; ++r) {
        if (wave < 6) wa.before(r); else wb.before(r);
        lds_barrier();  // x row r + 1 landed everywhere; t1 row r (and r - 1) complete
        if (r + 1 < IW) conv1(r + 1);
        lds_barrier();  // t1 row r + 1 complete
        // conv2 of row r: tap (kh, kw), channel half c: K-step 2 (3 kh + kw) + c; rows outside the image read the zero row
        {
            f32x4_t acc = (f32x4_t){b2.x, b2.y, b2.z, b2.w};
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) {
                const int row = r + kh - 1;
                const int slot = (unsigned)row < (unsigned)IW ? row % 3 : 3;
                const char* ts = smem + T1_OFF + slot * TROW + lg * TPL + px * 16;
#pragma unroll
                for (int kw = 0; kw < 3; ++kw)
#pragma unroll
                    for (int c = 0; c < 2; ++c)
                        acc = T::mfma(w2[2 * (3 * kh + kw) + c], *(const frag*)(ts + 4 * c * TPL + kw * 16), acc);
            }
            if (pv)
                *(uint2*)(smem + T2_OFF + (2 * q + (lg >> 1)) * TPL + px * 16 + (lg & 1) * 8) =
                    pack4<F16>(fmaxf(acc[0], 0.f), fmaxf(acc[1], 0.f), fmaxf(acc[2], 0.f), fmaxf(acc[3], 0.f));
        }
        lds_barrier();  // t2 row r complete
        // conv3 of row r onto bias + the residual x row r, into the staging row
        {
            f32x4_t acc[4];
            const char* xs = smem + X_OFF + (r & 3) * XROW + px * 16 + (lg & 1) * 8;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const uint2 xv = *(const uint2*)(xs + (2 * (4 * q + i) + (lg >> 1)) * XPL);  // (px >= 28: never stored)
                float f[8];
                T::unpack8(make_uint4(xv.x, xv.y, 0, 0), f);
                acc[i] = (f32x4_t){b3[i].x + f[0], b3[i].y + f[1], b3[i].z + f[2], b3[i].w + f[3]};
            }
#pragma unroll
            for (int s = 0; s < 2; ++s) {
                const frag bq = *(const frag*)(smem + T2_OFF + (4 * s + lg) * TPL + px * 16);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[i] = T::mfma(w3[s][i], bq, acc[i]);
            }
            if (pv) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t ch = 16 * (4 * q + i) + 4 * lg;  // 4 channels: chunk ch / 8, half (ch & 4)
                    *(uint2*)(smem + Y_OFF + px * 512 + (((ch >> 3) ^ ysw) << 4) + (ch & 4) * 2) =
                        pack4<F16>(fmaxf(acc[i][0], 0.f), fmaxf(acc[i][1], 0.f), fmaxf(acc[i][2], 0.f), fmaxf(acc[i][3], 0.f));
                }
            }
        }
        lds_barrier();  // staging row r complete; x row r consumed (its slot takes row r + 4)
        dma_row(r + 4);
        // row r -> y: 896 16-B pieces, contiguous in global; thread t stores pieces t and t + 512
        bf16_t* yr = p.y + ((size_t)b * IW + r) * IW * CX;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int k = threadIdx.x + 512 * u;
            if (k < XPIECES) {
                const int x = k >> 5, c = k & 31;
                *(uint4*)(yr + (size_t)k * 8) = *(const uint4*)(smem + Y_OFF + x * 512 + ((c ^ (x & 31)) << 4));
            }
        }
    }
    wait_vm<0>();
}

}  // namespace

bool bneck28_supported(int H, int W, int C, int P) { return H == IW && W == IW && C == CX && P == CP; }

size_t bneck28_weight_elems(int nblk) { return (size_t)nblk * 4 * NFR * 512; }

// One block's member convs ([Npad][Kpad] rows, K order (kh, kw, c)) into the per-quarter register images:
// [blk][quarter q][34 fragments][64 lanes][8]; fragment = 16 output rows x 32 K, lane (g, r) holds rows[row0 + r][kb(g) ..
// + 7] (conv1: x planes s + 8 g, the kernel's spread order)
void bneck28_pack_block(const bf16_t* r1, int kp1, const bf16_t* r2, int kp2, const bf16_t* r3, int kp3, int blk,
                        bf16_t* out) {
    auto frag = [](bf16_t* dst, const bf16_t* rows, int kp, int row0, auto kb) {
        for (int l = 0; l < 64; ++l)
            for (int e = 0; e < 8; ++e) dst[l * 8 + e] = rows[(size_t)(row0 + (l & 15)) * kp + kb(l >> 4) + e];
    };
    for (int q = 0; q < 4; ++q) {
        bf16_t* o = out + (size_t)(blk * 4 + q) * NFR * 512;
        int f = 0;
        for (int s = 0; s < 8; ++s) frag(o + (size_t)(f++) * 512, r1, kp1, 16 * q, [&](int g) { return 8 * (s + 8 * g); });
        for (int s = 0; s < 18; ++s) frag(o + (size_t)(f++) * 512, r2, kp2, 16 * q, [&](int g) { return 32 * s + 8 * g; });
        for (int s = 0; s < 2; ++s)
            for (int i = 0; i < 4; ++i)
                frag(o + (size_t)(f++) * 512, r3, kp3, 16 * (4 * q + i), [&](int g) { return 32 * s + 8 * g; });
    }
}

hipError_t launch_bneck28(const Chain17Args& a, int blk, hipStream_t s) {
    if (a.B <= 0 || !a.x || !a.y || !a.w || !a.bias || blk < 0) return hipErrorInvalidValue;
    auto k = a.f16 ? bneck28_kernel<true> : bneck28_kernel<false>;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, BN28_LDS);
        attr[a.f16 ? 1 : 0] = true;
    }
    // blockIdx.y selects the block's weights and biases (grid.y = 1, offset through the pointers)
    Chain17Args b = a;
    b.w = a.w + (size_t)blk * 4 * NFR * 512;
    b.bias = a.bias + (size_t)blk * 384;
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), BN28_LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, b);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), BN28_LDS, s, b);
    return hipGetLastError();
}

}  // namespace fr
