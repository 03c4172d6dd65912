// ResNet-50 ArcFace stem -- conv1 (7x7 / s2 / p3, 3 -> 64, BN folded) + ReLU + maxpool (3x3 / s2 / p1) at 112x112
// (arcface_model.py:118-132, the torchvision resnet50 stem) -- in one launch.  As member ops at bs = 256 the conv is
// ~100 us (profiles/r06_r50_layer_profile.txt: K = 392 per pixel, its 51 MB output written and re-read) and the
// max-pool ~31 us.  Here one 512-thread workgroup per image walks the pooled rows:
//   * phase m: conv rows 2m and 2m + 1 (waves 0-3 / 4-7; per wave two 16-channel fragments x two of the four
//     16-pixel fragments of the 56-pixel row, so each B fragment read feeds two MFMAs) into a 6-row ring, then pooled row m - 1 from conv rows 2m - 3 .. 2m - 1 with
//     one 16-B store per (pixel, 8 channels); one barrier per phase;
//   * the prepared input rows (launch_preprocess's 8-channel [v v v v v v 0 0] pixels, the stem's hi/lo weight
//     split; from u8 crops the kernel prepares them itself, one phase behind the raw rows' DMA, and the preprocess
//     launch is skipped) arrive by LDS-DMA into a 20-row ring two phases ahead, columns de-interleaved by parity with the 3-pixel
//     zero pad written by the DMA itself (out-of-range offsets read 0), so a stride-2 tap reads 16 consecutive
//     pixels' 16-B chunks: B fragment = one conflict-free ds_read_b128;
//   * the conv's weight rows ([Npad][Kpad], K = (tap, 8 channels), taps 49 .. 51 zero) stay in registers (2 x 13
//     fragments per wave);
//   * the max-pool compares the stored 16-bit values as unsigned integers: after ReLU (written as +0 for v <= 0)
//     bf16 / f16 bit patterns order like the values, and the padding never wins a window that holds a value >= 0.
// Same operands, weights, rounding point (the conv output in the storage format) as the member ops: only the f32
// summation order of the conv differs.  Bounds: 2 x 3136 x 64 x 392 = 157 MFLOP (of which 52 / 49 padding) per
// image, 200 KB in, 100 KB out: at bs = 256 40 GFLOP and 77 MB of HBM.
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int IH = 112;                      // input rows / columns
constexpr int CWD = 56;                      // conv output rows / columns
constexpr int PWD = 28;                      // pooled rows / columns
constexpr int CO = 64;                       // channels
constexpr int XPAR = 64 * 16;                // one parity plane of a padded input row: 64 columns x 16 B
constexpr int XROWB = 2 * XPAR;              // 2048
constexpr int XR = 20;                       // input ring rows
constexpr int CROWB = CWD * CO * 2;          // 7168: one conv row, [56 px][64 ch], 16-B chunks XOR-swizzled by px
constexpr int CR = 6;                        // conv ring rows
constexpr int X_OFF = 0;
constexpr int C_OFF = X_OFF + XR * XROWB;    // 40960
constexpr int RAW_OFF = C_OFF + CR * CROWB;  // 83968: u8 input, 2 slots of one DMA group (4 rows, 1344 B)
constexpr int RAWB = 2048;                   // (two waves' DMA spans)
constexpr int SR50_LDS = RAW_OFF + 2 * RAWB; // 88064
constexpr int KS = 13;                       // K-steps: 52 tap slots of 8 channels (49 used)
constexpr int NWV = 8;

typedef int v4i32 __attribute__((ext_vector_type(4)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
// 16-byte LDS-DMA (lane l lands at lds_addr + 16 l), invisible to the compiler's waitcnt pass (conv_trans.hip)
__device__ __forceinline__ void dma16(const v4i32& rsrc, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
                 : "memory", "m0");
}
#pragma clang diagnostic pop

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Phase m waits for input group G(m) = rows 4m + 2 .. 4m + 5 (issued in phase m - 2; G(-2) .. G(1) before the
// loop).  VMEM ops per phase: one DMA instruction (G(m + 2)), then, for m >= 1, S pooled-row stores (waves 0-3: one,
// 4-7: none).
template <int S>
__device__ __forceinline__ void wait_group(int m) {
    if (m >= 3) wait_vm<1 + 2 * S>();
    else if (m == 2) wait_vm<1 + S>();
    else wait_vm<1>();
}

// u8 input: phase m waits for the raw group G(m + 1) (issued in phase m - 1; G(1) after the prologue's conversions);
// younger: phase m - 1's pooled-row store (waves 0-1 issue the raw DMA and store in every phase m >= 1)
__device__ __forceinline__ void wait_raw(int m) {
    if (m >= 2) wait_vm<1>();
    else wait_vm<0>();
}

template <bool F16, bool U8>
__global__ __launch_bounds__(64 * NWV, 1) void stem_r50_kernel(StemR50Args p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, l15 = lane & 15, lg = lane >> 4;
    const int b = blockIdx.x;
    if (b >= p.B) return;
    // conv row 2m + sel, channel fragments 2 np and 2 np + 1, pixel fragments 2 ph and 2 ph + 1 (each B fragment read
    // feeds two MFMAs)
    const int sel = wave >> 2, np = (wave >> 1) & 1, ph = wave & 1;

    // ---- weights (2 x 13 fragments) and biases, into registers once, before the first DMA
    frag wa[2][KS];
    float4 bias[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            wa[i][ks] = *(const frag*)(p.w + (size_t)(16 * (2 * np + i) + l15) * p.Kpad + 32 * ks + 8 * lg);
        bias[i] = *(const float4*)(p.bias + 16 * (2 * np + i) + 4 * lg);
    }
    // consumed here, so the compiler's wait for these loads sits before the loop (its waitcnt pass does not see the
    // DMAs: a wait at a first use inside the loop would be a vmcnt(0) in every phase)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" : "+v"(wa[i][ks]));
        asm volatile("" : "+v"(bias[i].x), "+v"(bias[i].y), "+v"(bias[i].z), "+v"(bias[i].w));
    }

    // ---- input DMA: group G(k) = rows 4k + 2 .. 4k + 5; wave w moves row 4k + 2 + (w >> 1), parity plane w & 1: lane
    // i = padded column 2i + (w & 1), pixel 2i + (w & 1) - 3 (outside the row or the image: offset out of range, 0)
    const uint64_t xp = (uint64_t)p.x;
    const v4i32 xr = {(int)(uint32_t)xp, (int)((xp >> 32) & 0xffff), (int)((size_t)p.B * IH * IH * 16), 0x00020000};
    const int dpx = 2 * lane + (wave & 1) - 3;
    auto dma_group = [&](int k) {
        const int row = 4 * k + 2 + (wave >> 1);
        const bool ok = (unsigned)row < (unsigned)IH && (unsigned)dpx < (unsigned)IH;
        const uint32_t off = ok ? (uint32_t)((((size_t)b * IH + row) * IH + dpx) * 16) : 0x80000000u;
        dma16(xr, (uint32_t)(uintptr_t)(smem + X_OFF + ((row + 8) % XR) * XROWB + (wave & 1) * XPAR), off);
    };
    // ---- u8 crops (U8): group G(k) = 1344 contiguous bytes (21 16-B chunks per row) into raw slot k & 1 by waves 0-1,
    // then converted in LDS to the prepared pixels [v v v v v v 0 0], v = 2q - 255 (launch_preprocess's values)
    const uint64_t up = (uint64_t)p.u8;
    const v4i32 ur = {(int)(uint32_t)up, (int)((up >> 32) & 0xffff), (int)((size_t)p.B * IH * IH * 3), 0x00020000};
    auto dma_raw = [&](int k) {
        if (wave < 2) {
            const int e = 64 * wave + lane, row = 4 * k + 2 + e / 21;
            const bool ok = e < 84 && (unsigned)row < (unsigned)IH;
            const uint32_t off = ok ? (uint32_t)(((size_t)b * IH + 4 * k + 2) * IH * 3 + 16 * e) : 0x80000000u;
            dma16(ur, (uint32_t)(uintptr_t)(smem + RAW_OFF + (k & 1) * RAWB + 1024 * wave), off);
        }
    };
    auto convert = [&](int k) {  // thread t: row 4k + 2 + (t >> 7), parity plane (t >> 6) & 1, column index t & 63
        const int t = threadIdx.x, rr = t >> 7, par = (t >> 6) & 1, i = t & 63;
        const int row = 4 * k + 2 + rr, px = 2 * i + par - 3;
        uint4 v = make_uint4(0u, 0u, 0u, 0u);
        if ((unsigned)row < (unsigned)IH && (unsigned)px < (unsigned)IH) {
            const uint8_t* qb = (const uint8_t*)(smem + RAW_OFF + (k & 1) * RAWB + rr * (IH * 3) + 3 * px);
            const uint32_t a = T::cvt(2.0f * (float)qb[0] - 255.0f), c1 = T::cvt(2.0f * (float)qb[1] - 255.0f),
                           c2 = T::cvt(2.0f * (float)qb[2] - 255.0f);
            v = make_uint4(a | (c1 << 16), c2 | (a << 16), c1 | (c2 << 16), 0u);
        }
        *(uint4*)(smem + X_OFF + ((row + 8) % XR) * XROWB + par * XPAR + i * 16) = v;
    };
    if (U8) {
        dma_raw(-1);
        dma_raw(0);
        wait_vm<0>();
        lds_barrier();
        convert(-2);  // (all rows outside the image: zeros)
        convert(-1);
        convert(0);
        lds_barrier();  // raw slot 1 read before G(1) overwrites it
        dma_raw(1);
    } else {
#pragma unroll
        for (int k = -2; k <= 1; ++k) dma_group(k);
    }

    // per lane and K-step: tap 4 ks + lg (taps past 48 read tap 48's pixels: their weights are zero), row offset kh,
    // column offset (kw & 1) plane + (kw >> 1) chunks
    auto tap_off = [&](int ks, int& kh) {
        const int t = min(4 * ks + lg, 48);
        kh = (t * 37) >> 8;  // t / 7 for t < 49
        const int kw = t - 7 * kh;
        return (kw & 1) * XPAR + ((kw >> 1) + l15) * 16;
    };

    for (int m = 0; m <= PWD; ++m) {
        if (U8) {
            if (wave < 2) wait_raw(m);
        } else if (wave < 4) {
            wait_group<1>(m);
        } else {
            wait_group<0>(m);
        }
        lds_barrier();  // G(m) landed everywhere (U8: raw G(m + 1)); conv rows 2m - 3 .. 2m - 1 complete; the slots
                        // written below were last read in phase m - 1
        if (U8) {
            dma_raw(m + 2);  // into the slot of G(m), converted in phase m - 1
            convert(m + 1);  // read by the next phase's conv
        } else {
            dma_group(m + 2);  // (past the image: zero rows into free slots)
        }

        if (m < PWD) {
            const int y = 2 * m + sel;
            const int s0 = (2 * y + 5) % XR;  // slot of input row 2y - 3 (kh = 0)
            f32x4_t acc[2][2];
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) acc[i][j] = (f32x4_t){bias[i].x, bias[i].y, bias[i].z, bias[i].w};
            frag bq[3][2];
            auto rd = [&](int ks, frag (&d)[2]) {
                int kh;
                const int o = tap_off(ks, kh);
                const int sl = s0 + kh >= XR ? s0 + kh - XR : s0 + kh;
                const char* src = smem + X_OFF + sl * XROWB + o + 512 * ph;
#pragma unroll
                for (int j = 0; j < 2; ++j) d[j] = *(const frag*)(src + 256 * j);  // pixel fragment 2 ph + j: + 16 chunks
            };
            rd(0, bq[0]);
            rd(1, bq[1]);
#pragma unroll
            for (int ks = 0; ks < KS; ++ks) {
                __builtin_amdgcn_sched_barrier(0);  // keep each step's reads in that step
                if (ks + 2 < KS) rd(ks + 2, bq[(ks + 2) % 3]);
#pragma unroll
                for (int i = 0; i < 2; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j) acc[i][j] = T::mfma(wa[i][ks], bq[ks % 3][j], acc[i][j]);
            }
            __builtin_amdgcn_sched_barrier(0);
            // epilogue: ReLU (v <= 0 -> +0) into conv ring row y; lane = channels 16 (2 np + i) + 4 lg .. + 3 of pixel
            // 16 (2 ph + j) + l15
            char* const cr = smem + C_OFF + (y % CR) * CROWB;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int n = 16 * (2 * np + i) + 4 * lg;
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int px = 16 * (2 * ph + j) + l15;
                    if (px < CWD) {
                        float v[8];
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = relu_bits(acc[i][j][e]);  // +0 for v <= 0
                        const uint4 pk = T::pack8(v);
                        *(uint2*)(cr + px * 128 + (((n >> 3) ^ (px & 7)) << 4) + (n & 4) * 2) = make_uint2(pk.x, pk.y);
                    }
                }
            }
        }
        // pooled row m - 1: thread t < 224 -> pixel t >> 3, channels 8 (t & 7) ..; windows over conv rows / columns
        // 2j - 1 .. 2j + 1 (index -1: the padding, skipped)
        if (m >= 1 && threadIdx.x < PWD * 8) {
            const int mp = m - 1, j = threadIdx.x >> 3, cg = threadIdx.x & 7;
            typedef unsigned short us8 __attribute__((ext_vector_type(8)));
            us8 mx = (us8)0;
#pragma unroll
            for (int dr = -1; dr <= 1; ++dr) {
                const int rr = 2 * mp + dr;
                if (rr < 0) continue;
                const char* cr = smem + C_OFF + (rr % CR) * CROWB;
#pragma unroll
                for (int dc = -1; dc <= 1; ++dc) {
                    const int cc = 2 * j + dc;
                    if (cc < 0) continue;
                    const us8 v = __builtin_bit_cast(us8, *(const uint4*)(cr + cc * 128 + ((cg ^ (cc & 7)) << 4)));
                    mx = __builtin_elementwise_max(mx, v);
                }
            }
            *(uint4*)(p.y + (((size_t)b * PWD + mp) * PWD + j) * CO + 8 * cg) = __builtin_bit_cast(uint4, mx);
        }
    }
    wait_vm<0>();  // (the trailing zero-row DMAs too) -- nothing in flight when the workgroup ends
}

}  // namespace

bool stem_r50_supported(int H, int W, int Cin, int K, int Kpad, int Cout) {
    return H == IH && W == IH && Cin == 8 && K == 392 && Kpad >= 32 * KS && Cout == CO;
}

hipError_t launch_stem_r50(const StemR50Args& a, hipStream_t s) {
    if (a.B <= 0 || (!a.x && !a.u8) || !a.y || !a.w || !a.bias || a.Kpad < 32 * KS) return hipErrorInvalidValue;
    if ((size_t)a.B * IH * IH * 16 >= 0x80000000ull) return hipErrorInvalidValue;  // 31-bit buffer offsets
    auto k = a.u8 ? (a.f16 ? stem_r50_kernel<true, true> : stem_r50_kernel<false, true>)
                  : (a.f16 ? stem_r50_kernel<true, false> : stem_r50_kernel<false, false>);
    static bool attr[4] = {false, false, false, false};
    const int ai = (a.u8 ? 2 : 0) + (a.f16 ? 1 : 0);
    if (!attr[ai]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, SR50_LDS);
        attr[ai] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), SR50_LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(64 * NWV), SR50_LDS, s, a);
    return hipGetLastError();
}

}  // namespace fr
