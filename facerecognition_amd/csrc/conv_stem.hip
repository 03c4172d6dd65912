// Fused preprocess + IResNet stem for uint8 NHWC crops (CDNA4 / gfx950).
//
// Replaces two launches of the u8 path: preprocess_u8_kernel (misc.hip: q -> 2q - 255 into an 8-channel
// [q q 0 0] bf16 image) and the stem conv ("conv1", 3x3 / s1 / p1, 3 -> 64 @112x112, bias + PReLU) as an
// implicit GEMM with Cin = 8 (K = 72), which at K = 72 is all address arithmetic and runs far below the
// HBM rate of its 411 MB output (profiles/r01_bench_kernel_stats.csv, "conv_igemm tile1").
// Reference: get_transform() Resize/ToTensor/Normalize(0.5) + the backbone's first conv + BN + PReLU
// (inference/extract_embeddings.py get_transform; insightface IResNet stem).
// Same operands and weights as the two-launch path: the input values 2q - 255 are exact integers in
// bf16/f16, the weight rows are the engine's stem rows (w/255 split hi/lo over channels 0-2 / 3-5,
// K = (tap, c) with c fastest, zero past K = 72), so only the f32 summation order differs.
// Tile = 2 output rows of one image (224 pixels = 14 m-frags) x 64 channels (4 n-frags); 3 persistent
// blocks per CU loop over tiles, staging the weights once and prefetching the next tile's input:
//   * the 64 x 96 weight rows go to LDS once per block, the 4 input rows (dword loads) once per tile; the input
//     becomes 2q - 255 in the activation dtype with a zero halo, [row][col][4];
//   * MFMA operand B for K-step ks, k-group g is tap 4ks + g of one pixel = [v0 v1 v2 v0 v1 v2 0 0],
//     built from one 8-byte LDS read; operand A = 12 weight fragments per lane, read once per tile;
//   * 3 K-steps of v_mfma_f32_16x16x32_{bf16,f16} per tile; the epilogue (bias, PReLU) stages the
//     224 x 64 tile in LDS (16-B chunks XOR-swizzled by pixel) and writes it with 16-B coalesced stores.
#include "kernels.h"

#include <hip/hip_ext.h>

#include <cstdlib>
#include <type_traits>

namespace fr {
namespace {

constexpr int SW = 112;       // image width = height
constexpr int SCO = 64;       // output channels
constexpr int SROWS = 2;      // output rows per tile
constexpr int SPIX = SROWS * SW;  // 224
constexpr int WROW = 104;          // LDS weight row: 96 bf16 + pad (208 B: conflict-free 16-lane reads)

// Workgroup barrier that waits for LDS only: __syncthreads()'s fence also drains vmcnt, i.e. every 16-B
// output store of the previous tile (gfx950 counts stores in vmcnt) and the next tile's prefetched input
// rows, so each tile's 28 KiB of stores would run exposed instead of behind the next tile's work.
constexpr int OFF_SY = 0;                                     // 28672
constexpr int OFF_SWT = OFF_SY + SPIX * 8 * 16;               // 13312
constexpr int OFF_SX = OFF_SWT + SCO * WROW * 2;              // 3648
constexpr int OFF_SBS = OFF_SX + (SROWS + 2) * (SW + 2) * 8;  // 512
constexpr int OFF_RAW = OFF_SBS + 2 * SCO * 4;                // 2048
constexpr int STEM_LDS = OFF_RAW + 2 * 2 * 256 * 4;              // sraw: two tile buffers
static_assert(OFF_SX % 16 == 0 && OFF_SBS % 16 == 0 && OFF_RAW % 16 == 0, "16-B aligned LDS arrays");

// 4-byte LDS-DMA (buffer_load_dword ... lds; lane l lands at lds_addr + 4 l) issued from inline asm: the
// compiler then does not know about the LDS write, and its waitcnt pass does not guard every later LDS
// access with a vmcnt(0) (which would also drain the output stores); the kernel's own waits cover the DMA
// (m0 is reserved to the compiler, hence the pragma; nothing else in this kernel uses m0)
typedef int v4i32 __attribute__((ext_vector_type(4)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma_dword(const v4i32& rsrc, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
                 : "memory", "m0");
}
#pragma clang diagnostic pop

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

template <bool F16>
// waves_per_eu(3): the persistent loop would otherwise grow past 168 VGPRs and lose the third block per CU
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void stem_u8_kernel(
    const uint8_t* __restrict__ in, const bf16_t* __restrict__ w, int Kpad, const float* __restrict__ bias,
    const float* __restrict__ slope, int act, bf16_t* __restrict__ y, int Cy, int y_off, int ntiles) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    // one dynamic LDS block (STEM_LDS bytes): with static __shared__ arrays the compiler cannot tell the
    // input DMA's target from the other arrays and puts a vmcnt(0) (which drains the output stores) before
    // every LDS access after the DMA issue
    extern __shared__ __attribute__((aligned(16))) char smem[];
    uint16_t(*sx)[SW + 2][4] = (uint16_t(*)[SW + 2][4])(smem + OFF_SX);  // [SROWS + 2][SW + 2][4]
    uint4* sy = (uint4*)(smem + OFF_SY);                                  // [SPIX * 8]
    uint16_t(*swt)[WROW] = (uint16_t(*)[WROW])(smem + OFF_SWT);          // [SCO][WROW] weight rows
    float(*sbs)[SCO] = (float(*)[SCO])(smem + OFF_SBS);                   // [2][SCO] bias, PReLU slope
    uint32_t* sraw = (uint32_t*)(smem + OFF_RAW);                         // [2][2 * 256] u8 rows as dwords + pad
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

    // the 64 x 96 weight rows, staged once per (persistent) block; the first tile's barrier after its
    // sraw loads publishes them
    for (int e = tid; e < SCO * 12; e += 256) {
        const int n = e / 12, c = e % 12;
        *(uint4*)&swt[n][8 * c] = *(const uint4*)(w + (size_t)n * Kpad + 8 * c);
    }
    // bias and slope in LDS too: global loads in the epilogue would make its vmcnt waits also wait for the
    // next tile's input prefetch (issued just before) and for nothing else
    float sl_t = 1.f;
    if (tid < SCO) {
        sbs[0][tid] = bias[tid];
        sbs[1][tid] = sl_t = act == 2 ? slope[tid] : 0.f;
    }
    // PReLU as max(v, s v) when every slope is in (0, 1]: the same bits as v > 0 ? v : s v (for v > 0,
    // s v <= v; for v <= 0, s v >= v; NaN stays NaN), one operation fewer per value
    const bool slope01 = act == 2 && __syncthreads_and(tid >= SCO || (sl_t > 0.f && sl_t <= 1.f));

    // a tile's input rows r0-1 .. r0+2 (336 contiguous bytes each) as dwords, two per thread
    constexpr int RAWD = (SROWS + 2) * (SW * 3 / 4);
    static_assert(RAWD <= 2 * 256, "two input dwords per thread");
    // The rows go straight to LDS by LDS-DMA (4 B per lane, linear: dword e = tid + 256 j of the tile's
    // sraw buffer), two tiles ahead (one DMA latency per tile, under write load, was most of a tile's
    // time), branch free: rows outside the image, the pad dwords and tiles past the end get an
    // out-of-range offset, which reads 0.  The waits are explicit (see the loop top).
    const uint64_t inp = (uint64_t)in;
    const v4i32 inr = {(int)(uint32_t)inp, (int)((inp >> 32) & 0xffff), (int)((ntiles / (SW / SROWS)) * (SW * SW * 3)),
                       0x00020000};
    auto dma_raw = [&](int t, int buf) {
        const int b = t / (SW / SROWS), r0 = (t % (SW / SROWS)) * SROWS;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int e = tid + 256 * j, rr = e / (SW * 3 / 4), d = e % (SW * 3 / 4), ir = r0 - 1 + rr;
            const bool ok = e < RAWD && (unsigned)ir < (unsigned)SW;
            const uint32_t off = ok ? (uint32_t)(((b * SW + ir) * SW * 3) + 4 * d) : 0x80000000u;
            dma_dword(inr, (uint32_t)(uintptr_t)&sraw[512 * buf + 256 * j + 64 * wave], off);
        }
    };
    dma_raw(blockIdx.x, 0);  // gridDim.x <= ntiles
    dma_raw(blockIdx.x + gridDim.x, 1);
    // the weight / table loads above went to registers first: done before the counted waits below
    // tiles t = blockIdx.x + j * gridDim.x; every wave runs the same trip count (block-uniform loop)
    int j = 0;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x, ++j) {
        const int b = t / (SW / SROWS), r0 = (t % (SW / SROWS)) * SROWS;
        const uint32_t* sr = sraw + 512 * (j & 1);
        // this tile's DMA landed.  VMEM order: DMA 0, DMA 1, then per tile i: DMA i + 2 (2 ops), 7 stores;
        // younger than DMA j: DMA 1 (j = 0); DMA 2 + stores 0 (j = 1); stores j-2, DMA j+1, stores j-1
        if (j == 0) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        else if (j == 1) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        // the previous tile's reads of sraw / sx / sy all precede a barrier every thread has passed
        lds_barrier();
        // -> 2q - 255 in the activation dtype, zero halo columns (rows outside the image were zeroed above
        // but must also become 0, not -255)
        for (int e = tid; e < (SROWS + 2) * (SW + 2); e += 256) {
            const int rr = e / (SW + 2), cc = e % (SW + 2), ir = r0 - 1 + rr, ic = cc - 1;
            uint16_t v[3] = {0, 0, 0};
            if ((unsigned)ir < (unsigned)SW && (unsigned)ic < (unsigned)SW) {
                const uint8_t* q = (const uint8_t*)&sr[rr * (SW * 3 / 4)] + 3 * ic;
#pragma unroll
                for (int c = 0; c < 3; ++c) v[c] = T::cvt(2.0f * (float)q[c] - 255.0f);
            }
            *(uint2*)&sx[rr][cc][0] = make_uint2((uint32_t)v[0] | ((uint32_t)v[1] << 16), (uint32_t)v[2]);
        }
        // weight fragments from the block's LDS copy, re-read per tile (held across tiles they would add
        // 48 live VGPRs and cost the third block per CU): n = 16i + (lane&15), k = 32ks + 8g .. +7
        frag wa[4][3];
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int ks = 0; ks < 3; ++ks)
                wa[i][ks] = *(const frag*)&swt[16 * i + (lane & 15)][32 * ks + 8 * (lane >> 4)];
        lds_barrier();

        // wave w: m-frags w, w+4, w+8, w+12 (< 14)
        f32x4_t acc[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[u][i] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int f = wave + 4 * u;
            if (f >= SPIX / 16) break;  // wave-uniform
            const int px = 16 * f + (lane & 15), pr = px / SW, pc = px % SW;
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) {
                const int tap = 4 * ks + (lane >> 4);
                uint4 q = make_uint4(0u, 0u, 0u, 0u);
                if (tap < 9) {
                    const uint2 v = *(const uint2*)&sx[pr + tap / 3][pc + tap % 3][0];
                    const uint32_t v0 = v.x & 0xffff, v1 = v.x >> 16, v2 = v.y & 0xffff;
                    q = make_uint4(v.x, v2 | (v0 << 16), v1 | (v2 << 16), 0u);
                }
                const frag bq = __builtin_bit_cast(frag, q);
#pragma unroll
                for (int i = 0; i < 4; ++i) acc[u][i] = T::mfma(wa[i][ks], bq, acc[u][i]);
            }
        }
        dma_raw(t + 2 * gridDim.x, j & 1);  // unconditional (uniform wait counts); this buffer's reads are behind barrier 2
        // epilogue: lane holds channels 16i + 4(lane>>4) .. +3 of pixel 16f + (lane&15).  One branch per
        // tile picks the activation form (MODE 0: PReLU as max(v, s v); 1: PReLU by select; 2: ReLU;
        // 3: none), so the unrolled (i, u) body is straight code
        auto epilogue = [&](auto mode_tag) {
            constexpr int MODE = decltype(mode_tag)::value;
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int n = 16 * i + 4 * (lane >> 4);
                const float4 bb = *(const float4*)&sbs[0][n];
                const float4 sl = *(const float4*)&sbs[1][n];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int f = wave + 4 * u;
                    if (f >= SPIX / 16) break;
                    const int px = 16 * f + (lane & 15);
                    // bias and slope products as packed pairs (v_pk_add_f32 / v_pk_mul_f32: the same IEEE
                    // operations per element, half the instructions; the epilogue is most of the VALU)
                    typedef float f2 __attribute__((ext_vector_type(2)));
                    const f2 v01 = (f2){acc[u][i][0], acc[u][i][1]} + (f2){bb.x, bb.y};
                    const f2 v23 = (f2){acc[u][i][2], acc[u][i][3]} + (f2){bb.z, bb.w};
                    float v[8] = {v01.x, v01.y, v23.x, v23.y, 0, 0, 0, 0};
                    if (MODE == 0) {
                        const f2 p01 = v01 * (f2){sl.x, sl.y}, p23 = v23 * (f2){sl.z, sl.w};
                        // v_max_f32 directly: fmaxf would first canonicalize both operands (two more
                        // instructions each); these operands are arithmetic results, never signalling NaNs
                        asm("v_max_f32 %0, %1, %2" : "=v"(v[0]) : "v"(v01.x), "v"(p01.x));
                        asm("v_max_f32 %0, %1, %2" : "=v"(v[1]) : "v"(v01.y), "v"(p01.y));
                        asm("v_max_f32 %0, %1, %2" : "=v"(v[2]) : "v"(v23.x), "v"(p23.x));
                        asm("v_max_f32 %0, %1, %2" : "=v"(v[3]) : "v"(v23.y), "v"(p23.y));
                    } else if (MODE == 1) {
                        v[0] = v[0] > 0.f ? v[0] : v[0] * sl.x;
                        v[1] = v[1] > 0.f ? v[1] : v[1] * sl.y;
                        v[2] = v[2] > 0.f ? v[2] : v[2] * sl.z;
                        v[3] = v[3] > 0.f ? v[3] : v[3] * sl.w;
                    } else if (MODE == 2) {
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
                    }
                    const uint4 pk = T::pack8(v);
                    // 16-B chunk n/8 of the pixel's 128-B row, XOR-swizzled by pixel; this lane owns half of it
                    char* dst = (char*)&sy[px * 8 + ((n >> 3) ^ (px & 7))] + (n & 4) * 2;
                    *(uint2*)dst = make_uint2(pk.x, pk.y);
                }
            }
        };
        if (slope01) epilogue(std::integral_constant<int, 0>{});
        else if (act == 2) epilogue(std::integral_constant<int, 1>{});
        else if (act == 1) epilogue(std::integral_constant<int, 2>{});
        else epilogue(std::integral_constant<int, 3>{});
        lds_barrier();
        // coalesced stores: 224 pixels x 8 chunks of 16 B
        const size_t row0 = ((size_t)b * SW + r0) * SW;
        static_assert(SPIX * 8 % 256 == 0, "whole store rounds");
#pragma unroll
        for (int q = 0; q < SPIX * 8 / 256; ++q) {
            const int e = tid + 256 * q, px = e >> 3, ch = e & 7;
            *(uint4*)(y + (row0 + px) * Cy + y_off + 8 * ch) = sy[px * 8 + (ch ^ (px & 7))];
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (out-of-range) DMAs land before the LDS is released
}

}  // namespace

bool stem_u8_supported(int H, int W, int Cin, int K, int Kpad, int Cout, int Cy, int y_off) {
    return H == SW && W == SW && Cin == 8 && K == 72 && Kpad >= 96 && Cout == SCO && Cy % 8 == 0 && y_off % 8 == 0 &&
           y_off + SCO <= Cy;
}

hipError_t launch_stem_u8(const uint8_t* in, int B, const bf16_t* w, int Kpad, const float* bias, const float* slope,
                          int act, bf16_t* y, int Cy, int y_off, int f16, hipStream_t s) {
    // persistent blocks: 3 per CU (the VGPR limit), trip counts balanced so no block runs an extra
    // round; FR_AB stem_persist=0 launches one block per tile (weights re-staged per tile)
    static const bool persist = [] { return ab_int("stem_persist", 1) != 0; }();
    if ((size_t)B * SW * SW * 3 >= 0x80000000ull) return hipErrorInvalidValue;  // buffer offsets are 31-bit
    const int ntiles = B * (SW / SROWS);
    int nblk = ntiles;
    if (persist && ntiles > 768) {
        const int trips = (ntiles + 767) / 768;
        nblk = (ntiles + trips - 1) / trips;
    }
    const dim3 grid(nblk);
    if (f16)
        hipLaunchKernelGGL(stem_u8_kernel<true>, grid, dim3(256), STEM_LDS, s, in, w, Kpad, bias, slope, act, y, Cy, y_off, ntiles);
    else
        hipLaunchKernelGGL(stem_u8_kernel<false>, grid, dim3(256), STEM_LDS, s, in, w, Kpad, bias, slope, act, y, Cy, y_off, ntiles);
    return hipGetLastError();
}

}  // namespace fr
