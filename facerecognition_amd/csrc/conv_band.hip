// Row-band direct 3x3 convolution (stride 1, pad 1) for CDNA4 (gfx950).
//
// The dominant IResNet100 layers (3x3 s1 256->256 @14x14 = 55.5 % of FLOPs,
// 128->128 @28x28 = 22.9 %, 64->64 @56/@112 = 7.6 %) are 3x3 / stride 1 / pad 1.  An implicit GEMM
// re-gathers every input pixel for all 9 taps (9x the activation bytes through L2 -> LDS) and, at
// bs=256, its 128x128 tiles quantize badly on 256 CUs.  This kernel instead gives each block TH full
// output rows of ONE image (TH*W ~ 200 pixels: one whole 14x14 image, 7 rows of 28, 4 of 56, 2 of 112)
// x BN output channels, so the tile count is always a multiple of the batch (256 images -> whole
// rounds of 256 CUs), and:
//   * the (TH+2) x (W+2) input patch (zero halo) of one 64-channel chunk is DMA'd into LDS once and
//     read by all 9 taps at shifted positions;
//   * per (chunk, tap) K-step only the [BN][64] weight slice streams in (double buffered);
//   * the next chunk's patch DMA overlaps the current chunk's 9 K-steps (double buffered).
// MFMA: v_mfma_f32_16x16x32_{bf16,f16}; operand A = weight rows (n), operand B = patch rows (pixels),
// so each lane ends with 4 consecutive channels of one pixel and the fused epilogue (bias, residual,
// ReLU/PReLU, second affine output) stores 8-byte groups straight from registers.
// LDS rows are 128 B (64 channels); chunk index XOR (row>>1)&7, applied to the per-lane DMA source.
#include "kernels.h"

#include <hip/hip_ext.h>

#include <cstdlib>

namespace fr {
namespace {

constexpr uint32_t OOB = 0x80000000u;
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int swzb(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// ... with a wave-uniform byte offset in soffset (memory address only; the instruction's immediate
// offset would also shift the LDS destination)
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, soff, 0, 0);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
    else if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
    else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
    else if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if constexpr (N == 7) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
}

constexpr int MAXPW = 8;  // max patch DMA instructions per wave per chunk

// Fused epilogue straight from registers (lane = 4 consecutive channels of one pixel): bias, residual,
// ReLU/PReLU, bf16/f16 store, optional second affine output.  Channel-outer so the per-channel vectors
// load once per fragment column; residual loads are unconditional (invalid lanes read pixel 0) so the
// FM loads of a column are in flight together; only the stores are predicated.
template <class T, int W, int Wp, int Mv, int FM, int FN>
__device__ __forceinline__ void band_epilogue(const ConvArgs& p, const f32x4_t (&acc)[FN][FM], int lane, int wm,
                                              int wn, size_t pix0, int n0) {
    int pix_off[FM];
    bool pv[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
        const int m = 16 * (wm * FM + j) + (lane & 15);
        const int r = m / Wp, c = m - r * Wp;
        pv[j] = m < Mv && c < W;
        pix_off[j] = pv[j] ? r * W + c : 0;
    }
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int n_raw = n0 + wn * 16 * FN + 16 * i + 4 * (lane >> 4);
        const bool nv = n_raw < p.Cout;
        const int n = nv ? n_raw : 0;
        float4 bb = make_float4(0.f, 0.f, 0.f, 0.f), sl = bb, as = bb, ab = bb;
        if (p.bias && !p.bias9) bb = *(const float4*)(p.bias + n);
        if (p.act == 2) sl = *(const float4*)(p.slope + n);
        if (p.y2) { as = *(const float4*)(p.aff_s + n); ab = *(const float4*)(p.aff_b + n); }
        uint2 rr[FM];
        if (p.res) {
#pragma unroll
            for (int j = 0; j < FM; ++j)
                rr[j] = *(const uint2*)(p.res + (pix0 + pix_off[j]) * p.Cres + p.res_off + n);
        }
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            float v[4] = {acc[i][j][0] + bb.x, acc[i][j][1] + bb.y, acc[i][j][2] + bb.z, acc[i][j][3] + bb.w};
            if (p.bias9) {
                const int po = pix_off[j], oh = (int)((pix0 / W) % p.Ho) + po / W;
                const float4 b9 = *(const float4*)(p.bias9 + (size_t)border_class(oh, po % W, p.Ho, W) * p.Npad + n);
                v[0] += b9.x; v[1] += b9.y; v[2] += b9.z; v[3] += b9.w;
            }
            if (p.res) {
                float f[8];
                T::unpack8(make_uint4(rr[j].x, rr[j].y, 0, 0), f);
                v[0] += f[0]; v[1] += f[1]; v[2] += f[2]; v[3] += f[3];
            }
            if (p.act == 1) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
            } else if (p.act == 2) {
                v[0] = v[0] > 0.f ? v[0] : v[0] * sl.x;
                v[1] = v[1] > 0.f ? v[1] : v[1] * sl.y;
                v[2] = v[2] > 0.f ? v[2] : v[2] * sl.z;
                v[3] = v[3] > 0.f ? v[3] : v[3] * sl.w;
            }
            if (pv[j] && nv) {
                const size_t pix = pix0 + pix_off[j];
                float o8[8] = {v[0], v[1], v[2], v[3], 0, 0, 0, 0};
                const uint4 pk = T::pack8(o8);
                *(uint2*)(p.y + pix * p.Cy + p.y_off + n) = make_uint2(pk.x, pk.y);
                if (p.y2) {
                    float u8[8] = {v[0] * as.x + ab.x, v[1] * as.y + ab.y, v[2] * as.z + ab.z, v[3] * as.w + ab.w,
                                   0, 0, 0, 0};
                    const uint4 pk2 = T::pack8(u8);
                    *(uint2*)(p.y2 + pix * p.Cy2 + p.y2_off + n) = make_uint2(pk2.x, pk2.y);
                }
            }
        }
    }
}

// LDS-staged epilogue for the 4-wave band kernel.  Passes over (channel half wn, row group mp): the
// owning waves park their f32 accumulators in LDS (rows of 16*FN floats, padded by 16 B against bank
// conflicts), then all threads emit coalesced 8-channel groups: 16-B loads of the residual (issued
// before the LDS round trip), 16-B stores of y / y2, per-channel vectors loaded once per pass (a
// thread's channel group is fixed).  Row groups (MP > 1) keep the staged rows within the LDS.
template <class T, int W, int Wp, int Mv, int FM, int FN, int WM, int WN>
__device__ __forceinline__ void band_epilogue_lds(const ConvArgs& p, const f32x4_t (&acc)[FN][FM], char* smem,
                                                  int tid, int lane, int wm, int wn, size_t pix0, int n0) {
    constexpr int NT = 64 * WM * WN;
    constexpr int CH = 16 * FN;              // channels per pass
    constexpr int G = CH / 8;                // 8-channel groups per row
    constexpr int ROWS = 16 * FM * WM;       // MFMA rows (pixel positions incl. the discarded columns)
    constexpr int LD = CH * 4 + 16;          // bytes per LDS row
    constexpr int MP = ROWS * LD <= 160 * 1024 ? 1 : 2;  // row groups
    constexpr int GR = ROWS / MP;            // staged rows per pass
    static_assert(GR * LD <= 160 * 1024 && WM % MP == 0, "epilogue staging fits LDS");
    static_assert(NT % G == 0, "fixed channel group per thread");
    constexpr int RS = NT / G;               // rows per sweep
    constexpr int IT = (GR + RS - 1) / RS;   // sweeps over a row group
    const int g = tid % G, r0 = tid / G;
#pragma unroll 1
    for (int pass = 0; pass < WN * MP; ++pass) {
        const int pn = pass / MP, mp = pass % MP;
        const int mbase = mp * GR;
        const int n = n0 + pn * CH + 8 * g;
        const bool nv = n < p.Cout;
        const int nn = nv ? n : 0;
        // residual of this thread's rows first: its latency overlaps the LDS round trip
        uint4 rr[IT];
        int pixo[IT];
        bool ok[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int m = mbase + r0 + it * RS;
            const int r = m / Wp, c = m - r * Wp;
            ok[it] = r0 + it * RS < GR && m < Mv && c < W && nv;
            pixo[it] = ok[it] ? r * W + c : 0;
            if (p.res) rr[it] = *(const uint4*)(p.res + (pix0 + pixo[it]) * p.Cres + p.res_off + nn);
        }
        float b8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, s8[8], as8[8], ab8[8];
        if (p.bias && !p.bias9) {
            const float4 x0 = *(const float4*)(p.bias + nn), x1 = *(const float4*)(p.bias + nn + 4);
            b8[0] = x0.x; b8[1] = x0.y; b8[2] = x0.z; b8[3] = x0.w; b8[4] = x1.x; b8[5] = x1.y; b8[6] = x1.z; b8[7] = x1.w;
        }
        if (p.act == 2) {
            const float4 x0 = *(const float4*)(p.slope + nn), x1 = *(const float4*)(p.slope + nn + 4);
            s8[0] = x0.x; s8[1] = x0.y; s8[2] = x0.z; s8[3] = x0.w; s8[4] = x1.x; s8[5] = x1.y; s8[6] = x1.z; s8[7] = x1.w;
        }
        if (p.y2) {
            const float4 x0 = *(const float4*)(p.aff_s + nn), x1 = *(const float4*)(p.aff_s + nn + 4);
            const float4 y0 = *(const float4*)(p.aff_b + nn), y1 = *(const float4*)(p.aff_b + nn + 4);
            as8[0] = x0.x; as8[1] = x0.y; as8[2] = x0.z; as8[3] = x0.w; as8[4] = x1.x; as8[5] = x1.y; as8[6] = x1.z; as8[7] = x1.w;
            ab8[0] = y0.x; ab8[1] = y0.y; ab8[2] = y0.z; ab8[3] = y0.w; ab8[4] = y1.x; ab8[5] = y1.y; ab8[6] = y1.z; ab8[7] = y1.w;
        }
        if (wn == pn && wm / (WM / MP) == mp) {
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    const int m = 16 * (wm * FM + j) + (lane & 15) - mbase;
                    *(f32x4_t*)(smem + m * LD + (16 * i + 4 * (lane >> 4)) * 4) = acc[i][j];
                }
        }
        __syncthreads();
#pragma unroll
        for (int it = 0; it < IT; ++it) {
            const int ml = r0 + it * RS;
            if (ml < GR) {
                const float4 v0 = *(const float4*)(smem + ml * LD + g * 32);
                const float4 v1 = *(const float4*)(smem + ml * LD + g * 32 + 16);
                float v[8] = {v0.x + b8[0], v0.y + b8[1], v0.z + b8[2], v0.w + b8[3],
                              v1.x + b8[4], v1.y + b8[5], v1.z + b8[6], v1.w + b8[7]};
                if (p.bias9) {
                    const int po = pixo[it], oh = (int)((pix0 / W) % p.Ho) + po / W;
                    const float* bb = p.bias9 + (size_t)border_class(oh, po % W, p.Ho, W) * p.Npad + nn;
                    const float4 x0 = *(const float4*)bb, x1 = *(const float4*)(bb + 4);
                    v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
                    v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
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
                    for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * s8[e];
                }
                if (ok[it]) {
                    const size_t pix = pix0 + pixo[it];
                    *(uint4*)(p.y + pix * p.Cy + p.y_off + n) = T::pack8(v);
                    if (p.y2) {
                        float u[8];
#pragma unroll
                        for (int e = 0; e < 8; ++e) u[e] = v[e] * as8[e] + ab8[e];
                        *(uint4*)(p.y2 + pix * p.Cy2 + p.y2_off + n) = T::pack8(u);
                    }
                }
            }
        }
        __syncthreads();
    }
}

// Patch LDS image, chunk-major: [8 chunks of 8 channels][P64 positions][16 B].  A tap shift is then a
// pure position offset, i.e. an immediate on ds_read_b128, and 16 lanes reading 16 consecutive
// positions of one chunk hit 16 distinct 16-B slots (planes are whole 1-KiB DMA blocks, so aligned).
// Weight slices stay row-major [BN][64] with the (row>>1)&7 chunk XOR; their read addresses are
// step-invariant and precomputed.
template <bool F16, int W, int TH, int WM, int WN, int FM, int FN, int WS>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv3x3_band_kernel(ConvArgs p, int ntn) {
    constexpr int NW = WM * WN;
    constexpr int BN = 16 * FN * WN;
    constexpr int Wp = W + 2;
    constexpr int P = (TH + 2) * Wp;
    constexpr int P64 = (P + 63) / 64 * 64;     // a DMA instruction fills 64 positions (1 KiB)
    constexpr int PLANE = P64 * 16;             // bytes of one chunk plane
    constexpr int PATCH = 8 * PLANE;            // bytes of one patch buffer
    constexpr int NPB = P64 / 64;               // 64-position DMA blocks per chunk plane
    constexpr int PI = 8 * NPB;                 // patch DMA instructions
    constexpr int NPW = (PI + NW - 1) / NW;     // patch DMA instructions per wave (upper bound)
    static_assert(NPW <= MAXPW, "patch too large");
    constexpr int WSL = BN * 128;
    constexpr int NWI = BN / 8 / NW;
    static_assert(NWI * 8 * NW == BN, "weight slice rows must split evenly over waves");
    // MFMA row m <-> patch position m (tap (0,0) of output pixel (m / Wp, m % Wp)): columns W, W+1 of
    // each row are computed and discarded.  Consecutive m are consecutive LDS slots (conflict-free
    // ds_read_b128) and a tap is a constant position shift.
    constexpr int Mv = TH * Wp - 2;
    static_assert(16 * FM * WM >= Mv, "MFMA rows must cover the band");
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [patch0][patch1][wsl0..wsl{WS-1}]

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int H = p.H;
    const int bands = H / TH;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int tn = lid % ntn;
    const int rest = lid / ntn;
    const int band = rest % bands, b = rest / bands;
    const int oh0 = band * TH, n0 = tn * BN;

    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * H * W * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const uint32_t w_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.Npad * p.Kpad * 2);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, w_bytes, 0x00020000);

    // Patch DMA: instruction q -> chunk plane c = q / NPB, positions 64*(q % NPB) + lane.  The
    // source offsets are recomputed per chunk (Wp is a compile-time constant) to save registers.
    auto patch_src = [&](int u) -> uint32_t {
        const int q = wave + NW * u;
        const int c = q / NPB, pos = 64 * (q - c * NPB) + lane;
        const int ih = oh0 - 1 + pos / Wp, iw = pos % Wp - 1;
        const bool ok = q < PI && pos < P && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        return ok ? (uint32_t)((((b * H + ih) * W + iw) * p.Cx + p.x_off + 8 * c) * 2) : OOB;
    };
    // Weight slice DMA (row-major, swizzled source chunk).
    uint32_t woff[NWI];
#pragma unroll
    for (int u = 0; u < NWI; ++u) {
        const int row = 8 * (wave + NW * u) + (lane >> 3);
        const int cl = (lane & 7) ^ ((row >> 1) & 7);
        woff[u] = (uint32_t)(((n0 + row) * p.Kpad + 8 * cl) * 2);
    }
    // Fragment read offsets (bytes within a buffer) for kk = 0; kk = 1 is +4 chunk planes for the
    // patch and an XOR of byte bit 6 for the swizzled weight rows ((4+x)^k == (x^k)^4 for x < 4).
    int aoff[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
        const int m = 16 * (wm * FM + j) + (lane & 15);
        aoff[j] = (lane >> 4) * PLANE + (m < Mv ? m : 0) * 16;
    }
    int boff[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int row = wn * 16 * FN + 16 * i + (lane & 15);
        boff[i] = row * 128 + swzb(row, lane >> 4) * 16;
    }

    const int npw = __builtin_amdgcn_readfirstlane((PI - wave + NW - 1) / NW);  // this wave's patch instrs
    auto issue_patch = [&](int chunk, int pb) {
        const uint32_t cadd = (uint32_t)(chunk * 64 * 2);
        char* dst = smem + pb * PATCH;
#pragma unroll
        for (int u = 0; u < NPW; ++u)
            if (u < npw) {
                const uint32_t src = patch_src(u);
                dma16(xr, dst + (wave + NW * u) * 1024, src == OOB ? OOB : src + cadd);
            }
    };
    auto issue_w = [&](int step, int wb) {
        const int chunk = step / 9, tap = step - chunk * 9;
        const uint32_t kadd = (uint32_t)((tap * p.Cin + chunk * 64) * 2);
        char* dst = smem + 2 * PATCH + wb * WSL;
#pragma unroll
        for (int u = 0; u < NWI; ++u) dma16(wr, dst + (wave + NW * u) * 1024, woff[u] + kadd);
    };

    f32x4_t acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    auto mma_tap = [&](const char* pa, const char* wa, int shift_bytes) {
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            frag af[FN], bfr[FM];
#pragma unroll
            for (int i = 0; i < FN; ++i) af[i] = *(const frag*)(wa + (boff[i] ^ (kk * 64)));
#pragma unroll
            for (int j = 0; j < FM; ++j) bfr[j] = *(const frag*)(pa + aoff[j] + kk * 4 * PLANE + shift_bytes);
#pragma unroll
            for (int i = 0; i < FN; ++i)
#pragma unroll
                for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(af[i], bfr[j], acc[i][j]);
        }
    };

    const int nchunk = p.Cin / 64;
    const int nsteps = nchunk * 9;
    // Prologue: patch 0 and the first WS-1 weight slices.
    issue_patch(0, 0);
    for (int s = 0; s < WS - 1 && s < nsteps; ++s) issue_w(s, s);
    // Warm this XCD's L2 with the block's whole [BN][K] weight panel while the prologue DMA is in
    // flight: every CU would otherwise miss on the same cold 32-KiB slice in lockstep at each K-step.
    // Blocks b, b+8, ... share an XCD (round-robin dispatch; a speed assumption only); the 32 blocks of
    // an XCD each touch one 4-byte word per 128-B line of a 1/32 share of the panel.
    {
        const uint32_t panel = (uint32_t)BN * p.Kpad * 2;
        const uint32_t share = (panel + 31) / 32;
        const uint32_t base = (uint32_t)n0 * p.Kpad * 2 + (uint32_t)((blockIdx.x / 8) % 32) * share;
        const uint32_t stride = (uint32_t)NW * 64 * 128;
        unsigned dummy;
        for (uint32_t o = (uint32_t)(wave * 64 + lane) * 128; o < share; o += stride) {
            asm volatile("buffer_load_dword %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                         : "=&v"(dummy) : "v"(base + o), "s"(wr) : "memory");
        }
    }
    wait_vm<0>();
    __syncthreads();
    int step = 0;
    for (int chunk = 0; chunk < nchunk; ++chunk) {
        const char* pa = smem + (chunk & 1) * PATCH;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap, ++step) {
            const int ahead = step + WS - 1;  // slice to prefetch now
            if (ahead < nsteps) issue_w(ahead, ahead % WS);
            const bool np = tap == 0 && chunk + 1 < nchunk;
            if (np) issue_patch(chunk + 1, (chunk + 1) & 1);
            mma_tap(pa, smem + 2 * PATCH + (step % WS) * WSL, ((tap / 3) * Wp + (tap % 3)) * 16);
            // Retire slice step+1 (and, at the chunk's last tap, the next patch).  Younger groups
            // allowed in flight: the slices step+2..step+WS-1 (WS=3: one) and a patch issued this step.
            const int younger_w = (WS == 3 && step + 2 < nsteps && ahead >= step + 2) ? NWI : 0;
            if (tap == 8) {
                wait_vm<0>();
            } else if (np) {
                // order of issue this step: slice `ahead`, then patch -> both may stay outstanding
                if (NWI + NPW <= 8 && younger_w + npw <= 8) {
                    if (younger_w + npw == 8) wait_vm<8>(); else if (younger_w + npw == 7) wait_vm<7>();
                    else if (younger_w + npw == 6) wait_vm<6>(); else if (younger_w + npw == 5) wait_vm<5>();
                    else if (younger_w + npw == 4) wait_vm<4>(); else if (younger_w + npw == 3) wait_vm<3>();
                    else if (younger_w + npw == 2) wait_vm<2>(); else if (younger_w + npw == 1) wait_vm<1>();
                    else wait_vm<0>();
                } else {
                    wait_vm<0>();
                }
            } else {
                if (younger_w == 4) wait_vm<4>(); else if (younger_w == 2) wait_vm<2>();
                else if (younger_w == 1) wait_vm<1>(); else wait_vm<0>();
            }
            __syncthreads();
        }
    }

    band_epilogue<T, W, Wp, Mv, FM, FN>(p, acc, lane, wm, wn, (size_t)(b * H + oh0) * W, n0);
}

template <int N>
__device__ __forceinline__ void wait_vmn() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Software-pipelined band kernel: one wave per SIMD (4 waves, 512-register budget), each wave owning
// a 16*FM (pixel rows) x 16*FN (channels) register tile.  Per K-step s = (chunk, tap), K = 64 as two
// MFMA k-halves:
//   [ DMA slice s+2 | (tap 0) DMA next patch ]  [ ds_read k-half 1 frags | 56 MFMA on k-half 0 ]
//   s_waitcnt vmcnt(younger than slice s+1), lgkmcnt(0); s_barrier (raw: no vmcnt(0) drain)
//   [ ds_read next step's k-half 0 frags | 56 MFMA on k-half 1 ]
// so LDS reads always overlap MFMAs, the weight ring keeps two slices in flight across the barrier,
// and every DMA count is static (the last steps re-fetch the final slice / patch into free buffers
// instead of skipping, keeping the vmcnt arithmetic compile-time).
template <bool F16, int W, int TH, int WM, int WN, int FM, int FN, int WS>
__global__ __launch_bounds__(64 * WM * WN, 1) void conv3x3_bandp_kernel(ConvArgs p, int ntn) {
    static_assert(WS == 2 || WS == 3, "weight ring depth");
    constexpr int NW = WM * WN;
    constexpr int BN = 16 * FN * WN;
    constexpr int Wp = W + 2;
    constexpr int P = (TH + 2) * Wp;
    constexpr int P64 = (P + 63) / 64 * 64;
    constexpr int PLANE = P64 * 16;
    constexpr int PATCH = 8 * PLANE;
    constexpr int NPB = P64 / 64;
    constexpr int PI = 8 * NPB;
    static_assert(PI % NW == 0, "patch DMA must split evenly over waves");
    constexpr int NPW = PI / NW;
    static_assert(NPW <= 2 * FN && BN / 8 / NW <= 2 * FN, "at most two DMA pieces per MFMA group");
    constexpr int WSL = BN * 128;
    constexpr int NWI = BN / 8 / NW;
    static_assert(NWI * 8 * NW == BN, "weight slice rows must split evenly over waves");
    static_assert((WS - 2) * NWI + 2 * NPW <= 63, "vmcnt range");
    constexpr int Mv = TH * Wp - 2;
    static_assert(16 * FM * WM >= Mv, "MFMA rows must cover the band");
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [patch0][patch1][wsl0][wsl1][wsl2]

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int H = p.H;
    const int bands = H / TH;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int tn = lid % ntn;
    const int rest = lid / ntn;
    const int band = rest % bands, b = rest / bands;
    const int oh0 = band * TH, n0 = tn * BN;

    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * H * W * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const uint32_t w_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.Npad * p.Kpad * 2);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, w_bytes, 0x00020000);

    // Patch DMA: wave w owns position blocks w*NBW .. w*NBW+NBW-1 (64 positions each) of all 8 channel
    // planes; a piece's plane only changes the source channel offset, carried in soffset.
    static_assert(NPB % NW == 0, "patch position blocks must split evenly over waves");
    constexpr int NBW = NPB / NW;
    uint32_t psrc[NBW];
#pragma unroll
    for (int u = 0; u < NBW; ++u) {
        const int pos = 64 * (wave * NBW + u) + lane;
        const int ih = oh0 - 1 + pos / Wp, iw = pos % Wp - 1;
        const bool ok = pos < P && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        psrc[u] = ok ? (uint32_t)((((b * H + ih) * W + iw) * p.Cx + p.x_off) * 2) : OOB;
    }
    // Weight DMA: piece u covers rows 8*(wave + NW*u) + lane/8 -> a constant row stride per piece.
    const int wrow0 = 8 * wave + (lane >> 3);
    const uint32_t woff0 = (uint32_t)(((n0 + wrow0) * p.Kpad + 8 * ((lane & 7) ^ ((wrow0 >> 1) & 7))) * 2);
    const uint32_t wstride = (uint32_t)(8 * NW * p.Kpad * 2);
    int aoff[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) {
        const int m = 16 * (wm * FM + j) + (lane & 15);
        aoff[j] = (lane >> 4) * PLANE + (m < Mv ? m : 0) * 16;
    }
    int boff[FN], boff1[FN];  // k-half 1 = chunk ^ 4 = byte bit 6 of the swizzled row
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int row = wn * 16 * FN + 16 * i + (lane & 15);
        boff[i] = row * 128 + swzb(row, lane >> 4) * 16;
        boff1[i] = boff[i] ^ 64;
    }

    // one 1-KiB DMA piece of the next chunk's patch / of a weight slice (u < NPW / NWI); the pieces are
    // issued one per 7-MFMA group inside the k-halves so their issue cost hides behind MFMAs
    auto patch_piece = [&](int chunk, int pb, int u) {
        const int c = u % 8, blk = u / 8;
        dma16s(xr, smem + pb * PATCH + c * PLANE + (wave * NBW + blk) * 1024, psrc[blk],
               (uint32_t)(chunk * 64 * 2 + c * 16));
    };
    auto w_piece = [&](int chunk, int tap, int wb, int u) {
        const uint32_t kadd = (uint32_t)((tap * p.Cin + chunk * 64) * 2);
        dma16s(wr, smem + 2 * PATCH + wb * WSL + (wave + NW * u) * 1024, woff0, kadd + u * wstride);
    };
    auto issue_patch = [&](int chunk, int pb) {
#pragma unroll
        for (int u = 0; u < NPW; ++u) patch_piece(chunk, pb, u);
    };
    auto issue_w = [&](int chunk, int tap, int wb) {
#pragma unroll
        for (int u = 0; u < NWI; ++u) w_piece(chunk, tap, wb, u);
    };

    f32x4_t acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    // Fragments: the 7 patch fragments are double-buffered (pA / pB by k-half parity); each of the 8
    // weight fragments is refilled in place for the next k-half right after its last MFMA use.  Every
    // LDS read is (per-lane base) + (compile-time immediate) after the unrolling below.
    frag wf[FN], pA[FM], pB[FM];
    // ring slot of step s = s % WS: with WS = 3 this is tap % 3 (9 % 3 == 0, compile-time); with
    // WS = 2 it is (chunk + tap) & 1 (runtime parity, an add per weight read)
    auto wread = [&](frag& f, int i, int wslot, int kk) {
        f = *(const frag*)(smem + 2 * PATCH + wslot * WSL + (kk ? boff1[i] : boff[i]));
    };
    auto pread = [&](frag (&pf)[FM], int pbuf, int kk, int tap) {
        const int shift = ((tap / 3) * Wp + (tap % 3)) * 16;
        const char* pa = smem + pbuf * PATCH + kk * 4 * PLANE + shift;
#pragma unroll
        for (int j = 0; j < FM; ++j) pf[j] = *(const frag*)(pa + aoff[j]);
    };
    // one k-half: MFMAs on (wf, cur) while the next k-half's patch fragments land in `nxt` and each wf[i]
    // is reloaded (from wslot_n / kk_n) after its 7 MFMAs; `has_next` false on the very last half
    // one k-half: MFMAs on (wf, cur) while the next k-half's patch fragments land in `nxt`, each wf[i] is
    // reloaded (wslot_n / kk_n) after its 7 MFMAs, and DMA piece i (dma(i), i < n_dma) is issued after
    // group i.  Program order keeps LDS reads before the DMAs that may overwrite LDS; the sched-group
    // pattern places one LDS read per MFMA gap in group 0 and one read + one DMA after every group.
    auto half_step = [&](frag (&cur)[FM], frag (&nxt)[FM], bool has_next, int pbuf_n, int wslot_n, int kk_n,
                         int tap_n, int n_dma, auto&& dma) {
        if (has_next) pread(nxt, pbuf_n, kk_n, tap_n);
#pragma unroll
        for (int i = 0; i < FN; ++i) {
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(wf[i], cur[j], acc[i][j]);
            if (has_next) wread(wf[i], i, wslot_n, kk_n);
#pragma unroll
            for (int d = 0; d < (NPW > FN || NWI > FN ? 2 : 1); ++d)
                if (i + d * FN < n_dma) dma(i + d * FN);
        }
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            if (i == 0 && has_next) {
#pragma unroll
                for (int q = 0; q < FM; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
            } else {
                __builtin_amdgcn_sched_group_barrier(0x008, FM, 0);
            }
            if (has_next) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            if (i + FN < n_dma) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
            else if (i < n_dma) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        }
    };

    const int nchunk = p.Cin / 64;
    issue_patch(0, 0);
#pragma unroll
    for (int t = 0; t < WS; ++t) issue_w(0, t, t);
    {  // warm this XCD's L2 with a 1/32 share of the block's weight panel (see conv3x3_band_kernel)
        const uint32_t panel = (uint32_t)BN * p.Kpad * 2;
        const uint32_t share = (panel + 31) / 32;
        const uint32_t base = (uint32_t)n0 * p.Kpad * 2 + (uint32_t)((blockIdx.x / 8) % 32) * share;
        const uint32_t stride = (uint32_t)NW * 64 * 128;
        unsigned dummy;
        for (uint32_t o = (uint32_t)(wave * 64 + lane) * 128; o < share; o += stride) {
            asm volatile("buffer_load_dword %0, %1, %2, 0 offen\n\ts_waitcnt vmcnt(0)"
                         : "=&v"(dummy) : "v"(base + o), "s"(wr) : "memory");
        }
    }
    wait_vmn<0>();
    asm volatile("s_barrier" ::: "memory");
    pread(pA, 0, 0, 0);
#pragma unroll
    for (int i = 0; i < FN; ++i) wread(wf[i], i, 0, 0);

    // one K-step (chunk, tap): slot / slot_n = ring slots of this and the next step
    auto kstep = [&](int chunk, int tap, int pb, bool last_chunk, int slot, int slot_n) {
        // k-half 0: prefetch k-half 1 of this step; at tap 0 the next chunk's patch DMA rides along
        // (the last chunk re-fetches its own patch into the free buffer: static vmcnt counts)
        const int pch = last_chunk ? chunk : chunk + 1;
        half_step(pA, pB, true, pb, slot, 1, tap, tap == 0 ? NPW : 0,
                  [&](int u) { patch_piece(pch, pb ^ 1, u); });
        // slice step+1 (and, before a new chunk, its patch: older) has landed for this wave.
        // Younger: slices step+2 .. step+WS-1 and the patch pieces issued in the last WS-1 steps
        // (at tap 0 of this chunk).
        if (WS == 3) {
            if (tap == 0 || tap == 1) wait_vmn<(WS - 2) * NWI + NPW>();
            else wait_vmn<(WS - 2) * NWI>();
        } else {
            if (tap == 0) wait_vmn<NPW>();
            else wait_vmn<0>();
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // k-half 1: prefetch k-half 0 of the next step; this step's slot (read-complete before the
        // barrier) receives slice step+WS (clamped to the last slice at the tail)
        const bool nxt = tap < 8 || !last_chunk;
        const int tw = tap + WS < 9 ? tap + WS : tap + WS - 9;
        const int cw = tap + WS < 9 ? chunk : chunk + 1;
        const bool okw = cw < nchunk;
        half_step(pB, pA, nxt, tap < 8 ? pb : pb ^ 1, slot_n, 0, tap < 8 ? tap + 1 : 0, NWI,
                  [&](int u) { w_piece(okw ? cw : nchunk - 1, okw ? tw : 8, slot, u); });
    };
    if constexpr (WS == 3) {
        // ring slot of step (chunk, tap) = tap % 3 because 9 % 3 == 0
        for (int chunk = 0; chunk < nchunk; ++chunk) {
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) kstep(chunk, tap, chunk & 1, chunk + 1 == nchunk, tap % 3, (tap + 1) % 3);
        }
    } else {
        // two chunks (18 steps) per iteration: patch buffer and ring slot are compile-time (Cin % 128 == 0)
        for (int c2 = 0; c2 < nchunk; c2 += 2) {
#pragma unroll
            for (int half = 0; half < 2; ++half)
#pragma unroll
                for (int tap = 0; tap < 9; ++tap) {
                    const int st = half * 9 + tap;
                    kstep(c2 + half, tap, half, c2 + half + 1 == nchunk, st & 1, (st + 1) & 1);
                }
        }
    }
    wait_vmn<0>();  // the tail re-fetches must land before the workgroup's LDS is released

    __syncthreads();  // every wave is past its last LDS read before the staging overwrites the ring
    band_epilogue_lds<T, W, Wp, Mv, FM, FN, WM, WN>(p, acc, smem, threadIdx.x, lane, wm, wn,
                                                     (size_t)(b * H + oh0) * W, n0);
}

template <bool F16, int W, int TH, int WM, int WN, int FM, int FN, int WS>
static hipError_t launch_bandp_k(const ConvArgs& a, hipStream_t s) {
    constexpr int BN = 16 * FN * WN;
    constexpr int P64 = ((TH + 2) * (W + 2) + 63) / 64 * 64;
    constexpr int LDS = 2 * 8 * P64 * 16 + WS * BN * 128;
    static_assert(LDS <= 160 * 1024, "band LDS budget");
    auto k = conv3x3_bandp_kernel<F16, W, TH, WM, WN, FM, FN, WS>;
    static bool attr = false;
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
        attr = true;
    }
    const int ntn = (a.Cout + BN - 1) / BN;
    dim3 grid(a.B * (a.H / TH) * ntn);
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, dim3(64 * WM * WN), LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a, ntn);
    else
        hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), LDS, s, a, ntn);
    return hipGetLastError();
}

// Supported bands: (W, TH) with TH*(W+2)-2 <= the variant's MFMA rows.
//   variant 0: 2x4 waves, FM 7, FN 4 -> 224 pixel rows x 256 channels
//   variant 1: 2x4 waves, FM 7, FN 2 -> 224 x 128
//   variant 2: 4x2 waves, FM 4, FN 2 -> 256 x 64
template <bool F16, int W, int TH, int V, int WS>
static hipError_t launch_band_k(const ConvArgs& a, hipStream_t s) {
    constexpr int WM = V == 2 ? 4 : 2, WN = V == 2 ? 2 : 4, FM = V == 2 ? 4 : 7, FN = V == 0 ? 4 : 2;
    constexpr int BN = 16 * FN * WN;
    constexpr int P64 = ((TH + 2) * (W + 2) + 63) / 64 * 64;
    constexpr int LDS = 2 * 8 * P64 * 16 + WS * BN * 128;
    static_assert(LDS <= 160 * 1024, "band LDS budget");
    auto k = conv3x3_band_kernel<F16, W, TH, WM, WN, FM, FN, WS>;
    static bool attr = false;  // opt in to > 64 KiB dynamic LDS once per instantiation
    if (!attr) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
        attr = true;
    }
    const int ntn = (a.Cout + BN - 1) / BN;
    dim3 grid(a.B * (a.H / TH) * ntn);
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, dim3(64 * WM * WN), LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a, ntn);
    else
        hipLaunchKernelGGL(k, grid, dim3(64 * WM * WN), LDS, s, a, ntn);
    return hipGetLastError();
}

}  // namespace

// Applicability: 3x3 / stride 1 / pad 1, Cin % 64 == 0, a supported (W, TH) band, Cout a multiple of
// the variant's BN.  Returns the band config id (see launch_conv_band).
static bool band_legacy() {
    static const bool on = [] { return ab_int("band_legacy", 0) != 0; }();
    return on;
}

bool band_plan(const ConvArgs& a, int* cfg, int* variant) {
    if (a.Kh != 3 || a.Kw != 3 || a.sh != 1 || a.sw != 1 || a.ph != 1 || a.pw != 1) return false;
    if (a.Cin % 64 != 0 || a.Ho != a.H || a.Wo != a.W || a.partial || a.x2) return false;
    int v;
    if (a.Cout % 256 == 0) v = 0;
    else if (a.Cout % 128 == 0) v = 1;
    else if (a.Cout % 64 == 0) v = 2;
    else return false;
    int c;
    if (a.W == 14 && a.H % 14 == 0) c = 0;
    else if (a.W == 28 && a.H % 7 == 0) c = 1;
    else if (a.W == 56 && a.H % 4 == 0) c = 2;
    else if (a.W == 112 && a.H % 2 == 0) c = 3;
    else return false;
    if (c == 0 && v == 2) return false;  // 14x14x64: 196 rows of a 256-row tile, not worth it
    // software-pipelined 4-wave variant 3 = 14x14 x 256 channels.  (A 28x28 instance -- 14-row bands,
    // 4x1 waves, 2-slot ring -- measured 610 TFLOP/s on layer2 vs 692 for the igemm 128x128 tile:
    // half-length blocks in two rounds pay the prologue/epilogue twice; not instantiated.)
    if (!band_legacy() && c == 0 && v == 0) v = 3;
    if ((c == 2 || c == 3) && v != 2) return false;  // 4x58 / 2x114 rows exceed the 224-row variants
    *cfg = c;
    *variant = v;
    return true;
}

template <bool F16>
static hipError_t launch_band_t(const ConvArgs& a, int c, int v, hipStream_t s) {
    // 3: 14x14 images, 2x2 waves of 112 rows x 128 channels, 3-slot weight ring
    if (v == 3) return c == 0 ? launch_bandp_k<F16, 14, 14, 2, 2, 7, 8, 3>(a, s) : hipErrorInvalidValue;
    switch (c * 3 + v) {
        case 0: return launch_band_k<F16, 14, 14, 0, 3>(a, s);
        case 1: return launch_band_k<F16, 14, 14, 1, 3>(a, s);
        case 3: return launch_band_k<F16, 28, 7, 0, 2>(a, s);
        case 4: return launch_band_k<F16, 28, 7, 1, 3>(a, s);
        case 5: return launch_band_k<F16, 28, 7, 2, 3>(a, s);
        case 8: return launch_band_k<F16, 56, 4, 2, 3>(a, s);
        case 11: return launch_band_k<F16, 112, 2, 2, 2>(a, s);
        default: return hipErrorInvalidValue;
    }
}

hipError_t launch_conv_band(const ConvArgs& a, int cfg, int variant, hipStream_t s) {
    return a.f16 ? launch_band_t<true>(a, cfg, variant, s) : launch_band_t<false>(a, cfg, variant, s);
}

}  // namespace fr
