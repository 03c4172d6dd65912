// Persistent weight-resident 3x3 / stride 1 / pad 1 convolution with 64 input channels: IResNet100 layer1
// (layer1.0.conv1 at 112x112, layer1.{1,2}.conv{1,2} at 56x56, 64 -> 64) and layer2.0.conv1 (56x56,
// 64 -> 128): 13.6 % of the network's FLOPs (insightface IBasicBlock; bn1 folded as a border-class bias).
//
// As an implicit GEMM these convs have K = 576 only: every 128-pixel tile re-gathers its 9 taps from L2
// (9x the activation bytes) and re-streams the weights, and its prologue / epilogue are as long as its
// 9 K-steps, so they ran at 20-25 % of the MFMA peak while their HBM floor is far below that.  Here:
//   * one workgroup per CU (grid = CU count), 4 waves; the n-group's weights (64 output channels x 576,
//     72 KiB, pre-packed as 18 K-step slice images [4 groups of 8 ch][64 rows][16 B]) are DMA'd into LDS
//     once and stay there for all of the workgroup's units;
//   * a unit = 4 output rows x 56 columns of one image (224 pixels = 14 MFMA fragments, no padding;
//     112-wide images are two column halves); its input patch (6 rows x 58 positions x 64 channels,
//     zero halo by out-of-range DMA offsets) is DMA'd into one of two LDS buffers while the previous
//     unit computes (2 x 44 KiB + 72 KiB = exactly 160 KiB);
//   * the 64 channels of a position are one 128-B LDS row whose 16-B chunks are XOR-swizzled with the
//     position (chunk ^ (pos & 7), applied to the DMA's per-lane SOURCE), which makes every fragment
//     read conflict-free for all 9 tap shifts;
//   * 2 x 2 waves: wave (wm, wn) computes pixels [112 wm, 112 wm + 112) x channels [32 wn, 32 wn + 32):
//     7 x 2 fragments, 14 v_mfma_f32_16x16x32 per K-step, 18 K-steps per unit; the K loop has no
//     barrier and no DMA wait (only the unit boundary does);
//   * the accumulators are seeded with the bias of the pixel's border class (and the residual for the
//     block's conv2); those loads for the next unit are issued before the epilogue so their latency
//     overlaps it; the epilogue applies the activation (v > 0 ? v : v * negf), stages the unit's output
//     tile in the finished patch buffer and stores whole 128-B pixel rows, 16 B per lane;
//   * built with -mllvm -amdgpu-mfma-vgpr-form (Makefile): the 56 accumulators live in VGPRs, so the
//     epilogue and the seeding need no AGPR <-> VGPR moves (280 per unit otherwise).
#include "kernels.h"

#include <hip/hip_ext.h>

#include <cstdlib>

namespace fr {
namespace {

constexpr int RCOLS = 56;                                      // output columns per unit
constexpr int RROWS = 4;                                       // output rows per unit
constexpr int PROWS = RROWS + 2;                               // patch rows
constexpr int PPOS = RCOLS + 2;                                // patch positions per row
constexpr int PSLOTS = PROWS * PPOS * 8;                       // 16-B slots of a patch (2784)
constexpr int PPIECES = (PSLOTS + 255) / 256 * 4;              // 1-KiB DMA pieces, a multiple of 4 (44)
constexpr int PATCH_B = PPIECES * 1024;                        // 45056
constexpr int WSLICE_B = 4 * 64 * 16;                          // 4096: one K-step slice
constexpr int NKS = 18;                                        // K-steps (2 channel groups x 9 taps)
constexpr int W_B = NKS * WSLICE_B;                            // 73728
constexpr int ROWS_LDS = W_B + 2 * PATCH_B;                    // 163840 = all of the CU's LDS
constexpr uint32_t OOB = 0x80000000u;

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, 0, 0, 0);
}

struct Unit {
    int b, r0, c0;
};

// unit k of one n-group: (image, row block, column half)
__device__ __forceinline__ Unit unit_of(int k, int H, int W) {
    const int halves = W / RCOLS, rbs = H / RROWS;
    Unit u;
    u.c0 = (k % halves) * RCOLS;
    const int t = k / halves;
    u.r0 = (t % rbs) * RROWS;
    u.b = t / rbs;
    return u;
}

template <bool RES, int ACT>  // ACT: 0 none, 2 PReLU / ReLU (negf = slope or 0)
__global__ __launch_bounds__(256, 1) void conv_rows_kernel(ConvArgs p, int NG, int units) {
    typedef Num<false> T;
    typedef T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [weights 72 KiB][patch 0][patch 1]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const int H = p.H, W = p.W;
    // n-group of this workgroup and its units k = k0, k0 + kstride, ...
    const int ng = blockIdx.x % NG, k0 = blockIdx.x / NG, kstride = gridDim.x / NG;
    if (k0 >= units) return;

    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * H * W * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.wimg + (size_t)ng * (W_B / 2)), 0, (uint32_t)W_B, 0x00020000);

    // ---- DMA of a unit's patch into buffer `buf`: slot q = (row, pos, chunk'), logical 8-channel
    // group = chunk' ^ (pos & 7) (the swizzle lives in the source offset; the DMA destination is linear)
    auto issue_patch = [&](const Unit& u, int buf) {
        int ln = lane;
        asm volatile("" : "+v"(ln));  // opaque: the offsets are recomputed per unit, not kept live
#pragma unroll
        for (int t = 0; t < PPIECES / 4; ++t) {
            const int piece = 4 * t + wave, q = piece * 64 + ln;
            const int row = q / (PPOS * 8), rem = q - row * (PPOS * 8), pos = rem >> 3, ch = rem & 7;
            const int g = ch ^ (pos & 7);
            const int ir = u.r0 - 1 + row, ic = u.c0 - 1 + pos;
            const bool in = q < PSLOTS && (unsigned)ir < (unsigned)H && (unsigned)ic < (unsigned)W;
            const uint32_t off =
                in ? (uint32_t)(((((size_t)u.b * H + ir) * W + ic) * p.Cx + p.x_off + g * 8) * 2) : OOB;
            dma16(xr, smem + W_B + buf * PATCH_B + piece * 1024, off);
        }
    };

    // lane's output pixels (unit-relative): fragment j holds pixel m = 112 wm + 16 j + (lane & 15) =
    // row rr_j, column c_j of the unit, at offset rr_j * W + c_j from the unit's first pixel
    int prr[7], pcc[7], poff[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        const int m = 112 * wm + 16 * j + (lane & 15);
        prr[j] = m / RCOLS;
        pcc[j] = m - prr[j] * RCOLS;
        poff[j] = prr[j] * W + pcc[j];
    }
    const int nl = 64 * ng + 32 * wn + 4 * (lane >> 4);  // + 16 i: the lane's 4 channels of fragment i

    // ---- accumulator seeds of a unit: bias of the output pixel's border class (ep [9][Npad]) plus the
    // residual (RES)
    float4 sb[2][7];
    uint2 sr[2][7];
    auto load_seeds = [&](const Unit& u) {
        const size_t base = ((size_t)u.b * H + u.r0) * W + u.c0;
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const int oh = u.r0 + prr[j], ow = u.c0 + pcc[j];
            const int cls = border_class(oh, ow, H, W);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int n = nl + 16 * i;
                sb[i][j] = *(const float4*)(p.ep + cls * p.Npad + n);
                if (RES) sr[i][j] = *(const uint2*)(p.res + (base + poff[j]) * p.Cres + p.res_off + n);
            }
        }
    };
    f32x4_t acc[2][7];
    auto seed = [&](int i, int j) {
        float4 s = sb[i][j];
        if (RES) {
            float f[8];
            T::unpack8(make_uint4(sr[i][j].x, sr[i][j].y, 0, 0), f);
            s.x += f[0]; s.y += f[1]; s.z += f[2]; s.w += f[3];
        }
        acc[i][j] = (f32x4_t){s.x, s.y, s.z, s.w};
    };

    // ---- prologue: the n-group's weights (18 pieces per wave), the first patch, the first seeds
#pragma unroll
    for (int t = 0; t < W_B / 1024 / 4; ++t) {
        const int piece = 4 * t + wave;
        dma16(wr, smem + piece * 1024, (uint32_t)(piece * 1024 + lane * 16));
    }
    Unit cur = unit_of(k0, H, W);
    issue_patch(cur, 0);
    load_seeds(cur);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 7; ++j) seed(i, j);

    // fragment addresses (unit-independent): B = patch, pixel m of fragment j at tap (dh, dw) reads
    // row rr + dh, position c + dw, 8-channel group 4 cg + (lane >> 4): chunk ((4 cg + g) ^ (pos & 7)),
    // i.e. the cg = 1 address is the cg = 0 one with bit 6 flipped; A = weights, rows 32 wn + 16 i +
    // (lane & 15), group lane >> 4 of slice s
    int pa[7][3];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        const int m = 112 * wm + 16 * j + (lane & 15), rr = m / RCOLS, c = m - rr * RCOLS;
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
            const int pos = c + dw;
            pa[j][dw] = W_B + (rr * PPOS + pos) * 128 + (((lane >> 4) ^ (pos & 7)) * 16);
        }
    }
    const int wa = (lane >> 4) * 1024 + (32 * wn + (lane & 15)) * 16;

    frag fa[2][2], fb[2][7];
    auto read_step = [&](int s, int buf, int sl) {
        const int cg = s / 9, tap = s % 9, dh = tap / 3, dw = tap % 3;
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[sl][i] = *(const frag*)(smem + wa + s * WSLICE_B + i * 256);
#pragma unroll
        for (int j = 0; j < 7; ++j)
            fb[sl][j] = *(const frag*)(smem + ((pa[j][dw] + buf * PATCH_B + dh * (PPOS * 128)) ^ (cg << 6)));
    };

    int buf = 0;
#pragma unroll 1
    for (int k = k0; k < units; k += kstride) {
        const bool has_next = k + kstride < units;
        Unit nxt = has_next ? unit_of(k + kstride, H, W) : cur;
        if (has_next) issue_patch(nxt, buf ^ 1);
        // ---- K loop: 18 steps, the next step's 9 fragments read during this step's 14 MFMAs
        read_step(0, buf, 0);
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            __builtin_amdgcn_sched_barrier(0);
            if (s + 1 < NKS) read_step(s + 1, buf, (s + 1) & 1);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 7; ++j) acc[i][j] = T::mfma(fa[s & 1][i], fb[s & 1][j], acc[i][j]);
            // pinned order: one next-step fragment read behind each of the first 9 MFMAs (left to
            // itself the scheduler sinks each read to just before its use and waits on it there)
            if (s + 1 < NKS) {
#pragma unroll
                for (int q = 0; q < 9; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 5, 0);
            }
        }
        // ---- epilogue: the next unit's seeds load meanwhile
        {
            if (has_next) load_seeds(nxt);
            const size_t base = ((size_t)cur.b * H + cur.r0) * W + cur.c0;
            // every wave is past its K-loop reads of `buf`: it becomes the unit's output staging tile
            // [224 pixels][64 channels] (128-B rows, 16-B chunks swizzled with the pixel: conflict-free
            // 8-B writes), so the global stores below are whole 128-B pixel rows, 16 B per lane (8-B
            // scattered stores took as long as the K loop)
            asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            char* stg = smem + W_B + buf * PATCH_B;
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int nloc = 32 * wn + 16 * i + 4 * (lane >> 4), cl = nloc >> 3, half = (nloc >> 2) & 1;
                float4 nf = make_float4(1.f, 1.f, 1.f, 1.f);
                if (ACT) nf = *(const float4*)(p.negf + 64 * ng + nloc);
#pragma unroll
                for (int j = 0; j < 7; ++j) {
                    const int m = 112 * wm + 16 * j + (lane & 15);
                    float o[8] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3], 0, 0, 0, 0};
                    if (ACT) {
                        o[0] = o[0] > 0.f ? o[0] : o[0] * nf.x;
                        o[1] = o[1] > 0.f ? o[1] : o[1] * nf.y;
                        o[2] = o[2] > 0.f ? o[2] : o[2] * nf.z;
                        o[3] = o[3] > 0.f ? o[3] : o[3] * nf.w;
                    }
                    const uint4 pk = T::pack8(o);
                    *(uint2*)(stg + m * 128 + ((cl ^ (m & 7)) * 16) + half * 8) = make_uint2(pk.x, pk.y);
                    if (has_next) seed(i, j);
                }
            }
            // every load of this unit (the next patch's DMA, then the seeds) has landed before the
            // copy-out stores issue, so the unit's end need not drain them (vmcnt would: gfx950 counts
            // stores in vmcnt, and a load/store mix may retire out of order)
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
            // copy-out: 224 x 8 chunks of 16 B, 8 consecutive lanes per pixel row
#pragma unroll
            for (int q = 0; q < 7; ++q) {
                const int idx = (int)threadIdx.x + 256 * q, m = idx >> 3, cl = idx & 7;
                const int rr = m / RCOLS, c = m - rr * RCOLS;
                const uint4 v = *(const uint4*)(stg + m * 128 + ((cl ^ (m & 7)) * 16));
                *(uint4*)(p.y + (base + rr * W + c) * p.Cy + p.y_off + 64 * ng + cl * 8) = v;
            }
        }
        // every wave is past its copy-out reads of `buf`, which the next iteration's DMA overwrites (the
        // next patch landed before the copy-out; its stores stay in flight)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        cur = nxt;
        buf ^= 1;
    }
}

// Ping-pong variant (FR_AB rows_pp, default): 8 waves = two groups of 4, each with its own patch buffer,
// processing alternate units of the workgroup's list, synchronised by LDS-counter group barriers instead of
// s_barrier.  A SIMD then holds one wave of each group: while one group waits for its patch DMA or runs
// its epilogue and copy-out, the other group's K loop keeps the MFMA pipe busy (the single-group kernel
// above issues all of them from one wave per SIMD, so they add up, per the timing builds of round 2).  No patch
// prefetch within a group (the other group covers the DMA); the group counters live in the unused tail
// of each patch buffer (its DMA lanes past PSLOTS are masked off).
constexpr int PP_SPIN_LIMIT = 1 << 22;  // group-barrier spins (x s_sleep 1) before giving up (a bug, not a wait)

template <bool RES, int ACT>
__global__ __launch_bounds__(512, 1) void conv_rows_pp_kernel(ConvArgs p, int NG, int units) {
    typedef Num<false> T;
    typedef T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [weights 72 KiB][patch 0][patch 1]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = wave >> 2, gw = wave & 3;
    const int wm = gw & 1, wn = gw >> 1;
    const int H = p.H, W = p.W;
    const int ng = blockIdx.x % NG, k0 = blockIdx.x / NG, kstride = gridDim.x / NG;
    if (k0 >= units) return;

    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * H * W * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void*)(p.wimg + (size_t)ng * (W_B / 2)), 0, (uint32_t)W_B, 0x00020000);
    const int pbase = W_B + grp * PATCH_B;  // this group's patch buffer (LDS byte offset)
    typedef __attribute__((address_space(3))) int lds_int;
    lds_int* const gctr = (lds_int*)(uintptr_t)(pbase + PSLOTS * 16);

    // the n-group's weights: 72 pieces over the 8 waves; the group counters start at 0
#pragma unroll
    for (int t = 0; t < W_B / 1024 / 8; ++t) {
        const int piece = 8 * t + wave;
        dma16(wr, smem + piece * 1024, (uint32_t)(piece * 1024 + lane * 16));
    }
    if (lane == 0 && gw == 0) *gctr = 0;
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();

    int gphase = 0;
    // group barrier: every wave's LDS work (and, with vm, its vector-memory ops) done, then the 4 waves meet
    auto gbar = [&](bool vm) {
        if (vm) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        else asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __atomic_fetch_add(gctr, 1, __ATOMIC_RELAXED);
        gphase += 4;
        for (int it = 0; it < PP_SPIN_LIMIT; ++it) {
            if (__atomic_load_n(gctr, __ATOMIC_RELAXED) >= gphase) break;
            __builtin_amdgcn_s_sleep(1);
        }
        asm volatile("" ::: "memory");
    };
    // DMA of a unit's patch into the group's buffer (slots past PSLOTS masked: the counters live there)
    auto issue_patch = [&](const Unit& u) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int t = 0; t < PPIECES / 4; ++t) {
            const int piece = 4 * t + gw, q = piece * 64 + ln;
            const int row = q / (PPOS * 8), rem = q - row * (PPOS * 8), pos = rem >> 3, ch = rem & 7;
            const int g = ch ^ (pos & 7);
            const int ir = u.r0 - 1 + row, ic = u.c0 - 1 + pos;
            const bool in = (unsigned)ir < (unsigned)H && (unsigned)ic < (unsigned)W;
            const uint32_t off =
                in ? (uint32_t)(((((size_t)u.b * H + ir) * W + ic) * p.Cx + p.x_off + g * 8) * 2) : OOB;
            if (q < PSLOTS) dma16(xr, smem + pbase + piece * 1024, off);
        }
    };

    int prr[7], pcc[7], poff[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        const int m = 112 * wm + 16 * j + (lane & 15);
        prr[j] = m / RCOLS;
        pcc[j] = m - prr[j] * RCOLS;
        poff[j] = prr[j] * W + pcc[j];
    }
    const int nl = 64 * ng + 32 * wn + 4 * (lane >> 4);
    int pa[7][3];
#pragma unroll
    for (int j = 0; j < 7; ++j) {
        const int m = 112 * wm + 16 * j + (lane & 15), rr = m / RCOLS, c = m - rr * RCOLS;
#pragma unroll
        for (int dw = 0; dw < 3; ++dw) {
            const int pos = c + dw;
            pa[j][dw] = pbase + (rr * PPOS + pos) * 128 + (((lane >> 4) ^ (pos & 7)) * 16);
        }
    }
    const int wa = (lane >> 4) * 1024 + (32 * wn + (lane & 15)) * 16;
    f32x4_t acc[2][7];
    frag fa[2][2], fb[2][7];
    auto read_step = [&](int s, int sl) {
        const int cg = s / 9, tap = s % 9, dh = tap / 3, dw = tap % 3;
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[sl][i] = *(const frag*)(smem + wa + s * WSLICE_B + i * 256);
#pragma unroll
        for (int j = 0; j < 7; ++j) fb[sl][j] = *(const frag*)(smem + ((pa[j][dw] + dh * (PPOS * 128)) ^ (cg << 6)));
    };

#pragma unroll 1
    for (int k = k0 + grp * kstride; k < units; k += 2 * kstride) {
        const Unit cur = unit_of(k, H, W);
        issue_patch(cur);
        // accumulator seeds: bias of the pixel's border class (+ the residual), loaded while the DMA flies
        {
            const size_t base = ((size_t)cur.b * H + cur.r0) * W + cur.c0;
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                const int cls = border_class(cur.r0 + prr[j], cur.c0 + pcc[j], H, W);
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const int n = nl + 16 * i;
                    float4 sb = *(const float4*)(p.ep + cls * p.Npad + n);
                    if (RES) {
                        const uint2 r = *(const uint2*)(p.res + (base + poff[j]) * p.Cres + p.res_off + n);
                        float f[8];
                        T::unpack8(make_uint4(r.x, r.y, 0, 0), f);
                        sb.x += f[0]; sb.y += f[1]; sb.z += f[2]; sb.w += f[3];
                    }
                    acc[i][j] = (f32x4_t){sb.x, sb.y, sb.z, sb.w};
                }
            }
        }
        gbar(true);  // every wave's patch pieces landed
        read_step(0, 0);
#pragma unroll
        for (int s = 0; s < NKS; ++s) {
            __builtin_amdgcn_sched_barrier(0);
            if (s + 1 < NKS) read_step(s + 1, (s + 1) & 1);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 7; ++j) acc[i][j] = T::mfma(fa[s & 1][i], fb[s & 1][j], acc[i][j]);
            if (s + 1 < NKS) {
#pragma unroll
                for (int q = 0; q < 9; ++q) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 5, 0);
            }
        }
        gbar(false);  // every wave of the group is past its patch reads: the buffer becomes the output tile
        const size_t base = ((size_t)cur.b * H + cur.r0) * W + cur.c0;
        char* stg = smem + pbase;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int nloc = 32 * wn + 16 * i + 4 * (lane >> 4), cl = nloc >> 3, half = (nloc >> 2) & 1;
            float4 nf = make_float4(1.f, 1.f, 1.f, 1.f);
            if (ACT) nf = *(const float4*)(p.negf + 64 * ng + nloc);
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                const int m = 112 * wm + 16 * j + (lane & 15);
                float o[8] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3], 0, 0, 0, 0};
                if (ACT) {
                    o[0] = o[0] > 0.f ? o[0] : o[0] * nf.x;
                    o[1] = o[1] > 0.f ? o[1] : o[1] * nf.y;
                    o[2] = o[2] > 0.f ? o[2] : o[2] * nf.z;
                    o[3] = o[3] > 0.f ? o[3] : o[3] * nf.w;
                }
                const uint4 pk = T::pack8(o);
                *(uint2*)(stg + m * 128 + ((cl ^ (m & 7)) * 16) + half * 8) = make_uint2(pk.x, pk.y);
            }
        }
        gbar(false);  // the output tile is complete
        const int gt = gw * 64 + lane;
#pragma unroll
        for (int q = 0; q < 7; ++q) {
            const int idx = gt + 256 * q, m = idx >> 3, cl = idx & 7;
            const int rr = m / RCOLS, c = m - rr * RCOLS;
            const uint4 v = *(const uint4*)(stg + m * 128 + ((cl ^ (m & 7)) * 16));
            *(uint4*)(p.y + (base + rr * W + c) * p.Cy + p.y_off + 64 * ng + cl * 8) = v;
        }
        gbar(false);  // the copy-out reads are done before the next unit's DMA overwrites the buffer
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// out[ng][s = cg*9 + tap][g][n][e] = w[64 ng + n][tap*64 + 32 cg + 8 g + e]
__global__ __launch_bounds__(256) void rows_pack_kernel(const bf16_t* __restrict__ w, int Kpad, int NG,
                                                        bf16_t* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x, total = NG * NKS * 4 * 64;
    if (i >= total) return;
    const int n = i % 64, g = (i / 64) % 4, s = (i / 256) % NKS, ng = i / (256 * NKS);
    const int cg = s / 9, tap = s % 9;
    *(uint4*)(out + (size_t)i * 8) = *(const uint4*)(w + (size_t)(64 * ng + n) * Kpad + tap * 64 + 32 * cg + 8 * g);
}

}  // namespace

bool rows_supported(const ConvArgs& a) {
    return !a.x2 && a.Kh == 3 && a.Kw == 3 && a.sh == 1 && a.sw == 1 && a.ph == 1 && a.pw == 1 && a.Cin == 64 &&
           a.Cout % 64 == 0 && a.Npad >= a.Cout && a.H == a.Ho && a.W == a.Wo && a.H % RROWS == 0 &&
           a.W % RCOLS == 0 && a.Cx % 8 == 0 && a.x_off % 8 == 0 && a.x_off + 64 <= a.Cx && a.Cy % 8 == 0 &&
           a.y_off % 8 == 0 && a.y_off + a.Cout <= a.Cy && !a.y2 && !a.partial && !a.w8 && !a.y_amax && !a.f16 &&
           a.B > 0 && a.Kpad >= 576 &&
           (!a.res || (a.Cres % 4 == 0 && a.res_off % 4 == 0 && a.res_off + a.Cout <= a.Cres));
}

size_t rows_packed_elems(int Cout) { return (size_t)(Cout / 64) * NKS * 4 * 64 * 8; }

hipError_t rows_pack_weights(const bf16_t* w, int Kpad, int Cout, bf16_t* out, hipStream_t s) {
    const int total = (Cout / 64) * NKS * 4 * 64;
    hipLaunchKernelGGL(rows_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, s, w, Kpad, Cout / 64, out);
    return hipGetLastError();
}

hipError_t launch_conv_rows(const ConvArgs& a, int n_cu, hipStream_t s) {
    if (!rows_supported(a) || !a.wimg || !a.ep || !a.negf) return hipErrorInvalidValue;
    const int NG = a.Cout / 64;
    const int units = a.B * (a.H / RROWS) * (a.W / RCOLS);
    int grid = (n_cu / NG) * NG;                       // every workgroup owns one n-group
    if (grid > units * NG) grid = units * NG;
    const bool act = a.act != 0;
    static const bool pp = [] { return ab_int("rows_pp", 1) != 0; }();
    auto k = pp ? (a.res ? (act ? conv_rows_pp_kernel<true, 2> : conv_rows_pp_kernel<true, 0>)
                         : (act ? conv_rows_pp_kernel<false, 2> : conv_rows_pp_kernel<false, 0>))
                : (a.res ? (act ? conv_rows_kernel<true, 2> : conv_rows_kernel<true, 0>)
                         : (act ? conv_rows_kernel<false, 2> : conv_rows_kernel<false, 0>));
    const int threads = pp ? 512 : 256;
    const int v = (a.res ? 2 : 0) + (act ? 1 : 0);
    static bool attr[4] = {false, false, false, false};
    if (!attr[v]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, ROWS_LDS);
        attr[v] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(grid), dim3(threads), ROWS_LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a, NG,
                              units);
    else
        hipLaunchKernelGGL(k, dim3(grid), dim3(threads), ROWS_LDS, s, a, NG, units);
    return hipGetLastError();
}

}  // namespace fr
