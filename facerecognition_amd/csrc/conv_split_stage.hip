// Split LDS-resident stages for the stride-1 IBasicBlocks of IResNet100 layer2 (28x28x128, layer2.1 ..
// layer2.12: 24 convs, 22.9 % of the network's FLOPs) and layer1 (56x56x64, layer1.1 .. layer1.2: 4 convs).
//
// insightface IBasicBlock: bn1 -> conv3x3 -> bn2 -> PReLU -> conv3x3 -> bn3 -> + identity, BNs folded as
// in the layer3 stage (conv_stage.hip).  As separate launches (conv_img.hip / conv_rows.hip) each conv
// pays a cold prologue and a store/reload of the whole activation.  One image's activation (196 KiB /
// 392 KiB) does not fit one CU's 160 KiB LDS, so an image is split into PARTS workgroups of 14 output rows
// each (2 for layer2, 4 for layer1), on PARTS CUs, and each part keeps its rows resident for the stage:
//   * LDS patch: 16 stored rows (halo above, 14 own, halo below) x PC positions (column 0 = the zero left
//     halo, 1..IW = image columns, IW+1 = the zero right halo, the rest spare; PC = 32 / 64) of all C
//     channels, plane-major [C/8 planes][16 x PC positions][16 B] = 128 KiB; 16-pixel fragments never
//     straddle a row (16 | PC), so a virtual pixel v = PC * row + col reads tap (dh, dw) at position
//     v + PC dh + dw;
//   * weights: a 3-slot ring of K-steps (32 input channels x one tap x C output channels, 4 C x 16 B),
//     pre-packed in the LDS image (stage_pack_weights), one LDS-DMA instruction per wave per step (1 KiB,
//     or 512 B on 32 lanes for C = 64), three steps ahead across conv boundaries, one mid-step barrier
//     per K-step.  (Weights straight into registers, the layer3 stage's scheme, was 1.5 % slower for layer2:
//     with 4 pixel groups per channel group every weight byte is loaded by 4 waves);
//   * 8 waves = (8 / NG) pixel groups (7 fragments each) x NG = C / 64 channel groups (4 fragments):
//     28 v_mfma_f32_16x16x32 per wave per K-step, 112 f32 accumulators;
//   * epilogues as in the layer3 stage (conv1: PReLU -> patch, the identity read first and seeded with
//     conv2's bias into the accumulators; conv2: accumulator -> patch), plus the boundary-row exchange:
//     after every conv but the last, each part writes its first row (for the part above) and its last
//     row (for the part below) to xchg, publishes a per-part counter, waits for its neighbours'
//     counters (bounded, overruns counted in spin_timeouts) and copies their rows into its halo rows.
//     Rows are double-buffered by conv parity: a part rewrites a parity only after its neighbours have
//     consumed it (they have published the next conv, which needs it).  The hand-off uses no cache
//     maintenance (MI355X_MICROARCH.md, "valid forms", first row of the sc1 hand-off table; one
//     workgroup per CU, hipMalloc memory): rows are stored sc1 and every storing wave waits for them, a
//     barrier, one lane stores the counter sc1; the neighbour's wave 0 polls it with sc1 loads, the
//     other waves join it at a barrier, and every load of the rows is an sc1 load.  (An agent release +
//     acquire pair, buffer_wbl2 / buffer_inv per exchange per CU, cost 0.3 ms more on layer2.)
// Co-residency: the parts of an image are workgroups 8 PARTS q + 8 p + x (x < 8): 8 ids apart, so under
// the round-robin XCD dispatch they share an XCD, and in dispatch order a waiting part's neighbours are at
// most 8 (PARTS - 1) ids behind it, so the neighbours of every resident workgroup are resident or next in
// line whatever the grid size (layer2 at B = 256: 512 workgroups on 256 CUs = two full rounds).
#include "kernels.h"

#include <hip/hip_ext.h>

#include <algorithm>
#include <type_traits>

namespace fr {
namespace {

template <int IW_, int C_, int PARTS_, int PC_>
struct SplitGeo {
    static constexpr int IW = IW_, C = C_, PARTS = PARTS_, PC = PC_;
    static constexpr int HR = IW / PARTS;            // output rows per workgroup
    static constexpr int PR = HR + 2;                // stored rows
    static constexpr int PPOS = PR * PC;             // positions per plane
    static constexpr int PLANE_B = PPOS * 16;
    static constexpr int NPL = C / 8;                // planes
    static constexpr int PATCH_B = NPL * PLANE_B;
    static constexpr int SLICE_B = 4 * C * 16;       // one K-step: [4 groups of 8 ch][C rows][16 B]
    static constexpr int NSLOT = 3;
    static constexpr int LDS = PATCH_B + NSLOT * SLICE_B;
    static constexpr int KSTEPS = (C / 32) * 9;
    static constexpr int NG = C / 64;                // channel groups of 64
    static constexpr int MG = 8 / NG;                // pixel groups
    static constexpr int QPR = PC / 16;              // fragments per stored row
    static constexpr int FM = HR * PC / 16 / MG;     // pixel fragments per wave
    static constexpr int XROW = IW * C;              // exchanged row (elements)
    static_assert(HR * PARTS == IW && PR == 16 && PC >= IW + 2 && PC % 16 == 0 && FM == 7, "geometry");
    static_assert(KSTEPS % 3 == 0 && (C / 32) % 2 == 0 && (SLICE_B == 8192 || SLICE_B == 4096) && LDS <= 163840,
                  "schedule");
    static_assert(IW * NPL <= 512, "halo import: one 16-B slot per thread and row");
};
typedef SplitGeo<28, 128, 2, 32> Split28;  // layer2: 4 pixel groups x 2 channel groups
typedef SplitGeo<56, 64, 4, 64> Split56;   // layer1: 8 pixel groups x 1 channel group

constexpr int NW = 8;                     // waves
constexpr int FN = 4;                     // channel fragments per wave
constexpr uint32_t OOB = 0x80000000u;
constexpr int SPIN_LIMIT = 1 << 21;       // x s_sleep 1 (64 cycles): ~0.1 s, then counted and abandoned
constexpr int SC1 = 16;                   // buffer-load cache policy: sc1 (L1 bypass; gfx940+ cpol bit 4)

#ifndef FR_SPLIT_EXP
#define FR_SPLIT_EXP 0  // timing-only experiments (WRONG results): 1 exchange rows without the counter
                        // synchronisation, 2 no exchange at all
#endif

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ float4 sel4(bool c, float4 a, float4 b) {
    return make_float4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

// K-step order within a pair of 32-channel groups (18 positions): the 3 dh = 1 taps of both groups first
// (they read own rows only), then dh = 0 and dh = 2 (which also read the halo rows).  The halo rows of a
// conv are imported while positions 2 .. 4 of its first pair run (run_conv).  The weights are packed in
// this order (split_stage_pack_weights).
__host__ __device__ constexpr int pos_cg(int q) { return q < 3 ? 0 : (q < 6 ? 1 : (q < 12 ? 0 : 1)); }
__host__ __device__ constexpr int pos_tap(int q) {
    return q < 6 ? 3 + q % 3 : ((q - 6) % 6 < 3 ? (q - 6) % 6 : 3 + (q - 6) % 6);
}
constexpr int HALO_POS = 2;  // the import is issued between positions 1 and 2 and lands by position 4

// xchg layout: [B][PARTS][which: 0 = first row, 1 = last row][parity][IW][C]
template <typename G>
__host__ __device__ constexpr size_t xchg_elems(int B) { return (size_t)B * G::PARTS * 2 * 2 * G::XROW; }

template <bool F16, typename G>
__global__ __launch_bounds__(64 * NW, 1) void split_stage_kernel(StageArgs p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    constexpr int IW = G::IW, C = G::C, PARTS = G::PARTS, PC = G::PC, HR = G::HR, PR = G::PR, PPOS = G::PPOS;
    constexpr int PLANE_B = G::PLANE_B, NPL = G::NPL, PATCH_B = G::PATCH_B, SLICE_B = G::SLICE_B;
    constexpr int NSLOT = G::NSLOT, KSTEPS = G::KSTEPS, MG = G::MG, QPR = G::QPR, FM = G::FM, XROW = G::XROW;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [patch][slot0][slot1][slot2]

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave % MG, wn = wave / MG;
    const int blk = blockIdx.x;
    const int b = blk / (8 * PARTS) * 8 + (blk & 7), part = (blk >> 3) % PARTS;
    if (b >= p.B) return;  // grid padding (whole images)
    const int r0 = part * HR;
    const int nconv = 2 * p.nblk;
    const int total = nconv * KSTEPS;

    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)total * SLICE_B), 0x00020000);

    // ---- initial patch: image rows r0-1 .. r0+14 (out-of-image rows and halo columns read as zeros)
    {
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)p.x, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * IW * IW * C * 2), 0x00020000);
        for (int u = 0; u < PATCH_B / 1024 / NW; ++u) {
            const int piece = wave + NW * u, q = piece * 64 + lane;
            const int plane = q / PPOS, pos = q % PPOS, ir = r0 - 1 + pos / PC, ic = pos % PC - 1;
            const uint32_t src = (unsigned)ir < (unsigned)IW && (unsigned)ic < (unsigned)IW
                                     ? (uint32_t)((((b * IW + ir) * IW + ic) * C + plane * 8) * 2)
                                     : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(smem + piece * 1024), 16, src, 0, 0, 0);
        }
    }
    // each wave DMAs SLICE_B / 8 bytes of a K-step (lanes beyond that idle: 512 B for C = 64)
    constexpr int WB = SLICE_B / NW;
    auto issue_w = [&](int g, int slot) {
        if (WB == 1024 || lane < WB / 16)
            dma16s(wr, smem + PATCH_B + slot * SLICE_B + wave * WB, (uint32_t)(wave * WB + lane * 16), (uint32_t)g * SLICE_B);
    };
    issue_w(0, 0);
    issue_w(1, 1);
    issue_w(2, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // fragment addresses: B (patch) fragment f = FM wm + j covers virtual pixels 16f + (lane & 15) at plane
    // (lane >> 4) of the K-step's 4-plane group; A (weights) rows n = 64 wn + 16 i + (lane & 15)
    const int aoff = (lane >> 4) * PLANE_B + (16 * FM * wm + (lane & 15)) * 16;
    const int boff = PATCH_B + (lane >> 4) * (C * 16) + (64 * wn + (lane & 15)) * 16;

    f32x4_t acc[FN][FM];
    frag wf[FN], pA[FM], pB[FM];
    auto pread = [&](frag (&pf)[FM], int cg, int tap) {
        const char* a = smem + cg * 4 * PLANE_B + ((tap / 3) * PC + tap % 3) * 16 + aoff;
#pragma unroll
        for (int j = 0; j < FM; ++j) pf[j] = *(const frag*)(a + j * 256);
    };
    auto wread = [&](int i, int slot) { wf[i] = *(const frag*)(smem + boff + slot * SLICE_B + i * 256); };

    // one K-step (the layer3 stage's former schedule): MFMAs of the first half of the weight fragments on
    // `cur` while `nxt` is read; mid-step barrier (the issuing waves' slice g+1 landed, every wave is
    // past its reads of slot g % 3); DMA of slice g+3 into that slot; refills of wf with slice g+1
    // halo: vector-memory ops younger than this step's weight slice that may stay in flight (the halo-row
    // DMAs issued between positions 1 and 2 of a conv's first pair: 0, 1, 2 or 4 per wave)
    auto kstep = [&](int g, int slot, frag (&cur)[FM], frag (&nxt)[FM], int cg_n, int tap_n, int halo) {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        pread(nxt, cg_n, tap_n);
#pragma unroll
        for (int i = 0; i < FN / 2; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(wf[i], cur[j], acc[i][j]);
        // the FM youngest LDS reads are this step's pread(nxt); older refills of slot `slot` must be done
        if (halo == 0) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(7)\n\ts_barrier" ::: "memory");
        else if (halo == 1) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(7)\n\ts_barrier" ::: "memory");
        else if (halo == 2) asm volatile("s_waitcnt vmcnt(3) lgkmcnt(7)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(5) lgkmcnt(7)\n\ts_barrier" ::: "memory");
        issue_w(g + 3 < total ? g + 3 : total - 1, slot);
        const int nslot = slot == NSLOT - 1 ? 0 : slot + 1;
#pragma unroll
        for (int i = 0; i < FN / 2; ++i) wread(i, nslot);
#pragma unroll
        for (int i = FN / 2; i < FN; ++i) {
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(wf[i], cur[j], acc[i][j]);
            wread(i, nslot);
        }
    };

    // Epilogue tables ep[cv][9][C] (bias per border class) / slope[cv][C], as in the layer3 stage.
    // Fragment f = FM wm + j lies in row f / QPR, columns 16 (f % QPR) + (lane & 15): its column class
    // is left for f % QPR == 0 and lane column 0, right for f % QPR == QPR - 1 at column IW - 1, else
    // interior; its row class is the image border only for the first row of part 0 and the last row of
    // the last part.  Per channel fragment i a lane needs 6 biases: {interior, border row} x {first,
    // middle, last fragment of a row}.
    auto load_ep = [&](int cv, int i, float4 (&e)[6]) {
        int ln = lane;
        asm volatile("" : "+v"(ln));  // opaque copy: the addresses are not hoisted into the K loop
        const int cl = ln & 15, ccf = cl == 0 ? 0 : 1, ccl = cl == (IW - 1) % 16 ? 2 : 1;
        const int br = part == 0 ? 0 : 6;  // border-row class of this part (used by part 0 / the last part)
        const float* ep = p.ep + (size_t)cv * 9 * C + 64 * wn + 16 * i + 4 * (ln >> 4);
        e[0] = *(const float4*)(ep + (3 + ccf) * C);
        e[2] = *(const float4*)(ep + (3 + ccl) * C);
        e[3] = *(const float4*)(ep + (br + ccf) * C);
        e[5] = *(const float4*)(ep + (br + ccl) * C);
        if (QPR > 2) {  // rows with interior-only fragments
            e[1] = *(const float4*)(ep + 4 * C);
            e[4] = *(const float4*)(ep + (br + 1) * C);
        } else {
            e[1] = e[4] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
    };
    auto pick = [&](const float4 (&e)[6], int j) {
        const int f = FM * wm + j, q = f % QPR;
        const bool border = (part == 0 && f < QPR) || (part == PARTS - 1 && f >= (HR - 1) * QPR);
        // component selects on values: a dynamic index, or a select of element addresses, would keep
        // e in scratch memory
        const float4 e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3], e4 = e[4], e5 = e[5];
        const float4 in = sel4(q == 0, e0, QPR > 2 ? sel4(q == QPR - 1, e2, e1) : e2);
        const float4 bo = sel4(q == 0, e3, QPR > 2 ? sel4(q == QPR - 1, e5, e4) : e5);
        return sel4(border, bo, in);
    };
    auto seed_bias = [&](int cv) {
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            float4 e[6];
            load_ep(cv, i, e);
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const float4 bb = pick(e, j);
                acc[i][j] = (f32x4_t){bb.x, bb.y, bb.z, bb.w};
            }
        }
    };

    const bool has_up = part > 0, has_dn = part < PARTS - 1;
    int* const my_flag = p.flags + b * PARTS + part;
    const __amdgpu_buffer_rsrc_t xr_x = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.xchg, 0, (uint32_t)min((size_t)0x7fffffff, xchg_elems<G>(p.B) * 2), 0x00020000);
    // element offset of row `which` of part `pt`, parity `par`
    auto xrow_off = [&](int pt, int which, int par) { return (((size_t)(b * PARTS + pt) * 2 + which) * 2 + par) * XROW; };

    // Halo import of conv cv's boundary rows (published by the neighbours at the end of conv cv), issued
    // inside conv cv+1 between positions 1 and 2: wave 0 polls the neighbours' counters, the other waves
    // join it at a barrier, then every wave LDS-DMAs its planes' halo rows (sc1, straight into the patch:
    // one instruction per (plane, row), 512 B on 32 lanes for PC = 32) and returns the count it issued.
    // Positions 2 and 3 leave those DMAs in flight (kstep's halo slack); position 4's wait and barrier
    // complete them before position 5 reads position 6, the first halo tap.
    auto import_halo = [&](int cv) {
        if (wave == 0 && lane < 2 && !(FR_SPLIT_EXP & 1) && (lane == 0 ? has_up : has_dn)) {
            const int* nf = my_flag + (lane == 0 ? -1 : 1);
            int it = 0;
            while (__hip_atomic_load(nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cv + 1) {
                if (++it == SPIN_LIMIT) {
                    __hip_atomic_fetch_add(p.spin_timeouts, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        // raw barrier: __syncthreads() would first drain every wave's in-flight weight DMAs
        asm volatile("s_barrier" ::: "memory");
        int n = 0;
        const int pos = lane, px = pos - 1;  // patch column pos <- image column pos - 1 (halo columns: zeros)
        const bool lane_on = pos < PC;
#pragma unroll
        for (int u = 0; u < NPL / NW; ++u) {
            const int pl = wave + NW * u;
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                if (side == 0 ? !has_up : !has_dn) continue;
                const size_t row = side == 0 ? xrow_off(part - 1, 1, cv & 1) : xrow_off(part + 1, 0, cv & 1);
                const uint32_t off = (unsigned)px < (unsigned)IW ? (uint32_t)((row + px * C + pl * 8) * 2) : OOB;
                char* dst = smem + pl * PLANE_B + (side == 0 ? 0 : (PR - 1) * PC * 16);
                if (lane_on)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr_x, (lds_void*)dst, 16, off, 0, 0, SC1);
                ++n;
            }
        }
        return n;
    };
    int pending = -1;  // conv whose boundary rows are still to be imported (-1: none)

    auto run_conv = [&](int cv, auto second_tag) {
        constexpr bool second = decltype(second_tag)::value;
        if (!second) seed_bias(cv);  // conv2's seed (x + its bias) comes from conv1's epilogue
        pread(pA, pos_cg(0), pos_tap(0));
#pragma unroll
        for (int i = 0; i < FN; ++i) wread(i, 0);  // step 0 of every conv sits in slot 0 (KSTEPS % 3 == 0)
        const int g0 = cv * KSTEPS;
        int halo = 0;
#pragma unroll 1
        for (int cg = 0; cg < C / 32; cg += 2) {
#pragma unroll
            for (int t = 0; t < 18; ++t) {
                if (t == HALO_POS && cg == 0 && pending >= 0 && !(FR_SPLIT_EXP & 2)) {
                    halo = import_halo(pending);
                    pending = -1;
                }
                const int cgn = t == 17 ? (cg + 2 < C / 32 ? cg + 2 : 0) : cg + pos_cg(t + 1);
                const int tapn = t == 17 ? pos_tap(0) : pos_tap(t + 1);
                const int hs = t == HALO_POS || t == HALO_POS + 1 ? halo : 0;
                if (t & 1) kstep(g0 + cg * 9 + t, t % 3, pB, pA, cgn, tapn, hs);
                else kstep(g0 + cg * 9 + t, t % 3, pA, pB, cgn, tapn, hs);
            }
            halo = 0;
        }
        // ---- epilogue (every wave is past its last patch read)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int cl = ln & 15;
        bf16_t* dbg = nullptr;
        if (p.dbg_x) dbg = second ? p.dbg_x[cv >> 1] : p.dbg_t[cv >> 1];
        const bool store_y = second && cv == nconv - 1;
        const bool exch = cv < nconv - 1;
        bf16_t* const xo_up = p.xchg + xrow_off(part, 0, cv & 1);  // first row, for the part above
        bf16_t* const xo_dn = p.xchg + xrow_off(part, 1, cv & 1);  // last row, for the part below
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const int n = 64 * wn + 16 * i + 4 * (ln >> 4);
            uint2 xin[FM];
            float4 sl, e[6];  // conv1: this fragment's slope and conv2's biases (its accumulator seed)
            if (!second) {
                load_ep(cv + 1, i, e);
                sl = *(const float4*)(p.slope + (size_t)cv * C + n);
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    const int f = FM * wm + j, col = 16 * (f % QPR) + cl;
                    const char* slot = smem + (n >> 3) * PLANE_B + ((f / QPR + 1) * PC + col + 1) * 16 + (n & 7) * 2;
                    xin[j] = col < IW ? *(const uint2*)slot : make_uint2(0u, 0u);
                }
            }
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int f = FM * wm + j, row = f / QPR, col = 16 * (f % QPR) + cl;
                char* slot = smem + (n >> 3) * PLANE_B + ((row + 1) * PC + col + 1) * 16 + (n & 7) * 2;
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                if (!second) {  // PReLU: max(v, 0) + s * min(v, 0)
                    v[0] = fmaf(sl.x, fminf(v[0], 0.f), fmaxf(v[0], 0.f));
                    v[1] = fmaf(sl.y, fminf(v[1], 0.f), fmaxf(v[1], 0.f));
                    v[2] = fmaf(sl.z, fminf(v[2], 0.f), fmaxf(v[2], 0.f));
                    v[3] = fmaf(sl.w, fminf(v[3], 0.f), fmaxf(v[3], 0.f));
                }
                float o8[8] = {v[0], v[1], v[2], v[3], 0, 0, 0, 0};
                const uint4 pk = T::pack8(o8);
                const uint2 pk2 = make_uint2(pk.x, pk.y);
                if (!second) {
                    float fx[8];
                    T::unpack8(make_uint4(xin[j].x, xin[j].y, 0, 0), fx);
                    const float4 bb = pick(e, j);
                    acc[i][j] = (f32x4_t){fx[0] + bb.x, fx[1] + bb.y, fx[2] + bb.z, fx[3] + bb.w};
                }
                if (col < IW) {
                    *(uint2*)slot = pk2;
                    const size_t go = ((size_t)(b * IW + r0 + row) * IW + col) * C + n;
                    if (store_y) *(uint2*)(p.y + go) = pk2;
                    if (dbg) *(uint2*)(dbg + go) = pk2;
                    // boundary rows for the neighbours: sc1 stores (the hand-off rule, header)
                    const uint64_t pk64 = (uint64_t)pk2.x | ((uint64_t)pk2.y << 32);
                    if (exch && has_up && row == 0)
                        __hip_atomic_store((uint64_t*)(xo_up + col * C + n), pk64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (exch && has_dn && row == HR - 1)
                        __hip_atomic_store((uint64_t*)(xo_dn + col * C + n), pk64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        if (exch && !(FR_SPLIT_EXP & 2)) {
            // publish: every storing wave's rows are complete, a barrier, one sc1 counter store; the
            // neighbours' rows are imported during the next conv (import_halo)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0 && !(FR_SPLIT_EXP & 1))
                __hip_atomic_store(my_flag, cv + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pending = cv;
        }
        // the new activation is visible to every wave before the next conv reads it
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
#pragma unroll 1
    for (int blkc = 0; blkc < p.nblk; ++blkc) {
        run_conv(2 * blkc, std::false_type{});
        run_conv(2 * blkc + 1, std::true_type{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail DMAs land before the LDS is released
}

template <typename G>
hipError_t launch_split_t(const StageArgs& a, hipStream_t s) {
    auto k = a.f16 ? split_stage_kernel<true, G> : split_stage_kernel<false, G>;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
        attr[a.f16 ? 1 : 0] = true;
    }
    hipError_t e = hipMemsetAsync(a.flags, 0, (size_t)G::PARTS * a.B * sizeof(int), s);
    if (e != hipSuccess) return e;
    const dim3 grid((a.B + 7) / 8 * 8 * G::PARTS);
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, dim3(64 * NW), G::LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, grid, dim3(64 * NW), G::LDS, s, a);
    return hipGetLastError();
}

}  // namespace

// Per conv: pairs of 32-channel groups, 18 positions each in the pos_cg / pos_tap order, each position the
// K-step image [4 groups g][C rows n][8 channels] of channels 32 (2 pair + pos_cg) + 8 g + e at tap pos_tap.
void split_stage_pack_weights(const bf16_t* rows, int Kpad, int C, bf16_t* out) {
    for (int pair = 0; pair < C / 64; ++pair)
        for (int q = 0; q < 18; ++q) {
            const int cg = 2 * pair + pos_cg(q), tap = pos_tap(q);
            bf16_t* s = out + (size_t)(pair * 18 + q) * 4 * C * 8;
            for (int g = 0; g < 4; ++g)
                for (int n = 0; n < C; ++n)
                    for (int e = 0; e < 8; ++e)
                        s[(g * C + n) * 8 + e] = rows[(size_t)n * Kpad + tap * C + cg * 32 + g * 8 + e];
        }
}

int split_stage_parts(int H, int W, int C) {
    if (H == Split28::IW && W == Split28::IW && C == Split28::C) return Split28::PARTS;
    if (H == Split56::IW && W == Split56::IW && C == Split56::C) return Split56::PARTS;
    return 0;
}

size_t split_stage_weight_bytes(int C, int nconv) { return (size_t)nconv * (C / 32) * 9 * 4 * C * 16; }

size_t split_stage_xchg_elems(int B) { return std::max(xchg_elems<Split28>(B), xchg_elems<Split56>(B)); }

hipError_t launch_split_stage(const StageArgs& a, int H, int C, hipStream_t s) {
    if (a.B <= 0 || !a.xchg || !a.flags || !a.spin_timeouts) return hipErrorInvalidValue;
    if (H == Split28::IW && C == Split28::C) return launch_split_t<Split28>(a, s);
    if (H == Split56::IW && C == Split56::C) return launch_split_t<Split56>(a, s);
    return hipErrorInvalidValue;
}

}  // namespace fr
