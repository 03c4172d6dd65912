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
//     counters (bounded: spin_limit sleeps) and copies their rows into its halo rows.  A wait that runs
//     out is counted (spin_timeouts), raises the host-mapped fail_host flag, and poisons the part's
//     stage output with NaN, so the image's embedding is NaN rather than a plausible wrong vector
//     (engine.cpp: fr_embed re-runs the forward without split stages, or latches FR_ERR_STAGE).
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
    static constexpr int TROW = C * 4 + 32;          // table row bytes, two 16-B bank slots of padding: the rows
                                                     // of different border classes a fragment's lanes read at
                                                     // once fall on different banks (C * 4 is 0 mod 256 B; one
                                                     // slot would meet the lanes reading 4 channels further on)
    static constexpr int TAB_ROWS_B = 6 * TROW;      // the 6 border classes a part can meet, [6][C] f32 (padded)
    static constexpr int TS = TAB_ROWS_B + C * 4;      // + one row: the PReLU slope of the conv before
    static constexpr int TAB = PATCH_B + NSLOT * SLICE_B;
    static constexpr int FAILED = TAB + 2 * TS;      // int: this part's bounded wait ran out
    static constexpr int LDS = FAILED + 16;
    static constexpr int KSTEPS = (C / 32) * 9;
    static constexpr int NG = C / 64;                // channel groups of 64
    static constexpr int MG = 8 / NG;                // pixel groups
    static constexpr int QPR = PC / 16;              // fragments per stored row
    static constexpr int FM = HR * PC / 16 / MG;     // pixel fragments per wave
    static constexpr int XROW = IW * C;              // exchanged row (elements)
    static constexpr bool TAIL = IW == 28;           // a tail conv can follow (layer2 -> layer3.0.conv1)
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
constexpr int SPIN_LIMIT = 1 << 21;       // default: x s_sleep 1 (64 cycles): ~0.1 s, then the wait has run out
constexpr int SC1 = 16;                   // buffer-load cache policy: sc1 (L1 bypass; gfx940+ cpol bit 4)


typedef __attribute__((address_space(3))) void lds_void;

// threadIdx.x through an empty asm: loop-invariant copy-out addresses are recomputed where they are used
// instead of being hoisted to the kernel's start and spilled across the K loops
__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, soff, 0, 0);
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

// xchg layout: [B][PARTS][which: 0 = first row, 1 = last row][parity][C / 8 planes][IW][8]
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
    const int nconv = 2 * p.nblk;  // the blocks' convs; then p.ntail tail halves (run_tail)
    const int nconv_all = nconv + (G::TAIL ? p.ntail : 0);
    const int total = nconv_all * KSTEPS;

    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)total * SLICE_B), 0x00020000);

    // ---- initial patch: image rows r0-1 .. r0+14 (out-of-image rows and halo columns read as zeros)
    {
        // (the resources span this image only: 32-bit offsets at any batch size)
        const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.x + (size_t)b * IW * IW * C), 0, IW * IW * C * 2, 0x00020000);
        for (int u = 0; u < PATCH_B / 1024 / NW; ++u) {
            const int piece = wave + NW * u, q = piece * 64 + lane;
            const int plane = q / PPOS, pos = q % PPOS, ir = r0 - 1 + pos / PC, ic = pos % PC - 1;
            const uint32_t src = (unsigned)ir < (unsigned)IW && (unsigned)ic < (unsigned)IW
                                     ? (uint32_t)(((ir * IW + ic) * C + plane * 8) * 2)
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

    // Epilogue tables ep[cv][9][C] (bias per border class, class = 3 row class + column class) and
    // slope[cv][C], staged in LDS per conv: slot 0 holds the conv1 biases of the current block (its
    // accumulator seeds), slot 1 the conv2 biases (seeded in conv1's epilogue) plus conv1's slopes.  A part
    // meets 6 classes at most (row classes tbase, tbase + 1: top + interior for part 0, interior + bottom
    // for the others), so a slot holds those 6 rows.  Slot 1 is DMA'd at conv1's start, slot 0 (the next
    // block's) at conv2's start; the K loop's per-step vmcnt waits and barriers complete them.
    const int tbase = part == 0 ? 0 : 1;
    const __amdgpu_buffer_rsrc_t epr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.ep, 0, (uint32_t)((size_t)nconv_all * 9 * C * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t slr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.slope, 0, (uint32_t)((size_t)nconv_all * C * 4), 0x00020000);
    auto issue_tab = [&](int cv, int cv_slope, int slot) {
        char* dst = smem + G::TAB + slot * G::TS;
        int lane = opaque_tid() & 63;  // opaque: the DMA offsets are not hoisted out of the block loop
        if (wave < 6 && lane * 16 < C * 4)  // wave r: table row r (padded rows: one DMA per row)
            dma16s(epr, dst + wave * G::TROW, (uint32_t)(wave * C * 4 + lane * 16), (uint32_t)((cv * 9 + 3 * tbase) * C * 4));
        if (cv_slope >= 0 && wave == NW - 1 && lane * 16 < C * 4)
            dma16s(slr, dst + G::TAB_ROWS_B, (uint32_t)(lane * 16), (uint32_t)(cv_slope * C * 4));
    };
    // table-row byte offset of fragment j's output pixel for this lane: row class (wave-uniform) and
    // column class (the lane's column: left edge, interior, right edge)
    auto tab_row = [&](int j, int ln) {  // ln: an opaque lane copy (keeps LICM from hoisting + spilling)
        const int f = FM * wm + j, q = f % QPR, cl = ln & 15;
        const int rc = (part == 0 && f < QPR) ? 0 : ((part == PARTS - 1 && f >= (HR - 1) * QPR) ? 2 : 1);
        const int cc = (q == 0 && cl == 0) ? 0 : ((q == QPR - 1 && cl == (IW - 1) % 16) ? 2 : 1);
        return ((rc - tbase) * 3 + cc) * G::TROW;
    };
    auto seed_bias = [&](int slot) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const char* t = smem + G::TAB + slot * G::TS;
        const int nl4 = (64 * wn + 4 * (ln >> 4)) * 4;  // + 64 i: the lane's channel bytes in a table row
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int tr = tab_row(j, ln);
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const float4 bb = *(const float4*)(t + tr + nl4 + 64 * i);
                acc[i][j] = (f32x4_t){bb.x, bb.y, bb.z, bb.w};
            }
        }
    };

    issue_w(0, 0);
    issue_w(1, 1);
    issue_w(2, 2);
    issue_tab(0, -1, 0);
    if (threadIdx.x == 0) *(int*)(smem + G::FAILED) = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int spin_limit = p.spin_limit > 0 ? p.spin_limit : (p.spin_limit == 0 ? SPIN_LIMIT : 0);

    const bool has_up = part > 0, has_dn = part < PARTS - 1;
    int* const my_flag = p.flags + b * PARTS + part;
    // Progress counters are never reset: each launch counts on from the value its own counter holds at
    // the start (f0: only this workgroup writes it, and every part of an image has run the same convs in
    // every launch of this stage), so no memset has to precede the launch.  A neighbour's counter
    // reaching f0 + cv + 1 means its conv cv rows are published.
    const int f0 = __hip_atomic_load(my_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const __amdgpu_buffer_rsrc_t xr_x = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.xchg + (size_t)b * PARTS * 2 * 2 * XROW), 0, PARTS * 2 * 2 * XROW * 2, 0x00020000);
    // element offset (within this image's exchange rows) of row `which` of part `pt`, parity `par`
    auto xrow_off = [&](int pt, int which, int par) { return ((pt * 2 + which) * 2 + par) * XROW; };

    // Halo import of conv cv's boundary rows (published by the neighbours at the end of conv cv), issued
    // inside conv cv+1 between positions 1 and 2: wave 0 polls the neighbours' counters, the other waves
    // join it at a barrier, then every wave LDS-DMAs its planes' halo rows (sc1, straight into the patch:
    // one instruction per (plane, row), 512 B on 32 lanes for PC = 32) and returns the count it issued.
    // Positions 2 and 3 leave those DMAs in flight (kstep's halo slack); position 4's wait and barrier
    // complete them before position 5 reads position 6, the first halo tap.
    auto import_halo = [&](int cv) {
        if (wave == 0 && lane < 2 && (lane == 0 ? has_up : has_dn)) {
            const int* nf = my_flag + (lane == 0 ? -1 : 1);
            int it = 0;
            while (p.spin_limit < 0 ||
                   (int)((unsigned)__hip_atomic_load(nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - (unsigned)f0) < cv + 1) {
                if (it++ >= spin_limit) {  // ran out: count it, flag the host, poison this part's output
                    __hip_atomic_fetch_add(p.spin_timeouts, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    *(volatile int*)p.fail_host = 1;
                    *(volatile int*)(smem + G::FAILED) = 1;
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        // raw barrier: __syncthreads() would first drain every wave's in-flight weight DMAs
        asm volatile("s_barrier" ::: "memory");
        int n = 0;
        int ln = lane;
        asm volatile("" : "+v"(ln));  // opaque: the offsets are recomputed per import, not kept live (spills)
        const int pos = ln, px = pos - 1;  // patch column pos <- image column pos - 1 (halo columns: zeros)
        const bool lane_on = pos < PC;
#pragma unroll
        for (int u = 0; u < NPL / NW; ++u) {
            const int pl = wave + NW * u;
#pragma unroll
            for (int side = 0; side < 2; ++side) {
                if (side == 0 ? !has_up : !has_dn) continue;
                const int row = side == 0 ? xrow_off(part - 1, 1, cv & 1) : xrow_off(part + 1, 0, cv & 1);
                const uint32_t off = (unsigned)px < (unsigned)IW ? (uint32_t)((row + (pl * IW + px) * 8) * 2) : OOB;
                char* dst = smem + pl * PLANE_B + (side == 0 ? 0 : (PR - 1) * PC * 16);
                if (lane_on)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr_x, (lds_void*)dst, 16, off, 0, 0, SC1);
                ++n;
            }
        }
        return n;
    };
    int pending = -1;  // conv whose boundary rows are still to be imported (-1: none)

    // the K loop of conv cv over the patch (with the previous conv's halo import and counter publish)
    auto kloop = [&](int cv) __attribute__((always_inline)) {
        pread(pA, pos_cg(0), pos_tap(0));
#pragma unroll
        for (int i = 0; i < FN; ++i) wread(i, 0);  // step 0 of every conv sits in slot 0 (KSTEPS % 3 == 0)
        const int g0 = cv * KSTEPS;
        int halo = 0;
#pragma unroll 1
        for (int cg = 0; cg < C / 32; cg += 2) {
#pragma unroll
            for (int t = 0; t < 18; ++t) {
                if (t == HALO_POS && cg == 0 && pending >= 0) {
                    halo = import_halo(pending);
                    pending = -1;
                }
                const int cgn = t == 17 ? (cg + 2 < C / 32 ? cg + 2 : 0) : cg + pos_cg(t + 1);
                const int tapn = t == 17 ? pos_tap(0) : pos_tap(t + 1);
                const int hs = t == HALO_POS || t == HALO_POS + 1 ? halo : 0;
                if (t & 1) kstep(g0 + cg * 9 + t, t % 3, pB, pA, cgn, tapn, hs);
                else kstep(g0 + cg * 9 + t, t % 3, pA, pB, cgn, tapn, hs);
                // publish the previous conv's boundary rows: step 1's wait (vmcnt(1): everything but the
                // step-0 weight DMA) and barrier have completed every wave's row stores, so the counter can
                // go out without a drain of its own (a vmcnt(0) + barrier after the epilogue also drained
                // the weight ring and cost ~6 % of the stage in a timing build)
                if (t == 1 && cg == 0 && pending >= 0 && threadIdx.x == 0)
                    __hip_atomic_store(my_flag, (int)((unsigned)f0 + (unsigned)(pending + 1)), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            halo = 0;
        }
    };
    auto run_conv = [&](int cv, auto second_tag) {
        constexpr bool second = decltype(second_tag)::value;
        if (!second) {
            seed_bias(0);  // conv2's seed (x + its bias) comes from conv1's epilogue
            if (cv + 1 < nconv_all) issue_tab(cv + 1, cv, 1);
        } else if (cv + 1 < nconv_all) {
            issue_tab(cv + 1, -1, 0);  // the next block's conv1 biases (or the tail's first half)
        }
        kloop(cv);
        // ---- epilogue (every wave is past its last patch read): accumulators -> patch only; the global
        // copies (boundary rows, stage output, intermediates) are read back from the patch afterwards
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        {
            int ln = lane;
            asm volatile("" : "+v"(ln));
            const int cl = ln & 15;
            const char* t2 = smem + G::TAB + G::TS;  // conv2's biases, conv1's slopes
            int tr[FM];
            if (!second) {
#pragma unroll
                for (int j = 0; j < FM; ++j) tr[j] = tab_row(j, ln);
            }
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int n = 64 * wn + 16 * i + 4 * (ln >> 4);
                char* const slot0 = smem + (n >> 3) * PLANE_B + (PC + cl + 1) * 16 + (n & 7) * 2;
                uint2 xin[FM];
                float4 s1;  // conv1: slope - 1, PReLU(v) = v + (s - 1) min(v, 0)
                if (!second) {
                    const float4 sl = *(const float4*)(t2 + G::TAB_ROWS_B + n * 4);
                    s1 = make_float4(sl.x - 1.f, sl.y - 1.f, sl.z - 1.f, sl.w - 1.f);
#pragma unroll
                    for (int j = 0; j < FM; ++j) {
                        const int f = FM * wm + j;
                        xin[j] = *(const uint2*)(slot0 + ((f / QPR) * PC + 16 * (f % QPR)) * 16);
                    }
                }
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    const int f = FM * wm + j, q = f % QPR;
                    char* slot = slot0 + ((f / QPR) * PC + 16 * q) * 16;
                    float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                    if (!second) {
                        v[0] = fmaf(s1.x, min0_raw(v[0]), v[0]);
                        v[1] = fmaf(s1.y, min0_raw(v[1]), v[1]);
                        v[2] = fmaf(s1.z, min0_raw(v[2]), v[2]);
                        v[3] = fmaf(s1.w, min0_raw(v[3]), v[3]);
                    }
                    float o8[8] = {v[0], v[1], v[2], v[3], 0, 0, 0, 0};
                    const uint4 pk = T::pack8(o8);
                    uint2 pk2 = make_uint2(pk.x, pk.y);
                    // lanes past the image's last column write the zero right halo / spare positions
                    if (IW % 16 != 0 && q == QPR - 1 && cl >= IW % 16) pk2 = make_uint2(0u, 0u);
                    if (!second) {
                        float fx[8];
                        T::unpack8(make_uint4(xin[j].x, xin[j].y, 0, 0), fx);
                        const float4 bb = *(const float4*)(t2 + tr[j] + n * 4);
                        acc[i][j] = (f32x4_t){fx[0] + bb.x, fx[1] + bb.y, fx[2] + bb.z, fx[3] + bb.w};
                    }
                    *(uint2*)slot = pk2;
                }
            }
        }
        // the conv's output is in the patch for every wave (the next conv's reads, the copies below)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        const bool exch = cv < nconv_all - 1;  // (with a tail, the last block's rows are its halo)
        if (exch) {
            // boundary rows for the neighbours, plane-major [NPL][IW][8] per row (16-B chunks, positions
            // fastest: conflict-free LDS reads, contiguous stores), sc1 stores (the hand-off rule, header)
            for (int c = opaque_tid(); c < 2 * NPL * IW; c += 64 * NW) {
                const int side = c / (NPL * IW), rem = c - side * (NPL * IW), pl = rem / IW, pos = rem - pl * IW;
                if (side == 0 ? has_up : has_dn) {
                    const uint4 v = *(const uint4*)(smem + pl * PLANE_B + ((side == 0 ? 1 : HR) * PC + pos + 1) * 16);
                    const uint32_t off = (uint32_t)((xrow_off(part, side, cv & 1) + (pl * IW + pos) * 8) * 2);
                    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                    __builtin_amdgcn_raw_buffer_store_b128((u32x4){v.x, v.y, v.z, v.w}, xr_x, off, 0, SC1);
                }
            }
        }
        bf16_t* dbg = nullptr;
        if (p.dbg_x) dbg = second ? p.dbg_x[cv >> 1] : p.dbg_t[cv >> 1];
        bf16_t* const yo = second && cv == nconv - 1 ? p.y : dbg;
        if (yo) {  // the part's rows, NHWC (once per stage; every conv for intermediates)
            // a part whose halo wait ran out writes NaN (16-bit quiet NaN in both dtypes' high half)
            const uint32_t nan_or = *(const volatile int*)(smem + G::FAILED) ? 0x7FC07FC0u : 0u;
            // 16 pixels x 4 planes per wave instruction (16 lanes of one plane read 16 positions: distinct
            // banks; plane-fastest put every lane of a 16-lane group on one bank slot)
            constexpr int NPIX = HR * IW, NIT = (NPIX + 15) / 16 * 16 * NPL;
            for (int c = opaque_tid(); c < NIT; c += 64 * NW) {
                const int r = c >> 6, pix = (r / (NPL / 4)) * 16 + (c & 15), pl = (r % (NPL / 4)) * 4 + ((c >> 4) & 3);
                if (pix >= NPIX) continue;
                const int row = pix / IW, pos = pix - row * IW;
                uint4 v = *(const uint4*)(smem + pl * PLANE_B + ((row + 1) * PC + pos + 1) * 16);
                v.x |= nan_or; v.y |= nan_or; v.z |= nan_or; v.w |= nan_or;
                *(uint4*)(yo + ((size_t)(b * IW + r0 + row) * IW + pos) * C + pl * 8) = v;
            }
            if (dbg && yo != dbg) {
                for (int c = opaque_tid(); c < HR * IW * NPL; c += 64 * NW) {
                    const int pix = c / NPL, pl = c - pix * NPL, row = pix / IW, pos = pix - row * IW;
                    const uint4 v = *(const uint4*)(smem + pl * PLANE_B + ((row + 1) * PC + pos + 1) * 16);
                    *(uint4*)(dbg + ((size_t)(b * IW + r0 + row) * IW + pos) * C + pl * 8) = v;
                }
            }
        }
        if (exch) {
            // the rows are published at the next conv's K-step 1 (above), once every wave's stores are
            // complete; the neighbours' rows are imported at its K-step 2 (import_halo)
            pending = cv;
        }
    };
    // Tail (p.ntail = 2, layer2 -> IResNet100 layer3.0.conv1: 3x3/s1 C -> 2C, border-class bias + PReLU): the
    // conv after the stage reads the stage output, which sits in the patch with its halo rows imported at the
    // first half's K-step 2 (the last block published them); two C-channel halves run as convs nconv and
    // nconv + 1 and store the part's rows to p.y2 ([B][IW][IW][2C]).  Tables as in conv_stage.hip's tail.
    auto run_tail = [&](int cv, int half) __attribute__((always_inline)) {
        if (half == 0) {
            seed_bias(0);
            issue_tab(cv + 1, cv, 1);
        } else {
            seed_bias(1);
            issue_tab(cv, cv, 0);
        }
        kloop(cv);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int cl = ln & 15;
        const char* tsl = smem + G::TAB + (half == 0 ? G::TS : 0) + G::TAB_ROWS_B;
        const uint32_t nan_or = *(const volatile int*)(smem + G::FAILED) ? 0x7FC07FC0u : 0u;
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const int n = 64 * wn + 16 * i + 4 * (ln >> 4);
            const float4 sl = *(const float4*)(tsl + n * 4);
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int f = FM * wm + j, row = f / QPR, col = 16 * (f % QPR) + cl;
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                v[0] = fmaf(sl.x - 1.f, min0_raw(v[0]), v[0]);
                v[1] = fmaf(sl.y - 1.f, min0_raw(v[1]), v[1]);
                v[2] = fmaf(sl.z - 1.f, min0_raw(v[2]), v[2]);
                v[3] = fmaf(sl.w - 1.f, min0_raw(v[3]), v[3]);
                float o8[8] = {v[0], v[1], v[2], v[3], 0, 0, 0, 0};
                const uint4 pk = T::pack8(o8);
                if (col < IW)
                    *(uint2*)(p.y2 + ((size_t)(b * IW + r0 + row) * IW + col) * (2 * C) + half * C + n) =
                        make_uint2(pk.x | nan_or, pk.y | nan_or);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
#pragma unroll 1
    for (int blkc = 0; blkc < p.nblk; ++blkc) {
        run_conv(2 * blkc, std::false_type{});
        run_conv(2 * blkc + 1, std::true_type{});
    }
    if (G::TAIL && p.ntail) {
        run_tail(nconv, 0);
        run_tail(nconv + 1, 1);
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
    // (no flag reset: the counters run on across launches, see f0 in the kernel)
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
    if (a.B <= 0 || !a.xchg || !a.flags || !a.spin_timeouts || !a.fail_host) return hipErrorInvalidValue;
    if (H == Split28::IW && C == Split28::C) return launch_split_t<Split28>(a, s);
    if (H == Split56::IW && C == Split56::C) return launch_split_t<Split56>(a, s);
    return hipErrorInvalidValue;
}

}  // namespace fr
