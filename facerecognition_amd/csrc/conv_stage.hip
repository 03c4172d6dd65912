// LDS-resident stage kernel for the stride-1 IBasicBlocks of IResNet100 layer3 (14x14x256).
//
// Replaces, per image, the chain of 2*nblk row-band convolutions of layer3.1 .. layer3.29
// (insightface IBasicBlock: bn1 -> conv3x3 -> bn2 -> PReLU -> conv3x3 -> bn3 -> + identity; the BNs are
// folded into the conv weights by weights.fold_state_dict, bn1 as a border-class bias table).  These
// convs are 55 % of the network's FLOPs.  As separate launches every conv pays a lockstep prologue
// (patch + first weight slices, cold) and a lockstep epilogue (residual read + output write) on all
// 256 CUs at once: measured ~15 us of a ~65 us launch (profiles/r01_*).  A layer3 conv of image b only
// reads image b's previous activation, so one workgroup per image runs the whole stage:
//   * the activation lives in LDS as 14 rows x 16 positions (columns 0 and 15 are the zero left/right
//     halo) of all 256 channels ([32 planes of 8 channels][224 positions][16 B] = 112 KiB); the
//     top/bottom halo rows are not stored: the two (wave, m-frag, tap) combinations that read them
//     (wave-uniform) read the zero slot at position 0 instead; conv1's epilogue writes t =
//     PReLU(conv1(x)) straight into it, after reading x from the same positions to seed conv2's
//     accumulators (the identity), and conv2's epilogue writes x' = (x + conv2(t)) + bias back: no
//     global traffic at all between the first patch load and the last block's NHWC store;
//   * the weights of one K-step (32 input channels x one tap x 256 output channels, 16 KiB, pre-packed
//     as [4 channel groups][256 rows][16 B]) go straight from L2 into registers: each wave loads the
//     four 16-channel A fragments of its 64 output channels (4 x 16 B per lane) into a 3-step register
//     ring, two steps ahead and across conv boundaries.  Every CU runs the same K-step of the same
//     weights at about the same time, so the stream is L2-resident.  The patch is the only LDS data and
//     it is read-only inside a conv: the K loop has no barrier at all (a 3-slot LDS-DMA ring with one
//     mid-step barrier per K-step ran 2.50 ms vs 2.38 ms for this at bs = 256, same box);
//   * 8 waves = 2 pixel halves (7 rows = 7 m-frags of 16 positions, columns 14/15 computed and
//     discarded) x 4 channel groups (64 channels = 4 n-frags): 28 v_mfma_f32_16x16x32_{bf16,f16} per wave
//     per K-step, two waves per SIMD (the second hides the first's LDS and L2 waits); operand A =
//     weight rows, operand B = patch positions, so a lane ends with 4 consecutive channels of one pixel.
#include "kernels.h"

#include <hip/hip_ext.h>

#include <type_traits>

namespace fr {
namespace {

constexpr int SW = 14;                       // image width = height
constexpr int SWP = 16;                      // patch row stride (positions)
constexpr int SC = 256;                      // channels
constexpr int SPIX = SW * SW;                // 196
constexpr int PPOS = SW * SWP;               // 224 stored positions per plane (rows 0..13)
constexpr int PLANE_B = PPOS * 16;           // 3584: one 8-channel plane
constexpr int PATCH_B = (SC / 8) * PLANE_B;  // 114688
constexpr int SLICE_B = 4 * 256 * 16;        // 16384: one K-step of packed weights [4 groups of 8 ch][256 rows][16 B]
constexpr int PAD_B = 256;                   // zeros written by the epilogue's discarded lanes past the patch
constexpr int TAB_ROWS_B = 9 * SC * 4;       // epilogue table: bias per border class [9][256] f32
constexpr int TS = TAB_ROWS_B + SC * 4;      // + the PReLU slopes of the conv before [256]
constexpr int TAB = PATCH_B + PAD_B;
constexpr int STAGE_LDS = TAB + 2 * TS;      // 134400
constexpr int KSTEPS = (SC / 32) * 9;        // 72 per conv
constexpr uint32_t OOB = 0x80000000u;
constexpr int SNW = 8;                       // waves per workgroup: 2 pixel halves x 4 channel groups
constexpr int FN = 4;                        // 16-channel fragments per wave
constexpr int NPW = 16 * FN;                 // output channels per wave

// weight-ring depths (K-steps; loads RING - 1 ahead): the 7-fragment waves of the 13-fragment kernel, which
// wait ~30 % of each conv at the epilogue barrier for the 6-fragment ones, take 2 and fit 256 VGPRs without
// epilogue spills; the 6-fragment waves 3; the one-wave-per-SIMD variant 6
constexpr int RING7 = 2, RING6 = 3, RING13 = 6;

typedef __attribute__((address_space(3))) void lds_void;

// The lane id / thread id recomputed where used (v_mbcnt; volatile, so never hoisted, CSE'd or kept
// live across the conv loop): a long-lived copy of threadIdx.x gets spilled, and each scratch reload
// waits for every outstanding VMEM load (vmcnt(0)), i.e. drains the weight prefetch ring.
__device__ __forceinline__ int fresh_lane() {
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}
__device__ __forceinline__ int opaque_tid() {
    return (__builtin_amdgcn_readfirstlane(threadIdx.x) & ~63) + fresh_lane();
}

template <bool F16>
__global__ __launch_bounds__(64 * SNW, 1) void stage_kernel(StageArgs p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // the patch

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave & 1, wn = wave >> 1;
    const int b = blockIdx.x;
    const int nconv = 2 * p.nblk;
    const int total = nconv * KSTEPS;

    const uint32_t w_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)total * SLICE_B);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, w_bytes, 0x00020000);

    // ---- initial patch: x of this image; the patch is 7168 16-B slots (plane-major), 112 pieces of 64
    {
        // (the resource spans this image only: 32-bit offsets at any batch size)
        const __amdgpu_buffer_rsrc_t xr =
            __builtin_amdgcn_make_buffer_rsrc((void*)(p.x + (size_t)b * SPIX * SC), 0, SPIX * SC * 2, 0x00020000);
        for (int u = 0; u < PATCH_B / 1024 / SNW; ++u) {
            const int piece = wave + SNW * u, q = piece * 64 + lane;
            const int plane = q / PPOS, pos = q - plane * PPOS, r = pos / SWP, c = pos % SWP - 1;
            const uint32_t src = (unsigned)c < (unsigned)SW ? (uint32_t)((((r * SW + c) * SC) + plane * 8) * 2) : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(smem + piece * 1024), 16, src, 0, 0, 0);
        }
    }
    // ---- the pad after the patch (written by discarded lanes) needs no init; first conv1 table below
    // fragment addresses: B (patch) rows m = wm*112 + 16j + (lane&15) at plane (lane>>4) of the group;
    // A (weights) rows n = wn*64 + 16i + (lane&15) in group (lane>>4) of the K-step's packed image
    int aoff[7];
#pragma unroll
    for (int j = 0; j < 7; ++j) aoff[j] = (lane >> 4) * PLANE_B + ((wm * 7 + j) * SWP + (lane & 15)) * 16;
    const int zoff = (lane >> 4) * PLANE_B;  // position 0 = left halo of row 0: a zero slot in every plane
    const uint32_t wvo = (uint32_t)((lane >> 4) * 4096 + (wn * NPW + (lane & 15)) * 16);

    f32x4_t acc[FN][7];
    frag pA[7], pB[7];
    // patch fragments of (cg, tap): output row r = wm*7 + j reads source row r + dh - 1; rows -1 and 14
    // (wave 0 frag 0 at dh = 0, wave 1 frag 6 at dh = 2) are halo -> the zero slot
    auto pread = [&](frag (&pf)[7], int cg, int tap) {
        const int dh = tap / 3, dw = tap % 3;
        const char* pl = smem + cg * 4 * PLANE_B;
        const char* pa = pl + ((dh - 1) * SWP + dw) * 16;
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const char* a = pa + aoff[j];
            if (j == 0 && dh == 0) a = wm == 0 ? pl + zoff : a;
            if (j == 6 && dh == 2) a = wm == 1 ? pl + zoff : a;
            pf[j] = *(const frag*)a;
        }
    };
    // weight fragments of global K-step g: a 3-step register ring, loads two steps ahead.  The ring slot
    // of step g is g % 3 = tap % 3 (9 and 72 are multiples of 3): compile-time after unrolling
    frag wq[3][FN];
    auto wload = [&](frag (&w)[FN], int g) {
#pragma unroll
        for (int i = 0; i < FN; ++i)
            w[i] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(wr, wvo + i * 256, (uint32_t)g * SLICE_B, 0));
    };
    // one K-step: nxt <- patch fragments of (cg_n, tap_n) (after a conv's last step: unused reads, no
    // branch); weights of step g+2 (clamped: the tail re-fetches the last step); 28 MFMAs on (wq[r], cur)
    auto kstep = [&](int g, int r, frag (&cur)[7], frag (&nxt)[7], int cg_n, int tap_n) {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        pread(nxt, cg_n, tap_n);
        wload(wq[(r + 2) % 3], g + 2 < total ? g + 2 : total - 1);
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < 7; ++j) acc[i][j] = T::mfma(wq[r][i], cur[j], acc[i][j]);
    };

    const size_t img = (size_t)b * SPIX * SC;
    // Epilogue tables (built at load time): ep[cv][9][256] = the conv's bias for each border class of the
    // output pixel (bias9 of the folded pre-conv BN, or the plain bias in all 9 rows); slope[cv][256] =
    // the activation's negative-side factor.  Staged in LDS per conv: slot 0 = the conv1 biases of the
    // current block (its accumulator seeds), slot 1 = the conv2 biases (seeded in conv1's epilogue) and
    // conv1's slopes; slot 1 is DMA'd at conv1's start, slot 0 (the next block's) at conv2's start, and
    // both land long before use (loads retire in order; the weight loads behind them are waited on).
    // A lane's 4 channels n..n+3 of fragment i and its column class are fixed, and its output row is
    // interior except for fragment j = 0 of wave row 0 (image row 0) and j = 6 of wave row 1 (row 13).
    const __amdgpu_buffer_rsrc_t epr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.ep, 0, (uint32_t)((size_t)nconv * TAB_ROWS_B), 0x00020000);
    const __amdgpu_buffer_rsrc_t slr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.slope, 0, (uint32_t)((size_t)nconv * SC * 4), 0x00020000);
    auto issue_tab = [&](int cv, int cv_slope, int slot) {
        char* dst = smem + TAB + slot * TS;
        int lane = opaque_tid() & 63;  // opaque: the DMA offsets are not hoisted out of the block loop
#pragma unroll
        for (int u = 0; u < (TAB_ROWS_B / 1024 + SNW - 1) / SNW; ++u) {
            const int piece = wave + SNW * u;
            if (piece < TAB_ROWS_B / 1024)
                __builtin_amdgcn_raw_ptr_buffer_load_lds(epr, (lds_void*)(dst + piece * 1024), 16,
                                                         (uint32_t)(piece * 1024 + lane * 16), (uint32_t)(cv * TAB_ROWS_B), 0, 0);
        }
        if (cv_slope >= 0 && wave == SNW - 1)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(slr, (lds_void*)(dst + TAB_ROWS_B), 16, (uint32_t)(lane * 16),
                                                     (uint32_t)(cv_slope * SC * 4), 0, 0);
    };
    // table-row byte offsets of the lane's output pixels: interior rows, and this wave's border row (the
    // fragment j = 0 / 6 of wave row 0 / 1); ln: an opaque lane copy, keeps LICM from hoisting them
    auto is_edge = [&](int j) { return (j == 0 && wm == 0) || (j == 6 && wm == 1); };
    auto tab_rows = [&](int ln, int& tri, int& tre) {
        const int cc = ln & 15, ccls = cc == 0 ? 0 : (cc == SW - 1 ? 2 : 1);
        tri = (3 + ccls) * SC * 4;
        tre = ((wm ? 6 : 0) + ccls) * SC * 4;
    };
    auto seed_bias = [&]() {
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const char* t = smem + TAB + (wn * NPW + 4 * (ln >> 4)) * 4;
        int tri, tre;
        tab_rows(ln, tri, tre);
#pragma unroll
        for (int j = 0; j < 7; ++j) {
            const int tr = is_edge(j) ? tre : tri;
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const float4 bb = *(const float4*)(t + tr + 64 * i);
                acc[i][j] = (f32x4_t){bb.x, bb.y, bb.z, bb.w};
            }
        }
    };
    issue_tab(0, -1, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    wload(wq[0], 0);
    wload(wq[1], 1);

    auto run_conv = [&](int cv, auto second_tag) {
        constexpr bool second = decltype(second_tag)::value;
        if (!second) {  // conv1 starts from its bias (conv2 from x + its bias, seeded by conv1's epilogue)
            seed_bias();
            if (cv + 1 < nconv) issue_tab(cv + 1, cv, 1);
        } else if (cv + 1 < nconv) {
            issue_tab(cv + 1, -1, 0);  // the next block's conv1 biases
        }
        pread(pA, 0, 0);
        const int g0 = cv * KSTEPS;
#pragma unroll 1
        for (int cg = 0; cg < SC / 32; cg += 2) {
#pragma unroll
            for (int t = 0; t < 18; ++t) {
                const int cgl = cg + t / 9, tap = t % 9;
                const int cgn = t == 8 ? cg + 1 : (t == 17 ? cg + 2 : cgl);
                const int tapn = t == 8 || t == 17 ? 0 : tap + 1;
                if (t & 1) kstep(g0 + cgl * 9 + tap, tap % 3, pB, pA, cgn, tapn);
                else kstep(g0 + cgl * 9 + tap, tap % 3, pA, pB, cgn, tapn);
            }
        }
        // ---- epilogue: every wave is past its last patch read before the patch is overwritten.
        // The accumulators already hold the bias (seeded at conv1's start / by conv1's epilogue), so
        // conv1: t = PReLU(acc) -> patch; the lane first reads x (the same positions and channels it is
        //        about to overwrite -- no other lane touches them) and seeds conv2's accumulators with
        //        x + conv2's bias, so conv2 accumulates onto the identity: x' = x + b2 + conv2(t);
        // conv2: x' -> patch (and NHWC global for the last block / intermediates), no arithmetic.
        // (build_stage checks that every conv1 is PReLU and every conv2 has no activation.)
        // No activation traffic between the stage's first patch load and its last block (global loads:
        // the weight stream and the small epilogue tables).  The barrier only needs every wave's patch
        // reads drained (the weight loads in flight go to registers).
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        int ln = lane;
        asm volatile("" : "+v"(ln));
        const int cc = ln & 15;
        const bool okc = cc < SW;
        const char* t2 = smem + TAB + TS;  // conv2's biases, conv1's slopes
        int tri = 0, tre = 0;
        if (!second) tab_rows(ln, tri, tre);
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const int n = wn * NPW + 16 * i + 4 * (ln >> 4);
            char* slot0 = smem + (n >> 3) * PLANE_B + (wm * 112 + cc + 1) * 16 + (n & 7) * 2;
            // conv1: all 7 identity reads of this n-fragment first (one LDS latency per fragment); lanes of
            // the discarded columns 14/15 read (and later zero) the halo slots
            uint2 xin[7];
            float4 s1;  // conv1: slope - 1, PReLU(v) = v + (s - 1) min(v, 0)
            if (!second) {
                const float4 sl = *(const float4*)(t2 + TAB_ROWS_B + n * 4);
                s1 = make_float4(sl.x - 1.f, sl.y - 1.f, sl.z - 1.f, sl.w - 1.f);
#pragma unroll
                for (int j = 0; j < 7; ++j) xin[j] = *(const uint2*)(slot0 + j * 256);
            }
#pragma unroll
            for (int j = 0; j < 7; ++j) {
                char* slot = slot0 + j * 256;  // position m + 1 = wm*112 + 16j + cc + 1
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                if (!second) {
                    v[0] = fmaf(s1.x, min0_raw(v[0]), v[0]);
                    v[1] = fmaf(s1.y, min0_raw(v[1]), v[1]);
                    v[2] = fmaf(s1.z, min0_raw(v[2]), v[2]);
                    v[3] = fmaf(s1.w, min0_raw(v[3]), v[3]);
                }
                float o8[8] = {v[0], v[1], v[2], v[3], 0, 0, 0, 0};
                const uint4 pk = T::pack8(o8);
                // columns 14/15 write zeros: the right halo, the next row's left halo (past the last row:
                // the pad after the patch)
                const uint2 pk2 = okc ? make_uint2(pk.x, pk.y) : make_uint2(0u, 0u);
                if (!second) {
                    float f[8];
                    T::unpack8(make_uint4(xin[j].x, xin[j].y, 0, 0), f);
                    const float4 bb = *(const float4*)(t2 + (is_edge(j) ? tre : tri) + n * 4);
                    acc[i][j] = (f32x4_t){f[0] + bb.x, f[1] + bb.y, f[2] + bb.z, f[3] + bb.w};
                }
                *(uint2*)slot = pk2;
            }
        }
        // the new activation is visible to every wave before the next conv reads it (and the copies below)
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        bf16_t* dbg = nullptr;
        if (p.dbg_x) dbg = second ? p.dbg_x[cv >> 1] : p.dbg_t[cv >> 1];
        bf16_t* const yo = second && cv == nconv - 1 ? p.y : dbg;
        if (yo) {  // NHWC copies from the patch (the stage output once; intermediates every conv)
            for (int c = opaque_tid(); c < SPIX * (SC / 8); c += 64 * SNW) {
                const int pix = c / (SC / 8), pl = c - pix * (SC / 8), r = pix / SW, col = pix - r * SW;
                const uint4 v = *(const uint4*)(smem + pl * PLANE_B + (r * SWP + col + 1) * 16);
                *(uint4*)(yo + img + (size_t)pix * SC + pl * 8) = v;
            }
            if (dbg && yo != dbg) {
                for (int c = opaque_tid(); c < SPIX * (SC / 8); c += 64 * SNW) {
                    const int pix = c / (SC / 8), pl = c - pix * (SC / 8), r = pix / SW, col = pix - r * SW;
                    const uint4 v = *(const uint4*)(smem + pl * PLANE_B + (r * SWP + col + 1) * 16);
                    *(uint4*)(dbg + img + (size_t)pix * SC + pl * 8) = v;
                }
            }
            // drained here, in this rarely taken branch: with global stores possibly pending at the K loop's
            // head, the compiler's waitcnt pass treats vmcnt as out of order there and emits vmcnt(0) (the whole
            // weight prefetch ring) at every cg-loop head
            __builtin_amdgcn_s_waitcnt(0);
        }
    };
#pragma unroll 1
    for (int blk = 0; blk < p.nblk; ++blk) {
        run_conv(2 * blk, std::false_type{});
        run_conv(2 * blk + 1, std::true_type{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the tail's weight loads retire before the wave ends
}


// ---------------------------------------------------------------------------------------------------
// 13-fragment stage kernel (default).  The 196 pixels of an image are packed into 13 fragments of 16
// (208 slots, 12 spare) instead of one fragment per 16-position row (14 fragments, 2 halo columns each
// computed and discarded): 7 % fewer MFMAs.  The patch stores the halo too, so every tap of every lane is
// base(pixel) + a compile-time shift: no per-lane border selects in the K loop.  Waves 0-3 take
// fragments 0-6, waves 4-7 fragments 7-12 (one body per count): waves w and w + 4 share a SIMD (the
// dispatcher places a workgroup's waves 0->2->1->3 cyclically), so every SIMD runs one 7- and one
// 6-fragment wave, 13 fragments per SIMD (was 14).  Same K-steps, MFMA sequence per output and epilogue
// arithmetic as stage_kernel: bit-identical results (tests/test_gpu_stage.py).
//
// Bank-conflict-free patch reads.  A ds_read_b128 is served in 4 lane groups of 16 lanes (lanes 0-3,12-15
// of one 8-channel plane with lanes 4-11 of the next, and the other way round, MI355X_MICROARCH.md "LDS"),
// one LDS cycle per group iff its 16 lanes hit 16 different 16-B bank slots (byte address / 16 mod 16).
// With 16-position rows (a row = 256 B) the slot is the pixel's column: a fragment of 16 consecutive
// pixels spans two rows and two column pairs collide, every read took 2 cycles per group (r04:
// SQ_LDS_BANK_CONFLICT 52 % of SQ_LDS_IDX_ACTIVE).  Now:
//   * rows are 15 positions (column 14 of a row is column -1 of the next, both zero), so pixel (r, c) sits
//     at position (r + 1) * 15 + c + 1, whose slot is (c - r) mod 16 -- its "residue";
//   * planes are 248 positions (3968 B = 8 slots mod 256 B), so the next plane's lanes land 8 slots over;
//   * a fragment is not a run of pixels but one pixel of every residue (each residue has exactly 12
//     pixels once four are set aside for fragment 12), placed on lanes so that residues x and x + 8 share
//     a lane half (L2R13): in every lane group the 8 lanes of one plane and the 8 of the other then cover
//     all 16 slots.  Fragment 12 holds the 4 set-aside pixels; its 12 spare lanes read free slots (and
//     write nothing).
// Which pixel a lane owns does not change its arithmetic (each output is its own dot product), so the
// results stay bit-identical.
constexpr int RS13 = 15;                        // patch row stride (positions)
constexpr int PPOS13 = 248;                     // positions per plane: 241 used (rows -1..14 + the last halo)
constexpr int PLANE13_B = PPOS13 * 16;          // 3968
constexpr int PATCH13_B = (SC / 8) * PLANE13_B; // 126976
constexpr int TAB13 = PATCH13_B;
// epilogue table in LDS: the 9 border-class bias rows 1024 + 32 B apart (lanes of one lane group whose pixels
// have different classes read different bank slots), then the slopes
constexpr int TROW13 = SC * 4 + 32;             // 1056
constexpr int TSL13 = 9 * TROW13;               // slopes
constexpr int TS13 = TSL13 + SC * 4;            // 10528
constexpr int STAGE13_LDS = TAB13 + 2 * TS13;   // 148032
constexpr int SPARE13 = 0xff;                   // border class of a spare lane

__host__ __device__ constexpr int pix_pos13(int r, int c) { return (r + 1) * RS13 + c + 1; }

// lane -> residue within a full fragment: lanes 0-3,12-15 take residue pairs {x, x + 8} for x = 0..3,
// lanes 4-11 those for x = 4..7
constexpr int L2R13[16] = {0, 8, 1, 9, 4, 12, 5, 13, 6, 14, 7, 15, 2, 10, 3, 11};

struct Map13 {
    uint8_t pos[13][16];  // patch position of lane l's pixel in fragment f
    uint8_t cls[13][16];  // its bias-table border class 3 * rowclass + colclass (SPARE13: spare lane)
    uint8_t pix[13][16];  // its pixel index r * 14 + c (SPARE13: spare lane)
};

__host__ __device__ constexpr int border_cls13(int r, int c) {
    return 3 * (r == 0 ? 0 : (r == SW - 1 ? 2 : 1)) + (c == 0 ? 0 : (c == SW - 1 ? 2 : 1));
}

constexpr Map13 make_map13() {
    Map13 m{};
    int r2l[16] = {};
    for (int l = 0; l < 16; ++l) r2l[L2R13[l]] = l;
    int cnt[16] = {};
    for (int r = 0; r < SW; ++r)
        for (int c = 0; c < SW; ++c) {
            if (r >= SW - 2 && c >= SW - 2) continue;  // (12,12) (12,13) (13,12) (13,13): fragment 12
            const int x = (c - r + 16) & 15, k = cnt[x]++, l = r2l[x];
            m.pos[k][l] = (uint8_t)pix_pos13(r, c);
            m.cls[k][l] = (uint8_t)border_cls13(r, c);
            m.pix[k][l] = (uint8_t)(r * SW + c);
        }
    // fragment 12: residues 0 (lane 0), 1 (lane 2), 0 (lane 4), 15 (lane 11); the spare lanes read
    // residues 2,3,4,5,6,9 (lanes 1,3,12..15) and 2..7 (lanes 5..10) at interior positions 112 + x
    const int vl[4] = {0, 2, 4, 11}, vr[4] = {12, 12, 13, 13}, vc[4] = {12, 13, 13, 12};
    const int sl[12] = {1, 3, 12, 13, 14, 15, 5, 6, 7, 8, 9, 10}, sx[12] = {2, 3, 4, 5, 6, 9, 2, 3, 4, 5, 6, 7};
    for (int i = 0; i < 4; ++i) {
        m.pos[12][vl[i]] = (uint8_t)pix_pos13(vr[i], vc[i]);
        m.cls[12][vl[i]] = (uint8_t)border_cls13(vr[i], vc[i]);
        m.pix[12][vl[i]] = (uint8_t)(vr[i] * SW + vc[i]);
    }
    for (int i = 0; i < 12; ++i) {
        m.pos[12][sl[i]] = (uint8_t)(112 + sx[i]);
        m.cls[12][sl[i]] = (uint8_t)SPARE13;
        m.pix[12][sl[i]] = (uint8_t)SPARE13;
    }
    return m;
}
__constant__ Map13 kMap13 = make_map13();

// compile-time check of the layout: every lane group of every fragment hits 16 different bank slots, and
// the 13 fragments own every pixel exactly once
constexpr bool map13_ok() {
    constexpr Map13 m = make_map13();
    const int half0[8] = {0, 1, 2, 3, 12, 13, 14, 15}, half1[8] = {4, 5, 6, 7, 8, 9, 10, 11};
    for (int f = 0; f < 13; ++f)
        for (int swap = 0; swap < 2; ++swap) {
            bool seen[16] = {};
            for (int i = 0; i < 8; ++i) {
                const int a = (swap ? half1 : half0)[i], b = (swap ? half0 : half1)[i];
                const int sa = m.pos[f][a] % 16, sb = (PPOS13 + m.pos[f][b]) % 16;
                if (seen[sa]) return false;
                seen[sa] = true;
                if (seen[sb]) return false;
                seen[sb] = true;
            }
        }
    int owned[SPIX] = {};
    for (int f = 0; f < 13; ++f)
        for (int l = 0; l < 16; ++l) {
            const int q = m.pos[f][l];
            if (q < 16 || q > 224) return false;  // every tap stays inside the plane
            if (m.cls[f][l] == SPARE13) continue;
            const int r = q / RS13 - 1, c = q % RS13 - 1;
            if (r < 0 || r >= SW || c < 0 || c >= SW || m.cls[f][l] != border_cls13(r, c) || m.pix[f][l] != r * SW + c)
                return false;
            ++owned[r * SW + c];
        }
    for (int i = 0; i < SPIX; ++i)
        if (owned[i] != 1) return false;
    return true;
}
static_assert(map13_ok(), "13-fragment map: bank conflict or pixel not owned exactly once");

// FM pixel fragments per wave starting at fragment f0 x FN 16-channel fragments (channel group wn), NWV waves
template <bool F16, int FM, int NWV, int FN = fr::FN, int RING_ = 0>
__device__ __forceinline__ void stage13_body(const StageArgs& p, char* smem, const int wave, const int lane,
                                             const int wn, const int f0) {
    constexpr int NPW = 16 * FN;  // output channels per wave
    typedef Num<F16> T;
    typedef typename T::frag frag;
    const int b = blockIdx.x;
    const int nconv = 2 * p.nblk;               // the blocks' convs; then p.ntail tail halves (run_tail)
    const int nconv_all = nconv + p.ntail;
    const int total = nconv_all * KSTEPS;
    const uint32_t w_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)total * SLICE_B);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, w_bytes, 0x00020000);

    // ---- initial patch (halo rows and columns read as zeros): 128 pieces of 1 KiB
    {
        // (the resource spans this image only: 32-bit offsets at any batch size)
        const __amdgpu_buffer_rsrc_t xr =
            __builtin_amdgcn_make_buffer_rsrc((void*)(p.x + (size_t)b * SPIX * SC), 0, SPIX * SC * 2, 0x00020000);
        for (int u = 0; u < (PATCH13_B / 1024 + NWV - 1) / NWV; ++u) {
            const int piece = wave + NWV * u, q = piece * 64 + lane;
            if (piece >= PATCH13_B / 1024) break;
            const int plane = q / PPOS13, pos = q - plane * PPOS13, r = pos / RS13 - 1, c = pos % RS13 - 1;
            const uint32_t src = (unsigned)r < (unsigned)SW && (unsigned)c < (unsigned)SW
                                     ? (uint32_t)((((r * SW + c) * SC) + plane * 8) * 2)
                                     : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(smem + piece * 1024), 16, src, 0, 0, 0);
        }
    }
    // B (patch) fragment j: lane (lane & 15)'s pixel of fragment f0 + j at plane (lane >> 4) of the K-step's group
    int aoff[FM];
#pragma unroll
    for (int j = 0; j < FM; ++j) aoff[j] = (lane >> 4) * PLANE13_B + kMap13.pos[f0 + j][lane & 15] * 16;
    const uint32_t wvo = (uint32_t)((lane >> 4) * 4096 + (wn * NPW + (lane & 15)) * 16);

    f32x4_t acc[FN][FM];
    frag pA[FM];
    auto pread = [&](frag (&pf)[FM], int cg, int tap) {
        const char* pa = smem + cg * 4 * PLANE13_B + ((tap / 3 - 1) * RS13 + tap % 3 - 1) * 16;
#pragma unroll
        for (int j = 0; j < FM; ++j) pf[j] = *(const frag*)(pa + aoff[j]);
    };
    constexpr int RING = RING_ ? RING_ : (FM == 13 ? RING13 : (FM == 7 ? RING7 : RING6));
    frag wq[RING][FN];
    auto wload = [&](frag (&w)[FN], int g) {
#pragma unroll
        for (int i = 0; i < FN; ++i)
            w[i] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(wr, wvo + i * 256,
                                                                                  (uint32_t)g * SLICE_B, 0));
    };
    // ONE fragment set, refilled in place -- the 4 MFMAs of fragment j (one per weight fragment),
    // then fragment j of the next step is read into the same registers, 4 (FM - 1) MFMAs of this wave
    // before the next step uses it (the order is pinned: left alone, the scheduler sinks every read to
    // the end of the step and the next step waits for them)
    auto kstep1 = [&](int g, int r, frag (&pf)[FM], int cg_n, int tap_n) {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        wload(wq[(r + RING - 1) % RING], g + RING - 1 < total ? g + RING - 1 : total - 1);
        const char* pa = smem + cg_n * 4 * PLANE13_B + ((tap_n / 3 - 1) * RS13 + tap_n % 3 - 1) * 16;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
#pragma unroll
            for (int i = 0; i < FN; ++i)
                acc[i][j] = T::mfma(wq[r][i], pf[j], acc[i][j]);
            pf[j] = *(const frag*)(pa + aoff[j]);
        }
        __builtin_amdgcn_sched_group_barrier(0x020, FN, 0);
#pragma unroll
        for (int q = 0; q < FM; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
    };

    const size_t img = (size_t)b * SPIX * SC;
    const __amdgpu_buffer_rsrc_t epr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.ep, 0, (uint32_t)((size_t)nconv_all * TAB_ROWS_B), 0x00020000);
    const __amdgpu_buffer_rsrc_t slr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.slope, 0, (uint32_t)((size_t)nconv_all * SC * 4), 0x00020000);
    auto issue_tab = [&](int cv, int cv_slope, int slot) {
        char* dst = smem + TAB13 + slot * TS13;
        int ln = fresh_lane();
#pragma unroll
        for (int u = 0; u < (TAB_ROWS_B / 1024 + NWV - 1) / NWV; ++u) {
            const int piece = wave + NWV * u;
            if (piece < TAB_ROWS_B / 1024)  // piece = class row
                __builtin_amdgcn_raw_ptr_buffer_load_lds(epr, (lds_void*)(dst + piece * TROW13), 16,
                                                         (uint32_t)(piece * 1024 + ln * 16), (uint32_t)(cv * TAB_ROWS_B), 0, 0);
        }
        if (cv_slope >= 0 && wave == NWV - 1)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(slr, (lds_void*)(dst + TSL13), 16, (uint32_t)(ln * 16),
                                                     (uint32_t)(cv_slope * SC * 4), 0, 0);
    };
    // table-row byte offset of the border class of the lane's pixel in fragment j (ln: an opaque lane copy)
    // (a spare lane takes the interior row 4: it only seeds accumulators nobody stores)
    auto tab_row = [&](int j, int ln) {
        const int k = kMap13.cls[f0 + j][ln & 15];
        return (k == SPARE13 ? 4 : k) * TROW13;
    };
    auto seed_bias = [&](int slot) {
        int ln = fresh_lane();
        const char* t = smem + TAB13 + slot * TS13 + (wn * NPW + 4 * (ln >> 4)) * 4;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int tr = tab_row(j, ln);
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const float4 bb = *(const float4*)(t + tr + 64 * i);
                acc[i][j] = (f32x4_t){bb.x, bb.y, bb.z, bb.w};
            }
        }
    };
    issue_tab(0, -1, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    wload(wq[0], 0);
    static_assert(18 % RING == 0, "ring slot = K-step % RING must be compile-time in the 18-step body");
#pragma unroll
    for (int q = 1; q < RING - 1; ++q) wload(wq[q], q);

    // the K loop of conv cv over the patch
    auto kloop = [&](int cv) {
        pread(pA, 0, 0);
        const int g0 = cv * KSTEPS;
#pragma unroll 1
        for (int cg = 0; cg < SC / 32; cg += 2) {
#pragma unroll
            for (int t = 0; t < 18; ++t) {
                const int cgl = cg + t / 9, tap = t % 9;
                const int cgn = t == 8 ? cg + 1 : (t == 17 ? cg + 2 : cgl);
                const int tapn = t == 8 || t == 17 ? 0 : tap + 1;
                const int rs = RING == 3 ? tap % 3 : t % RING;  // = global K-step % RING (72, 9 and 18 are multiples)
                kstep1(g0 + cgl * 9 + tap, rs, pA, cgn, tapn);
            }
        }
    };
    auto run_conv = [&](int cv, auto second_tag) {
        constexpr bool second = decltype(second_tag)::value;
        if (!second) {
            seed_bias(0);
            if (cv + 1 < nconv_all) issue_tab(cv + 1, cv, 1);
        } else if (cv + 1 < nconv_all) {
            issue_tab(cv + 1, -1, 0);
        }
        kloop(cv);
        // ---- epilogue (as stage_kernel's): accumulators -> patch; spare-slot lanes write nothing
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        // Fragment-major: the lane's slot for (j, i) is its B-fragment base aoff[j] moved to the output
        // channel plane (n >> 3 = 8 wn + 2 i + (g >> 1), byte (n & 7) * 2 = (g & 1) * 8), and x (conv1) is
        // read right where it is consumed (preloaded per n-fragment, the 7 x were spilled to scratch)
        int ln = fresh_lane();
        const int cl = ln & 15, g = ln >> 4;
        const char* t2 = smem + TAB13 + TS13;
        const int cb = (NPW / 8 * wn + (g >> 1) - g) * PLANE13_B + (g & 1) * 8;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            char* const sj = smem + aoff[j] + cb;
            const int tr = second ? 0 : tab_row(j, ln);
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int n = wn * NPW + 16 * i + 4 * g;
                char* const slot = sj + 2 * i * PLANE13_B;
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                if (!second) {
                    const float4 sl = *(const float4*)(t2 + TSL13 + n * 4);
                    v[0] = fmaf(sl.x - 1.f, min0_raw(v[0]), v[0]);
                    v[1] = fmaf(sl.y - 1.f, min0_raw(v[1]), v[1]);
                    v[2] = fmaf(sl.z - 1.f, min0_raw(v[2]), v[2]);
                    v[3] = fmaf(sl.w - 1.f, min0_raw(v[3]), v[3]);
                }
                float o8[8] = {v[0], v[1], v[2], v[3], 0, 0, 0, 0};
                const uint4 pk = T::pack8(o8);
                if (!second) {
                    const uint2 xin = *(const uint2*)slot;
                    float f[8];
                    T::unpack8(make_uint4(xin.x, xin.y, 0, 0), f);
                    const float4 bb = *(const float4*)(t2 + tr + n * 4);
                    acc[i][j] = (f32x4_t){f[0] + bb.x, f[1] + bb.y, f[2] + bb.z, f[3] + bb.w};
                }
                if (f0 + j < 12 || kMap13.cls[12][cl] != SPARE13)
                    *(uint2*)slot = make_uint2(pk.x, pk.y);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        bf16_t* dbg = nullptr;
        if (p.dbg_x) dbg = second ? p.dbg_x[cv >> 1] : p.dbg_t[cv >> 1];
        bf16_t* const yo = second && cv == nconv - 1 ? p.y : dbg;
        if (yo) {
            for (int c = opaque_tid(); c < SPIX * (SC / 8); c += 64 * NWV) {
                const int pix = c / (SC / 8), pl = c - pix * (SC / 8);
                const uint4 v = *(const uint4*)(smem + pl * PLANE13_B + pix_pos13(pix / SW, pix % SW) * 16);
                *(uint4*)(yo + img + (size_t)pix * SC + pl * 8) = v;
            }
            if (dbg && yo != dbg) {
                for (int c = opaque_tid(); c < SPIX * (SC / 8); c += 64 * NWV) {
                    const int pix = c / (SC / 8), pl = c - pix * (SC / 8);
                    const uint4 v = *(const uint4*)(smem + pl * PLANE13_B + pix_pos13(pix / SW, pix % SW) * 16);
                    *(uint4*)(dbg + img + (size_t)pix * SC + pl * 8) = v;
                }
            }
            // drained here, in this rarely taken branch: with global stores possibly pending at the K loop's
            // head, the compiler's waitcnt pass treats vmcnt as out of order there and emits vmcnt(0) (the whole
            // weight prefetch ring) at every cg-loop head
            __builtin_amdgcn_s_waitcnt(0);
        }
    };
    // Tail (p.ntail = 2): the next conv in the network reads the stage output, which sits in the patch, as a
    // 3x3/s1 conv 256 -> 512 with a border-class bias and PReLU (IResNet100 layer4.0.conv1): its two 256-channel
    // halves run as convs nconv and nconv + 1 over the same patch and store to p.y2 ([B][196][512]) directly.
    // Tables: the last conv2 DMA'd half 0's bias rows into slot 0; half 0 puts half 1's bias rows and its own
    // slopes into slot 1; half 1 seeds from slot 1 and DMAs its slopes into slot 0.
    auto run_tail = [&](int cv, int half) {
        if (half == 0) {
            seed_bias(0);
            issue_tab(cv + 1, cv, 1);
        } else {
            seed_bias(1);
            issue_tab(cv, cv, 0);
        }
        kloop(cv);
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        int ln = fresh_lane();
        const int cl = ln & 15, g = ln >> 4;
        const char* tsl = smem + TAB13 + (half == 0 ? TS13 : 0) + TSL13;
        bf16_t* const yb = p.y2 + (size_t)blockIdx.x * SPIX * (2 * SC) + half * SC;
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int P = kMap13.pix[f0 + j][cl];
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int n = wn * NPW + 16 * i + 4 * g;
                const float4 sl = *(const float4*)(tsl + n * 4);
                float v[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
                v[0] = fmaf(sl.x - 1.f, min0_raw(v[0]), v[0]);
                v[1] = fmaf(sl.y - 1.f, min0_raw(v[1]), v[1]);
                v[2] = fmaf(sl.z - 1.f, min0_raw(v[2]), v[2]);
                v[3] = fmaf(sl.w - 1.f, min0_raw(v[3]), v[3]);
                float o8[8] = {v[0], v[1], v[2], v[3], 0, 0, 0, 0};
                const uint4 pk = T::pack8(o8);
                if (P != SPARE13) *(uint2*)(yb + (size_t)P * (2 * SC) + n) = make_uint2(pk.x, pk.y);
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
#pragma unroll 1
    for (int blk = 0; blk < p.nblk; ++blk) {
        run_conv(2 * blk, std::false_type{});
        run_conv(2 * blk + 1, std::true_type{});
    }
    if (p.ntail) {
        run_tail(nconv, 0);
        run_tail(nconv + 1, 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool F16>
__global__ __launch_bounds__(64 * SNW, 1) void stage13_kernel(StageArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (wave < 4) stage13_body<F16, 7, SNW>(p, smem, wave, lane, wave, 0);  // fragments 0..6
    else stage13_body<F16, 6, SNW>(p, smem, wave, lane, wave - 4, 7);       // fragments 7..12
}

// One wave per SIMD (variant 2): 4 waves, each all 13 pixel fragments x its 64 output channels (52 MFMAs per
// K-step, accumulators in AGPRs, up to 512 registers per wave).  Every weight fragment is loaded by ONE wave
// per CU (the 8-wave kernel loads each twice, once per pixel half, ~1/3 of a conv apart: two L2 reads) and
// the ring runs 5 K-steps ahead; no second wave shares the SIMD, so none waits at the epilogue barrier
// for its partner's K loop either.
// Channel-split variant (3): 8 waves, each all 13 pixel fragments x 32 output channels (26 MFMAs per K-step).
// Every weight fragment is loaded by ONE wave per CU (the default kernel's waves w and w + 4 load the same 64
// channels for their pixel halves: twice the L2 -> CU weight stream), at the price of twice the patch reads.
template <bool F16>
__global__ __launch_bounds__(64 * SNW, 1) void stage13c_kernel(StageArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    stage13_body<F16, 13, SNW, 2, 3>(p, smem, wave, lane, wave, 0);
}

template <bool F16>
__global__ __launch_bounds__(256, 1) void stage13w_kernel(StageArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    stage13_body<F16, 13, 4>(p, smem, wave, lane, wave, 0);
}

}  // namespace


bool stage_supported(int B, int H, int W, int C) { return B > 0 && H == SW && W == SW && C == SC; }

size_t stage_weight_bytes(int nconv) { return (size_t)nconv * KSTEPS * SLICE_B; }

// Packs one conv's [C][Kpad] row-major weights (K order (kh, kw, c)) into a stage's K-step image:
// step s = cg*9 + tap, [4 groups g][C rows n][8 channels] with channel 32cg + 8g + e (C = 256 here,
// 128 for the layer2 stage, conv_stage28.hip).
void stage_pack_weights(const bf16_t* rows, int Kpad, int C, bf16_t* out) {
    for (int cg = 0; cg < C / 32; ++cg)
        for (int tap = 0; tap < 9; ++tap) {
            bf16_t* s = out + (size_t)(cg * 9 + tap) * 4 * C * 8;
            for (int g = 0; g < 4; ++g)
                for (int n = 0; n < C; ++n)
                    for (int e = 0; e < 8; ++e)
                        s[(g * C + n) * 8 + e] = rows[(size_t)n * Kpad + tap * C + cg * 32 + g * 8 + e];
        }
}

hipError_t launch_stage(const StageArgs& a, hipStream_t s) {
    // variant 1: the legacy 14-fragment kernel; 2: the one-wave-per-SIMD 13-fragment kernel (both
    // bit-identical; FR_OPT_STAGE_VARIANT)
    const int v = a.variant >= 1 && a.variant <= 3 ? a.variant : 0;
    if (a.ntail && (a.ntail != 2 || v == 1 || !a.y2)) return hipErrorInvalidValue;  // the legacy kernel has no tail
    auto k = v == 1   ? (a.f16 ? stage_kernel<true> : stage_kernel<false>)
             : v == 2 ? (a.f16 ? stage13w_kernel<true> : stage13w_kernel<false>)
             : v == 3 ? (a.f16 ? stage13c_kernel<true> : stage13c_kernel<false>)
                      : (a.f16 ? stage13_kernel<true> : stage13_kernel<false>);
    const int lds = v == 1 ? STAGE_LDS : STAGE13_LDS;
    const int threads = v == 2 ? 256 : 64 * SNW;
    static bool attr[8] = {false, false, false, false, false, false, false, false};
    const int ai = 2 * v + (a.f16 ? 1 : 0);
    if (!attr[ai]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr[ai] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(a.B), dim3(threads), lds, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, dim3(a.B), dim3(threads), lds, s, a);
    return hipGetLastError();
}

}  // namespace fr
