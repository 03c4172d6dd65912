// Split LDS-resident stage for the stride-1 IBasicBlocks of IResNet100 layer2 (28x28x128).
//
// layer2.1 .. layer2.12 are 24 3x3 convs on 28x28x128 (22.9 % of the network's FLOPs; insightface
// IBasicBlock: bn1 -> conv3x3 -> bn2 -> PReLU -> conv3x3 -> bn3 -> + identity, BNs folded as in the
// layer3 stage, conv_stage.hip).  As separate launches (conv_img.hip) each conv pays a cold prologue and
// a store/reload of the 51 MB activation.  One image's activation (28 x 28 x 128 bf16 = 196 KiB) does
// not fit one CU's 160 KiB LDS, so an image is split into two workgroups of 14 output rows each, on two
// CUs, and the halves keep their rows resident for the whole stage:
//   * LDS patch: 16 stored rows (halo above, 14 own, halo below) x 32 positions (column 0 and 29 = the
//     zero left/right halo, 1..28 = image columns, 30..31 spare) of all 128 channels, plane-major
//     [16 planes of 8 channels][512 positions][16 B] = 128 KiB; 16-pixel fragments never straddle a row
//     (32 | 16 * 2), so a virtual pixel v = 32 * row + col reads tap (dh, dw) at position v + 32 dh + dw;
//   * weights: a 3-slot ring of 8 KiB K-steps (32 input channels x one tap x 128 output channels),
//     pre-packed in the LDS image (stage_pack_weights), one 1-KiB DMA piece per wave per K-step, three
//     steps ahead across conv boundaries (the layer3 stage's schedule: one mid-step barrier per step);
//   * 8 waves = 4 pixel groups (7 fragments = 3.5 rows each) x 2 channel groups (64 channels, 4
//     fragments): 28 v_mfma_f32_16x16x32 per wave per K-step, 112 f32 accumulators;
//   * epilogues as in the layer3 stage (conv1: PReLU -> patch, the identity read first and seeded with
//     conv2's bias into the accumulators; conv2: accumulator -> patch), plus the boundary-row exchange:
//     after every conv but the last, each half writes the row its partner needs (half 0: row 13, half 1:
//     row 14 of the image) to xchg, publishes a per-half counter with an agent-scope release, waits for
//     the partner's counter (acquire; bounded, overruns counted in spin_timeouts) and copies the
//     partner's row into its halo row.  Rows are double-buffered by conv parity: a half rewrites a
//     parity only after the partner has consumed it (it has published the next conv, which needs it).
// Co-residency: the two halves of an image are workgroups 16q + x and 16q + 8 + x (x < 8): 8 ids apart,
// so under the round-robin XCD dispatch they share an XCD (and its L2), and in dispatch order a waiting
// half's partner is at most 8 ids behind it, so the partners of every resident workgroup are resident or
// next in line whatever the grid size (B = 256: 512 workgroups on 256 CUs = two full rounds).
#include "kernels.h"

#include <hip/hip_ext.h>

#include <type_traits>

namespace fr {
namespace {

constexpr int IW = 28;                   // image width = height
constexpr int HR = 14;                   // output rows per workgroup
constexpr int C = 128;                   // channels
constexpr int PC = 32;                   // patch row stride (positions)
constexpr int PR = HR + 2;               // stored rows
constexpr int PPOS = PR * PC;            // 512 positions per plane
constexpr int PLANE_B = PPOS * 16;       // 8192
constexpr int NPL = C / 8;               // 16 planes
constexpr int PATCH_B = NPL * PLANE_B;   // 131072
constexpr int SLICE_B = 4 * C * 16;      // 8192: [4 groups of 8 ch][128 rows][16 B]
constexpr int NSLOT = 3;
constexpr int LDS_B = PATCH_B + NSLOT * SLICE_B;  // 155648
constexpr int KSTEPS = (C / 32) * 9;     // 36 per conv
constexpr int NW = 8;                    // waves
constexpr int FM = 7, FN = 4;            // pixel / channel fragments per wave
constexpr int XROW = IW * C;             // exchanged row (elements)
constexpr uint32_t OOB = 0x80000000u;
constexpr int SPIN_LIMIT = 1 << 21;      // x s_sleep 1 (64 cycles): ~0.1 s, then counted and abandoned

constexpr int SC1 = 16;                  // buffer-load cache policy: sc1 (L1 bypass; gfx940+ cpol bit 4)

#ifndef FR_S28_EXP
#define FR_S28_EXP 0  // timing-only experiments (WRONG results): 1 exchange rows without the flag
                      // synchronisation, 2 no exchange at all
#endif

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, soff, 0, 0);
}

__device__ __forceinline__ float4 sel4(bool c, float4 a, float4 b) {
    return make_float4(c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z, c ? a.w : b.w);
}

__host__ __device__ constexpr size_t stage28_xchg_bytes(int B) { return (size_t)B * 2 * 2 * XROW * 2; }

template <bool F16>
__global__ __launch_bounds__(64 * NW, 1) void stage28_kernel(StageArgs p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [patch][slot0][slot1][slot2]

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave & 3, wn = wave >> 2;
    const int blk = blockIdx.x;
    const int b = (blk >> 4) * 8 + (blk & 7), half = (blk >> 3) & 1;
    if (b >= p.B) return;  // grid padding (whole pairs)
    const int r0 = half * HR;
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
    auto issue_w = [&](int g, int slot) {
        dma16s(wr, smem + PATCH_B + slot * SLICE_B + wave * 1024, (uint32_t)(wave * 1024 + lane * 16), (uint32_t)g * SLICE_B);
    };
    issue_w(0, 0);
    issue_w(1, 1);
    issue_w(2, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // fragment addresses: B (patch) fragment f = 7 wm + j covers virtual pixels 16f + (lane & 15) at plane
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

    // one K-step (the layer3 stage's schedule, conv_stage.hip): MFMAs of the first half of the weight
    // fragments on `cur` while `nxt` is read; mid-step barrier (this wave's slice g+1 landed, every wave
    // is past its reads of slot g % 3); DMA of slice g+3 into that slot; refills of wf with slice g+1
    auto kstep = [&](int g, int slot, frag (&cur)[FM], frag (&nxt)[FM], int cg_n, int tap_n) {
        asm volatile("" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        pread(nxt, cg_n, tap_n);
#pragma unroll
        for (int i = 0; i < FN / 2; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(wf[i], cur[j], acc[i][j]);
        // the FM youngest LDS reads are this step's pread(nxt); older refills of slot `slot` must be done
        asm volatile("s_waitcnt vmcnt(1) lgkmcnt(7)\n\ts_barrier" ::: "memory");
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

    // Epilogue tables ep[cv][9][128] (bias per border class) / slope[cv][128], as in the layer3 stage.
    // Fragment f = 7 wm + j lies in row f >> 1, columns 16 (f & 1) + (lane & 15): its column class
    // depends on the parity of f (= parity of wm + j) and the lane; its row class is the image border
    // only for rows 0 (half 0: f = 0, 1) and 27 (half 1: f = 26, 27).  Per channel fragment i a lane
    // needs 4 biases: {interior, border row} x {even, odd fragment}.
    auto load_ep = [&](int cv, int i, float4 (&e)[4]) {
        int ln = lane;
        asm volatile("" : "+v"(ln));  // opaque copy: the addresses are not hoisted into the K loop
        const int cl = ln & 15, cce = cl == 0 ? 0 : 1, cco = cl == 11 ? 2 : 1, br = half ? 6 : 0;
        const float* ep = p.ep + (size_t)cv * 9 * C + 64 * wn + 16 * i + 4 * (ln >> 4);
        e[0] = *(const float4*)(ep + (3 + cce) * C);
        e[1] = *(const float4*)(ep + (3 + cco) * C);
        e[2] = *(const float4*)(ep + (br + cce) * C);
        e[3] = *(const float4*)(ep + (br + cco) * C);
    };
    auto pick = [&](const float4 (&e)[4], int j) {
        const bool border = half == 0 ? (wm == 0 && j < 2) : (wm == 3 && j >= 5);
        const bool odd = (wm + j) & 1;
        // component selects on values: a dynamic index, or a select of element addresses, would keep
        // e in scratch memory
        const float4 e0 = e[0], e1 = e[1], e2 = e[2], e3 = e[3];
        const float4 in = sel4(odd, e1, e0), bo = sel4(odd, e3, e2);
        return sel4(border, bo, in);
    };
    auto seed_bias = [&](int cv) {
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            float4 e[4];
            load_ep(cv, i, e);
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const float4 bb = pick(e, j);
                acc[i][j] = (f32x4_t){bb.x, bb.y, bb.z, bb.w};
            }
        }
    };

    const int hrow = half ? 0 : PR - 1;       // stored row that receives the partner's row
    const int xrow = half ? 0 : HR - 1;       // own output row the partner needs
    int* const my_flag = p.flags + 2 * b + half;
    const __amdgpu_buffer_rsrc_t xr_x = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.xchg, 0, (uint32_t)min((size_t)0x7fffffff, stage28_xchg_bytes(p.B)), 0x00020000);
    const int* const partner_flag = p.flags + 2 * b + (half ^ 1);

    auto run_conv = [&](int cv, auto second_tag) {
        constexpr bool second = decltype(second_tag)::value;
        if (!second) seed_bias(cv);  // conv2's seed (x + its bias) comes from conv1's epilogue
        pread(pA, 0, 0);
#pragma unroll
        for (int i = 0; i < FN; ++i) wread(i, 0);  // step 0 of every conv sits in slot 0 (36 % 3 == 0)
        const int g0 = cv * KSTEPS;
#pragma unroll 1
        for (int cg = 0; cg < C / 32; cg += 2) {
#pragma unroll
            for (int t = 0; t < 18; ++t) {
                const int cgl = cg + t / 9, tap = t % 9;
                const int cgn = t == 8 ? cg + 1 : (t == 17 ? (cg + 2 < C / 32 ? cg + 2 : 0) : cgl);
                const int tapn = t == 8 || t == 17 ? 0 : tap + 1;
                if (t & 1) kstep(g0 + cgl * 9 + tap, tap % 3, pB, pA, cgn, tapn);
                else kstep(g0 + cgl * 9 + tap, tap % 3, pA, pB, cgn, tapn);
            }
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
        bf16_t* const xo = p.xchg + ((size_t)(2 * b + half) * 2 + (cv & 1)) * XROW;
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const int n = 64 * wn + 16 * i + 4 * (ln >> 4);
            uint2 xin[FM];
            float4 sl, e[4];  // conv1: this fragment's slope and conv2's biases (its accumulator seed)
            if (!second) {
                load_ep(cv + 1, i, e);
                sl = *(const float4*)(p.slope + (size_t)cv * C + n);
#pragma unroll
                for (int j = 0; j < FM; ++j) {
                    const int f = FM * wm + j, col = 16 * (f & 1) + cl;
                    const char* slot = smem + (n >> 3) * PLANE_B + (((f >> 1) + 1) * PC + col + 1) * 16 + (n & 7) * 2;
                    xin[j] = col < IW ? *(const uint2*)slot : make_uint2(0u, 0u);
                }
            }
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int f = FM * wm + j, row = f >> 1, col = 16 * (f & 1) + cl;
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
                    if (exch && row == xrow)  // sc1 store (the exchange's hand-off rule, below)
                        __hip_atomic_store((uint64_t*)(xo + col * C + n), (uint64_t)pk2.x | ((uint64_t)pk2.y << 32),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
        }
        if (exch && !(FR_S28_EXP & 2)) {
            // Hand-off without cache-maintenance fences (MI355X_MICROARCH.md, "valid forms", first row of
            // the sc1 hand-off table; one workgroup per CU, hipMalloc memory): the row bytes are stored
            // sc1 (above) and every storing wave waits for them, a barrier, one lane stores the flag sc1;
            // the partner's wave 0 polls it with sc1 loads, the other waves join it at a barrier, and
            // every load of the row is an sc1 load.  (An agent release + acquire pair costs ~0.4 ms
            // over the stage's 23 exchanges: buffer_wbl2 / buffer_inv per exchange per CU.)
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (threadIdx.x == 0 && !(FR_S28_EXP & 1))
                __hip_atomic_store(my_flag, cv + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (wave == 0 && lane == 0 && !(FR_S28_EXP & 1)) {
                int it = 0;
                while (__hip_atomic_load(partner_flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < cv + 1) {
                    if (++it == SPIN_LIMIT) {
                        __hip_atomic_fetch_add(p.spin_timeouts, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                }
            }
            __syncthreads();
            // the partner's row into the halo row: 448 threads x 16 B (28 pixels x 16 planes; pixel-major,
            // 16 threads read one pixel's 256 B)
            const int t = threadIdx.x;
            if (t < IW * NPL) {
                const int px = t >> 4, pl = t & 15;
                const uint32_t off = (uint32_t)((((2 * b + (half ^ 1)) * 2 + (cv & 1)) * XROW + px * C + pl * 8) * 2);
                const uint4 v = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(xr_x, off, 0, SC1));
                *(uint4*)(smem + pl * PLANE_B + (hrow * PC + px + 1) * 16) = v;
            }
        }
        // the new activation (and halo row) is visible to every wave before the next conv reads it
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
#pragma unroll 1
    for (int blkc = 0; blkc < p.nblk; ++blkc) {
        run_conv(2 * blkc, std::false_type{});
        run_conv(2 * blkc + 1, std::true_type{});
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail DMAs land before the LDS is released
}

}  // namespace

bool stage28_supported(int H, int W, int Cc) { return H == IW && W == IW && Cc == C; }

size_t stage28_weight_bytes(int nconv) { return (size_t)nconv * KSTEPS * SLICE_B; }

size_t stage28_xchg_elems(int B) { return (size_t)B * 2 * 2 * XROW; }

hipError_t launch_stage28(const StageArgs& a, hipStream_t s) {
    if (a.B <= 0 || !a.xchg || !a.flags || !a.spin_timeouts) return hipErrorInvalidValue;
    auto k = a.f16 ? stage28_kernel<true> : stage28_kernel<false>;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_B);
        attr[a.f16 ? 1 : 0] = true;
    }
    hipError_t e = hipMemsetAsync(a.flags, 0, (size_t)2 * a.B * sizeof(int), s);
    if (e != hipSuccess) return e;
    const dim3 grid((2 * a.B + 15) / 16 * 16);
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, dim3(64 * NW), LDS_B, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, grid, dim3(64 * NW), LDS_B, s, a);
    return hipGetLastError();
}

}  // namespace fr
