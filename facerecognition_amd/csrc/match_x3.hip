// Fast exact gallery match for large galleries (BASELINE config 4: 2048 probes x a 125k-row shard of a
// 1M x 512 gallery per rank).  The exact f32 path (match.hip, v_mfma_f32_16x16x4_f32) runs at the f32
// MFMA rate, 1/16 of bf16.  Here:
//   1. candidates: s~ = ph.gh, ONE v_mfma_f32_16x16x32_bf16 per 32 dims (probe and gallery row each rounded to
//      bf16).  The bound is measured, not worst-case: s - ph.gh = p.(g - gh) + (p - ph).gh, so
//      |s~ - s| <= eps(p) = ||p|| EG + ||p - ph|| GN + c (||p|| + ||p - ph||) GN, with EG = max over rows of
//      ||g - gh|| and GN = max ||gh|| (split_x3_kernel keeps both in the buffer's header) and c = 2048 2^-24
//      for the f32 accumulation of 512 exact products (twice the gamma_512 bound).  For unit rows this is
//      ~3.9e-3 ||p|| -- the band of the former 2-product pass (ph.gh + pl.gh, eps 4.0e-3 worst case) at half
//      its MFMAs and probe registers; per (probe, split)
//      the top-KO by s~ of four sub-lists
//      of KP (rows 16j + 4 sub + r of each tile, kept by the lane whose accumulators hold them) and a floor: every row
//      dropped from a sub-list, or by the filter, has s~ <= floor = the larger of the best last entry of the full
//      sub-lists and the least (KP/2)-th entry (the filter's second bar; round 6: before, rows that bar dropped were
//      not covered, a gap only a 16-row near-tie within 2 eps in one split could have exposed);
//   2. rescore (one wave per probe): the global top-KC by s~ are rescored exactly with the k-ordered f32
//      fmaf chain of the exact kernel (same order, so the scores are bit-identical to match.hip) and
//      the top-k is taken by (score desc, index asc);
//   3. proof: every row outside the KC candidates has s~ <= T (the KC-th candidate's s~, or the largest
//      floor if higher), so its exact
//      score is <= T + eps.  Unless the k-th exact score exceeds T + 2 eps (i.e. more than KC - k rows tie
//      with it within 2 eps), the wave rescans the whole gallery exactly for that probe (counted).  The
//      result is therefore always the exact top-k of the f32 scores.
// Block = 8 waves, 16 PF probes per wave (PF = 1: 128 per block) as bf16 fragments in registers for the
// whole kernel; gallery chunks (64 rows x 128 dims of gh, 16 KiB) stream through a 7-slot LDS-DMA ring
// six chunks ahead (counted vmcnt, raw barriers; XOR-swizzled 16-B chunks): the ring depth, not HBM,
// sets the stream rate (in flight / L2 latency).  Blocks of one gallery split share an XCD (xcd_remap), so each XCD streams its
// splits from HBM once and the other probe blocks hit its L2.
#include "kernels.h"

#include <algorithm>
#include <float.h>
#include <stdlib.h>
#include <limits.h>

namespace fr {
namespace {


constexpr int XW = 8;         // waves per block
// probe fragments (16 probes each) per wave: every gallery fragment read feeds PF MFMAs.  PF = 2 (256 probes per
// block, 32-entry lists per lane) measured the same (2048 x 125k 0.44 vs 0.45 ms, 256 x 1M 0.48 vs 0.47): the kernel
// is bound by the filter's VALU work (7 VALU per MFMA), not the LDS reads, and halving the probe blocks doubles
// the splits and so the list fills
constexpr int PF = 1;
constexpr int XP = 16 * PF * XW;  // probes per block
constexpr int XG = 64;        // gallery rows per tile
// dims per LDS chunk: 128 (16-KiB chunks, 7-slot ring) since the 1-product pass halved the MFMAs per barrier;
// 64 (8 KiB, 13 slots) measured 2.5 % slower (2048 x 125k 0.450 vs 0.438 ms; it was 1.5-3 % faster at 2 products)
constexpr int XC = 128;
constexpr int XNC = 512 / XC;  // chunks per 64-row tile
constexpr int XGR = XC / 8;    // 16-B groups per chunk row
constexpr int XD = 512;       // embedding dim (the kernel is specialised)
constexpr int KP = 8;         // candidates per (probe, split, sub-lane): 4 sub-lanes per probe
constexpr int KO = 16;        // candidates written per (probe, split) ...
constexpr int KS = KO + 1;    // ... plus one floor entry (index -2)
constexpr int KC = 32;        // candidates rescored per probe (a 2 eps band of ~8e-3 needs more than 16: with
                              // 16, random 1M-row galleries put the 5th score within 2 eps of the 16th often
                              // enough to trigger rescans)
constexpr float X_ACC = 2048.f / 16777216.f;  // c of the header: f32 accumulation of 512 exact products
// header of the chunk buffer (elements; 8 KiB keeps the chunks 8-KiB aligned): uint32 [0] = EG, [1] = GN as
// f32 bits (non-negative: integer max == float max), raised by every split_x3_kernel launch
constexpr int X3_HEAD = 4096;

__device__ __forceinline__ bool better(float s1, int i1, float s2, int i2) {
    return s1 > s2 || (s1 == s2 && i1 < i2);
}

template <int KMAX>
__device__ __forceinline__ void insert(float (&ls)[KMAX], int (&li)[KMAX], float s, int idx) {
    if (!better(s, idx, ls[KMAX - 1], li[KMAX - 1])) return;
    float cs = s;
    int ci = idx;
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
        if (better(cs, ci, ls[q], li[q])) {
            const float ts = ls[q];
            const int ti = li[q];
            ls[q] = cs;
            li[q] = ci;
            cs = ts;
            ci = ti;
        }
    }
}

// score-only sorted insert for the candidate scan (ties with the last entry are dropped: the floor
// covers them)
template <int KMAX>
__device__ __forceinline__ void insert_s(float (&ls)[KMAX], int (&li)[KMAX], float s, int idx) {
    if (!(s > ls[KMAX - 1])) return;
    bool b[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) b[q] = s > ls[q];
#pragma unroll
    for (int q = KMAX - 1; q >= 0; --q) {
        const float sh = q > 0 && b[q - 1] ? ls[q - 1] : s;
        const int ih = q > 0 && b[q - 1] ? li[q - 1] : idx;
        ls[q] = b[q] ? sh : ls[q];
        li[q] = b[q] ? ih : li[q];
    }
}


typedef __attribute__((ext_vector_type(8))) __bf16 bf8v;

// The candidate pass's gallery copy, in its chunk order: gh = bf16(g) (|g - gh| <= 2^-8 |g|), chunk (tile
// T = 64 rows, dims 64c ..) = 8 KiB contiguous at (8T + c) x 8 KiB, [64 rows x 128 B], a row's eight 16-B
// groups stored at slot group ^ xswz_row(row): the LDS-DMA copies a chunk linearly and the fragment reads
// stay conflict-free.  (Row-major gh / gl arrays put a chunk's 64
// rows 1 KiB apart: its 128-B pieces fell on a few HBM / L2 channels, every block of a split on the same
// ones.)  Rows past the gallery in the last tile are never candidates (the kernel masks them).
constexpr int XCHUNK_E = 64 * XC;  // bf16 elements per chunk
// 128-B rows: rows r, r + 1 are 32 banks apart, so (r >> 1) & 7 separates the rest; 256-B rows start on one bank
__device__ __forceinline__ int xswz_row(int row) { return XGR == 16 ? row & 15 : (row >> 1) & 7; }

__global__ __launch_bounds__(256) void split_x3_kernel(const float* __restrict__ G, int64_t row0, int64_t n,
                                                       bf16_t* __restrict__ T, uint32_t* __restrict__ stats) {
    // one thread per 8 dims of one row (a wave = one row: the grid stride is a multiple of 64)
    float eg = 0.f, gn = 0.f;  // this lane's running max of ||g - gh|| and ||gh|| over its rows
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n * 64; i += (int64_t)gridDim.x * 256) {
        const int64_t r = row0 + i / 64;
        const int grp = (int)(i % 64), c = grp / XGR, g = grp % XGR, rr = (int)(r & 63);
        const float* src = G + r * 512 + 8 * grp;
        const float4 a = *(const float4*)src, b = *(const float4*)(src + 4);
        const float v[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint16_t hb[8];
        float e2 = 0.f, h2 = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
            const __bf16 h = (__bf16)v[e];
            hb[e] = __builtin_bit_cast(uint16_t, h);
            const float hf = (float)h, d = v[e] - hf;
            e2 = fmaf(d, d, e2);
            h2 = fmaf(hf, hf, h2);
        }
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            e2 += __shfl_xor(e2, o);
            h2 += __shfl_xor(h2, o);
        }
        eg = fmaxf(eg, sqrtf(e2));
        gn = fmaxf(gn, sqrtf(h2));
        bf16_t* dst = T + ((r >> 6) * XNC + c) * XCHUNK_E + rr * XC + (g ^ xswz_row(rr)) * 8;
        uint4 hv;
        hv.x = hb[0] | (uint32_t)hb[1] << 16; hv.y = hb[2] | (uint32_t)hb[3] << 16;
        hv.z = hb[4] | (uint32_t)hb[5] << 16; hv.w = hb[6] | (uint32_t)hb[7] << 16;
        *(uint4*)dst = hv;
    }
    // (the norms' own f32 rounding: 1e-4 relative margin)
    if ((threadIdx.x & 63) == 0 && gn > 0.f) {
        atomicMax((int*)stats, __float_as_int(eg * 1.0001f));
        atomicMax((int*)stats + 1, __float_as_int(gn * 1.0001f));
    }
}

constexpr int XSLOT = XC == 128 ? 7 : 13;  // LDS ring depth (chunks): XSLOT - 1 in flight (96 KiB)
constexpr int XCHUNK_B = XG * XC * 2;          // 8 KiB: [64 rows x 128 B]
static_assert(XCHUNK_B == XCHUNK_E * 2, "chunk layout");
constexpr int XRB = XC * 2;                    // LDS row bytes
constexpr int XPPW = XCHUNK_B / 1024 / 8;      // 1-KiB DMA pieces per wave per chunk
typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ int xswz(int row, int chunk) { return chunk ^ xswz_row(row); }

__global__ __launch_bounds__(512) void match_x3_kernel(const float* __restrict__ P, int B, const bf16_t* __restrict__ GT,
                                                       int64_t N, int64_t index_base,
                                                       int64_t rows_per_split, int n_split, int npb,
                                                       float* __restrict__ cs, int32_t* __restrict__ ci) {
    // ONE LDS array (a second __shared__ object can make hipcc drain vmcnt before ds_reads)
    __shared__ __attribute__((aligned(16))) char smem[XSLOT * XCHUNK_B];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: no waterfall around the DMAs
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int split = lid / npb, pb = lid - split * npb;
    const int p0 = pb * XP;
    const int64_t g_begin = (int64_t)split * rows_per_split;
    const int64_t g_end = g_begin + rows_per_split < N ? g_begin + rows_per_split : N;

    // probe fragments (the MFMA's B operand): fragment f, k-step t (32 dims) of probe
    // p0 + 16 (PF wave + f) + (lane & 15), dims 32t + 8(lane>>4) .. +8
    constexpr int KT = XD / 32;
    bf8v ph[PF][KT];
    const int my_sub = lane >> 4;  // the lane's sub-list: rows 16j + 4*my_sub + r of every tile
    auto my_q = [&](int f) { return 16 * (PF * wave + f) + (lane & 15); };  // its probe of fragment f (block-local)
#pragma unroll
    for (int f = 0; f < PF; ++f) {
        const int p = p0 + my_q(f);
#pragma unroll
        for (int t = 0; t < KT; ++t) {
            float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            if (p < B) {
                const float* src = P + (size_t)p * XD + 32 * t + 8 * (lane >> 4);
                const float4 a = *(const float4*)src, b = *(const float4*)(src + 4);
                v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) ph[f][t][e] = (__bf16)v[e];
        }
    }

    float ls[PF][KP];
    int li[PF][KP];
#pragma unroll
    for (int f = 0; f < PF; ++f)
#pragma unroll
        for (int q = 0; q < KP; ++q) { ls[f][q] = -INFINITY; li[f][q] = INT_MAX; }

    // LDS-DMA of chunk (tile t0, dims 64c..): a linear copy of its 16 KiB (split_x3_kernel's layout), 16
    // pieces of 1 KiB, wave w issues pieces 2w, 2w+1.  The resource starts at the split's first chunk
    // (32-bit offsets); look-ahead chunks past the gallery read 0, past the split are never used.
    const size_t g_chunk0 = (size_t)(g_begin / XG) * XNC;
    const size_t g_left = ((size_t)((N + XG - 1) / XG) * XNC - g_chunk0) * XCHUNK_B;
    const __amdgpu_buffer_rsrc_t rg = __builtin_amdgcn_make_buffer_rsrc((void*)(GT + g_chunk0 * XCHUNK_E), 0,
                                                                        (int)min(g_left, (size_t)0x7fffffff), 0x00020000);
    auto issue_chunk = [&](int64_t t0, int c, int slot) {
        const uint32_t cbase = (uint32_t)((((t0 - g_begin) / XG) * XNC + c) * XCHUNK_B);
#pragma unroll
        for (int u = 0; u < XPPW; ++u) {
            const int piece = XPPW * wave + u;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rg, (lds_void*)(smem + slot * XCHUNK_B + piece * 1024), 16,
                                                     cbase + piece * 1024 + 16 * lane, 0, 0, 0);
        }
    };
    // prologue: the first XSLOT - 1 chunks (slots are uniform run-time values: one VALU add per chunk)
    int64_t t_issue = g_begin;  // tile of the next chunk to issue
    int c_issue = 0, s_issue = 0, s_read = 0;
    auto issue_next = [&]() {
        issue_chunk(t_issue, c_issue, s_issue);
        if (++c_issue == XD / XC) { c_issue = 0; t_issue += XG; }
        if (++s_issue == XSLOT) s_issue = 0;
    };
#pragma unroll
    for (int i = 0; i < XSLOT - 1; ++i) issue_next();

    // Lane reductions over a probe's 4 sub-list lanes (lane ^ 16, ^ 32, ^ 48): two v_permlane{32,16}_swap (max and
    // min are symmetric, so the swapped halves pair up as xor 32 / 16), no LDS round trip on the tile's critical path.
    auto red4 = [](float x, bool mx) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
        const float y = mx ? fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]))
                           : fminf(__uint_as_float(r[0]), __uint_as_float(r[1]));
        auto q = __builtin_amdgcn_permlane16_swap(__float_as_uint(y), __float_as_uint(y), false, false);
        return mx ? fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1])) : fminf(__uint_as_float(q[0]), __uint_as_float(q[1]));
    };
    // the tile's candidate filter and sorted inserts (a = its accumulators, tb = its first row)
    auto filter_tile = [&](f32x4_t (&a)[4], float (&ls)[KP], int (&li)[KP], int64_t tb) {
        // a[j][r] = s~(the lane's probe, row tb + 16*j + 4*my_sub + r).  A row not above the best KP-th score
        // of the probe's 4 sub-lists (lanes lane ^ 16, ^ 32) is never needed: the floor (>= that score)
        // covers it in the proof -- ties included, so the scan compares scores only.  The sorted insert
        // runs once per hit of the wave's busiest lane.
        if (g_end - tb < XG) {  // last tile of the split: rows past it are zero-filled, never candidates
            const int lim = (int)(g_end - tb);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int r = 0; r < 4; ++r)
                    if (16 * j + 4 * my_sub + r >= lim) a[j][r] = -INFINITY;
        }
        // also: when every sub-list holds >= KP/2 entries above x, the probe's top KO = 2 KP (the merge
        // keeps exactly those) are all above x, so min over the sub-lists of the (KP/2)-th score is a
        // valid (usually higher) bar too
        const float thr = fmaxf(red4(ls[KP - 1], true), red4(ls[KP / 2 - 1], false));
        uint32_t m = 0;
#pragma unroll
        for (int e = 0; e < 16; ++e) m |= a[e >> 2][e & 3] > thr ? 1u << e : 0u;
        // one pass per hit of the busiest lane (usually one): pick the score by a select tree of bitfield
        // inserts on the raw bits (written as ternaries over array elements, the compiler folded the selects
        // into a dynamically indexed array and spilled it through LDS: two LDS round trips per insert)
        while (m) {
            const int e = __builtin_ctz(m);
            m &= m - 1;
            const uint32_t m3 = 0u - (uint32_t)((e >> 3) & 1), m2 = 0u - (uint32_t)((e >> 2) & 1);
            const uint32_t m1 = 0u - (uint32_t)((e >> 1) & 1), m0 = 0u - (uint32_t)(e & 1);
            auto bsel = [](uint32_t msk, uint32_t x, uint32_t y) { return (msk & x) | (~msk & y); };
            uint32_t v8[8], v4[4], v2[2];
#pragma unroll
            for (int q = 0; q < 8; ++q)
                v8[q] = bsel(m3, __float_as_uint(a[(q + 8) >> 2][(q + 8) & 3]), __float_as_uint(a[q >> 2][q & 3]));
#pragma unroll
            for (int q = 0; q < 4; ++q) v4[q] = bsel(m2, v8[q + 4], v8[q]);
#pragma unroll
            for (int q = 0; q < 2; ++q) v2[q] = bsel(m1, v4[q + 2], v4[q]);
            const float sc = __uint_as_float(bsel(m0, v2[1], v2[0]));
            insert_s<KP>(ls, li, sc, (int)(tb + index_base) + 16 * (e >> 2) + 4 * my_sub + (e & 3));
        }
    };
    for (int64_t t0 = g_begin; t0 < g_end; t0 += XG) {
        f32x4_t acc[PF][4];
#pragma unroll
        for (int f = 0; f < PF; ++f)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[f][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int c = 0; c < XD / XC; ++c) {
            // chunk c landed (the XPPW x (XSLOT - 2) younger chunks' DMA pieces may stay in flight); every wave
            // has its reads of chunk c - 1 back (lgkmcnt(0): the compiler may sink that chunk's MFMAs, and with
            // them its own waits, below this barrier), so chunk c - 1's slot takes chunk c + XSLOT - 1
            static_assert(XPPW * (XSLOT - 2) < 64, "vmcnt range");
            asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(XPPW * (XSLOT - 2)) : "memory");
            issue_next();
            const char* ch = smem + s_read * XCHUNK_B;
            if (++s_read == XSLOT) s_read = 0;
#pragma unroll
            for (int tt = 0; tt < XC / 32; ++tt) {
                const int t = c * (XC / 32) + tt;
                const int kch = 4 * tt + (lane >> 4);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int row = 16 * j + (lane & 15);
                    const int o = row * XRB + xswz(row, kch) * 16;
                    const bf8v gh = *(const bf8v*)(ch + o);
                    // gallery rows as the A operand: D[row][probe], so each lane's accumulators belong to
                    // ONE probe (its own candidate sub-list) and the filter never leaves the registers
#pragma unroll
                    for (int f = 0; f < PF; ++f)
                        acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(gh, ph[f][t], acc[f][j], 0, 0, 0);
                }
            }
        }
#pragma unroll
        for (int f = 0; f < PF; ++f) filter_tile(acc[f], ls[f], li[f], t0);
    }
    // the look-ahead DMAs (zeros past the split) land everywhere before the ring is reused as scratch
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    // merge the 4 sub-lists of each probe into its top KO: park them in the (drained) ring and let one
    // lane per probe insert all four (a rolled loop: one inlined insert)
    float* ms = (float*)smem;                    // [XP][4][KP] scores (the drained DMA ring)
    int* mi = (int*)(smem + XP * 4 * KP * 4);    // [XP][4][KP] indices
    static_assert(2 * XP * 4 * KP * 4 <= XSLOT * XCHUNK_B, "merge scratch fits the ring");
    static_assert(KO == 2 * KP, "the scan's second bar assumes 4 sub-lists x KP/2 = KO");
#pragma unroll
    for (int f = 0; f < PF; ++f)
#pragma unroll
        for (int q = 0; q < KP; ++q) {
            ms[(my_q(f) * 4 + my_sub) * KP + q] = ls[f][q];
            mi[(my_q(f) * 4 + my_sub) * KP + q] = li[f][q];
        }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    // lanes of sub-list 0 merge the probe of fragment 0, sub-list 1 that of fragment 1, ...
    const int mf = my_sub % PF, mq = my_q(mf), p = p0 + mq;
    if (my_sub < PF && p < B) {
        float os[KO];
        int oi[KO];
#pragma unroll
        for (int q = 0; q < KO; ++q) { os[q] = -INFINITY; oi[q] = INT_MAX; }
        // every row the scan dropped scores at most the final bar: a full sub-list dropped rows up to its last
        // entry, and the filter's second bar (the least (KP/2)-th entry) dropped rows up to at most its final value
        float floor_s = -INFINITY, half = INFINITY;
#pragma unroll 1
        for (int e = 0; e < 4 * KP; ++e) {
            const float sc = ms[mq * 4 * KP + e];
            const int ix = mi[mq * 4 * KP + e];
            if (e % KP == KP / 2 - 1) half = fminf(half, ix == INT_MAX ? -INFINITY : sc);
            if (ix == INT_MAX) continue;
            insert<KO>(os, oi, sc, ix);
            if (e % KP == KP - 1) floor_s = fmaxf(floor_s, sc);
        }
        floor_s = fmaxf(floor_s, half);
        const size_t o = ((size_t)p * n_split + split) * KS;
#pragma unroll
        for (int q = 0; q < KO; ++q) {
            const bool valid = oi[q] != INT_MAX;
            cs[o + q] = valid ? os[q] : -INFINITY;
            ci[o + q] = valid ? oi[q] : -1;
        }
        cs[o + KO] = floor_s;
        ci[o + KO] = -2;
    }
}

// Exact score in the order of match.hip's v_mfma_f32_16x16x4_f32 sequence: per 16-dim block t16 the MFMAs take
// components comp = 0..3 of the lanes' float4 k-groups kq = 0..3, each a k-ordered fmaf chain (exact_dot_lds
// below, with the probe row in LDS).

// wave-wide pop of the best (score desc, index asc) entry of per-lane sorted lists
template <int KMAX>
__device__ __forceinline__ void wave_pop(float (&ls)[KMAX], int (&li)[KMAX], int& head, float& ws, int& wi) {
    float bs = -INFINITY;
    int bi = INT_MAX;
#pragma unroll
    for (int h = 0; h < KMAX; ++h)
        if (h == head) { bs = ls[h]; bi = li[h]; }
    ws = bs;
    wi = bi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const float os = __shfl_xor(ws, o);
        const int oi = __shfl_xor(wi, o);
        if (better(os, oi, ws, wi)) { ws = os; wi = oi; }
    }
    if (wi == bi && bi != INT_MAX) ++head;  // indices are unique: the owner pops
}

// The exact score with the probe row in LDS (every lane reads the same address: a broadcast) and four 16-dim steps
// of gallery loads in flight
__device__ __forceinline__ float exact_dot_lds(const float* p, const float* __restrict__ g) {
    float acc = 0.f;
#pragma unroll 4
    for (int t16 = 0; t16 < XD / 16; ++t16) {
        float4 a[4], b[4];
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) {
            a[kq] = *(const float4*)(p + 16 * t16 + 4 * kq);
            b[kq] = *(const float4*)(g + 16 * t16 + 4 * kq);
        }
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) acc = fmaf(a[kq].x, b[kq].x, acc);
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) acc = fmaf(a[kq].y, b[kq].y, acc);
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) acc = fmaf(a[kq].z, b[kq].z, acc);
#pragma unroll
        for (int kq = 0; kq < 4; ++kq) acc = fmaf(a[kq].w, b[kq].w, acc);
    }
    return acc;
}

constexpr int KL = 8;  // rescore: per-lane candidate list depth (a lane's dropped entries join the floor)

__global__ __launch_bounds__(256) void rescore_kernel(const float* __restrict__ P, int B, const float* __restrict__ G,
                                                      int64_t N, int64_t index_base, const float* __restrict__ cs,
                                                      const int32_t* __restrict__ ci, int n_lists, int k,
                                                      float* __restrict__ out_s, int32_t* __restrict__ out_i,
                                                      int* __restrict__ n_fallback, const uint32_t* __restrict__ stats) {
    __shared__ __attribute__((aligned(16))) float prow_s[4][XD];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int p = blockIdx.x * 4 + wave;
    if (p >= B) return;
    const float* prow = P + (size_t)p * XD;
    float* const pl = prow_s[wave];
    for (int d = 4 * lane; d < XD; d += 256) *(float4*)(pl + d) = *(const float4*)(prow + d);
    // (a) global top-KC by approximate score; T = the KC-th (or -inf with fewer candidates).  Each lane keeps its
    // best KL of the entries it reads (eight loads in flight per round); an entry a full list drops scores at
    // most lane_floor, which joins the floor, so the proof below stays valid (a lane holding more than KL of
    // the KC best can only make it fail, and then the probe is rescanned).
    float ls[KL];
    int li[KL];
#pragma unroll
    for (int q = 0; q < KL; ++q) { ls[q] = -INFINITY; li[q] = INT_MAX; }
    const int n = n_lists * KS;
    float floor_s = -INFINITY;  // every row no list holds has s~ <= floor_s
    const float* csp = cs + (size_t)p * n;
    const int32_t* cip = ci + (size_t)p * n;
    for (int c0 = lane; c0 < n; c0 += 64 * 8) {
        float vs[8];
        int vi[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int c = c0 + 64 * u;
            vi[u] = c < n ? cip[c] : -1;
            vs[u] = c < n ? csp[c] : -INFINITY;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if (vi[u] >= 0) {
                if (better(vs[u], vi[u], ls[KL - 1], li[KL - 1])) {
                    if (li[KL - 1] != INT_MAX) floor_s = fmaxf(floor_s, ls[KL - 1]);  // pushed out of the list
                    insert<KL>(ls, li, vs[u], vi[u]);
                } else {
                    floor_s = fmaxf(floor_s, vs[u]);
                }
            } else if (vi[u] == -2) {
                floor_s = fmaxf(floor_s, vs[u]);
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) floor_s = fmaxf(floor_s, __shfl_xor(floor_s, o));
    int head = 0, my_idx = -1;
    float T = -INFINITY;
    for (int q = 0; q < KC; ++q) {
        float ws;
        int wi;
        wave_pop<KL>(ls, li, head, ws, wi);
        if (lane == q) my_idx = wi == INT_MAX ? -1 : wi;
        if (q == KC - 1) T = wi == INT_MAX ? -INFINITY : ws;
    }
    T = fmaxf(T, floor_s);
    // (b) exact rescoring: lane q < KC holds candidate q
    float rs[1] = {-INFINITY};
    int ri[1] = {INT_MAX};
    if (lane < KC && my_idx >= 0) {
        rs[0] = exact_dot_lds(pl, G + (size_t)(my_idx - index_base) * XD);
        ri[0] = my_idx;
    }
    float pp = 0.f, ll = 0.f;  // ||p||^2, ||p - ph||^2 (ph as the candidate pass rounds it)
    for (int d = lane; d < XD; d += 64) {
        const float v = prow[d], r = v - (float)(__bf16)v;
        pp = fmaf(v, v, pp);
        ll = fmaf(r, r, ll);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        pp += __shfl_xor(pp, o);
        ll += __shfl_xor(ll, o);
    }
    const float EG = __uint_as_float(stats[0]), GN = __uint_as_float(stats[1]);
    const float np = sqrtf(pp), nl = sqrtf(ll);
    const float eps = (np * EG + nl * GN + X_ACC * (np + nl) * GN) * 1.001f;  // header
    // (c) exact top-k among the candidates
    int h1 = 0;
    float kth = INFINITY, outs = -INFINITY;
    int outi = -1;
    for (int q = 0; q < k; ++q) {
        float ws;
        int wi;
        wave_pop<1>(rs, ri, h1, ws, wi);
        if (lane == q) {
            outs = wi == INT_MAX ? -INFINITY : ws;
            outi = wi == INT_MAX ? -1 : wi;
        }
        if (q == k - 1) kth = ws;
    }
    // (d) an excluded row scores <= T + eps; ties need the index order, so require kth > T + 2 eps
    if (!(T == -INFINITY || kth > T + 2.f * eps)) {
        // (e) widened: candidates KC .. 2 KC - 1 on lanes KC .. 2 KC - 1 (the lists hold up to 64 x KL entries), T
        // from the 2 KC-th; a one-wave rescan of the whole gallery (milliseconds at 1M rows) only if that fails too
        static_assert(2 * KC == 64, "one candidate per lane");
        float T2 = -INFINITY;
        for (int q = KC; q < 2 * KC; ++q) {
            float ws;
            int wi;
            wave_pop<KL>(ls, li, head, ws, wi);
            if (lane == q) my_idx = wi == INT_MAX ? -1 : wi;
            if (q == 2 * KC - 1) T2 = wi == INT_MAX ? -INFINITY : ws;
        }
        T2 = fmaxf(T2, floor_s);
        if (lane >= KC && my_idx >= 0) {
            rs[0] = exact_dot_lds(pl, G + (size_t)(my_idx - index_base) * XD);
            ri[0] = my_idx;
        }
        h1 = 0;
        for (int q = 0; q < k; ++q) {
            float ws;
            int wi;
            wave_pop<1>(rs, ri, h1, ws, wi);
            if (lane == q) {
                outs = wi == INT_MAX ? -INFINITY : ws;
                outi = wi == INT_MAX ? -1 : wi;
            }
            if (q == k - 1) kth = ws;
        }
        T = T2;
    }
    if (!(T == -INFINITY || kth > T + 2.f * eps)) {
        if (lane == 0 && n_fallback) atomicAdd(n_fallback, 1);
        float fs[KC];
        int fi[KC];
#pragma unroll
        for (int q = 0; q < KC; ++q) { fs[q] = -INFINITY; fi[q] = INT_MAX; }
#pragma unroll 1
        for (int64_t r = lane; r < N; r += 64)
            insert<KC>(fs, fi, exact_dot_lds(pl, G + (size_t)r * XD), (int)(r + index_base));
        int hh = 0;
        for (int q = 0; q < k; ++q) {
            float ws;
            int wi;
            wave_pop<KC>(fs, fi, hh, ws, wi);
            if (lane == q) {
                outs = wi == INT_MAX ? -INFINITY : ws;
                outi = wi == INT_MAX ? -1 : wi;
            }
        }
    }
    if (lane < k) {
        out_s[(size_t)p * k + lane] = outs;
        out_i[(size_t)p * k + lane] = outi;
    }
}

// Small-batch exact match (B <= 4 probes: the reference's online recognize path at bs = 1,
// recognition_engine.py:328-381).  match_p512_kernel keeps 64 probes per block in MFMA fragments, so at B = 1 a
// block scores 63 padding probes and the split plan leaves ~80 blocks each walking 128 rows through an LDS ring
// (32 us for 10k rows).  Here each lane scores one row at a time (R rows per lane, WPB waves per block) for every
// probe with exact_dot_lds's k-ordered fmaf chain (the f32 kernels' order: the scores are theirs bit for bit; 8 16-dim
// steps of loads in flight measured 15.7 vs 13.9 us for 1 x 10k), and keeps per-lane sorted lists; each wave's top-k per probe goes to LDS, wave 0
// merges the block's WPB lists and writes one candidate list per block for topk_merge_kernel.  WPB = 1 while the
// waves fit the CUs (each CU then streams one wave's 128 KiB of rows), more waves per block (fewer lists) beyond.
template <int NB, int KL, int WPB>
__global__ __launch_bounds__(64 * WPB) void match_rows_kernel(const float* __restrict__ P, int B, const float* __restrict__ G,
                                                         int64_t N, int64_t index_base, int k, int R,
                                                         float* __restrict__ cand_s, int32_t* __restrict__ cand_i) {
    __shared__ float xs[NB][WPB][KL];
    __shared__ int xi[NB][WPB][KL];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t r0 = ((int64_t)blockIdx.x * WPB + wave) * 64 * R;
    float ls[NB][KL];
    int li[NB][KL];
#pragma unroll
    for (int b = 0; b < NB; ++b)
#pragma unroll
        for (int q = 0; q < KL; ++q) { ls[b][q] = -INFINITY; li[b][q] = INT_MAX; }
    for (int j = 0; j < R; ++j) {
        const int64_t r = r0 + 64 * j + lane;
        if (r >= N) break;
        const float* g = G + (size_t)r * XD;
        float acc[NB];
#pragma unroll
        for (int b = 0; b < NB; ++b) acc[b] = 0.f;
#pragma unroll 2
        for (int t16 = 0; t16 < XD / 16; ++t16) {
            float4 gv[4];
#pragma unroll
            for (int kq = 0; kq < 4; ++kq) gv[kq] = *(const float4*)(g + 16 * t16 + 4 * kq);
#pragma unroll
            for (int b = 0; b < NB; ++b) {
                if (b >= B) break;
                float4 pv[4];
#pragma unroll
                for (int kq = 0; kq < 4; ++kq) pv[kq] = *(const float4*)(P + (size_t)b * XD + 16 * t16 + 4 * kq);
                // exact_dot_lds's order: k = 16 t + 4 kq + c, c outer
#pragma unroll
                for (int kq = 0; kq < 4; ++kq) acc[b] = fmaf(pv[kq].x, gv[kq].x, acc[b]);
#pragma unroll
                for (int kq = 0; kq < 4; ++kq) acc[b] = fmaf(pv[kq].y, gv[kq].y, acc[b]);
#pragma unroll
                for (int kq = 0; kq < 4; ++kq) acc[b] = fmaf(pv[kq].z, gv[kq].z, acc[b]);
#pragma unroll
                for (int kq = 0; kq < 4; ++kq) acc[b] = fmaf(pv[kq].w, gv[kq].w, acc[b]);
            }
        }
#pragma unroll
        for (int b = 0; b < NB; ++b)
            if (b < B) insert<KL>(ls[b], li[b], acc[b], (int)(r + index_base));
    }
    // each wave's top-k per probe -> LDS
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (b >= B) break;
        int head = 0;
        for (int q = 0; q < k; ++q) {
            float ws;
            int wi;
            wave_pop<KL>(ls[b], li[b], head, ws, wi);
            if (lane == 0) { xs[b][wave][q] = ws; xi[b][wave][q] = wi; }
        }
    }
    __syncthreads();
    if (wave) return;
    // wave 0: lane 16 w + q holds entry q of wave w's list; k pops give the block's top-k
#pragma unroll
    for (int b = 0; b < NB; ++b) {
        if (b >= B) break;
        float ms[1] = {-INFINITY};
        int mi[1] = {INT_MAX};
        const int w = lane >> 4, q = lane & 15;
        if (w < WPB && q < k) { ms[0] = xs[b][w][q]; mi[0] = xi[b][w][q]; }
        int head = 0;
        float outs = -INFINITY;
        int outi = -1;
        for (int q2 = 0; q2 < k; ++q2) {
            float ws;
            int wi;
            wave_pop<1>(ms, mi, head, ws, wi);
            if (lane == q2) {
                outs = wi == INT_MAX ? -INFINITY : ws;
                outi = wi == INT_MAX ? -1 : wi;
            }
        }
        if (lane < k) {
            const size_t o = ((size_t)b * gridDim.x + blockIdx.x) * k + lane;
            cand_s[o] = outs;
            cand_i[o] = outi;
        }
    }
}

}  // namespace

size_t x3_gallery_elems(int64_t rows) { return X3_HEAD + (size_t)((rows + XG - 1) / XG) * XNC * XCHUNK_E; }

hipError_t launch_split_x3(const float* G, int64_t row0, int64_t n, bf16_t* T, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    int64_t blocks = (n * 64 + 255) / 256;
    if (blocks > 16384) blocks = 16384;
    hipLaunchKernelGGL(split_x3_kernel, dim3((unsigned)blocks), dim3(256), 0, s, G, row0, n, T + X3_HEAD, (uint32_t*)T);
    return hipGetLastError();
}

void match_x3_plan(int B, int64_t N, int* n_split, int64_t* rows_per_split) {
    const int npb = (B + XP - 1) / XP;
    int64_t want = (256 + npb - 1) / npb;  // one 512-thread block per CU
    const int64_t tiles = (N + XG - 1) / XG;
    if (want > tiles) want = tiles;
    if (want < 1) want = 1;
    const int64_t rps = ((tiles + want - 1) / want) * XG;
    *rows_per_split = rps;
    *n_split = (int)((N + rps - 1) / rps);
}

// match_rows_kernel's plan: R rows per lane so that at most ~1024 blocks run (one list each), WPB waves per block
bool match_rows_supported(int B, int D, int k) { return B >= 1 && B <= 4 && D == XD && k >= 1 && k <= 8; }

static int rows_wpb(int64_t N) {
    const int64_t waves = (N + 63) / 64;
    return waves <= 256 ? 1 : waves <= 512 ? 2 : 4;
}

void match_rows_plan(int64_t N, int* n_lists, int* R) {
    const int64_t per = 64LL * rows_wpb(N) * 1024;
    *R = (int)std::max<int64_t>(1, (N + per - 1) / per);
    *n_lists = (int)((N + 64LL * rows_wpb(N) * *R - 1) / (64LL * rows_wpb(N) * *R));
}

hipError_t launch_match_rows(const float* P, int B, const float* G, int64_t N, int D, int k, int64_t index_base,
                             float* cand_s, int32_t* cand_i, int n_lists, int R, hipStream_t s) {
    if (!match_rows_supported(B, D, k) || n_lists < 1) return hipErrorInvalidValue;
    typedef void (*Kern)(const float*, int, const float*, int64_t, int64_t, int, int, float*, int32_t*);
    const int wpb = rows_wpb(N);
    const Kern tab[3][4] = {
        {match_rows_kernel<1, 5, 1>, match_rows_kernel<1, 8, 1>, match_rows_kernel<4, 5, 1>, match_rows_kernel<4, 8, 1>},
        {match_rows_kernel<1, 5, 2>, match_rows_kernel<1, 8, 2>, match_rows_kernel<4, 5, 2>, match_rows_kernel<4, 8, 2>},
        {match_rows_kernel<1, 5, 4>, match_rows_kernel<1, 8, 4>, match_rows_kernel<4, 5, 4>, match_rows_kernel<4, 8, 4>}};
    const Kern kern = tab[wpb == 1 ? 0 : wpb == 2 ? 1 : 2][(B == 1 ? 0 : 2) + (k <= 5 ? 0 : 1)];
    hipLaunchKernelGGL(kern, dim3(n_lists), dim3(64 * wpb), 0, s, P, B, G, N, index_base, k, R, cand_s, cand_i);
    return hipGetLastError();
}

int match_x3_candidates() { return KS; }

hipError_t launch_match_x3(const float* P, int B, const float* G, const bf16_t* GT, int64_t N, int D,
                           int k, int64_t index_base, float* cand_s, int32_t* cand_i, int n_split,
                           int64_t rows_per_split, float* out_s, int32_t* out_i, int* n_fallback, hipStream_t s) {
    if (D != XD || k > KC || k < 1) return hipErrorInvalidValue;
    const int npb = (B + XP - 1) / XP;
    hipLaunchKernelGGL(match_x3_kernel, dim3(npb * n_split), dim3(512), 0, s, P, B, GT + X3_HEAD, N, index_base,
                       rows_per_split, n_split, npb, cand_s, cand_i);
    hipLaunchKernelGGL(rescore_kernel, dim3((B + 3) / 4), dim3(256), 0, s, P, B, G, N, index_base, cand_s, cand_i,
                       n_split, k, out_s, out_i, n_fallback, (const uint32_t*)GT);
    return hipGetLastError();
}

}  // namespace fr
