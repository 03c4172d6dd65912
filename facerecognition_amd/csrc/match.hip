// Gallery match: probes P[B,D] · galleryᵀ G[N,D] → per-probe top-k (score desc, index asc).
//
// Replaces:
//   RecognitionEngine.recognize_with_db   inference/recognition_engine.py:267-289 (Python loop
//                                          over db rows + stable sort(reverse=True) + top-5)
//   recognize_with_faiss / IndexFlatIP     recognition_engine.py:291-326, extract_embeddings.py:595-645
//   notebook batched np.dot + argmax/argsort evaluate_arcface_kaggle.ipynb cells 15-16
//
// Scores are exact f32 (v_mfma_f32_16x16x4_f32: an fmaf chain per lane group, no reduced-
// precision path).  Each block owns 64 probes x one gallery split; it walks the split in
// 64-row tiles (D staged through LDS in 64-float chunks), writes the 64x64 score tile to
// LDS, and 4 threads per probe keep sorted register top-k lists (strict comparator with
// index tie-break, so equal scores keep the lower index first exactly like np.argmax and
// Python's stable sort).  A merge kernel (also used after the multi-GPU all-gather) folds
// the per-split lists.
#include "kernels.h"
#include <float.h>
#include <limits.h>

#include <algorithm>
#include <cstdlib>

namespace fr {
namespace {

constexpr int MP = 64;  // probes per block
constexpr int MG = 64;  // gallery rows per tile
constexpr int KC = 64;  // D chunk (floats)
constexpr int LD = KC + 4;

__device__ __forceinline__ bool better(float s1, int i1, float s2, int i2) {
    return s1 > s2 || (s1 == s2 && i1 < i2);
}

// Insert (s, idx) into a list sorted by better(): branch-free.  b[q] = the candidate beats entry q is
// monotone in q, so entry q becomes entry q-1 (b[q-1]), the candidate (first b), or stays.  (A swap chain
// compiled to a full list copy per step behind branches: the top-k filter then cost more than the MFMAs.)
template <int KMAX>
__device__ __forceinline__ void topk_insert(float (&ls)[KMAX], int (&li)[KMAX], float s, int idx) {
    bool b[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) b[q] = better(s, idx, ls[q], li[q]);
#pragma unroll
    for (int q = KMAX - 1; q > 0; --q) {
        const float sh = b[q - 1] ? ls[q - 1] : s;
        const int ih = b[q - 1] ? li[q - 1] : idx;
        ls[q] = b[q] ? sh : ls[q];
        li[q] = b[q] ? ih : li[q];
    }
    ls[0] = b[0] ? s : ls[0];
    li[0] = b[0] ? idx : li[0];
}

template <int KMAX>
__global__ __launch_bounds__(256) void match_partial_kernel(const float* __restrict__ P, int B,
                                                            const float* __restrict__ G, int64_t N, int D, int k,
                                                            int64_t index_base, int64_t rows_per_split, int n_split,
                                                            float* __restrict__ cs, int32_t* __restrict__ ci) {
    // LDS: sP[64][68] + sG[64][68] floats (34.8 KB), reused for the candidate merge;
    //      sS[64][65] score tile.
    __shared__ __attribute__((aligned(16))) float sPG[2 * MP * LD];
    __shared__ float sS[MP * (MG + 1)];
    float* sP = sPG;
    float* sG = sPG + MP * LD;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int p0 = blockIdx.x * MP;
    const int split = blockIdx.y;
    const int64_t g_begin = (int64_t)split * rows_per_split;
    int64_t g_end = g_begin + rows_per_split;
    if (g_end > N) g_end = N;

    float ls[KMAX];
    int li[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) { ls[q] = -INFINITY; li[q] = INT_MAX; }
    const int my_p = tid >> 2, my_sub = tid & 3;

    for (int64_t t0 = g_begin; t0 < g_end; t0 += MG) {
        f32x4_t acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        for (int d0 = 0; d0 < D; d0 += KC) {
            // stage P[p0:p0+64][d0:d0+64] and G[t0:t0+64][d0:d0+64]
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int q = tid + 256 * i;
                const int row = q >> 4, c4 = (q & 15) * 4;
                float4 pv = make_float4(0.f, 0.f, 0.f, 0.f), gv = pv;
                if (p0 + row < B && d0 + c4 < D) pv = *(const float4*)(P + (size_t)(p0 + row) * D + d0 + c4);
                if (t0 + row < g_end && d0 + c4 < D) gv = *(const float4*)(G + (size_t)(t0 + row) * D + d0 + c4);
                *(float4*)(sP + row * LD + c4) = pv;
                *(float4*)(sG + row * LD + c4) = gv;
            }
            __syncthreads();
#pragma unroll
            for (int t16 = 0; t16 < KC / 16; ++t16) {
                const int kof = 16 * t16 + 4 * (lane >> 4);
                const float4 a4 = *(const float4*)(sP + (16 * wave + (lane & 15)) * LD + kof);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float4 b4 = *(const float4*)(sG + (16 * j + (lane & 15)) * LD + kof);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, acc[j], 0, 0, 0);
                    acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, acc[j], 0, 0, 0);
                }
            }
            __syncthreads();
        }
        // acc[j][r] = score(probe 16*wave + 4*(lane>>4) + r, gallery row t0 + 16*j + (lane&15))
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                sS[(16 * wave + 4 * (lane >> 4) + r) * (MG + 1) + 16 * j + (lane & 15)] = acc[j][r];
        __syncthreads();
        // filter against this lane's current K-th best first: after the lists fill almost no score
        // qualifies, and the (divergent) sorted insert runs only for the few that do
        {
            const float thr = ls[KMAX - 1];
            const int thri = li[KMAX - 1];
            uint32_t mask = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int g = my_sub * 16 + i;
                if (t0 + g < g_end && better(sS[my_p * (MG + 1) + g], (int)(t0 + g + index_base), thr, thri))
                    mask |= 1u << i;
            }
            while (mask) {
                const int i = __builtin_ctz(mask);
                mask &= mask - 1;
                const int g = my_sub * 16 + i;
                topk_insert<KMAX>(ls, li, sS[my_p * (MG + 1) + g], (int)(t0 + g + index_base));
            }
        }
        __syncthreads();
    }

    // merge the 4 sub-lists of each probe
    float* ms = sPG;                       // [64][4][KMAX]
    int* mi = (int*)(sPG + MP * 4 * KMAX);  // [64][4][KMAX]
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
        ms[(my_p * 4 + my_sub) * KMAX + q] = ls[q];
        mi[(my_p * 4 + my_sub) * KMAX + q] = li[q];
    }
    __syncthreads();
    if (my_sub == 0) {
        for (int o = 1; o < 4; ++o)
            for (int q = 0; q < KMAX; ++q)
                topk_insert<KMAX>(ls, li, ms[(my_p * 4 + o) * KMAX + q], mi[(my_p * 4 + o) * KMAX + q]);
        const int p = p0 + my_p;
        if (p < B) {
            for (int q = 0; q < k; ++q) {
                const size_t o = ((size_t)p * n_split + split) * k + q;
                const bool valid = li[q] != INT_MAX;
                cs[o] = valid ? ls[q] : -INFINITY;
                ci[o] = valid ? li[q] : -1;
            }
        }
    }
}

// D = 512 variant of match_partial_kernel with the same scores bit for bit (the same v_mfma_f32_16x16x4f32
// sequence per output: k = 16 t16 + 4 (lane >> 4) + c) and the same candidate lists.  Each wave keeps its
// 16 probes' A fragments in registers for the whole split (32 float4 per lane, loaded once), so only
// gallery rows move through LDS: 64-row x 64-float chunks (256-B rows, 16-B slots XOR-swizzled with the
// row: conflict-free fragment reads) LDS-DMA'd three chunks ahead into a 4-buffer ring, counted vmcnt
// waits and one LDS-only barrier per chunk.  (The old kernel staged both operands per chunk through
// registers behind full barriers; register prefetch one chunk ahead left each block one 16-KB load in
// flight and ran 74 us at 256 x 10k, latency bound.)
constexpr int D512 = 512;
constexpr int NBUF = 4;                    // chunk ring depth (3 chunks in flight)
constexpr int CHUNK_B = MG * KC * 4;       // 16384
constexpr int P512_LDS = NBUF * CHUNK_B + MP * (MG + 1) * 4;
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 16-B LDS-DMA from inline asm (lane l lands at lds_addr + 16 l): the compiler does not see the LDS write,
// so it adds no vmcnt(0) before later LDS accesses; the kernel's own counted waits cover it
typedef int v4i32 __attribute__((ext_vector_type(4)));
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16_asm(const v4i32& rsrc, uint32_t lds_addr, uint32_t voff) {
    asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
                 :
                 : "v"(voff), "s"(rsrc), "s"(__builtin_amdgcn_readfirstlane(lds_addr))
                 : "memory", "m0");
}
#pragma clang diagnostic pop

template <int KMAX>
__global__ __launch_bounds__(256, 1) void match_p512_kernel(const float* __restrict__ P, int B,
                                                            const float* __restrict__ G, int64_t N, int k,
                                                            int64_t index_base, int64_t rows_per_split, int n_split,
                                                            float* __restrict__ cs, int32_t* __restrict__ ci) {
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [NBUF chunks][sS]
    float* sS = (float*)(smem + NBUF * CHUNK_B);

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int p0 = blockIdx.x * MP;
    const int split = blockIdx.y;
    const int64_t g_begin = (int64_t)split * rows_per_split;
    int64_t g_end = g_begin + rows_per_split;
    if (g_end > N) g_end = N;
    const int rows = (int)(g_end - g_begin);  // <= 64 tiles of 64 rows (the plan's bound)
    const int ntiles = (rows + MG - 1) / MG;

    // the wave's A fragments: pa[t] = P[p0 + 16 wave + (lane & 15)][16 t + 4 (lane >> 4) .. + 3]
    float4 pa[D512 / 16];
    {
        const int p = p0 + 16 * wave + (lane & 15);
        const float* src = P + (size_t)min(p, B - 1) * D512 + 4 * (lane >> 4);
#pragma unroll
        for (int t = 0; t < D512 / 16; ++t) pa[t] = *(const float4*)(src + 16 * t);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the DMA wait counts below see only DMAs
        const float z = p < B ? 1.f : 0.f;  // rows past the batch: zero probes (no branch around the loads)
#pragma unroll
        for (int t = 0; t < D512 / 16; ++t) pa[t] = make_float4(pa[t].x * z, pa[t].y * z, pa[t].z * z, pa[t].w * z);
    }

    // the split's rows as a buffer resource: rows past the split read 0 (out of range)
    const uint64_t gp = (uint64_t)(G + (size_t)g_begin * D512);
    const v4i32 gr = {(int)(uint32_t)gp, (int)((gp >> 32) & 0xffff), rows * D512 * 4, 0x00020000};
    const uint32_t smem_base = (uint32_t)(uintptr_t)smem;
    // chunk c = (tile c / 8, floats 64 (c % 8) ..) into ring buffer c % NBUF: wave w issues pieces w + 4u,
    // piece q = rows 4q .. 4q + 3, lane -> row 4q + (lane >> 4), slot lane & 15 = column group
    // (lane & 15) ^ (row & 15).  Chunks past the split are issued anyway (all out of range) so that every
    // wait count is the same.
    auto issue_chunk = [&](int c) {
        const int t = c >> 3, d0 = (c & 7) * KC;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int q = wave + 4 * u, row = 4 * q + (lane >> 4), g = (lane & 15) ^ (row & 15);
            const uint32_t off = (uint32_t)((t * MG + row) * (D512 * 4) + (d0 + 4 * g) * 4);
            dma16_asm(gr, smem_base + (c % NBUF) * CHUNK_B + q * 1024, off);
        }
    };
#pragma unroll
    for (int c = 0; c < NBUF - 1; ++c) issue_chunk(c);

    float ls[KMAX];
    int li[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) { ls[q] = -INFINITY; li[q] = INT_MAX; }
    const int my_p = tid >> 2, my_sub = tid & 3;

    for (int tl = 0; tl < ntiles; ++tl) {
        const int64_t t0 = g_begin + (int64_t)tl * MG;
        f32x4_t acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ch = 0; ch < D512 / KC; ++ch) {
            // chunk 8 tl + ch landed: only the two chunks issued after it (8 DMAs) may be in flight
            __builtin_amdgcn_sched_barrier(0);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
            lds_barrier();
            issue_chunk(8 * tl + ch + NBUF - 1);  // into the buffer read last chunk
            const char* buf = smem + (ch % NBUF) * CHUNK_B;
            // all 16 B fragments of the chunk first, one LDS wait (left alone the compiler waits before every
            // 4 MFMAs, and one wave per SIMD cannot hide that), then the MFMAs with the 4 accumulators
            // interleaved (a dependent f32 MFMA waits 40 cycles, the issue is 32): per accumulator the order
            // is unchanged, x y z w per t16
            float4 b4[KC / 16][4];
#pragma unroll
            for (int t16 = 0; t16 < KC / 16; ++t16) {
                const int slot = (4 * t16 + (lane >> 4)) ^ (lane & 15);
#pragma unroll
                for (int j = 0; j < 4; ++j) b4[t16][j] = *(const float4*)(buf + (16 * j + (lane & 15)) * 256 + slot * 16);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);  // nothing crosses the wait (MFMAs are not memory operations)
#pragma unroll
            for (int t16 = 0; t16 < KC / 16; ++t16) {
                const float4 a4 = pa[(KC / 16) * ch + t16];
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4[t16][j].x, acc[j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4[t16][j].y, acc[j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4[t16][j].z, acc[j], 0, 0, 0);
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4[t16][j].w, acc[j], 0, 0, 0);
            }
        }
        // scores -> LDS (its previous readers are 8 barriers back), then the filtered top-k insert
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                sS[(16 * wave + 4 * (lane >> 4) + r) * (MG + 1) + 16 * j + (lane & 15)] = acc[j][r];
        lds_barrier();
        {
            // filter (no branches: all 16 scores read, 32-bit indices), then the few inserts.  Threshold:
            // the best of the probe's 4 sub-lists' last entries (lanes 4p .. 4p+3): that sub-list holds
            // KMAX >= k entries at least that good, so nothing worse can reach the split's top k
            float thr = ls[KMAX - 1];
            int thri = li[KMAX - 1];
#pragma unroll
            for (int o = 1; o <= 2; o <<= 1) {
                const float os = __shfl_xor(thr, o);
                const int oi = __shfl_xor(thri, o);
                if (better(os, oi, thr, thri)) { thr = os; thri = oi; }
            }
            const int ibase = (int)(t0 + index_base) + my_sub * 16;
            const int lim = (int)min((int64_t)MG, g_end - t0) - my_sub * 16;
            const float* row = sS + my_p * (MG + 1) + my_sub * 16;
            uint32_t mask = 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) mask |= (((i < lim) & better(row[i], ibase + i, thr, thri)) ? 1u : 0u) << i;
            while (mask) {
                const int i = __builtin_ctz(mask);
                mask &= mask - 1;
                topk_insert<KMAX>(ls, li, row[i], ibase + i);
            }
        }
    }

    // merge the 4 sub-lists of each probe in the ring's LDS: the trailing (out-of-range) DMAs land first
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float* ms = (float*)smem;                 // [64][4][KMAX]
    int* mi = (int*)(smem + MP * 4 * KMAX * 4);  // [64][4][KMAX]
#pragma unroll
    for (int q = 0; q < KMAX; ++q) {
        ms[(my_p * 4 + my_sub) * KMAX + q] = ls[q];
        mi[(my_p * 4 + my_sub) * KMAX + q] = li[q];
    }
    __syncthreads();
    if (my_sub == 0) {
        for (int o = 1; o < 4; ++o)
            for (int q = 0; q < KMAX; ++q)
                topk_insert<KMAX>(ls, li, ms[(my_p * 4 + o) * KMAX + q], mi[(my_p * 4 + o) * KMAX + q]);
        const int p = p0 + my_p;
        if (p < B) {
            for (int q = 0; q < k; ++q) {
                const size_t o = ((size_t)p * n_split + split) * k + q;
                const bool valid = li[q] != INT_MAX;
                cs[o] = valid ? ls[q] : -INFINITY;
                ci[o] = valid ? li[q] : -1;
            }
        }
    }
}

// One wave per probe: lanes insert strided candidates into local lists, then k rounds of a
// wave-wide (score desc, index asc) argmax pop.  Candidate j of list l of probe p is at
// p * probe_stride + l * list_stride + j (elements) in cs / ci: [P][n_lists][k] for fr_topk_merge
// (probe_stride = n_lists k, list_stride = k), the all-gathered [rank][2][P][k] exchange block for
// fr_topk_merge_ranks (probe_stride = k, list_stride = 2 P k, ci = cs + P k).
template <int KMAX>
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ cs, const int32_t* __restrict__ ci,
                                                         int B, int n_lists, int k, int64_t probe_stride,
                                                         int64_t list_stride, float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_i) {
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= B) return;
    float ls[KMAX];
    int li[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) { ls[q] = -INFINITY; li[q] = INT_MAX; }
    const int n = n_lists * k;
    // 8 candidates per lane in flight per round (their loads issued together, then the inserts): one
    // load at a time exposed the L2 latency per candidate
    const float* ps = cs + (size_t)p * probe_stride;
    const int32_t* pi = ci + (size_t)p * probe_stride;
    for (int c0 = 0; c0 < n; c0 += 64 * 8) {
        float sv[8];
        int iv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int c = c0 + 64 * u + lane;
            const bool ok = c < n;
            const int l = c / k;
            const size_t o = (size_t)l * list_stride + (c - l * k);
            sv[u] = ok ? ps[o] : -INFINITY;
            iv[u] = ok ? pi[o] : -1;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (iv[u] >= 0) topk_insert<KMAX>(ls, li, sv[u], iv[u]);
    }
    int head = 0;
    for (int q = 0; q < k; ++q) {
        float bs = -INFINITY;
        int bi = INT_MAX;
#pragma unroll
        for (int h = 0; h < KMAX; ++h)
            if (h == head) { bs = ls[h]; bi = li[h]; }
        float ws = bs;
        int wi = bi;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            const float os = __shfl_xor(ws, o);
            const int oi = __shfl_xor(wi, o);
            if (better(os, oi, ws, wi)) { ws = os; wi = oi; }
        }
        if (wi == bi && bi != INT_MAX) ++head;  // indices are unique: the owner pops
        if (lane == 0) {
            out_s[(size_t)p * k + q] = wi == INT_MAX ? -INFINITY : ws;
            out_i[(size_t)p * k + q] = wi == INT_MAX ? -1 : wi;
        }
    }
}

}  // namespace

static bool p512_enabled() {
    static const bool on = [] { return ab_int("match_p512", 1) != 0; }();
    return on;
}

// Split plan of the exact match.  match_p512_kernel (D = 512, k <= 8) keeps a wave's probes in registers,
// so a split should span several 64-row tiles: choose the tiles per split r minimising (rounds of 256
// resident blocks) x r, ties to the larger r (fewer candidate lists for the merge); e.g. 256 x 10k: 3
// tiles per split, 212 blocks (one per CU) instead of 628 one-tile blocks.
void match_split_plan(int B, int64_t N, int D, int k, int* n_split, int64_t* rows_per_split) {
    if (D == D512 && k <= 8 && p512_enabled() && B > 0 && N > 0) {
        const int64_t pb = (B + MP - 1) / MP, T = (N + MG - 1) / MG;
        int64_t best_r = 1;
        double best = 1e30;
        static const int env_r = ab_int("match_tiles", 0);  // experiments: tiles per split
        for (int64_t r = 1; r <= T && r <= 64; ++r) {
            if (env_r > 0 && r != std::min<int64_t>(env_r, std::min<int64_t>(T, 64))) continue;
            const int64_t blocks = pb * ((T + r - 1) / r);
            const double cost = (double)((blocks + 255) / 256) * r + 0.02 * (double)((T + r - 1) / r);
            if (cost <= best) { best = cost; best_r = r; }
        }
        *rows_per_split = best_r * MG;
        *n_split = (int)((T + best_r - 1) / best_r);
        return;
    }
    match_split_plan(B, N, n_split, rows_per_split);
}

void match_split_plan(int B, int64_t N, int* n_split, int64_t* rows_per_split) {
    const int pt = (B + MP - 1) / MP;
#ifndef FR_MATCH_BLOCKS
#define FR_MATCH_BLOCKS 1024
#endif
    int64_t want = (FR_MATCH_BLOCKS + pt - 1) / pt;  // aim for ~4 blocks per CU (256 x 10k: 105 -> 87 us vs 2)
    int64_t tiles = (N + MG - 1) / MG;
    if (want > tiles) want = tiles;
    if (want < 1) want = 1;
    int64_t rps = ((tiles + want - 1) / want) * MG;
    if (rps < MG) rps = MG;
    *rows_per_split = rps;
    *n_split = (int)((N + rps - 1) / rps);
    if (*n_split < 1) *n_split = 1;
}

hipError_t launch_match_topk(const float* P, int B, const float* G, int64_t N, int D, int k, int64_t index_base,
                             float* cand_s, int32_t* cand_i, int n_split, int64_t rows_per_split, hipStream_t s) {
    dim3 grid((B + MP - 1) / MP, n_split);
    if (D == D512 && p512_enabled() && B > 0 && k <= 8) {  // (16-deep lists would spill next to the register probes)
        if (rows_per_split > 64 * MG) return hipErrorInvalidValue;  // the plan's bound (32-bit DMA offsets)
        // lists exactly as deep as needed for the usual k <= 5 (top-5 is the reference's default)
        auto kern = k <= 5 ? match_p512_kernel<5> : match_p512_kernel<8>;
        static bool attr[2] = {false, false};
        if (!attr[k <= 5]) {
            (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, P512_LDS);
            attr[k <= 5] = true;
        }
        hipLaunchKernelGGL(kern, grid, dim3(256), P512_LDS, s, P, B, G, N, k, index_base, rows_per_split, n_split,
                           cand_s, cand_i);
        return hipGetLastError();
    }
    if (k <= 8)
        hipLaunchKernelGGL(match_partial_kernel<8>, grid, dim3(256), 0, s, P, B, G, N, D, k, index_base,
                           rows_per_split, n_split, cand_s, cand_i);
    else
        hipLaunchKernelGGL(match_partial_kernel<16>, grid, dim3(256), 0, s, P, B, G, N, D, k, index_base,
                           rows_per_split, n_split, cand_s, cand_i);
    return hipGetLastError();
}

static hipError_t merge_strided(const float* cs, const int32_t* ci, int B, int n_lists, int k, int64_t probe_stride,
                                int64_t list_stride, float* out_s, int32_t* out_i, hipStream_t s) {
    dim3 grid((B + 3) / 4);
    if (k <= 8)
        hipLaunchKernelGGL(topk_merge_kernel<8>, grid, dim3(256), 0, s, cs, ci, B, n_lists, k, probe_stride, list_stride,
                           out_s, out_i);
    else
        hipLaunchKernelGGL(topk_merge_kernel<16>, grid, dim3(256), 0, s, cs, ci, B, n_lists, k, probe_stride,
                           list_stride, out_s, out_i);
    return hipGetLastError();
}

hipError_t launch_topk_merge(const float* cs, const int32_t* ci, int B, int n_lists, int k, float* out_s,
                             int32_t* out_i, hipStream_t s) {
    return merge_strided(cs, ci, B, n_lists, k, (int64_t)n_lists * k, k, out_s, out_i, s);
}

hipError_t launch_topk_merge_ranks(const void* xchg, int n_ranks, int B, int k, float* out_s, int32_t* out_i,
                                   hipStream_t s) {
    const float* cs = (const float*)xchg;
    return merge_strided(cs, (const int32_t*)(cs + (size_t)B * k), B, n_ranks, k, k, 2 * (int64_t)B * k, out_s,
                         out_i, s);
}

// ---------------------------------------------------------------------------------------------------
// Large k (17 .. FR_TOPK_LARGE_MAX): IndexFlatIP.search with any k (recognition_engine.py:291-326 passes
// the caller's k straight to faiss).  Register top-k lists do not scale past 16, so the large path
// materialises the exact score rows -- the SAME v_mfma_f32_16x16x4f32 sequence per output as
// match_partial_kernel, so a large-k list starts with exactly the small-k list -- and selects per probe
// with a radix select on the order-preserving u32 image of the score (3 digit passes of 11/11/10 bits
// over the row, histograms in LDS), takes every score above the k-th and the lowest-index ties at it,
// and bitonic-sorts the k survivors (score desc, index asc) in LDS.
namespace {

__global__ __launch_bounds__(256) void match_scores_kernel(const float* __restrict__ P, int B, const float* __restrict__ G,
                                                           int64_t N, int D, float* __restrict__ S) {
    __shared__ __attribute__((aligned(16))) float sPG[2 * MP * LD];
    float* sP = sPG;
    float* sG = sPG + MP * LD;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int p0 = blockIdx.x * MP;
    const int64_t t0 = (int64_t)blockIdx.y * MG;
    const int64_t g_end = N;
    f32x4_t acc[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    for (int d0 = 0; d0 < D; d0 += KC) {  // match_partial_kernel's tile, operation for operation
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int q = tid + 256 * i;
            const int row = q >> 4, c4 = (q & 15) * 4;
            float4 pv = make_float4(0.f, 0.f, 0.f, 0.f), gv = pv;
            if (p0 + row < B && d0 + c4 < D) pv = *(const float4*)(P + (size_t)(p0 + row) * D + d0 + c4);
            if (t0 + row < g_end && d0 + c4 < D) gv = *(const float4*)(G + (size_t)(t0 + row) * D + d0 + c4);
            *(float4*)(sP + row * LD + c4) = pv;
            *(float4*)(sG + row * LD + c4) = gv;
        }
        __syncthreads();
#pragma unroll
        for (int t16 = 0; t16 < KC / 16; ++t16) {
            const int kof = 16 * t16 + 4 * (lane >> 4);
            const float4 a4 = *(const float4*)(sP + (16 * wave + (lane & 15)) * LD + kof);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float4 b4 = *(const float4*)(sG + (16 * j + (lane & 15)) * LD + kof);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.x, b4.x, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.y, b4.y, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.z, b4.z, acc[j], 0, 0, 0);
                acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4.w, b4.w, acc[j], 0, 0, 0);
            }
        }
        __syncthreads();
    }
    // acc[j][r] = score(probe 16 wave + 4 (lane >> 4) + r, row t0 + 16 j + (lane & 15))
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int p = p0 + 16 * wave + 4 * (lane >> 4) + r;
            const int64_t g = t0 + 16 * j + (lane & 15);
            if (p < B && g < N) S[(size_t)p * N + g] = acc[j][r];
        }
}

// order-preserving u32 image of a score (-0 folds onto +0: the small-k comparator ties them)
__device__ __forceinline__ uint32_t skey(float v) {
    const uint32_t b = __float_as_uint(v == 0.f ? 0.f : v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}

constexpr int TK_THREADS = 1024;

// Block-wide exclusive prefix sum of one int per thread (+ the total).
__device__ __forceinline__ int block_excl_scan(int v, int* red, int* total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) red[wave] = x;
    __syncthreads();
    int before = 0, all = 0;
    for (int w = 0; w < TK_THREADS / 64; ++w) {
        const int c = red[w];
        before += w < wave ? c : 0;
        all += c;
    }
    __syncthreads();
    *total = all;
    return before + x - v;
}

__global__ __launch_bounds__(TK_THREADS) void topk_large_kernel(const float* __restrict__ S, int64_t N, int k,
                                                                int64_t index_base, float* __restrict__ out_s,
                                                                int32_t* __restrict__ out_i) {
    __shared__ uint32_t hist[2048];
    __shared__ unsigned long long keys[FR_TOPK_LARGE_MAX];
    __shared__ int red[TK_THREADS / 64];
    __shared__ int sel[3];
    const int tid = threadIdx.x;
    const float* row = S + (size_t)blockIdx.x * N;
    const int kk = (int)(N < (int64_t)k ? N : (int64_t)k);
    uint32_t prefix = 0, pmask = 0;
    int kr = kk;
    // ---- radix select: the exact u32 key T of the kk-th largest score, and how many ties at T to take
    for (int pass = 0; pass < 3; ++pass) {
        const int shift = pass == 0 ? 21 : (pass == 1 ? 10 : 0);
        const int nb = pass < 2 ? 2048 : 1024;
        for (int i = tid; i < 2048; i += TK_THREADS) hist[i] = 0;
        __syncthreads();
        for (int64_t i = tid; i < N; i += TK_THREADS) {
            const uint32_t u = skey(row[i]);
            if ((u & pmask) == prefix) atomicAdd(&hist[(u >> shift) & (nb - 1)], 1u);
        }
        __syncthreads();
        if (tid < 64) {  // wave 0: lane l owns bins nb-1-l*per .. (descending), find where the count reaches kr
            const int per = nb / 64;
            int c = 0;
            for (int q = 0; q < per; ++q) c += (int)hist[nb - 1 - tid * per - q];
            int x = c;
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o);
                if (tid >= o) x += y;
            }
            const int before = x - c;
            if (before < kr && x >= kr) {
                int acc = before;
                for (int q = 0; q < per; ++q) {
                    const int d = nb - 1 - tid * per - q;
                    const int h = (int)hist[d];
                    if (acc + h >= kr) {
                        sel[0] = d;
                        sel[1] = acc;
                        break;
                    }
                    acc += h;
                }
            }
        }
        __syncthreads();
        prefix |= (uint32_t)sel[0] << shift;
        pmask |= (uint32_t)(nb - 1) << shift;
        kr -= sel[1];
        __syncthreads();
    }
    const uint32_t T = prefix;
    // ---- gather: every key above T (unordered), then the kr lowest-index rows equal to T (ordered scan)
    if (tid == 0) sel[2] = 0;
    __syncthreads();
    for (int64_t i = tid; i < N; i += TK_THREADS) {
        const uint32_t u = skey(row[i]);
        if (u > T) {
            const int slot = atomicAdd(&sel[2], 1);
            keys[slot] = ((unsigned long long)u << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)i);
        }
    }
    __syncthreads();
    const int above = sel[2];
    int taken = 0;
    for (int64_t c0 = 0; c0 < N && taken < kr; c0 += TK_THREADS) {
        const int64_t i = c0 + tid;
        const int eq = i < N && skey(row[i]) == T;
        int total;
        const int pos = block_excl_scan(eq, red, &total);
        if (eq && taken + pos < kr)
            keys[above + taken + pos] = ((unsigned long long)T << 32) | (uint32_t)(0xFFFFFFFFu - (uint32_t)i);
        taken += total;
    }
    __syncthreads();
    // ---- bitonic sort of the kk keys, descending (pad with 0: below every real key)
    int P2 = 1;
    while (P2 < kk) P2 <<= 1;
    for (int i = kk + tid; i < P2; i += TK_THREADS) keys[i] = 0ull;
    __syncthreads();
    for (int size = 2; size <= P2; size <<= 1)
        for (int stride = size >> 1; stride > 0; stride >>= 1) {
            for (int i = tid; i < P2; i += TK_THREADS) {
                const int j = i ^ stride;
                if (j > i) {
                    const bool desc = (i & size) == 0;
                    const unsigned long long a = keys[i], b = keys[j];
                    if (desc ? a < b : a > b) {
                        keys[i] = b;
                        keys[j] = a;
                    }
                }
            }
            __syncthreads();
        }
    for (int q = tid; q < k; q += TK_THREADS) {
        float sc = -INFINITY;
        int32_t ix = -1;
        if (q < kk) {
            const unsigned long long kv = keys[q];
            const uint32_t u = (uint32_t)(kv >> 32);
            const uint32_t b = (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u;
            sc = __uint_as_float(b);
            ix = (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)kv) + index_base);
        }
        out_s[(size_t)blockIdx.x * k + q] = sc;
        out_i[(size_t)blockIdx.x * k + q] = ix;
    }
}

}  // namespace

// S: B x N f32 scratch (the caller's, stream-ordered).  out: [B][k].
hipError_t launch_match_topk_large(const float* P, int B, const float* G, int64_t N, int D, int k, int64_t index_base,
                                   float* S, float* out_s, int32_t* out_i, hipStream_t s) {
    if (B <= 0 || N <= 0 || k <= 0 || k > FR_TOPK_LARGE_MAX || N > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(match_scores_kernel, dim3((B + MP - 1) / MP, (unsigned)((N + MG - 1) / MG)), dim3(256), 0, s, P,
                       B, G, N, D, S);
    hipLaunchKernelGGL(topk_large_kernel, dim3(B), dim3(TK_THREADS), 0, s, S, N, k, index_base, out_s, out_i);
    return hipGetLastError();
}

}  // namespace fr
