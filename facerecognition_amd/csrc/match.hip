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

namespace fr {
namespace {

constexpr int MP = 64;  // probes per block
constexpr int MG = 64;  // gallery rows per tile
constexpr int KC = 64;  // D chunk (floats)
constexpr int LD = KC + 4;

__device__ __forceinline__ bool better(float s1, int i1, float s2, int i2) {
    return s1 > s2 || (s1 == s2 && i1 < i2);
}

template <int KMAX>
__device__ __forceinline__ void topk_insert(float (&ls)[KMAX], int (&li)[KMAX], float s, int idx) {
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

// One wave per probe: lanes insert strided candidates into local lists, then k rounds of a
// wave-wide (score desc, index asc) argmax pop.
template <int KMAX>
__global__ __launch_bounds__(256) void topk_merge_kernel(const float* __restrict__ cs, const int32_t* __restrict__ ci,
                                                         int B, int n_lists, int k, float* __restrict__ out_s,
                                                         int32_t* __restrict__ out_i) {
    const int lane = threadIdx.x & 63;
    const int p = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (p >= B) return;
    float ls[KMAX];
    int li[KMAX];
#pragma unroll
    for (int q = 0; q < KMAX; ++q) { ls[q] = -INFINITY; li[q] = INT_MAX; }
    const int n = n_lists * k;
    for (int c = lane; c < n; c += 64) {
        const int idx = ci[(size_t)p * n + c];
        if (idx >= 0) topk_insert<KMAX>(ls, li, cs[(size_t)p * n + c], idx);
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
    if (k <= 8)
        hipLaunchKernelGGL(match_partial_kernel<8>, grid, dim3(256), 0, s, P, B, G, N, D, k, index_base,
                           rows_per_split, n_split, cand_s, cand_i);
    else
        hipLaunchKernelGGL(match_partial_kernel<16>, grid, dim3(256), 0, s, P, B, G, N, D, k, index_base,
                           rows_per_split, n_split, cand_s, cand_i);
    return hipGetLastError();
}

hipError_t launch_topk_merge(const float* cs, const int32_t* ci, int B, int n_lists, int k, float* out_s,
                             int32_t* out_i, hipStream_t s) {
    dim3 grid((B + 3) / 4);
    if (k <= 8)
        hipLaunchKernelGGL(topk_merge_kernel<8>, grid, dim3(256), 0, s, cs, ci, B, n_lists, k, out_s, out_i);
    else
        hipLaunchKernelGGL(topk_merge_kernel<16>, grid, dim3(256), 0, s, cs, ci, B, n_lists, k, out_s, out_i);
    return hipGetLastError();
}

}  // namespace fr
