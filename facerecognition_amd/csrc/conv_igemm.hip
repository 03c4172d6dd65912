// Implicit-GEMM convolution for CDNA4 (gfx950): NHWC 16-bit activations, KRSC 16-bit weights,
// f32 accumulation on v_mfma_f32_16x16x32_{bf16,f16}, fused epilogue.
//
// Replaces the torch conv+BN+ReLU/PReLU+residual chains of the reference backbones:
//   ResNetBackbone.forward            models/arcface/arcface_model.py:118-132 (torchvision Bottleneck)
//   FaceNet InceptionResnetV1 trunk   models/facenet/facenet_model.py:12-16 (BasicConv2d/Block35/17/8)
//   insightface IBasicBlock (IResNet100, README.md:72; no reference code)
//
// GEMM view: C[n][m] = sum_k W[n][k] * X[m][k]; m = output pixel (b, oh, ow), n = output channel,
// k = (r, s, c) with c fastest.  MFMA operand A = weight rows (n), operand B = gathered activation
// rows (m): each lane's 4 accumulator registers are 4 consecutive channels of one pixel.
//
// Staging: both operand tiles go global → LDS by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per
// wave instruction = 8 tile rows of 128 B), two LDS stages, one barrier per 64-deep K-step: the DMA
// for step t+1 is issued before the MFMAs of step t.  The im2col gather is the per-lane source
// offset; a padding tap or a row past M gets an out-of-range offset and the buffer unit returns
// zeros (no select, no zero page).  LDS rows are 128 B; the 16-B chunk index is XOR-swizzled with
// (row>>1)&7 by permuting the per-lane SOURCE chunk (the DMA destination is lane-linear), which
// makes the MFMA-fragment ds_read_b128 loads bank-conflict free.
// FASTK (Cin % 64 == 0): a K-step is one (r, s) tap and 64 channels, tracked in scalars.
#include "kernels.h"

#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>

namespace fr {
typedef unsigned int v4u32_t __attribute__((ext_vector_type(4)));

namespace {

constexpr int BK = 64;
constexpr uint32_t OOB = 0x80000000u;  // buffer offset past num_records → the DMA writes zeros

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

template <int N>
__device__ __forceinline__ void wait_vmn() {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, 0, 0, 0);
}

// Shared fused epilogue for 8 consecutive channels n..n+7 of output pixel m.
template <bool F16>
__device__ __forceinline__ void epilogue8(const ConvArgs& p, float* v, int m, int n) {
    typedef Num<F16> T;
    if (p.bias9) {
        const int HoWo = p.Ho * p.Wo, r = m % HoWo;
        const float* bb = p.bias9 + (size_t)border_class(r / p.Wo, r % p.Wo, p.Ho, p.Wo) * p.Npad + n;
        const float4 b0 = *(const float4*)bb, b1 = *(const float4*)(bb + 4);
        v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
        v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    } else if (p.bias) {
        const float4 b0 = *(const float4*)(p.bias + n), b1 = *(const float4*)(p.bias + n + 4);
        v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
        v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
    }
    if (p.res) {
        const uint4 r = *(const uint4*)(p.res + (size_t)m * p.Cres + p.res_off + n);
        float f[8];
        T::unpack8(r, f);
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += f[e];
    }
    if (p.act == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
    } else if (p.act == 2) {
        const float4 s0 = *(const float4*)(p.slope + n), s1 = *(const float4*)(p.slope + n + 4);
        const float sl[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * sl[e];
    }
    *(uint4*)(p.y + (size_t)m * p.Cy + p.y_off + n) = F16 && p.y_bf16 ? Num<false>::pack8(v) : T::pack8(v);
    if (p.y2) {
        const float4 a0 = *(const float4*)(p.aff_s + n), a1 = *(const float4*)(p.aff_s + n + 4);
        const float4 c0 = *(const float4*)(p.aff_b + n), c1 = *(const float4*)(p.aff_b + n + 4);
        float u[8] = {v[0] * a0.x + c0.x, v[1] * a0.y + c0.y, v[2] * a0.z + c0.z, v[3] * a0.w + c0.w,
                      v[4] * a1.x + c1.x, v[5] * a1.y + c1.y, v[6] * a1.z + c1.z, v[7] * a1.w + c1.w};
        *(uint4*)(p.y2 + (size_t)m * p.Cy2 + p.y2_off + n) = T::pack8(u);
    }
}

template <int BM, int BN, int WM, int WN, int STAGES>
struct ConvGeom {
    static constexpr int NW = WM * WN, NT = 64 * NW;
    static constexpr int STAGE = (BM + BN) * BK * 2;  // bytes per LDS stage
    static constexpr int LDS_A = STAGES * STAGE, LDS_E = BM * (BN + 4) * 4;
    static constexpr int LDS_BYTES = LDS_A > LDS_E ? LDS_A : LDS_E;
    static constexpr int BLOCKS_PER_CU = (160 * 1024) / LDS_BYTES > 2 ? 2 : (160 * 1024) / LDS_BYTES;
    static constexpr int MIN_WAVES_PER_SIMD = BLOCKS_PER_CU * NW / 4;
};

template <bool F16, int BM, int BN, int WM, int WN, int STAGES, bool FASTK>
__global__ __launch_bounds__(64 * WM * WN, (ConvGeom<BM, BN, WM, WN, STAGES>::MIN_WAVES_PER_SIMD))
void conv_igemm_kernel(ConvArgs p, int tiles_n, int kt_per_split) {
    typedef ConvGeom<BM, BN, WM, WN, STAGES> Gm;
    constexpr int NW = Gm::NW, NT = Gm::NT;
    static_assert(NW == 4 || NW == 8, "4 or 8 waves");
    typedef Num<F16> T;
    typedef typename T::frag frag;
    constexpr int TWM = BM / WM, TWN = BN / WN;  // wave tile (pixels, channels)
    constexpr int FM = TWM / 16, FN = TWN / 16;  // MFMA tiles per wave
    constexpr int NA = BM / (8 * NW), NB = BN / (8 * NW);  // DMA instructions per wave per K-step
    static_assert(NA * 8 * NW == BM && NB * 8 * NW == BN, "tile rows must split evenly over the waves");
    constexpr int STAGE_A = BM * BK * 2, STAGE = Gm::STAGE;
    constexpr int EPI_LD = BN + 4;
    constexpr int LDS_BYTES = Gm::LDS_BYTES;
    __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];  // the ONLY LDS object (guide §5 trap 4a)

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int wm = wave % WM, wn = wave / WM;
    const int lid = xcd_remap(blockIdx.x, gridDim.x);
    const int tm = lid / tiles_n, tn = lid - tm * tiles_n;
    const int m0 = tm * BM, n0 = tn * BN;
    const int split = blockIdx.y;
    const int nkt = p.Kpad / BK;
    const int kt0 = split * kt_per_split;
    const int kt1 = min(nkt, kt0 + kt_per_split);

    // Lane's DMA slot: rows 8*(wave + NW*i) + (lane>>3); the logical chunk it fetches is the same for
    // every i (the swizzle term (row>>1)&7 = (4*wave + 4*NW*i + (lane>>4)) & 7 does not depend on i).
    const int lrow = lane >> 3;
    const int cl = (lane & 7) ^ ((4 * wave + (lane >> 4)) & 7);

    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * p.H * p.W * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const uint32_t w_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.Npad * p.Kpad * 2);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc((void*)p.w, 0, w_bytes, 0x00020000);

    const int HoWo = p.Ho * p.Wo;
    int a_ih[NA], a_iw[NA];
    uint32_t a_base[NA];  // byte offset of (b, ih0, iw0, x_off [+ 8*cl]) — wraps if ih0/iw0 < 0, only used when valid
    uint32_t a_base2[NA];  // FASTK + x2: byte offset of (b, oh*st2, ow*st2, x2_off + 8*cl) in x2, OOB past M
#pragma unroll
    for (int i = 0; i < NA; ++i) {
        const int m = m0 + 8 * (wave + NW * i) + lrow;
        if (m < p.M) {
            const int b = m / HoWo, r = m - b * HoWo;
            const int oh = r / p.Wo, ow = r - oh * p.Wo;
            a_ih[i] = oh * p.sh - p.ph;
            a_iw[i] = ow * p.sw - p.pw;
            // FASTK: c_cur is the K-step's channel base, the lane adds its chunk here;
            // generic: c_cur already is the lane's own channel.
            a_base[i] = (uint32_t)((((b * p.H + a_ih[i]) * p.W + a_iw[i]) * p.Cx + p.x_off + (FASTK ? 8 * cl : 0)) * 2);
            a_base2[i] = FASTK && p.x2
                             ? (uint32_t)((((b * p.H2 + oh * p.st2) * p.W2 + ow * p.st2) * p.Cx2 + p.x2_off + 8 * cl) * 2)
                             : OOB;
        } else {
            a_ih[i] = -(1 << 28);
            a_iw[i] = 0;
            a_base[i] = 0;
            a_base2[i] = OOB;
        }
    }
    // K-steps from kt_x2 on read x2 (the K-concatenated 1x1 projection)
    const int kt_x2 = FASTK && p.x2 ? p.K1 / BK : nkt;
    const __amdgpu_buffer_rsrc_t x2r = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.x2 ? p.x2 : p.x), 0,
        (uint32_t)min((size_t)0x7fffffff, p.x2 ? (size_t)p.B * p.H2 * p.W2 * p.Cx2 * 2 : (size_t)0), 0x00020000);
    uint32_t b_base[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) b_base[j] = (uint32_t)(((n0 + 8 * (wave + NW * j) + lrow) * p.Kpad + 8 * cl) * 2);

    // K-step position: FASTK → wave-uniform (r, s, c0); generic → per-lane (r, s, c) of k = kt*64 + 8*cl.
    int r_cur, s_cur, c_cur;
    {
        const int k = kt0 * BK + (FASTK ? 0 : 8 * cl);
        const int rs = k / p.Cin;
        c_cur = k - rs * p.Cin;
        r_cur = rs / p.Kw;
        s_cur = rs - r_cur * p.Kw;
    }
    int k_cur = kt0 * BK + 8 * cl;

    auto issue = [&](int kt, int buf) {
        const char* sA = smem + buf * STAGE;
        const char* sB = sA + STAGE_A;
        if (FASTK && kt >= kt_x2) {  // projection K-steps: x2 at the output's stride-st2 position
            const uint32_t c2 = (uint32_t)((kt - kt_x2) * BK * 2);
#pragma unroll
            for (int i = 0; i < NA; ++i)
                dma16(x2r, sA + (wave + NW * i) * 1024, a_base2[i] == OOB ? OOB : a_base2[i] + c2);
        } else {
            const int soff = ((r_cur * p.W + s_cur) * p.Cx + c_cur) * 2;
#pragma unroll
            for (int i = 0; i < NA; ++i) {
                const int ih = a_ih[i] + r_cur, iw = a_iw[i] + s_cur;
                bool ok = (unsigned)ih < (unsigned)p.H && (unsigned)iw < (unsigned)p.W;
                if (!FASTK) ok = ok && k_cur < p.K;
                const uint32_t off = ok ? a_base[i] + (uint32_t)soff : OOB;
                dma16(xr, sA + (wave + NW * i) * 1024, off);
            }
        }
#pragma unroll
        for (int j = 0; j < NB; ++j)
            dma16(wr, sB + (wave + NW * j) * 1024, b_base[j] + (uint32_t)(kt * BK * 2));
        // advance one K-step
        if (FASTK) {
            c_cur += BK;
            if (c_cur == p.Cin) {
                c_cur = 0;
                if (++s_cur == p.Kw) { s_cur = 0; ++r_cur; }
            }
        } else {
            k_cur += BK;
            c_cur += BK;
            while (c_cur >= p.Cin) {
                c_cur -= p.Cin;
                if (++s_cur == p.Kw) { s_cur = 0; ++r_cur; }
            }
        }
    };

    f32x4_t acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

    auto compute = [&](int buf) {
        const bf16_t* sA = (const bf16_t*)(smem + buf * STAGE);
        const bf16_t* sW = (const bf16_t*)(smem + buf * STAGE + STAGE_A);
        frag af[2][FN], bfr[2][FM];
        auto rd = [&](int kk) {
            const int ch = kk * 4 + (lane >> 4);
#pragma unroll
            for (int i = 0; i < FN; ++i) {
                const int row = wn * TWN + i * 16 + (lane & 15);
                af[kk][i] = *(const frag*)(sW + row * BK + swz(row, ch) * 8);
            }
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int row = wm * TWM + j * 16 + (lane & 15);
                bfr[kk][j] = *(const frag*)(sA + row * BK + swz(row, ch) * 8);
            }
        };
        // pinned order: the first half-step's fragments, then its MFMAs with the second half-step's
        // fragment reads spread between them (left to itself the scheduler issues each read just before
        // its use and waits on it there)
        __builtin_amdgcn_sched_barrier(0);
        rd(0);
        __builtin_amdgcn_sched_barrier(0);
        rd(1);
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(af[0][i], bfr[0][j], acc[i][j]);
        constexpr int R = FN + FM, MF = FN * FM, PER = MF / R > 0 ? MF / R : 1;
#pragma unroll
        for (int q = 0; q < R; ++q) {
            __builtin_amdgcn_sched_group_barrier(0x008, PER, 0);
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        if constexpr (MF > PER * R) __builtin_amdgcn_sched_group_barrier(0x008, MF - PER * R, 0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(af[1][i], bfr[1][j], acc[i][j]);
    };

    constexpr int G = BN / 8;            // 8-channel groups per tile row
    constexpr int RS = NT / G;           // tile rows per pass
    constexpr int ITER = BM / RS;        // passes
    static_assert(NT % G == 0 && BM % RS == 0, "epilogue mapping");
    const int g = tid % G, ml0 = tid / G;
    const int n = n0 + g * 8;
    const bool nv = n < p.Cout;
    // Epilogue mapping (fixed 8-channel group per thread).  The per-channel vectors load now and the
    // residual tile during the last two K-steps, so the epilogue does not wait on them.
    const int nn = nv ? n : 0;
    float bias8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sl8[8], as8[8], ab8[8];
    if (p.bias && !p.bias9) {
        const float4 b0 = *(const float4*)(p.bias + nn), b1 = *(const float4*)(p.bias + nn + 4);
        bias8[0] = b0.x; bias8[1] = b0.y; bias8[2] = b0.z; bias8[3] = b0.w;
        bias8[4] = b1.x; bias8[5] = b1.y; bias8[6] = b1.z; bias8[7] = b1.w;
    }
    if (p.act == 2) {
        const float4 s0 = *(const float4*)(p.slope + nn), s1 = *(const float4*)(p.slope + nn + 4);
        sl8[0] = s0.x; sl8[1] = s0.y; sl8[2] = s0.z; sl8[3] = s0.w;
        sl8[4] = s1.x; sl8[5] = s1.y; sl8[6] = s1.z; sl8[7] = s1.w;
    }
    if (p.y2) {
        const float4 a0 = *(const float4*)(p.aff_s + nn), a1 = *(const float4*)(p.aff_s + nn + 4);
        const float4 c0 = *(const float4*)(p.aff_b + nn), c1 = *(const float4*)(p.aff_b + nn + 4);
        as8[0] = a0.x; as8[1] = a0.y; as8[2] = a0.z; as8[3] = a0.w; as8[4] = a1.x; as8[5] = a1.y; as8[6] = a1.z; as8[7] = a1.w;
        ab8[0] = c0.x; ab8[1] = c0.y; ab8[2] = c0.z; ab8[3] = c0.w; ab8[4] = c1.x; ab8[5] = c1.y; ab8[6] = c1.z; ab8[7] = c1.w;
    }
    uint4 rr[ITER];
    const bool want_res = p.res && !p.partial;
    const bool pre_res = want_res;  // the residual rides behind the last K-steps' DMA
    auto load_res = [&]() {
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const int m = m0 + ml0 + it * RS;
            rr[it] = *(const uint4*)(p.res + (size_t)(m < p.M ? m : 0) * p.Cres + p.res_off + nn);
        }
    };
    if constexpr (STAGES == 2) {
        // DMA for step t+1 overlaps the MFMAs of step t; one vmcnt(0) + barrier per step.
        if (kt0 < kt1) {
            issue(kt0, 0);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        int buf = 0;
        const int kres = max(kt0, kt1 - 2);  // residual loads ride behind this step's DMA
        for (int kt = kt0; kt < kt1; ++kt) {
            if (kt + 1 < kt1) issue(kt + 1, buf ^ 1);
            if (pre_res && kt == kres) load_res();
            compute(buf);
            // next stage landed (this wave's DMA; the younger residual loads may stay in flight), then
            // every wave's; raw barrier: __syncthreads() would also drain the residual loads
            if (pre_res && kt >= kres) wait_vmn<ITER>();
            else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            asm volatile("s_barrier" ::: "memory");
            buf ^= 1;
        }
    } else {
        // 3-stage ring: two K-steps of DMA in flight; at step t wait only for step t's group
        // (vmcnt(NA+NB) leaves step t+1's group outstanding), raw s_barrier (no vmcnt drain), then
        // issue step t+2 into the stage step t-1 used (every wave has passed its MFMAs).
        constexpr int GROUP = NA + NB;
        if (kt0 < kt1) issue(kt0, 0);
        if (kt0 + 1 < kt1) issue(kt0 + 1, 1);
        int buf = 0;
        for (int kt = kt0; kt < kt1; ++kt) {
            if (kt + 1 < kt1) {
                static_assert(GROUP >= 2 && GROUP <= 9 && GROUP != 7, "counted wait for this DMA group size");
                if constexpr (GROUP == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
                else if constexpr (GROUP == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
                else if constexpr (GROUP == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                else if constexpr (GROUP == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
                else if constexpr (GROUP == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
                else if constexpr (GROUP == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
            } else {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            __builtin_amdgcn_s_barrier();
            __builtin_amdgcn_sched_barrier(0);
            if (kt + 2 < kt1) issue(kt + 2, buf == 0 ? 2 : buf - 1);
            compute(buf);
            buf = buf == 2 ? 0 : buf + 1;
        }
        __syncthreads();
    }

    if (want_res && (STAGES != 2 || !pre_res)) load_res();
    // Epilogue: accumulators → LDS f32 tile [BM][EPI_LD] → coalesced 8-channel groups.
    float* sE = (float*)smem;
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int ml = wm * TWM + j * 16 + (lane & 15);
            const int nl = wn * TWN + i * 16 + 4 * (lane >> 4);
            *(f32x4_t*)(sE + ml * EPI_LD + nl) = acc[i][j];
        }
    __syncthreads();
    if (p.partial) {
        // in-launch reduction: the partial slabs go through sc1 (write-through, coherent across XCDs) buffer stores
        // and loads (cdna_hip_programming.md §6 Guideline 16 R1), besides the release / acquire pair below
        const __amdgpu_buffer_rsrc_t pr = __builtin_amdgcn_make_buffer_rsrc(
            (void*)p.partial, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)gridDim.y * p.M * p.Npad * 4), 0x00020000);
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const int ml = ml0 + it * RS, m = m0 + ml;
            if (m >= p.M || !nv) continue;
            const float4 v0 = *(const float4*)(sE + ml * EPI_LD + g * 8);
            const float4 v1 = *(const float4*)(sE + ml * EPI_LD + g * 8 + 4);
            const size_t e = ((size_t)split * p.M + m) * p.Npad + n;
            if (p.splitk_cnt) {
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, v0), pr, (uint32_t)(e * 4), 0, 16);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u32_t, v1), pr, (uint32_t)(e * 4 + 16), 0, 16);
            } else {
                *(float4*)(p.partial + e) = v0;
                *(float4*)(p.partial + e + 4) = v1;
            }
        }
        if (!p.splitk_cnt) return;
        // In-launch split-K reduction (cdna_hip_programming.md §6 Guideline 16, counter hand-off): every slice
        // publishes its partial tile (agent-scope release before the ticket); the slice that draws the last
        // ticket acquires, sums the tile's partials in split order and runs the split-K epilogue's arithmetic
        // (splitk_epilogue_kernel: the same bits), one kernel boundary per split conv fewer.
        wait_vmn<0>();
        __syncthreads();  // every wave's partial stores issued and waited; sE no longer read
        volatile int* flag = (volatile int*)smem;
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            wait_vmn<0>();
            const int t = __hip_atomic_fetch_add(p.splitk_cnt + lid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = t == (int)gridDim.y - 1;
            if (last) {
                __hip_atomic_store(p.splitk_cnt + lid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                wait_vmn<0>();
            }
            *flag = last;
        }
        __syncthreads();
        if (!*flag) return;
        float amax = 0.f;
#pragma unroll
        for (int it = 0; it < ITER; ++it) {
            const int m = m0 + ml0 + it * RS;
            if (m >= p.M || !nv) continue;
            float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
            for (int s2 = 0; s2 < (int)gridDim.y; ++s2) {
                const uint32_t o = (uint32_t)((((size_t)s2 * p.M + m) * p.Npad + n) * 4);
                const float4 a = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(pr, o, 0, 16));
                const float4 b = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(pr, o + 16, 0, 16));
                v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
                v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
            }
            epilogue8<F16>(p, v, m, n);
#pragma unroll
            for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
        }
        if (p.y_amax) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
            if ((tid & 63) == 0)
                atomicMax((unsigned int*)p.y_amax + blockIdx.x % max(p.amax_slots, 1), __float_as_uint(amax));
        }
        return;
    }
    float amax = 0.f;  // max |y| of this thread's stores (fp8 consumers' dynamic activation scale)
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
        const int ml = ml0 + it * RS, m = m0 + ml;
        const float4 v0 = *(const float4*)(sE + ml * EPI_LD + g * 8);
        const float4 v1 = *(const float4*)(sE + ml * EPI_LD + g * 8 + 4);
        float v[8] = {v0.x + bias8[0], v0.y + bias8[1], v0.z + bias8[2], v0.w + bias8[3],
                      v1.x + bias8[4], v1.y + bias8[5], v1.z + bias8[6], v1.w + bias8[7]};
        if (p.bias9) {  // border-class bias (bias8 is zero then)
            const int mm = m < p.M ? m : 0, HoWo = p.Ho * p.Wo, r = mm % HoWo;
            const float* bb = p.bias9 + (size_t)border_class(r / p.Wo, r % p.Wo, p.Ho, p.Wo) * p.Npad + nn;
            const float4 b0 = *(const float4*)bb, b1 = *(const float4*)(bb + 4);
            v[0] += b0.x; v[1] += b0.y; v[2] += b0.z; v[3] += b0.w;
            v[4] += b1.x; v[5] += b1.y; v[6] += b1.z; v[7] += b1.w;
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
            for (int e = 0; e < 8; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * sl8[e];
        }
        if (m < p.M && nv) {
#pragma unroll
            for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
            *(uint4*)(p.y + (size_t)m * p.Cy + p.y_off + n) = F16 && p.y_bf16 ? Num<false>::pack8(v) : T::pack8(v);
            if (p.y2) {
                float u[8];
#pragma unroll
                for (int e = 0; e < 8; ++e) u[e] = v[e] * as8[e] + ab8[e];
                *(uint4*)(p.y2 + (size_t)m * p.Cy2 + p.y2_off + n) = T::pack8(u);
            }
        }
    }
    if (p.y_amax) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
        if ((tid & 63) == 0)
            atomicMax((unsigned int*)p.y_amax + (blockIdx.x + gridDim.x * blockIdx.y) % max(p.amax_slots, 1),
                      __float_as_uint(amax));
    }
}

template <bool F16>
__global__ __launch_bounds__(256) void splitk_epilogue_kernel(ConvArgs p) {
    const int G = p.Cout / 8;
    const size_t total = (size_t)p.M * G;
    float amax = 0.f;  // as the conv epilogue: max |y| for an fp8 consumer's activation scale
    for (size_t it = blockIdx.x * 256ull + threadIdx.x; it < total; it += (size_t)gridDim.x * 256) {
        const int m = (int)(it / G), n = (int)(it - (size_t)m * G) * 8;
        float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int s = 0; s < p.split_k; ++s) {
            const float* src = p.partial + ((size_t)s * p.M + m) * p.Npad + n;
            const float4 a = *(const float4*)src, b = *(const float4*)(src + 4);
            v[0] += a.x; v[1] += a.y; v[2] += a.z; v[3] += a.w;
            v[4] += b.x; v[5] += b.y; v[6] += b.z; v[7] += b.w;
        }
        epilogue8<F16>(p, v, m, n);
#pragma unroll
        for (int e = 0; e < 8; ++e) amax = fmaxf(amax, fabsf(v[e]));
    }
    if (p.y_amax) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) amax = fmaxf(amax, __shfl_xor(amax, o));
        if ((threadIdx.x & 63) == 0)
            atomicMax((unsigned int*)p.y_amax + blockIdx.x % max(p.amax_slots, 1), __float_as_uint(amax));
    }
}

template <bool F16, int BM, int BN, int WM, int WN, int STAGES>
hipError_t launch_variant(const ConvArgs& a, hipStream_t s) {
    if (a.x2 && (a.Cin % 64 != 0 || a.K1 != a.Kh * a.Kw * a.Cin || a.C2 % 64 != 0 || a.K1 + a.C2 > a.Kpad))
        return hipErrorInvalidValue;  // the projection K-steps need the FASTK path
    if (a.y_bf16 && (!a.f16 || a.res || a.y2)) return hipErrorInvalidValue;  // bf16 output of an f16 conv only
    const int tiles_m = (a.M + BM - 1) / BM, tiles_n = (a.Cout + BN - 1) / BN;
    const int nkt = a.Kpad / BK;
    const int split = a.split_k > 1 ? a.split_k : 1;
    const int per = (nkt + split - 1) / split;
    dim3 grid(tiles_m * tiles_n, split);
    dim3 block(64 * WM * WN);
    auto k = a.Cin % 64 == 0 ? conv_igemm_kernel<F16, BM, BN, WM, WN, STAGES, true>
                             : conv_igemm_kernel<F16, BM, BN, WM, WN, STAGES, false>;
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, block, 0, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a, tiles_n, per);
    else
        hipLaunchKernelGGL(k, grid, block, 0, s, a, tiles_n, per);
    return hipGetLastError();
}

template <bool F16>
hipError_t launch_dtype(const ConvArgs& a, hipStream_t s) {
    switch (a.tile) {
        case TILE_256x64: return launch_variant<F16, 256, 64, 4, 1, 2>(a, s);
        case TILE_128x64: return launch_variant<F16, 128, 64, 2, 2, 2>(a, s);
        case TILE_64x128: return launch_variant<F16, 64, 128, 2, 2, 2>(a, s);
        case TILE_128x128_S3: return launch_variant<F16, 128, 128, 2, 2, 3>(a, s);
        case TILE_256x128: return launch_variant<F16, 256, 128, 4, 2, 3>(a, s);
        case TILE_128x256: return launch_variant<F16, 128, 256, 2, 4, 3>(a, s);
        case TILE_128x64_S3: return launch_variant<F16, 128, 64, 2, 2, 3>(a, s);
        case TILE_64x128_S3: return launch_variant<F16, 64, 128, 2, 2, 3>(a, s);
        case TILE_64x64_S3: return launch_variant<F16, 64, 64, 2, 2, 3>(a, s);
        case TILE_64x64: return launch_variant<F16, 64, 64, 2, 2, 2>(a, s);
        case TILE_32x64_S3: return launch_variant<F16, 32, 64, 2, 2, 3>(a, s);
        default: return launch_variant<F16, 128, 128, 2, 2, 2>(a, s);
    }
}

}  // namespace

int conv_tile_bm(int tile) {
    switch (tile) {
        case TILE_256x64: case TILE_256x128: return 256;
        case TILE_64x128: case TILE_64x128_S3: case TILE_64x64_S3: case TILE_64x64: return 64;
        case TILE_32x64_S3: return 32;
        default: return 128;
    }
}
int conv_tile_bn(int tile) {
    switch (tile) {
        case TILE_256x64: case TILE_128x64: case TILE_128x64_S3: case TILE_64x64_S3: case TILE_64x64: case TILE_32x64_S3:
            return 64;
        case TILE_128x256: return 256;
        default: return 128;
    }
}
static int tile_blocks_per_cu(int tile) {
    switch (tile) {
        case TILE_128x128_S3: case TILE_256x128: case TILE_128x256: return 1;
        default: return 2;
    }
}

// Tile + split-K choice: minimise rounds-of-resident-blocks x per-block work / tile efficiency,
// plus a charge for split-K (partials round trip + reduce kernel + prologue/epilogue amortised over
// fewer K-steps).  A forced variant via FR_AB conv_tile=<id> (env) is honoured for experiments.
static int env_tile_id() {
    static const int t = [] { return ab_int("conv_tile", -1); }();
    return t;
}

bool conv_tile_forced() { return env_tile_id() >= 0; }

// Tiles worth timing for a conv with Cout output channels (the autotuner's candidate set).
int conv_tile_candidates(int Cout, int* out) {
    // the 3-stage LDS rings of the small tiles first: the tuner keeps the first of candidates within 1 %, and
    // its repeated launches run with warm caches, where the deeper ring's latency hiding does not show; in the
    // forward (cold operands) the 3-stage tile is the faster one (IRV1 Block17 1x7 / 7x1: 12.0 vs 17.4 us)
    static const int tiles[] = {TILE_128x64_S3, TILE_64x128_S3, TILE_128x128, TILE_256x64, TILE_128x64, TILE_64x128,
                                TILE_256x128, TILE_128x256, TILE_64x64_S3, TILE_64x64, TILE_32x64_S3};
    int n = 0;
    for (int t : tiles) {
        const int BN = conv_tile_bn(t);
        if (BN >= 128 && Cout <= 64) continue;
        if (BN == 256 && Cout <= 128) continue;
        out[n++] = t;
    }
    return n;
}

void conv_plan(int M, int Cout, int Kpad, int* tile, int* split) {
    const int env_tile = env_tile_id();
    static const int tiles[] = {TILE_128x128, TILE_256x64, TILE_128x64, TILE_64x128, TILE_128x128_S3, TILE_256x128,
                                TILE_128x256, TILE_128x64_S3, TILE_64x128_S3};
    // relative MFMA efficiency per tile, calibrated on the IResNet100 bs=256 per-layer sweep
    // (tools/tile_sweep.sh, profiles/r01_tile_sweep.txt); the 3-stage 128x128 ring is the slowest
    // (0 = not in the cost model; the autotuner, tune_conv, still times the 3-stage 128x64 / 64x128
    // tiles: layer1.0's stride-2 transition runs 161 -> 152 us on the 3-stage 128x64)
    static const double eff[] = {1.0, 0.93, 0.92, 0.9, 0.7, 0.9, 0.92, 0.0, 0.0};
    constexpr int NV = sizeof(tiles) / sizeof(tiles[0]);
    const int nkt = Kpad / BK;
    double best = 1e30;
    int bt = TILE_128x128, bs = 1;
    for (int v = 0; v < NV; ++v) {
        if (env_tile >= 0 && tiles[v] != env_tile) continue;
        if (env_tile < 0 && eff[v] == 0.0) continue;
        const int BM = conv_tile_bm(tiles[v]), BN = conv_tile_bn(tiles[v]);
        if (BN >= 128 && Cout <= 64) continue;
        if (BN == 256 && Cout <= 128) continue;
        const long nt = (long)((M + BM - 1) / BM) * ((Cout + BN - 1) / BN);
        const int slots = 256 * tile_blocks_per_cu(tiles[v]);
        for (int sk = 1; sk <= 16; sk *= 2) {
            if (sk > 1 && nkt / sk < 8) break;
            const long blocks = nt * sk;
            const double rounds = (double)((blocks + slots - 1) / slots);
            const double ksteps = (double)((nkt + sk - 1) / sk) + 6.0;  // + prologue/epilogue ~ 6 K-steps
            const double per_block = (double)BM * BN * ksteps / (eff[v] > 0.0 ? eff[v] : 1.0) / (512.0 / slots);
            const double cost = rounds * per_block + (sk > 1 ? 0.25 * (double)M * Cout * sk / 2048.0 : 0.0);
            if (cost < best * 0.999) { best = cost; bt = tiles[v]; bs = sk; }
        }
    }
    *tile = bt;
    *split = bs;
}

// The embedding head (M = batch, N = 512, K = 25,088 at 7x7x512): a few output tiles over a very long K, so
// split-K wide enough to give every CU a block (conv_plan stopped at 16 splits of the 2-stage tile: 256 blocks
// of 24 K-steps at bs = 256, 43 us); splits that divide the K-steps evenly, >= 4 K-steps each.  FR_AB head_plan=tile:split
// overrides (experiments).
void head_plan(int M, int Cout, int Kpad, int* tile, int* split) {
    struct EnvPlan { int tile = -1, split = -1; };
    static const EnvPlan env = [] {
        EnvPlan e;
        const char* v = ab_str("head_plan");  // "tile:split"
        int t = -1, sp = -1;
        if (v && sscanf(v, "%d:%d", &t, &sp) == 2 && t >= 0 && sp >= 1) { e.tile = t; e.split = sp; }
        return e;
    }();
    if (env.tile >= 0) {
        *tile = env.tile;
        *split = env.split;
        return;
    }
    // 3-stage 128x64 tiles, at most one block per CU (tools/head_sweep.sh at bs = 256: 14 splits 28.8 us,
    // the 2-stage tile with 28 splits 31.3 us, 56 splits 37 us)
    const int nkt = Kpad / BK;
    const long tiles = (long)((M + 127) / 128) * ((Cout + 63) / 64);
    int best = 1;
    for (int sp = 1; sp <= nkt / 4; ++sp) {
        if (nkt % sp) continue;
        if (tiles * sp > 256) break;
        best = sp;
    }
    if (best == 1) {  // no even split: fall back to the generic plan
        conv_plan(M, Cout, Kpad, tile, split);
        return;
    }
    *tile = TILE_128x64_S3;
    *split = best;
}

hipError_t launch_conv(const ConvArgs& a, hipStream_t s) {
    if (a.tile == TILE_WRING) {  // conv_wring.hip (an autotuner pick)
        ConvArgs w = a;
        w.wimg = a.wring_;
        return launch_conv_wring(w, s);
    }
    if (a.tile == TILE_DIRECT) return launch_conv_direct(a, 0, s);  // conv_direct.hip (an autotuner pick)
    return a.f16 ? launch_dtype<true>(a, s) : launch_dtype<false>(a, s);
}

hipError_t launch_splitk_epilogue(const ConvArgs& a, hipStream_t s) {
    const size_t total = (size_t)a.M * (a.Cout / 8);
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    if (a.f16)
        hipLaunchKernelGGL(splitk_epilogue_kernel<true>, dim3(blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(splitk_epilogue_kernel<false>, dim3(blocks), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace fr
