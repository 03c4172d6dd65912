// LDS-resident Inception-ResNet blocks (CDNA4 / gfx950): FaceNet IRV1's Block35 (17x17), Block17 (8x8) and
// Block8 (3x3) as one launch each (reference: facenet_model.py:28-36 -> facenet-pytorch InceptionResnetV1).
// Per conv the per-conv path writes the branch tensors to HBM and reads them back, and the 32-128-channel
// branch convs are small GEMMs that leave most of the chip idle (profiles/r03_final_irv1_layer_profile.txt:
// Block35 75 us, Block17 65 us, 11-18 % of the bf16 peak).  Here one workgroup owns G images (G = 1 for
// Block35 / Block17) and runs the block's convs as a short program: the block input is read from global
// memory, every branch intermediate (the concatenation and the second-stage tensors) stays in LDS, and only
// the block output goes back to HBM.  The weights stream from L2 (one XCD's 32 CUs share them).
//
// A conv is an implicit GEMM over the workgroup's pixels: 8 waves take units of MF pixel fragments x NF
// 16-channel fragments; per 32-deep K-step a unit loads MF activation fragments (ds_read_b128 from LDS, or a
// buffer load from the block input) and NF weight fragments (buffer loads, D steps ahead) and issues MF*NF
// v_mfma_f32_16x16x32.  Convs of one program step are independent (Block35's two 3x3 branches) and share the
// waves; a barrier separates the steps.  LDS rows are the workgroup's pixels, ld % 32 == 16 elements so the 16
// consecutive pixels of a fragment hit 16 distinct 16-byte bank groups; out-of-image taps read a zeroed
// 64-byte area.  Per output the MFMA chain runs over k in order and the epilogue is conv_igemm's (acc + bias,
// + residual, activation), so every conv equals conv_igemm tile 0 bit for bit (the padded K-steps beyond
// K, which add 0 * 0, are skipped).
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int WAVES = 8;
constexpr uint32_t OOB = 0x80000000u;

typedef __attribute__((address_space(3))) char lds_char;

typedef unsigned int u32x4_v __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2_v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ u32x4_v lds_read16(const lds_char* lds, uint32_t byte) {
    return *(const __attribute__((address_space(3))) u32x4_v*)(lds + byte);
}

template <bool F16, int MF, int NF, bool GSRC>
__device__ __forceinline__ void block_unit(const BlockArgs& p, const BlockConv& c, int mu, int nu, lds_char* lds,
                                           uint32_t zoff, uint32_t ptab, int lane, int npx, int img0) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    const int g = lane >> 4;
    const int HW = p.H * p.W;
    const int K = c.kh * c.kw * c.Cin;
    const int nks = (K + 31) / 32;
    const int n0 = nu * NF * 16;
    const int ld = GSRC ? p.Cx : p.ld;
    // per pixel fragment: the lane's pixel byte offset (channel 8 g) and a mask of the taps that land inside its
    // image (0 for a pixel past the workgroup's last), so a K-step costs the step table's scalar tap offset plus
    // a bit test per fragment.  The pixel's (row, column) comes from the workgroup's LDS table.
    uint32_t base[MF], vmask[MF];
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        const int q = 16 * (mu * MF + i) + (lane & 15);
        const bool pv = q < npx;
        const int qq = pv ? q : 0;
        const uint32_t pc = *(const __attribute__((address_space(3))) uint32_t*)(lds + ptab + 4 * qq);
        const int oh = pc & 0xffff, ow = pc >> 16;
        base[i] = (uint32_t)((qq * ld + c.src_off + 8 * g) * 2);
        // taps (tr, tc) inside the image: tr in [r0, r1], tc in [c0, c1]
        const int r0 = max(0, c.ph - oh), r1 = min(c.kh - 1, p.H - 1 + c.ph - oh);
        const int c0 = max(0, c.pw - ow), c1 = min(c.kw - 1, p.W - 1 + c.pw - ow);
        const uint32_t cols = c1 >= c0 ? (2u << c1) - (1u << c0) : 0u;
        uint32_t m = 0;
        for (int tr = 0; tr < c.kh; ++tr) m |= (tr >= r0 && tr <= r1) ? cols << (tr * c.kw) : 0u;
        vmask[i] = pv ? m : 0u;
    }
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)c.w, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)c.Npad * c.Kpad * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.x + (size_t)img0 * HW * p.Cx), 0, (uint32_t)min((size_t)0x7fffffff, (size_t)npx * p.Cx * 2),
        0x00020000);
    const uint32_t wbase = (uint32_t)(((n0 + (lane & 15)) * c.Kpad + 8 * g) * 2);
    const uint32_t zaddr = zoff + 16u * g;

    // Operand ring of D K-steps.  The steady-state loop issues the loads of step s + D right after the MFMAs of
    // step s, unconditionally (steps past the end read zeros: an out-of-range buffer offset / the LDS zero
    // area), so the loop body has no branch and the compiler waits for exactly the loads each step consumes.
    constexpr int D = MF * NF <= 8 ? 4 : 2;
    frag wa[D][NF], xb[D][MF];
    auto load_step = [&](int s, int slot) {
        const bool live = s < nks;
        const int2 st = c.steps[s];  // {tap offset, tap} (tap 31 past the end: no mask bit), wave-uniform
        const uint32_t toff = (uint32_t)__builtin_amdgcn_readfirstlane(st.x);
        const uint32_t bit = 1u << __builtin_amdgcn_readfirstlane(st.y);
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const bool ok = (vmask[i] & bit) != 0u;
            if (GSRC) {
                const uint32_t off = ok ? base[i] + toff : OOB;
                xb[slot][i] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
            } else {
                const uint32_t off = ok ? base[i] + toff : zaddr;
                xb[slot][i] = __builtin_bit_cast(frag, lds_read16(lds, off));
            }
        }
        const uint32_t so = live ? (uint32_t)(s * 64) : OOB;
#pragma unroll
        for (int j = 0; j < NF; ++j)
            wa[slot][j] = __builtin_bit_cast(
                frag, __builtin_amdgcn_raw_buffer_load_b128(wr, wbase + (uint32_t)(j * 16 * c.Kpad * 2), so, 0));
    };
    f32x4_t acc[MF][NF];
#pragma unroll
    for (int i = 0; i < MF; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    auto mfmas = [&](int q) {
#pragma unroll
        for (int i = 0; i < MF; ++i)
#pragma unroll
            for (int j = 0; j < NF; ++j) acc[i][j] = T::mfma(wa[q][j], xb[q][i], acc[i][j]);
    };
    // the epilogue's global operands (bias, residual), loaded before the K loop: issued after the block's output
    // stores they could alias, each would be a full memory round trip per fragment
    float4 bz[NF];
    uint2 rz[MF][NF];
#pragma unroll
    for (int j = 0; j < NF; ++j) {
        const int n = n0 + 16 * j + 4 * g;
        bz[j] = c.bias ? *(const float4*)(c.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (c.res) {
#pragma unroll
        for (int i = 0; i < MF; ++i) {
            const int q = 16 * (mu * MF + i) + (lane & 15);
#pragma unroll
            for (int j = 0; j < NF; ++j)
                rz[i][j] = q < npx ? *(const uint2*)(p.x + ((size_t)img0 * HW + q) * p.Cx + c.res_off + n0 + 16 * j + 4 * g)
                                   : make_uint2(0u, 0u);
        }
    }
#pragma unroll
    for (int q = 0; q < D; ++q) load_step(q, q);
    int s0 = 0;
    for (; s0 + D <= nks; s0 += D) {
#pragma unroll
        for (int q = 0; q < D; ++q) {
            mfmas(q);
            load_step(s0 + q + D, q);
        }
    }
#pragma unroll
    for (int q = 0; q < D - 1; ++q)
        if (s0 + q < nks) mfmas(q);
    // epilogue (conv_igemm's arithmetic): lane holds channels n .. n + 3 of fragment j for pixel q of fragment i
#pragma unroll
    for (int i = 0; i < MF; ++i) {
        const int q = 16 * (mu * MF + i) + (lane & 15);
        if (q >= npx) continue;
#pragma unroll
        for (int j = 0; j < NF; ++j) {
            const int n = n0 + 16 * j + 4 * g;
            float v[4] = {acc[i][j][0] + bz[j].x, acc[i][j][1] + bz[j].y, acc[i][j][2] + bz[j].z, acc[i][j][3] + bz[j].w};
            if (c.res) {
                float f[8];
                T::unpack8(make_uint4(rz[i][j].x, rz[i][j].y, 0u, 0u), f);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] += f[e];
            }
            if (c.act == 1) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
            } else if (c.act == 2) {
#pragma unroll
                for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : v[e] * c.slope[n + e];
            }
            float o8[8] = {v[0], v[1], v[2], v[3], 0.f, 0.f, 0.f, 0.f};
            const uint4 pk = T::pack8(o8);
            if (c.dst_lds)
                *(__attribute__((address_space(3))) u32x2_v*)(lds + (q * p.ld + c.dst_off + n) * 2) = (u32x2_v){pk.x, pk.y};
            else
                *(uint2*)(p.y + ((size_t)img0 * HW + q) * p.Cy + c.dst_off + n) = make_uint2(pk.x, pk.y);
        }
    }
}

template <bool F16, bool GSRC>
__device__ __forceinline__ void block_unit_shape(const BlockArgs& p, const BlockConv& c, int mu, int nu, lds_char* lds,
                                                 uint32_t zoff, uint32_t ptab, int lane, int npx, int img0) {
    switch (c.mf * 8 + c.nf) {
        case 8 + 1: block_unit<F16, 1, 1, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
        case 8 + 2: block_unit<F16, 1, 2, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
        case 8 + 4: block_unit<F16, 1, 4, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
        case 16 + 1: block_unit<F16, 2, 1, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
        case 16 + 2: block_unit<F16, 2, 2, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
        case 16 + 4: block_unit<F16, 2, 4, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
        case 32 + 1: block_unit<F16, 4, 1, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
        case 32 + 2: block_unit<F16, 4, 2, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
        default: block_unit<F16, 4, 4, GSRC>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0); break;
    }
}

template <bool F16>
__global__ __launch_bounds__(WAVES * 64) void block_kernel(BlockArgs p) {
    extern __shared__ __attribute__((aligned(16))) char lds_generic[];
    lds_char* lds = (lds_char*)lds_generic;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int img0 = blockIdx.x * p.G;
    const int G = min(p.G, p.B - img0);
    const int npx = G * p.H * p.W, n_mf = (npx + 15) / 16;
    const uint32_t zoff = (uint32_t)npx * p.ld * 2;  // 64 zero bytes after the pixel rows
    if (threadIdx.x < 16) *(__attribute__((address_space(3))) uint32_t*)(lds + zoff + 4 * threadIdx.x) = 0u;
    const uint32_t ptab = zoff + 64;  // per pixel: row | column << 16
    for (int q = threadIdx.x; q < npx; q += WAVES * 64) {
        const int r = q % (p.H * p.W), oh = r / p.W;
        *(__attribute__((address_space(3))) uint32_t*)(lds + ptab + 4 * q) = (uint32_t)oh | (uint32_t)(r - oh * p.W) << 16;
    }
    __syncthreads();
    for (int st = 0; st < p.nstep; ++st) {
        int base = 0;  // the step's units, numbered across its convs; unit u goes to wave u % WAVES
        for (int ci = 0; ci < p.nconv; ++ci) {
            const BlockConv& c = p.c[ci];
            if (c.step != st) continue;
            const int mus = (n_mf + c.mf - 1) / c.mf, nus = c.Cout / (16 * c.nf), n = mus * nus;
            for (int u = (wave - base % WAVES + WAVES) % WAVES; u < n; u += WAVES) {
                const int mu = u % mus, nu = u / mus;
                if (c.src_lds)
                    block_unit_shape<F16, false>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0);
                else
                    block_unit_shape<F16, true>(p, c, mu, nu, lds, zoff, ptab, lane, npx, img0);
            }
            base += n;
        }
        __syncthreads();
    }
}

}  // namespace

size_t block_lds_bytes(int G, int H, int W, int ld) { return (size_t)G * H * W * (ld * 2 + 4) + 64; }

bool block_supported(const BlockArgs& a) {
    if (a.nconv < 1 || a.nconv > FR_BLOCK_MAX_CONVS || a.nstep < 1 || a.G < 1 || a.B < 1 || a.ld % 32 != 16 ||
        a.Cx % 4 != 0 || a.Cy % 4 != 0 || block_lds_bytes(a.G, a.H, a.W, a.ld) > 160 * 1024)
        return false;
    // 31-bit buffer records / offsets: past 2 GiB an operand would read zeros, silently
    if ((size_t)a.B * a.H * a.W * a.Cx * 2 > 0x7fffffffull || (size_t)a.B * a.H * a.W * a.Cy * 2 > 0x7fffffffull) return false;
    for (int i = 0; i < a.nconv; ++i) {
        const BlockConv& c = a.c[i];
        const int nfr = c.Cout / 16;
        if (c.Cin % 32 != 0 || c.Cout % 16 != 0 || c.kh * c.kw > 31 || c.Kpad % 32 != 0 || c.Kpad < c.kh * c.kw * c.Cin ||
            c.Npad < c.Cout || !c.steps || c.step < 0 || c.step >= a.nstep || (c.mf != 1 && c.mf != 2 && c.mf != 4) ||
            (c.nf != 1 && c.nf != 2 && c.nf != 4) || nfr % c.nf != 0 || c.src_off % 8 != 0 || c.dst_off % 4 != 0 ||
            (c.act == 2 && !c.slope) || c.act < 0 || c.act > 2)
            return false;
        if (c.src_lds ? c.src_off + c.Cin > a.ld : c.src_off + c.Cin > a.Cx) return false;
        if (c.dst_lds ? c.dst_off + c.Cout > a.ld : c.dst_off + c.Cout > a.Cy) return false;
        if (c.res && (c.res_off % 4 != 0 || c.res_off + c.Cout > a.Cx)) return false;
    }
    return true;
}

hipError_t launch_block(const BlockArgs& a, hipStream_t s) {
    if (!block_supported(a)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((a.B + a.G - 1) / a.G));
    const size_t lds = block_lds_bytes(a.G, a.H, a.W, a.ld);
    auto k = a.f16 ? block_kernel<true> : block_kernel<false>;
    static bool attr[2] = {false, false};
    if (!attr[a.f16 ? 1 : 0]) {
        hipError_t e = hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        if (e != hipSuccess) return e;
        attr[a.f16 ? 1 : 0] = true;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, dim3(WAVES * 64), lds, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, grid, dim3(WAVES * 64), lds, s, a);
    return hipGetLastError();
}

}  // namespace fr
