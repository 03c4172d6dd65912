// Row-band direct 3x3 convolution (stride 1, pad 1) for the 28x28x128 IBasicBlock convs of IResNet100
// layer2 (layer2.1 .. layer2.12: 24 convs, 22.9 % of the network's FLOPs).
//
// As an implicit GEMM these convs re-gather every input pixel for all 9 taps (9x the activation bytes
// L2 -> LDS: at the MFMA rate ~99 GB/s per CU, above the ~70 GB/s an LDS-DMA gather sustains per CU,
// MI355X_MICROARCH.md "Indexed rows").  Here a workgroup owns a quarter image (7 output rows x 28) x
// all 128 output channels, two workgroups per CU (4B workgroups = 4 per CU at bs = 256, so one
// workgroup's epilogue overlaps the other's main loop):
//   * per 32-input-channel chunk the 9 x 30 zero-haloed patch is DMA'd into LDS once ([4 planes of 8
//     channels][9 rows][32 positions][16 B]) and read by all 9 taps at shifted positions; the next
//     chunk's patch (double buffer) streams in during the current chunk's 9 K-steps;
//   * per K-step (chunk, tap) the [128 out][32 in] weight slice (8 KiB), pre-packed at load time in
//     its LDS image (img_pack_weights: 1-KiB contiguous DMA pieces), streams into a 3-slot ring, three steps
//     ahead; one mid-step s_barrier per K-step (the stage kernel's schedule, conv_stage.hip);
//   * 2x2 waves: wave (wm, wn) computes 7 virtual-pixel frags (rows 0..6 x 32 columns, 28 valid) x
//     64 output channels (4 n-frags): 28 v_mfma_f32_16x16x32_bf16 per K-step, 112 f32 accumulators;
//   * operand A = weight rows, operand B = patch positions, so a lane ends with 4 consecutive channels
//     of one pixel; the epilogue (bias or border-class bias9, residual, ReLU/PReLU) stores 8 B per lane.
#include "kernels.h"

#include <hip/hip_ext.h>

#include <cstdlib>

namespace fr {
namespace {


// Geometry of one instance: IW x IW images with IC input = output channels; a workgroup owns QR output
// rows x all IC channels, laid out as QR rows x PCOL virtual columns (IW valid + pad) = 16-pixel frags;
// 4 waves = PG pixel groups x (4 / PG) channel groups.
template <int IW_, int IC_, int QR_, int PCOL_, int PG_>
struct ImgGeo {
    static constexpr int IW = IW_, IC = IC_, QR = QR_, PC = PCOL_, PG = PG_, CG = 4 / PG_;
    static constexpr int PPOS = (QR + 2) * PC;                      // positions per plane (halo rows)
    static constexpr int PLANE_B = PPOS * 16;                       // a multiple of 256 B
    static constexpr int PATCH_PIECES = (4 * PLANE_B / 1024 + 3) / 4 * 4;  // 1-KiB pieces, 4 | count
    static constexpr int PATCH_B = PATCH_PIECES * 1024;
    static constexpr int SLICE_B = 4 * IC * 16;                     // [4 groups of 8 ch][IC rows][16 B]
    static constexpr int WP = SLICE_B / 1024 / 4;                   // weight pieces per wave per step
    static constexpr int PP = PATCH_PIECES / 4;                     // patch pieces per wave per chunk
    static constexpr int NSLOT = 3;
    static constexpr int LDS = 2 * PATCH_B + NSLOT * SLICE_B;
    static constexpr int NCH = IC / 32;
    static constexpr int NSTEP = NCH * 9;
    static constexpr int FM = QR * PC / 16 / PG;                    // pixel frags per wave
    static constexpr int FN = IC / 16 / CG;                         // channel frags per wave
    static constexpr int BANDS = IW / QR;                           // workgroups per image
    static_assert(PLANE_B % 256 == 0 && IW % QR == 0 && PC % 16 == 0 && PC >= IW + 2 && FN % 2 == 0, "geometry");
};
typedef ImgGeo<28, 128, 7, 32, 2> Geo28;  // layer2: 2 x 2 waves of 7 frags x 64 channels, 64 KiB LDS
typedef ImgGeo<56, 64, 4, 64, 4> Geo56;   // layer1: 4 waves of 4 frags (one virtual row) x 64 channels

constexpr uint32_t OOB = 0x80000000u;
typedef __attribute__((address_space(3))) void lds_void;

// LDS-DMA of 16 B per lane; soff: a wave-uniform byte offset (memory address only)
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t rsrc, const char* lds, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds, 16, voff, soff, 0, 0);
}

// mid-step wait: vmcnt(N); LDS ops older than the step's L youngest (its next-step patch reads, which
// no DMA of this step touches) complete -- the weight refills of the slot about to be overwritten and
// the staged patch writes that the next barrier publishes
template <int N, int L>
__device__ __forceinline__ void wait_vm_barrier() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(%1)\n\ts_barrier" ::"n"(N), "n"(L) : "memory");
}

// RES: residual input (IBasicBlock conv2); B9: border-class bias table (conv1 with bn1 folded).  The
// epilogue is specialised on them so its loads issue together instead of behind per-pixel branches.
template <bool F16, bool RES, bool B9, typename G>
__global__ __launch_bounds__(256, 2) void conv_img_kernel(ConvArgs p) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    constexpr int IW = G::IW, IC = G::IC, PC = G::PC, FM = G::FM, FN = G::FN, NCH = G::NCH, NSTEP = G::NSTEP;
    constexpr int NSLOT = G::NSLOT, PATCH_B = G::PATCH_B, SLICE_B = G::SLICE_B, PLANE_B = G::PLANE_B;
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [patch 0][patch 1][slot 0..2]
    char* const slots = smem + 2 * PATCH_B;

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int wm = wave % G::PG, wn = wave / G::PG;  // pixel frags FM*wm.., output channels 16*FN*wn..
    const int b = blockIdx.x / G::BANDS, r0 = G::QR * (blockIdx.x % G::BANDS);

    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * IW * IW * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t wr =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.wimg, 0, (uint32_t)(NSTEP * SLICE_B), 0x00020000);

    // patch of chunk cc (input channels 32cc..): PP pieces per wave, plane-major [4 planes][QR+2 rows]
    // [PC positions][16 B]; halo, pad and spare pieces read out of range (zeros).  Offsets recomputed
    // per chunk (no live registers); the chunk's channel offset in the scalar offset.
    auto issue_patch = [&](int cc, int buf) {
        int ln = lane;
        asm volatile("" : "+v"(ln));  // opaque copy: the offsets are not hoisted (registers for the MFMAs)
#pragma unroll
        for (int u = 0; u < G::PP; ++u) {
            const int piece = 4 * u + wave, sl = piece * 64 + ln;
            const int plane = sl / G::PPOS, pos = sl % G::PPOS, pr = pos / PC, pc = pos % PC;
            const int ir = r0 - 1 + pr, ic = pc - 1;
            const bool in = plane < 4 && (unsigned)ir < (unsigned)IW && (unsigned)ic < (unsigned)IW;
            const uint32_t off =
                in ? (uint32_t)((((size_t)b * IW * IW + ir * IW + ic) * p.Cx + p.x_off + plane * 8) * 2) : OOB;
            dma16s(xr, smem + buf * PATCH_B + piece * 1024, off, (uint32_t)(cc * 32 * 2));
        }
    };
    // chunks >= 1 go through registers instead: 4 consecutive lanes load one pixel's 64 contiguous bytes
    // (16 segments per wave-load instead of the DMA's 64 scattered 16-B pieces), loaded at the chunk
    // start and written plane-major into the free patch buffer three K-steps later
    typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_t;
    constexpr int PH = (G::PP + 1) / 2;  // pieces per phase (two phases: register budget)
    u32x4_t pst[PH];
    auto load_patch = [&](int cc, int ph) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int uu = 0; uu < PH; ++uu) {
            const int u = PH * ph + uu;
            if (u >= G::PP) break;
            const int sl = (4 * u + wave) * 64 + ln, pos = sl >> 2, plane = sl & 3, pr = pos / PC, pc = pos % PC;
            const int ir = r0 - 1 + pr, ic = pc - 1;
            const bool in = pos < G::PPOS && (unsigned)ir < (unsigned)IW && (unsigned)ic < (unsigned)IW;
            const uint32_t off =
                in ? (uint32_t)((((size_t)b * IW * IW + ir * IW + ic) * p.Cx + p.x_off + plane * 8) * 2) : OOB;
            pst[uu] = __builtin_amdgcn_raw_buffer_load_b128(xr, off, cc * 32 * 2, 0);
        }
    };
    auto store_patch = [&](int buf, int ph) {
        int ln = lane;
        asm volatile("" : "+v"(ln));
#pragma unroll
        for (int uu = 0; uu < PH; ++uu) {
            const int u = PH * ph + uu;
            if (u >= G::PP) break;
            const int sl = (4 * u + wave) * 64 + ln, pos = sl >> 2, plane = sl & 3;
            if (pos < G::PPOS) *(u32x4_t*)(smem + buf * PATCH_B + plane * PLANE_B + pos * 16) = pst[uu];
        }
    };
    // weight slice of K-step s: pre-packed in the LDS image [g][n][16 B] (img_pack_weights), so each
    // of the WP pieces per wave is 1 KiB contiguous; the step in soffset
    auto issue_w = [&](int s, int slot) {
#pragma unroll
        for (int u = 0; u < G::WP; ++u) {
            const int piece = G::WP * wave + u;
            dma16s(wr, slots + slot * SLICE_B + piece * 1024, (uint32_t)(piece * 1024 + lane * 16), (uint32_t)(s * SLICE_B));
        }
    };

    // fragment addresses: B (patch) virtual frag f = FM*wm + j -> positions 16f + (lane&15) (linear:
    // one base + compile-time offsets), plane (lane>>4); A (weights) rows 16*FN*wn + 16i + (lane&15),
    // group (lane>>4)
    const int pbase = (lane >> 4) * PLANE_B + (16 * FM * wm + (lane & 15)) * 16;
    const int woff = (lane >> 4) * (IC * 16) + (16 * FN * wn + (lane & 15)) * 16;

    // accumulator seeds, loaded while the prologue DMA is in flight: the bias (B9: of the output pixel's
    // border class) plus (RES) the residual, so the epilogue only applies the activation and stores.
    // Pad columns read a valid pixel (their results are never stored).
    const size_t img = (size_t)b * IW * IW;
    f32x4_t acc[FN][FM];
    {
        int ln = lane;
        asm volatile("" : "+v"(ln));  // opaque copy: the seed addresses are not kept live in the loop
#pragma unroll
        for (int i = 0; i < FN; ++i) {
            const int n = 16 * FN * wn + 16 * i + 4 * (ln >> 4);
            float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
            if (!B9 && p.bias) bb = *(const float4*)(p.bias + n);
#pragma unroll
            for (int j = 0; j < FM; ++j) {
                const int f = FM * wm + j, v = 16 * f + (ln & 15), c = v % PC, r = r0 + v / PC;
                const int cc = c < IW ? c : 0;
                float4 s = bb;
                if (B9) s = *(const float4*)(p.bias9 + border_class(r, c, IW, IW) * p.Npad + n);
                if (RES) {
                    const uint2 rr = *(const uint2*)(p.res + (img + r * IW + cc) * p.Cres + p.res_off + n);
                    float f8[8];
                    T::unpack8(make_uint4(rr.x, rr.y, 0, 0), f8);
                    s.x += f8[0]; s.y += f8[1]; s.z += f8[2]; s.w += f8[3];
                }
                acc[i][j] = (f32x4_t){s.x, s.y, s.z, s.w};
            }
        }
    }
    frag wf[FN], pA[FM], pB[FM];
    auto pread = [&](frag (&pf)[FM], int buf, int tap) {
        const int dh = tap / 3, dw = tap % 3;
        const char* a = smem + buf * PATCH_B + pbase + (dh * PC + dw) * 16;
#pragma unroll
        for (int j = 0; j < FM; ++j) pf[j] = *(const frag*)(a + j * 256);
    };
    auto wread = [&](int i, int slot) { wf[i] = *(const frag*)(slots + slot * SLICE_B + woff + i * 256); };

    // prologue: chunk 0's patch and the first three weight slices
    issue_patch(0, 0);
    issue_w(0, 0);
    issue_w(1, 1);
    issue_w(2, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    pread(pA, 0, 0);
#pragma unroll
    for (int i = 0; i < FN; ++i) wread(i, 0);

    // one K-step s (slot s % 3, chunk c = s / 9, tap t = s % 9): nxt <- patch fragments of step s+1;
    // MFMAs of the first half of the weight frags; mid-step barrier: this wave's slice s+1 landed
    // (younger: slice s+2 and the patch loads of steps s-2, s-1), every wave is
    // past its reads of slot s % 3 and of the previous chunk's patch buffer; DMA of slice s+3 into slot
    // s % 3; at t == 0 the next chunk's patch loads into registers, at t == 3 it is written to the other
    // buffer; wf <- slice s+1 (first half now, second half in place after their MFMAs).  The next
    // chunk's patch is read at the start of its t == 8 step: the t == 7 barrier covered it.
    auto kstep = [&](int s, frag (&cur)[FM], frag (&nxt)[FM]) {
        const int t = s % 9, c = s / 9, slot = s % NSLOT, nslot = (s + 1) % NSLOT;
        // compiler fence: the previous step's refills and staged patch writes stay ahead of this
        // step's reads, so "all but the FM youngest LDS ops" below means exactly those
        asm volatile("" ::: "memory");
        if (s + 1 < NSTEP) pread(nxt, t == 8 ? (c + 1) & 1 : c & 1, t == 8 ? 0 : t + 1);
#pragma unroll
        for (int i = 0; i < FN / 2; ++i)
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(wf[i], cur[j], acc[i][j]);
        // younger than slice s+1 (issued at step s-2): slice s+2 and the patch loads of steps s-2, s-1
        if (t == 1 || t == 2) wait_vm_barrier<G::WP + PH, FM>();
        else if (t == 4 || t == 5) wait_vm_barrier<G::WP + (G::PP - PH), FM>();
        else if (t == 7) wait_vm_barrier<G::WP, 0>();  // publishes the staged patch (read from t == 8)
        else wait_vm_barrier<G::WP, FM>();
        issue_w(s + 3 < NSTEP ? s + 3 : NSTEP - 1, slot);  // tail: harmless re-fetch (uniform counts)
        // next chunk's patch in two register phases: load at t == 0 / 3, store at t == 3 / 6 (the loads
        // have landed by then: they precede the slices waited for), read from t == 8 on
        const int cn = c + 1 < NCH ? c + 1 : NCH - 1;
        if (t == 3 || t == 6) store_patch((c + 1) & 1, t == 3 ? 0 : 1);
        if (t == 0 || t == 3) load_patch(cn, t == 0 ? 0 : 1);
#pragma unroll
        for (int i = 0; i < FN / 2; ++i) wread(i, nslot);
#pragma unroll
        for (int i = FN / 2; i < FN; ++i) {
#pragma unroll
            for (int j = 0; j < FM; ++j) acc[i][j] = T::mfma(wf[i], cur[j], acc[i][j]);
            wread(i, nslot);
        }
    };
#pragma unroll
    for (int s = 0; s < NSTEP; s += 2) {
        kstep(s, pA, pB);
        kstep(s + 1, pB, pA);
    }

    // ---- epilogue: straight from the accumulators (no LDS), 8 B per lane and (i, j).  Bias and
    // residual are already in the accumulators; the activation is v > 0 ? v : v * negf (negf = PReLU
    // slope, 0 for ReLU, 1 for none: one branch-free form, its 4 loads issued together).
    int ln = lane;
    asm volatile("" : "+v"(ln));  // opaque copy: keeps the per-(i, j) addresses from being hoisted
    float4 nf[FN];
#pragma unroll
    for (int i = 0; i < FN; ++i) nf[i] = *(const float4*)(p.negf + 16 * FN * wn + 16 * i + 4 * (ln >> 4));
#pragma unroll
    for (int i = 0; i < FN; ++i) {
        const int n = 16 * FN * wn + 16 * i + 4 * (ln >> 4);
#pragma unroll
        for (int j = 0; j < FM; ++j) {
            const int f = FM * wm + j, v = 16 * f + (ln & 15), c = v % PC, r = r0 + v / PC;
            float o[4] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]};
            o[0] = fmaf(nf[i].x, fminf(o[0], 0.f), fmaxf(o[0], 0.f));
            o[1] = fmaf(nf[i].y, fminf(o[1], 0.f), fmaxf(o[1], 0.f));
            o[2] = fmaf(nf[i].z, fminf(o[2], 0.f), fmaxf(o[2], 0.f));
            o[3] = fmaf(nf[i].w, fminf(o[3], 0.f), fmaxf(o[3], 0.f));
            float o8[8] = {o[0], o[1], o[2], o[3], 0, 0, 0, 0};
            const uint4 pk = T::pack8(o8);
            if (c < IW) *(uint2*)(p.y + (img + r * IW + c) * p.Cy + p.y_off + n) = make_uint2(pk.x, pk.y);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail DMAs land before the LDS is released
}

template <typename G>
bool img_supported_t(const ConvArgs& a) {
    constexpr int IW = G::IW, IC = G::IC;
    return a.wimg && !a.x2 && a.Kh == 3 && a.Kw == 3 && a.sh == 1 && a.sw == 1 && a.ph == 1 && a.pw == 1 && a.H == IW && a.W == IW &&
           a.Ho == IW && a.Wo == IW && a.Cin == IC && a.Cout == IC && a.Npad >= IC && a.Kpad >= 9 * IC &&
           a.Cx % 8 == 0 && a.x_off % 8 == 0 && a.x_off + IC <= a.Cx && a.Cy % 4 == 0 && a.y_off % 4 == 0 &&
           a.y_off + IC <= a.Cy && !a.y2 && !a.partial && !a.w8 && !a.y_amax && a.B > 0 && !a.f16 &&
           !(a.res && a.bias9) && (!a.res || (a.Cres % 4 == 0 && a.res_off % 4 == 0 && a.res_off + IC <= a.Cres)) &&
           a.negf;
}

template <typename G>
hipError_t launch_img_t(const ConvArgs& a, hipStream_t s) {
    auto k = a.res ? conv_img_kernel<false, true, false, G>
                   : (a.bias9 ? conv_img_kernel<false, false, true, G> : conv_img_kernel<false, false, false, G>);
    const int v = a.res ? 0 : (a.bias9 ? 1 : 2);
    static bool attr[3] = {false, false, false};
    if (!attr[v]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, G::LDS);
        attr[v] = true;
    }
    const dim3 grid(G::BANDS * a.B);
    if (a.ev0)
        hipExtLaunchKernelGGL(k, grid, dim3(256), G::LDS, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a);
    else
        hipLaunchKernelGGL(k, grid, dim3(256), G::LDS, s, a);
    return hipGetLastError();
}

// out[s = cc*9 + tap][g][n][e] = w[n][tap*IC + 32cc + 8g + e]
__global__ __launch_bounds__(256) void img_pack_kernel(const bf16_t* __restrict__ w, int Kpad, int ic,
                                                       bf16_t* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x, total = (ic / 32) * 9 * 4 * ic;
    if (i >= total) return;
    const int n = i % ic, g = (i / ic) % 4, s = i / (4 * ic), cc = s / 9, tap = s % 9;
    *(uint4*)(out + (size_t)i * 8) = *(const uint4*)(w + (size_t)n * Kpad + tap * ic + 32 * cc + 8 * g);
}

}  // namespace

bool img_shape_ok(const ConvArgs& a, int* ic) {
    ConvArgs t = a;
    t.wimg = (const bf16_t*)1;
    t.negf = (const float*)1;
    if (img_supported_t<Geo28>(t)) { *ic = 128; return true; }
    if (img_supported_t<Geo56>(t)) { *ic = 64; return true; }
    return false;
}

size_t img_packed_elems(int ic) { return (size_t)(ic / 32) * 9 * 4 * ic * 8; }

hipError_t img_pack_weights(const bf16_t* w, int Kpad, int ic, bf16_t* out, hipStream_t s) {
    const int total = (ic / 32) * 9 * 4 * ic;
    hipLaunchKernelGGL(img_pack_kernel, dim3((total + 255) / 256), dim3(256), 0, s, w, Kpad, ic, out);
    return hipGetLastError();
}

bool img28_supported(const ConvArgs& a) { return img_supported_t<Geo28>(a); }
bool img56_supported(const ConvArgs& a) { return img_supported_t<Geo56>(a); }

hipError_t launch_conv_img28(const ConvArgs& a, hipStream_t s) {
    return img28_supported(a) ? launch_img_t<Geo28>(a, s) : hipErrorInvalidValue;
}
hipError_t launch_conv_img56(const ConvArgs& a, hipStream_t s) {
    return img56_supported(a) ? launch_img_t<Geo56>(a, s) : hipErrorInvalidValue;
}

}  // namespace fr
