// Persistent small-K direct convolution (CDNA4 / gfx950): any Kh x Kw, stride, padding, Cin % 8 == 0,
// K = Kh*Kw*Cin <= 384 (Kpad / 32 <= 12 K-steps), Cout % (16 NF) == 0.
//
// For these shapes (FaceNet InceptionResnetV1: the stem convs at 160..38 px with 8..80 channels, the
// Block35 3x3 32 -> 32 convs and the 1x1 convs with K <= 384) the implicit GEMM re-gathers the taps
// and re-streams the weights per 128-pixel tile for 2..6 K-steps only, so each tile is mostly prologue
// and epilogue: 2-6 x below the HBM floor of these layers (profiles/r03_irv1_layer_profile.txt).
// Here, as in conv_rows.hip:
//   * one workgroup per CU (4 waves, one per SIMD, up to 512 registers each) owns one group of 16 NF
//     output channels for the whole launch; its weights go from the [Npad][Kpad] rows straight into
//     VGPRs once (K-step ks, lane group g: the 16-B A fragment W[n][32 ks + 8 g .. +8]);
//   * a unit = 64 FW consecutive output pixels of one image (row-major); the input rows it reads (all
//     columns, zero halo from out-of-range DMA offsets) are LDS-DMA'd into one of two buffers while the
//     previous unit computes; wave w computes the unit's pixel fragments [FW w, FW w + FW);
//   * operand B of K-step ks for a lane is the 8 channels 32 ks + 8 g .. of the flattened K = (kh, kw, c)
//     at its pixel: a per-lane byte offset (tap shift + channel) computed once per launch, added to the
//     fragment's base position;
//   * patch positions are CINB + 32 bytes apart when CINB / 16 is even (CINB = 2 Cin): 16 consecutive
//     positions x 4 lane groups then hit 16 distinct 16-B bank groups (conflict-free ds_read_b128);
//   * the K order (32-deep MFMA chunks of the flattened K) and the epilogue arithmetic (bias, then the
//     activation, as conv_igemm's epilogue8) are the implicit GEMM's, so the output equals conv_igemm
//     tile 0 bit for bit and the per-shape autotuner can time this kernel beside the igemm tiles.
#include "kernels.h"

#include <hip/hip_ext.h>

namespace fr {
namespace {

constexpr int DNW = 4;    // waves, one per SIMD
constexpr int KSR1 = 12;  // register-resident K-steps at one workgroup per CU: Kpad <= 384
constexpr int KSR2 = 10;  // ... at two (NF = 2 only): Kpad <= 320
constexpr uint32_t OOB = 0x80000000u;

typedef __attribute__((address_space(3))) void lds_void;

struct DGeo {
    int PST;      // bytes per patch position (CINB, + 32 when CINB / 16 is even)
    int PCH;      // 16-B slots per position (PST / 16)
    int CH16;     // data slots per position (Cin / 8)
    int PW;       // positions per patch row (W + 2 pw)
    int PATCH_B;  // bytes per patch buffer (a multiple of 1024)
    int KS;       // K-steps of 32
    int upi;      // units per image
    int units;    // B * upi
    int ngroups;  // Cout / (16 NF)
};

template <int NF, int FW>
__host__ __device__ constexpr int direct_upx() { return 16 * FW * DNW; }

// OCC: workgroups per CU (2: up to 256 registers per wave, 10 register K-steps; for the small convs whose
// per-unit DMA latency one workgroup cannot hide)
template <bool F16, int NF, int FW, int OCC>
__global__ __launch_bounds__(64 * DNW, OCC) void conv_direct_kernel(ConvArgs p, DGeo g) {
    constexpr int KSR = OCC == 2 ? KSR2 : KSR1;
    typedef Num<F16> T;
    typedef typename T::frag frag;
    constexpr int UPX = direct_upx<NF, FW>();
    extern __shared__ __attribute__((aligned(16))) char smem[];  // [patch 0][patch 1]
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lg = lane >> 4, lr = lane & 15;
    const int ng = blockIdx.x % g.ngroups, k0 = blockIdx.x / g.ngroups, kstride = gridDim.x / g.ngroups;
    if (k0 >= g.units) return;
    const int H = p.H, W = p.W, Wo = p.Wo, HoWo = p.Ho * p.Wo;
    const int n0 = ng * 16 * NF;

    // ---- weights -> VGPRs (K-steps past Kpad / 32 are zero and never used)
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.w, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)p.Npad * p.Kpad * 2), 0x00020000);
    frag wa[KSR][NF];
#pragma unroll
    for (int ks = 0; ks < KSR; ++ks)
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const uint32_t off = ks < g.KS ? (uint32_t)(((n0 + 16 * i + lr) * p.Kpad + 32 * ks + 8 * lg) * 2) : OOB;
            wa[ks][i] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
        }
    // the lane's bias / PReLU slopes (loaded once: a global load in the epilogue would wait for the next
    // unit's patch DMA and this unit's stores, which vmcnt counts in order with it)
    float4 bias4[NF], slope4[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int n = n0 + 16 * i + 4 * lg;
        bias4[i] = p.bias ? *(const float4*)(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        slope4[i] = p.act == 2 ? *(const float4*)(p.slope + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    // ---- the lane's operand-B byte offset per K-step: flattened K index 32 ks + 8 lg = (tap, c); taps
    // past Kh*Kw (the zero-weight K padding) read tap 0
    int koff[KSR];
    {
        const int taps = p.Kh * p.Kw;
#pragma unroll
        for (int ks = 0; ks < KSR; ++ks) {
            const int kk = 32 * ks + 8 * lg;
            int t = kk / p.Cin, c = kk - t * p.Cin;
            if (t >= taps) t = 0, c = 0;
            const int kh = t / p.Kw, kw = t - kh * p.Kw;
            koff[ks] = (kh * g.PW + kw) * g.PST + c * 2;
        }
    }

    const uint32_t x_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.B * H * W * p.Cx * 2);
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)p.x, 0, x_bytes, 0x00020000);
    const uint32_t y_bytes = (uint32_t)min((size_t)0x7fffffff, (size_t)p.M * p.Cy * 2);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc((void*)p.y, 0, y_bytes, 0x00020000);

    struct Unit {
        int b, p0, p1, oh0, ih0, rows;
    };
    auto unit_of = [&](int k) {
        Unit u;
        u.b = k / g.upi;
        u.p0 = (k - u.b * g.upi) * UPX;
        u.p1 = min(u.p0 + UPX, HoWo);
        u.oh0 = u.p0 / Wo;
        const int oh1 = (u.p1 - 1) / Wo;
        u.ih0 = u.oh0 * p.sh - p.ph;
        u.rows = (oh1 - u.oh0) * p.sh + p.Kh;
        return u;
    };
    // DMA of a unit's input rows into buffer buf: 16-B slot q = (row, position, chunk); chunks past Cin / 8
    // (the bank-conflict pad) and positions outside the image read as zeros
    auto issue_patch = [&](const Unit& u, int buf) {
        const int per_row = g.PW * g.PCH, nslots = u.rows * per_row;
        int ln = lane;
        asm volatile("" : "+v"(ln));
        for (int piece = wave; piece * 64 < nslots; piece += DNW) {
            const int q = piece * 64 + ln;
            const int row = q / per_row, rem = q - row * per_row, pos = rem / g.PCH, ch = rem - pos * g.PCH;
            const int ih = u.ih0 + row, iw = pos - p.pw;
            const bool in = q < nslots && ch < g.CH16 && (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
            const uint32_t off = in ? (uint32_t)(((((size_t)u.b * H + ih) * W + iw) * p.Cx + p.x_off + 8 * ch) * 2) : OOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (lds_void*)(smem + buf * g.PATCH_B + piece * 1024), 16, off, 0, 0, 0);
        }
    };

    Unit cur = unit_of(k0);
    issue_patch(cur, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    int buf = 0;
    f32x4_t acc[NF][FW];
#pragma unroll 1
    for (int k = k0; k < g.units; k += kstride) {
        const bool has_next = k + kstride < g.units;
        const Unit nxt = has_next ? unit_of(k + kstride) : cur;
        if (has_next) issue_patch(nxt, buf ^ 1);
        // fragment base positions (bytes) of the lane's pixels; pixels past the unit repeat its last
        int pb[FW];
#pragma unroll
        for (int j = 0; j < FW; ++j) {
            int px = cur.p0 + 16 * (FW * wave + j) + lr;
            px = px < cur.p1 ? px : cur.p1 - 1;
            const int oh = px / Wo, ow = px - oh * Wo;
            pb[j] = buf * g.PATCH_B + ((oh - cur.oh0) * p.sh * g.PW + ow * p.sw) * g.PST;
        }
#pragma unroll
        for (int i = 0; i < NF; ++i)
#pragma unroll
            for (int j = 0; j < FW; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        // ---- K loop: fragments of step ks + 1 read during step ks's MFMAs
        frag fb[2][FW];
#pragma unroll
        for (int j = 0; j < FW; ++j) fb[0][j] = *(const frag*)(smem + pb[j] + koff[0]);
#pragma unroll
        for (int ks = 0; ks < KSR; ++ks) {
            if (ks < g.KS) {
                if (ks + 1 < KSR && ks + 1 < g.KS) {
#pragma unroll
                    for (int j = 0; j < FW; ++j) fb[(ks + 1) & 1][j] = *(const frag*)(smem + pb[j] + koff[ks + 1]);
                }
#pragma unroll
                for (int i = 0; i < NF; ++i)
#pragma unroll
                    for (int j = 0; j < FW; ++j) acc[i][j] = T::mfma(wa[ks][i], fb[ks & 1][j], acc[i][j]);
            }
        }
        // ---- epilogue (conv_igemm epilogue8's arithmetic): bias, activation, pack, 8-B buffer stores
        // (pixels past the unit: out-of-range offsets, so every wave issues exactly NF * FW stores)
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int n = n0 + 16 * i + 4 * lg;
            const float4 bb = bias4[i], sl = slope4[i];
#pragma unroll
            for (int j = 0; j < FW; ++j) {
                float v[8] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3], 0.f, 0.f, 0.f, 0.f};
                if (p.bias) {
                    v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
                }
                if (p.act == 1) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
                } else if (p.act == 2) {
                    v[0] = v[0] > 0.f ? v[0] : v[0] * sl.x;
                    v[1] = v[1] > 0.f ? v[1] : v[1] * sl.y;
                    v[2] = v[2] > 0.f ? v[2] : v[2] * sl.z;
                    v[3] = v[3] > 0.f ? v[3] : v[3] * sl.w;
                }
                const uint4 pk = F16 && p.y_bf16 ? Num<false>::pack8(v) : T::pack8(v);
                const int px = cur.p0 + 16 * (FW * wave + j) + lr;
                const uint32_t off =
                    px < cur.p1 ? (uint32_t)((((size_t)cur.b * HoWo + px) * p.Cy + p.y_off + n) * 2) : OOB;
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64((u32x2){pk.x, pk.y}, yr, off, 0, 0);
            }
        }
        // the next unit's rows landed (they precede this unit's NF * FW stores, which stay in flight) and
        // every wave is past its reads of `buf`, which the next iteration's DMA overwrites
        if constexpr (NF * FW == 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
        else if constexpr (NF * FW == 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
        else if constexpr (NF * FW == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        else if constexpr (NF * FW == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        cur = nxt;
        buf ^= 1;
    }
}

// 1x1 / stride-1 / unpadded convs: a unit's pixels are contiguous NHWC rows, so operand B goes straight
// from global memory into registers (no patch, no LDS): every K-step's fragment of the unit at once,
// the next unit's during this unit's MFMAs (two register sets).  Units run over all B * H * W pixels.
// Epilogue as conv_igemm's epilogue8: bias, residual, activation.
template <bool F16, int NF, int FW, int KSR>  // KSR: K-steps compiled (>= Kpad / 32; the rest read zeros)
__global__ __launch_bounds__(64 * DNW, 1) void conv_direct1_kernel(ConvArgs p, DGeo g) {
    typedef Num<F16> T;
    typedef typename T::frag frag;
    constexpr int UPX = 16 * FW * DNW;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lg = lane >> 4, lr = lane & 15;
    const int ng = blockIdx.x % g.ngroups, k0 = blockIdx.x / g.ngroups, kstride = gridDim.x / g.ngroups;
    if (k0 >= g.units) return;
    const int n0 = ng * 16 * NF, M = p.M;

    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.w, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)p.Npad * p.Kpad * 2), 0x00020000);
    frag wa[KSR][NF];
#pragma unroll
    for (int ks = 0; ks < KSR; ++ks)
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const uint32_t off = ks < g.KS ? (uint32_t)(((n0 + 16 * i + lr) * p.Kpad + 32 * ks + 8 * lg) * 2) : OOB;
            wa[ks][i] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(wr, off, 0, 0));
        }
    float4 bias4[NF], slope4[NF];
#pragma unroll
    for (int i = 0; i < NF; ++i) {
        const int n = n0 + 16 * i + 4 * lg;
        bias4[i] = p.bias ? *(const float4*)(p.bias + n) : make_float4(0.f, 0.f, 0.f, 0.f);
        slope4[i] = p.act == 2 ? *(const float4*)(p.slope + n) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.x, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)M * p.Cx * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t yr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)p.y, 0, (uint32_t)min((size_t)0x7fffffff, (size_t)M * p.Cy * 2), 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(p.res ? p.res : p.y), 0, (uint32_t)(p.res ? min((size_t)0x7fffffff, (size_t)M * p.Cres * 2) : 0), 0x00020000);
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

    auto load_unit = [&](int k, frag (&fb)[KSR][FW], u32x2 (&rs)[NF][FW]) {
#pragma unroll
        for (int j = 0; j < FW; ++j) {
            const int px = k * UPX + 16 * (FW * wave + j) + lr;
            const bool ok = px < M;
#pragma unroll
            for (int ks = 0; ks < KSR; ++ks) {  // branch free: steps past Kpad / 32 read zeros
                const uint32_t off =
                    ok && ks < g.KS ? (uint32_t)(((size_t)px * p.Cx + p.x_off + 32 * ks + 8 * lg) * 2) : OOB;
                fb[ks][j] = __builtin_bit_cast(frag, __builtin_amdgcn_raw_buffer_load_b128(xr, off, 0, 0));
            }
            if (p.res) {
#pragma unroll
                for (int i = 0; i < NF; ++i) {
                    const uint32_t off =
                        ok ? (uint32_t)(((size_t)px * p.Cres + p.res_off + n0 + 16 * i + 4 * lg) * 2) : OOB;
                    rs[i][j] = __builtin_amdgcn_raw_buffer_load_b64(rr, off, 0, 0);
                }
            }
        }
    };
    auto run_unit = [&](int k, const frag (&fb)[KSR][FW], const u32x2 (&rs)[NF][FW]) {
        f32x4_t acc[NF][FW];
#pragma unroll
        for (int i = 0; i < NF; ++i)
#pragma unroll
            for (int j = 0; j < FW; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KSR; ++ks)
#pragma unroll
            for (int i = 0; i < NF; ++i)
#pragma unroll
                for (int j = 0; j < FW; ++j) acc[i][j] = T::mfma(wa[ks][i], fb[ks][j], acc[i][j]);
#pragma unroll
        for (int i = 0; i < NF; ++i) {
            const int n = n0 + 16 * i + 4 * lg;
            const float4 bb = bias4[i], sl = slope4[i];
#pragma unroll
            for (int j = 0; j < FW; ++j) {
                float v[8] = {acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3], 0.f, 0.f, 0.f, 0.f};
                if (p.bias) {
                    v[0] += bb.x; v[1] += bb.y; v[2] += bb.z; v[3] += bb.w;
                }
                if (p.res) {
                    float f[8];
                    T::unpack8(make_uint4(rs[i][j].x, rs[i][j].y, 0u, 0u), f);
                    v[0] += f[0]; v[1] += f[1]; v[2] += f[2]; v[3] += f[3];
                }
                if (p.act == 1) {
#pragma unroll
                    for (int e = 0; e < 4; ++e) v[e] = v[e] > 0.f ? v[e] : 0.f;
                } else if (p.act == 2) {
                    v[0] = v[0] > 0.f ? v[0] : v[0] * sl.x;
                    v[1] = v[1] > 0.f ? v[1] : v[1] * sl.y;
                    v[2] = v[2] > 0.f ? v[2] : v[2] * sl.z;
                    v[3] = v[3] > 0.f ? v[3] : v[3] * sl.w;
                }
                const uint4 pk = F16 && p.y_bf16 ? Num<false>::pack8(v) : T::pack8(v);
                const int px = k * UPX + 16 * (FW * wave + j) + lr;
                const uint32_t off = px < M ? (uint32_t)(((size_t)px * p.Cy + p.y_off + n) * 2) : OOB;
                __builtin_amdgcn_raw_buffer_store_b64((u32x2){pk.x, pk.y}, yr, off, 0, 0);
            }
        }
    };
    frag fA[KSR][FW], fB[KSR][FW];
    u32x2 rA[NF][FW], rB[NF][FW];
    int k = k0;
    load_unit(k, fA, rA);
#pragma unroll 1
    while (true) {
        if (k + kstride < g.units) load_unit(k + kstride, fB, rB);
        run_unit(k, fA, rA);
        k += kstride;
        if (k >= g.units) break;
        if (k + kstride < g.units) load_unit(k + kstride, fA, rA);
        run_unit(k, fB, rB);
        k += kstride;
        if (k >= g.units) break;
    }
}

struct DCfg;
DGeo direct_geo(const ConvArgs& a, const DCfg& c, int* lds);

// configuration of a shape: NF (16-channel fragments per wave = channels per workgroup / 16) and FW
// (pixel fragments per wave); 0 = unsupported
struct DCfg {
    int nf, fw, occ, mode;  // mode 1: 1x1 / stride 1 / unpadded, operand B from global (conv_direct1_kernel)
};
static bool direct1_shape(const ConvArgs& a) {
    return a.Kh == 1 && a.Kw == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0 && a.Ho == a.H && a.Wo == a.W;
}
DCfg direct_cfg(const ConvArgs& a) {
    DCfg c{0, 0, 1, 0};
    if (a.res && (!direct1_shape(a) || a.Cres % 4 || a.res_off % 4)) return c;  // residual: the 1x1 kernel only
    if (a.Kh <= 0 || a.Kw <= 0 || a.x2 || a.y2 || a.partial || a.w8 || a.y_amax || a.bias9 || a.Cin % 8 || a.Cx % 8 || a.x_off % 8 ||
        a.Cy % 4 || a.y_off % 4 || a.Kpad % 32 || a.Kpad / 32 > KSR1 || a.K > a.Kpad || a.sh < 1 || a.sw < 1 ||
        a.B <= 0 || a.Ho <= 0 || a.Wo <= 0)
        return c;
    c.nf = a.Cout % 64 == 0 ? 4 : (a.Cout % 32 == 0 ? 2 : 0);
    if (!c.nf) return c;
    if (direct1_shape(a)) {  // no patch: one or two fragments per wave (the registers hold two units' operands)
        c.mode = 1;
        c.fw = c.nf == 4 ? 1 : 2;
        return c;
    }
    // pixel fragments per wave: the largest unit (8, 4, 2 or 1 fragments per wave; larger units re-read
    // fewer halo rows) whose padded pixel count is
    // within 5 % of the least padded one and whose two patch buffers fit the LDS
    const int hw = a.Ho * a.Wo;
    int best_u = 1 << 30;
    const int fw_max = c.nf == 4 ? 4 : 8;  // NF = 4 with 8 fragments per wave spills at 512 registers
    for (int fw = fw_max; fw >= 1; fw /= 2) best_u = min(best_u, (hw + 64 * fw - 1) / (64 * fw) * 64 * fw);
    for (int fw = fw_max; fw >= 1; fw /= 2) {
        const int u = (hw + 64 * fw - 1) / (64 * fw) * 64 * fw;
        if (u * 100 > best_u * 105) continue;
        DCfg t{c.nf, fw, 1};
        int lds = 0;
        (void)direct_geo(a, t, &lds);
        if (lds <= 160 * 1024) {
            c.fw = fw;
            break;
        }
    }
    if (!c.fw) c.nf = 0;
    // two workgroups per CU when their registers (NF = 2, <= 10 K-steps) and LDS allow
    if (c.nf == 2 && c.fw <= 4 && a.Kpad / 32 <= KSR2) {
        int lds = 0;
        (void)direct_geo(a, c, &lds);
        if (2 * lds <= 160 * 1024) c.occ = 2;
    }
    return c;
}

DGeo direct_geo(const ConvArgs& a, const DCfg& c, int* lds) {
    DGeo g{};
    if (c.mode == 1) {
        g.KS = a.Kpad / 32;
        g.units = (a.M + 16 * c.fw * DNW - 1) / (16 * c.fw * DNW);
        g.upi = g.units;
        g.ngroups = a.Cout / (16 * c.nf);
        *lds = 0;
        return g;
    }
    const int cinb = a.Cin * 2;
    g.CH16 = a.Cin / 8;
    // 16-B slots per position: for >= 4 data chunks the next count = 2 (mod 4), so that 16 consecutive
    // positions' (position x slots + lane group) values are 16 distinct bank groups
    // (below 8 chunks the pad would cost more DMA traffic than the 2-way conflicts it avoids: these
    // convs are bound by the patch stream)
    g.PCH = g.CH16 < 8 ? g.CH16 : g.CH16 + (6 - g.CH16 % 4) % 4;
    g.PST = g.PCH * 16;
    g.PW = a.W + 2 * a.pw;
    (void)cinb;
    const int upx = 16 * c.fw * DNW;
    // rows of the largest unit: its pixels span at most ceil(upx / Wo) + 1 output rows
    const int orows = min(a.Ho, (upx + a.Wo - 1) / a.Wo + 1);
    const int prow = (orows - 1) * a.sh + a.Kh;
    g.PATCH_B = (prow * g.PW * g.PST + 1023) / 1024 * 1024;
    g.KS = a.Kpad / 32;
    g.upi = (a.Ho * a.Wo + upx - 1) / upx;
    g.units = a.B * g.upi;
    g.ngroups = a.Cout / (16 * c.nf);
    *lds = 2 * g.PATCH_B;
    return g;
}

}  // namespace

bool direct_supported(const ConvArgs& a) {
    const DCfg c = direct_cfg(a);
    if (!c.nf) return false;
    int lds = 0;
    const DGeo g = direct_geo(a, c, &lds);
    (void)g;
    return lds <= 160 * 1024 && (size_t)a.B * a.H * a.W * a.Cx * 2 < 0x7fffffffull &&
           (size_t)a.M * a.Cy * 2 < 0x7fffffffull && (!a.res || (size_t)a.M * a.Cres * 2 < 0x7fffffffull);
}

hipError_t launch_conv_direct(const ConvArgs& a, int n_cu, hipStream_t s) {
    if (!direct_supported(a)) return hipErrorInvalidValue;
    const DCfg c = direct_cfg(a);
    int lds = 0;
    const DGeo g = direct_geo(a, c, &lds);
    if (n_cu <= 0) {  // the launching device's CU count (queried once per device)
        static int cus[64] = {0};
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (dev < 0 || dev >= 64) dev = 0;
        if (!cus[dev]) {
            hipDeviceProp_t prop;
            cus[dev] = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
        }
        n_cu = cus[dev];
    }
    int grid = (c.occ * n_cu / g.ngroups) * g.ngroups;
    if (grid < g.ngroups) grid = g.ngroups;
    if (grid > g.units * g.ngroups) grid = g.units * g.ngroups;
    typedef void (*KFn)(ConvArgs, DGeo);
    static const KFn kt[2][4][2] = {
        {{conv_direct_kernel<false, 2, 1, 1>, conv_direct_kernel<true, 2, 1, 1>},
         {conv_direct_kernel<false, 2, 2, 1>, conv_direct_kernel<true, 2, 2, 1>},
         {conv_direct_kernel<false, 2, 4, 1>, conv_direct_kernel<true, 2, 4, 1>},
         {conv_direct_kernel<false, 2, 8, 1>, conv_direct_kernel<true, 2, 8, 1>}},
        {{conv_direct_kernel<false, 4, 1, 1>, conv_direct_kernel<true, 4, 1, 1>},
         {conv_direct_kernel<false, 4, 2, 1>, conv_direct_kernel<true, 4, 2, 1>},
         {conv_direct_kernel<false, 4, 4, 1>, conv_direct_kernel<true, 4, 4, 1>},
         {conv_direct_kernel<false, 4, 4, 1>, conv_direct_kernel<true, 4, 4, 1>}}};  // (FW = 8: not used with NF = 4)
    static const KFn kt2[3][2] = {{conv_direct_kernel<false, 2, 1, 2>, conv_direct_kernel<true, 2, 1, 2>},
                                  {conv_direct_kernel<false, 2, 2, 2>, conv_direct_kernel<true, 2, 2, 2>},
                                  {conv_direct_kernel<false, 2, 4, 2>, conv_direct_kernel<true, 2, 4, 2>}};
    const int ni = c.nf == 4 ? 1 : 0, fi = c.fw == 8 ? 3 : (c.fw == 4 ? 2 : (c.fw == 2 ? 1 : 0)), di = a.f16 ? 1 : 0;
#define D1(F16, NF, FW) \
    { conv_direct1_kernel<F16, NF, FW, 2>, conv_direct1_kernel<F16, NF, FW, 4>, conv_direct1_kernel<F16, NF, FW, 8>, \
      conv_direct1_kernel<F16, NF, FW, 12> }
    static const KFn kt1[2][2][4] = {{D1(false, 2, 2), D1(true, 2, 2)}, {D1(false, 4, 1), D1(true, 4, 1)}};
#undef D1
    const int ks = a.Kpad / 32, ki = ks <= 2 ? 0 : (ks <= 4 ? 1 : (ks <= 8 ? 2 : 3));
    const KFn k = c.mode == 1 ? kt1[ni][di][ki] : (c.occ == 2 ? kt2[fi][di] : kt[ni][fi][di]);
    static int attr_lds[32] = {0};  // the largest size set per instantiation
    const int ai = ((c.occ == 2 ? 2 : 0) + ni) * 8 + fi * 2 + di;
    if (c.mode == 0 && lds > attr_lds[ai]) {
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
        attr_lds[ai] = lds;
    }
    if (a.ev0)
        hipExtLaunchKernelGGL(k, dim3(grid), dim3(64 * DNW), lds, s, (hipEvent_t)a.ev0, (hipEvent_t)a.ev1, 0, a, g);
    else
        hipLaunchKernelGGL(k, dim3(grid), dim3(64 * DNW), lds, s, a, g);
    return hipGetLastError();
}

}  // namespace fr
