// Shared device/host helpers for the frhip kernels (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cmath>
#include <string>

typedef uint16_t bf16_t;  // 16-bit activation/weight storage (bf16 or f16 bits, per handle dtype)
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_t;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_t;
typedef __attribute__((ext_vector_type(4))) float f32x4_t;

namespace fr {

// Thread-local last-error plumbing (defined in engine.cpp).
void set_error(const std::string& msg);
// A/B switches from the FR_AB environment variable (engine.cpp): "key" or "key=value", comma separated
const char* ab_str(const char* key);
int ab_int(const char* key, int dflt);

#define FR_HIP_CHECK(expr)                                                        \
    do {                                                                          \
        hipError_t _e = (expr);                                                   \
        if (_e != hipSuccess) {                                                   \
            ::fr::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));   \
            return FR_ERR_HIP;                                                    \
        }                                                                         \
    } while (0)

// f32 -> bf16 round-to-nearest-even on the host (weights packing).
static inline bf16_t host_f2bf(float f) {
    uint32_t u;
    __builtin_memcpy(&u, &f, 4);
    if ((u & 0x7f800000u) == 0x7f800000u) return (bf16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
    u += 0x7fffu + ((u >> 16) & 1u);
    return (bf16_t)(u >> 16);
}

// f32 -> OCP e4m3fn (gfx950 fp8) round-to-nearest-even on the host, saturating to +-448 (no NaN from
// weights).  Exact for values that are already e4m3-representable (weights.quantize_fp8 output).
static inline uint8_t host_f2e4m3(float f) {
    const uint8_t s = f < 0.f ? 0x80 : 0;
    float a = f < 0.f ? -f : f;
    if (!(a == a)) return 0x7f;
    if (a >= 448.f) return s | 0x7e;
    int e;
    const float m = frexpf(a, &e);  // a = m * 2^e, m in [0.5, 1)
    int E = e - 1;                  // a = (2m) * 2^E, 2m in [1, 2)
    if (a == 0.f || E < -6) {       // subnormal: step 2^-9
        const int q = (int)nearbyintf(a * 512.f);
        return s | (uint8_t)q;      // q == 8 is the smallest normal (exp 1, mantissa 0): same bits
    }
    int q = (int)nearbyintf((2.f * m - 1.f) * 8.f);
    if (q == 8) { q = 0; ++E; }
    if (E > 8 || (E == 8 && q == 7)) return s | 0x7e;
    return s | (uint8_t)(((E + 7) << 3) | q);
}

// f32 -> f16 round-to-nearest-even on the host, saturating to ±65504 (no inf from weights).
static inline uint16_t host_f2h(float f) {
    if (f > 65504.f) f = 65504.f;
    if (f < -65504.f) f = -65504.f;
    _Float16 h = (_Float16)f;
    uint16_t r;
    __builtin_memcpy(&r, &h, 2);
    return r;
}
static inline float host_h2f(uint16_t v) {
    _Float16 h;
    __builtin_memcpy(&h, &v, 2);
    return (float)h;
}
static inline float host_bf2f(bf16_t v) {
    uint32_t u = ((uint32_t)v) << 16;
    float f;
    __builtin_memcpy(&f, &u, 4);
    return f;
}

// min(v, 0) as a raw v_min_f32: fminf first canonicalizes its operand (one more VALU op per value); the
// epilogues apply it to MFMA accumulators, which are never signalling NaNs, so the result bits are the same
__device__ __forceinline__ float min0_raw(float v) {
    float r;
    asm("v_min_f32 %0, 0, %1" : "=v"(r) : "v"(v));
    return r;
}
__device__ __forceinline__ float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// Pack two floats into two bf16 (RNE): one v_cvt_pk_bf16_f32 on gfx950 (two scalar casts can come out
// as two converts plus shifts and ors).
__device__ __forceinline__ uint32_t pack2_bf16(float a, float b) {
    typedef float f32x2_v __attribute__((ext_vector_type(2)));
    typedef __bf16 bf16x2_v __attribute__((ext_vector_type(2)));
    const f32x2_v v = {a, b};
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_v));
}

__device__ __forceinline__ void unpack8_bf16(const uint4& v, float* f) {
    f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
    f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
    f[4] = __uint_as_float(v.z << 16); f[5] = __uint_as_float(v.z & 0xffff0000u);
    f[6] = __uint_as_float(v.w << 16); f[7] = __uint_as_float(v.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 pack8_bf16(const float* f) {
    uint4 r;
    r.x = pack2_bf16(f[0], f[1]); r.y = pack2_bf16(f[2], f[3]);
    r.z = pack2_bf16(f[4], f[5]); r.w = pack2_bf16(f[6], f[7]);
    return r;
}

// 16-bit number formats of the compute path.  Both run v_mfma_f32_16x16x32_{bf16,f16} at the
// same rate with f32 accumulation; f16 carries 3 more mantissa bits, bf16 more range.
template <bool F16>
struct Num;

template <>
struct Num<false> {  // bf16
    typedef bf16x8_t frag;
    static __device__ __forceinline__ f32x4_t mfma(const frag& a, const frag& b, const f32x4_t& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ void unpack8(const uint4& v, float* f) { unpack8_bf16(v, f); }
    static __device__ __forceinline__ uint4 pack8(const float* f) { return pack8_bf16(f); }
    static __device__ __forceinline__ uint16_t cvt(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }
};

// ReLU as one v_max_i32 on the bits (a negative float is a negative int; -0 becomes +0).  fmaxf(v, 0.f) first
// canonicalizes v in IEEE mode: two VALU per value in the fused kernels' epilogues
__device__ __forceinline__ float relu_bits(float v) { return __builtin_bit_cast(float, max(__builtin_bit_cast(int, v), 0)); }

__device__ __forceinline__ uint32_t pack2_f16(float a, float b) {
    a = fminf(fmaxf(a, -65504.f), 65504.f);  // saturate: an overflow must not become inf
    b = fminf(fmaxf(b, -65504.f), 65504.f);
    _Float16 x = (_Float16)a, y = (_Float16)b;
    return (uint32_t)__builtin_bit_cast(uint16_t, x) | ((uint32_t)__builtin_bit_cast(uint16_t, y) << 16);
}

template <>
struct Num<true> {  // f16
    typedef f16x8_t frag;
    static __device__ __forceinline__ f32x4_t mfma(const frag& a, const frag& b, const f32x4_t& c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
    }
    static __device__ __forceinline__ float h2f(uint32_t bits16) {
        return (float)__builtin_bit_cast(_Float16, (uint16_t)bits16);
    }
    static __device__ __forceinline__ void unpack8(const uint4& v, float* f) {
        f[0] = h2f(v.x & 0xffff); f[1] = h2f(v.x >> 16); f[2] = h2f(v.y & 0xffff); f[3] = h2f(v.y >> 16);
        f[4] = h2f(v.z & 0xffff); f[5] = h2f(v.z >> 16); f[6] = h2f(v.w & 0xffff); f[7] = h2f(v.w >> 16);
    }
    static __device__ __forceinline__ uint4 pack8(const float* f) {
        uint4 r;
        r.x = pack2_f16(f[0], f[1]); r.y = pack2_f16(f[2], f[3]);
        r.z = pack2_f16(f[4], f[5]); r.w = pack2_f16(f[6], f[7]);
        return r;
    }
    static __device__ __forceinline__ uint16_t cvt(float f) {
        f = fminf(fmaxf(f, -65504.f), 65504.f);
        return __builtin_bit_cast(uint16_t, (_Float16)f);
    }
};

// Border class of output pixel (oh, ow) for a bias9 table (3x3 / stride 1 / pad 1 with the input BN
// folded into the weights): 3*rc + cc, rc = 0 top row, 1 interior, 2 bottom row (cc for columns).
__device__ __forceinline__ int border_class(int oh, int ow, int Ho, int Wo) {
    const int rc = oh == 0 ? 0 : (oh == Ho - 1 ? 2 : 1);
    const int cc = ow == 0 ? 0 : (ow == Wo - 1 ? 2 : 1);
    return 3 * rc + cc;
}

// Bijective XCD-aware block remap (cdna_hip_programming.md §5, "XCD swizzle must be
// bijective"): blocks that share an XCD (raw id ≡ mod 8) get consecutive logical ids.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    if (nwg <= 8) return bid;
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, loc = bid / 8;
    return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + loc;
}

}  // namespace fr
