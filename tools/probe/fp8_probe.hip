// Probe (run once on the GPU box): lane->k map of v_mfma_scale_f32_16x16x128_f8f6f4 with fp8 e4m3
// operands, and v_cvt_scalef32_pk_fp8_bf16 scale direction / saturation.  Exact small-integer data.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <cmath>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) short i16x2;

// e4m3fn encode for small integers 0..7 and 1: value v -> bits
static unsigned char enc(float v) {
    if (v == 0) return 0;
    int s = v < 0; v = fabsf(v);
    int e = (int)floorf(log2f(v)); float m = v / ldexpf(1, e) - 1; // 1.m
    int em = e + 7; int mm = (int)lrintf(m * 8);
    if (mm == 8) { mm = 0; em++; }
    return (unsigned char)((s << 7) | (em << 3) | mm);
}

__global__ void mm(const unsigned char* A, const unsigned char* B, float* D, int mode) {
    // A: 16 x 128 row-major bytes, B: 16 (cols) x 128 (k) bytes; mode 0: lane l takes A[l&15][32*(l>>4)+j]
    const int l = threadIdx.x;
    unsigned char a[32], b[32];
    for (int j = 0; j < 32; ++j) {
        int k = mode == 0 ? 32 * (l >> 4) + j : (j / 8) * 32 + 8 * (l >> 4) + (j % 8);
        a[j] = A[(l & 15) * 128 + k];
        b[j] = B[(l & 15) * 128 + k];
    }
    i32x8 av, bv;
    memcpy(&av, a, 32); memcpy(&bv, b, 32);
    f32x4 c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 127, 0, 127);
    for (int r = 0; r < 4; ++r) D[(4 * (l >> 4) + r) * 16 + (l & 15)] = c[r];
}

__global__ void cvt(const float* x, unsigned* y, float s) {
    const int l = threadIdx.x;
    bf16x2 v = {(__bf16)x[2 * l], (__bf16)x[2 * l + 1]};
    i16x2 o = {0, 0};
    o = __builtin_amdgcn_cvt_scalef32_pk_fp8_bf16(o, v, s, false);
    y[l] = (unsigned)__builtin_bit_cast(unsigned, o) & 0xffff;
}

int main() {
    unsigned char hA[16 * 128], hB[16 * 128];
    float ref[256];
    srand(1);
    float fa[16][128], fb[16][128];
    for (int i = 0; i < 16; ++i) for (int k = 0; k < 128; ++k) {
        fa[i][k] = (float)(rand() % 7 - 3); fb[i][k] = (float)(rand() % 5 - 2);
        hA[i * 128 + k] = enc(fa[i][k]); hB[i * 128 + k] = enc(fb[i][k]);
    }
    for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) {
        float s = 0; for (int k = 0; k < 128; ++k) s += fa[i][k] * fb[j][k]; ref[i * 16 + j] = s;
    }
    unsigned char *dA, *dB; float* dD;
    hipMalloc(&dA, 2048); hipMalloc(&dB, 2048); hipMalloc(&dD, 1024);
    hipMemcpy(dA, hA, 2048, hipMemcpyHostToDevice); hipMemcpy(dB, hB, 2048, hipMemcpyHostToDevice);
    for (int mode = 0; mode < 2; ++mode) {
        hipLaunchKernelGGL(mm, dim3(1), dim3(64), 0, 0, dA, dB, dD, mode);
        float hD[256]; hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
        int bad = 0; for (int i = 0; i < 256; ++i) bad += hD[i] != ref[i];
        printf("mfma16x16x128 fp8 lane map mode %d (0: k=32*(l>>4)+j, 1: interleaved 8s): mismatches %d / 256\n", mode, bad);
    }
    float hx[128] = {1.0f, 2.0f, 0.5f, 3.0f, 448.0f, 500.0f, 1000.0f, -1000.0f, 0.001953125f, 0.0009765625f, 1e-6f, -3.0f, 240.f, 464.f, 0, 0};
    for (int i = 16; i < 128; ++i) hx[i] = 0;
    float* dx; unsigned* dy; hipMalloc(&dx, 512); hipMalloc(&dy, 256);
    hipMemcpy(dx, hx, 512, hipMemcpyHostToDevice);
    for (float s : {1.0f, 2.0f}) {
        hipLaunchKernelGGL(cvt, dim3(1), dim3(64), 0, 0, dx, dy, s);
        unsigned hy[64]; hipMemcpy(hy, dy, 256, hipMemcpyDeviceToHost);
        printf("cvt_scalef32_pk_fp8_bf16 scale %.1f:", s);
        for (int i = 0; i < 7; ++i) printf(" (%g->%02x %g->%02x)", hx[2 * i], hy[i] & 0xff, hx[2 * i + 1], hy[i] >> 8);
        printf("\n");
    }
    return 0;
}
