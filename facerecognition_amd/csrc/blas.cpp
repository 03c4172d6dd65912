// 1x1 stride-1 convolutions as plain library GEMMs (hipBLASLt), an autotuner candidate beside the hand-written
// kernels (engine.cpp tune_conv).  A 1x1 conv over NHWC activations is exactly a GEMM: Y[M x N] = X[M x K] W^T
// with M = B*H*W pixels, K = Cin, N = Cout, activations row-major with their tensors' channel strides (channel
// slices of concat tensors are leading-dimension views), the folded weights [Npad][Kpad] row-major.  Column-major
// (hipBLASLt's convention): D^T (N x M, ld Cy) = op(A) B with A = W^T (K x N, ld Kpad, transposed) and B = X^T
// (K x M, ld Cx); the epilogue is the library's: bias (f32, the folded BN shift) + ReLU, the residual as
// beta * C (C = the residual slice, ld Cres, beta = 1).  Only the f32 summation order differs from the implicit
// GEMM.  Used where it measures faster: IRV1's and ResNet-50's 1x1 convs (IResNet100 has none; its PReLU is not a
// library epilogue anyway).
#include <hipblaslt/hipblaslt.h>

#include <cstring>
#include <mutex>
#include <vector>

#include "kernels.h"

namespace fr {

namespace {

struct BlasEnt {
    const void* w;
    int M, N, K, Kpad, Cx, Cy, Cres, act, has_res, f16;
    const void* bias;
    hipblasLtMatmulDesc_t op = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, lc = nullptr, ld = nullptr;
    hipblasLtMatmulAlgo_t algo;
    bool ok = false;
};

struct BlasState {
    hipblasLtHandle_t lt = nullptr;
    void* ws = nullptr;
    size_t ws_bytes = 0;
    std::vector<BlasEnt> ents;
};

constexpr size_t WS_BYTES = 32u << 20;  // preallocated: no allocation inside a captured forward

bool same(const BlasEnt& e, const ConvArgs& a) {
    return e.w == a.w && e.M == a.M && e.N == a.Cout && e.K == a.Cin && e.Kpad == a.Kpad && e.Cx == a.Cx &&
           e.Cy == a.Cy && e.Cres == (a.res ? a.Cres : 0) && e.act == a.act && e.has_res == (a.res != nullptr) &&
           e.f16 == a.f16 && e.bias == (const void*)a.bias;
}

void destroy_ent(BlasEnt& e) {
    if (e.la) hipblasLtMatrixLayoutDestroy(e.la);
    if (e.lb) hipblasLtMatrixLayoutDestroy(e.lb);
    if (e.lc) hipblasLtMatrixLayoutDestroy(e.lc);
    if (e.ld) hipblasLtMatrixLayoutDestroy(e.ld);
    if (e.op) hipblasLtMatmulDescDestroy(e.op);
    e.la = e.lb = e.lc = e.ld = nullptr;
    e.op = nullptr;
}

// descriptors, layouts and the heuristic's first algorithm for this conv (host-side only: no device work)
bool build(BlasState& st, BlasEnt& e, const ConvArgs& a) {
    const hipDataType dt = a.f16 ? HIP_R_16F : HIP_R_16BF;
    if (hipblasLtMatmulDescCreate(&e.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return false;
    const hipblasOperation_t ta = HIPBLAS_OP_T, tb = HIPBLAS_OP_N;
    hipblasLtMatmulDescSetAttribute(e.op, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta));
    hipblasLtMatmulDescSetAttribute(e.op, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb));
    hipblasLtEpilogue_t epi = a.bias ? (a.act == 1 ? HIPBLASLT_EPILOGUE_RELU_BIAS : HIPBLASLT_EPILOGUE_BIAS)
                                     : (a.act == 1 ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT);
    hipblasLtMatmulDescSetAttribute(e.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &epi, sizeof(epi));
    if (a.bias) {
        const void* bp = a.bias;
        const int32_t bt = HIP_R_32F;
        hipblasLtMatmulDescSetAttribute(e.op, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp));
        hipblasLtMatmulDescSetAttribute(e.op, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
    }
    if (hipblasLtMatrixLayoutCreate(&e.la, dt, a.Cin, a.Cout, a.Kpad) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&e.lb, dt, a.Cin, a.M, a.Cx) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&e.lc, dt, a.Cout, a.M, a.res ? a.Cres : a.Cy) != HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutCreate(&e.ld, dt, a.Cout, a.M, a.Cy) != HIPBLAS_STATUS_SUCCESS)
        return false;
    hipblasLtMatmulPreference_t pref = nullptr;
    if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return false;
    const uint64_t wsb = st.ws_bytes;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wsb, sizeof(wsb));
    hipblasLtMatmulHeuristicResult_t res[4];
    int n = 0;
    const hipblasStatus_t hs = hipblasLtMatmulAlgoGetHeuristic(st.lt, e.op, e.la, e.lb, e.lc, e.ld, pref, 4, res, &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (hs != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS || res[0].workspaceSize > st.ws_bytes)
        return false;
    e.algo = res[0].algo;
    return true;
}

}  // namespace

bool blas_supported(const ConvArgs& a) {
    return a.Kh == 1 && a.Kw == 1 && a.sh == 1 && a.sw == 1 && a.ph == 0 && a.pw == 0 && a.H == a.Ho && a.W == a.Wo &&
           a.K == a.Cin && !a.x2 && !a.y2 && !a.partial && !a.w8 && !a.y_amax && !a.bias9 && !a.y_bf16 &&
           (a.act == 0 || a.act == 1) && a.Cin % 8 == 0 && a.Cx % 8 == 0 && a.x_off % 8 == 0 && a.Cy % 8 == 0 &&
           a.y_off % 8 == 0 && a.Cout % 8 == 0 && a.Kpad % 8 == 0 && a.M > 0 &&
           (!a.res || (a.Cres % 8 == 0 && a.res_off % 8 == 0));
}

void* blas_create() { return new BlasState(); }

void blas_destroy(void* p) {
    auto* st = (BlasState*)p;
    if (!st) return;
    for (auto& e : st->ents) destroy_ent(e);
    if (st->ws) (void)hipFree(st->ws);
    if (st->lt) hipblasLtDestroy(st->lt);
    delete st;
}

hipError_t launch_conv_blas(void* p, const ConvArgs& a, hipStream_t s) {
    auto* st = (BlasState*)p;
    if (!st || !blas_supported(a)) return hipErrorInvalidValue;
    if (!st->lt) {
        if (hipblasLtCreate(&st->lt) != HIPBLAS_STATUS_SUCCESS) return hipErrorInitializationError;
        if (hipMalloc(&st->ws, WS_BYTES) != hipSuccess) return hipErrorOutOfMemory;
        st->ws_bytes = WS_BYTES;
    }
    BlasEnt* e = nullptr;
    for (auto& x : st->ents)
        if (same(x, a)) e = &x;
    if (!e) {
        BlasEnt n{};
        n.w = a.w; n.M = a.M; n.N = a.Cout; n.K = a.Cin; n.Kpad = a.Kpad; n.Cx = a.Cx; n.Cy = a.Cy;
        n.Cres = a.res ? a.Cres : 0; n.act = a.act; n.has_res = a.res != nullptr; n.f16 = a.f16; n.bias = a.bias;
        n.ok = build(*st, n, a);
        st->ents.push_back(n);
        e = &st->ents.back();
    }
    if (!e->ok) return hipErrorNotSupported;
    const float alpha = 1.f, beta = a.res ? 1.f : 0.f;
    const bf16_t* X = a.x + a.x_off;
    bf16_t* Y = a.y + a.y_off;
    const bf16_t* C = a.res ? a.res + a.res_off : Y;
    const hipblasStatus_t hs = hipblasLtMatmul(st->lt, e->op, &alpha, a.w, e->la, X, e->lb, &beta, C, e->lc, Y, e->ld,
                                               &e->algo, st->ws, st->ws_bytes, s);
    return hs == HIPBLAS_STATUS_SUCCESS ? hipSuccess : hipErrorLaunchFailure;
}

}  // namespace fr
