// Internal launcher interface between the C-ABI/graph runner (engine.cpp) and the
// HIP kernels (conv_igemm.hip, misc.hip, match.hip).  Not part of the public ABI.
#pragma once
#include "common.h"

namespace fr {

// Conv tile variants (BM pixels x BN channels, 4 waves each).
enum { TILE_128x128 = 0, TILE_256x64 = 1, TILE_128x64 = 2, TILE_64x128 = 3,
       TILE_128x128_S3 = 4, TILE_256x128 = 5, TILE_128x256 = 6,  // *_S3 / 8-wave tiles: 3-stage DMA ring
       TILE_128x64_S3 = 8, TILE_64x128_S3 = 9, NUM_TILE_IDS = 10,     // (7 = the band kernel's id in the ABI)
       TILE_WRING = 13,    // conv_wring.hip (= FR_TILE_WRING), an autotuner candidate beside the igemm tiles
       TILE_DIRECT = 14,   // conv_direct.hip (= FR_TILE_DIRECT), the same
       TILE_64x64_S3 = 17, TILE_64x64 = 18, TILE_32x64_S3 = 19 };  // round 6: small-M GEMMs (IRV1 Block8: M = 2304) over more CUs

// Implicit-GEMM convolution, NHWC bf16 in/out, f32 accumulate, fused epilogue.
// GEMM view: M = B*Ho*Wo output pixels, N = Cout, K = Kh*Kw*Cin (c fastest).
struct ConvArgs {
    const bf16_t* x; int B, H, W, Cx, x_off, Cin;
    const bf16_t* w; int Kh, Kw, sh, sw, ph, pw, K, Kpad;
    int Ho, Wo, M, Cout, Npad;
    const float* bias; const float* slope; int act;  // act: 0 none, 1 relu, 2 prelu
    const float* bias9;           // [9][Npad] border-class bias (replaces bias; see frhip.h), or null
    const bf16_t* res; int Cres, res_off;
    bf16_t* y; int Cy, y_off;
    bf16_t* y2; int Cy2, y2_off; const float* aff_s; const float* aff_b;
    float* partial; int split_k;  // partial != null: raw f32 partials [split][M][Npad], no epilogue
    int f16;                      // 0: bf16 storage + bf16 MFMA; 1: f16 storage + f16 MFMA
    int tile;                     // TILE_* variant (conv_plan)
    void* ev0;                    // optional hipEvent_t pair stamped by the dispatch itself
    void* ev1;                    //   (hipExtLaunchKernel; fr_prof_* timing), null normally
    // fp8 path (conv_fp8.hip): e4m3 weights [Npad][Kpad] (Kpad = bytes per row, % 128), per-channel
    // scale, dynamic per-tensor amax of the input (power-of-two activation scale) and of the output
    const uint8_t* w8;
    const float* wscale;
    const float* x_amax;
    float* y_amax;                // non-null: the epilogue atomically records max |y| (both dtypes)
    int amax_slots;               // x_amax / y_amax are arrays of this many partial maxima (block % slots)
    const bf16_t* wimg;           // conv_img.hip: weights pre-packed as K-step slice images (img_pack_weights)
    const float* negf;            // conv_img / conv_rows: [Npad] activation negative-side factor (slope / 0 / 1)
    const float* ep;              // conv_rows.hip: [9][Npad] bias per border class (bias9, or bias x 9)
    const bf16_t* wrows_;         // engine: the conv's conv_rows weight image when it has one (else null)
    // K-concatenated 1x1 projection (a residual block's downsample folded into its last conv; igemm with
    // Cin % 64 == 0 only): K steps [K1, K1 + C2) read x2 [B][H2][W2][Cx2] at (oh * st2, ow * st2),
    // channels x2_off.., and the weight rows hold [W_conv | W_downsample] (bias = the sum)
    const bf16_t* x2;
    int H2, W2, Cx2, x2_off, C2, st2, K1;
    int y_bf16;                   // f16 input / MFMA, bf16 output (igemm; the end of an f16 plan section)
    const bf16_t* wring_;         // engine: the conv's conv_wring weight image when it has one (else null)
    // split-K (partial != null): per-tile arrival counters (zero between launches).  Non-null: the last of a tile's
    // split workgroups sums the partials and runs the epilogue in the same launch (no launch_splitk_epilogue)
    int* splitk_cnt;
};
// Implicit GEMM with the weights streamed from L2 into a register ring (conv_wring.hip): Cin % 64 == 0,
// Cout % 256 == 0, Kpad = K (+ the K-concatenated projection) % 128 == 0; a.wimg = the packed image.
bool wring_supported(const ConvArgs& a);
size_t wring_packed_elems(int Kpad, int Npad);
hipError_t wring_pack_weights(const bf16_t* w, int Kpad, int Npad, bf16_t* out, hipStream_t s);
hipError_t launch_conv_wring(const ConvArgs& a, hipStream_t s);
// Persistent small-K direct conv (conv_direct.hip): any Kh x Kw / stride / padding, Cin % 8 == 0, Kpad <= 384,
// Cout % 32 == 0, bias + activation epilogue only; equal to conv_igemm tile 0 bit for bit.  n_cu <= 0: queried.
bool direct_supported(const ConvArgs& a);
hipError_t launch_conv_direct(const ConvArgs& a, int n_cu, hipStream_t s);
// Persistent weight-resident 3x3/s1/p1 conv with 64 input channels (conv_rows.hip); a.wimg = the
// rows_pack_weights image, a.ep / a.negf set.
bool rows_supported(const ConvArgs& a);
size_t rows_packed_elems(int Cout);
hipError_t rows_pack_weights(const bf16_t* w, int Kpad, int Cout, bf16_t* out, hipStream_t s);
hipError_t launch_conv_rows(const ConvArgs& a, int n_cu, hipStream_t s);
// Small-M implicit GEMM (conv_small.hip): one wave per 16 pixels x 64 channels over the whole K, operands straight
// from global memory (no LDS); Cin % 32 == 0, Cout % 64 == 0; ks = 1: equal to conv_igemm tile 0 bit for bit;
// ks = 4 / 8: that many waves split each tile's K and sum through LDS (a split-K summation order).
// conv_small.hip: split = KS (waves sharing a tile's K) | NF << 8 (16-channel fragments per tile; 0 = 4)
bool small_supported(const ConvArgs& a, int nf = 4);
bool small_split_ok(int split);
hipError_t launch_conv_small(const ConvArgs& a, int split, hipStream_t s);
constexpr int FR_AMAX_SLOTS = 64;  // engine: spreads the producers' atomics over 64 addresses
// max |x| of n (% 8) bf16/f16 values into amax[0 .. slots) (misc.hip): for tensors an fp8 conv reads whose
// producer has no amax epilogue (an LDS-resident stage)
hipError_t launch_amax(const bf16_t* x, size_t n, int f16, float* amax, int slots, hipStream_t s);

// FP8 (e4m3 x e4m3, v_mfma_scale_f32_16x16x128_f8f6f4) implicit GEMM; Cin % 64 == 0.
int conv_fp8_tile(int M, int Cout);
hipError_t launch_conv_fp8(const ConvArgs& a, hipStream_t s);

// Choose tile variant and split-K factor for a GEMM of M x Cout x Kpad.
bool conv_tile_forced();
int conv_tile_candidates(int Cout, int* out);
void conv_plan(int M, int Cout, int Kpad, int* tile, int* split);
void head_plan(int M, int Cout, int Kpad, int* tile, int* split);  // the embedding head's split-K
int conv_tile_bm(int tile);
int conv_tile_bn(int tile);

// Launches a.tile with a.split_k; returns hipError_t.
hipError_t launch_conv(const ConvArgs& a, hipStream_t s);
// Row-band direct 3x3/s1/p1 conv (conv_band.hip): applicability/params, launch.
bool band_plan(const ConvArgs& a, int* cfg, int* variant);
hipError_t launch_conv_band(const ConvArgs& a, int cfg, int variant, hipStream_t s);
// Image-per-workgroup direct 3x3/s1/p1 conv for 28x28, 128 -> 128 channels (conv_img.hip).
bool img28_supported(const ConvArgs& a);
hipError_t launch_conv_img28(const ConvArgs& a, hipStream_t s);
// ... and for 56x56, 64 -> 64 channels (layer1), 4-row bands.
bool img56_supported(const ConvArgs& a);
hipError_t launch_conv_img56(const ConvArgs& a, hipStream_t s);
// Shape checks without the packed weights, their size, and the device packer ([Npad][Kpad] rows ->
// [36 or 18 K-steps][4 groups][IC rows][8 channels]).
bool img_shape_ok(const ConvArgs& a, int* ic);
size_t img_packed_elems(int ic);
hipError_t img_pack_weights(const bf16_t* w, int Kpad, int ic, bf16_t* out, hipStream_t s);
// LDS-resident stage kernel (conv_stage.hip): the stride-1 IBasicBlocks of a 14x14x256 stage, one
// workgroup per image, activation kept in LDS across all 2*nblk convs.
struct StageConv {
    const float* bias;   // [256] (null when bias9 carries the full bias)
    const float* bias9;  // [9][256] border-class bias (conv1: folded pre-conv BN), or null
    const float* slope;  // [256] PReLU slopes (act == 2), or null
    int act, pad_;
};
struct StageArgs {
    const bf16_t* x;           // stage input [B][14][14][256]
    bf16_t* y;                 // stage output [B][14][14][256] (written by the last block)
    const bf16_t* w;           // packed K-step images of all convs (stage_pack_weights)
    const StageConv* conv;     // [2*nblk] device table
    const float* ep;           // [2*nblk][9][256] epilogue bias per border class (bias9, or bias broadcast)
    const float* slope;        // [2*nblk][256] negative-side factor: PReLU slope, 0 (ReLU) or 1 (none)
    const float* wscale;       // fp8 stage (conv_stage8.hip) only: [2*nblk][256] per-channel e4m3 weight scales
    bf16_t* const* dbg_x;      // optional [nblk] per-block outputs / [nblk] conv1 outputs (device
    bf16_t* const* dbg_t;      //   pointer tables; null = do not materialise intermediates)
    // split stages (conv_split_stage.hip) only: boundary-row exchange between an image's workgroups
    bf16_t* xchg;              // [B][parts][2 rows][2 parities][W][C]
    int* flags;                // [B][parts] per-part progress (convs published), zeroed by the launcher
    int* spin_timeouts;        // bounded-wait overruns (fr_debug_stage_timeouts); 0 when healthy
    int* fail_host;            // host-mapped flag: set to 1 (plain vector store) by any part whose wait ran out
    int spin_limit;            // sleeps before a wait counts as run out; < 0: every wait runs out (debug)
    int variant;               // kernel variant (FR_OPT_STAGE_VARIANT): 0 default, 1 the legacy layout
    // layer3 stage only (conv_stage.hip stage13 kernels): ntail = 2 runs the next conv (3x3/s1 256 -> 512,
    // border-class bias + PReLU, IResNet100 layer4.0.conv1) on the final patch as two 256-channel halves,
    // weights / tables appended as convs 2 nblk and 2 nblk + 1; its output y2 [B][14][14][512]
    int ntail;
    bf16_t* y2;
    int B, nblk, f16;
    void* ev0;
    void* ev1;
};
bool stage_supported(int B, int H, int W, int C);
size_t stage_weight_bytes(int nconv);
void stage_pack_weights(const bf16_t* rows, int Kpad, int C, bf16_t* out);
hipError_t launch_stage(const StageArgs& a, hipStream_t s);
// The same stage with e4m3 weights and activations (conv_stage8.hip, BASELINE config 5): a.w = the
// stage8_pack_weights images of all convs, a.wscale their per-channel scales; the residual stays bf16.
size_t stage8_weight_bytes(int nconv);
void stage8_pack_weights(const uint8_t* rows, int Kpad8, uint8_t* out);
hipError_t launch_stage8(const StageArgs& a, hipStream_t s);
// Split LDS-resident stages (conv_split_stage.hip): 28x28x128 (IResNet100 layer2.1 .. layer2.12) in two
// workgroups per image, 56x56x64 (layer1.1 .. layer1.2) in four, 14 output rows each, exchanging their
// boundary rows per conv through xchg / flags.  split_stage_parts: workgroups per image, 0 = unsupported.
int split_stage_parts(int H, int W, int C);
size_t split_stage_weight_bytes(int C, int nconv);
void split_stage_pack_weights(const bf16_t* rows, int Kpad, int C, bf16_t* out);  // the split stages' K order
size_t split_stage_xchg_elems(int B);  // enough for either geometry
hipError_t launch_split_stage(const StageArgs& a, int H, int C, hipStream_t s);
// Fused IResNet100 transition block layer1.0 (conv_trans.hip): conv1 3x3/s1 + PReLU (t rows kept in LDS) ->
// conv2 3x3/s2 + the K-concatenated 1x1/s2 downsample + bias, one workgroup per image; x [B][112][112][64] ->
// y [B][56][56][64].  w1 / w2 = trans_pack_weights images of conv1 (K 576) and conv2 + downsample (K 640).
struct TransArgs {
    const bf16_t* x;
    bf16_t* y;
    const bf16_t* w1;
    const bf16_t* w2;
    const float* ep1;     // [9][64] conv1 bias per border class (bn1 folded)
    const float* slope1;  // [64] conv1 PReLU slopes
    const float* b2;      // [64] conv2 + downsample bias
    int B, f16;
    void* ev0;
    void* ev1;
};
bool trans_supported(int B, int H, int W, int Cin, int Cmid, int Cout, int K1, int K2);
size_t trans_packed_elems(int K);
hipError_t trans_pack_weights(const bf16_t* w, int Kpad, int K, bf16_t* out, hipStream_t s);
hipError_t launch_trans(const TransArgs& a, hipStream_t s);
// FaceNet IRV1 repeat_2 (Block17 x nblk at 8x8x896) as one launch (conv_chain.hip): one workgroup per image, the
// block input resident in LDS across all blocks; w = chain17_pack_block streams, bias = [nblk][A B C D (128 each)
// | E (896)] f32 (the member convs' folded biases: branch1.0, 1x7, 7x1, branch0, conv2d).
struct Chain17Args {
    const bf16_t* x;      // [B][8][8][896] (mixed_6a)
    bf16_t* y;            // [B][8][8][896] (the last block's output)
    const bf16_t* w;
    const float* bias;
    int B, nblk, f16;
    void* ev0;
    void* ev1;
};
bool chain17_supported(int H, int W, int C, int nblk);
size_t chain17_weight_elems(int nblk);
size_t chain17_bias_floats(int nblk);
void chain17_pack_block(const bf16_t* rA, int kpA, const bf16_t* r17, int kp17, const bf16_t* r71, int kp71,
                        const bf16_t* rE, int kpE, int blk, int nblk, bf16_t* out);
hipError_t launch_chain17(const Chain17Args& a, hipStream_t s);
// ResNet-50 layer3.1 .. layer3.5 (five Bottlenecks at 7x7x1024) as one launch, one workgroup per image
// (conv_chain_r50.hip); the args are Chain17Args' (x = layer3.0's output, y = the last block's, w =
// chain_r50_pack_block streams, bias = [nblk][conv1 256 | conv2 256 | conv3 1024] f32)
bool chain_r50_supported(int H, int W, int C, int nblk);
size_t chain_r50_weight_elems(int nblk);
size_t chain_r50_bias_floats(int nblk);
void chain_r50_pack_block(const bf16_t* r1, int kp1, const bf16_t* r2, int kp2, const bf16_t* r3, int kp3, int blk,
                          int nblk, bf16_t* out);
hipError_t launch_chain_r50(const Chain17Args& a, hipStream_t s);
// ResNet-50 layer1 Bottlenecks (28x28: 1.1 / 1.2 256 -> 64 -> 64 -> 256 + x; ds: 1.0, 64 -> 64 -> 64 -> 256 with the
// downsample K-concatenated into conv3) as one launch per block, one workgroup per image walking its rows
// (conv_bneck28.hip); Chain17Args' x / y are the block's input / output, w = its bneck28_pack_block images
// (bneck28_block_elems), bias = its [conv1 64 | conv2 64 | conv3 256] f32
bool bneck28_supported(int H, int W, int C, int P);
size_t bneck28_block_elems(bool ds);
void bneck28_pack_block(const bf16_t* r1, int kp1, const bf16_t* r2, int kp2, const bf16_t* r3, int kp3, bool ds,
                        bf16_t* out);
hipError_t launch_bneck28(const Chain17Args& a, bool ds, hipStream_t s);
// ResNet-50 stem (conv1 7x7/s2 3 -> 64 + ReLU + maxpool 3x3/s2) in one launch, one workgroup per image
// (conv_stem_r50.hip): x = the prepared [B][112][112][8] input (launch_preprocess's stem format) or u8, y = the pooled
// [B][28][28][64], w / Kpad / bias = the conv's [Npad][Kpad] rows (stem hi/lo split) and folded bias
struct StemR50Args {
    const bf16_t* x;
    const uint8_t* u8;  // u8 crops [B][112][112][3] (non-null: prepared in-kernel, x unused)
    bf16_t* y;
    const bf16_t* w;
    const float* bias;
    int Kpad, B, f16;
    void* ev0;
    void* ev1;
};
bool stem_r50_supported(int H, int W, int Cin, int K, int Kpad, int Cout);
hipError_t launch_stem_r50(const StemR50Args& a, hipStream_t s);
// FaceNet IRV1 stem at 160x160 (conv_stem160.hip): conv2d_1a (3x3/s2 8 -> 32) + conv2d_2a (3x3 32 -> 32) +
// conv2d_2b (3x3/p1 32 -> 64) + maxpool_3a (3x3/s2) + conv2d_3b (1x1 64 -> 80), each conv + bias + ReLU, as one
// launch, one workgroup per image; input: u8 crops [B][160][160][3] (u8 != null: the preparation is done in-kernel)
// or the prepared 8-channel input x [B][160][160][8]; y = conv2d_3b's [B][38][38][80]; w* = the member convs'
// [Npad][Kpad] rows (kp* = Kpad), b* their folded biases.
struct Stem160Args {
    const bf16_t* x;
    const uint8_t* u8;
    bf16_t* y;
    const bf16_t* w1; const bf16_t* w2; const bf16_t* w3; const bf16_t* w4;
    const float* b1; const float* b2; const float* b3; const float* b4;
    int kp1, kp2, kp3, kp4;
    int B, f16;
    void* ev0;
    void* ev1;
};
bool stem160_supported(int H, int W, int Cin, int K1, int K2, int K3, int K4, int C1, int C2, int C3, int C4);
hipError_t launch_stem160(const Stem160Args& a, hipStream_t s);
// FaceNet IRV1 repeat_1 (Block35 x nblk at 17x17x256) as one launch (conv_chain35.hip): one workgroup per image, the
// branch tensors in LDS, the block outputs through global memory (io[0] = the NHWC input, io[1..nblk-1] = the
// intermediate block outputs, stored plane-major [32][289][8], io[nblk] = the NHWC output); w / bias =
// chain35_pack_block / chain35_pack_bias images of the member convs.
struct Chain35Args {
    const bf16_t* io[9];
    const bf16_t* w;
    const float* bias;
    int B, nblk, f16;
    void* ev0;
    void* ev1;
};
bool chain35_supported(int H, int W, int C, int nblk);
size_t chain35_weight_elems(int nblk);
size_t chain35_bias_floats(int nblk);
void chain35_pack_block(const bf16_t* r1, int kp1, const bf16_t* r21, int kp21, const bf16_t* r22, int kp22,
                        const bf16_t* r3, int kp3, const bf16_t* r4, int kp4, int blk, bf16_t* out);
void chain35_pack_bias(const float* b1, const float* b21, const float* b22, const float* b3, const float* b4, int blk,
                       float* out);
hipError_t launch_chain35(const Chain35Args& a, hipStream_t s);
// Split-K reduction + the same fused epilogue as the conv kernel.
hipError_t launch_splitk_epilogue(const ConvArgs& a, hipStream_t s);
// Number of K-tiles of 64 (for split-k planning).
inline int conv_k_tiles(int Kpad) { return Kpad / 64; }

// Input prep: channels [q0,q1,q2,q0,q1,q2,0,0] with q = 2u-255 (u8: exact in bf16/f16) or
// q = 255*x (normalized f32).  The stem conv folds 1/255 and a hi/lo weight split into the
// duplicated channels, so x = (u/255-0.5)/0.5 enters the first conv without rounding.
hipError_t launch_preprocess(const void* in, int in_fmt, int B, int H, int W, bf16_t* out, int f16, hipStream_t s);
// Fused u8 preprocess + IResNet stem conv (conv_stem.hip).
bool stem_u8_supported(int H, int W, int Cin, int K, int Kpad, int Cout, int Cy, int y_off);
hipError_t launch_stem_u8(const uint8_t* in, int B, const bf16_t* w, int Kpad, const float* bias, const float* slope,
                          int act, bf16_t* y, int Cy, int y_off, int f16, hipStream_t s);
// y_bf16: f16 input, bf16 output (3x3 only: the end of an f16 plan section)
hipError_t launch_maxpool(const bf16_t* x, int B, int H, int W, int Cx, int x_off, int C, int k, int stride,
                          int pad, bf16_t* y, int Cy, int y_off, int Ho, int Wo, int f16, hipStream_t s, int y_bf16 = 0);
hipError_t launch_avgpool(const bf16_t* x, int B, int H, int W, int C, bf16_t* y, int f16, hipStream_t s);
// Sum split-K partials [split][B][Npad] + bias, optional L2 normalize → out [B][N] f32.
bool head_gemv_supported(int B, int K, int Kpad, int Npad);
hipError_t launch_head_gemv(const bf16_t* x, int B, int K, const bf16_t* w, int Kpad, int N, int Npad, int S, int f16,
                            float* partial, hipStream_t s);
hipError_t launch_head_finalize(const float* partial, int split, int B, int N, int Npad, const float* bias,
                                int normalize, float* out, hipStream_t s);
// FaceNet projection: out = x W^T + bias (f32), optional F.normalize (eps 1e-12).  K <= 1024.
hipError_t launch_proj_l2(const float* x, int B, int K, const float* W, const float* bias, int N, int normalize,
                          float* out, hipStream_t s);
// Row-wise L2 normalize in place (F.normalize, eps 1e-12).
hipError_t launch_l2norm_rows(float* x, int B, int D, hipStream_t s);

// Gallery match.
hipError_t launch_match_topk(const float* P, int B, const float* G, int64_t N, int D, int k,
                             int64_t index_base, float* cand_s, int32_t* cand_i, int n_split,
                             int64_t rows_per_split, hipStream_t s);
hipError_t launch_topk_merge(const float* cs, const int32_t* ci, int B, int n_lists, int k, float* out_s,
                             int32_t* out_i, hipStream_t s);
// The same merge over the all-gathered exchange block [n_ranks][2][B][k] (scores f32, then indices i32).
hipError_t launch_topk_merge_ranks(const void* xchg, int n_ranks, int B, int k, float* out_s, int32_t* out_i,
                                   hipStream_t s);
// k > 16 (match.hip): exact score rows S [B][N] (the caller's scratch) + a per-probe radix select.
constexpr int FR_TOPK_LARGE_MAX = 4096;
hipError_t launch_match_topk_large(const float* P, int B, const float* G, int64_t N, int D, int k, int64_t index_base,
                                   float* S, float* out_s, int32_t* out_i, hipStream_t s);
// Large-gallery match (match_x3.hip): bf16x3 candidates, exact f32 rescoring with a proof / fallback.
constexpr int64_t X3_MIN_ROWS = 32768;  // below: the exact f32 kernel is as fast (10k x 256: 0.105 vs 0.16 ms)
// bf16 hi/lo copy of gallery rows [row0, row0 + n) of G (f32 [rows][512]) into the candidate pass's
// chunk-ordered buffer T of x3_gallery_elems(capacity) bf16 (match_x3.hip)
size_t x3_gallery_elems(int64_t rows);
hipError_t launch_split_x3(const float* G, int64_t row0, int64_t n, bf16_t* T, hipStream_t s);
void match_x3_plan(int B, int64_t N, int* n_split, int64_t* rows_per_split);
bool match_rows_supported(int B, int D, int k);
void match_rows_plan(int64_t N, int* n_lists, int* R);
hipError_t launch_match_rows(const float* P, int B, const float* G, int64_t N, int D, int k, int64_t index_base,
                             float* cand_s, int32_t* cand_i, int n_lists, int R, hipStream_t s);
int match_x3_candidates();
hipError_t launch_match_x3(const float* P, int B, const float* G, const bf16_t* GT, int64_t N, int D,
                           int k, int64_t index_base, float* cand_s, int32_t* cand_i, int n_split,
                           int64_t rows_per_split, float* out_s, int32_t* out_i, int* n_fallback, hipStream_t s);
// Choose n_split / rows_per_split for a (B, N) match.
void match_split_plan(int B, int64_t N, int* n_split, int64_t* rows_per_split);
void match_split_plan(int B, int64_t N, int D, int k, int* n_split, int64_t* rows_per_split);  // exact path
hipError_t launch_segment_mean_normalize(const float* E, int D, const int32_t* seg_start, int n_seg,
                                         float* out, hipStream_t s);
// Gallery preparation: rows with |‖g‖-1| >= 1e-3 divided by ‖g‖ (cosine_similarity semantics).
hipError_t launch_gallery_prepare(float* G, int64_t N, int D, hipStream_t s);
// Crop preparation (preprocess.hip): Pillow-exact bilinear resize, cv2-exact affine warp (u8 RGB NHWC).
size_t resize_u8_workspace(int B, int H, int W, int OH, int OW);
hipError_t launch_resize_u8(const uint8_t* in, int B, int H, int W, uint8_t* out, int OH, int OW, void* ws,
                            hipStream_t s);
hipError_t launch_warp_affine_u8(const uint8_t* in, int B, int H, int W, const double* M, uint8_t* out, int OH, int OW,
                                 hipStream_t s);

// MTCNN face-detector building blocks (mtcnn.hip): f32 NHWC.
hipError_t launch_area_resample(const uint8_t* img, int H, int W, const int32_t* regions, int n, int oh, int ow,
                                float* out, hipStream_t s);
hipError_t launch_mtcnn_conv(const float* x, int B, int H, int W, int Cin, const float* w, const float* bias,
                             const float* slope, int Cout, int kh, int kw, float* y, hipStream_t s);
hipError_t launch_mtcnn_maxpool(const float* x, int B, int H, int W, int C, int k, int st, int Ho, int Wo, float* y,
                                hipStream_t s);
hipError_t launch_mtcnn_dense(const float* x, int B, int K, const float* w, const float* bias, const float* slope,
                              int N, float* y, hipStream_t s);
hipError_t launch_mtcnn_head(const float* x, int64_t M, int C, const float* w, const float* bias, int NO, float* out,
                             hipStream_t s);
int pool_ceil_out(int H, int k, int s);

}  // namespace fr
