/*
 * frhip.h — C ABI of the MI355X-native face-embedding + gallery-match path.
 *
 * This is the drop-in boundary for the hot path of sin0235/FaceRecognition
 * (SURVEY.md §8a/§8b).  The reference has no FFI layer: its boundary is the
 * Python call `model(x, labels=None)` / `model(x)` plus the match loops.
 * Each entry point below names the reference interface it replaces
 * (paths relative to the reference root).  Plain C types only: device
 * buffers are passed as raw pointers (e.g. torch `tensor.data_ptr()`),
 * streams as `void*` (a hipStream_t, e.g. torch `current_stream().cuda_stream`),
 * and every function returns FR_OK (0) or a negative FR_ERR_* code with a
 * thread-local message in fr_last_error().
 */
#ifndef FRHIP_H
#define FRHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FR_ABI_VERSION 1

/* ---- status codes (reference error convention: SURVEY.md §8b row "Error convention") ---- */
#define FR_OK 0
#define FR_ERR_ARG (-1)     /* bad argument / unsupported shape              */
#define FR_ERR_HIP (-2)     /* a HIP runtime call failed                      */
#define FR_ERR_WEIGHTS (-3) /* weight blob malformed or tensor missing        */
#define FR_ERR_STATE (-4)   /* call order violated (no weights, no gallery)   */
#define FR_ERR_OOM (-5)     /* device allocation failed                       */
#define FR_ERR_STAGE (-6)   /* a split stage's bounded halo wait ran out in an FR_EMBED_ASYNC forward:
                             * that forward's affected embeddings are NaN (see fr_sync_check)   */

/* ---- backbone architectures ---- */
#define FR_ARCH_RESNET50_ARCFACE 0 /* models/arcface/arcface_model.py:65-202 (ArcFaceModel, ResNet-50 trunk) */
#define FR_ARCH_IRESNET100 1       /* insightface iresnet100 (README.md:72 only; no reference code)         */
#define FR_ARCH_IRV1_FACENET 2     /* models/facenet/facenet_model.py:7-36 (facenet_pytorch InceptionResnetV1) */

/* ---- compute dtypes ---- */
#define FR_DTYPE_BF16 0 /* bf16 activations/weights, f32 accumulate (v_mfma_f32_16x16x32_bf16) */
#define FR_DTYPE_FP8 2  /* BASELINE config 5: e4m3 weights (per-output-channel scale) x e4m3 activations
                         * (dynamic per-tensor power-of-two scale) on v_mfma_scale_f32_16x16x128_f8f6f4,
                         * f32 accumulate; activations stay bf16 in memory (residual stream at bf16);
                         * the stem and the 25088->512 head stay bf16.  Weight blob convs carrying
                         * "<name>.wscale" run fp8 (values in "<name>.w" must be e4m3-representable). */
#define FR_DTYPE_F16 1  /* f16 activations/weights, f32 accumulate (v_mfma_f32_16x16x32_f16): same MFMA
                           rate, 3 more mantissa bits; stores saturate at +-65504 */

/* ---- input formats accepted by fr_embed ---- */
#define FR_IN_U8_NHWC 0  /* aligned crops, u8 [B,H,W,3] RGB; ToTensor+Normalize(0.5,0.5) fused (extract_embeddings.py:170-185) */
#define FR_IN_F32_NCHW 1 /* already-normalized f32 [B,3,H,W], i.e. the output of get_transform()                             */

/* ---- fr_embed flags ---- */
#define FR_EMBED_RAW 1 /* return the un-normalized head output (= model(x, labels=None)); default is F.normalize'd */
/* Return as soon as the forward is enqueued.  Without this flag, a forward that runs an IResNet100 split
 * stage (layer1 / layer2: several workgroups per image waiting for each other's boundary rows, bounded)
 * is waited for before fr_embed returns, and if any of those waits ran out the forward is run again on
 * the per-conv path (no waits), so the returned embeddings are always valid (fr_debug_stage_reruns counts
 * the re-runs).  With it, a part whose wait ran out writes NaN into its image's activations (the
 * embedding is NaN, never a plausible wrong vector) and the handle latches FR_ERR_STAGE, returned once by
 * fr_sync_check or by the next fr_embed / fr_embed_match on the handle. */
#define FR_EMBED_ASYNC 2

typedef struct fr_handle fr_handle;

/* Thread-local message describing the last failure on this thread ("" if none). */
const char* fr_last_error(void);
int fr_abi_version(void);

/* Create a handle bound to HIP device `device`.
 * Replaces: ArcFaceModel(...)/FaceNetModel(...) construction in
 * load_arcface_model (inference/extract_embeddings.py:80-123) and
 * load_facenet_model (:126-167). */
int fr_create(fr_handle** out, int device, int arch, int dtype);
void fr_destroy(fr_handle* h);

/* Load BN-folded weights (FRW1 blob written by facerecognition_amd/weights.py).
 * Replaces: model.load_state_dict(checkpoint['model_state_dict'])
 * (inference/extract_embeddings.py:104-106, :150-153). */
int fr_load_weights(fr_handle* h, const void* blob, size_t nbytes);

/* Pre-allocate activation workspace for batches up to max_batch (no allocation
 * happens inside fr_embed once reserved, so it can be stream-captured). */
int fr_reserve(fr_handle* h, int max_batch);

/* Embedding dimension (512) and the square input side the arch expects (112/160). */
int fr_embed_dim(const fr_handle* h);
int fr_input_size(const fr_handle* h);

/* Forward pass: `in` (device) → `out` (device f32 [B, embed_dim]).
 * Replaces: `model(x, labels=None)` + `F.normalize(p=2, dim=1)` in
 * extract_embedding_single (inference/extract_embeddings.py:377-382) and
 * extract_embeddings_batch (:430-435); FaceNetModel.forward (facenet_model.py:28-36). */
int fr_embed(fr_handle* h, const void* in, int in_fmt, int B, int H, int W,
             float* out, int flags, void* stream);

/* Synchronize `stream`, then report (once) a split-stage wait that ran out in an FR_EMBED_ASYNC forward
 * of this handle since the last report: FR_ERR_STAGE, else FR_OK. */
int fr_sync_check(fr_handle* h, void* stream);

/* ---- gallery + match (replaces RecognitionEngine.recognize_with_db's loop,
 *      recognition_engine.py:267-289, the notebook np.dot+argmax/argsort,
 *      evaluate_arcface_kaggle.ipynb cells 15-16, and faiss IndexFlatIP.search,
 *      recognition_engine.py:291-326) ---- */

/* Install gallery rows G [N, D] f32 (host or device memory).  Rows whose L2
 * norm differs from 1 by >= 1e-3 are divided by their norm so that the stored
 * dot product equals cosine_similarity (recognition_engine.py:41-63); zero rows
 * stay zero (score 0.0).  `index_base` is added to every returned index (gallery
 * sharding: rank r passes the global row of its first shard row). */
int fr_gallery_set(fr_handle* h, const float* G, int64_t N, int D, int64_t index_base, int g_on_device);
int64_t fr_gallery_rows(const fr_handle* h);

/* Write rows [row0, row0 + n) of the gallery from G [n, D] (host or device): an in-place update of
 * existing rows and/or a contiguous append (row0 <= fr_gallery_rows).  Only the written rows are
 * prepared as in fr_gallery_set (and split for the bf16x3 path); appends grow the allocation
 * geometrically.  Replaces the rebuild-per-edit of the reference's dict db / IndexFlatIP.add
 * (recognition_engine.py:406-418 add_to_db; extract_embeddings.py:625-632). */
int fr_gallery_write(fr_handle* h, const float* G, int64_t row0, int64_t n, int D, int g_on_device);

/* Top-k of P [B, D] (device f32, L2-normalized probes) against the gallery.
 * Results (device): scores [B, k] f32 descending, idx [B, k] int32; ties are
 * broken by lower index (stable sort(reverse=True) / np.argmax semantics).
 * Rows past the gallery end come back as score -inf, idx -1.  1 <= k <= 4096 (faiss
 * IndexFlatIP.search takes any k, recognition_engine.py:291,304): k <= 16 keeps register
 * top-k lists; larger k materialises the exact score rows in stream-ordered scratch
 * (<= 256 MiB per probe chunk) and radix-selects per probe -- the same scores bit for bit,
 * so a large-k list starts with the small-k list.  k > 16 needs N < 2^31. */
int fr_match_topk(fr_handle* h, const float* P, int B, int k, float* scores, int32_t* idx, void* stream);

/* Merge n_lists candidate lists per probe: cand_s/cand_i [B, n_lists, k] → [B, k]
 * with the same (score desc, index asc) order.  Used after the RCCL all-gather of
 * per-shard candidates. */
int fr_topk_merge(const float* cand_s, const int32_t* cand_i, int B, int n_lists, int k,
                  float* scores, int32_t* idx, void* stream);

/* The same merge over the multi-GPU candidate exchange block as all-gathered (SURVEY.md §8e step
 * 3-4, one collective): xchg = [n_ranks][2][B][k] 4-byte words, rank r's block holding its shard's
 * top-k scores (f32 [B][k]) followed by their global indices (int32 [B][k]).  Each rank writes its
 * block with fr_match_topk straight into the send buffer; the all-gather output is merged as is
 * (no repacking, no permute).  Replaces the per-shard exchange the reference does not have
 * (single-process recognize_with_db / IndexFlatIP.search, recognition_engine.py:267-326). */
int fr_topk_merge_ranks(const void* xchg, int n_ranks, int B, int k, float* scores, int32_t* idx,
                        void* stream);

/* Fused convenience: fr_embed (normalized) then fr_match_topk on the same stream. */
int fr_embed_match(fr_handle* h, const void* in, int in_fmt, int B, int H, int W, int k,
                   float* emb_out, float* scores, int32_t* idx, void* stream);

/* Segmented mean + renormalize (gallery construction: extract_embedding_for_folder
 * inference/extract_embeddings.py:755-760, compute_prototypes :555-592,
 * RecognitionEngine.add_to_db recognition_engine.py:411-413):
 * out[s] = m / (||m|| + 1e-8), m = mean of E[seg_start[s] .. seg_start[s+1]) (device). */
int fr_segment_mean_normalize(const float* E, int D, const int32_t* seg_start, int n_seg,
                              float* out, void* stream);

/* ---- crop preparation on the device (u8 RGB NHWC in and out) ---- */

/* Bytes of device workspace fr_resize_u8 needs for this shape (0 when the width is unchanged). */
size_t fr_resize_u8_workspace(int B, int H, int W, int OH, int OW);
/* Replaces: PIL Image.resize((OW, OH), Image.BILINEAR) inside get_transform / get_facenet_transform's
 * Resize (inference/extract_embeddings.py:170-185): Pillow's two-pass antialiased bilinear resampler,
 * bit-exact (coefficients in double as Pillow, 22-bit fixed point, horizontal pass first).  in: device
 * [B,H,W,3] u8; out: device [B,OH,OW,3] u8; ws: device workspace of fr_resize_u8_workspace bytes. */
int fr_resize_u8(const uint8_t* in, int B, int H, int W, uint8_t* out, int OH, int OW, void* ws, size_t ws_bytes,
                 void* stream);
/* Replaces: cv2.warpAffine(image, M, (OW, OH), borderValue=0) of align_face (extract_embeddings.py:216-242,
 * recognition_engine.py:169-204; INTER_LINEAR, BORDER_CONSTANT 0), restating OpenCV's fixed-point path
 * (1/32-pixel grid, 15-bit weights).  M: device [B][2][3] float64, the FORWARD source->destination matrices
 * (SimilarityTransform(src landmarks -> ARCFACE_TEMPLATE).params[:2], as the reference passes them). */
int fr_warp_affine_u8(const uint8_t* in, int B, int H, int W, const double* M, uint8_t* out, int OH, int OW,
                      void* stream);

/* ---- face detection before the path: the building blocks of the device MTCNN
 *      (facerecognition_amd/face_detector.py), replacing facenet-pytorch's MTCNN behind
 *      FaceDetector._detect_mtcnn (preprocessing/face_detector.py:78-97, 144-210).  f32 NHWC tensors. ---- */

/* F.interpolate(mode='area') of u8 RGB regions + (x - 127.5) * 0.0078125 (detect_face's imresample and
 * normalisation): regions (device int32 [n][5]) = image index, y0, x0, h, w inside img [*, H, W, 3];
 * out (device f32) [n, oh, ow, 3].  Bit-identical to torch's CPU adaptive average pooling. */
int fr_area_resample_u8(const uint8_t* img, int H, int W, const int32_t* regions, int n, int oh, int ow, float* out,
                        void* stream);
/* Valid (unpadded) stride-1 conv, weights [Cout][kh][kw][Cin], + bias, then PReLU when slope != NULL. */
int fr_mtcnn_conv(const float* x, int B, int H, int W, int Cin, const float* w, const float* bias, const float* slope,
                  int Cout, int kh, int kw, float* y, void* stream);
/* MaxPool2d(k, stride, ceil_mode=True): y [B, Ho, Wo, C] with Ho = ceil((H - k) / stride) + 1 (torch's rule). */
int fr_mtcnn_maxpool(const float* x, int B, int H, int W, int C, int k, int stride, float* y, void* stream);
/* Linear: y [B, N] = x [B, K] . w [N, K]^T + bias, then PReLU when slope != NULL. */
int fr_mtcnn_dense(const float* x, int B, int K, const float* w, const float* bias, const float* slope, int N, float* y,
                   void* stream);
/* Net heads: out [M, n_out] = x [M, C] . w [n_out, C]^T + bias, columns 0-1 replaced by their softmax
 * (face probability in column 1), the rest raw (box regression, landmarks). */
int fr_mtcnn_head(const float* x, int64_t M, int C, const float* w, const float* bias, int n_out, float* out,
                  void* stream);

/* Greedy NMS on the host (detect_face's batched_nms / batched_nms_numpy): boxes [n][4] (x1, y1, x2, y2) float32,
 * order = the candidates' score order; a box is dropped when a kept box earlier in the order overlaps it with
 * IoU > thresh (min_mode = 0: torchvision's areas and test, a 0 / 0 IoU keeps) or unless intersection / min
 * area <= thresh (min_mode = 1: nms_numpy's 'Min', +1-pixel extents), float32 arithmetic as numpy's.  keep [n] receives the kept indices in
 * order, *n_keep their count.  Grid-bucketed: O(n) for boxes of bounded size. */
int fr_nms_host(const float* boxes, int64_t n, const int64_t* order, float thresh, int min_mode, int64_t* keep,
                int64_t* n_keep);

/* ---- op-level entry points (kernel parity tests and custom graphs) ---- */

/* Implicit-GEMM convolution on NHWC bf16 with fused epilogue:
 *   y = act( conv(x, w) + bias + res )   written to y[..., y_off : y_off+Cout]
 *   y2 = y * aff_s + aff_b                (optional second output, bf16)
 * Weights: bf16 [Npad][Kpad], row n = output channel, K ordered (r, s, c) with
 * c fastest (KRSC), zero padded; Npad % 128 == 0, Kpad % 64 == 0.
 * Requirements: Cin % 8 == 0, Cx/x_off/Cy/y_off/Cres/res_off % 8 == 0, Cout % 8 == 0. */
typedef struct fr_conv_desc {
    const void* x; int B, H, W, Cx, x_off, Cin;  /* input tensor [B,H,W,Cx], channels [x_off, x_off+Cin) */
    const void* w; int Cout, Kh, Kw, stride_h, stride_w, pad_h, pad_w, Npad, Kpad;
    const float* bias;   /* [Cout] or NULL */
    int act;             /* 0 none, 1 relu, 2 prelu (slope) */
    const float* slope;  /* [Cout] for prelu */
    const void* res; int Cres, res_off; /* residual [B,Ho,Wo,Cres] bf16 or NULL */
    void* y; int Cy, y_off;             /* output [B,Ho,Wo,Cy] bf16 */
    void* y2; int Cy2, y2_off; const float* aff_s; const float* aff_b; /* optional */
    int Ho, Wo;          /* filled by fr_conv_out_shape if 0 */
    int split_k;         /* 0/1 = fused epilogue; >1 = f32 partials into `partial` then reduce */
    float* partial;      /* workspace [split_k, B*Ho*Wo, Npad] f32 when split_k > 1 */
    int dtype;           /* FR_DTYPE_BF16 / FR_DTYPE_F16: element type of x, w, res, y, y2 */
    int tile;            /* 0 = automatic (cost model); 1 + FR_TILE_* forces a tile variant */
    /* Border-class bias for a 3x3 / stride 1 / pad 1 conv whose input BN was folded into the weights
     * (the BN shift meets the zero padding only at the image border): [9][Npad] f32, class
     * 3*rc + cc with rc = 0 / 1 / 2 for output row 0 / interior / Ho-1 (cc likewise for columns).
     * When set it replaces `bias`.  NULL otherwise. */
    const float* bias9;
    /* dtype == FR_DTYPE_FP8: w is e4m3 bytes [Npad][Kpad] (Kpad % 128 == 0, Cin % 64 == 0), wscale [Npad]
     * per-output-channel f32 scales, x_amax -> the input's max |x| (device f32; the activation scale is
     * the power of two 2^e with max|x| / 2^e <= 448); x, res, y, y2 are bf16.  y_amax (any dtype, may
     * be NULL): the epilogue atomically raises it to max |y| of what it stores (caller zeroes it). */
    const float* wscale;
    const float* x_amax;
    float* y_amax;
} fr_conv_desc;

/* conv tile variants (pixels x channels per 256-thread block) */
#define FR_TILE_128x128 0
#define FR_TILE_256x64 1
#define FR_TILE_128x64 2
#define FR_TILE_64x128 3
#define FR_TILE_128x128_S3 4 /* 3-stage DMA ring, 1 block/CU */
#define FR_TILE_256x128 5    /* 8 waves, 3-stage ring */
#define FR_TILE_128x256 6    /* 8 waves, 3-stage ring */
#define FR_TILE_BAND 7       /* row-band direct 3x3/s1/p1 kernel (conv_band.hip); auto-selected when applicable */
#define FR_TILE_128x64_S3 8  /* 3-stage DMA ring, 2 blocks/CU */
#define FR_TILE_64x128_S3 9  /* 3-stage DMA ring, 2 blocks/CU */
#define FR_TILE_IMG56 11     /* the same for 56x56x64->64 (layer1), 4-row bands */
#define FR_TILE_IMG28 10     /* row-band direct 3x3/s1/p1 28x28x128->128 bf16 kernel (conv_img.hip); auto-selected (FR_AB no_img28: off) */
#define FR_TILE_ROWS 12      /* persistent weight-resident 3x3/s1/p1 kernel for Cin = 64, Cout % 64 == 0, W % 56 == 0,
                              * H % 4 == 0, bf16 (conv_rows.hip); auto-selected (FR_AB no_rows: off) */
#define FR_TILE_WRING 13     /* implicit GEMM with a register weight ring (conv_wring.hip): Cin % 64 == 0, Cout % 256 == 0;
                                autotuned per shape against the igemm tiles (FR_AB no_wring: off) */
#define FR_TILE_DIRECT 14    /* persistent small-K direct conv (conv_direct.hip): Cin % 8 == 0, Kpad <= 384, Cout % 32 == 0,
                                bias + activation epilogue; autotuned per shape (FR_AB no_direct: off) */
/* 15: retired (round 5; a hipBLASLt candidate that never won a whole forward) */
#define FR_TILE_64x64_S3 17  /* 3-stage DMA ring, 64 x 64 tiles (round 6: small-M GEMMs over more CUs) */
#define FR_TILE_64x64 18
#define FR_TILE_32x64_S3 19
#define FR_TILE_SMALL 16     /* small-M implicit GEMM, one wave per 16 px x 64 ch over the whole K (conv_small.hip); bit-identical to tile 0.
                                split_k = KS | NF << 8: KS (4 / 8 / 16) waves share a tile's K (split-K summation order), NF
                                (2 / 1; 0 = 4) 16-channel fragments per tile: 1, 4, 8, 1|2<<8, 4|2<<8, 8|2<<8, 1|1<<8, 4|1<<8,
                                8|1<<8, 16|1<<8 */

int fr_op_conv2d(const fr_conv_desc* d, void* stream);

/* u8 NHWC [B,H,W,3] or f32 NCHW [B,3,H,W] → 16-bit NHWC [B,H,W,8] = [q0,q1,q2,q0,q1,q2,0,0] with
 * q = 2u-255 (u8; exact) or q = 255*x (normalized f32), i.e. q = 255 * ((u/255-0.5)/0.5).  The stem
 * conv weights carry 1/255 as a hi/lo pair on the duplicated channels (exact first layer). */
int fr_op_preprocess(const void* in, int in_fmt, int B, int H, int W, void* out, int dtype, void* stream);

/* Max pool NHWC bf16 (padding never wins, as torch MaxPool2d). */
int fr_op_maxpool(const void* x, int B, int H, int W, int Cx, int x_off, int C,
                  int k, int stride, int pad, void* y, int Cy, int y_off, int Ho, int Wo, int dtype, void* stream);

/* Global average pool NHWC bf16 [B,H,W,C] → bf16 [B,C]. */
int fr_op_avgpool(const void* x, int B, int H, int W, int C, void* y, int dtype, void* stream);

/* Linear head: out[B,N] = x[B,K] (bf16) · w[Npad,Kpad]ᵀ (bf16) + bias, f32 out, optional L2
 * normalize (F.normalize eps 1e-12).  `partial` must hold split_k*B*Npad floats. */
int fr_op_linear(const void* x, int B, int K, const void* w, int N, int Npad, int Kpad,
                 const float* bias, int normalize, float* out, int split_k, float* partial, int dtype, void* stream);

/* ---- execution options (no reference counterpart: plan choices of this build) ----------------
 * FR_OPT_STAGE (default 1; FR_AB no_stage starts at 0): run the stride-1 IResNet100 layer3 blocks
 *   as one LDS-resident stage kernel per image instead of 58 separate conv launches.  Numerically the
 *   same op sequence and bf16 rounding points (f32 accumulation in a different K order).  0 = never,
 *   1 = auto: at every batch of at most one image per CU (measured faster than the per-conv launches
 *   down to B = 1), and above that only when the rounds of one image per CU are at least
 *   FR_OPT_STAGE_MIN_FILL percent full (B = 257 on 256 CUs takes the per-conv launches), 2 = always.
 * FR_OPT_STAGE_MIN_FILL (default 80): the auto threshold above, in percent.
 * FR_OPT_KEEP_INTERMEDIATES (default 0): the stage kernel also writes every block output and conv1
 *   output to its named tensor (per-layer drift tests; costs HBM writes).
 * Changing an option drops the captured hipGraph replays.  fr_get_option returns the value (FR_OPT_STAGE
 * reads 0 when the plan has no stage) or FR_ERR_ARG. */
#define FR_OPT_STAGE 1
#define FR_OPT_KEEP_INTERMEDIATES 2
/* FR_OPT_MATCH_EXACT (default 0): galleries of >= FR_OPT_X3_MIN_ROWS rows (D = 512) are matched by a bf16x3 candidate
 * pass (|error| <= 1.25e-4 ||p||) plus exact f32 rescoring of the top-16 candidates per probe, with a
 * per-probe proof that no excluded row can enter the top-k (else an exact rescan of that probe): the
 * results equal the exact f32 kernel's.  1 forces the f32-MFMA kernel for every gallery. */
#define FR_OPT_MATCH_EXACT 3
/* FR_OPT_X3_MIN_ROWS (default 32768): smallest gallery given the bf16x3 path (its hi/lo copy is made by
 * the next fr_gallery_set); below it the f32 kernel is as fast. */
#define FR_OPT_X3_MIN_ROWS 4
#define FR_OPT_STAGE_MIN_FILL 5
/* FR_OPT_STAGE_SPIN_LIMIT (default 0 = the kernel's bound, ~0.1 s): sleeps (64 cycles each) a split-stage
 * part waits for a neighbour's boundary rows before the wait counts as run out.  < 0 makes every wait
 * run out at once (debug: exercises the NaN poisoning, the re-run and FR_ERR_STAGE deterministically). */
#define FR_OPT_STAGE_SPIN_LIMIT 6
/* FR_OPT_STAGE_VARIANT (default 0): the layer3 stage kernel's pixel layout -- 0: 13 fragments of 16 pixels
 * per image (196 of 208 slots used), 1: the legacy 14 rows of 16 positions (2 halo columns computed and
 * discarded per row), 2: the 13-fragment layout at one wave per SIMD (each weight fragment loaded once per
 * CU), 3: 8 waves split by output channel (32 each) over all 13 fragments (each weight fragment loaded once
 * per CU, twice the patch reads).  All give the same bits (A/B and regression tests). */
#define FR_OPT_STAGE_VARIANT 7
/* FR_OPT_SPLITK_INLAUNCH (default 1; FR_AB splitk_inlaunch=0 starts at 0): a split-K implicit-GEMM conv may reduce
 * its partials in the same launch (the last workgroup of each tile sums them in split order) where the
 * per-shape tuning measured that faster than a second launch; 0 = always the second launch.  The same bits
 * either way.  fr_debug_plan prints an in-launch split as a negative split count. */
#define FR_OPT_SPLITK_INLAUNCH 8
/* FR_OPT_BATCH_INVARIANT (default 0): batch-size-independent embeddings.  Every conv runs a kernel that sums K in
 * the implicit GEMM's order (igemm tiles, register-ring, direct and small-M kernels unsplit; no split-K, no LDS-resident
 * stage / transition / block kernels) and the head uses bs = 256's split plan at every batch, so a face's embedding
 * is the same bits whatever batch it is in (the reference's recognize_batch is a loop over recognize,
 * recognition_engine.py:383-389).  Slower than the default, which measures the fastest kernels per batch size.
 * FR_DTYPE_FP8 handles refuse value 1 (FR_ERR_ARG): their e4m3 convs scale activations by a per-batch amax. */
#define FR_OPT_BATCH_INVARIANT 9
/* FR_OPT_FUSED_MASK (default 127): which kinds of fused multi-conv kernels a forward may run (each still measured
 * against its member convs per batch size under FR_OPT_STAGE 1): bit 0 the IResNet100 LDS-resident stages and the
 * fused layer1.0 transition, bit 1 the IRV1 stem (conv_stem160.hip), bit 2 IRV1 repeat_1 (conv_chain35.hip), bit 3
 * IRV1 repeat_2 (conv_chain.hip), bit 4 ResNet-50 layer3.1-3.5 (conv_chain_r50.hip), bit 5 ResNet-50 layer1.0-1.2
 * (conv_bneck28.hip), bit 6 the ResNet-50 stem conv + max-pool (conv_stem_r50.hip).  For A/B timing and for tests
 * that check one fused kernel against its members. */
#define FR_OPT_FUSED_MASK 10
int fr_set_option(fr_handle* h, int option, int value);
int fr_get_option(const fr_handle* h, int option);
/* Number of probes (since the gallery was first split) whose bf16x3 candidate proof failed and were
 * rescanned exactly (synchronizes the device). */
int fr_debug_match_fallbacks(fr_handle* h);
/* Number of bounded waits of the split stage kernels (layer2: two workgroups per image, layer1: four,
 * exchanging boundary rows per conv) that ran out before the partner published; 0 on a healthy device
 * (synchronizes the device).  Each one was either re-run (fr_embed's default) or reported as
 * FR_ERR_STAGE with NaN embeddings (FR_EMBED_ASYNC): never returned as a valid embedding. */
int fr_debug_stage_timeouts(fr_handle* h);
/* Number of forwards fr_embed ran again on the per-conv path because a split-stage wait ran out. */
int fr_debug_stage_reruns(fr_handle* h);

/* ---- debug: named intermediate tensors of the forward plan (per-layer drift tests) ----
 * Tensor names are the reference/oracle module whose output the tensor equals
 * (e.g. "backbone.layer2.0", "layer3.7.prelu", "model.repeat_1.2"); "" for internal buffers. */
/* ---- measurement: per-kernel-class timing with HIP events (bench.py roofline) --------------
 * No reference counterpart (the reference has no profiler hook); used by bench.py to time the
 * dominant kernel live, on the stream it is launched on.  fr_prof_enable(h, n) (n >= 1) resets and
 * starts recording an event pair around every n-th launch of fr_embed (conv launches are stamped by
 * their dispatch via hipExtLaunchKernel; n > 1 samples to keep the overhead small); n = 0 stops.
 * Profiled forwards launch eagerly (no hipGraph replay).  fr_prof_collect() waits for the pending
 * events and returns the number of kernel classes; fr_prof_get() reads class i: name (matches the
 * kernel instantiation), summed milliseconds, launch count, summed algorithmic FLOPs (2*M*N*K). */
int fr_prof_enable(fr_handle* h, int on);
/* Restrict timing to one kernel class (name as returned by fr_prof_get; NULL or "" = all).
 * Each event pair serializes the stream slightly, so bench.py times only the dominant class. */
int fr_prof_only(fr_handle* h, const char* kernel_class);
int fr_prof_collect(fr_handle* h);
/* Graph-slot timing (bench.py's timed steps, which replay hipGraphs like the product path):
 * fr_prof_slots(h, class, n) makes n event pairs (n = 0 frees them); with slot i selected
 * (fr_prof_slot_select, -1 = none) a forward records pair i around launch i mod L of `class` (L = the
 * class's launches per forward, counted by the first slot forward) -- captured into slot i's own graph, so
 * every replay of that graph re-stamps the pair on the launching stream; fr_prof_slot_ms reads pair i
 * (milliseconds between the two events), fr_prof_slot_work the timed launch's algorithmic FLOPs and bytes. */
int fr_prof_slots(fr_handle* h, const char* kernel_class, int n);
int fr_prof_slot_select(fr_handle* h, int slot);
int fr_prof_slot_ms(fr_handle* h, int slot, float* ms);
int fr_prof_slot_work(fr_handle* h, int slot, double* flops, double* bytes);
int fr_prof_get(const fr_handle* h, int i, char* name, size_t n, double* total_ms, int64_t* launches,
                double* flops);
/* Algorithmic HBM bytes of class i over its timed launches (each input / weight / output byte once;
 * re-reads through L2 and the Infinity Cache are not counted), for the class's HBM-roofline fraction. */
int fr_prof_get_bytes(const fr_handle* h, int i, double* bytes);

int fr_debug_tensor_count(const fr_handle* h);
/* Text dump of the forward plan at batch B, one line per op:
 * "conv|head M N K Kpad tile split KhxKw name", "stage M 256 2304 2304 nconv 1 3x3 name" or
 * "pre|maxpool|avgpool". */
int fr_debug_plan(fr_handle* h, int B, char* buf, size_t n);
const char* fr_debug_tensor_name(const fr_handle* h, int t);
int fr_debug_tensor_shape(const fr_handle* h, int t, int* H, int* W, int* C);
/* Copy the first B samples of tensor t (bf16 NHWC) to dst (device) after an fr_embed. */
/* Storage dtype of tensor t (FR_DTYPE_BF16 / FR_DTYPE_F16): a bf16 IRV1 plan keeps its high-resolution stem
 * tensors in f16, so fr_debug_copy_tensor's 16-bit elements are to be read in this dtype. */
int fr_debug_tensor_dtype(const fr_handle* h, int t);
int fr_debug_copy_tensor(fr_handle* h, int t, int B, void* dst, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* FRHIP_H */
