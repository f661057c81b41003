/*
 * dclip.h — C ABI of libdclip.so, the MI355X (gfx950) DenseCLIP ViT hot path.
 *
 * Every entry point takes plain device pointers, element counts/strides and a
 * hipStream_t (passed as void*), launches asynchronously on that stream and returns
 * 0 on success or a negative DCLIP_ERR_* code; dclip_last_error() then holds a
 * message (thread-local).  No entry point allocates, synchronises or touches the
 * host side of a tensor, so a caller may capture any sequence in a hipGraph.
 *
 * dtype codes: DCLIP_F32 / DCLIP_F16 / DCLIP_BF16.  Matrices are row-major with
 * explicit leading dimensions (in elements).
 *
 * Reference interface each entry point replaces (paths relative to
 * /root/reference/segmentation):
 *   dclip_layernorm_fwd/bwd    denseclip/models.py:243-249  LayerNorm.forward (fp32 math)
 *   dclip_gemm                 nn.Linear in models.py:275-281 (MHA in/out proj, c_fc,
 *                              c_proj), conv1 patchify models.py:407/546 as GEMM,
 *                              vis_proj / global_proj denseclip.py:198-199,605-616,
 *                              and every weight/input gradient of those
 *   dclip_attn_fwd/bwd         nn.MultiheadAttention core (SDPA) models.py:287-289
 *   dclip_conv3x3(_wgrad)      ViTFeatureFusionNeck 3x3 ConvBNReLU convs models.py:741-745
 *   dclip_upsample_ce/silog    logits/depth resize + CE / SILog losses denseclip.py:843-868,
 *                              train_denseclip.py:1265-1314, losses.py:21-78
 *   dclip_im2col               conv1 (16x16, stride 16, no bias) models.py:407,546
 *   dclip_tokens_fwd/bwd       flatten/transpose + CLS + pos add, models.py:548-556
 *   dclip_pos_interp_fwd/bwd   interpolate_pos_encoding models.py:514-540
 *   dclip_transpose            per-layer read-out NLC->NCHW models.py:568-582 (and its
 *                              gradient), NCHW->NHWC for vis_proj, GEMM operand
 *                              transposes with fused bias-gradient column sums
 *   dclip_row_mean             F.adaptive_avg_pool2d(...,(1,1)) denseclip.py:596
 *   dclip_score_map            F.normalize x2 + einsum('bchw,bkc->bkhw')
 *                              denseclip.py:672-675
 *   dclip_score_concat         upsample + torch.cat of the score map onto a read-out map
 *                              denseclip.py:684-694
 *   dclip_bilinear_fwd/bwd     F.interpolate(bilinear, align_corners=False)
 *                              denseclip.py:847,860,899,909 (logits/depth upsample)
 *   dclip_cast                 dtype conversion of operands (.type()/.to() casts)
 *   dclip_cityscapes_prepare   Cityscapes label remap, disparity->depth, crop/flip/normalise
 */
#ifndef DCLIP_H
#define DCLIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DCLIP_F32 0
#define DCLIP_F16 1
#define DCLIP_BF16 2
#define DCLIP_U8 3    /* dclip_cityscapes_augment only: the uint8 HWC crop, before ColorJitter / Normalize */

#define DCLIP_OK 0
#define DCLIP_ERR_ARG (-1)
#define DCLIP_ERR_HIP (-2)

/* GEMM epilogues (dclip_gemm) */
#define DCLIP_EPI_STORE 0      /* C = acc (+ bias[n])                                  */
#define DCLIP_EPI_GELU 1       /* C = z = acc + bias ; C2 = z * sigmoid(1.702 z) ; C null: C2 only */
#define DCLIP_EPI_RESIDUAL 2   /* C(f32) = aux(f32) + acc + bias (aux may alias C); C2, when set, gets the same values in ab_dt */
#define DCLIP_EPI_GELU_BWD 3   /* C = acc * quick_gelu'(aux)       (aux = z)           */
#define DCLIP_EPI_SPLITK 4     /* C(f32) = sum over K splits (+ bias): partial f32 slabs
                                  in the caller's workspace aux (splits*M*N f32), then
                                  one deterministic combine pass (weight gradients)    */
#define DCLIP_EPI_STORE_SCALED 5 /* C = (acc + bias[n]) * aux[n], aux = f32 per-column scale
                                  (the q columns of the in-projection pre-multiplied by
                                  d^-0.5 * log2(e) for dclip_attn_*)                    */

const char* dclip_last_error(void);
int dclip_abi_version(void);

/* Kernel-variant knobs for A/B tuning in one process (process-global, not thread-safe;
 * 0 restores the default).  Results do not depend on them beyond fp32 summation order.  */
#define DCLIP_OPT_ATTN_FWD_WAVES 0   /* 4 or 8 (default) waves = 128 / 256 queries per workgroup */
#define DCLIP_OPT_ATTN_DQ_WAVES 1    /* 4 or 8 (default): dQ pass queries per workgroup / 32      */
#define DCLIP_OPT_ATTN_DKDV_WAVES 2  /* 4 (default) or 8: dK/dV pass keys per workgroup / 32      */
#define DCLIP_OPT_GEMM_TILE 3        /* dclip_gemm tiles: 0 auto (default: 6, 1 below 4096 rows), 1 128x128, 2 256x256, 3 256x128, 4 256x256 k32x4, 5 256x256 ping-pong, 6 persistent 256x256, 7 the same with 4 waves of 128x128, 8 / 9 persistent with pipelined fragment reads (8 / 4 waves) */
#define DCLIP_OPT_GEMM_TN_TILE 4     /* dclip_gemm_tn tiles: 0 auto (default: 256x256 when M, N >= 256), 1 128x128, 2 256x256 with 32-row K-steps in a 4-deep ring, 3 the same 5-deep, 4 256x256 on 4 waves of 128x128, 5 the weight-gradient kernels (256x256 and 128x128) and the conv weight-gradient kernel with the LDS-DMA builtin instead of the asm form (round 6 late: the builtin made every K-step wait for the next one's staging) */
#define DCLIP_OPT_ATTN_DKDV_QS 5     /* dK/dV pass query rows per barrier: 64 (default) or 128 */
#define DCLIP_OPT_ATTN_BWD_KERNEL 7  /* 0 (default): CLS-split passes for N >= 257 (a ragged N-1 with the default pass variants only); 1: generic */
#define DCLIP_OPT_ATTN_FWD_KERNEL 6  /* 0 (default): CLS-split kernels (the pipelined attn_fwd3 when N - 1 is a multiple of 256, else attn_fwd2, ragged N-1 included); 1: generic; 2: attn_fwd3 4 waves x 64 rows; 3: attn_fwd3 8 waves; 4: attn_fwd2 always */
#define DCLIP_OPT_ATTN_BWD_BLOCK 8   /* CLS-split backward: 0 (default, round 6) / 10: the one-pass backward (attention_bwd1.hip: dK, dV and per-key-block dQ partials in one pipelined key-major sweep, an ordered dQ reduction; dclip_attn_bwd_workspace includes the partials, 3.2 GB at B=8, N=8193, H=12); 9: its unpipelined sweep; 6: the two-pass dQ + dK/dV passes, 64 keys per wave, AGPR dK / dV (attention_dkdv6.hip); 7: its software-pipelined schedule; 8: its ring DMA inside R4; 5: software-pipelined 32 keys per wave; 1: the unpipelined one */
#define DCLIP_OPT_GEMM_TN_COLSUM 9   /* 0 (default): the 256x256 weight-gradient kernel sums dY's columns (bias gradient) itself; 1: a separate pass */
#define DCLIP_OPT_GEMM_EPI 10      /* persistent NT GEMM epilogue: 0 (default) row-major through LDS, whole 128-B lines per store, streaming (nontemporal) stores for the wide forward outputs (N >= 2048, not RESIDUAL / GELU_BWD); 1 the accumulator-layout stores (16 rows x 64 B); 2 row-major, streaming stores for every output; 3 row-major, no streaming stores */
#define DCLIP_OPT_GEMM_TAIL 11     /* persistent NT GEMM M tail (<= 16 rows): 0 (default) one latency-shaped MFMA launch (16 columns per workgroup, every K-slice load issued up front, side inputs prefetched); 1 the 256-row split-K tile + combine pair; 2 round 4's one launch (64 columns per workgroup, 8 waves, K % 256 == 0) */
#define DCLIP_OPT_ATTN_FP8_QK 12   /* dclip_attn_fwd_fp8: 0 (default) S = QK^T on the 16-bit MFMA, P V on the fp8 one; 1 both on fp8 (the round-3 kernel) */
#define DCLIP_OPT_ATTN_DQ_ISSUE 13  /* CLS-split dQ pass LDS-DMA issue: 0 (default) a ragged-tile branch; 1 branch-free per-lane select */
#define DCLIP_OPT_ATTN_DQ_ROWS 14   /* CLS-split dQ pass query rows per wave: 32 (default; 8 waves, two per SIMD) or 64 (4 waves, one per SIMD) */
#define DCLIP_OPT_ATTN_DQ_DEFER 15  /* CLS-split dQ pass: 0 (default) a unit's dQ MFMAs right after its softmax; 1 half a step later, beside the next unit's S / dP chains */
#define DCLIP_OPT_GEMM_SCHED 16     /* persistent NT GEMM tile walk: 0 (default) static (round * G + block); 1 work-conserving (every tile claimed: round-0 ownership bitmap, XCD-local ranges, stealing) */
#define DCLIP_OPT_GEMM_KLOOP 17     /* 8-wave GEMM K-loops: 0 (default) the persistent NT kernel with its fragment reads issued one 8-MFMA group ahead except on the GELU epilogue, the TN kernel as compiled; 1 read-ahead in every NT and TN K-loop; 2 none */
#define DCLIP_OPT_ATTN_DQ_REDUCE 18 /* one-pass backward dQ reduction: 0 (default) 8 lanes per query, each lane its 8 columns over the key blocks; 1 8 queries per workgroup, their partial runs read contiguously into LDS (1 KiB per wave-instruction), then 2 columns per lane summed in the same key-block order (bitwise equal) */
#define DCLIP_OPT_ATTN_PREP_ORDER 19 /* one-pass backward prep pass: 0 (default) query blocks of one head on adjacent workgroups; 1 the heads of one query block on adjacent workgroups (same per-workgroup work, bitwise equal) */
#define DCLIP_OPT_COUNT 20
int dclip_set_option(int id, int value);

/* LayerNorm over the last dim (cols), eps, affine w/b (fp32).  y = (x-mu)*rstd*w+b.
 * mean/rstd (rows) are written when non-null.                                        */
int dclip_layernorm_fwd(const void* x, int x_dt, const float* w, const float* b,
                        void* y, int y_dt, float* mean, float* rstd,
                        int64_t rows, int64_t cols, float eps, void* stream);

/* LayerNorm backward.  dy: grad wrt y (dy_dt), x: the LN input (x_dt), mean/rstd from
 * the forward.  dx (f32) is overwritten (accumulate=0) or added to (accumulate=1).
 * dw/db (f32, cols) are ACCUMULATED (callers zero them first).                       */
int dclip_layernorm_bwd(const void* dy, int dy_dt, const void* x, int x_dt,
                        const float* w, const float* mean, const float* rstd,
                        float* dx, int accumulate, float* dw, float* db,
                        int64_t rows, int64_t cols, void* stream);
/* The same with the residual branch's gradient fused in: dx = res + LN^T(dy) (res f32, may be
 * null or alias dx) and, when lp is non-null, a 16-bit copy lp = (lp_dt) dx (lp_dt F16 or
 * BF16) — the next GEMM's operand, without a separate clone / cast pass (the
 * x + f(LN(x)) residual of models.py:292-293, backward).                              */
int dclip_layernorm_bwd_res(const void* dy, int dy_dt, const float* dy_scale, int64_t dy_ntok,
                            const void* x, int x_dt, const float* w, const float* mean, const float* rstd,
                            const float* res, float* dx, void* lp, int lp_dt, float* dw, float* db,
                            float* ws, int64_t rows, int64_t cols, void* stream);
/* dy_scale, dy_ntok (ABI 6; dclip_layernorm_bwd_res, _scaled, _scaled_add): dy is read as
 * dy * (*dy_scale) when dy_scale is non-null (an f16 dy still on its gradient scale s, dy_scale
 * pointing at 1/s: the fp16 backward's dX GEMMs write their output for the LN backward in f16 on
 * the scale their operand carries), and rows with row % dy_ntok == 0 read as 0 when dy_ntok > 0
 * (a token-buffer gradient whose CLS rows are not part of it: the ln_post read-out's).  NULL / 0:
 * dy as given.  Need cols in {512, 768, 1024}.                                               */
/* ws (ABI 5; dclip_layernorm_bwd_res, _scaled, _add, _scaled_add): the caller's scratch of
 * dclip_layernorm_bwd_ws_floats(rows, cols) floats (contents on entry irrelevant, clobbered) for
 * the per-workgroup dw / db partials, summed into dw / db in a fixed order (deterministic) by a
 * second launch on the same stream; private to the call, so concurrent calls on different
 * streams or graph replays never share it.  NULL: the workgroups add atomically into dw / db
 * (correct, summation order not fixed).  Widths without the fast kernels (cols not 512 / 768 /
 * 1024; the query returns 0 for them) always add atomically.                               */
int64_t dclip_layernorm_bwd_ws_floats(int64_t rows, int64_t cols);

/* C[m][n] = alpha * sum_k A[m][k] * B[n][k]  ("NT": both operands k-contiguous, ab_dt in
 * {F16, BF16}), m < M, n < N, k < K (K % 64 == 0, lda/ldb % 8 == 0), then the
 * epilogue.  bias: f32[N] or null.  aux: epilogue side input (see DCLIP_EPI_*).
 * alpha undoes a gradient scale carried by an operand (fp16 backward; 1 otherwise); when
 * alpha_ptr is non-null the factor is alpha * *alpha_ptr, read on the device (the 1/s entry
 * of a dclip_grad_scale pair: no host round trip).
 * splits > 1 (EPI_SPLITK only) splits K into `splits` equal 64-multiple chunks.      */
int dclip_gemm(int epilogue, int ab_dt,
               const void* A, int64_t lda, const void* B, int64_t ldb,
               int64_t M, int64_t N, int64_t K, int splits, float alpha, const float* alpha_ptr,
               const float* bias, const void* aux, int aux_dt, int64_t ld_aux,
               void* C, int c_dt, int64_t ldc, void* C2, int64_t ldc2, void* stream);

/* C[m][n] = alpha * sum_k A[k][m] * B[k][n] ("TN": reduction over the ROWS of both operands —
 * the weight-gradient shape dW = dY^T X without transposed copies).  A: (K, lda >= M),
 * B: (K, ldb >= N), M % 8 == N % 8 == 0.  The K range is split into `splits` chunks of
 * K_pad / splits (K_pad >= K, multiple of 64*splits; rows >= K contribute zero).
 * epilogue STORE (f32 C, splits == 1) or SPLITK (f32 slabs in ws, then a combine that adds
 * bias[n] when non-null; ws holds splits*(M*N + M) floats: the slabs, then (ABI 5) the column
 * sums' per-split partials).  colsum_a (f32, M), when non-null, receives += alpha * the column
 * sums of A over the K rows (the bias gradient of dY) — in a fixed order (deterministic) on the
 * 256x256 path (M, N >= 256), by per-row-chunk atomics on the small-tile path.  alpha_ptr as in
 * dclip_gemm.                                                                          */
/* The K-split plan dclip_gemm_tn runs best with for an M x N output over K rows
 * (splits, and K_pad = K rounded up to 64*splits); host-side only, no GPU work.      */
int dclip_gemm_tn_plan(int64_t M, int64_t N, int64_t K, int* splits, int64_t* K_pad);

int dclip_gemm_tn(int epilogue, int ab_dt, const void* A, int64_t lda, const void* B, int64_t ldb,
                  int64_t M, int64_t N, int64_t K, int64_t K_pad, int splits, float alpha,
                  const float* alpha_ptr, const float* bias,
                  void* ws, void* C, int64_t ldc, float* colsum_a, void* stream);

/* Fused multi-head attention over a packed QKV buffer.
 * qkv: (B*N, 3*H*D) row-major, [q | k | v] each (H, D) head-major (the layout of
 *      x @ in_proj_weight^T + in_proj_bias, models.py:289 / F.multi_head_attention_forward)
 *      with the q columns PRE-MULTIPLIED by c = scale * log2(e) ("log2-domain queries",
 *      produced for free by the in-projection GEMM's DCLIP_EPI_STORE_SCALED epilogue)
 * o:   (B*N, H*D) softmax(q k^T * scale) v, heads concatenated
 * lse: (B, H, N) f32, log2-domain row statistic  max*c + log2(sum), c = scale*log2(e)
 * D must be 64.                                                                      */
int dclip_attn_fwd(int dt, const void* qkv, void* o, float* lse,
                   int B, int N, int H, int D, float scale, void* stream);

/* Attention backward (flash-style recompute from lse; no N x N buffer, no atomics): for N >= 257
 * (the CLS split) by default the one-pass backward (round 6: a prep pass writing delta =
 * rowsum(dout*o) and the statistics, one key-major sweep for dK, dV and 16-bit dQ partials per
 * 256-key block, an ordered reduction of the partials); with DCLIP_OPT_ATTN_BWD_BLOCK 6, and below
 * N = 257, a query-major dQ pass (which also writes delta) and a key-major dK/dV pass.  dout:
 * (B*N, H*D) dt.  delta_ws: f32 workspace of dclip_attn_bwd_workspace(B, N, H) floats — query it
 * after setting options: it includes the one-pass form's partials (B*H*ceil((N-1)/256)*
 * (1+64*ceil((N-1)/64))*128 bytes, 3.2 GB at B = 8, N = 8193, H = 12) when that form runs.  Its
 * first B*H*N floats receive delta; the rest holds the CLS-split row-0 partials, the negated lse /
 * delta planes, key 0's dS column and the dQ partials.
 * qkv as for dclip_attn_fwd (q pre-multiplied by scale*log2(e)); `scale` = d^-0.5.
 * dqkv: (B*N, 3*H*D) dt output, [dq | dk | dv] in the qkv layout: gradients with
 * respect to the UNSCALED q, k, v (i.e. the in-projection output before the q scale).  */
int dclip_attn_bwd(int dt, const void* qkv, const void* o, const void* dout,
                   const float* lse, float* delta_ws, void* dqkv,
                   int B, int N, int H, int D, float scale, void* stream);

/* configs[4]'s attention backward (ABI 7): dclip_attn_bwd's contract and results within e4m3
 * rounding — on the CLS-split path (N >= 257) the dK / dV pass runs dV = P^T dO and dK = dS^T q' on
 * the block-scaled e4m3 MFMA (v_mfma_scale_f32_32x32x64_f8f6f4, MX E8M0 scales per 32 queries: the
 * Q / dO rows' from a pack pass, P's fixed at 2^-8, dS's per key from its amax), S, dP and the dQ
 * pass stay 16-bit; elsewhere it is dclip_attn_bwd.  ws: dclip_attn_bwd_fp8_workspace(B, N, H)
 * floats, 16-B aligned (dclip_attn_bwd's workspace, then the slices' e4m3 images).  Replaces the
 * backward of models.py:287-289 under the fp8 attention of BASELINE configs[4].               */
int64_t dclip_attn_bwd_fp8_workspace(int B, int N, int H);
int dclip_attn_bwd_fp8(int dt, const void* qkv, const void* o, const void* dout, const float* lse, float* ws,
                       void* dqkv, int B, int N, int H, int D, float scale, void* stream);
int64_t dclip_attn_bwd_workspace(int B, int N, int H);

/* fp8 attention forward (BASELINE config 5; inference only — there is no fp8 backward).
 * Same qkv / o / lse contract as dclip_attn_fwd (q pre-multiplied by d^-0.5*log2(e)), computed
 * on the block-scaled e4m3 MFMA v_mfma_scale_f32_32x32x64_f8f6f4: q, k, v are quantised to
 * OCP e4m3 with one scale per (image, head, q|k|v) = 448 / amax, P to e4m3 unscaled (P <= 1).
 * ws: dclip_attn_fwd_fp8_workspace(B, N, H) bytes, 256-byte aligned (the packed q8 / k8 /
 * transposed v8 planes and the amax table).  H <= 64, D must be 64.                      */
int dclip_attn_fwd_fp8(int dt, const void* qkv, void* o, float* lse, void* ws,
                       int B, int N, int H, int D, void* stream);
int64_t dclip_attn_fwd_fp8_workspace(int B, int N, int H);

/* Non-overlapping p x p patches of img (B, Cin, Hin, Win) (img_dt) ->
 * out (B*gh*gw, ldo) (out_dt), column order (c, ky, kx) = conv weight flattening,
 * gh = Hin / p, gw = Win / p (floor, as Conv2d stride p).  Columns Cin*p*p .. ldo-1
 * are written as zeros: ldo = the patch GEMM's K padded to 64 (p = 14: 588 -> 640).
 * ldo % 4 == 0.                                                                        */
int dclip_im2col(const void* img, int img_dt, void* out, int out_dt, int64_t ldo,
                 int B, int Cin, int Hin, int Win, int p, void* stream);

/* Token assembly: x[b][0] = cls + pos[0]; x[b][1+i] = patch[b*P+i] + pos[1+i]
 * x: f32 (B*(P+1), C).  patch: (B*P, C) patch_dt.  pos: f32 (P+1, C).              */
int dclip_tokens_fwd(const void* patch, int patch_dt, const float* cls, const float* pos,
                     float* x, int B, int P, int C, void* stream);

/* Token assembly backward: dpatch[b*P+i] = dpatch_scale * dx[b][1+i] (dpatch_dt; times
 * *dpatch_scale_ptr when non-null, read on the device);
 * dcls += sum_b dx[b][0]; dpos[t] += sum_b dx[b][t]  (dcls/dpos f32, accumulated)   */
int dclip_tokens_bwd(const float* dx, void* dpatch, int dpatch_dt, float dpatch_scale,
                     const float* dpatch_scale_ptr, float* dcls, float* dpos, int B, int P, int C,
                     void* stream);

/* Bilinear (align_corners=False) resize of the g x g patch grid of pos (g*g+1, C)
 * to H x W; out (H*W+1, C), row 0 = pos row 0.                                       */
int dclip_pos_interp_fwd(const float* pos, float* out, int g, int C, int H, int W,
                         void* stream);
/* Its gradient: dpos (g*g+1, C) += interp^T(dout); dout (H*W+1, C).                 */
int dclip_pos_interp_bwd(const float* dout, float* dpos, int g, int C, int H, int W,
                         void* stream);

/* Batched transpose: out[b][c][r] (=, or += if accumulate) in[b][r0 + r][c]
 * for r < rows, c < cols; rows..rows_pad-1 of every out row are written as 0.
 * colsum (f32, cols) += sum over b, r of in[b][r0+r][c] when non-null.
 * Strides in elements.  accumulate requires out_dt == F32.                          */
int dclip_transpose(const void* in, int in_dt, int64_t in_bstride, int64_t in_ld, int64_t r0,
                    void* out, int out_dt, int64_t out_bstride, int64_t out_ld,
                    int batch, int64_t rows, int64_t rows_pad, int64_t cols,
                    int accumulate, float* colsum, void* stream);

/* Compute-dtype weight copies after an optimizer step (no reference counterpart: the reference
 * runs fp32 weights; replaces one cast and one transpose launch per weight per step).  desc:
 * n entries of 8 int64 ON THE DEVICE: [src (f32, rows x cols, contiguous, 16-B aligned),
 * plain dst (out_dt, rows x cols) or 0, transposed dst (out_dt, cols x rows) or 0, rows, cols,
 * first tile, column tiles = ceil(cols / 64), 0]; entry e covers tiles [first, first +
 * ceil(rows / 64) * column tiles), the entries in order, tiles = the total.  One launch.      */
int dclip_weight_refresh(const int64_t* desc, int n, int64_t tiles, int out_dt, void* stream);

/* Strided pixel rows: row r (< rows) of image b is X + b*bstride + (row_off + r)*ld (elements; a ViT
 * token buffer (B*N, C) has bstride N*C, row_off 1 (skips CLS), ld C).  16-bit X, 16-byte aligned rows.
 *
 * out[b][c] (f32) = mean over r < rows of row r of image b  (F.adaptive_avg_pool2d(x, (1, 1)),
 * denseclip.py:596); ws: dclip_row_mean_workspace(B, rows, C) floats (fixed-order chunk sums).
 * C % 8 == 0, C <= 2048.                                                                       */
int64_t dclip_row_mean_workspace(int B, int64_t rows, int C);
int dclip_row_mean(const void* x, int x_dt, int64_t bstride, int64_t row_off, int64_t ld, int B, int64_t rows,
                   int C, float* ws, float* out, void* stream);

/* Pixel-text score map (F.normalize x2 + einsum('bchw,bkc->bkhw'), denseclip.py:672-675) as a
 * batched MFMA product.  v: strided pixel rows as above (HW rows per image, v_dt F16/BF16),
 * t: f32 (B, K, C).  score f32 (B, K, HW) = <v/max(|v|,eps), t/max(|t|,eps)>.  K <= 32,
 * C % 16 == 0, C <= 2048.                                                                      */
int dclip_score_map(const void* v, int v_dt, int64_t bstride, int64_t row_off, int64_t ld, const float* t,
                    float* score, int B, int HW, int C, int K, float eps, void* stream);

/* The score_concat_index branch's torch.cat([x_i, F.interpolate(score, (h, w)).to(x_i.dtype)], 1)
 * (denseclip.py:684-694) in one pass: out (B*h*w, C + K) channels-last rows, 16-bit (dt) = the
 * strided pixel rows of x_i (as dclip_row_mean: image b's pixel p at b*bstride + (row_off + p)*ld)
 * followed by the bilinearly resized (align_corners=False) f32 score (B, K, hs, ws), K <= 64.      */
int dclip_score_concat(const void* rows, int dt, int64_t bstride, int64_t row_off, int64_t ld, int C,
                       const float* score, int K, int hs, int ws, void* out, int B, int h, int w, void* stream);

/* Bilinear resize, align_corners=False, of NC planes (NC, Hi, Wi) -> (NC, Ho, Wo).   */
int dclip_bilinear_fwd(const void* in, int in_dt, void* out, int out_dt,
                       int64_t NC, int Hi, int Wi, int Ho, int Wo, void* stream);
/* Its gradient: din f32 (NC, Hi, Wi) = resize^T(dout).  ws: f32 (NC, Ho, Wi).        */
int dclip_bilinear_bwd(const void* dout, int dout_dt, float* din, float* ws,
                       int64_t NC, int Hi, int Wi, int Ho, int Wo, void* stream);

/* 3x3 / stride 1 / pad 1 convolution as an implicit GEMM on channels-last pixel rows
 * (the ViTFeatureFusionNeck's per-level convs, reference models.py:741-745 / 13-20, run on
 * the ViT token read-out without NCHW copies).  Input pixel (b, y, x) of the B x H x W image
 * is the row X + b*x_bstride + x_off + (y*W + x)*x_ld (elements, all multiples of 8); for a
 * ViT token buffer (B*N, C): x_bstride = N*C, x_off = C (skips CLS), x_ld = C.
 *   mode 0 (forward):  out[p][n] = sum_{tap, c} X[p + d(tap)][c] * Wt[n][tap*Cin + c]
 *   mode 1 (dgrad):    out[p][n] = sum_{tap, c} X[p - d(tap)][c] * Wt[n][tap*Cin + c]
 *                      (X = dOut with Cin = Cout channels, Wt[ci][tap*Cout + co] = w[co][ci][tap])
 * d(tap) = (tap/3 - 1, tap%3 - 1); out-of-image taps read zeros.  Cin % 64 == 0.
 * Output row of pixel p: p, or with out_gap > 0: p + (p / (H*W))*out_gap + out_off (e.g.
 * gap 1, off 1 writes into rows 1.. of each batch of a (B*N, C) token buffer); out_ld is
 * its row pitch.  out_dt: f32 or the operand dtype; accumulate=1 (f32 only) adds.        */
int dclip_conv3x3(int mode, int ab_dt, const void* X, int64_t x_bstride, int64_t x_off, int64_t x_ld,
                  int B, int H, int W, int Cin, const void* Wt, int Nout, void* out, int out_dt,
                  int64_t out_ld, int out_gap, int out_off, int accumulate, void* stream);

/* Weight gradient of the 3x3 conv: dW[co][tap*Cin + c] = sum_p dY[p][co] * X[p + d(tap)][c]
 * (f32, Nout x 9*Cin), pixels split into `splits` chunks summed through ws
 * (splits * Nout * 9*Cin f32) in a fixed order.  Cin % 128 == 0.  oihw = 1 writes torch's
 * weight layout instead, dW[co][c][tap] (Nout, Cin, 3, 3), times *alpha_ptr when given (the 1/s
 * entry of an fp16 gradient-scale pair; alpha_ptr needs oihw = 1).                       */
int dclip_conv3x3_wgrad(int ab_dt, const void* dY, int64_t ldy, int Nout, const void* X, int64_t x_bstride,
                        int64_t x_off, int64_t x_ld, int B, int H, int W, int Cin, float* dW, void* ws,
                        int splits, int oihw, const float* alpha_ptr, void* stream);

/* Fused bilinear upsample (align_corners=False) + loss + gradient of the heads
 * (denseclip.py:843-868 resize, train_denseclip.py:1265-1314 losses), without materialising
 * the upsampled tensors.  logits: (B, K, h, w) low_dt; labels: (B, H, W) int64 (lab_dt 0),
 * int32 (1) or uint8 (2); pixels whose label is ignore_index (or outside [0, K)) are skipped.
 *   dclip_upsample_ce:    loss_sum (f64[1]) += sum of -log softmax(up(logits))[label],
 *                         count (u32[1]) += #valid, grad (f32, B*K*h*w, accumulated)
 *                         += up^T(softmax - onehot)   (the caller scales by 1/count)
 *   dclip_upsample_silog: pred (B, 1, h, w); target f32 (B, H, W); mask u8 (B, H, W) or null.
 *                         pass 0: sums (f64[3]) += (sum d, sum d^2, T), d = log(max(up(pred),
 *                         eps)) - log(max(target, eps)) on the mask; pass 1 (sums complete):
 *                         grad (f32, B*h*w) += up^T((2d/T - 2 lambd S/T^2) / up(pred))
 *                         (zero where up(pred) < eps).  K == 19 for the CE kernel.
 * ws (ABI 7): the caller's scratch of dclip_upsample_ws_floats(B, K, h, w) floats (K = 1 for
 * SILog), 8-byte aligned, contents undefined on entry: every workgroup writes its loss partials
 * and its low-res gradient tile there and two short launches add them in a fixed order, so the
 * loss and the gradient are bitwise reproducible (ABI 6 used float atomics).  Stream-ordered:
 * one ws per call in flight.                                                            */
int64_t dclip_upsample_ws_floats(int B, int K, int h, int w);
int dclip_upsample_ce(int low_dt, const void* logits, int B, int K, int h, int w, const void* labels, int lab_dt,
                      int H, int W, int ignore_index, double* loss_sum, unsigned* count, float* grad, float* ws,
                      void* stream);
int dclip_upsample_silog(int pass, int low_dt, const void* pred, int B, int h, int w, const float* target,
                         const uint8_t* mask, int H, int W, float eps, float lambd, double* sums, float* grad,
                         float* ws, void* stream);

/* Cityscapes depth + segmentation batch preparation (datasets/cityscapes_depth_seg.py:129-170,
 * 218 and the trainer's RandomCrop / HorizontalFlip / Normalize / ToTensorV2,
 * train_denseclip.py:143-149).  Inputs: decoded planes of B images of H x W — img uint8
 * (B, H, W, 3) RGB, ids uint8 (B, H, W) Cityscapes label ids, disp uint16 (B, H, W) disparity;
 * crop int32 (B, 3) = (y0, x0, flip) per image, window [y0, y0 + h) x [x0, x0 + w) inside the
 * image (mirrored when flip != 0).  Outputs for the h x w crops: out_img (B, 3, h, w) out_dt
 * = (x - 255 mean) * (1 / (255 std)); out_seg int64 (B, h, w) train ids (ids >= 34 -> 255);
 * out_depth f32 (B, h, w) = bf / ((d - 1) / 256 + 1e-6) where d > 0, (d - 1) / 256 > 1e-3 and
 * the depth <= depth_max, else 0; out_mask uint8 (B, h, w) = depth > 0.  All device pointers
 * (mean, stdv: 3 host floats).                                                          */
int dclip_cityscapes_prepare(const uint8_t* img, const uint8_t* ids, const uint16_t* disp, int B, int H, int W,
                             const int* crop, int h, int w, const float* mean, const float* stdv, float bf,
                             float depth_max, void* out_img, int out_dt, int64_t* out_seg, float* out_depth,
                             uint8_t* out_mask, void* stream);

/* dclip_cityscapes_prepare with the trainer's whole spatial pipeline in front of the crop
 * (train_denseclip.py:138-149): RandomScale -> PadIfNeeded -> RandomCrop -> HorizontalFlip.
 * params int32 (B, 7) on the device = (Hs, Ws, pad_top, pad_left, y0, x0, flip) per image: the
 * image is resized to Hs x Ws (cv2 INTER_CUBIC on uint8, the flag the reference's
 * interpolation=Image.BILINEAR (= 2) selects; label ids and disparity INTER_NEAREST), padded by
 * pad_top / pad_left (image 0, seg 255, depth 255 -> mask 1, as PadIfNeeded(value=0,
 * mask_value=255) followed by the reference's depth > 0 validity), and the h x w window at
 * (y0, x0) of the padded image is taken (mirrored when flip).  Same outputs as
 * dclip_cityscapes_prepare; identity params (H, W, 0, 0, y0, x0, flip) give its result.   */
int dclip_cityscapes_augment(const uint8_t* img, const uint8_t* ids, const uint16_t* disp, int B, int H, int W,
                             const int* params, int h, int w, const float* mean, const float* stdv, float bf,
                             float depth_max, void* out_img, int out_dt, int64_t* out_seg, float* out_depth,
                             uint8_t* out_mask, void* stream);

/* ColorJitter (albumentations, train_denseclip.py:152-155; `color_jitter: true`) in place on a
 * uint8 HWC batch img (B, h, w, 3) RGB: params (B, 8) f64 on the device = brightness, contrast,
 * saturation, hue factors and the order of the four (0 brightness, 1 contrast, 2 saturation,
 * 3 hue) per image; identity factors (1, 1, 1, 0) leave an image untouched.  uint8 arithmetic of
 * albumentations' *_torchvision functions and OpenCV's 8-bit RGB<->GRAY / HSV conversions.
 * ws: B uint64 (per-image gray sums for the contrast mean).                             */
int dclip_color_jitter(uint8_t* img, int B, int h, int w, const double* params, unsigned long long* ws,
                       void* stream);

/* Normalize + ToTensorV2 of a uint8 HWC batch (B, h, w, 3): out (B, 3, h, w) out_dt =
 * (x - 255 mean) * (1 / (255 std)) (mean, stdv: 3 host floats).                           */
int dclip_normalize_u8(const uint8_t* img, int B, int h, int w, const float* mean, const float* stdv, void* out,
                       int out_dt, void* stream);

/* Element-wise dtype conversion of n elements: out = (out_dt)(in * scale), times *scale_ptr
 * when non-null (read on the device).  A power-of-two scale keeps fp16 gradients out of the
 * subnormal range (see dclip_grad_scale and dclip_gemm's alpha).                      */
int dclip_cast(const void* in, int in_dt, void* out, int out_dt, int64_t n, float scale,
               const float* scale_ptr, void* stream);

/* Eval-mode BatchNorm2d (+ ReLU when relu != 0) from the running statistics, on the same rows
 * as dclip_bn_fwd: y = x * w / sqrt(running_var + eps) + (b - running_mean * that scale), f32
 * arithmetic, 16-bit I/O.  ws: dclip_bn_workspace(rows, C) floats.  (nn.BatchNorm2d.eval() of
 * the neck's ConvModules and the FCN heads, models.py:13-20.)                            */
int dclip_bn_eval(int dt, const void* x, int64_t rows, int C, int64_t ld, const float* w, const float* b, float eps,
                  const float* running_mean, const float* running_var, float* ws, void* y, int relu, void* stream);

/* Stochastic depth (drop_path, reference models.py:257-268, 291-294 on the LND layout: one keep
 * value per token position): out[r][c] = (x ? x[r][c] : 0) + s[r % ntok] * y[r][c], f32
 * (rows, cols) row-major, rows a multiple of ntok, cols % 4 == 0; out may alias x or y. */
int dclip_row_scale_add(const float* x, const float* y, const float* s, int ntok, float* out, int64_t rows,
                        int cols, void* stream);

/* Power-of-two scale for the fp16 cast of an f32 gradient g (n elements, 16-byte aligned),
 * computed on the device: ws[0] = s = 2^clamp(floor(log2(target / max|g|)), -60, 60),
 * ws[1] = 1/s (s = 1 when max|g| is 0 or not finite).  ws: 4 floats, ws[2..3] zero on entry
 * (left zero on exit, so one buffer serves successive calls on a stream).  Pass ws to
 * dclip_cast / dclip_tokens_bwd as scale_ptr and ws + 1 to dclip_gemm / dclip_gemm_tn as
 * alpha_ptr.  (No reference counterpart: the reference trains in fp32.)              */
int dclip_grad_scale(const float* g, int64_t n, float target, float* ws, void* stream);
/* Read-out gradient folded into a block's incoming gradient (replaces the autograd sum of the
 * two uses of a block output, models.py:565 -> 577-597, plus the backward's cast): sum = a + b
 * with b's CLS rows (row % ntok == 0) read as 0, lp = (lp_dt)(sum * scale).  a, sum: f32
 * (rows, cols); b: (rows, cols) token buffer, f32/bf16/f16; cols % 8 == 0; sum may alias a. */
int dclip_add_readout_cast(const float* a, const void* b, int b_dt, float* sum, void* lp, int lp_dt,
                           int64_t rows, int cols, int ntok, float scale, void* stream);

/* The fp16 backward's form of the same fold: sum = a + b * (*b_scale_ptr, or 1 when null) with
 * b's CLS rows read as 0, and in the same pass ws = the dclip_grad_scale pair (s, 1/s, 0, 0) of
 * sum for its fp16 cast (ws zeroed before first use, left reusable).  b_scale_ptr: the 1/s entry
 * of the fp16 heads' gradient scale (the map gradient arrives scaled).  cols % 8 == 0.      */
int dclip_add_readout_amax(const float* a, const void* b, int b_dt, const float* b_scale_ptr, float* sum,
                           int64_t rows, int cols, int ntok, float target, float* ws, void* stream);

/* DELAYED-scale fp16 casts of the backward's block gradients (the fp16 line; replaces a
 * dclip_grad_scale + dclip_cast pair, or dclip_add_readout_amax + dclip_cast, per block branch).
 * st: the state of one gradient site, DCLIP_DS_STATE_FLOATS floats that persist across training
 * steps (3 x 64 shards of |x|-maximum bits, then 3 used scales); `use` counts the site's calls
 * from 1.  Call k casts with s = 2^clamp(floor(log2(target / max_{k-1})), -60, 60), the scale of
 * call k-1's own maximum (call k-1's scale again when that maximum was 0 or not finite), writes
 * (s, 1/s) to spair (2 floats: what the consumers of lp unscale by) and records its maximum in st
 * for call k+1 — no fences, no arrival counter.  Seeding for call 1 (after an exact two-pass cast
 * with scale s0): st all zero except st[0] = target / s0 and st[192] = s0.  A gradient that grew
 * by more than 65504 / target between two calls overflows to inf in lp (the fp16 train step
 * then checks its gradients and skips, train.step_unless_nonfinite).  (No reference
 * counterpart: the reference trains in fp32.)
 *   dclip_add_readout_cast_scaled: sum = a (+ b * (*b_scale_ptr), b's CLS rows read as 0; b may be
 *     null, then sum is not written), lp = (f16)(sum * s).  models.py:565 -> 577-597 as
 *     dclip_add_readout_cast.  cols % 8 == 0.
 *   dclip_layernorm_bwd_scaled: dclip_layernorm_bwd_res with an f32 x, dy f32 or (ABI 6) f16 on
 *     dy_scale, and lp = (f16)(dx * s) (models.py:243-249 backward).  cols in {512, 768, 1024}. */
#define DCLIP_DS_STATE_FLOATS 196
int dclip_add_readout_cast_scaled(const float* a, const void* b, int b_dt, const float* b_scale_ptr, float* sum,
                                  void* lp, int64_t rows, int cols, int ntok, float target, float* st, int use,
                                  float* spair, void* stream);
int dclip_layernorm_bwd_scaled(const void* dy, int dy_dt, const float* dy_scale, const void* x, int x_dt,
                               const float* w, const float* mean, const float* rstd, const float* res, float* dx,
                               void* lp, float* dw, float* db, float* ws, int64_t rows, int64_t cols, float target,
                               float* st, int use, float* spair, void* stream);

/* LayerNorm backward of a block's ln_1 with the PREVIOUS block's read-out map gradient folded in
 * (models.py:243-249 backward + the models.py:565 -> 577-597 read-out's gradient):
 *   dx = (res + LN^T(dy)) + add,  lp = (lp_dt) dx
 * add: a bf16 (rows, cols) token buffer whose rows with row % ntok == 0 (CLS) read as 0.  One pass
 * in place of dclip_layernorm_bwd_res + dclip_add_readout_cast (bitwise their result: the same
 * fp32 additions in the same order).  dy f32 or bf16, x f32, cols in {512, 768, 1024}; lp required.
 * dw / db accumulate as in dclip_layernorm_bwd_res (may be NULL). */
int dclip_layernorm_bwd_add(const void* dy, int dy_dt, const float* x, const float* w, const float* mean,
                            const float* rstd, const float* res, const void* add, int ntok, float* dx, void* lp,
                            int lp_dt, float* dw, float* db, float* ws, int64_t rows, int64_t cols, void* stream);
/* The fp16 backward's form: dclip_layernorm_bwd_scaled (dy f32 or f16 on dy_scale, f32 x, lp = (f16)(dx * s) on the
 * delayed scale of st's use `use`, (s, 1/s) to spair) with dx = (res + LN^T(dy)) + add * (*add_scale)
 * (add: f16 or bf16 (add_dt), CLS rows read as 0; add_scale may be NULL = 1) — in place of
 * dclip_layernorm_bwd_res + dclip_add_readout_cast_scaled on the same site state.  cols in
 * {512, 768, 1024}. */
int dclip_layernorm_bwd_scaled_add(const void* dy, int dy_dt, const float* dy_scale, const float* x,
                                   const float* w, const float* mean, const float* rstd, const float* res,
                                   const void* add, int add_dt, const float* add_scale, int ntok, float* dx,
                                   void* lp, float* dw, float* db, float* ws, int64_t rows, int64_t cols,
                                   float target, float* st, int use, float* spair, void* stream);

/* Train-mode BatchNorm2d (+ optionally the ReLU after it) on a channels-last 16-bit map viewed as
 * rows (B*H*W) of C channels at a row pitch of ld elements (ld = C for a whole map; larger for a
 * channel slice of a wider buffer, e.g. one level of the neck's concatenation).  Replaces
 * nn.BatchNorm2d + nn.ReLU in the neck's ConvModules (models.py:13-20) and the FCN heads;
 * torch.nn.functional.batch_norm semantics: biased batch variance for the normalisation,
 * unbiased for running_var, running = (1 - momentum) running + momentum batch.  C % 8 == 0,
 * C <= 2048, ld % 8 == 0.  w, b, running_mean / running_var may be NULL.  ws:
 * dclip_bn_workspace(rows, C) floats.  Forward: y = [relu](bn(x)) (same pitch as x), mean /
 * rstd (f32, C) for the backward.  Backward (relu: dy masked where bn(x) <= 0, recomputed from x):
 * dx (dt, same pitch) and, when non-null, dw / db (f32, C). */
int64_t dclip_bn_workspace(int64_t rows, int C);
int dclip_bn_fwd(int dt, const void* x, int64_t rows, int C, int64_t ld, const float* w, const float* b,
                 float eps, float momentum, float* running_mean, float* running_var, float* ws, float* mean,
                 float* rstd, void* y, int relu, void* stream);
/* gscale (nullable): dw and db are multiplied by *gscale (the 1/s entry of the fp16 heads'
 * gradient-scale pair; dx keeps the scale of dy).                                         */
int dclip_bn_bwd(int dt, const void* dy, const void* x, int64_t rows, int C, int64_t ld, const float* w,
                 const float* b, const float* mean, const float* rstd, float* ws, void* dx, float* dw,
                 float* db, int relu, const float* gscale, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* DCLIP_H */
