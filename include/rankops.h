/*
 * rankops.h — C ABI of the MI355X (gfx950) CTR feature-interaction engine.
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t passed
 * as `void*` (NULL = the default stream).  Nothing here knows about torch: the
 * Python host layer (the rankops Python package) binds these with ctypes, exactly as the
 * reference's `nn.Module.forward()` bodies would bind them.
 * All work is enqueued asynchronously on `stream`; no entry point allocates
 * device memory or synchronises, so every forward can be captured in a hipGraph.
 *
 * Return value: RK_OK (0) or an RK_ERR_* code; rk_last_error() gives the text.
 * Out-of-range embedding indices never fault: the row is read as zeros and
 * RK_FLAG_INDEX_OOB is raised in the device flag word (rk_error_flags), the
 * analogue of nn.Embedding's IndexError / device assert.
 *
 * Reference interfaces replaced (file:line in the reference snapshot):
 *   rk_concat_gather   nn.Embedding lookups + torch.cat       dcn.py:163-169, deepcrossing.py:148-155,
 *                                                            din.py:296-305,310, bst.py:218-224,243
 *   rk_dcn_cross       cross_layer() loop + output_layer part dcn.py:25-50,171-173,177-178
 *   rk_fm_gather       DeepFM first/second-order FM + concat deepfm.py:122-142
 *   rk_fm_pack_table, rk_fm_gather_packed  the same over one packed [V, pad4(D+1)] table per field
 *   rk_linear          nn.Linear (+BatchNorm1d eval, ReLU/LeakyReLU/Dice/PReLU, residual,
 *                      LayerNorm, sum/mean pooling, final Linear(*,1)+sigmoid) dcn.py:144-152,175-180;
 *                      deepfm.py:100-112,143-151; din.py:26-36,272-285,312-316; deepcrossing.py:25-42,161-162;
 *                      bst.py:59-64,73-75,86-90,203-214,238-247
 *   rk_din_attention   din_attention() with the history gathered from the table  din.py:42-84,300-305
 *   rk_din_attention_dense  din_attention(query, keys[B,T,H], keys_length, is_softmax)  din.py:42-84
 *   rk_dice_forward    Dice.forward() in eval (BatchNorm running statistics)           din.py:26-36
 *   rk_row_l2norm_mean DIN mini-batch-aware l2 term          din.py:318-322
 *   rk_afm_forward     AFM.forward()                         afm.py:92-119
 *   rk_bst_attention   BSTTransformer scores/mask/softmax/AV bst.py:73-84 (mask from seq_length, bst.py:228-229)
 *   rk_bst_attention_masked  the same with BSTTransformer.forward's key_padding_mask  bst.py:66-84
 *   rk_bst_forward_blocks  all BSTTransformer blocks + pooling, fused bst.py:66-91,224-241
 *   rk_bst_forward_blocks_packed  the same on pre-packed projection weights
 *   rk_linear_tiled    one wide MLP layer (2D-tiled)          deepfm.py:100-112 (first deep layer)
 *   rk_fm_linear_packed  the DeepFM front end in one launch: packed-table gather, fm1, fm2 and the
 *                      first deep layer (the deep input never reaches HBM)  deepfm.py:100-112,122-142
 *   rk_deepfm_forward  DeepFM.forward() in one launch at configs[1]'s shape   deepfm.py:121-151
 *   rk_eval_batch, rk_auc  evaluate(): loss / accuracy / AUC on the device  dcn.py:214-239
 *   rk_fwfm_forward    FwFM.forward()                        fwfm.py:114-139
 *   training (loss.backward() + optimizer.step() of the train() loops, dcn.py:196-201):
 *   rk_gemm            the Linear backward GEMMs (dX = dZ W, dW = dZ^T X, db)   dcn.py:147-150
 *   rk_gemm_wgrad      dW = dZ^T X, db over long reductions (one tile owner per row slab)
 *   rk_logit_head_backward  output_layer + sigmoid backward      dcn.py:177-179
 *   rk_dcn_cross_backward   cross_layer backward w.r.t. x0        dcn.py:46-49
 *   rk_relu_backward   ReLU backward (residual_unit's outer ReLU) deepcrossing.py:41
 *   rk_embedding_backward   nn.Embedding dense weight gradient    dcn.py:131-138,163-166
 *   rk_embedding_backward_seq  the same for a [batch, T] behaviour sequence (runs pre-summed)
 *   rk_embedding_backward_sorted  the same for long, skewed index lists (behaviour sequences)
 *                      as a sorted segment-reduce                din.py:300-303, bst.py:224
 *   rk_adam_step       torch.optim.Adam step (all tensors, one launch)  dcn.py:275
 *   rk_bn_act_train_forward / rk_bn_act_backward  Linear -> BatchNorm1d (train) -> ReLU -> Dropout
 *                      and its backward                       deepfm.py:100-109
 *   rk_fm_backward, rk_fm_combine_backward  FM and final_layer + sigmoid backward  deepfm.py:122-151
 *   rk_rng_next, rk_dropout_mask  dropout stream counter / explicit mask
 *   rk_dice_train_forward / rk_dice_backward  Dice with batch statistics and its backward  din.py:26-36
 *   rk_prelu_train_forward / rk_prelu_backward  the activation='prelu' option (nn.PReLU)  din.py:277-279
 *   rk_din_att_cross, rk_din_att_pool_forward, rk_din_att_pool_backward, rk_din_cross_fold
 *                      din_attention() train forward pieces and backward   din.py:42-84
 *   rk_row_l2norm_backward  DIN mini-batch-aware l2 term backward           din.py:318-322
 *   rk_fwfm_backward   FwFM backward (embedding rows, pair weights, bias)  fwfm.py:114-139,150-156
 *   rk_afm_pairs, rk_afm_pool_forward, rk_afm_pool_backward, rk_afm_pair_fold
 *   rk_bst_add_pos, rk_bst_gather_pos, rk_bst_attn_train_forward / _backward, rk_bst_res_dropout_ln_forward,
 *   rk_linear_res_dropout_ln (projection + residual LayerNorm fused),
 *   rk_bst_ln_backward, rk_bst_pool_ln_backward, rk_bst_pos_backward, rk_bst_leaky_dropout,
 *   rk_bst_pool / _backward
 *                      BSTTransformer train forward (activations kept) and backward  bst.py:66-91,238-241
 *                      AFM train forward (activations kept) and backward  afm.py:92-119,173
 *   rk_bn_fold         BatchNorm1d eval affine (running stats) deepfm.py:105, din.py:31,281, bst.py:208
 */
#ifndef RANKOPS_H
#define RANKOPS_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RK_ABI_VERSION 1

#define RK_OK 0
#define RK_ERR_INVALID 1     /* bad argument (shape, null pointer, limit) */
#define RK_ERR_LAUNCH 2      /* hipLaunch / hipGetLastError failure */
#define RK_ERR_RUNTIME 3     /* other HIP runtime failure */
#define RK_ERR_UNSUPPORTED 4 /* shape outside the implemented envelope */

#define RK_FLAG_INDEX_OOB 1u /* an embedding index was < 0 or >= table rows */

#define RK_ACT_NONE 0
#define RK_ACT_RELU 1
#define RK_ACT_LEAKY 2 /* LeakyReLU(slope) */
#define RK_ACT_DICE 3  /* Dice: a*(1-p)*x + p*x, p = sigmoid(x*act_scale + act_shift) */
#define RK_ACT_PRELU 4 /* PReLU(act_alpha) */

#define RK_MAX_SEGMENTS 64

/* One column block of a concatenated feature row.
 * Table segment (idx != NULL): out[b, out_col:out_col+dim] = src[idx[b*idx_stride]*src_ld : +dim]
 * Dense segment (idx == NULL): out[b, out_col:out_col+dim] = src[b*src_ld : +dim]           */
typedef struct rk_segment {
  const float* src;
  const int64_t* idx;
  int64_t idx_stride;
  int64_t src_ld;
  int64_t rows; /* table rows (bounds check); ignored for dense segments */
  int32_t dim;
  int32_t out_col;
} rk_segment;

/* Fused GEMM epilogue, applied in this order to z = x.W^T:
 *   z += bias[n]; z += residual[m, n] (+ residual_periodic[m % period, n]);
 *   z = z*pre_scale[n] + pre_shift[n];   (BatchNorm1d eval before the activation)
 *   z = act(z);
 *   z = z*post_scale[n] + post_shift[n]; (BatchNorm1d eval after the activation: DIN)
 * then the optional row epilogues (need the whole row in one workgroup, N <= 256):
 *   LayerNorm over n (ln_gamma/ln_beta, ln_eps);
 *   pool: pool_out[g, n] = sum over rows m of group g (pool_rows consecutive rows),
 *         divided by pool_len[g] when pool_mean;
 *   head: logit[m] = sum_n z[m,n]*head_w[n] + head_b[0] (+ head_partial[m]);
 *         DeepFM combine when fm1 != NULL: head_aux[m] = logit (deep logit),
 *         logit = final_w[0]*fm1[m] + final_w[1]*fm2[m] + final_w[2]*deep + final_b[0];
 *         head_prob[m] = sigmoid(logit).
 * y may be NULL when only row-epilogue outputs are wanted.                              */
typedef struct rk_epilogue {
  const float* bias;
  const float* residual;
  int64_t ld_residual;
  const float* residual_periodic;
  int32_t residual_period;
  const float* pre_scale;
  const float* pre_shift;
  int32_t act;
  float slope;
  const float* act_scale;
  const float* act_shift;
  const float* act_alpha;
  int32_t act_alpha_len;
  const float* post_scale;
  const float* post_shift;
  const float* ln_gamma;
  const float* ln_beta;
  float ln_eps;
  int32_t has_ln;
  float* pool_out;
  int64_t ld_pool;
  int32_t pool_rows;
  int32_t pool_mean;
  const int64_t* pool_len;
  const float* head_w;
  const float* head_b;
  const float* head_partial;
  const float* fm1;
  const float* fm2;
  const float* final_w;
  const float* final_b;
  float* head_logit;
  float* head_prob;
  float* head_aux;
} rk_epilogue;

/* One hidden layer of a fused MLP tail (rk_mlp_forward): y = act(x.W^T + bias) with the same
 * element-wise epilogue order as rk_epilogue; `residual` adds the input of the previous layer
 * (DeepCrossing's ReLU(x + L2(ReLU(L1 x))), deepcrossing.py:37-41).                        */
#define RK_MLP_MAX_LAYERS 8
typedef struct rk_mlp_layer {
  const float* w; /* [n, K] row-major */
  int64_t ldw;
  int32_t n;
  int32_t act;
  float slope;
  int32_t residual;
  const float* bias;
  const float* pre_scale;
  const float* pre_shift;
  const float* act_scale;
  const float* act_shift;
  const float* act_alpha;
  int32_t act_alpha_len;
  const float* post_scale;
  const float* post_shift;
  float* store; /* optional: this layer's activations also written to store[m * ld_store + n]
                   (the training forward keeps them for the backward) */
  int64_t ld_store;
} rk_mlp_layer;

/* ---- runtime ---- */
int32_t rk_abi_version(void);
/* Provenance of this build: "src=<sha256[:16] of the sources> arch=<gfx> extra=<flags>". */
const char* rk_build_info(void);
const char* rk_last_error(void);
int rk_init(int32_t device);
/* Reads (and optionally clears) the device flag word; synchronises the device. */
int rk_error_flags(int32_t device, uint32_t* flags, int32_t reset);

/* ---- embedding gather / interaction kernels ---- */
int rk_concat_gather(const rk_segment* segs, int32_t nseg, int64_t batch, float* out,
                     int64_t ld_out, void* stream);

/* x0 = concat(segs); x_0 = xl_in (or x0 when NULL); x_{l+1} = x0*(x_l.w_l) + b_l + x_l.
 * Optional outputs: x0 (the gathered row), xl_out (x_L), cross_partial = x_L.head_w.      */
int rk_dcn_cross(const rk_segment* segs, int32_t nseg, int64_t batch, int32_t width,
                 const float* cross_w, const float* cross_b, int32_t num_layers,
                 const float* head_w, float* x0, int64_t ld_x0, const float* xl_in,
                 int64_t ld_xl_in, float* xl_out, int64_t ld_xl_out, float* cross_partial,
                 void* stream);

/* Segments are either all embedding tables (idx != NULL) or all dense (row b of src); dim/4 a
 * power of two, dim <= 256, at most 32 fields. */
int rk_fm_gather(const rk_segment* second_order, const rk_segment* first_order,
                 int32_t num_fields, int32_t dim, int64_t batch, float* deep_in,
                 int64_t ld_deep, float* fm1, float* fm2, void* stream);

/* One field's DeepFM tables packed into one row-major [rows, ld_out] table (ld_out % 4 == 0,
 * ld_out >= dim + 1): second-order row at columns 0..dim-1, first-order weight at column dim,
 * zero padding.  Replaces the pair nn.Embedding(V, dim) + nn.Embedding(V, 1) of one field
 * (deepfm.py:90-98) as the storage the eval gather reads; a layout pass run once per weight
 * version (the host layer caches it like the packed MLP weights).                            */
int rk_fm_pack_table(const float* second, int64_t ld_second, const float* first, int64_t ld_first,
                     int64_t rows, int32_t dim, float* out, int64_t ld_out, void* stream);

/* rk_fm_gather over packed tables (deepfm.py:122-142): segment f = {packed table of field f,
 * its [B] int64 indices (unit stride), src_ld = the packed row stride, rows, dim, out_col}.  One
 * contiguous row read per (sample, field) gives both embedding orders.                          */
int rk_fm_gather_packed(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch,
                        float* deep_in, int64_t ld_deep, float* fm1, float* fm2, void* stream);

int rk_din_attention(const float* query, int64_t ld_query, const float* key_table,
                     int64_t key_rows, int64_t ld_key, const int64_t* seq, int64_t ld_seq,
                     int32_t T, const int64_t* seq_len, int64_t batch, int32_t H,
                     const float* w1, const float* b1, const float* w2, const float* b2,
                     const float* w3, const float* b3, int32_t use_softmax, float* out,
                     int64_t ld_out, void* stream);

/* din_attention(query, keys, keys_length, is_softmax) with a dense history tensor: key row t of
 * sample b at keys + b * ld_keys_b + t * ld_keys_t (16-B aligned rows).  H in {8,16,32,64}.   */
int rk_din_attention_dense(const float* query, int64_t ld_query, const float* keys, int64_t ld_keys_b,
                           int64_t ld_keys_t, int32_t T, const int64_t* keys_length, int64_t batch,
                           int32_t H, const float* w1, const float* b1, const float* w2,
                           const float* b2, const float* w3, const float* b3, int32_t use_softmax,
                           float* out, int64_t ld_out, void* stream);

/* Dice (din.py:26-36) in eval: p = sigmoid(x * bn_scale + bn_shift) with the BatchNorm folded
 * by rk_bn_fold, y = alpha * (1 - p) * x + p * x;  x, y: [rows, n].                          */
int rk_dice_forward(const float* x, int64_t ldx, int64_t rows, int32_t n, const float* bn_scale,
                    const float* bn_shift, const float* alpha, float* y, int64_t ldy, void* stream);

/* out_scalar = scale * mean_r ||x[r, col0:col0+ncols]||_2, deterministic two-stage sum;
 * workspace: RK_L2_WORKSPACE floats of device scratch.                                   */
#define RK_L2_WORKSPACE 512
int rk_row_l2norm_mean(const float* x, int64_t ld, int64_t rows, int32_t col0, int32_t ncols,
                       float scale, float* workspace, float* out_scalar, void* stream);

/* Whole DIN eval forward (din.py:294-323) in one launch:
 *   row[b] = concat(row_segs)  (width <= 255; target query at q_col, attention written at att_col)
 *   row[b, att_col:+H] = din_attention(row[b, q_col:+H], key_table[seq[b]], seq_len[b])
 *   head outputs = fcn layers (rk_mlp_layer, packed) + head (head_w/head_b/head_logit/head_prob)
 *   l2_out = l2_scale * mean_b ||row[b, l2_col0:width]||_2 when l2_out != NULL, finished in
 *     the same launch by the last workgroup.  l2_workspace: ceil(batch/16) floats of partials
 *     followed by one uint32 counter that must be 0 before the first call (the kernel leaves it
 *     0 again; keep one workspace per stream).  H in {8, 16, 32}.                          */
int rk_din_forward(const rk_segment* row_segs, int32_t nseg, int32_t width, int32_t q_col,
                   int32_t att_col, const float* key_table, int64_t key_rows, int64_t ld_key,
                   const int64_t* seq, int64_t ld_seq, int32_t T, const int64_t* seq_len,
                   int64_t batch, int32_t H, const float* w1, const float* b1, const float* w2,
                   const float* b2, const float* w3, const float* b3, int32_t use_softmax,
                   const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head,
                   int32_t l2_col0, float l2_scale, float* l2_workspace, float* l2_out,
                   const float* att_image, void* stream);

/* att_image (optional, NULL = split in the kernel from w1..w3): the attention weights pre-split
 * into the kernel's LDS layout by rk_din_pack_attention (rk_din_attention_image_floats(H)
 * floats, 16-B aligned), so the launch stages them with one round of coalesced copies.  The
 * layout splits W1 = [W1a | W1b | W1c | W1d] over [q, k, q-k, q*k] (din.py:56-64): WK = W1b - W1c,
 * WQK = W1d, WQ = W1a + W1c, then W2, b1, b2, w3 (b3 is read from its pointer).              */
int64_t rk_din_attention_image_floats(int32_t H);
int rk_din_pack_attention(const float* w1, const float* b1, const float* w2, const float* b2,
                          const float* w3, int32_t H, float* image, void* stream);

/* rk_din_forward with phase B's epilogue-parameter image packed by rk_mlp_pack_epilogue from the
 * same layer stack (NULL: resolved per column at launch, as rk_din_forward): the kernel copies it
 * into LDS by LDS-DMA after the attention phase.  Ignored when phase B does not run on the
 * compiled [512, 256, 128] plan.  Same outputs, bit for bit.                                  */
int rk_din_forward_ex(const rk_segment* row_segs, int32_t nseg, int32_t width, int32_t q_col,
                      int32_t att_col, const float* key_table, int64_t key_rows, int64_t ld_key,
                      const int64_t* seq, int64_t ld_seq, int32_t T, const int64_t* seq_len,
                      int64_t batch, int32_t H, const float* w1, const float* b1, const float* w2,
                      const float* b2, const float* w3, const float* b3, int32_t use_softmax,
                      const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head,
                      int32_t l2_col0, float l2_scale, float* l2_workspace, float* l2_out,
                      const float* att_image, const float* epi_image, void* stream);

/* A prepared rk_din_forward: the same arguments, validated once, launched later by
 * rk_din_plan_launch on any stream at the cost of one kernel launch — the one-kernel analogue of
 * a captured hipGraph without the graph's per-replay launch gap (~9 us on this forward).  Like a
 * graph, a plan binds the pointers it was made with: keep every buffer alive, and make a new plan
 * after the weights move or their packed images are rebuilt.                                  */
int rk_din_forward_plan(const rk_segment* row_segs, int32_t nseg, int32_t width, int32_t q_col,
                        int32_t att_col, const float* key_table, int64_t key_rows, int64_t ld_key,
                        const int64_t* seq, int64_t ld_seq, int32_t T, const int64_t* seq_len,
                        int64_t batch, int32_t H, const float* w1, const float* b1, const float* w2,
                        const float* b2, const float* w3, const float* b3, int32_t use_softmax,
                        const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head,
                        int32_t l2_col0, float l2_scale, float* l2_workspace, float* l2_out,
                        const float* att_image, void** plan);
int rk_din_plan_launch(const void* plan, void* stream);
void rk_din_plan_destroy(void* plan);
/* Binds the plan's phase-B epilogue-parameter image, packed by rk_mlp_pack_epilogue from the same
 * layer stack (NULL unbinds): its launches then copy it into LDS by LDS-DMA after the attention
 * phase instead of resolving every column's bias / BatchNorm / Dice parameters at launch.
 * RK_ERR_UNSUPPORTED for a plan without a streamed phase B.                                     */
int rk_din_plan_set_epilogue_image(void* plan, const float* image);

int rk_afm_forward(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch,
                   const float* dense, int64_t ld_dense, int32_t num_dense,
                   const float* dense_w, const float* dense_b, const float* att_w,
                   const float* att_b, int32_t att_factor, const float* att_h,
                   const float* att_hb, const float* p_w, const float* p_b, float* logit,
                   float* prob, void* stream);

int rk_bst_attention(const float* qkv, int64_t ld_qkv, int64_t batch, int32_t T,
                     int32_t d_model, int32_t heads, const int64_t* seq_len, float* ctx,
                     int64_t ld_ctx, void* stream);
/* key_padding_mask: [batch, ld_mask] bytes, nonzero = masked key (torch bool); NULL = none.
 * A row with every key masked gives NaN context, as torch's softmax over all -inf.          */
int rk_bst_attention_masked(const float* qkv, int64_t ld_qkv, int64_t batch, int32_t T,
                            int32_t d_model, int32_t heads, const uint8_t* key_padding_mask,
                            int64_t ld_mask, float* ctx, int64_t ld_ctx, void* stream);

/* The whole BSTModel eval forward at the reference script's d_model 16 (bst.py:192, 216-247) in one
 * launch: the DNN row [dense | category embeddings] gathered by `row_segs` over columns
 * [0, width), every transformer block and the pooling (as rk_bst_forward_blocks at d_model 16)
 * written to columns [width, width + 16), then `layers` (packed by rk_mlp_pack_weight, BatchNorm
 * folded, LeakyReLU) and the output layer + sigmoid of `head` (head_w/head_b/head_logit/head_prob).
 * Envelope: heads 1/2/4/8, 1 <= T <= 64, nblocks <= 4, nseg <= 8, width + 16 in (64, 128] with
 * hidden units [512, 256, 128] (else RK_ERR_UNSUPPORTED: rk_concat_gather +
 * rk_bst_forward_blocks + rk_mlp_forward compute the same).                                  */
int rk_bst_small_forward(const rk_segment* row_segs, int32_t nseg, int32_t width, const float* table,
                         int64_t table_rows, int64_t ld_table, const int64_t* seq, int64_t ld_seq,
                         int32_t T, const int64_t* seq_len, int64_t batch, int32_t heads,
                         int32_t nblocks, const float* const* block_params,
                         const float* block_scalars, int32_t pool_mean, const rk_mlp_layer* layers,
                         int32_t nlayers, const rk_epilogue* head, void* stream);

/* Every transformer block of BSTModel.forward plus the pooling (bst.py:66-91, 224-241) in one
 * launch, one workgroup per sample, activations kept in LDS:
 *   x = table[seq[b, :T]];  for each block i: x = block_i(x)  (mask keys >= seq_len[b])
 *   pool_out[b, 0:128] = sum_t x[t]  (/ seq_len[b] when pool_mean)
 * block_params: host array of 17 device pointers per block, in this order:
 *   pos[max_len,128], wq, bq, wk, bk, wv, bv, wo, bo, w1 (ffn.0), b1, w2 (ffn.3), b2,
 *   ln1_gamma, ln1_beta, ln2_gamma, ln2_beta   (nn.Linear [out,in] row-major, 16-B aligned)
 * block_scalars: host array of 3 floats per block: ln1_eps, ln2_eps, leaky slope.
 * Envelope: d_model 128, heads 4, 1 <= T <= 64, nblocks <= 4 (else RK_ERR_UNSUPPORTED).
 * Replaces the rk_linear x5 + rk_bst_attention sequence of one block.                     */
int rk_bst_forward_blocks(const float* table, int64_t table_rows, int64_t ld_table,
                          const int64_t* seq, int64_t ld_seq, int32_t T, const int64_t* seq_len,
                          int64_t batch, int32_t d_model, int32_t heads, int32_t nblocks,
                          const float* const* block_params, const float* block_scalars,
                          float* pool_out, int64_t ld_pool, int32_t pool_mean, void* stream);
/* rk_bst_forward_blocks (d_model 128 only) with the six projection weights of every block (wq, wk,
 * wv, wo, w1, w2) in rk_bst_pack_block_weight's layout; same outputs, bit for bit.            */
int rk_bst_forward_blocks_packed(const float* table, int64_t table_rows, int64_t ld_table,
                                 const int64_t* seq, int64_t ld_seq, int32_t T,
                                 const int64_t* seq_len, int64_t batch, int32_t d_model,
                                 int32_t heads, int32_t nblocks, const float* const* block_params,
                                 const float* block_scalars, float* pool_out, int64_t ld_pool,
                                 int32_t pool_mean, void* stream);
/* A [128, 128] projection weight (nn.Linear [out, in], contiguous) in the order the block kernel's
 * 32x32x2 MFMA lanes load it: float 4096 j + 1024 g + 256 c + 4 l + e of `out` (16384 floats) is
 * W[32 j + l % 32][32 g + 8 c + 4 (l / 32) + e] — each wave load one contiguous 1 KiB.  Not in place. */
int rk_bst_pack_block_weight(const float* w, float* out, void* stream);

/* ---- dense layers ---- */
int rk_linear(const float* x, int64_t ldx, const float* x_periodic, int32_t x_period,
              const float* w, int64_t ldw, int64_t M, int32_t N, int32_t K,
              const rk_epilogue* ep, float* y, int64_t ldy, void* stream);

/* Packed layout of a fused-MLP weight: pad64(n) x pad64(k) floats, zero filled (rows and K
 * padded to 64 so the kernel's loads are unconditional aligned float4s), fragment-major: the
 * 16-column x 16-k block (t, c) is 256 contiguous floats in the order the MFMA lanes load it
 * (float i of the block = W[16t + ((i>>2)&15)][16c + 4((i>>2)>>4) + (i&3)]).  Pack once at load
 * time; rows/cols of rk_mlp_packed_size give the size and ldw = cols.                       */
int rk_mlp_packed_size(int32_t n, int32_t k, int64_t* rows, int64_t* cols);
int rk_mlp_pack_weight(const float* w, int64_t ldw, int32_t n, int32_t k, float* out, void* stream);

/* The per-column epilogue parameters of a layer stack with a compiled streamed plan (hidden units
 * [512, 256, 128] over an input of <= 256, or [256, 128] over 512), resolved and laid out as the
 * streamed tail's LDS image ([column][8] floats: bias, pre scale/shift, Dice scale/shift, slope,
 * post scale/shift).  rk_mlp_epilogue_image_floats: its size in floats (0: no compiled plan).    */
int rk_mlp_epilogue_image_floats(const rk_mlp_layer* layers, int32_t nlayers, int32_t K0);
int rk_mlp_pack_epilogue(const rk_mlp_layer* layers, int32_t nlayers, int32_t K0, float* out, void* stream);

/* Whole MLP tail in one launch: layers[0..nlayers) on x [M, K0] (K0 <= 1024, widths <= 512;
 * every layers[l].w packed by rk_mlp_pack_weight, ldw = pad64(K)), then the head of `head`
 * (head_w/head_b/head_partial/fm combine/head_logit/head_prob/head_aux) when head->head_w is
 * set, else the last activation is written to y.                                          */
int rk_mlp_forward(const float* x, int64_t ldx, int64_t M, int32_t K0, const rk_mlp_layer* layers,
                   int32_t nlayers, const rk_epilogue* head, float* y, int64_t ldy, void* stream);

/* rk_concat_gather + rk_mlp_forward in one launch (eval, generic tail with residual layers, a head):
 * each 16-row workgroup gathers its rows' `width` columns from the segments (rk_concat_gather's
 * column map: the last covering segment wins, uncovered columns are zero, out-of-range rows are
 * zero and raise RK_FLAG_INDEX_OOB) straight into the first layer's LDS buffer.  nseg <= 16,
 * width <= 256, head->head_w required, no layer stores.  Replaces the reference's
 * torch.cat(dense, embeddings) + residual stack + output layer (deepcrossing.py:146-163).       */
int rk_mlp_forward_gather(const rk_segment* segs, int32_t nseg, int32_t width, int64_t batch,
                          const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head, void* stream);

/* Whole DCN eval forward in one launch (DCNModel.forward, dcn.py:161-180): gather of the row from
 * segs (out_col ascending from 0, at most 8 segments, width <= 256), num_layers cross layers
 * (weights [L, width] as rk_dcn_cross), the MLP tail as rk_mlp_forward (layers packed) and the head:
 * logit = x_L . cross_head_w + (h . head->head_w + head->head_b), prob = sigmoid(logit), written to
 * head->head_logit / head->head_prob.  cross_head_w = output_layer.weight[0, :width].           */
int rk_dcn_forward(const rk_segment* segs, int32_t nseg, int64_t batch, int32_t width, const float* cross_w,
                   const float* cross_b, int32_t num_layers, const float* cross_head_w,
                   const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head, void* stream);

/* One MLP layer as a 2D-tiled GEMM (64-row x 128-column tiles): y[M, n] = epilogue(x . W^T) with
 * W packed by rk_mlp_pack_weight (ldw = pad64(K)) and the element-wise part of the rk_mlp_layer
 * epilogue (bias, BatchNorm affines, activation; no residual).  For a wide first layer
 * (deepfm.py:100-112, 960 -> 512) it reads every weight 64 times per 4096 rows instead of 256. */
int rk_linear_tiled(const float* x, int64_t ldx, int64_t M, int32_t K, const rk_mlp_layer* layer,
                    float* y, int64_t ldy, void* stream);

/* The DeepFM eval front end as one 2D-tiled launch (deepfm.py:122-142 then deepfm.py:100-112 for the
 * first deep layer): for every sample b, fm1[b] = sum_f first-order weight, fm2[b] = 0.5 sum_d
 * ((sum_f e_f)^2 - sum_f e_f^2)[d], and y[b, :] = epilogue(concat_f(e_f) . W^T) with
 * e_f = row idx_f[b] of field f's packed table (rk_fm_pack_table layout, as rk_fm_gather_packed:
 * segment f = {packed table, unit-stride index, rows, dim, src_ld >= dim + 1, out_col = f * dim}).
 * A segment with idx = NULL is a dense block of packed rows (row b at src + b * src_ld, b < batch):
 * the rows ShardedDeepFM receives from a field's owner rank over the row all-to-all.
 * The layer is packed by rk_mlp_pack_weight for K = num_fields * dim (no residual).  dim a power of
 * two in [4, 256], num_fields <= 32.  The concatenated deep input is staged in LDS only.
 * Out-of-range indices read zero rows and raise RK_FLAG_INDEX_OOB.                               */
int rk_fm_linear_packed(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch,
                        const rk_mlp_layer* layer, float* y, int64_t ldy, float* fm1, float* fm2,
                        void* stream);

/* The whole DeepFM eval forward in one launch (DeepFM.forward, deepfm.py:121-151): fields as for
 * rk_fm_linear_packed (packed tables with unit-stride indices, or dense blocks of packed rows),
 * layers = the three deep layers (Linear + BatchNorm folded + ReLU, deepfm.py:100-112), head =
 * deep_output_layer (head_w, head_b) with final_layer (final_w, final_b) and the outputs
 * head_logit / head_prob / head_aux (the deep logit); fm1 / fm2 [batch] are written (its own
 * fm1 / fm2 fields are ignored).  Compiled plan: 960 -> 512 -> 256 -> 128 (configs[1]: 30 fields
 * x 32); other shapes return RK_ERR_UNSUPPORTED (use rk_fm_linear_packed + rk_mlp_forward). */
int rk_deepfm_forward(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch,
                      const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head, float* fm1,
                      float* fm2, void* stream);

/* ---- table-sharded DeepFM, the local steps around the all-to-alls (rankops.sharded; the
 * reference's DeepFM.forward, deepfm.py:121-151, runs on one device) ---- */
/* The index all-to-all's send buffer in one launch: slot q (fields in owner-major order) copies
 * idx[q][0..batch) as int32 to out[base[q] + b * stride[q]] (base = batch * start_r + j,
 * stride = F_r: blocks [r][b][f_r]).  An index outside [0, 2^31) is sent as -1, so the owner's
 * rk_shard_gather_rows writes a zero row and raises RK_FLAG_INDEX_OOB instead of wrapping. */
int rk_shard_pack_indices(const int64_t* const* idx, const int64_t* base, const int32_t* stride,
                          int32_t num_fields, int64_t batch, int32_t* out, void* stream);
/* The row all-to-all's send buffer for samples [b0, b0 + bc) of every source: out[s][b'][j][0..row_floats)
 * = packed row idx[(s * source_batch + b0 + b') * num_fields + j] of table j (tables[j]: packed
 * rk_fm_pack_table layout, src_ld >= row_floats, 16-B aligned; idx / out / dim fields unused).
 * Out-of-range indices write zero rows and raise RK_FLAG_INDEX_OOB. */
int rk_shard_gather_rows(const rk_segment* tables, int32_t num_fields, int32_t row_floats, const int32_t* idx,
                         int32_t num_sources, int64_t source_batch, int64_t b0, int64_t bc, float* out,
                         void* stream);

/* The split wire format of the row exchange (round 5): out per source s = [bc][j][dim] second-order
 * rows straight from second[j] (the [V, dim] nn.Embedding weight, src_ld >= dim, 16-B aligned), then
 * pad4(bc) floats: per sample the sum over j = 0..num_fields-1 (in order) of the first-order weight
 * first[j].src[row * first[j].src_ld].  dim % 4 == 0.  Out-of-range indices give zero
 * rows / weights and raise RK_FLAG_INDEX_OOB. */
int rk_shard_gather_rows_split(const rk_segment* second, const rk_segment* first, int32_t num_fields,
                               int32_t dim, const int32_t* idx, int32_t num_sources, int64_t source_batch,
                               int64_t b0, int64_t bc, float* out, void* stream);
/* rk_deepfm_forward with the first-order weight of field f read from first[f][r * first_ld[f]]
 * (r = the field's index, or the sample for a dense block) instead of the packed row's column dim;
 * first[f] == NULL contributes 0 (ShardedDeepFM's split rows: the owner's partial sum on its first
 * field).  Rows then need src_ld >= dim only. */
int rk_deepfm_forward_fo(const rk_segment* fields, const float* const* first, const int64_t* first_ld,
                         int32_t num_fields, int32_t dim, int64_t batch, const rk_mlp_layer* layers,
                         int32_t nlayers, const rk_epilogue* head, float* fm1, float* fm2, void* stream);

/* FwFM.forward (fwfm.py:114-139): per sample, logit = sum_f linear[f] row + sum_{i<j} field_weight[p]
 * <embeddings[i] row, embeddings[j] row> + bias[0] (p runs i-major over i < j, fwfm.py:129-136),
 * prob = sigmoid(logit).  embeddings[f]: table segments of width dim (out_col ignored);
 * linear[f]: the first-order tables (dim 1).  2 <= num_fields <= 16, 1 <= dim <= 256 (dim > 64
 * needs 16-byte aligned rows).  logit may be NULL.  Out-of-range indices read zero rows and raise
 * RK_FLAG_INDEX_OOB.                                                                             */
int rk_fwfm_forward(const rk_segment* embeddings, const rk_segment* linear, int32_t num_fields,
                    int32_t dim, int64_t batch, const float* field_weight, const float* bias,
                    float* logit, float* prob, void* stream);

/* ---- training (§8(f) #2) ---------------------------------------------------------------- */
/* C[m, n] (+)= sum_r opA(m, r) * opB(n, r) on FP32 MFMA, with
 *   opA(m, r) = trans_a ? A[r*lda + m] : A[m*lda + r], times [A_mask(m, r) > 0] when A_mask
 *               (same layout and lda as A: the ReLU backward dz = dh * [h > 0]) is non-NULL;
 *   opB(n, r) = trans_b ? B[r*ldb + n] : B[n*ldb + r];
 *   row_sums[m] (+)= sum_r opA(m, r) when non-NULL (bias gradients).
 * nn.Linear backward: dX = dZ W  -> rk_gemm(0, 1, B, K, N, dZ, ldz, mask, W, K, dX, ...);
 *                     dW = dZ^T X -> rk_gemm(1, 1, N, K, B, dZ, ldz, mask, X, ldx, dW, K, db, ...).
 * split <= 0 picks a reduction split (float atomics) that fills the GPU; accumulate = 0
 * overwrites C / row_sums.                                                                  */
int rk_gemm(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t R, const float* A,
            int64_t lda, const float* A_mask, const float* B, int64_t ldb, float* C, int64_t ldc,
            float* row_sums, int32_t accumulate, int32_t split, void* stream);

/* Weight-gradient GEMM (every nn.Linear's dW / db in loss.backward(), e.g. bst.py:59-64,73-90,
 * dcn.py:147-150): C[n, k] (+)= sum_r opA(r, n) B[r * ldb + k] and row_sums[n] (+)= sum_r opA(r, n),
 * opA(r, n) = A[r * lda + n] (times [A_mask[r * lda + n] > 0] when A_mask != NULL), for a long
 * reduction R.  Same result as rk_gemm(1, 1, N, K, R, ...) but each 128 x 128 output tile is owned
 * by one workgroup per row slab and the slabs' partials are summed in a fixed order
 * (deterministic).  Needs N, K, lda, ldb, ldc % 4 == 0 and 16-B aligned pointers
 * (RK_ERR_UNSUPPORTED otherwise); workspace: rk_gemm_wgrad_workspace_floats(N, K, R) floats.  */
int rk_gemm_wgrad(int64_t N, int64_t K, int64_t R, const float* A, int64_t lda, const float* A_mask,
                  const float* B, int64_t ldb, float* C, int64_t ldc, float* row_sums,
                  int32_t accumulate, float* workspace, int64_t workspace_floats, void* stream);
int64_t rk_gemm_wgrad_workspace_floats(int64_t N, int64_t K, int64_t R);

/* out[i] (+)= dy[i] * [y[i] > 0] over n contiguous floats (ReLU backward from its output; the
 * residual path of residual_unit, deepcrossing.py:41).                                        */
int rk_relu_backward(const float* dy, const float* y, float* out, int64_t n, int32_t accumulate,
                     void* stream);

/* Linear(ka + kb, 1) + sigmoid head over rows [xa | xb] (kb may be 0):
 * g = dlogit + dprob * (1 - prob) * prob (either grad may be NULL); dxa/dxb = g w (NULL: not
 * written); dw[ka + kb] = sum_b g x; db[0] = sum_b g (both overwritten); g_out[b] = g.       */
int rk_logit_head_backward(const float* dlogit, const float* dprob, const float* prob, int64_t batch,
                           const float* xa, int64_t ld_xa, int32_t ka, const float* xb, int64_t ld_xb,
                           int32_t kb, const float* w, float* dxa, int64_t ld_dxa, float* dxb,
                           int64_t ld_dxb, float* dw, float* db, float* g_out, void* stream);

/* nn.Embedding gradient of a behaviour sequence without sorting (bst.py:224): grad[idx[b*stride + t]]
 * += dx[b*T + t, out_col : out_col + dim] for b < batch, t < T (grad->idx_stride = the row stride
 * of the [batch, T] index matrix).  Runs of equal consecutive ids in a sample (a padded tail) are
 * summed before their atomics.  Needs an even dim <= 128 and 8-B aligned rows
 * (RK_ERR_UNSUPPORTED otherwise: use rk_embedding_backward_sorted).                            */
int rk_embedding_backward_seq(const rk_segment* grad, int64_t batch, int32_t T, const float* dx,
                              int64_t ld_dx, void* stream);
/* Sorted segment-reduce form of rk_embedding_backward for ONE table segment and a long index list
 * with hot rows (padded behaviour sequences): grad[idx[i]] += dx[i, out_col:+dim] for i < n, via a
 * radix sort of the indices and one atomic per (distinct row in a 64-position chunk, column).
 * workspace: rk_embedding_backward_sorted_workspace_size(n) bytes.  Out-of-range indices are skipped
 * and raise RK_FLAG_INDEX_OOB.                                                               */
int rk_embedding_backward_sorted_workspace_size(int64_t n, int64_t* bytes);
int rk_embedding_backward_sorted(const rk_segment* grad, int64_t n, const float* dx, int64_t ld_dx,
                                 void* workspace, int64_t ws_bytes, void* stream);

/* Gradient of num_layers cross layers (rk_dcn_cross's stack, weights [L, width]) w.r.t. x0 given
 * dL/dx_L; written to dx0 (added when accumulate).  width <= 256, num_layers <= 8.           */
int rk_dcn_cross_backward(const float* x0, int64_t ld_x0, int64_t batch, int32_t width,
                          const float* cross_w, const float* cross_b, int32_t num_layers,
                          const float* dxl, int64_t ld_dxl, float* dx0, int64_t ld_dx0,
                          int32_t accumulate, void* stream);

/* Dense nn.Embedding weight gradients: for every table segment (src = the [rows, dim] gradient
 * buffer, written with float atomics — zero it first), grad[idx[b]] += dx[b, out_col:+dim].
 * Dense segments (idx == NULL) are skipped; out-of-range indices raise RK_FLAG_INDEX_OOB.   */
int rk_embedding_backward(const rk_segment* grads, int32_t nseg, int64_t batch, const float* dx,
                          int64_t ld_dx, void* stream);

/* Dropout streams: *slot = *counter; *counter += 1 (one thread, stream-ordered, graph-safe). */
int rk_rng_next(int64_t* counter, int64_t* slot, void* stream);

/* The keep mask a dropout stream draws, as the multiplier it applies: out[b*n + j] = 1/(1-p) or 0.
 * keep(i) = mix64(seed, *stream_slot, i) >= p * 2^32 (splitmix64 finaliser; not torch's Philox). */
int rk_dropout_mask(uint64_t seed, const int64_t* stream_slot, int64_t batch, int32_t n,
                    double dropout_p, float* out, void* stream);

/* y = Dropout_p(act(BatchNorm1d_train(z + bias))) over [batch, n] (deepfm.py:101-108; BST's
 * LeakyReLU units bst.py:207-211): batch statistics (biased variance) in fp64, save_mean /
 * save_invstd written, running_mean / running_var updated with momentum and the unbiased variance
 * (both may be NULL); batch_norm = 0 skips the normalisation, act = RK_ACT_NONE / RK_ACT_RELU /
 * RK_ACT_LEAKY (negative slope `slope`), dropout_p = 0 the dropout.  workspace: 2n doubles.
 * gamma / beta may be NULL (affine = False).                                                  */
int rk_bn_act_train_forward(const float* z, int64_t ldz, int64_t batch, int32_t n, const float* bias,
                            int32_t batch_norm, const float* gamma, const float* beta, float eps,
                            float momentum, float* running_mean, float* running_var,
                            double* workspace, float* save_mean, float* save_invstd, int32_t act,
                            float slope, double dropout_p, uint64_t seed, const int64_t* stream_slot, float* y,
                            int64_t ldy, void* stream);

/* Backward of rk_bn_act_train_forward given dy: dz (gradient w.r.t. z, i.e. the Linear output
 * before its bias), dgamma / dbeta (may be NULL).  Same seed / stream slot as the forward.    */
int rk_bn_act_backward(const float* dy, int64_t lddy, const float* z, int64_t ldz, int64_t batch,
                       int32_t n, const float* bias, int32_t batch_norm, const float* gamma,
                       const float* beta, const float* save_mean, const float* save_invstd,
                       int32_t act, float slope, double dropout_p, uint64_t seed,
                       const int64_t* stream_slot,
                       double* workspace, float* dz, int64_t lddz, float* dgamma, float* dbeta,
                       void* stream);

/* DeepFM FM backward (deepfm.py:122-140): out[b, f*dim + d] = d_deep[b, f*dim + d] +
 * dfm2[b] * (S_d - e_{f,d}), e = the saved deep input (concatenated second-order rows),
 * S_d = sum_f e_{f,d}.  d_deep / dfm2 may be NULL (zero).                                      */
int rk_fm_backward(const float* deep_in, int64_t ld_in, const float* d_deep, int64_t ld_d,
                   const float* dfm2, int64_t batch, int32_t num_fields, int32_t dim, float* out,
                   int64_t ld_out, void* stream);

/* final_layer(cat[fm1, fm2, deep]) + sigmoid backward (deepfm.py:147-150) with incoming grads of
 * all five outputs (each may be NULL): g = dtotal + dprob (1 - p) p; dfm1 = dfm1_in + g w0,
 * dfm2 = dfm2_in + g w1, ddeep = ddeep_in + g w2; dfinal_w[3], dfinal_b[1] overwritten.        */
int rk_fm_combine_backward(const float* dprob, const float* dtotal, const float* dfm1_in,
                           const float* dfm2_in, const float* ddeep_in, const float* prob,
                           const float* fm1, const float* fm2, const float* deep,
                           const float* final_w, int64_t batch, float* dfm1, float* dfm2,
                           float* ddeep, float* dfinal_w, float* dfinal_b, void* stream);

/* Dice (din.py:26-36) in train mode: x = z + bias, xhat = BatchNorm1d(affine=False) with the batch
 * statistics (running stats updated with momentum), y = alpha * (1 - sigmoid(xhat)) * x +
 * sigmoid(xhat) * x.  workspace: 2n doubles (forward), 3n (backward).  Backward writes dz =
 * dL/d(z + bias) and dalpha (when non-NULL).                                                  */
int rk_dice_train_forward(const float* z, int64_t ldz, int64_t batch, int32_t n, const float* bias,
                          const float* alpha, float eps, float momentum, float* running_mean,
                          float* running_var, double* workspace, float* save_mean, float* save_invstd,
                          float* y, int64_t ldy, void* stream);
int rk_dice_backward(const float* dy, int64_t lddy, const float* z, int64_t ldz, int64_t batch,
                     int32_t n, const float* bias, const float* alpha, const float* save_mean,
                     const float* save_invstd, double* workspace, float* dz, int64_t lddz,
                     float* dalpha, void* stream);

/* DIN's PReLU activation option (din.py:277-279, nn.PReLU()) in train mode: x = z + bias,
 * y = x > 0 ? x : a x, with one shared weight (num_weights == 1, the reference's nn.PReLU()) or
 * one per column (num_weights == n).  Backward writes dz = dL/d(z + bias) and dweight[num_weights]
 * (when non-NULL); workspace: num_weights doubles.                                              */
int rk_prelu_train_forward(const float* z, int64_t ldz, int64_t batch, int32_t n, const float* bias,
                           const float* weight, int32_t num_weights, float* y, int64_t ldy, void* stream);
int rk_prelu_backward(const float* dy, int64_t lddy, const float* z, int64_t ldz, int64_t batch,
                      int32_t n, const float* bias, const float* weight, int32_t num_weights,
                      double* workspace, float* dz, int64_t lddz, float* dweight, void* stream);

/* din_attention train pieces (din.py:42-84).  keys [B, T, H] = key_table[seq] (gathered), cross
 * [B*T, 4H] = [q, k, q-k, q*k] with q = x[b, q_col:+H]; the att_net layers run on rk_linear.
 * pool_forward: s = a2 . w3 + b3, masked (softmax: padded with -2^32+1, / sqrt(H)) weights saved
 * to weights [B, T], out = sum_t w_t k_t written to x[b, att_col:+H].  T <= 1024, H <= 64.
 * pool_backward: from dout = dx[b, att_col:+H]: dkeys = w_t dout (overwritten) and
 * da2 = ds_t w3 [a2 > 0].  cross_fold: d(cross) -> dq added to dx[b, q_col:+H], dkeys added.  */
int rk_din_att_cross(const float* x, int64_t ldx, int32_t q_col, const float* key_table,
                     int64_t key_rows, int64_t ld_key, const int64_t* seq, int64_t ld_seq,
                     int64_t batch, int32_t T, int32_t H, float* keys, float* cross, void* stream);
int rk_din_att_pool_forward(const float* a2, int32_t a2_width, const float* w3, const float* b3,
                            const float* keys, const int64_t* seq_len, int64_t batch, int32_t T,
                            int32_t H, int32_t use_softmax, float* weights, float* x, int64_t ldx,
                            int32_t att_col, void* stream);
int rk_din_att_pool_backward(const float* dx, int64_t lddx, int32_t att_col, const float* weights,
                             const float* keys, const float* a2, int32_t a2_width, const float* w3,
                             const int64_t* seq_len, int64_t batch, int32_t T, int32_t H,
                             int32_t use_softmax, float* dkeys, float* da2, void* stream);
int rk_din_cross_fold(const float* dcross, const float* x, int64_t ldx, int32_t q_col,
                      const float* keys, int64_t batch, int32_t T, int32_t H, float* dkeys, float* dx,
                      int64_t lddx, void* stream);

/* Backward of out = scale * mean_r ||x[r, col0:+ncols]||_2 (rk_row_l2norm_mean): called with
 * scale / rows, adds grad_out[0] * scale * x / ||x_r|| to dx[r, col0 + c] (0 for a zero row).   */
int rk_row_l2norm_backward(const float* x, int64_t ldx, int64_t rows, int32_t col0, int32_t ncols,
                           float scale, const float* grad_out, float* dx, int64_t lddx, void* stream);

/* FwFM backward from dL/dprob [B] (BCELoss on rk_fwfm_forward's probabilities, fwfm.py:150-156):
 * dz = dprob * (1 - prob) * prob -> dz [B] (the first-order tables' gradient rows),
 * d_emb[b, f*dim + c] = dz * sum_{j != f} r_{pair(f,j)} E_j[c] (scatter with rk_embedding_backward),
 * d_field_weight [F(F-1)/2] and d_bias [1] (overwritten).                                   */
int rk_fwfm_backward(const rk_segment* embeddings, int32_t num_fields, int32_t dim, int64_t batch,
                     const float* field_weight, const float* prob, const float* dprob, float* d_emb,
                     int64_t ld_demb, float* dz, float* d_field_weight, float* d_bias, void* stream);

/* AFM training (afm.py:92-119).  pairs: emb [B, F*dim] (gathered rows) and pairs [B*P, dim]
 * (P = F(F-1)/2, i-major), 2 <= F <= 16.  The attention's first layer a1 = relu(pairs W1^T + b1)
 * runs on rk_linear; pool_forward: s = a1 . w2 + b2, softmax over the P pairs (weights [B, P]),
 * ws = sum_p w_p pair_p [B, dim], logit = dense . wd + bd + ws . wp + bp, pred = sigmoid(logit)
 * (dim, num_dense <= 64; logit may be NULL).  pool_backward from dpred and/or dtotal (either may
 * be NULL): d_pairs (direct part, overwritten), da1 = d a1 [B*P, A] (masked by a1 > 0), and
 * acc = [d wd (num_dense) | d bd | d wp (dim) | d bp | d w2 (A <= 256) | d b2] (overwritten).
 * pair_fold: d_emb[b, i*dim + d] = sum_j d_pairs[b, pair(i,j), d] * emb[b, j*dim + d].          */
int rk_afm_pairs(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch, float* emb,
                 float* pairs, void* stream);
int rk_afm_pool_forward(const float* a1, int32_t att_dim, const float* w2, const float* b2,
                        const float* pairs, int32_t num_pairs, int32_t dim, const float* dense,
                        int64_t ld_dense, int32_t num_dense, const float* wd, const float* bd,
                        const float* wp, const float* bp, int64_t batch, float* weights, float* ws,
                        float* logit, float* pred, void* stream);
int rk_afm_pool_backward(const float* dpred, const float* dtotal, const float* pred,
                         const float* weights, const float* ws, const float* pairs, const float* a1,
                         int32_t att_dim, const float* w2, const float* wp, const float* dense,
                         int64_t ld_dense, int32_t num_dense, int64_t batch, int32_t num_pairs,
                         int32_t dim, float* d_pairs, float* da1, float* acc, void* stream);
int rk_afm_pair_fold(const float* d_pairs, const float* emb, int32_t num_fields, int32_t dim,
                     int64_t batch, float* d_emb, void* stream);

/* BST training (bst.py:66-91, 238-241), rows = B*T of width d:
 *   add_pos: xp[m] = x[m] + pos[m % T].
 *   attn_train_forward: per (sample, head) P = softmax(mask(Q K^T / sqrt(dh))) saved to probs (or not
 *     saved when probs == NULL; T % 4 == 0, dh % 4 == 0)
 *     [B, heads, T, T] and ctx = P V [rows, d]; qkv is [rows, 3d] = [Q | K | V].  T <= 64,
 *     d / heads <= 64.  attn_train_backward: dqkv [rows, 3d] from dctx (overwritten).
 *   res_dropout_ln_forward: r = base + Dropout_p(o) (saved), y = LayerNorm(r) (gamma, beta, eps),
 *     mean / rstd [rows] saved.  d <= 256.
 *   ln_backward: dr = LayerNorm backward of dy (overwritten), d_o = Dropout_p-masked dr (NULL:
 *     skipped), dgamma / dbeta [d] (overwritten, summed in a fixed order: workspace 1024 * d floats).
 *   pos_backward: dpos[t] += sum_b dxp[b*T + t] for t < T (the position-embedding gradient; zero dpos first).
 *   leaky_dropout: forward out = Dropout_p(LeakyReLU_slope(f)); backward (backward = 1)
 *     out = in * keep * scale * (f > 0 ? 1 : slope).
 *   pool: row[b, col:+d] = sum_t x[b*T + t] (/ seq_len[b] when mean); pool_backward broadcasts.
 * Dropout masks: the counter hash of rk_dropout_mask with index m * d + k.                      */
int rk_bst_add_pos(const float* x, const float* pos, int32_t T, int64_t rows, int32_t d, float* xp,
                   void* stream);
/* Behaviour-sequence gather + position add of the first block's train forward (bst.py:224,73-75):
 * x[m] = table[idx[m]] (out-of-range: zeros + RK_FLAG_INDEX_OOB), xp[m] = x[m] + pos[m % T, :].
 * Needs d % 4 == 0 and 16-B aligned rows (RK_ERR_UNSUPPORTED otherwise).                       */
int rk_bst_gather_pos(const float* table, int64_t rows, int64_t ld_table, const int64_t* idx,
                      int64_t n, int32_t T, int32_t d, const float* pos, float* x, float* xp,
                      void* stream);
int rk_bst_attn_train_forward(const float* qkv, int64_t batch, int32_t T, int32_t d, int32_t heads,
                              const int64_t* seq_len, float* probs, float* ctx, void* stream);
int rk_bst_attn_train_backward(const float* qkv, const float* probs, const float* dctx,
                               int64_t batch, int32_t T, int32_t d, int32_t heads, float* dqkv,
                               void* stream);
/* The O / FFN2 projection and the residual LayerNorm after it in one launch (bst.py:84-90):
 * r = base + dropout(x W^T + bias), y = LayerNorm(r) (gamma, beta, eps), mean / rstd per row, for
 * d_model = N = 128: the projection output never reaches HBM.  x [M, K] (ld ldx), W [128, K] (ld
 * ldw), base / r / y [M, 128] contiguous; K in {32, 64, 128}, 16-B aligned rows
 * (RK_ERR_UNSUPPORTED otherwise: use rk_linear + rk_bst_res_dropout_ln_forward).
 * Same dropout mask as rk_bst_res_dropout_ln_forward for the same (seed, stream slot).          */
int rk_linear_res_dropout_ln(const float* x, int64_t ldx, int64_t M, int32_t K, const float* w, int64_t ldw,
                             const float* bias, const float* base, double dropout_p, uint64_t seed,
                             const int64_t* stream_slot, const float* gamma, const float* beta, float eps,
                             float* r, float* y, float* mean, float* rstd, void* stream);
int rk_bst_res_dropout_ln_forward(const float* base, const float* o, int64_t rows, int32_t d,
                                  double dropout_p, uint64_t seed, const int64_t* stream_slot,
                                  const float* gamma, const float* beta, float eps, float* r, float* y,
                                  float* mean, float* rstd, void* stream);
int rk_bst_ln_backward(const float* dy, const float* r, const float* mean, const float* rstd,
                       const float* gamma, int64_t rows, int32_t d, double dropout_p, uint64_t seed,
                       const int64_t* stream_slot, float* dr, float* d_o, float* dgamma, float* dbeta,
                       float* workspace, int64_t workspace_floats, void* stream);
/* rk_bst_ln_backward of the last block fused with the pooling backward (bst.py:238-241): the
 * incoming gradient of row m is drow[m / T, col:col+d] (/ seq_len[m / T] when mean_pool), so the
 * [rows, d] broadcast is never written.  rows = batch * T; needs d % 4 == 0 and 16-B aligned r /
 * dr / d_o rows (drow any alignment; RK_ERR_UNSUPPORTED otherwise: use rk_bst_pool_backward +
 * rk_bst_ln_backward).                                                                         */
int rk_bst_pool_ln_backward(const float* drow, int64_t ld_row, int32_t col, int32_t T,
                            const int64_t* seq_len, int32_t mean_pool, const float* r,
                            const float* mean, const float* rstd, const float* gamma, int64_t rows,
                            int32_t d, double dropout_p, uint64_t seed, const int64_t* stream_slot,
                            float* dr, float* d_o, float* dgamma, float* dbeta, float* workspace,
                            int64_t workspace_floats, void* stream);
/* Floats rk_bst_ln_backward / rk_bst_pool_ln_backward need in `workspace` for model width d. */
int64_t rk_bst_ln_backward_workspace_floats(int32_t d);
int rk_bst_pos_backward(const float* dxp, int64_t batch, int32_t T, int32_t d, float* dpos, void* stream);
int rk_bst_leaky_dropout(const float* in, const float* f, int64_t n, float slope, double dropout_p,
                         uint64_t seed, const int64_t* stream_slot, int32_t backward, float* out,
                         void* stream);
int rk_bst_pool(const float* x, int64_t batch, int32_t T, int32_t d, const int64_t* seq_len,
                int32_t mean, float* row, int64_t ld_row, int32_t col, void* stream);
int rk_bst_pool_backward(const float* drow, int64_t ld_row, int32_t col, int64_t batch, int32_t T,
                         int32_t d, const int64_t* seq_len, int32_t mean, float* dx, void* stream);

typedef struct rk_adam_tensor {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t numel;
  float* step; /* optional device step counter (torch capturable=True): incremented on the device,
                  bias corrections formed there; give it for all tensors of a call or for none */
} rk_adam_tensor;

/* One torch.optim.Adam step (amsgrad = maximize = False; L2 weight_decay added to the gradient)
 * for every tensor in the list; `step` is the 1-based step count after increment (ignored when
 * the tensors carry device step counters: then the call is graph-capturable).  Scalars are
 * doubles (Python floats): derived values (1 - beta, lr / bias_correction1, ...) are formed in
 * double and rounded to float once, as torch does.                                            */
int rk_adam_step(const rk_adam_tensor* tensors, int32_t n, double lr, double beta1, double beta2,
                 double eps, double weight_decay, int64_t step, void* stream);

/* ---- evaluation metrics (the reference's evaluate(): dcn.py:214-239, same in every model) ---- */
/* One batch into accum (3 x 8 bytes, zero it first): [0] double sum over batches of the batch's
 * mean loss — loss_kind 0: BCEWithLogitsLoss(logits, labels) (dcn.py:229, bst.py:300,
 * deepcrossing.py:212); 1: BCELoss(probs, labels), logs clamped at -100 (din.py:379, deepfm.py:198,
 * afm.py:203, fwfm.py:176; logits may be NULL) — plus *extra if non-NULL (DIN's l2_reg, din.py:380);
 * [1] uint64 count of rint(probs) == labels (accuracy_score(labels, np.round(probs)));
 * [2] uint64 number of batches.                                                            */
int rk_eval_batch(const float* logits, const float* probs, const float* labels, int64_t n,
                  int32_t loss_kind, const float* extra, void* accum, void* stream);
/* Exact roc_auc_score(labels, scores) (dcn.py:237) for n <= 2^32-1: Mann-Whitney U with ties
 * credited 1/2, from a radix sort and int64 counts; *out (device double) = NaN for a NaN score or a
 * single class.  workspace: rk_auc_workspace_size(n) bytes of device memory.                      */
int rk_auc_workspace_size(int64_t n, int64_t* bytes);
int rk_auc(const float* scores, const float* labels, int64_t n, void* workspace, int64_t ws_bytes,
           double* out, void* stream);

int rk_bn_fold(const float* mean, const float* var, const float* weight, const float* bias,
               float eps, int32_t n, float* scale, float* shift, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* RANKOPS_H */
