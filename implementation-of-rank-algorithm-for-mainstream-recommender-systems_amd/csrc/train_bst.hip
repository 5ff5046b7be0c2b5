// BST training pieces: BSTTransformer.forward in train mode with the
// activations its backward needs kept in HBM, and the backward (bst.py:66-91, pooling bst.py:238-241).
//
// Per block, x [M = B*T, d]:
//   xp = x + pos[t]                                   (bst_add_pos)
//   Q = xp Wq^T + bq, K = xp Wk^T + bk, V = x Wv^T + bv    (rk_linear)
//   P = softmax(mask(Q K^T / sqrt(dh))), ctx = P V     (bst_attn_train_fwd: P saved, [B, h, T, T])
//   o = ctx Wo^T + bo;  r1 = xp + dropout(o);  out1 = LN1(r1)        (bst_res_dropout_ln_fwd)
//   f1 = out1 W1^T + b1;  a = dropout(leaky(f1))                        (bst_leaky_dropout_fwd)
//   f2 = a W2^T + b2;  r2 = out1 + dropout(f2);  out = LN2(r2)
// Dropout masks are the counter hash of train_common.h (index m * d + k per site).
#include "train_common.h"

namespace rk {

constexpr int kBstTMax = 64;   // sequence length envelope of the train kernels
constexpr int kBstDhMax = 64;  // head width envelope
constexpr int kBstLd = 65;     // LDS row pitch (bank-conflict padding)

__global__ __launch_bounds__(256) void bst_add_pos_kernel(const float* __restrict__ x, const float* __restrict__ pos,
                                                          int T, int64_t M, int d, float* __restrict__ xp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * d) return;
  const int64_t m = i / d;
  const int k = (int)(i - m * d);
  xp[i] = x[i] + pos[(int64_t)(m % T) * d + k];
}

// Stage a [T, dh] head slice of a row-major [M, ld] matrix (columns col0..col0+dh) into LDS.
__device__ __forceinline__ void bst_stage(float* __restrict__ dst, const float* __restrict__ src, int64_t ld,
                                          int64_t row0, int col0, int T, int dh) {
  for (int i = threadIdx.x; i < T * dh; i += blockDim.x) {
    const int t = i / dh, k = i - t * dh;
    dst[t * kBstLd + k] = src[(row0 + t) * ld + col0 + k];
  }
}

// Workgroup per (sample, head).  Phase 1: wave w computes the probability rows w, w+4, ... (lane =
// key position) into LDS and HBM; phase 2: ctx = P V with lane = (row in a group of 64/dh rows,
// column), so every lane is busy at dh = 32.
__global__ __launch_bounds__(256) void bst_attn_train_fwd_kernel(const float* __restrict__ qkv, int64_t B, int T,
                                                                 int d, int heads,
                                                                 const int64_t* __restrict__ seq_len,
                                                                 float* __restrict__ P, float* __restrict__ ctx) {
  __shared__ float sQ[kBstTMax * kBstLd], sK[kBstTMax * kBstLd], sV[kBstTMax * kBstLd], sP[kBstTMax * kBstLd];
  const int64_t b = blockIdx.x / heads;
  const int h = (int)(blockIdx.x - b * heads);
  const int dh = d / heads;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t row0 = b * T, ld = 3 * (int64_t)d;
  bst_stage(sQ, qkv, ld, row0, h * dh, T, dh);
  bst_stage(sK, qkv, ld, row0, d + h * dh, T, dh);
  bst_stage(sV, qkv, ld, row0, 2 * d + h * dh, T, dh);
  __syncthreads();
  const int64_t len = seq_len[b];
  const float sq = sqrtf((float)dh);  // scores / math.sqrt(q.size(-1)), bst.py:77
  float* Pb = P + (b * heads + h) * (int64_t)T * T;
  for (int i = wv; i < T; i += 4) {
    float s = -INFINITY;
    if (lane < T) {
      float acc = 0.f;
      for (int k = 0; k < dh; ++k) acc = fmaf(sQ[i * kBstLd + k], sK[lane * kBstLd + k], acc);
      s = (int64_t)lane < len ? acc / sq : -INFINITY;  // masked_fill(key_padding_mask, -inf)
    }
    const float mx = wave_max(s);
    const float e = lane < T ? expf(s - mx) : 0.f;
    const float sum = wave_sum(e);
    const float p = e / sum;
    if (lane < T) {
      Pb[(int64_t)i * T + lane] = p;
      sP[i * kBstLd + lane] = p;
    }
  }
  __syncthreads();
  const int R = 64 / dh, rr = lane / dh, k = lane - rr * dh;
  for (int i0 = wv * R; i0 < T; i0 += 4 * R) {
    const int i = i0 + rr;
    if (rr < R && i < T) {
      float c = 0.f;
      for (int j = 0; j < T; ++j) c = fmaf(sP[i * kBstLd + j], sV[j * kBstLd + k], c);
      ctx[(row0 + i) * d + h * dh + k] = c;
    }
  }
}

// Backward of the above from dctx [M, d]: dqkv [M, 3d] (overwritten).
//   dP = dC V^T;  dS = P (dP - rowsum(P dP)) / sqrt(dh);  dQ = dS K;  dK = dS^T Q;  dV = P^T dC.
__global__ __launch_bounds__(256) void bst_attn_train_bwd_kernel(const float* __restrict__ qkv,
                                                                 const float* __restrict__ P,
                                                                 const float* __restrict__ dctx, int64_t B, int T,
                                                                 int d, int heads, float* __restrict__ dqkv) {
  __shared__ float sQ[kBstTMax * kBstLd], sK[kBstTMax * kBstLd], sV[kBstTMax * kBstLd];
  __shared__ float sC[kBstTMax * kBstLd], sP[kBstTMax * kBstLd], sS[kBstTMax * kBstLd];
  const int64_t b = blockIdx.x / heads;
  const int h = (int)(blockIdx.x - b * heads);
  const int dh = d / heads;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t row0 = b * T, ld = 3 * (int64_t)d;
  bst_stage(sQ, qkv, ld, row0, h * dh, T, dh);
  bst_stage(sK, qkv, ld, row0, d + h * dh, T, dh);
  bst_stage(sV, qkv, ld, row0, 2 * d + h * dh, T, dh);
  bst_stage(sC, dctx, d, row0, h * dh, T, dh);
  const float* Pb = P + (b * heads + h) * (int64_t)T * T;
  for (int i = threadIdx.x; i < T * T; i += blockDim.x) sP[(i / T) * kBstLd + i % T] = Pb[i];
  __syncthreads();
  const float sq = sqrtf((float)dh);
  for (int i = wv; i < T; i += 4) {
    float dp = 0.f, p = 0.f;
    if (lane < T) {
      for (int k = 0; k < dh; ++k) dp = fmaf(sC[i * kBstLd + k], sV[lane * kBstLd + k], dp);
      p = sP[i * kBstLd + lane];
    }
    const float D = wave_sum(p * dp);
    if (lane < T) sS[i * kBstLd + lane] = p * (dp - D) / sq;
  }
  __syncthreads();
  // lane = (row in a group of 64/dh rows, column): every lane busy at dh = 32
  const int R = 64 / dh, rr = lane / dh, c = lane - rr * dh;
  for (int i0 = wv * R; i0 < T; i0 += 4 * R) {
    const int i = i0 + rr;
    if (rr < R && i < T) {
      float q = 0.f, kk = 0.f, v = 0.f;
      for (int j = 0; j < T; ++j) {
        q = fmaf(sS[i * kBstLd + j], sK[j * kBstLd + c], q);   // dQ[i] = sum_j dS[i, j] K[j]
        kk = fmaf(sS[j * kBstLd + i], sQ[j * kBstLd + c], kk);  // dK[i] = sum_j dS[j, i] Q[j]
        v = fmaf(sP[j * kBstLd + i], sC[j * kBstLd + c], v);    // dV[i] = sum_j P[j, i] dC[j]
      }
      float* o = dqkv + (row0 + i) * ld + h * dh + c;
      o[0] = q;
      o[d] = kk;
      o[2 * d] = v;
    }
  }
}

// One wave per row: r = base + dropout(o); y = LayerNorm(r) (biased variance, eps); saves r, mean, rstd.
__global__ __launch_bounds__(256) void bst_res_dropout_ln_fwd_kernel(
    const float* __restrict__ base, const float* __restrict__ o, int64_t M, int d, uint64_t seed,
    const int64_t* __restrict__ stream_slot, uint32_t threshold, float scale, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ r_out, float* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int64_t m = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (m >= M) return;
  const uint64_t stream = threshold ? (uint64_t)*stream_slot : 0;
  float v[4];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int k = lane + 64 * c;
    v[c] = 0.f;
    if (k < d) {
      float ov = o[m * d + k];
      if (threshold) ov = dropout_keep(seed, stream, (uint64_t)m * d + k, threshold) ? ov * scale : 0.f;
      v[c] = base[m * d + k] + ov;
      r_out[m * d + k] = v[c];
      s += v[c];
    }
  }
  const float mean = wave_sum(s) / (float)d;
  float q = 0.f;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    if (lane + 64 * c < d) q += (v[c] - mean) * (v[c] - mean);
  const float rstd = 1.0f / sqrtf(wave_sum(q) / (float)d + eps);
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int k = lane + 64 * c;
    if (k < d) y[m * d + k] = (v[c] - mean) * rstd * gamma[k] + beta[k];
  }
  if (lane == 0) {
    mean_out[m] = mean;
    rstd_out[m] = rstd;
  }
}

// LayerNorm backward from dy: dr = rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma; d_o =
// dropout-masked dr (the residual branch's gradient).  Waves walk rows grid-stride; each lane keeps
// its columns' dgamma = sum dy xhat and dbeta = sum dy in registers, the workgroup combines them
// in LDS and writes one partial row per workgroup to ws [kLnBlocks][2d], summed in block order by
// bst_ln_param_kernel (deterministic; per-row atomics on the same 2d addresses serialised).
constexpr int kLnBlocks = 512;

__global__ __launch_bounds__(256) void bst_ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ r,
                                                         const float* __restrict__ mean_in,
                                                         const float* __restrict__ rstd_in,
                                                         const float* __restrict__ gamma, int64_t M, int d,
                                                         uint64_t seed, const int64_t* __restrict__ stream_slot,
                                                         uint32_t threshold, float scale, float* __restrict__ dr,
                                                         float* __restrict__ d_o, float* __restrict__ ws) {
  __shared__ float red[4][2][256];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t stream = threshold ? (uint64_t)*stream_slot : 0;
  float pg[4] = {0.f, 0.f, 0.f, 0.f}, pb[4] = {0.f, 0.f, 0.f, 0.f}, gm[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) gm[c] = lane + 64 * c < d ? gamma[lane + 64 * c] : 0.f;
  for (int64_t m = (int64_t)blockIdx.x * 4 + wv; m < M; m += (int64_t)gridDim.x * 4) {
    const float mean = mean_in[m], rstd = rstd_in[m];
    float g[4], xh[4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = lane + 64 * c;
      g[c] = xh[c] = 0.f;
      if (k < d) {
        const float dyv = dy[m * d + k];
        xh[c] = (r[m * d + k] - mean) * rstd;
        g[c] = dyv * gm[c];
        s1 += g[c];
        s2 += g[c] * xh[c];
        pg[c] = fmaf(dyv, xh[c], pg[c]);
        pb[c] += dyv;
      }
    }
    const float k1 = wave_sum(s1) / (float)d, k2 = wave_sum(s2) / (float)d;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = lane + 64 * c;
      if (k < d) {
        const float v = rstd * (g[c] - k1 - xh[c] * k2);
        dr[m * d + k] = v;
        if (d_o)
          d_o[m * d + k] = threshold ? (dropout_keep(seed, stream, (uint64_t)m * d + k, threshold) ? v * scale : 0.f)
                                     : v;
      }
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    red[wv][0][lane + 64 * c] = pg[c];
    red[wv][1][lane + 64 * c] = pb[c];
  }
  __syncthreads();
  for (int k = threadIdx.x; k < d; k += blockDim.x) {
    ws[(int64_t)blockIdx.x * 2 * d + k] = red[0][0][k] + red[1][0][k] + red[2][0][k] + red[3][0][k];
    ws[(int64_t)blockIdx.x * 2 * d + d + k] = red[0][1][k] + red[1][1][k] + red[2][1][k] + red[3][1][k];
  }
}

// 16 waves per workgroup, each summing every 16th block partial of 64 columns; LDS combine.
__global__ __launch_bounds__(1024) void bst_ln_param_kernel(const float* __restrict__ ws, int nblocks, int d,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (k < 2 * d)
    for (int blk = wv; blk < nblocks; blk += 16) s += ws[(int64_t)blk * 2 * d + k];
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && k < 2 * d) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    if (k < d)
      dgamma[k] = t;
    else
      dbeta[k - d] = t;
  }
}

// Position-embedding gradient: dpos[t, k] += sum over a chunk of samples of dxp[b*T + t, k] (rows
// t < T; the caller zeroes dpos).  grid.y splits the batch into kPosChunks chunks (one float
// atomic per chunk and element).
constexpr int kPosChunks = 64;

__global__ __launch_bounds__(256) void bst_pos_grad_kernel(const float* __restrict__ dxp, int64_t B, int T, int d,
                                                           float* __restrict__ dpos) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= T * d) return;
  const int64_t per = (B + gridDim.y - 1) / gridDim.y;
  const int64_t b0 = blockIdx.y * per, b1 = min<int64_t>(B, b0 + per);
  float s = 0.f;
  for (int64_t b = b0; b < b1; ++b) s += dxp[b * T * d + i];
  atomicAdd(dpos + i, s);
}

// a = dropout(leaky(f)) forward; backward df = da * keep * scale * (f > 0 ? 1 : slope).
template <bool BWD>
__global__ __launch_bounds__(256) void bst_leaky_dropout_kernel(const float* __restrict__ in,
                                                                const float* __restrict__ f, int64_t n, float slope,
                                                                uint64_t seed, const int64_t* __restrict__ stream_slot,
                                                                uint32_t threshold, float scale,
                                                                float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool keep = threshold ? dropout_keep(seed, (uint64_t)*stream_slot, (uint64_t)i, threshold) : true;
  const float s = threshold ? scale : 1.f;
  const float fv = f[i];
  if (BWD)
    out[i] = keep ? in[i] * s * (fv > 0.f ? 1.f : slope) : 0.f;
  else
    out[i] = keep ? (fv > 0.f ? fv : fv * slope) * s : 0.f;
}

// Pooling over all T rows of a sample (bst.py:238-241): sum, or sum / len (mean).
__global__ __launch_bounds__(256) void bst_pool_fwd_kernel(const float* __restrict__ out, int64_t B, int T, int d,
                                                           const int64_t* __restrict__ seq_len, int mean,
                                                           float* __restrict__ row, int64_t ld_row, int col) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * d) return;
  const int64_t b = i / d;
  const int k = (int)(i - b * d);
  float s = 0.f;
  for (int t = 0; t < T; ++t) s += out[(b * T + t) * d + k];
  if (mean) s = s / (float)seq_len[b];
  row[b * ld_row + col + k] = s;
}

__global__ __launch_bounds__(256) void bst_pool_bwd_kernel(const float* __restrict__ drow, int64_t ld_row, int col,
                                                           int64_t B, int T, int d,
                                                           const int64_t* __restrict__ seq_len, int mean,
                                                           float* __restrict__ dout) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T * d) return;
  const int64_t m = i / d;
  const int k = (int)(i - m * d);
  const int64_t b = m / T;
  float g = drow[b * ld_row + col + k];
  if (mean) g = g / (float)seq_len[b];
  dout[i] = g;
}

static inline unsigned grid_of(int64_t n, int per = 256) { return (unsigned)((n + per - 1) / per); }

}  // namespace rk

using namespace rk;

RK_API int rk_bst_add_pos(const float* x, const float* pos, int32_t T, int64_t rows, int32_t d, float* xp,
                          void* stream) {
  if (!x || !pos || !xp || T <= 0 || rows < 0 || d <= 0) return fail(RK_ERR_INVALID, "rk_bst_add_pos: bad arguments");
  if (rows == 0) return RK_OK;
  bst_add_pos_kernel<<<grid_of(rows * d), 256, 0, (hipStream_t)stream>>>(x, pos, T, rows, d, xp);
  return check_launch("rk_bst_add_pos");
}

RK_API int rk_bst_attn_train_forward(const float* qkv, int64_t batch, int32_t T, int32_t d, int32_t heads,
                                     const int64_t* seq_len, float* probs, float* ctx, void* stream) {
  if (!qkv || !seq_len || !probs || !ctx || batch < 0 || T <= 0 || T > kBstTMax || heads <= 0 || d % heads ||
      d / heads > kBstDhMax)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_attn_train_forward: T <= %d, d %% heads == 0, d/heads <= %d", kBstTMax,
                kBstDhMax);
  if (batch == 0) return RK_OK;
  bst_attn_train_fwd_kernel<<<(unsigned)(batch * heads), 256, 0, (hipStream_t)stream>>>(qkv, batch, T, d, heads,
                                                                                        seq_len, probs, ctx);
  return check_launch("rk_bst_attn_train_forward");
}

RK_API int rk_bst_attn_train_backward(const float* qkv, const float* probs, const float* dctx, int64_t batch,
                                      int32_t T, int32_t d, int32_t heads, float* dqkv, void* stream) {
  if (!qkv || !probs || !dctx || !dqkv || batch < 0 || T <= 0 || T > kBstTMax || heads <= 0 || d % heads ||
      d / heads > kBstDhMax)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_attn_train_backward: T <= %d, d/heads <= %d", kBstTMax, kBstDhMax);
  if (batch == 0) return RK_OK;
  bst_attn_train_bwd_kernel<<<(unsigned)(batch * heads), 256, 0, (hipStream_t)stream>>>(qkv, probs, dctx, batch, T,
                                                                                        d, heads, dqkv);
  return check_launch("rk_bst_attn_train_backward");
}

RK_API int rk_bst_res_dropout_ln_forward(const float* base, const float* o, int64_t rows, int32_t d,
                                         double dropout_p, uint64_t seed, const int64_t* stream_slot,
                                         const float* gamma, const float* beta, float eps, float* r, float* y,
                                         float* mean, float* rstd, void* stream) {
  if (!base || !o || !gamma || !beta || !r || !y || !mean || !rstd || rows < 0 || d <= 0 || d > 256 ||
      !(dropout_p >= 0.0 && dropout_p < 1.0) || (dropout_p > 0.0 && !stream_slot))
    return fail(RK_ERR_INVALID, "rk_bst_res_dropout_ln_forward: bad arguments (d <= 256)");
  if (rows == 0) return RK_OK;
  bst_res_dropout_ln_fwd_kernel<<<grid_of(rows, 4), 256, 0, (hipStream_t)stream>>>(
      base, o, rows, d, seed, stream_slot, dropout_threshold(dropout_p), (float)(1.0 / (1.0 - dropout_p)), gamma,
      beta, eps, r, y, mean, rstd);
  return check_launch("rk_bst_res_dropout_ln_forward");
}

RK_API int64_t rk_bst_ln_backward_workspace_floats(int32_t d) { return (int64_t)kLnBlocks * 2 * (d > 0 ? d : 0); }

RK_API int rk_bst_ln_backward(const float* dy, const float* r, const float* mean, const float* rstd,
                              const float* gamma, int64_t rows, int32_t d, double dropout_p, uint64_t seed,
                              const int64_t* stream_slot, float* dr, float* d_o, float* dgamma, float* dbeta,
                              float* workspace, int64_t workspace_floats, void* stream) {
  if (!dy || !r || !mean || !rstd || !gamma || !dr || !dgamma || !dbeta || !workspace || rows < 0 || d <= 0 ||
      d > 256 || !(dropout_p >= 0.0 && dropout_p < 1.0) || (dropout_p > 0.0 && !stream_slot))
    return fail(RK_ERR_INVALID, "rk_bst_ln_backward: bad arguments (d <= 256)");
  if (workspace_floats < rk_bst_ln_backward_workspace_floats(d))
    return fail(RK_ERR_INVALID, "rk_bst_ln_backward: workspace of %lld floats, needs %lld (%d * 2d)",
                (long long)workspace_floats, (long long)rk_bst_ln_backward_workspace_floats(d), kLnBlocks);
  hipStream_t st = (hipStream_t)stream;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>(kLnBlocks, (rows + 3) / 4));
  bst_ln_bwd_kernel<<<blocks, 256, 0, st>>>(dy, r, mean, rstd, gamma, rows, d, seed, stream_slot,
                                            dropout_threshold(dropout_p), (float)(1.0 / (1.0 - dropout_p)), dr, d_o,
                                            workspace);
  bst_ln_param_kernel<<<grid_of(2 * d, 64), 1024, 0, st>>>(workspace, blocks, d, dgamma, dbeta);
  return check_launch("rk_bst_ln_backward");
}

RK_API int rk_bst_pos_backward(const float* dxp, int64_t batch, int32_t T, int32_t d, float* dpos, void* stream) {
  if (!dxp || !dpos || batch < 0 || T <= 0 || d <= 0) return fail(RK_ERR_INVALID, "rk_bst_pos_backward: bad arguments");
  if (batch == 0) return RK_OK;
  const dim3 grid(grid_of((int64_t)T * d), (unsigned)std::min<int64_t>(kPosChunks, batch));
  bst_pos_grad_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(dxp, batch, T, d, dpos);
  return check_launch("rk_bst_pos_backward");
}

RK_API int rk_bst_leaky_dropout(const float* in, const float* f, int64_t n, float slope, double dropout_p,
                                uint64_t seed, const int64_t* stream_slot, int32_t backward, float* out,
                                void* stream) {
  if (!f || !out || (backward && !in) || n < 0 || !(dropout_p >= 0.0 && dropout_p < 1.0) ||
      (dropout_p > 0.0 && !stream_slot))
    return fail(RK_ERR_INVALID, "rk_bst_leaky_dropout: bad arguments");
  if (n == 0) return RK_OK;
  const uint32_t thr = dropout_threshold(dropout_p);
  const float scale = (float)(1.0 / (1.0 - dropout_p));
  hipStream_t st = (hipStream_t)stream;
  if (backward)
    bst_leaky_dropout_kernel<true><<<grid_of(n), 256, 0, st>>>(in, f, n, slope, seed, stream_slot, thr, scale, out);
  else
    bst_leaky_dropout_kernel<false><<<grid_of(n), 256, 0, st>>>(in, f, n, slope, seed, stream_slot, thr, scale, out);
  return check_launch("rk_bst_leaky_dropout");
}

RK_API int rk_bst_pool(const float* out, int64_t batch, int32_t T, int32_t d, const int64_t* seq_len, int32_t mean,
                       float* row, int64_t ld_row, int32_t col, void* stream) {
  if (!out || !seq_len || !row || batch < 0 || T <= 0 || d <= 0 || col < 0 || col + d > ld_row)
    return fail(RK_ERR_INVALID, "rk_bst_pool: bad arguments");
  if (batch == 0) return RK_OK;
  bst_pool_fwd_kernel<<<grid_of(batch * d), 256, 0, (hipStream_t)stream>>>(out, batch, T, d, seq_len, mean, row,
                                                                          ld_row, col);
  return check_launch("rk_bst_pool");
}

RK_API int rk_bst_pool_backward(const float* drow, int64_t ld_row, int32_t col, int64_t batch, int32_t T, int32_t d,
                                const int64_t* seq_len, int32_t mean, float* dout, void* stream) {
  if (!drow || !seq_len || !dout || batch < 0 || T <= 0 || d <= 0 || col < 0 || col + d > ld_row)
    return fail(RK_ERR_INVALID, "rk_bst_pool_backward: bad arguments");
  if (batch == 0) return RK_OK;
  bst_pool_bwd_kernel<<<grid_of(batch * T * d), 256, 0, (hipStream_t)stream>>>(drow, ld_row, col, batch, T, d,
                                                                              seq_len, mean, dout);
  return check_launch("rk_bst_pool_backward");
}
