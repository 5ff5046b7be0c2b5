// AFM training pieces: the train-mode AFM.forward with the activations its
// backward needs kept in HBM, and the backward (afm.py:92-119, loss: BCELoss on the prediction,
// afm.py:173,258).
//
//   pair_p = e_i * e_j (i < j, i-major)            [B, P, D]
//   a1 = relu(pair W1^T + b1) (rk_linear),  s_p = a1 . w2 + b2,  w = softmax_p(s)
//   ws = sum_p w_p pair_p,  total = (dense . wd + bd) + (ws . wp + bp),  pred = sigmoid(total)
//
// Backward: the per-sample chain (sigmoid, the two heads, softmax, the score layer) runs one
// wave per sample and emits d(pair) (direct part) and d(a1); the first attention layer's weight
// gradient and input gradient are rk_gemm calls; the pair gradients fold into the field
// embeddings' row gradients (d e_i = sum_j d pair_ij * e_j) for rk_embedding_backward.
#include "common.h"

namespace rk {

constexpr int kAfmMaxFields = 16;
constexpr int kAfmMaxPairs = kAfmMaxFields * (kAfmMaxFields - 1) / 2;
constexpr int kAfmMaxAtt = 256;
struct AfmTrainSegs {
  rk_segment s[kAfmMaxFields];
};

// E[b, f*D + d] = table_f[idx_f[b], d]; pairs[(b*P + p)*D + d] = e_i[d] * e_j[d].  Thread per (b, d).
__global__ __launch_bounds__(256) void afm_pairs_kernel(AfmTrainSegs segs, int F, int D, int64_t B,
                                                        float* __restrict__ E, float* __restrict__ pairs,
                                                        uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * D) return;
  const int64_t b = i / D;
  const int d = (int)(i - b * D);
  float e[kAfmMaxFields];
#pragma unroll
  for (int f = 0; f < kAfmMaxFields; ++f) {
    e[f] = 0.f;
    if (f < F) {
      const float* r = segment_row(segs.s[f], b, d == 0 ? flags : nullptr);
      if (r) e[f] = r[d];
      E[b * F * D + (int64_t)f * D + d] = e[f];
    }
  }
  const int P = F * (F - 1) / 2;
  int p = 0;
#pragma unroll
  for (int x = 0; x < kAfmMaxFields; ++x) {
    if (x >= F) break;
#pragma unroll
    for (int y = x + 1; y < kAfmMaxFields; ++y) {
      if (y >= F) break;
      pairs[(b * P + p) * D + d] = e[x] * e[y];
      ++p;
    }
  }
}

// One wave per sample: scores, softmax over pairs, weighted sum, both heads, sigmoid.
// Saves w [B, P] and ws [B, D].  D, nd <= 64, P <= 120.
__global__ __launch_bounds__(256) void afm_pool_forward_kernel(
    const float* __restrict__ a1, int A, const float* __restrict__ w2, const float* __restrict__ b2,
    const float* __restrict__ pairs, const float* __restrict__ dense, int64_t ld_dense, int nd,
    const float* __restrict__ wd, const float* __restrict__ bd, const float* __restrict__ wp,
    const float* __restrict__ bp, int64_t B, int P, int D, float* __restrict__ w_out, float* __restrict__ ws_out,
    float* __restrict__ logit, float* __restrict__ pred) {
  __shared__ float sw[4][kAfmMaxPairs];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * 4 + wv;
  const bool live = b0 < B;
  const int64_t b = live ? b0 : B - 1;
  float* S = sw[wv];
  const float* ab = a1 + b * P * A;
  for (int p = 0; p < P; ++p) {
    float s = 0.f;
    for (int a = lane; a < A; a += 64) s = fmaf(ab[(int64_t)p * A + a], w2[a], s);
    s = wave_sum(s);
    if (lane == 0) S[p] = s + b2[0];
  }
  __syncthreads();
  float mx = -INFINITY;
  for (int p = lane; p < P; p += 64) mx = fmaxf(mx, S[p]);
  mx = wave_max(mx);
  float sum = 0.f;
  for (int p = lane; p < P; p += 64) sum += expf(S[p] - mx);
  sum = wave_sum(sum);
  __syncthreads();
  for (int p = lane; p < P; p += 64) S[p] = expf(S[p] - mx) / sum;
  __syncthreads();
  if (!live) return;
  for (int p = lane; p < P; p += 64) w_out[b * P + p] = S[p];
  float ws = 0.f;
  if (lane < D) {
    const float* pb = pairs + b * P * D + lane;
    for (int p = 0; p < P; ++p) ws = fmaf(S[p], pb[(int64_t)p * D], ws);
    ws_out[b * D + lane] = ws;
  }
  const float al = wave_sum(lane < D ? ws * wp[lane] : 0.f) + bp[0];
  const float dl = wave_sum(lane < nd ? dense[b * ld_dense + lane] * wd[lane] : 0.f) + bd[0];
  if (lane == 0) {
    const float t = dl + al;
    if (logit) logit[b] = t;
    pred[b] = sigmoidf_ref(t);
  }
}

// One wave per sample, from dL/dpred and/or dL/dtotal:
//   dt = dtotal + dpred * (1 - pred) * pred;  grads of dense_layer and p (accumulated);
//   dws = dt * wp;  dw_p = dws . pair_p;  ds_p = w_p (dw_p - sum_q w_q dw_q);
//   d_pairs[p, d] = w_p dws[d] (overwrite);  da1[p, a] = ds_p w2[a] [a1 > 0];
//   dW2[a] += sum_p ds_p a1[p, a];  db2 += sum_p ds_p.
// acc layout (zeroed by the host): [dwd nd | dbd | dwp D | dbp | dw2 A | db2].
__global__ __launch_bounds__(256) void afm_pool_backward_kernel(
    const float* __restrict__ dpred, const float* __restrict__ dtotal, const float* __restrict__ pred,
    const float* __restrict__ w, const float* __restrict__ ws, const float* __restrict__ pairs,
    const float* __restrict__ a1, int A, const float* __restrict__ w2, const float* __restrict__ wp,
    const float* __restrict__ dense, int64_t ld_dense, int nd, int64_t B, int P, int D,
    float* __restrict__ d_pairs, float* __restrict__ da1, float* __restrict__ acc) {
  __shared__ float red[64 + 1 + 64 + 1 + kAfmMaxAtt + 1];
  __shared__ float sds[4][kAfmMaxPairs];
  __shared__ float sdws[4][64];
  const int nacc = nd + 1 + D + 1 + A + 1;
  for (int i = threadIdx.x; i < nacc; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * 4 + wv;
  const bool live = b0 < B;
  const int64_t b = live ? b0 : B - 1;
  float dt = 0.f;
  if (live) {
    const float y = pred[b];
    dt = (dtotal ? dtotal[b] : 0.f) + (dpred ? dpred[b] * (1.0f - y) * y : 0.f);
  }
  float* red_wd = red;
  float* red_wp = red + nd + 1;
  float* red_w2 = red + nd + 1 + D + 1;
  if (lane < nd) atomicAdd(red_wd + lane, dt * dense[b * ld_dense + lane]);
  if (lane < D) {
    atomicAdd(red_wp + lane, dt * ws[b * D + lane]);
    sdws[wv][lane] = dt * wp[lane];
  }
  if (lane == 0) {
    atomicAdd(red_wd + nd, dt);
    atomicAdd(red_wp + D, dt);
  }
  __syncthreads();
  const float* pb = pairs + b * P * D;
  const float* wb = w + b * P;
  float g = 0.f;
  for (int p = lane; p < P; p += 64) {
    float dw = 0.f;
    for (int d = 0; d < D; ++d) dw = fmaf(sdws[wv][d], pb[(int64_t)p * D + d], dw);
    sds[wv][p] = dw;
    g += wb[p] * dw;
  }
  g = wave_sum(g);
  for (int p = lane; p < P; p += 64) sds[wv][p] = wb[p] * (sds[wv][p] - g);
  __syncthreads();
  if (live) {
    for (int64_t i = lane; i < (int64_t)P * D; i += 64) {
      const int p = (int)(i / D), d = (int)(i - (int64_t)p * D);
      d_pairs[b * P * D + i] = wb[p] * sdws[wv][d];
    }
    const float* ab = a1 + b * P * A;
    for (int64_t i = lane; i < (int64_t)P * A; i += 64) {
      const int p = (int)(i / A), a = (int)(i - (int64_t)p * A);
      da1[b * P * A + i] = ab[i] > 0.f ? sds[wv][p] * w2[a] : 0.f;
    }
    for (int a = lane; a < A; a += 64) {
      float s = 0.f;
      for (int p = 0; p < P; ++p) s = fmaf(sds[wv][p], ab[(int64_t)p * A + a], s);
      atomicAdd(red_w2 + a, s);
    }
    float sp = 0.f;
    for (int p = lane; p < P; p += 64) sp += sds[wv][p];
    sp = wave_sum(sp);
    if (lane == 0) atomicAdd(red_w2 + A, sp);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nacc; i += blockDim.x) atomicAdd(acc + i, red[i]);
}

// dE[b, i*D + d] = sum_{j != i} d_pairs[b, pair(i, j), d] * e_j[d].  Thread per (b, d).
__global__ __launch_bounds__(256) void afm_pair_fold_kernel(const float* __restrict__ d_pairs,
                                                            const float* __restrict__ E, int F, int D, int64_t B,
                                                            float* __restrict__ dE) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * D) return;
  const int64_t b = i / D;
  const int d = (int)(i - b * D);
  const int P = F * (F - 1) / 2;
  float e[kAfmMaxFields], g[kAfmMaxFields];
#pragma unroll
  for (int f = 0; f < kAfmMaxFields; ++f) {
    e[f] = f < F ? E[b * F * D + (int64_t)f * D + d] : 0.f;
    g[f] = 0.f;
  }
  int p = 0;
#pragma unroll
  for (int x = 0; x < kAfmMaxFields; ++x) {
    if (x >= F) break;
#pragma unroll
    for (int y = x + 1; y < kAfmMaxFields; ++y) {
      if (y >= F) break;
      const float dp = d_pairs[(b * P + p) * D + d];
      g[x] = fmaf(dp, e[y], g[x]);
      g[y] = fmaf(dp, e[x], g[y]);
      ++p;
    }
  }
#pragma unroll
  for (int f = 0; f < kAfmMaxFields; ++f)
    if (f < F) dE[b * F * D + (int64_t)f * D + d] = g[f];
}

}  // namespace rk

using namespace rk;

RK_API int rk_afm_pairs(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch, float* emb,
                        float* pairs, void* stream) {
  if (!fields || num_fields < 2 || num_fields > kAfmMaxFields || dim <= 0 || !emb || !pairs || batch < 0)
    return fail(RK_ERR_INVALID, "rk_afm_pairs: bad arguments (2 <= fields <= %d)", kAfmMaxFields);
  AfmTrainSegs t;
  for (int f = 0; f < num_fields; ++f) {
    if (!fields[f].src || !fields[f].idx || fields[f].rows <= 0 || fields[f].dim != dim)
      return fail(RK_ERR_INVALID, "rk_afm_pairs: field %d table invalid", f);
    t.s[f] = fields[f];
  }
  const int64_t n = batch * dim;
  if (n == 0) return RK_OK;
  afm_pairs_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(t, num_fields, dim, batch, emb,
                                                                                 pairs, device_flags());
  return check_launch("rk_afm_pairs");
}

RK_API int rk_afm_pool_forward(const float* a1, int32_t att_dim, const float* w2, const float* b2, const float* pairs,
                               int32_t num_pairs, int32_t dim, const float* dense, int64_t ld_dense,
                               int32_t num_dense, const float* wd, const float* bd, const float* wp, const float* bp,
                               int64_t batch, float* weights, float* ws, float* logit, float* pred, void* stream) {
  if (!a1 || !w2 || !b2 || !pairs || !dense || !wd || !bd || !wp || !bp || !weights || !ws || !pred || batch < 0 ||
      att_dim <= 0 || num_pairs <= 0 || num_pairs > kAfmMaxPairs || dim <= 0 || dim > 64 || num_dense <= 0 ||
      num_dense > 64)
    return fail(RK_ERR_INVALID, "rk_afm_pool_forward: bad arguments (dim, dense <= 64, pairs <= %d)",
                kAfmMaxPairs);
  if (batch == 0) return RK_OK;
  afm_pool_forward_kernel<<<(unsigned)((batch + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      a1, att_dim, w2, b2, pairs, dense, ld_dense, num_dense, wd, bd, wp, bp, batch, num_pairs, dim, weights, ws,
      logit, pred);
  return check_launch("rk_afm_pool_forward");
}

RK_API int rk_afm_pool_backward(const float* dpred, const float* dtotal, const float* pred, const float* weights,
                                const float* ws, const float* pairs, const float* a1, int32_t att_dim,
                                const float* w2, const float* wp, const float* dense, int64_t ld_dense,
                                int32_t num_dense, int64_t batch, int32_t num_pairs, int32_t dim, float* d_pairs,
                                float* da1, float* acc, void* stream) {
  if ((!dpred && !dtotal) || !pred || !weights || !ws || !pairs || !a1 || !w2 || !wp || !dense || !d_pairs ||
      !da1 || !acc || batch < 0 || att_dim <= 0 || att_dim > kAfmMaxAtt || num_pairs <= 0 ||
      num_pairs > kAfmMaxPairs || dim <= 0 || dim > 64 || num_dense <= 0 || num_dense > 64)
    return fail(RK_ERR_INVALID, "rk_afm_pool_backward: bad arguments (attention factor <= %d)", kAfmMaxAtt);
  hipStream_t st = (hipStream_t)stream;
  const size_t nacc = (size_t)num_dense + 1 + dim + 1 + att_dim + 1;
  if (hipMemsetAsync(acc, 0, nacc * sizeof(float), st) != hipSuccess)
    return fail(RK_ERR_RUNTIME, "rk_afm_pool_backward: memset failed");
  if (batch == 0) return RK_OK;
  afm_pool_backward_kernel<<<(unsigned)((batch + 3) / 4), 256, 0, st>>>(
      dpred, dtotal, pred, weights, ws, pairs, a1, att_dim, w2, wp, dense, ld_dense, num_dense, batch, num_pairs, dim,
      d_pairs, da1, acc);
  return check_launch("rk_afm_pool_backward");
}

RK_API int rk_afm_pair_fold(const float* d_pairs, const float* emb, int32_t num_fields, int32_t dim, int64_t batch,
                            float* d_emb, void* stream) {
  if (!d_pairs || !emb || !d_emb || num_fields < 2 || num_fields > kAfmMaxFields || dim <= 0 || batch < 0)
    return fail(RK_ERR_INVALID, "rk_afm_pair_fold: bad arguments");
  const int64_t n = batch * dim;
  if (n == 0) return RK_OK;
  afm_pair_fold_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(d_pairs, emb, num_fields, dim,
                                                                                     batch, d_emb);
  return check_launch("rk_afm_pair_fold");
}
