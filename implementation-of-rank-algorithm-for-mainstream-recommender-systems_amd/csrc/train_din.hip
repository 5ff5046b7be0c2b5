// DIN training pieces: the train-mode din_attention forward with the
// activations the backward needs kept in HBM, its backward w.r.t. the query and the history
// keys, and the backward of the mini-batch-aware l2 term.
//
// Reference (din.py:42-84):
//   cross = cat[q, k, q - k, q * k]                (B, T, 4H)
//   a1 = relu(cross W1^T + b1), a2 = relu(a1 W2^T + b2), s = a2 w3^T + b3   (att_net, drawn per call)
//   softmax: w = softmax(where(mask, s, -2^32 + 1) / sqrt(H));  else w = masked_fill(s, ~mask, 0)
//   out = sum_t w_t k_t
// and l2 = lambda * mean_b ||[cat, target, att]_b||_2 (din.py:318-322).
//
// The att_net GEMMs run on rk_linear (forward) and rk_gemm (backward); this file holds the
// gather/cross build, the score -> weights -> weighted-sum step and its backward, the fold of
// d(cross) into d(query) / d(keys), and the l2 backward.  att_net's weights are not module
// parameters (fresh per call in the reference), so only input gradients are formed.
#include "common.h"

namespace rk {

// keys[b, t, :] = table[seq[b, t]] (zero row + flag when out of range);
// cross[b*T + t, :] = [q, k, q - k, q * k] with q = x[b, q_col : q_col + H].
__global__ __launch_bounds__(256) void din_att_cross_kernel(const float* __restrict__ x, int64_t ldx, int q_col,
                                                            const float* __restrict__ table, int64_t rows,
                                                            int64_t ld_tab, const int64_t* __restrict__ seq,
                                                            int64_t ld_seq, int64_t B, int T, int H,
                                                            float* __restrict__ keys, float* __restrict__ cross,
                                                            uint32_t* flags) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T * H) return;
  const int h = (int)(i % H);
  const int64_t bt = i / H;
  const int64_t b = bt / T;
  const int t = (int)(bt - b * T);
  const int64_t r = seq[b * ld_seq + t];
  float k = 0.f;
  if (r >= 0 && r < rows)
    k = table[r * ld_tab + h];
  else if (h == 0)
    flag_oob(flags);
  const float q = x[b * ldx + q_col + h];
  keys[i] = k;
  float* c = cross + bt * 4 * H;
  c[h] = q;
  c[H + h] = k;
  c[2 * H + h] = q - k;
  c[3 * H + h] = q * k;
}

// float4 form of din_att_cross_kernel (H % 4 == 0, 16-B aligned table rows / x row): a thread per
// (b, t, 4 columns), 128-bit loads and stores.
__global__ __launch_bounds__(256) void din_att_cross4_kernel(const float* __restrict__ x, int64_t ldx, int q_col,
                                                             const float* __restrict__ table, int64_t rows,
                                                             int64_t ld_tab, const int64_t* __restrict__ seq,
                                                             int64_t ld_seq, int64_t B, int T, int H,
                                                             float* __restrict__ keys, float* __restrict__ cross,
                                                             uint32_t* flags) {
  const int H4 = H / 4;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T * H4) return;
  const int h = 4 * (int)(i % H4);
  const int64_t bt = i / H4;
  const int64_t b = bt / T;
  const int t = (int)(bt - b * T);
  const int64_t r = seq[b * ld_seq + t];
  f32x4 k = {0.f, 0.f, 0.f, 0.f};
  if (r >= 0 && r < rows)
    k = *reinterpret_cast<const f32x4*>(table + r * ld_tab + h);
  else if (h == 0)
    flag_oob(flags);
  const float* qp = x + b * ldx + q_col + h;  // the feature row need not be 16-B aligned
  const f32x4 q = {qp[0], qp[1], qp[2], qp[3]};
  *reinterpret_cast<f32x4*>(keys + bt * H + h) = k;
  float* c = cross + bt * 4 * H;
  *reinterpret_cast<f32x4*>(c + h) = q;
  *reinterpret_cast<f32x4*>(c + H + h) = k;
  *reinterpret_cast<f32x4*>(c + 2 * H + h) = q - k;
  *reinterpret_cast<f32x4*>(c + 3 * H + h) = q * k;
}

// One wave per sample: s_t = a2[b, t] . w3 + b3; weights (masked, or masked softmax with the
// reference's -2^32 + 1 padding scaled by 1/sqrt(H)); out = sum_t w_t k_t written to
// x[b, att_col : att_col + H].  Saves w (B, T).  T <= kDinMaxT, H <= 64.
constexpr int kDinMaxT = 1024;

__global__ __launch_bounds__(256) void din_att_pool_forward_kernel(const float* __restrict__ a2, int A2,
                                                                   const float* __restrict__ w3,
                                                                   const float* __restrict__ b3,
                                                                   const float* __restrict__ keys,
                                                                   const int64_t* __restrict__ seq_len, int64_t B,
                                                                   int T, int H, int softmax, float sqrt_h,
                                                                   float* __restrict__ wts, float* __restrict__ x,
                                                                   int64_t ldx, int att_col, int vec_a2) {
  __shared__ float sw[4][kDinMaxT];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * 4 + wv;
  const bool live = b0 < B;
  const int64_t b = live ? b0 : B - 1;  // dead waves recompute the last sample and store nothing
  float* S = sw[wv];
  const int64_t len = seq_len[b];
  const float bias3 = b3[0];
  float mx = -INFINITY;
  const bool vec = vec_a2;  // A2 % 4 == 0 and a2 16-B aligned (host): float4 row reads, 4x fewer loads
  for (int t = lane; t < T; t += 64) {
    const float* row = a2 + (b * T + t) * A2;
    float s = 0.f;
    if (vec) {
      for (int j = 0; j < A2; j += 4) {
        const f32x4 r4 = *reinterpret_cast<const f32x4*>(row + j);
        s = fmaf(r4[0], w3[j], s);
        s = fmaf(r4[1], w3[j + 1], s);
        s = fmaf(r4[2], w3[j + 2], s);
        s = fmaf(r4[3], w3[j + 3], s);
      }
    } else {
      for (int j = 0; j < A2; ++j) s = fmaf(row[j], w3[j], s);
    }
    s += bias3;
    const bool m = t < len;
    float v;
    if (softmax) {
      v = (m ? s : -4294967295.0f) / sqrt_h;  // where(mask, s, -2**32 + 1) / embedding_dim**0.5
      mx = fmaxf(mx, v);
    } else {
      v = m ? s : 0.f;
    }
    S[t] = v;
  }
  if (softmax) {
    mx = wave_max(mx);
    float sum = 0.f;
    for (int t = lane; t < T; t += 64) {
      const float e = expf(S[t] - mx);
      S[t] = e;
      sum += e;
    }
    sum = wave_sum(sum);
    for (int t = lane; t < T; t += 64) S[t] = S[t] / sum;
  }
  __syncthreads();
  if (!live) return;
  for (int t = lane; t < T; t += 64) wts[b * T + t] = S[t];
  if (lane < H) {
    float o = 0.f;
    const float* kb = keys + b * T * H + lane;
    for (int t = 0; t < T; ++t) o = fmaf(S[t], kb[(int64_t)t * H], o);
    x[b * ldx + att_col + lane] = o;
  }
}

// One wave per sample, from dout = dx[b, att_col : att_col + H]:
//   dkeys[b, t, :] = w_t dout (overwrite); dw_t = dout . k_t;
//   ds_t = mask ? (softmax ? w_t (dw_t - sum_u w_u dw_u) / sqrt(H) : dw_t) : 0;
//   da2[b*T + t, j] = ds_t w3[j] [a2 > 0].
__global__ __launch_bounds__(256) void din_att_pool_backward_kernel(const float* __restrict__ dx, int64_t lddx,
                                                                    int att_col, const float* __restrict__ wts,
                                                                    const float* __restrict__ keys,
                                                                    const float* __restrict__ a2, int A2,
                                                                    const float* __restrict__ w3,
                                                                    const int64_t* __restrict__ seq_len, int64_t B,
                                                                    int T, int H, int softmax, float sqrt_h,
                                                                    float* __restrict__ dkeys,
                                                                    float* __restrict__ da2, int vec_keys,
                                                                    int vec_a2) {
  __shared__ float sd[4][kDinMaxT];
  __shared__ float so[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t b0 = (int64_t)blockIdx.x * 4 + wv;
  const bool live = b0 < B;
  const int64_t b = live ? b0 : B - 1;  // dead waves recompute the last sample and store nothing
  float* DS = sd[wv];
  if (lane < H) so[wv][lane] = dx[b * lddx + att_col + lane];
  __syncthreads();
  const int64_t len = seq_len[b];
  const float* kb = keys + b * T * H;
  const float* wb = wts + b * T;
  float g = 0.f;
  const bool vec = vec_keys;  // H % 4 == 0, keys and dkeys 16-B aligned (host): float4 reads
  for (int t = lane; t < T; t += 64) {
    float dw = 0.f;
    if (vec) {
      for (int h = 0; h < H; h += 4) {
        const f32x4 k4 = *reinterpret_cast<const f32x4*>(kb + (int64_t)t * H + h);
        dw = fmaf(so[wv][h], k4[0], dw);
        dw = fmaf(so[wv][h + 1], k4[1], dw);
        dw = fmaf(so[wv][h + 2], k4[2], dw);
        dw = fmaf(so[wv][h + 3], k4[3], dw);
      }
    } else {
      for (int h = 0; h < H; ++h) dw = fmaf(so[wv][h], kb[(int64_t)t * H + h], dw);
    }
    DS[t] = dw;
    g += wb[t] * dw;
  }
  if (softmax) g = wave_sum(g);
  for (int t = lane; t < T; t += 64) {
    const float dw = DS[t];
    float ds = softmax ? wb[t] * (dw - g) / sqrt_h : dw;
    DS[t] = t < len ? ds : 0.f;
  }
  __syncthreads();
  if (!live) return;
  if (vec && vec_a2) {  // float4 stores of dkeys and da2 (rows 16-B aligned)
    const int H4 = H / 4, A4 = A2 / 4;
    for (int i = lane; i < T * H4; i += 64) {
      const int t = i / H4, h = 4 * (i - t * H4);
      const float wt = wb[t];
      *reinterpret_cast<f32x4*>(dkeys + b * T * H + (int64_t)t * H + h) =
          f32x4{wt * so[wv][h], wt * so[wv][h + 1], wt * so[wv][h + 2], wt * so[wv][h + 3]};
    }
    for (int i = lane; i < T * A4; i += 64) {
      const int t = i / A4, j = 4 * (i - t * A4);
      const int64_t o = (b * T + t) * A2 + j;
      const f32x4 a = *reinterpret_cast<const f32x4*>(a2 + o);
      const float dt = DS[t];
      f32x4 r;
#pragma unroll
      for (int e = 0; e < 4; ++e) r[e] = a[e] > 0.f ? dt * w3[j + e] : 0.f;
      *reinterpret_cast<f32x4*>(da2 + o) = r;
    }
    return;
  }
  for (int64_t i = lane; i < (int64_t)T * H; i += 64) {
    const int t = (int)(i / H), h = (int)(i - (int64_t)t * H);
    dkeys[b * T * H + i] = wb[t] * so[wv][h];
  }
  for (int64_t i = lane; i < (int64_t)T * A2; i += 64) {
    const int t = (int)(i / A2), j = (int)(i - (int64_t)t * A2);
    const int64_t o = (b * T + t) * A2 + j;
    da2[o] = a2[o] > 0.f ? DS[t] * w3[j] : 0.f;
  }
}

// Workgroup-per-sample form (H <= 64, 256 / H position groups): every (t, h) of the sample is a
// thread's work (the dkeys update is elementwise), dq is summed per position group in registers
// and across the groups in LDS in a fixed order.
__global__ __launch_bounds__(256) void din_cross_fold_wg_kernel(const float* __restrict__ dcross,
                                                                const float* __restrict__ x, int64_t ldx, int q_col,
                                                                const float* __restrict__ keys, int64_t B, int T,
                                                                int H, float* __restrict__ dkeys,
                                                                float* __restrict__ dx, int64_t lddx) {
  __shared__ float red[256];
  const int64_t b = blockIdx.x;
  const int G = 256 / H;  // position groups
  const int h = threadIdx.x % H, tg = threadIdx.x / H;
  float dq = 0.f;
  if (tg < G) {
    const float q = x[b * ldx + q_col + h];
    for (int t = tg; t < T; t += G) {
      const int64_t bt = b * T + t;
      const float* dc = dcross + bt * 4 * H;
      const float k = keys[bt * H + h];
      const float d0 = dc[h], d1 = dc[H + h], d2 = dc[2 * H + h], d3 = dc[3 * H + h];
      dq += d0 + d2 + d3 * k;
      dkeys[bt * H + h] += d1 - d2 + d3 * q;
    }
  }
  red[threadIdx.x] = dq;
  __syncthreads();
  if (threadIdx.x < H) {
    float s = 0.f;
    for (int g = 0; g < G; ++g) s += red[g * H + threadIdx.x];
    dx[b * lddx + q_col + threadIdx.x] += s;
  }
}

// d(cross) -> d(query), d(keys): dq = sum_t (dc0 + dc2 + dc3 * k_t), added to dx[b, q_col + h];
// dkeys[b, t, h] += dc1 - dc2 + dc3 * q.  One thread per (b, h).
__global__ __launch_bounds__(256) void din_cross_fold_kernel(const float* __restrict__ dcross,
                                                             const float* __restrict__ x, int64_t ldx, int q_col,
                                                             const float* __restrict__ keys, int64_t B, int T, int H,
                                                             float* __restrict__ dkeys, float* __restrict__ dx,
                                                             int64_t lddx) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * H) return;
  const int64_t b = i / H;
  const int h = (int)(i - b * H);
  const float q = x[b * ldx + q_col + h];
  float dq = 0.f;
  for (int t = 0; t < T; ++t) {
    const int64_t bt = b * T + t;
    const float* dc = dcross + bt * 4 * H;
    const float k = keys[bt * H + h];
    const float d0 = dc[h], d1 = dc[H + h], d2 = dc[2 * H + h], d3 = dc[3 * H + h];
    dq += d0 + d2 + d3 * k;
    dkeys[bt * H + h] += d1 - d2 + d3 * q;
  }
  dx[b * lddx + q_col + h] += dq;
}

// l2 = scale * sum_b ||v_b|| (scale = lambda / B): dx[b, col0 + c] += g * scale * v / ||v|| (0 when
// ||v|| = 0, as torch.norm's backward).  One wave per row; g read from device memory.
__global__ __launch_bounds__(256) void row_l2norm_backward_kernel(const float* __restrict__ x, int64_t ldx,
                                                                  int64_t rows, int col0, int ncols, float scale,
                                                                  const float* __restrict__ gout,
                                                                  float* __restrict__ dx, int64_t lddx) {
  const int lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (r >= rows) return;
  const float* v = x + r * ldx + col0;
  float ss = 0.f;
  for (int c = lane; c < ncols; c += 64) ss = fmaf(v[c], v[c], ss);
  ss = wave_sum(ss);
  const float nrm = sqrtf(ss);
  if (nrm == 0.f) return;
  const float k = gout[0] * scale / nrm;
  for (int c = lane; c < ncols; c += 64) dx[r * lddx + col0 + c] += k * v[c];
}

}  // namespace rk

using namespace rk;

RK_API int rk_din_att_cross(const float* x, int64_t ldx, int32_t q_col, const float* key_table, int64_t key_rows,
                            int64_t ld_key, const int64_t* seq, int64_t ld_seq, int64_t batch, int32_t T, int32_t H,
                            float* keys, float* cross, void* stream) {
  if (!x || !key_table || !seq || !keys || !cross || batch < 0 || T <= 0 || H <= 0 || q_col < 0 || ld_seq < T ||
      key_rows <= 0)
    return fail(RK_ERR_INVALID, "rk_din_att_cross: bad arguments");
  const int64_t n = batch * T * H;
  if (n == 0) return RK_OK;
  if (H % 4 == 0 && ld_key % 4 == 0 &&
      ((reinterpret_cast<uintptr_t>(key_table) | reinterpret_cast<uintptr_t>(keys) |
        reinterpret_cast<uintptr_t>(cross)) & 15) == 0) {
    din_att_cross4_kernel<<<(unsigned)((n / 4 + 255) / 256), 256, 0, (hipStream_t)stream>>>(
        x, ldx, q_col, key_table, key_rows, ld_key, seq, ld_seq, batch, T, H, keys, cross, device_flags());
    return check_launch("rk_din_att_cross");
  }
  din_att_cross_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      x, ldx, q_col, key_table, key_rows, ld_key, seq, ld_seq, batch, T, H, keys, cross, device_flags());
  return check_launch("rk_din_att_cross");
}

RK_API int rk_din_att_pool_forward(const float* a2, int32_t a2_width, const float* w3, const float* b3,
                                   const float* keys, const int64_t* seq_len, int64_t batch, int32_t T, int32_t H,
                                   int32_t use_softmax, float* weights, float* x, int64_t ldx, int32_t att_col,
                                   void* stream) {
  if (!a2 || !w3 || !b3 || !keys || !seq_len || !weights || !x || batch < 0 || T <= 0 || T > kDinMaxT || H <= 0 ||
      H > 64 || a2_width <= 0)
    return fail(RK_ERR_INVALID, "rk_din_att_pool_forward: bad arguments (T <= %d, H <= 64)", kDinMaxT);
  if (batch == 0) return RK_OK;
  din_att_pool_forward_kernel<<<(unsigned)((batch + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      a2, a2_width, w3, b3, keys, seq_len, batch, T, H, use_softmax, sqrtf((float)H), weights, x, ldx,
      att_col, a2_width % 4 == 0 && aligned16(a2));
  return check_launch("rk_din_att_pool_forward");
}

RK_API int rk_din_att_pool_backward(const float* dx, int64_t lddx, int32_t att_col, const float* weights,
                                    const float* keys, const float* a2, int32_t a2_width, const float* w3,
                                    const int64_t* seq_len, int64_t batch, int32_t T, int32_t H, int32_t use_softmax,
                                    float* dkeys, float* da2, void* stream) {
  if (!dx || !weights || !keys || !a2 || !w3 || !seq_len || !dkeys || !da2 || batch < 0 || T <= 0 ||
      T > kDinMaxT || H <= 0 || H > 64 || a2_width <= 0)
    return fail(RK_ERR_INVALID, "rk_din_att_pool_backward: bad arguments (T <= %d, H <= 64)", kDinMaxT);
  if (batch == 0) return RK_OK;
  din_att_pool_backward_kernel<<<(unsigned)((batch + 3) / 4), 256, 0, (hipStream_t)stream>>>(
      dx, lddx, att_col, weights, keys, a2, a2_width, w3, seq_len, batch, T, H, use_softmax, sqrtf((float)H),
      dkeys, da2, H % 4 == 0 && aligned16(keys) && aligned16(dkeys), a2_width % 4 == 0 && aligned16(a2) &&
      aligned16(da2));
  return check_launch("rk_din_att_pool_backward");
}

RK_API int rk_din_cross_fold(const float* dcross, const float* x, int64_t ldx, int32_t q_col, const float* keys,
                             int64_t batch, int32_t T, int32_t H, float* dkeys, float* dx, int64_t lddx,
                             void* stream) {
  if (!dcross || !x || !keys || !dkeys || !dx || batch < 0 || T <= 0 || H <= 0)
    return fail(RK_ERR_INVALID, "rk_din_cross_fold: bad arguments");
  const int64_t n = batch * H;
  if (n == 0) return RK_OK;
  if (H <= 64) {
    din_cross_fold_wg_kernel<<<(unsigned)batch, 256, 0, (hipStream_t)stream>>>(dcross, x, ldx, q_col, keys, batch, T,
                                                                             H, dkeys, dx, lddx);
    return check_launch("rk_din_cross_fold");
  }
  din_cross_fold_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(dcross, x, ldx, q_col, keys,
                                                                                       batch, T, H, dkeys, dx, lddx);
  return check_launch("rk_din_cross_fold");
}

RK_API int rk_row_l2norm_backward(const float* x, int64_t ldx, int64_t rows, int32_t col0, int32_t ncols,
                                  float scale, const float* grad_out, float* dx, int64_t lddx, void* stream) {
  if (!x || !grad_out || !dx || rows < 0 || col0 < 0 || ncols <= 0 || col0 + ncols > ldx || col0 + ncols > lddx)
    return fail(RK_ERR_INVALID, "rk_row_l2norm_backward: bad arguments");
  if (rows == 0) return RK_OK;
  row_l2norm_backward_kernel<<<(unsigned)((rows + 3) / 4), 256, 0, (hipStream_t)stream>>>(x, ldx, rows, col0, ncols,
                                                                                         scale, grad_out, dx, lddx);
  return check_launch("rk_row_l2norm_backward");
}
