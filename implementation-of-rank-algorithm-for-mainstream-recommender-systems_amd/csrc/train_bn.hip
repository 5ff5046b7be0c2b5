// Training pieces of the DeepFM-style tails: train-mode BatchNorm1d + ReLU
// + Dropout (deepfm.py:100-109 in model.train()), their backward, the FM backward and the
// final_layer combine backward (deepfm.py:122-151).
//
// BatchNorm1d in training mode normalises with the batch statistics (biased variance) and
// updates running_mean / running_var with momentum (unbiased variance), as torch does.  The
// statistics are reduced in fp64 (atomics from row blocks): sum and sum of squares of z + bias.
//
// Dropout draws its keep mask from a counter-based hash, never stored: keep(b, n) =
// mix64(seed, stream, b * N + n) >= p * 2^32, recomputed identically by the backward; `stream`
// is read from device memory (rk_rng_next advances it), so a captured hipGraph draws a fresh
// mask on every replay.  The mask is not torch's Philox stream: dropout masks (like torch's
// CPU vs CUDA masks) are a random choice, parity tests feed the same mask to the oracle.
#include "train_common.h"

namespace rk {


constexpr int kBnCols = 64;   // columns per workgroup (one per lane)
constexpr int kBnRows = 64;   // rows per workgroup (16 per wave: B = 4096 gives 64 row blocks)

// sum[n] += sum_b (z[b, n] + bias[n]); sq[n] += sum_b (z + bias)^2   (fp64)
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ z, int64_t ldz, int64_t B, int N,
                                                       const float* __restrict__ bias, double* __restrict__ sum,
                                                       double* __restrict__ sq) {
  __shared__ double red[2][4][kBnCols];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * kBnCols + lane;
  const int64_t b0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t b1 = min<int64_t>(B, b0 + kBnRows);
  double s = 0.0, q = 0.0;
  if (n < N) {
    const float bb = bias ? bias[n] : 0.f;
    #pragma unroll 4
    for (int64_t b = b0 + w; b < b1; b += 4) {
      const double v = (double)(z[b * ldz + n] + bb);
      s += v;
      q += v * v;
    }
  }
  red[0][w][lane] = s;
  red[1][w][lane] = q;
  __syncthreads();
  if (w == 0 && n < N) {
    s = red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane];
    q = red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane];
    atomicAdd(sum + n, s);
    atomicAdd(sq + n, q);
  }
}

struct BnCol {
  float mean, invstd;
};

__device__ __forceinline__ BnCol bn_col(const double* sum, const double* sq, int n, int64_t B, float eps) {
  const double mean = sum[n] / (double)B;
  double var = sq[n] / (double)B - mean * mean;
  var = var < 0.0 ? 0.0 : var;
  BnCol c;
  c.mean = (float)mean;
  c.invstd = 1.0f / sqrtf((float)var + eps);
  return c;
}

// y = dropout(act(gamma * (z + bias - mean) * invstd + beta)); with bn == 0: dropout(act(z + bias)).
// act: RK_ACT_NONE, RK_ACT_RELU or RK_ACT_LEAKY(slope) (BST's DNN units, bst.py:207-211).
// Row block 0 also writes save_mean / save_invstd and updates the running statistics.
__global__ __launch_bounds__(256) void bn_apply_kernel(const float* __restrict__ z, int64_t ldz, int64_t B, int N,
                                                       const float* __restrict__ bias, int bn,
                                                       const double* __restrict__ sum, const double* __restrict__ sq,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, float momentum, float* __restrict__ running_mean,
                                                       float* __restrict__ running_var, float* __restrict__ save_mean,
                                                       float* __restrict__ save_invstd, int act, float slope, uint32_t threshold,
                                                       float scale, uint64_t seed,
                                                       const int64_t* __restrict__ stream_slot,
                                                       float* __restrict__ y, int64_t ldy) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * kBnCols + lane;
  if (n >= N) return;
  const int64_t b0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t b1 = min<int64_t>(B, b0 + kBnRows);
  const float bb = bias ? bias[n] : 0.f;
  float mean = 0.f, invstd = 1.f, g = 1.f, be = 0.f;
  if (bn) {
    const BnCol c = bn_col(sum, sq, n, B, eps);
    mean = c.mean;
    invstd = c.invstd;
    g = gamma ? gamma[n] : 1.f;
    be = beta ? beta[n] : 0.f;
    if (blockIdx.y == 0 && w == 0) {
      save_mean[n] = mean;
      save_invstd[n] = invstd;
      if (running_mean) {
        const double var_b = sq[n] / (double)B - (sum[n] / (double)B) * (sum[n] / (double)B);
        const float unbiased = (float)(B > 1 ? var_b * (double)B / (double)(B - 1) : var_b);
        running_mean[n] = momentum * mean + (1.f - momentum) * running_mean[n];
        running_var[n] = momentum * unbiased + (1.f - momentum) * running_var[n];
      }
    }
  }
  const uint64_t stream = threshold ? (uint64_t)*stream_slot : 0;
  #pragma unroll 4
    for (int64_t b = b0 + w; b < b1; b += 4) {
    float u = z[b * ldz + n] + bb;
    if (bn) u = (u - mean) * invstd * g + be;
    if (act == RK_ACT_RELU) u = u < 0.f ? 0.f : u;
    else if (act == RK_ACT_LEAKY) u = u > 0.f ? u : u * slope;
    if (threshold) u = dropout_keep(seed, stream, (uint64_t)b * N + n, threshold) ? u * scale : 0.f;
    y[b * ldy + n] = u;
  }
}

// Backward statistics: du = dy * keep * scale * act'(u); sum[n] += du; sq[n] += du * xhat.
template <bool STATS>
__global__ __launch_bounds__(256) void bn_backward_kernel(
    const float* __restrict__ dy, int64_t lddy, const float* __restrict__ z, int64_t ldz, int64_t B, int N,
    const float* __restrict__ bias, int bn, const float* __restrict__ save_mean, const float* __restrict__ save_invstd,
    const float* __restrict__ gamma, const float* __restrict__ beta, int act, float slope, uint32_t threshold, float scale,
    uint64_t seed, const int64_t* __restrict__ stream_slot, double* __restrict__ sum, double* __restrict__ sq,
    float* __restrict__ dz, int64_t lddz) {
  __shared__ double red[2][4][kBnCols];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * kBnCols + lane;
  const int64_t b0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t b1 = min<int64_t>(B, b0 + kBnRows);
  double s = 0.0, q = 0.0;
  if (n < N) {
    const float bb = bias ? bias[n] : 0.f;
    const float mean = bn ? save_mean[n] : 0.f, invstd = bn ? save_invstd[n] : 1.f;
    const float g = (bn && gamma) ? gamma[n] : 1.f, be = (bn && beta) ? beta[n] : 0.f;
    float k1 = 0.f, k2 = 0.f;
    if (!STATS && bn) {  // torch: (dy - mean_dy - xmu * invstd^2 * mean_dy_xmu) * invstd * weight
      k1 = (float)(sum[n] / (double)B);
      k2 = (float)(sq[n] / (double)B);
    }
    const uint64_t stream = threshold ? (uint64_t)*stream_slot : 0;
    #pragma unroll 4
    for (int64_t b = b0 + w; b < b1; b += 4) {
      const float xmu = z[b * ldz + n] + bb - mean;
      const float xhat = xmu * invstd;
      float du = dy[b * lddy + n];
      if (threshold) du = dropout_keep(seed, stream, (uint64_t)b * N + n, threshold) ? du * scale : 0.f;
      if (act == RK_ACT_RELU || act == RK_ACT_LEAKY) {
        const float u = bn ? xhat * g + be : xmu;
        du = u > 0.f ? du : (act == RK_ACT_RELU ? 0.f : du * slope);
      }
      if (STATS) {
        s += (double)du;
        q += (double)du * (double)xmu;
      } else {
        dz[b * lddz + n] = bn ? (du - k1 - xmu * invstd * invstd * k2) * invstd * g : du;
      }
    }
  }
  if (STATS) {
    red[0][w][lane] = s;
    red[1][w][lane] = q;
    __syncthreads();
    if (w == 0 && n < N) {
      atomicAdd(sum + n, red[0][0][lane] + red[0][1][lane] + red[0][2][lane] + red[0][3][lane]);
      atomicAdd(sq + n, red[1][0][lane] + red[1][1][lane] + red[1][2][lane] + red[1][3][lane]);
    }
  }
}

// dgamma = sum du * xhat = invstd * sum du * xmu; dbeta = sum du
__global__ void bn_param_grads_kernel(const double* __restrict__ sum, const double* __restrict__ sq,
                                      const float* __restrict__ save_invstd, int N, float* __restrict__ dgamma,
                                      float* __restrict__ dbeta) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  if (dbeta) dbeta[n] = (float)sum[n];
  if (dgamma) dgamma[n] = (float)(sq[n] * (double)save_invstd[n]);
}

__global__ void zero_f64_kernel(double* __restrict__ p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.0;
}

__global__ void rng_next_kernel(int64_t* __restrict__ counter, int64_t* __restrict__ slot) {
  *slot = *counter;
  *counter += 1;
}

// DeepFM FM backward: d e_{f,d} = d_deep[b, f D + d] + dfm2[b] * (S_d - e_{f,d}),
// S_d = sum_f e_{f,d}, e read back from the saved deep input (the concatenated embeddings).
__global__ __launch_bounds__(256) void fm_backward_kernel(const float* __restrict__ deep_in, int64_t ld_in,
                                                          const float* __restrict__ d_deep, int64_t ld_d,
                                                          const float* __restrict__ dfm2, int64_t B, int F, int D,
                                                          float* __restrict__ out, int64_t ld_out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= B * D) return;
  const int64_t b = i / D;
  const int d = (int)(i - b * D);
  const float* e = deep_in + b * ld_in + d;
  float S = 0.f;
  for (int f = 0; f < F; ++f) S += e[f * D];
  const float g2 = dfm2 ? dfm2[b] : 0.f;
  for (int f = 0; f < F; ++f)
    out[b * ld_out + f * D + d] = (d_deep ? d_deep[b * ld_d + f * D + d] : 0.f) + g2 * (S - e[f * D]);
}

// final_layer (Linear(3, 1) over [fm1, fm2, deep]) + sigmoid backward, with the incoming grads of
// all five outputs: g = dtotal + dprob (1 - p) p; d{fm1,fm2,deep} = d_in + g w_{0,1,2};
// dw = sum g [fm1, fm2, deep]; db = sum g  (block partial sums + atomics; zeroed by the host fn)
__global__ __launch_bounds__(256) void fm_combine_backward_kernel(
    const float* __restrict__ dprob, const float* __restrict__ dtotal, const float* __restrict__ dfm1_in,
    const float* __restrict__ dfm2_in, const float* __restrict__ ddeep_in, const float* __restrict__ prob,
    const float* __restrict__ fm1, const float* __restrict__ fm2, const float* __restrict__ deep,
    const float* __restrict__ w, int64_t B, float* __restrict__ dfm1, float* __restrict__ dfm2,
    float* __restrict__ ddeep, float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[4][4];
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (b < B) {
    float g = dtotal ? dtotal[b] : 0.f;
    if (dprob) {
      const float p = prob[b];
      g += dprob[b] * (1.f - p) * p;
    }
    dfm1[b] = (dfm1_in ? dfm1_in[b] : 0.f) + g * w[0];
    dfm2[b] = (dfm2_in ? dfm2_in[b] : 0.f) + g * w[1];
    ddeep[b] = (ddeep_in ? ddeep_in[b] : 0.f) + g * w[2];
    a0 = g * fm1[b];
    a1 = g * fm2[b];
    a2 = g * deep[b];
    a3 = g;
  }
  a0 = wave_sum(a0);
  a1 = wave_sum(a1);
  a2 = wave_sum(a2);
  a3 = wave_sum(a3);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) {
    red[wv][0] = a0;
    red[wv][1] = a1;
    red[wv][2] = a2;
    red[wv][3] = a3;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(threadIdx.x < 3 ? dw + threadIdx.x : db, v);
  }
}

__global__ void zero_f32_kernel(float* __restrict__ p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = 0.f;
}

__global__ void dropout_mask_kernel(uint64_t seed, const int64_t* __restrict__ stream_slot, int64_t B, int N,
                                    uint32_t threshold, float scale, float* __restrict__ out) {
  const uint64_t stream = (uint64_t)*stream_slot;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < B * N; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = dropout_keep(seed, stream, (uint64_t)i, threshold) ? scale : 0.f;
}



// ---- DIN's Dice activation in train mode (din.py:26-36): x = z + bias, xhat = BatchNorm1d(affine
// = False) of x with the batch statistics, p = sigmoid(xhat), y = alpha * (1 - p) * x + p * x.
// The Dice BatchNorm's running statistics are updated like bn_apply_kernel's.
__global__ __launch_bounds__(256) void dice_apply_kernel(const float* __restrict__ z, int64_t ldz, int64_t B, int N,
                                                         const float* __restrict__ bias, const double* __restrict__ sum,
                                                         const double* __restrict__ sq,
                                                         const float* __restrict__ alpha, float eps, float momentum,
                                                         float* __restrict__ running_mean,
                                                         float* __restrict__ running_var, float* __restrict__ save_mean,
                                                         float* __restrict__ save_invstd, float* __restrict__ y,
                                                         int64_t ldy) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * kBnCols + lane;
  if (n >= N) return;
  const int64_t b0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t b1 = min<int64_t>(B, b0 + kBnRows);
  const float bb = bias ? bias[n] : 0.f;
  const BnCol c = bn_col(sum, sq, n, B, eps);
  const float a = alpha[n];
  if (blockIdx.y == 0 && w == 0) {
    save_mean[n] = c.mean;
    save_invstd[n] = c.invstd;
    if (running_mean) {
      const double var_b = sq[n] / (double)B - (sum[n] / (double)B) * (sum[n] / (double)B);
      const float unbiased = (float)(B > 1 ? var_b * (double)B / (double)(B - 1) : var_b);
      running_mean[n] = momentum * c.mean + (1.f - momentum) * running_mean[n];
      running_var[n] = momentum * unbiased + (1.f - momentum) * running_var[n];
    }
  }
  #pragma unroll 4
    for (int64_t b = b0 + w; b < b1; b += 4) {
    const float x = z[b * ldz + n] + bb;
    const float p = 1.0f / (1.0f + expf(-((x - c.mean) * c.invstd)));
    y[b * ldy + n] = a * (1.0f - p) * x + p * x;
  }
}

// ---- Dice in eval (din.py:33-36): xhat = x * scale + shift (BatchNorm1d running statistics,
// folded by rk_bn_fold), p = sigmoid(xhat), y = alpha * (1 - p) * x + p * x.  Thread per element,
// rows over grid.y.
__global__ __launch_bounds__(256) void dice_eval_kernel(const float* __restrict__ x, int64_t ldx, int64_t B, int N,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift,
                                                        const float* __restrict__ alpha, float* __restrict__ y,
                                                        int64_t ldy) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= N) return;
  const float sc = scale[n], sh = shift[n], a = alpha[n];
  for (int64_t b = blockIdx.y; b < B; b += gridDim.y) {
    const float v = x[b * ldx + n];
    const float p = 1.0f / (1.0f + expf(-(v * sc + sh)));
    y[b * ldy + n] = a * (1.0f - p) * v + p * v;
  }
}

// Dice backward.  With g = dy: dx = g * (alpha (1 - p) + p)  [direct]
//   + invstd * (dxhat - mean_b dxhat - xhat * mean_b(dxhat * xhat))  [through the batch statistics],
// dxhat = g * x * (1 - alpha) * p * (1 - p);  dalpha = sum_b g * x * (1 - p).
// STATS pass: ws[0..N) += dxhat, ws[N..2N) += dxhat * xhat, ws[2N..3N) += g * x * (1 - p).
template <bool STATS>
__global__ __launch_bounds__(256) void dice_backward_kernel(const float* __restrict__ dy, int64_t lddy,
                                                            const float* __restrict__ z, int64_t ldz, int64_t B, int N,
                                                            const float* __restrict__ bias,
                                                            const float* __restrict__ alpha,
                                                            const float* __restrict__ save_mean,
                                                            const float* __restrict__ save_invstd,
                                                            double* __restrict__ ws, float* __restrict__ dz,
                                                            int64_t lddz) {
  __shared__ double red[3][4][kBnCols];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * kBnCols + lane;
  const int64_t b0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t b1 = min<int64_t>(B, b0 + kBnRows);
  double s1 = 0.0, s2 = 0.0, sa = 0.0;
  if (n < N) {
    const float bb = bias ? bias[n] : 0.f;
    const float mean = save_mean[n], invstd = save_invstd[n], a = alpha[n];
    float k1 = 0.f, k2 = 0.f;
    if (!STATS) {
      k1 = (float)(ws[n] / (double)B);
      k2 = (float)(ws[N + n] / (double)B);
    }
    #pragma unroll 4
    for (int64_t b = b0 + w; b < b1; b += 4) {
      const float x = z[b * ldz + n] + bb;
      const float xhat = (x - mean) * invstd;
      const float p = 1.0f / (1.0f + expf(-xhat));
      const float g = dy[b * lddy + n];
      const float dxhat = g * x * (1.0f - a) * p * (1.0f - p);
      if (STATS) {
        s1 += (double)dxhat;
        s2 += (double)dxhat * (double)xhat;
        sa += (double)(g * x * (1.0f - p));
      } else {
        dz[b * lddz + n] = g * (a * (1.0f - p) + p) + invstd * (dxhat - k1 - xhat * k2);
      }
    }
  }
  if (STATS) {
    red[0][w][lane] = s1;
    red[1][w][lane] = s2;
    red[2][w][lane] = sa;
    __syncthreads();
    if (w == 0 && n < N) {
#pragma unroll
      for (int k = 0; k < 3; ++k)
        atomicAdd(ws + (int64_t)k * N + n, red[k][0][lane] + red[k][1][lane] + red[k][2][lane] + red[k][3][lane]);
    }
  }
}

__global__ void f64_to_f32_kernel(const double* __restrict__ src, int n, float* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (float)src[i];
}

// ---- DIN's PReLU alternative (din.py:277-279, nn.PReLU(): one shared weight, or one per column
// when nw == N): x = z + bias, y = x > 0 ? x : a x.
__global__ __launch_bounds__(256) void prelu_apply_kernel(const float* __restrict__ z, int64_t ldz, int64_t B, int N,
                                                          const float* __restrict__ bias,
                                                          const float* __restrict__ weight, int nw,
                                                          float* __restrict__ y, int64_t ldy) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * kBnCols + lane;
  if (n >= N) return;
  const int64_t b0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t b1 = min<int64_t>(B, b0 + kBnRows);
  const float bb = bias ? bias[n] : 0.f;
  const float a = weight[nw == 1 ? 0 : n];
  #pragma unroll 4
  for (int64_t b = b0 + w; b < b1; b += 4) {
    const float x = z[b * ldz + n] + bb;
    y[b * ldy + n] = x > 0.f ? x : a * x;
  }
}

// PReLU backward: dz = dy * (x > 0 ? 1 : a); ws[nw == 1 ? 0 : n] += sum_b dy * min(x, 0)  (fp64;
// with one shared weight the columns are first summed across the wave).
__global__ __launch_bounds__(256) void prelu_backward_kernel(const float* __restrict__ dy, int64_t lddy,
                                                             const float* __restrict__ z, int64_t ldz, int64_t B,
                                                             int N, const float* __restrict__ bias,
                                                             const float* __restrict__ weight, int nw,
                                                             double* __restrict__ ws, float* __restrict__ dz,
                                                             int64_t lddz) {
  __shared__ double red[4][kBnCols];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int n = blockIdx.x * kBnCols + lane;
  const int64_t b0 = (int64_t)blockIdx.y * kBnRows;
  const int64_t b1 = min<int64_t>(B, b0 + kBnRows);
  double s = 0.0;
  if (n < N) {
    const float bb = bias ? bias[n] : 0.f;
    const float a = weight[nw == 1 ? 0 : n];
    #pragma unroll 4
    for (int64_t b = b0 + w; b < b1; b += 4) {
      const float x = z[b * ldz + n] + bb;
      const float g = dy[b * lddy + n];
      const bool pos = x > 0.f;
      dz[b * lddz + n] = pos ? g : g * a;
      s += pos ? 0.0 : (double)(g * x);
    }
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0) {
    s = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
    if (nw == 1) {
      #pragma unroll
      for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
      if (lane == 0) atomicAdd(ws, s);
    } else if (n < N) {
      atomicAdd(ws + n, s);
    }
  }
}

}  // namespace rk

using namespace rk;

RK_API int rk_rng_next(int64_t* counter, int64_t* slot, void* stream) {
  if (!counter || !slot) return fail(RK_ERR_INVALID, "rk_rng_next: null pointer");
  rng_next_kernel<<<1, 1, 0, (hipStream_t)stream>>>(counter, slot);
  return check_launch("rk_rng_next");
}

RK_API int rk_dropout_mask(uint64_t seed, const int64_t* stream_slot, int64_t batch, int32_t n, double dropout_p,
                           float* out, void* stream) {
  if (!stream_slot || !out || batch < 0 || n <= 0 || !(dropout_p > 0.0 && dropout_p < 1.0))
    return fail(RK_ERR_INVALID, "rk_dropout_mask: bad arguments");
  if (batch == 0) return RK_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>((batch * n + 255) / 256, 8 * num_cus());
  dropout_mask_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(seed, stream_slot, batch, n,
                                                               dropout_threshold(dropout_p),
                                                               (float)(1.0 / (1.0 - dropout_p)), out);
  return check_launch("rk_dropout_mask");
}

RK_API int rk_bn_act_train_forward(const float* z, int64_t ldz, int64_t batch, int32_t n, const float* bias,
                                   int32_t batch_norm, const float* gamma, const float* beta, float eps,
                                   float momentum, float* running_mean, float* running_var, double* workspace,
                                   float* save_mean, float* save_invstd, int32_t act, float slope,
                                   double dropout_p, uint64_t seed, const int64_t* stream_slot, float* y, int64_t ldy, void* stream) {
  if (!z || !y || batch <= 0 || n <= 0 || ldz < n || ldy < n || (batch_norm && (!workspace || !save_mean ||
      !save_invstd)) || !(dropout_p >= 0.0 && dropout_p < 1.0) || (dropout_p > 0.0 && !stream_slot) ||
      (running_mean != nullptr) != (running_var != nullptr))
    return fail(RK_ERR_INVALID, "rk_bn_act_train_forward: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((n + kBnCols - 1) / kBnCols), (unsigned)((batch + kBnRows - 1) / kBnRows));
  if (batch_norm) {
    zero_f64_kernel<<<(2 * n + 255) / 256, 256, 0, st>>>(workspace, 2 * n);
    bn_stats_kernel<<<grid, 256, 0, st>>>(z, ldz, batch, n, bias, workspace, workspace + n);
  }
  const uint32_t thr = dropout_threshold(dropout_p);
  const float scale = (float)(1.0 / (1.0 - dropout_p));
  bn_apply_kernel<<<grid, 256, 0, st>>>(z, ldz, batch, n, bias, batch_norm, workspace, workspace + n, gamma, beta, eps,
                                        momentum, running_mean, running_var, save_mean, save_invstd, act, slope, thr, scale,
                                        seed, stream_slot, y, ldy);
  return check_launch("rk_bn_act_train_forward");
}

RK_API int rk_bn_act_backward(const float* dy, int64_t lddy, const float* z, int64_t ldz, int64_t batch, int32_t n,
                              const float* bias, int32_t batch_norm, const float* gamma, const float* beta,
                              const float* save_mean, const float* save_invstd, int32_t act, float slope,
                              double dropout_p, uint64_t seed, const int64_t* stream_slot, double* workspace, float* dz, int64_t lddz,
                              float* dgamma, float* dbeta, void* stream) {
  if (!dy || !z || !dz || batch <= 0 || n <= 0 || (batch_norm && (!save_mean || !save_invstd || !workspace)) ||
      !(dropout_p >= 0.0 && dropout_p < 1.0) || (dropout_p > 0.0 && !stream_slot))
    return fail(RK_ERR_INVALID, "rk_bn_act_backward: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((n + kBnCols - 1) / kBnCols), (unsigned)((batch + kBnRows - 1) / kBnRows));
  const uint32_t thr = dropout_threshold(dropout_p);
  const float scale = (float)(1.0 / (1.0 - dropout_p));
  if (batch_norm) {
    zero_f64_kernel<<<(2 * n + 255) / 256, 256, 0, st>>>(workspace, 2 * n);
    bn_backward_kernel<true><<<grid, 256, 0, st>>>(dy, lddy, z, ldz, batch, n, bias, 1, save_mean, save_invstd, gamma,
                                                   beta, act, slope, thr, scale, seed, stream_slot, workspace,
                                                   workspace + n, nullptr, 0);
    if (dgamma || dbeta)
      bn_param_grads_kernel<<<(n + 255) / 256, 256, 0, st>>>(workspace, workspace + n, save_invstd, n, dgamma, dbeta);
  }
  bn_backward_kernel<false><<<grid, 256, 0, st>>>(dy, lddy, z, ldz, batch, n, bias, batch_norm, save_mean,
                                                  save_invstd, gamma, beta, act, slope, thr, scale, seed, stream_slot,
                                                  workspace, batch_norm ? workspace + n : nullptr, dz, lddz);
  return check_launch("rk_bn_act_backward");
}

RK_API int rk_fm_backward(const float* deep_in, int64_t ld_in, const float* d_deep, int64_t ld_d, const float* dfm2,
                          int64_t batch, int32_t num_fields, int32_t dim, float* out, int64_t ld_out, void* stream) {
  if (!deep_in || !out || batch < 0 || num_fields <= 0 || dim <= 0 || ld_in < num_fields * dim ||
      ld_out < num_fields * dim || (d_deep && ld_d < num_fields * dim))
    return fail(RK_ERR_INVALID, "rk_fm_backward: bad arguments");
  if (batch == 0) return RK_OK;
  const int64_t total = batch * dim;
  fm_backward_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(
      deep_in, ld_in, d_deep, ld_d, dfm2, batch, num_fields, dim, out, ld_out);
  return check_launch("rk_fm_backward");
}

RK_API int rk_fm_combine_backward(const float* dprob, const float* dtotal, const float* dfm1_in, const float* dfm2_in,
                                  const float* ddeep_in, const float* prob, const float* fm1, const float* fm2,
                                  const float* deep, const float* final_w, int64_t batch, float* dfm1, float* dfm2,
                                  float* ddeep, float* dfinal_w, float* dfinal_b, void* stream) {
  if (!prob || !fm1 || !fm2 || !deep || !final_w || !dfm1 || !dfm2 || !ddeep || !dfinal_w || !dfinal_b || batch < 0)
    return fail(RK_ERR_INVALID, "rk_fm_combine_backward: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  zero_f32_kernel<<<1, 64, 0, st>>>(dfinal_w, 3);
  zero_f32_kernel<<<1, 64, 0, st>>>(dfinal_b, 1);
  if (batch > 0)
    fm_combine_backward_kernel<<<(unsigned)((batch + 255) / 256), 256, 0, st>>>(
        dprob, dtotal, dfm1_in, dfm2_in, ddeep_in, prob, fm1, fm2, deep, final_w, batch, dfm1, dfm2, ddeep, dfinal_w,
        dfinal_b);
  return check_launch("rk_fm_combine_backward");
}

RK_API int rk_dice_train_forward(const float* z, int64_t ldz, int64_t batch, int32_t n, const float* bias,
                                 const float* alpha, float eps, float momentum, float* running_mean,
                                 float* running_var, double* workspace, float* save_mean, float* save_invstd,
                                 float* y, int64_t ldy, void* stream) {
  if (!z || !y || !alpha || !workspace || !save_mean || !save_invstd || batch <= 0 || n <= 0 || ldz < n ||
      ldy < n || (running_mean != nullptr) != (running_var != nullptr))
    return fail(RK_ERR_INVALID, "rk_dice_train_forward: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((n + kBnCols - 1) / kBnCols), (unsigned)((batch + kBnRows - 1) / kBnRows));
  zero_f64_kernel<<<(2 * n + 255) / 256, 256, 0, st>>>(workspace, 2 * n);
  bn_stats_kernel<<<grid, 256, 0, st>>>(z, ldz, batch, n, bias, workspace, workspace + n);
  dice_apply_kernel<<<grid, 256, 0, st>>>(z, ldz, batch, n, bias, workspace, workspace + n, alpha, eps, momentum,
                                          running_mean, running_var, save_mean, save_invstd, y, ldy);
  return check_launch("rk_dice_train_forward");
}

RK_API int rk_dice_backward(const float* dy, int64_t lddy, const float* z, int64_t ldz, int64_t batch, int32_t n,
                            const float* bias, const float* alpha, const float* save_mean, const float* save_invstd,
                            double* workspace, float* dz, int64_t lddz, float* dalpha, void* stream) {
  if (!dy || !z || !dz || !alpha || !save_mean || !save_invstd || !workspace || batch <= 0 || n <= 0)
    return fail(RK_ERR_INVALID, "rk_dice_backward: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((n + kBnCols - 1) / kBnCols), (unsigned)((batch + kBnRows - 1) / kBnRows));
  zero_f64_kernel<<<(3 * n + 255) / 256, 256, 0, st>>>(workspace, 3 * n);
  dice_backward_kernel<true><<<grid, 256, 0, st>>>(dy, lddy, z, ldz, batch, n, bias, alpha, save_mean, save_invstd,
                                                   workspace, nullptr, 0);
  if (dalpha) f64_to_f32_kernel<<<(n + 255) / 256, 256, 0, st>>>(workspace + 2 * n, n, dalpha);
  dice_backward_kernel<false><<<grid, 256, 0, st>>>(dy, lddy, z, ldz, batch, n, bias, alpha, save_mean, save_invstd,
                                                    workspace, dz, lddz);
  return check_launch("rk_dice_backward");
}

RK_API int rk_prelu_train_forward(const float* z, int64_t ldz, int64_t batch, int32_t n, const float* bias,
                                  const float* weight, int32_t num_weights, float* y, int64_t ldy, void* stream) {
  if (!z || !y || !weight || batch <= 0 || n <= 0 || ldz < n || ldy < n || (num_weights != 1 && num_weights != n))
    return fail(RK_ERR_INVALID, "rk_prelu_train_forward: bad arguments");
  dim3 grid((unsigned)((n + kBnCols - 1) / kBnCols), (unsigned)((batch + kBnRows - 1) / kBnRows));
  prelu_apply_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(z, ldz, batch, n, bias, weight, num_weights, y, ldy);
  return check_launch("rk_prelu_train_forward");
}

RK_API int rk_prelu_backward(const float* dy, int64_t lddy, const float* z, int64_t ldz, int64_t batch, int32_t n,
                             const float* bias, const float* weight, int32_t num_weights, double* workspace,
                             float* dz, int64_t lddz, float* dweight, void* stream) {
  if (!dy || !z || !dz || !weight || !workspace || batch <= 0 || n <= 0 || ldz < n || lddy < n || lddz < n ||
      (num_weights != 1 && num_weights != n))
    return fail(RK_ERR_INVALID, "rk_prelu_backward: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((n + kBnCols - 1) / kBnCols), (unsigned)((batch + kBnRows - 1) / kBnRows));
  zero_f64_kernel<<<(num_weights + 255) / 256, 256, 0, st>>>(workspace, num_weights);
  prelu_backward_kernel<<<grid, 256, 0, st>>>(dy, lddy, z, ldz, batch, n, bias, weight, num_weights, workspace, dz,
                                              lddz);
  if (dweight) f64_to_f32_kernel<<<(num_weights + 255) / 256, 256, 0, st>>>(workspace, num_weights, dweight);
  return check_launch("rk_prelu_backward");
}

RK_API int rk_dice_forward(const float* x, int64_t ldx, int64_t rows, int32_t n, const float* bn_scale,
                           const float* bn_shift, const float* alpha, float* y, int64_t ldy, void* stream) {
  if (!x || !y || !bn_scale || !bn_shift || !alpha || rows < 0 || n <= 0 || ldx < n || ldy < n)
    return fail(RK_ERR_INVALID, "rk_dice_forward: bad arguments");
  if (rows == 0) return RK_OK;
  dim3 grid((unsigned)((n + 255) / 256), (unsigned)std::min<int64_t>(rows, 4096));
  dice_eval_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(x, ldx, rows, n, bn_scale, bn_shift, alpha, y, ldy);
  return check_launch("rk_dice_forward");
}
