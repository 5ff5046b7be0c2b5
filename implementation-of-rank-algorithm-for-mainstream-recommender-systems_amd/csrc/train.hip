// Training: the backward of the forward path and the optimizer step that the
// reference's train() loops run through autograd (`loss.backward(); optimizer.step()`,
// dcn.py:196-201; the same in every script).
//
//   rk_gemm                 C (+)= op(A) . op(B)^T on FP32 MFMA, optional ReLU mask on A
//                           (dz = dh * [h > 0]) and row sums of op(A) (bias gradients); split
//                           over the reduction with float atomics when the output tile grid is
//                           too small to fill the GPU (weight gradients: reduction = batch)
//   rk_logit_head_backward  Linear(K, 1) + sigmoid head: g = dlogit + dprob * p (1 - p),
//                           dX = g w, dw = sum_b g x, db = sum_b g   (dcn.py:177-179)
//   rk_dcn_cross_backward   gradient of the cross stack w.r.t. x0 (dcn.py:46-49); the per-call
//                           cross weights are not module parameters, their gradients are dropped
//                           as in the reference
//   rk_embedding_backward   nn.Embedding's dense weight gradient: rows scattered with atomics
//   rk_adam_step            torch.optim.Adam (foreach / single-tensor math) over many tensors in
//                           one launch
#include "common.h"

namespace rk {

// ------------------------------------------------------------------------------------------
// GEMM: C[m, n] (+)= sum_r opA(m, r) * opB(n, r)
//   opA(m, r) = TA ? A[r * lda + m] : A[m * lda + r]   (times [mask(m, r) > 0] when masked)
//   opB(n, r) = TB ? B[r * ldb + n] : B[n * ldb + r]
// 64 x 64 output tile per 256-thread workgroup (2 x 2 waves of 32 x 32, v_mfma_f32_32x32x2_f32);
// the reduction is staged through LDS 32 at a time, k-major ([r][m], row stride 65) so both the
// transposed and the plain global layouts store without bank conflicts and the MFMA operand
// reads are consecutive across lanes.  The next tile's global loads are issued before the
// current tile's MFMAs.
// ------------------------------------------------------------------------------------------
constexpr int kGT = 64;       // output tile edge
constexpr int kGR = 64;       // reduction step (2048 MFMA cycles per wave: covers a global round trip)
constexpr int kGLD = kGT + 1;  // LDS row stride
constexpr int kGV = kGT * kGR / 256;  // staged values per thread and operand

template <bool T>
__device__ __forceinline__ void stage_load(const float* __restrict__ P, int64_t ld, const float* __restrict__ mask,
                                           int64_t rows, int64_t R, int64_t row0, int64_t r0, int tid,
                                           float (&v)[kGV]) {
  // 64 rows x 64 reduction values, kGV per thread, coalesced along the contiguous dim.  Loads
  // are unconditional (out-of-range lanes read element 0 and are zeroed afterwards) so all of
  // them, and the mask's, are in flight together instead of one branch + wait per element.
  int64_t off[kGV];
  bool ok[kGV];
#pragma unroll
  for (int i = 0; i < kGV; ++i) {
    int rr, mm;
    if (T) {  // contiguous along rows
      mm = tid & 63;
      rr = (tid >> 6) + 4 * i;
    } else {  // contiguous along the reduction
      rr = tid & 63;
      mm = (tid >> 6) + 4 * i;
    }
    const int64_t m = row0 + mm, r = r0 + rr;
    ok[i] = m < rows && r < R;
    off[i] = ok[i] ? (T ? r * ld + m : m * ld + r) : 0;
  }
#pragma unroll
  for (int i = 0; i < kGV; ++i) v[i] = P[off[i]];
  if (mask) {
    float mk[kGV];
#pragma unroll
    for (int i = 0; i < kGV; ++i) mk[i] = mask[off[i]];
#pragma unroll
    for (int i = 0; i < kGV; ++i) v[i] = (ok[i] && mk[i] > 0.f) ? v[i] : 0.f;
  } else {
#pragma unroll
    for (int i = 0; i < kGV; ++i) v[i] = ok[i] ? v[i] : 0.f;
  }
}

template <bool T>
__device__ __forceinline__ void stage_store(float* __restrict__ S, int tid, const float (&v)[kGV]) {
#pragma unroll
  for (int i = 0; i < kGV; ++i) {
    int rr, mm;
    if (T) {
      mm = tid & 63;
      rr = (tid >> 6) + 4 * i;
    } else {
      rr = tid & 63;
      mm = (tid >> 6) + 4 * i;
    }
    S[rr * kGLD + mm] = v[i];
  }
}

template <bool TA, bool TB, bool ATOMIC>
__global__ __launch_bounds__(256) void gemm_kernel(int64_t M, int64_t N, int64_t R, int64_t r_per_split,
                                                   const float* __restrict__ A, int64_t lda,
                                                   const float* __restrict__ A_mask, const float* __restrict__ B,
                                                   int64_t ldb, float* __restrict__ C, int64_t ldc,
                                                   float* __restrict__ row_sums, int accumulate) {
  __shared__ float As[kGR * kGLD];
  __shared__ float Bs[kGR * kGLD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * kGT, n0 = (int64_t)blockIdx.y * kGT;
  const int64_t rb = (int64_t)blockIdx.z * r_per_split;
  const int64_t re = min<int64_t>(R, rb + r_per_split);
  const bool sums = row_sums && blockIdx.y == 0;
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  float rsum = 0.f;
  float va[kGV], vb[kGV];
  if (rb < re) {
    stage_load<TA>(A, lda, A_mask, M, re, m0, rb, tid, va);
    stage_load<TB>(B, ldb, nullptr, N, re, n0, rb, tid, vb);
  }
  for (int64_t r0 = rb; r0 < re; r0 += kGR) {
    stage_store<TA>(As, tid, va);
    stage_store<TB>(Bs, tid, vb);
    __syncthreads();
    if (r0 + kGR < re) {  // next tile in flight during this tile's MFMAs
      stage_load<TA>(A, lda, A_mask, M, re, m0, r0 + kGR, tid, va);
      stage_load<TB>(B, ldb, nullptr, N, re, n0, r0 + kGR, tid, vb);
    }
    if (sums && tid < kGT) {
#pragma unroll 16
      for (int r = 0; r < kGR; ++r) rsum += As[r * kGLD + tid];
    }
    const float* a_col = As + wm * 32 + (lane & 31);
    const float* b_col = Bs + wn * 32 + (lane & 31);
    const int k1 = lane >> 5;
    // all operand reads of the step first: one wait, then 32 back-to-back MFMAs (reading them one
    // MFMA at a time put an LDS round trip in front of every MFMA)
    float av[kGR / 2], bv[kGR / 2];
#pragma unroll
    for (int k = 0; k < kGR / 2; ++k) {
      av[k] = a_col[(2 * k + k1) * kGLD];
      bv[k] = b_col[(2 * k + k1) * kGLD];
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < kGR / 2; ++k) acc = mfma32(av[k], bv[k], acc);
    __syncthreads();
  }
  const int64_t n = n0 + wn * 32 + (lane & 31);
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = m0 + wm * 32 + acc_row(r, lane);
    if (m < M && n < N) {
      float* c = C + m * ldc + n;
      if (ATOMIC)
        atomicAdd(c, acc[r]);
      else
        *c = accumulate ? *c + acc[r] : acc[r];
    }
  }
  if (sums && tid < kGT && m0 + tid < M) {
    if (ATOMIC)
      atomicAdd(row_sums + m0 + tid, rsum);
    else
      row_sums[m0 + tid] = accumulate ? row_sums[m0 + tid] + rsum : rsum;
  }
}

__global__ void zero2d_kernel(float* __restrict__ p, int64_t rows, int64_t cols, int64_t ld) {
  const int64_t n = rows * cols;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[(i / cols) * ld + i % cols] = 0.f;
}

__global__ void relu_backward_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                     float* __restrict__ out, int64_t n, int accumulate) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = y[i] > 0.f ? dy[i] : 0.f;
    out[i] = accumulate ? out[i] + v : v;
  }
}

static void zero2d(float* p, int64_t rows, int64_t cols, int64_t ld, hipStream_t st) {
  const int64_t n = rows * cols;
  if (n <= 0) return;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4 * num_cus());
  zero2d_kernel<<<blocks, 256, 0, st>>>(p, rows, cols, ld);
}

// ------------------------------------------------------------------------------------------
// Linear(K, 1) + sigmoid head backward over an input row made of up to two column blocks
// (DCN: [cross_vec | dnn_vec], dcn.py:177).  Each workgroup takes a block of rows; thread t
// owns columns t, t + 256; per-column partial sums of g * x are combined with atomics.
// ------------------------------------------------------------------------------------------
constexpr int kHeadRows = 64;

__global__ __launch_bounds__(256) void head_backward_kernel(
    const float* __restrict__ dlogit, const float* __restrict__ dprob, const float* __restrict__ prob, int64_t batch,
    const float* __restrict__ xa, int64_t ld_xa, int ka, const float* __restrict__ xb, int64_t ld_xb, int kb,
    const float* __restrict__ w, float* __restrict__ dxa, int64_t ld_dxa, float* __restrict__ dxb, int64_t ld_dxb,
    float* __restrict__ dw, float* __restrict__ db, float* __restrict__ g_out) {
  __shared__ float gs[kHeadRows];
  const int tid = threadIdx.x;
  const int64_t b0 = (int64_t)blockIdx.x * kHeadRows;
  const int rows = (int)min<int64_t>(kHeadRows, batch - b0);
  if (tid < rows) {
    const int64_t b = b0 + tid;
    float g = dlogit ? dlogit[b] : 0.f;
    if (dprob) {
      const float p = prob[b];
      g += dprob[b] * (1.f - p) * p;  // sigmoid_backward: grad * (1 - y) * y
    }
    gs[tid] = g;
    if (g_out) g_out[b] = g;
  }
  __syncthreads();
  const int K = ka + kb;
  for (int k = tid; k < K; k += 256) {
    const bool in_a = k < ka;
    const int c = in_a ? k : k - ka;
    const float* x = in_a ? xa : xb;
    const int64_t ldx = in_a ? ld_xa : ld_xb;
    float* dx = in_a ? dxa : dxb;
    const int64_t lddx = in_a ? ld_dxa : ld_dxb;
    const float wk = w[k];
    float s = 0.f;
    for (int i = 0; i < rows; ++i) {
      const int64_t b = b0 + i;
      const float g = gs[i];
      s = fmaf(g, x[b * ldx + c], s);
      if (dx) dx[b * lddx + c] = g * wk;
    }
    atomicAdd(dw + k, s);
  }
  if (tid == 0) {
    float s = 0.f;
    for (int i = 0; i < rows; ++i) s += gs[i];
    atomicAdd(db, s);
  }
}

// ------------------------------------------------------------------------------------------
// DCN cross stack backward (dcn.py:46-49): one wave per row, columns lane + 64 j.
//   forward  s_l = x_l . w_l;  x_{l+1} = (x0 * s_l + b_l) + x_l
//   backward g = dx_{l+1}:  dx0 += g s_l;  ds_l = g . x0;  dx_l = g + ds_l w_l;  dx0 += dx_0
// ------------------------------------------------------------------------------------------
constexpr int kCrossBwdPerLane = 4;
constexpr int kCrossBwdMaxLayers = 8;

__global__ __launch_bounds__(256) void cross_backward_kernel(const float* __restrict__ x0, int64_t ld_x0,
                                                             int64_t batch, int width,
                                                             const float* __restrict__ cw,
                                                             const float* __restrict__ cb, int L,
                                                             const float* __restrict__ dxl, int64_t ld_dxl,
                                                             float* __restrict__ dx0, int64_t ld_dx0,
                                                             int accumulate) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (gridDim.x * (int64_t)blockDim.x) >> 6;
  for (int64_t b = wave; b < batch; b += nwaves) {
    float x[kCrossBwdPerLane], xl[kCrossBwdPerLane], s[kCrossBwdMaxLayers];
#pragma unroll
    for (int j = 0; j < kCrossBwdPerLane; ++j) {
      const int c = lane + 64 * j;
      x[j] = c < width ? x0[b * ld_x0 + c] : 0.f;
      xl[j] = x[j];
    }
    // forward recompute: only the scalars s_l are needed
#pragma unroll
    for (int l = 0; l < kCrossBwdMaxLayers; ++l) {
      if (l >= L) break;
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < kCrossBwdPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) d = fmaf(xl[j], cw[(int64_t)l * width + c], d);
      }
      d = wave_sum(d);
      s[l] = d;
#pragma unroll
      for (int j = 0; j < kCrossBwdPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) xl[j] = (x[j] * d + cb[(int64_t)l * width + c]) + xl[j];
      }
    }
    float g[kCrossBwdPerLane], gx0[kCrossBwdPerLane];
#pragma unroll
    for (int j = 0; j < kCrossBwdPerLane; ++j) {
      const int c = lane + 64 * j;
      g[j] = c < width ? dxl[b * ld_dxl + c] : 0.f;
      gx0[j] = 0.f;
    }
#pragma unroll
    for (int l = kCrossBwdMaxLayers - 1; l >= 0; --l) {
      if (l >= L) continue;
      float ds = 0.f;
#pragma unroll
      for (int j = 0; j < kCrossBwdPerLane; ++j) {
        gx0[j] = fmaf(g[j], s[l], gx0[j]);
        ds = fmaf(g[j], x[j], ds);
      }
      ds = wave_sum(ds);
#pragma unroll
      for (int j = 0; j < kCrossBwdPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) g[j] = fmaf(ds, cw[(int64_t)l * width + c], g[j]);
      }
    }
#pragma unroll
    for (int j = 0; j < kCrossBwdPerLane; ++j) {
      const int c = lane + 64 * j;
      if (c < width) {
        float* o = dx0 + b * ld_dx0 + c;
        const float v = gx0[j] + g[j];
        *o = accumulate ? *o + v : v;
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// nn.Embedding dense weight gradient: grad[idx[b], j] += dx[b, out_col + j] (atomics).
// One workgroup row-block per segment (grid.y); threads over (row, column) of the segment.
// ------------------------------------------------------------------------------------------
struct GradSegs {
  rk_segment s[RK_MAX_SEGMENTS];
};

// Small tables (rows * dim <= kEmbLdsFloats: device, tags, ...) take every sample, so global
// atomics on them serialise: those are accumulated per workgroup in LDS first and flushed once
// (PRIV).  Large tables add straight into the gradient with global atomics; each thread issues
// kEmbUnroll index and dx loads before its first atomic, so the memory round trips overlap.
// Zero contributions are skipped (see below).
constexpr int kEmbLdsFloats = 8192;
constexpr int kEmbUnroll = 8;

template <bool PRIV>
__global__ __launch_bounds__(256) void embedding_backward_kernel(GradSegs segs, int64_t batch,
                                                                 const float* __restrict__ dx, int64_t ld_dx,
                                                                 uint32_t* flags) {
  __shared__ float acc[PRIV ? kEmbLdsFloats : 1];
  const rk_segment& s = segs.s[blockIdx.y];
  if (!s.idx) return;
  const int dim = s.dim;
  const int64_t n = batch * dim;
  float* grad = const_cast<float*>(s.src);
  if (PRIV != (s.rows * dim <= kEmbLdsFloats)) return;  // the other instantiation owns this segment
  if (PRIV) {
    for (int i = threadIdx.x; i < s.rows * dim; i += blockDim.x) acc[i] = 0.f;
    __syncthreads();
  }
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i0 < n; i0 += stride * kEmbUnroll) {
    int64_t r[kEmbUnroll];
    float v[kEmbUnroll];
    int j[kEmbUnroll];
#pragma unroll
    for (int u = 0; u < kEmbUnroll; ++u) {
      const int64_t i = i0 + u * stride;
      const int64_t b = i < n ? i / dim : 0;
      j[u] = (int)(i - b * dim);
      r[u] = i < n ? s.idx[b * s.idx_stride] : -1;
      v[u] = i < n ? dx[b * ld_dx + s.out_col + j[u]] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kEmbUnroll; ++u) {
      if (i0 + u * stride >= n) continue;
      if (r[u] < 0 || r[u] >= s.rows) {
        if (j[u] == 0) flag_oob(flags);
        continue;
      }
      // adding 0 changes nothing: padded history positions (index 0, zero gradient) would
      // otherwise all hit row 0 and serialise on its atomics
      if (v[u] == 0.f) continue;
      if (PRIV)
        atomicAdd(acc + r[u] * dim + j[u], v[u]);
      else
        atomicAdd(grad + r[u] * s.src_ld + j[u], v[u]);
    }
  }
  if (PRIV) {
    __syncthreads();
    for (int i = threadIdx.x; i < s.rows * dim; i += blockDim.x) {
      const float x = acc[i];
      if (x != 0.f) atomicAdd(grad + (i / dim) * s.src_ld + i % dim, x);
    }
  }
}

// ------------------------------------------------------------------------------------------
// Adam, torch.optim.Adam semantics (amsgrad = maximize = False):
//   g = grad (+ weight_decay * p);  m = lerp(m, g, 1 - beta1);  v = v * beta2 + (1 - beta2) g^2
//   p = p - step_size * m / (sqrt(v) / sqrt(bias_correction2) + eps),  step_size = lr / bc1
// Workgroups walk 4096-element chunks; the chunk -> tensor map is a prefix table in the args.
// ------------------------------------------------------------------------------------------
constexpr int kAdamMaxTensors = 64;
constexpr int64_t kAdamChunk = 4096;

struct AdamList {
  rk_adam_tensor t[kAdamMaxTensors];
  int64_t chunk_start[kAdamMaxTensors + 1];
};

// CAPTURABLE: the step count lives in device memory (torch's capturable=True layout, one float
// per tensor, incremented by adam_step_inc_kernel first) and the bias corrections are formed on
// the device in float in torch's capturable order:
//   step_size = 1 / ((beta1^t - 1) / lr);  bc2_sqrt = sqrt(-(beta2^t - 1));
//   p += m / ((sqrt(v) / bc2_sqrt + eps) / step_size)
template <bool CAPTURABLE>
__global__ __launch_bounds__(256) void adam_kernel(AdamList list, int n, float one_minus_b1, float beta1, float beta2,
                                                   float one_minus_b2, float eps, float weight_decay, float lr,
                                                   float step_size, float bc2_sqrt) {
  const int64_t chunk = blockIdx.x;
  int t = 0;
  while (t + 1 < n && list.chunk_start[t + 1] <= chunk) ++t;
  const rk_adam_tensor& T = list.t[t];
  if (CAPTURABLE) {
    const float st = *T.step;
    step_size = 1.f / ((powf(beta1, st) - 1.f) / lr);  // negative
    bc2_sqrt = sqrtf(-(powf(beta2, st) - 1.f));
  }
  const int64_t base = (chunk - list.chunk_start[t]) * kAdamChunk;
  const int64_t end = min<int64_t>(T.numel, base + kAdamChunk);
  for (int64_t i = base + threadIdx.x; i < end; i += blockDim.x) {
    float p = T.param[i];
    float g = T.grad[i];
    if (weight_decay != 0.f) g = g + weight_decay * p;
    float m = T.exp_avg[i];
    m = m + one_minus_b1 * (g - m);  // lerp, weight < 0.5 branch
    float v = T.exp_avg_sq[i] * beta2;
    v = v + one_minus_b2 * g * g;  // addcmul_: self + value * t1 * t2
    if (CAPTURABLE) {
      const float denom = (sqrtf(v) / bc2_sqrt + eps) / step_size;
      p = p + m / denom;
    } else {
      const float denom = sqrtf(v) / bc2_sqrt + eps;
      p = p + (-step_size) * (m / denom);
    }
    T.exp_avg[i] = m;
    T.exp_avg_sq[i] = v;
    T.param[i] = p;
  }
}

__global__ void adam_step_inc_kernel(AdamList list, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) *list.t[t].step += 1.f;
}

}  // namespace rk

using namespace rk;

RK_API int rk_gemm(int32_t trans_a, int32_t trans_b, int64_t M, int64_t N, int64_t R, const float* A, int64_t lda,
                   const float* A_mask, const float* B, int64_t ldb, float* C, int64_t ldc, float* row_sums,
                   int32_t accumulate, int32_t split, void* stream) {
  if (M < 0 || N < 0 || R < 0 || !C || ldc < N) return fail(RK_ERR_INVALID, "rk_gemm: bad shape / output");
  if (R > 0 && (!A || !B)) return fail(RK_ERR_INVALID, "rk_gemm: null operand");
  if (lda < (trans_a ? M : R) || ldb < (trans_b ? N : R))
    return fail(RK_ERR_INVALID, "rk_gemm: leading dimension too small (lda %lld, ldb %lld)", (long long)lda,
                (long long)ldb);
  hipStream_t st = (hipStream_t)stream;
  if (M == 0 || N == 0) return RK_OK;
  const int64_t tm = (M + kGT - 1) / kGT, tn = (N + kGT - 1) / kGT;
  if (tm > INT32_MAX || tn > 65535) return fail(RK_ERR_UNSUPPORTED, "rk_gemm: output too large");
  if (!trans_a && !row_sums && split <= 1 &&
      gemm_rows_try(A, lda, A_mask, nullptr, 0, B, ldb, trans_b, M, (int)N, (int)R, C, ldc, accumulate, nullptr, st))
    return check_launch("rk_gemm");
  if (split <= 0) {  // enough workgroups to cover the CUs twice, >= 256 reduction values each
    const int64_t want = (2 * num_cus() + tm * tn - 1) / (tm * tn);
    split = (int32_t)std::max<int64_t>(1, std::min<int64_t>({want, R / 256, 1024}));
  }
  int64_t rps = (R + split - 1) / split;
  rps = (rps + kGR - 1) / kGR * kGR;
  split = (int32_t)std::max<int64_t>(1, (R + rps - 1) / std::max<int64_t>(rps, 1));
  const bool atomic = split > 1;
  if (atomic && !accumulate) {
    zero2d(C, M, N, ldc, st);
    if (row_sums) zero2d(row_sums, 1, M, M, st);
  }
  dim3 grid((unsigned)tm, (unsigned)tn, (unsigned)split);
#define RK_GEMM_CASE(TA_, TB_)                                                                                 \
  if (!!trans_a == TA_ && !!trans_b == TB_) {                                                                  \
    if (atomic)                                                                                                \
      gemm_kernel<TA_, TB_, true><<<grid, 256, 0, st>>>(M, N, R, rps, A, lda, A_mask, B, ldb, C, ldc, row_sums, \
                                                        accumulate);                                          \
    else                                                                                                       \
      gemm_kernel<TA_, TB_, false><<<grid, 256, 0, st>>>(M, N, R, rps, A, lda, A_mask, B, ldb, C, ldc,         \
                                                         row_sums, accumulate);                               \
  }
  RK_GEMM_CASE(false, false)
  RK_GEMM_CASE(false, true)
  RK_GEMM_CASE(true, false)
  RK_GEMM_CASE(true, true)
#undef RK_GEMM_CASE
  return check_launch("rk_gemm");
}

RK_API int rk_relu_backward(const float* dy, const float* y, float* out, int64_t n, int32_t accumulate, void* stream) {
  if (n < 0 || (n > 0 && (!dy || !y || !out))) return fail(RK_ERR_INVALID, "rk_relu_backward: bad arguments");
  if (n == 0) return RK_OK;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 8 * num_cus());
  relu_backward_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(dy, y, out, n, accumulate);
  return check_launch("rk_relu_backward");
}

RK_API int rk_logit_head_backward(const float* dlogit, const float* dprob, const float* prob, int64_t batch,
                                  const float* xa, int64_t ld_xa, int32_t ka, const float* xb, int64_t ld_xb,
                                  int32_t kb, const float* w, float* dxa, int64_t ld_dxa, float* dxb, int64_t ld_dxb,
                                  float* dw, float* db, float* g_out, void* stream) {
  if (batch < 0 || ka <= 0 || kb < 0 || !xa || (kb > 0 && !xb) || !w || !dw || !db || (dprob && !prob))
    return fail(RK_ERR_INVALID, "rk_logit_head_backward: bad arguments");
  hipStream_t st = (hipStream_t)stream;
  zero2d(dw, 1, ka + kb, ka + kb, st);
  zero2d(db, 1, 1, 1, st);
  if (batch == 0) return check_launch("rk_logit_head_backward");
  const int64_t blocks = (batch + kHeadRows - 1) / kHeadRows;
  head_backward_kernel<<<(unsigned)blocks, 256, 0, st>>>(dlogit, dprob, prob, batch, xa, ld_xa, ka, xb, ld_xb, kb, w,
                                                         dxa, ld_dxa, dxb, ld_dxb, dw, db, g_out);
  return check_launch("rk_logit_head_backward");
}

RK_API int rk_dcn_cross_backward(const float* x0, int64_t ld_x0, int64_t batch, int32_t width, const float* cross_w,
                                 const float* cross_b, int32_t num_layers, const float* dxl, int64_t ld_dxl, float* dx0,
                                 int64_t ld_dx0, int32_t accumulate, void* stream) {
  if (!x0 || (num_layers > 0 && (!cross_w || !cross_b)) || !dxl || !dx0 || batch < 0)
    return fail(RK_ERR_INVALID, "rk_dcn_cross_backward: bad arguments");
  if (width <= 0 || width > 64 * kCrossBwdPerLane || num_layers < 0 || num_layers > kCrossBwdMaxLayers)
    return fail(RK_ERR_UNSUPPORTED, "rk_dcn_cross_backward: width %d (max %d), %d layers (max %d)", width,
                64 * kCrossBwdPerLane, num_layers, kCrossBwdMaxLayers);
  if (batch == 0) return RK_OK;
  const int64_t blocks = std::min<int64_t>((batch + 3) / 4, 8 * num_cus());
  cross_backward_kernel<<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(x0, ld_x0, batch, width, cross_w, cross_b,
                                                                           num_layers, dxl, ld_dxl, dx0, ld_dx0,
                                                                           accumulate);
  return check_launch("rk_dcn_cross_backward");
}

RK_API int rk_embedding_backward(const rk_segment* grads, int32_t nseg, int64_t batch, const float* dx, int64_t ld_dx,
                                 void* stream) {
  if (!grads || nseg <= 0 || nseg > RK_MAX_SEGMENTS || !dx || batch < 0)
    return fail(RK_ERR_INVALID, "rk_embedding_backward: bad arguments");
  GradSegs t;
  int64_t widest = 0;
  for (int i = 0; i < nseg; ++i) {
    const rk_segment& s = grads[i];
    if (s.idx && (!s.src || s.dim <= 0 || s.rows <= 0 || s.out_col < 0 || s.out_col + s.dim > ld_dx))
      return fail(RK_ERR_INVALID, "rk_embedding_backward: segment %d invalid", i);
    t.s[i] = s;
    if (s.idx) widest = std::max<int64_t>(widest, s.dim);
  }
  if (batch == 0 || widest == 0) return RK_OK;
  const int64_t per = batch * widest;
  bool any_priv = false, any_global = false;
  for (int i = 0; i < nseg; ++i)
    if (t.s[i].idx) (t.s[i].rows * t.s[i].dim <= kEmbLdsFloats ? any_priv : any_global) = true;
  hipStream_t st = (hipStream_t)stream;
  if (any_priv) {  // a few workgroups per small table: each flushes its whole LDS image once
    const unsigned bx = (unsigned)std::min<int64_t>((per + 255) / 256, 2 * num_cus());
    embedding_backward_kernel<true><<<dim3(bx, (unsigned)nseg), 256, 0, st>>>(t, batch, dx, ld_dx, device_flags());
  }
  if (any_global) {
    const unsigned bx = (unsigned)std::min<int64_t>((per + 256 * kEmbUnroll - 1) / (256 * kEmbUnroll), 8 * num_cus());
    embedding_backward_kernel<false><<<dim3(bx, (unsigned)nseg), 256, 0, st>>>(t, batch, dx, ld_dx, device_flags());
  }
  return check_launch("rk_embedding_backward");
}

RK_API int rk_adam_step(const rk_adam_tensor* tensors, int32_t n, double lr, double beta1, double beta2, double eps,
                        double weight_decay, int64_t step, void* stream) {
  if (!tensors || n < 0 || (step < 1 && !(n > 0 && tensors[0].step)) || !(beta1 >= 0.0 && beta1 < 1.0) ||
      !(beta2 >= 0.0 && beta2 < 1.0))
    return fail(RK_ERR_INVALID, "rk_adam_step: bad arguments");
  // every scalar derived in double like torch's Python-side arithmetic, then rounded to float
  // (the kernels' opmath): 1 - beta2 from a float beta2 would be off by 1e-5 relative
  const double bc1 = 1.0 - std::pow(beta1, (double)step);
  const double bc2 = 1.0 - std::pow(beta2, (double)step);
  const float step_size = (float)(lr / bc1);
  const float bc2_sqrt = (float)std::sqrt(bc2);
  const float omb1 = (float)(1.0 - beta1), omb2 = (float)(1.0 - beta2);
  hipStream_t st = (hipStream_t)stream;
  const bool capturable = n > 0 && tensors[0].step != nullptr;
  for (int base = 0; base < n; base += kAdamMaxTensors) {
    AdamList list;
    const int cnt = std::min(kAdamMaxTensors, n - base);
    int64_t chunks = 0;
    for (int i = 0; i < cnt; ++i) {
      const rk_adam_tensor& t = tensors[base + i];
      if (t.numel < 0 || (t.numel > 0 && (!t.param || !t.grad || !t.exp_avg || !t.exp_avg_sq)))
        return fail(RK_ERR_INVALID, "rk_adam_step: tensor %d invalid", base + i);
      if ((t.step != nullptr) != capturable)
        return fail(RK_ERR_INVALID, "rk_adam_step: device step counters must be given for all tensors or none");
      list.t[i] = t;
      list.chunk_start[i] = chunks;
      chunks += (t.numel + kAdamChunk - 1) / kAdamChunk;
    }
    list.chunk_start[cnt] = chunks;
    if (capturable) adam_step_inc_kernel<<<1, kAdamMaxTensors, 0, st>>>(list, cnt);
    if (chunks == 0) continue;
    if (capturable)
      adam_kernel<true><<<(unsigned)chunks, 256, 0, st>>>(list, cnt, omb1, (float)beta1, (float)beta2, omb2,
                                                          (float)eps, (float)weight_decay, (float)lr, 0.f, 0.f);
    else
      adam_kernel<false><<<(unsigned)chunks, 256, 0, st>>>(list, cnt, omb1, (float)beta1, (float)beta2, omb2,
                                                           (float)eps, (float)weight_decay, (float)lr, step_size,
                                                           bc2_sqrt);
  }
  return check_launch("rk_adam_step");
}
