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

__global__ __launch_bounds__(256) void bst_add_pos_kernel(const float* __restrict__ x, const float* __restrict__ pos,
                                                          int T, int64_t M, int d, float* __restrict__ xp) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * d) return;
  const int64_t m = i / d;
  const int k = (int)(i - m * d);
  xp[i] = x[i] + pos[(int64_t)(m % T) * d + k];
}

// Behaviour-sequence gather fused with the position add (bst.py:224 + 73-75): x[m] = table[idx[m]]
// (out-of-range -> zeros, flagged), xp[m] = x[m] + pos[m % T]; float4 per lane, d % 4 == 0.
__global__ __launch_bounds__(256) void bst_gather_pos_kernel(const float* __restrict__ table, int64_t rows,
                                                             int64_t ld_table, const int64_t* __restrict__ idx,
                                                             int64_t M, int T, int d, const float* __restrict__ pos,
                                                             float* __restrict__ x, float* __restrict__ xp,
                                                             uint32_t* flags) {
  const int q = d / 4;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= M * q) return;
  const int64_t m = e / q;
  const int k = 4 * (int)(e - m * q);
  const int64_t r = idx[m];
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (r >= 0 && r < rows)
    v = *reinterpret_cast<const f32x4*>(table + r * ld_table + k);
  else if (k == 0)
    flag_oob(flags);
  const f32x4 pv = *reinterpret_cast<const f32x4*>(pos + (int64_t)(m % T) * d + k);
  *reinterpret_cast<f32x4*>(x + m * d + k) = v;
  *reinterpret_cast<f32x4*>(xp + m * d + k) = v + pv;
}

// Attention train kernels on FP32 MFMA (v_mfma_f32_16x16x4_f32: lane l supplies A[l&15][k] and
// B[k][l&15] with hardware k = l>>4; accumulator register r of lane l is D[4*(l>>4) + r][l&15]).
// One 256-thread workgroup per (sample, head); T is padded to TP = 16*ceil(T/16) <= 64 positions and
// the head width to DP = 16*ceil(dh/16) <= 64 columns, zero-filled in LDS.  Wave w owns the 16-row
// strip w of the TP x TP score matrix.  Scores are formed transposed (S^T = K Q^T), so a lane's
// accumulators hold S[i = l&15][j = 16*jt + 4*(l>>4) + r]: the row-softmax reduces over registers
// and the lane pairs l^16, l^32, and the probabilities are already the A operand of P V (k = j) —
// no LDS round trip between the two products.
// LDS (dynamic): the [TP][DP + 4] operand tiles, and in the backward two [TP][TP + 4] tiles (P, dS).
__host__ __device__ constexpr int att_pad16(int v) { return (v + 15) & ~15; }
static size_t att_lds_bytes(int T, int dh, bool bwd) {
  const int TP = att_pad16(T), DP = att_pad16(dh);
  return sizeof(float) * (size_t)(bwd ? 4 * TP * (DP + 4) + 2 * TP * (TP + 4) : 3 * TP * (DP + 4));
}


__device__ __forceinline__ f32x4 mfma16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}


// Stage a [T, dh] head slice (columns col0..col0+dh of a row-major [M, ld] matrix) into a zero-padded
// [TP][DP] LDS tile of pitch ldt.
__device__ __forceinline__ void att_stage(float* __restrict__ dst, int ldt, const float* __restrict__ src, int64_t ld,
                                          int64_t row0, int col0, int T, int dh, int TP, int DP) {
  if (((dh | ld | col0) & 3) == 0) {  // float4 path (16-B aligned rows, dh a multiple of 4)
    const int q = DP / 4;
    for (int i = threadIdx.x; i < TP * q; i += blockDim.x) {
      const int t = i / q, k = 4 * (i - t * q);
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (t < T && k < dh) v = *reinterpret_cast<const f32x4*>(src + (row0 + t) * ld + col0 + k);
      *reinterpret_cast<f32x4*>(dst + t * ldt + k) = v;
    }
    return;
  }
  for (int i = threadIdx.x; i < TP * DP; i += blockDim.x) {
    const int t = i / DP, k = i - t * DP;
    dst[t * ldt + k] = (t < T && k < dh) ? src[(row0 + t) * ld + col0 + k] : 0.f;
  }
}

// Stage NT head slices at once (float4 path only: dh, ld and col0 multiples of 4): every tile's
// global loads are issued before the first LDS store, so the NT round trips overlap instead of
// running one after another.  TP * DP / 4 <= 1024 float4 per tile (4 per thread at 256 threads).
template <int NT>
__device__ __forceinline__ void att_stage_all(float* const (&dst)[NT], const float* const (&src)[NT],
                                              const int64_t (&ld)[NT], const int (&col0)[NT], int ldt, int64_t row0,
                                              int T, int dh, int TP, int DP) {
  const int q = DP / 4, n = TP * q;
  f32x4 v[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int r = i / q, k = 4 * (i - r * q);
      v[t][u] = (i < n && r < T && k < dh) ? *reinterpret_cast<const f32x4*>(src[t] + (row0 + r) * ld[t] + col0[t] + k)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int r = i / q, k = 4 * (i - r * q);
      if (i < n) *reinterpret_cast<f32x4*>(dst[t] + r * ldt + k) = v[t][u];
    }
}

// acc[jt] += rows(16*jt ..) of X  .  rows(16*w ..) of Y, contracted over DP columns (both [TP][ldt] LDS
// tiles): lane ends with D[j = 16*jt + 4*(l>>4) + r][i = l&15] = sum_c X[j][c] Y[i][c].
__device__ __forceinline__ void att_rowdot(f32x4 (&acc)[4], const float* __restrict__ X, const float* __restrict__ Y,
                                           int ldt, int w, int NS, int ND, int lane) {
  const int li = lane & 15, kq = 4 * (lane >> 4);
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) acc[jt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    if (c >= ND) break;
    const f32x4 b = *reinterpret_cast<const f32x4*>(Y + (16 * w + li) * ldt + 16 * c + kq);
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      if (jt >= NS) break;
      const f32x4 a = *reinterpret_cast<const f32x4*>(X + (16 * jt + li) * ldt + 16 * c + kq);
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[jt] = mfma16x4(a[e], b[e], acc[jt]);
    }
  }
}

// out[ct] = A (registers: lane holds A[i = l&15][k = 16*kt + 4*(l>>4) + e] in a[kt][e]) . B[k][16*ct + (l&15)]
// with B a [TP][ldb] LDS tile; lane ends with D[i = 4*(l>>4) + r][c = 16*ct + (l&15)].
__device__ __forceinline__ void att_regmm(f32x4 (&out)[4], const f32x4 (&a)[4], const float* __restrict__ B, int ldb,
                                         int NS, int ND, int lane) {
  const int li = lane & 15, kq = 4 * (lane >> 4);
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) out[ct] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    if (kt >= NS) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float* brow = B + (16 * kt + kq + e) * ldb + li;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        if (ct >= ND) break;
        out[ct] = mfma16x4(a[kt][e], brow[16 * ct], out[ct]);
      }
    }
  }
}

// out[ct] = sum_i At[i][16*w + (l&15)] . B[i][16*ct + (l&15)] over i < TP: the transposed-A product
// (dK = dS^T Q, dV = P^T dC) for the 16 output rows of strip w; At is [TP][lda], B is [TP][ldb] in LDS.
__device__ __forceinline__ void att_tmm(f32x4 (&out)[4], const float* __restrict__ At, int lda,
                                       const float* __restrict__ B, int ldb, int w, int NS, int ND, int lane) {
  const int li = lane & 15, kq = 4 * (lane >> 4);
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) out[ct] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kt = 0; kt < 4; ++kt) {
    if (kt >= NS) break;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = 16 * kt + kq + e;
      const float a = At[i * lda + 16 * w + li];
      const float* brow = B + i * ldb + li;
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        if (ct >= ND) break;
        out[ct] = mfma16x4(a, brow[16 * ct], out[ct]);
      }
    }
  }
}

// Store a strip result (lane holds D[16*w + 4*(l>>4) + r][16*ct + (l&15)]) into rows row0.. of a
// row-major matrix at column col0 (rows < T, columns < dh only).
__device__ __forceinline__ void att_store(const f32x4 (&v)[4], float* __restrict__ dst, int64_t ld, int64_t row0,
                                          int col0, int w, int T, int dh, int ND, int lane) {
  const int li = lane & 15, kq = 4 * (lane >> 4);
#pragma unroll
  for (int ct = 0; ct < 4; ++ct) {
    if (ct >= ND) break;
    const int c = 16 * ct + li;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * w + kq + r;
      if (i < T && c < dh) dst[(row0 + i) * ld + col0 + c] = v[ct][r];
    }
  }
}

// P = softmax(mask(Q K^T / sqrt(dh))) (saved, [B, h, T, T]) and ctx = P V.
__global__ __launch_bounds__(256) void bst_attn_train_fwd_kernel(const float* __restrict__ qkv, int64_t B, int T,
                                                                 int d, int heads,
                                                                 const int64_t* __restrict__ seq_len,
                                                                 float* __restrict__ P, float* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float att_sm[];
  const int64_t b = blockIdx.x / heads;
  const int h = (int)(blockIdx.x - b * heads);
  const int dh = d / heads;
  const int TP = (T + 15) & ~15, DP = (dh + 15) & ~15, ldt = DP + 4;
  const int NS = TP / 16, ND = DP / 16;
  float* const sQ = att_sm;
  float* const sK = sQ + TP * ldt;
  float* const sV = sK + TP * ldt;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t row0 = b * T, ld = 3 * (int64_t)d;
  if (((dh | d) & 3) == 0) {
    float* const dst[3] = {sQ, sK, sV};
    const float* const src[3] = {qkv, qkv, qkv};
    const int64_t lds[3] = {ld, ld, ld};
    const int c0[3] = {h * dh, d + h * dh, 2 * d + h * dh};
    att_stage_all<3>(dst, src, lds, c0, ldt, row0, T, dh, TP, DP);
  } else {
    att_stage(sQ, ldt, qkv, ld, row0, h * dh, T, dh, TP, DP);
    att_stage(sK, ldt, qkv, ld, row0, d + h * dh, T, dh, TP, DP);
    att_stage(sV, ldt, qkv, ld, row0, 2 * d + h * dh, T, dh, TP, DP);
  }
  __syncthreads();
  if (w >= NS) return;
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int64_t len = seq_len[b];
  const float sq = sqrtf((float)dh);  // scores / math.sqrt(q.size(-1)), bst.py:77
  f32x4 s[4];
  att_rowdot(s, sK, sQ, ldt, w, NS, ND, lane);  // s[jt][r] = S[i = 16w + li][j = 16jt + kq + r]
  float mx = -INFINITY;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jt + kq + r;
      const float v = (jt < NS && j < T) ? ((int64_t)j < len ? s[jt][r] / sq : -INFINITY) : -INFINITY;
      s[jt][r] = v;  // masked_fill(key_padding_mask, -inf), bst.py:80
      mx = fmaxf(mx, v);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
  mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
  float sum = 0.f;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jt + kq + r;
      const float e = (jt < NS && j < T) ? expf(s[jt][r] - mx) : 0.f;
      s[jt][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 16, kWave);
  sum += __shfl_xor(sum, 32, kWave);
  const int i = 16 * w + li;
  float* Pi = P + ((b * heads + h) * (int64_t)T + i) * T;
  const bool vec = (T & 3) == 0;  // rows of P are 16-B aligned: one float4 store per key tile
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    if (jt >= NS) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jt + kq + r;
      const float p = s[jt][r] / sum;
      s[jt][r] = j < T ? p : 0.f;
      if (!vec && i < T && j < T) Pi[j] = p;
    }
    if (vec && i < T && 16 * jt + kq < T) *reinterpret_cast<f32x4*>(Pi + 16 * jt + kq) = s[jt];
  }
  f32x4 c[4];
  att_regmm(c, s, sV, ldt, NS, ND, lane);
  att_store(c, ctx, d, row0, h * dh, w, T, dh, ND, lane);
}

// Backward of the above from dctx [M, d]: dqkv [M, 3d] (overwritten).
//   dP = dC V^T;  dS = P (dP - rowsum(P dP)) / sqrt(dh);  dQ = dS K;  dK = dS^T Q;  dV = P^T dC.
// Phase 1 (wave = query strip): dP (transposed form, as S above), P from HBM in the same register
// layout, dS, dQ = dS K with dS as the register A operand; P and dS go to LDS.  Phase 2 (wave = key
// strip): dK and dV from the LDS copies (transposed-A products).
__global__ __launch_bounds__(256) void bst_attn_train_bwd_kernel(const float* __restrict__ qkv,
                                                                 const float* __restrict__ P,
                                                                 const float* __restrict__ dctx, int64_t B, int T,
                                                                 int d, int heads, float* __restrict__ dqkv) {
  extern __shared__ __attribute__((aligned(16))) float att_sm[];
  const int64_t b = blockIdx.x / heads;
  const int h = (int)(blockIdx.x - b * heads);
  const int dh = d / heads;
  const int TP = (T + 15) & ~15, DP = (dh + 15) & ~15, ldt = DP + 4, ldp = TP + 4;
  const int NS = TP / 16, ND = DP / 16;
  float* const sQ = att_sm;
  float* const sK = sQ + TP * ldt;
  float* const sV = sK + TP * ldt;
  float* const sC = sV + TP * ldt;
  float* const sP = sC + TP * ldt;
  float* const sS = sP + TP * ldp;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int64_t row0 = b * T, ld = 3 * (int64_t)d;
  // this wave's P strip (register layout of the dP tile below) is loaded first, so its round trip
  // overlaps the operand staging
  const int i = 16 * w + li;
  const float* Pi = P + ((b * heads + h) * (int64_t)T + min(i, T - 1)) * T;
  f32x4 p[4];
  const bool pvec = (T & 3) == 0;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    p[jt] = (f32x4){0.f, 0.f, 0.f, 0.f};
    if (jt >= NS || i >= T || w >= NS) continue;
    if (pvec) {
      if (16 * jt + kq < T) p[jt] = *reinterpret_cast<const f32x4*>(Pi + 16 * jt + kq);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (16 * jt + kq + r < T) p[jt][r] = Pi[16 * jt + kq + r];
    }
  }
  if (((dh | d) & 3) == 0) {
    float* const dst[4] = {sQ, sK, sV, sC};
    const float* const src[4] = {qkv, qkv, qkv, dctx};
    const int64_t lds[4] = {ld, ld, ld, (int64_t)d};
    const int c0[4] = {h * dh, d + h * dh, 2 * d + h * dh, h * dh};
    att_stage_all<4>(dst, src, lds, c0, ldt, row0, T, dh, TP, DP);
  } else {
    att_stage(sQ, ldt, qkv, ld, row0, h * dh, T, dh, TP, DP);
    att_stage(sK, ldt, qkv, ld, row0, d + h * dh, T, dh, TP, DP);
    att_stage(sV, ldt, qkv, ld, row0, 2 * d + h * dh, T, dh, TP, DP);
    att_stage(sC, ldt, dctx, d, row0, h * dh, T, dh, TP, DP);
  }
  __syncthreads();
  const float sq = sqrtf((float)dh);
  if (w < NS) {
    f32x4 g[4];
    att_rowdot(g, sV, sC, ldt, w, NS, ND, lane);  // g[jt][r] = dP[i = 16w + li][j = 16jt + kq + r]
    float D = 0.f;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) D += p[jt][r] * g[jt][r];
    D += __shfl_xor(D, 16, kWave);
    D += __shfl_xor(D, 32, kWave);
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      if (jt >= NS) break;
#pragma unroll
      for (int r = 0; r < 4; ++r) g[jt][r] = p[jt][r] * (g[jt][r] - D) / sq;
      *reinterpret_cast<f32x4*>(sP + i * ldp + 16 * jt + kq) = p[jt];
      *reinterpret_cast<f32x4*>(sS + i * ldp + 16 * jt + kq) = g[jt];
    }
    f32x4 q[4];
    att_regmm(q, g, sK, ldt, NS, ND, lane);  // dQ[i] = sum_j dS[i, j] K[j]
    att_store(q, dqkv, ld, row0, h * dh, w, T, dh, ND, lane);
  }
  __syncthreads();
  if (w < NS) {
    f32x4 o[4];
    att_tmm(o, sS, ldp, sQ, ldt, w, NS, ND, lane);  // dK[j] = sum_i dS[i, j] Q[i]
    att_store(o, dqkv, ld, row0, d + h * dh, w, T, dh, ND, lane);
    att_tmm(o, sP, ldp, sC, ldt, w, NS, ND, lane);  // dV[j] = sum_i P[i, j] dC[i]
    att_store(o, dqkv, ld, row0, 2 * d + h * dh, w, T, dh, ND, lane);
  }
}

// ---- Persistent forms of the two attention train kernels (T % 4 == 0, dh % 4 == 0: float4 rows).
// A workgroup walks (sample, head) items grid-stride; while it computes item n, the global loads of
// item n + grid (its Q/K/V(/dC) slices and, in the backward, each wave's P strip) are already in
// flight in registers, so the staging round trip no longer sits between one item's compute and the
// next (the one-item-per-workgroup kernels above wait out a full round trip per item: latency-bound,
// SQ_WAIT_ANY 51% of wave time in the backward).  US = float4 slots per thread and tile.
template <int NT, int US>
__device__ __forceinline__ void att_load_regs(f32x4 (&v)[NT][US], const float* const (&src)[NT],
                                              const int64_t (&ld)[NT], const int (&col0)[NT], int64_t row0, int T,
                                              int dh, int TP, int DP) {
  const int q = DP / 4, n = TP * q;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int u = 0; u < US; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int r = i / q, k = 4 * (i - r * q);
      v[t][u] = (i < n && r < T && k < dh) ? *reinterpret_cast<const f32x4*>(src[t] + (row0 + r) * ld[t] + col0[t] + k)
                                           : f32x4{0.f, 0.f, 0.f, 0.f};
    }
}

template <int NT, int US>
__device__ __forceinline__ void att_store_regs(float* const (&dst)[NT], const f32x4 (&v)[NT][US], int ldt, int TP,
                                               int DP) {
  const int q = DP / 4, n = TP * q;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int u = 0; u < US; ++u) {
      const int i = threadIdx.x + 256 * u;
      const int r = i / q, k = 4 * (i - r * q);
      if (i < n) *reinterpret_cast<f32x4*>(dst[t] + r * ldt + k) = v[t][u];
    }
}

// Row softmax of the strip of wave w (bst.py:77-84): s[jt][r] = P[i = 16w + li][j = 16jt + kq + r],
// from the staged Q and K tiles; the same code for the forward (which may save P) and for the
// backward that recomputes P instead of reading it (bit-identical values).
__device__ __forceinline__ void att_softmax_strip(f32x4 (&s)[4], const float* __restrict__ sK,
                                                  const float* __restrict__ sQ, int ldt, int w, int NS, int ND,
                                                  int lane, int T, int64_t len, float sq) {
  const int kq = 4 * (lane >> 4);
  att_rowdot(s, sK, sQ, ldt, w, NS, ND, lane);  // s[jt][r] = S[i = 16w + li][j = 16jt + kq + r]
  float mx = -INFINITY;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jt + kq + r;
      const float x = (jt < NS && j < T) ? ((int64_t)j < len ? s[jt][r] / sq : -INFINITY) : -INFINITY;
      s[jt][r] = x;  // masked_fill(key_padding_mask, -inf), bst.py:80
      mx = fmaxf(mx, x);
    }
  mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
  mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
  float sum = 0.f;
#pragma unroll
  for (int jt = 0; jt < 4; ++jt)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jt + kq + r;
      const float e = (jt < NS && j < T) ? expf(s[jt][r] - mx) : 0.f;
      s[jt][r] = e;
      sum += e;
    }
  sum += __shfl_xor(sum, 16, kWave);
  sum += __shfl_xor(sum, 32, kWave);
#pragma unroll
  for (int jt = 0; jt < 4; ++jt) {
    if (jt >= NS) break;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = 16 * jt + kq + r;
      s[jt][r] = j < T ? s[jt][r] / sum : 0.f;
    }
  }
}

template <int US>
__global__ __launch_bounds__(256, 2) void bst_attn_train_fwd_pkernel(const float* __restrict__ qkv, int64_t B, int T,
                                                                  int d, int heads,
                                                                  const int64_t* __restrict__ seq_len,
                                                                  float* __restrict__ P, float* __restrict__ ctx) {
  extern __shared__ __attribute__((aligned(16))) float att_sm[];
  const int dh = d / heads;
  const int TP = (T + 15) & ~15, DP = (dh + 15) & ~15, ldt = DP + 4;
  const int NS = TP / 16, ND = DP / 16;
  float* const sQ = att_sm;
  float* const sK = sQ + TP * ldt;
  float* const sV = sK + TP * ldt;
  float* const dst[3] = {sQ, sK, sV};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int64_t items = B * heads, ld = 3 * (int64_t)d;
  const float sq = sqrtf((float)dh);  // scores / math.sqrt(q.size(-1)), bst.py:77
  const int64_t lds3[3] = {ld, ld, ld};
  const float* const src3[3] = {qkv, qkv, qkv};
  f32x4 v[3][US];
  int64_t it = blockIdx.x;
  if (it < items) {
    const int64_t b = it / heads;
    const int h = (int)(it - b * heads);
    const int c0[3] = {h * dh, d + h * dh, 2 * d + h * dh};
    att_load_regs<3, US>(v, src3, lds3, c0, b * T, T, dh, TP, DP);
  }
  for (; it < items; it += gridDim.x) {
    const int64_t b = it / heads;
    const int h = (int)(it - b * heads);
    const int64_t row0 = b * T;
    att_store_regs<3, US>(dst, v, ldt, TP, DP);
    __syncthreads();
    const int64_t nx = it + gridDim.x;
    if (nx < items) {
      const int64_t nb = nx / heads;
      const int nh = (int)(nx - nb * heads);
      const int c0[3] = {nh * dh, d + nh * dh, 2 * d + nh * dh};
      att_load_regs<3, US>(v, src3, lds3, c0, nb * T, T, dh, TP, DP);
    }
    if (w < NS) {
      f32x4 s[4];
      att_softmax_strip(s, sK, sQ, ldt, w, NS, ND, lane, T, seq_len[b], sq);
      const int i = 16 * w + li;
      if (P && i < T) {  // P == NULL: the backward recomputes it
        float* Pi = P + ((b * heads + h) * (int64_t)T + i) * T;
#pragma unroll
        for (int jt = 0; jt < 4; ++jt)
          if (jt < NS && 16 * jt + kq < T) *reinterpret_cast<f32x4*>(Pi + 16 * jt + kq) = s[jt];
      }
      f32x4 c[4];
      att_regmm(c, s, sV, ldt, NS, ND, lane);
      att_store(c, ctx, d, row0, h * dh, w, T, dh, ND, lane);
    }
    __syncthreads();  // the next item's staging overwrites the tiles
  }
}

template <int US>
__global__ __launch_bounds__(256, 2) void bst_attn_train_bwd_pkernel(const float* __restrict__ qkv,
                                                                  const float* __restrict__ P,
                                                                  const float* __restrict__ dctx, int64_t B, int T,
                                                                  int d, int heads, float* __restrict__ dqkv) {
  extern __shared__ __attribute__((aligned(16))) float att_sm[];
  const int dh = d / heads;
  const int TP = (T + 15) & ~15, DP = (dh + 15) & ~15, ldt = DP + 4, ldp = TP + 4;
  const int NS = TP / 16, ND = DP / 16;
  float* const sQ = att_sm;
  float* const sK = sQ + TP * ldt;
  float* const sV = sK + TP * ldt;
  float* const sC = sV + TP * ldt;
  float* const sP = sC + TP * ldt;
  float* const sS = sP + TP * ldp;
  float* const dst[4] = {sQ, sK, sV, sC};
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int64_t items = B * heads, ld = 3 * (int64_t)d;
  const float sq = sqrtf((float)dh);
  const int64_t lds4[4] = {ld, ld, ld, (int64_t)d};
  const float* const src4[4] = {qkv, qkv, qkv, dctx};
  const int i = 16 * w + li;
  const bool prow = w < NS && i < T;
  f32x4 v[4][US], pc[4];
  // item `x`'s operand slices, and this wave's P strip, into registers
  auto load_tiles = [&](int64_t x) {
    const int64_t b = x / heads;
    const int h = (int)(x - b * heads);
    const int c0[4] = {h * dh, d + h * dh, 2 * d + h * dh, h * dh};
    att_load_regs<4, US>(v, src4, lds4, c0, b * T, T, dh, TP, DP);
  };
  auto load_p = [&](int64_t x) {
    const float* Pi = P + (x * (int64_t)T + (prow ? i : 0)) * T;
#pragma unroll
    for (int jt = 0; jt < 4; ++jt)
      pc[jt] = (prow && jt < NS && 16 * jt + kq < T) ? *reinterpret_cast<const f32x4*>(Pi + 16 * jt + kq)
                                                      : f32x4{0.f, 0.f, 0.f, 0.f};
  };
  int64_t it = blockIdx.x;
  if (it < items) {
    load_tiles(it);
    load_p(it);
  }
  for (; it < items; it += gridDim.x) {
    const int64_t b = it / heads;
    const int h = (int)(it - b * heads);
    const int64_t row0 = b * T;
    const bool more = it + gridDim.x < items;
    att_store_regs<4, US>(dst, v, ldt, TP, DP);
    __syncthreads();
    if (more) load_tiles(it + gridDim.x);
    if (w < NS) {
      f32x4 g[4];
      att_rowdot(g, sV, sC, ldt, w, NS, ND, lane);  // g[jt][r] = dP[i = 16w + li][j = 16jt + kq + r]
      float D = 0.f;
#pragma unroll
      for (int jt = 0; jt < 4; ++jt)
#pragma unroll
        for (int r = 0; r < 4; ++r) D += pc[jt][r] * g[jt][r];
      D += __shfl_xor(D, 16, kWave);
      D += __shfl_xor(D, 32, kWave);
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        if (jt >= NS) break;
#pragma unroll
        for (int r = 0; r < 4; ++r) g[jt][r] = pc[jt][r] * (g[jt][r] - D) / sq;
        *reinterpret_cast<f32x4*>(sP + i * ldp + 16 * jt + kq) = pc[jt];
        *reinterpret_cast<f32x4*>(sS + i * ldp + 16 * jt + kq) = g[jt];
      }
      if (more) load_p(it + gridDim.x);  // pc is in LDS now: the next strip's loads overlap the rest
      f32x4 q[4];
      att_regmm(q, g, sK, ldt, NS, ND, lane);  // dQ[i] = sum_j dS[i, j] K[j]
      att_store(q, dqkv, ld, row0, h * dh, w, T, dh, ND, lane);
    }
    __syncthreads();
    if (w < NS) {
      f32x4 o[4];
      att_tmm(o, sS, ldp, sQ, ldt, w, NS, ND, lane);  // dK[j] = sum_i dS[i, j] Q[i]
      att_store(o, dqkv, ld, row0, d + h * dh, w, T, dh, ND, lane);
      att_tmm(o, sP, ldp, sC, ldt, w, NS, ND, lane);  // dV[j] = sum_i P[i, j] dC[i]
      att_store(o, dqkv, ld, row0, 2 * d + h * dh, w, T, dh, ND, lane);
    }
    __syncthreads();  // the next item's staging overwrites the tiles
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

// Row-group layout of the float4 LayerNorm kernels (d % 4 == 0, d <= 4L): a row is held by L lanes
// of 4 consecutive columns (lane li: columns 4li..4li+3), so a wave holds 64 / L rows at once, and
// each wave keeps NR such row groups in flight (all loads issued before the first reduction).
template <int L>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
  return v;
}

__device__ __forceinline__ f32x4 ld4(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
__device__ __forceinline__ void st4(float* p, f32x4 v) { *reinterpret_cast<f32x4*>(p) = v; }

constexpr int kLnNR = 4;  // row groups in flight per wave

template <int L>
__global__ __launch_bounds__(256) void bst_res_dropout_ln_fwd4_kernel(
    const float* __restrict__ base, const float* __restrict__ o, int64_t M, int d, uint64_t seed,
    const int64_t* __restrict__ stream_slot, uint32_t threshold, float scale, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float* __restrict__ r_out, float* __restrict__ y,
    float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int RPW = 64 / L;
  const int lane = threadIdx.x & 63, sub = lane / L, li = lane % L;
  const int k = 4 * li;
  const bool on = k < d;
  const uint64_t stream = threshold ? (uint64_t)*stream_slot : 0;
  const f32x4 g4 = on ? ld4(gamma + k) : f32x4{0.f, 0.f, 0.f, 0.f};
  const f32x4 b4 = on ? ld4(beta + k) : f32x4{0.f, 0.f, 0.f, 0.f};
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t step = nw * RPW;  // rows between a wave's consecutive row groups
  const float inv_d = 1.0f / (float)d;
  for (int64_t m0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + sub; m0 - sub < M; m0 += step * kLnNR) {
    f32x4 v[kLnNR];
#pragma unroll
    for (int i = 0; i < kLnNR; ++i) {
      const int64_t m = m0 + i * step;
      v[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (on && m < M) {
        const f32x4 ov = ld4(o + m * d + k), bv = ld4(base + m * d + k);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float t = ov[c];
          if (threshold) t = dropout_keep(seed, stream, (uint64_t)m * d + k + c, threshold) ? t * scale : 0.f;
          v[i][c] = bv[c] + t;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kLnNR; ++i) {
      const int64_t m = m0 + i * step;
      const float mean = group_sum<L>(v[i][0] + v[i][1] + v[i][2] + v[i][3]) * inv_d;
      float q = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) q += on ? (v[i][c] - mean) * (v[i][c] - mean) : 0.f;
      const float rstd = 1.0f / sqrtf(group_sum<L>(q) * inv_d + eps);
      if (m < M) {
        if (on) {
          f32x4 out;
#pragma unroll
          for (int c = 0; c < 4; ++c) out[c] = (v[i][c] - mean) * rstd * g4[c] + b4[c];
          st4(r_out + m * d + k, v[i]);
          st4(y + m * d + k, out);
        }
        if (li == 0) {
          mean_out[m] = mean;
          rstd_out[m] = rstd;
        }
      }
    }
  }
}

// LayerNorm backward from dy: dr = rstd (g - mean(g) - xhat mean(g xhat)), g = dy gamma; d_o =
// dropout-masked dr (the residual branch's gradient).  Waves walk rows grid-stride; each lane keeps
// its columns' dgamma = sum dy xhat and dbeta = sum dy in registers, the workgroup combines them
// in LDS and writes one partial row per workgroup to ws [kLnBlocks][2d], summed in block order by
// bst_ln_param_kernel (deterministic; per-row atomics on the same 2d addresses serialised).
constexpr int kLnBlocks = 2048;  // 8 per CU: enough row groups in flight for the HBM stream
constexpr int kLnRows = 4;  // rows in flight per wave

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
  // kLnRows rows per step, all of their loads issued before the first reduction: one row at a
  // time left each wave (2 per SIMD at 512 workgroups) waiting a full memory round trip per row
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t m0 = (int64_t)blockIdx.x * 4 + wv; m0 < M; m0 += stride * kLnRows) {
    float dyv[kLnRows][4], rv[kLnRows][4], mean[kLnRows], rstd[kLnRows];
#pragma unroll
    for (int i = 0; i < kLnRows; ++i) {
      const int64_t m = m0 + i * stride;
      const int64_t mm = m < M ? m : M - 1;
      mean[i] = mean_in[mm];
      rstd[i] = rstd_in[mm];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = lane + 64 * c;
        dyv[i][c] = k < d ? dy[mm * d + k] : 0.f;
        rv[i][c] = k < d ? r[mm * d + k] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < kLnRows; ++i) {
      const int64_t m = m0 + i * stride;
      if (m >= M) break;
      float g[4], xh[4];
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = lane + 64 * c;
        g[c] = xh[c] = 0.f;
        if (k < d) {
          xh[c] = (rv[i][c] - mean[i]) * rstd[i];
          g[c] = dyv[i][c] * gm[c];
          s1 += g[c];
          s2 += g[c] * xh[c];
          pg[c] = fmaf(dyv[i][c], xh[c], pg[c]);
          pb[c] += dyv[i][c];
        }
      }
      const float k1 = wave_sum(s1) / (float)d, k2 = wave_sum(s2) / (float)d;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = lane + 64 * c;
        if (k < d) {
          const float v = rstd[i] * (g[c] - k1 - xh[c] * k2);
          dr[m * d + k] = v;
          if (d_o)
            d_o[m * d + k] = threshold
                                 ? (dropout_keep(seed, stream, (uint64_t)m * d + k, threshold) ? v * scale : 0.f)
                                 : v;
        }
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

// float4 row-group form of bst_ln_bwd_kernel (same math, same workspace layout: one [2d] partial
// per workgroup).  When drow is non-NULL the incoming gradient is the pooling backward's broadcast
// dy[m] = drow[m / T, col:] (/ seq_len for mean pooling, bst.py:238-241) instead of dy.
template <int L>
__global__ __launch_bounds__(256) void bst_ln_bwd4_kernel(const float* __restrict__ dy,
                                                          const float* __restrict__ drow, int64_t ld_row, int col,
                                                          int T, const int64_t* __restrict__ seq_len, int mean_pool,
                                                          const float* __restrict__ r,
                                                          const float* __restrict__ mean_in,
                                                          const float* __restrict__ rstd_in,
                                                          const float* __restrict__ gamma, int64_t M, int d,
                                                          uint64_t seed, const int64_t* __restrict__ stream_slot,
                                                          uint32_t threshold, float scale, float* __restrict__ dr,
                                                          float* __restrict__ d_o, float* __restrict__ ws) {
  constexpr int RPW = 64 / L;
  __shared__ f32x4 red[4][2][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, sub = lane / L, li = lane % L;
  const int k = 4 * li;
  const bool on = k < d;
  const uint64_t stream = threshold ? (uint64_t)*stream_slot : 0;
  const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
  const f32x4 gm = on ? ld4(gamma + k) : zero;
  f32x4 pg = zero, pb = zero;
  const int64_t step = (int64_t)gridDim.x * 4 * RPW;
  const float inv_d = 1.0f / (float)d;
  for (int64_t m0 = ((int64_t)blockIdx.x * 4 + wv) * RPW + sub; m0 - sub < M; m0 += step * kLnNR) {
    f32x4 dyv[kLnNR], rv[kLnNR];
    float mean[kLnNR], rstd[kLnNR];
#pragma unroll
    for (int i = 0; i < kLnNR; ++i) {
      const int64_t m = m0 + i * step;
      const int64_t mm = m < M ? m : M - 1;
      mean[i] = mean_in[mm];
      rstd[i] = rstd_in[mm];
      dyv[i] = rv[i] = zero;
      if (on) {
        if (drow) {
          const int64_t b = mm / T;
          const float* src = drow + b * ld_row + col + k;  // the DNN row: any alignment (col = 50 in BST)
          dyv[i] = f32x4{src[0], src[1], src[2], src[3]};
          if (mean_pool) {
            const float inv = 1.0f / (float)seq_len[b];
#pragma unroll
            for (int c = 0; c < 4; ++c) dyv[i][c] = dyv[i][c] * inv;
          }
        } else {
          dyv[i] = ld4(dy + mm * d + k);
        }
        rv[i] = ld4(r + mm * d + k);
      }
    }
#pragma unroll
    for (int i = 0; i < kLnNR; ++i) {
      const int64_t m = m0 + i * step;
      const bool live = m < M;
      f32x4 g, xh;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        xh[c] = (rv[i][c] - mean[i]) * rstd[i];
        g[c] = dyv[i][c] * gm[c];
        s1 += g[c];
        s2 += g[c] * xh[c];
        if (live) {
          pg[c] = fmaf(dyv[i][c], xh[c], pg[c]);
          pb[c] += dyv[i][c];
        }
      }
      const float k1 = group_sum<L>(s1) * inv_d, k2 = group_sum<L>(s2) * inv_d;
      if (live && on) {
        f32x4 v, vo;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          v[c] = rstd[i] * (g[c] - k1 - xh[c] * k2);
          vo[c] = threshold ? (dropout_keep(seed, stream, (uint64_t)m * d + k + c, threshold) ? v[c] * scale : 0.f)
                            : v[c];
        }
        st4(dr + m * d + k, v);
        if (d_o) st4(d_o + m * d + k, vo);
      }
    }
  }
  // fold the wave's row groups (lanes li, li + L, ... hold the same columns), then the 4 waves
#pragma unroll
  for (int off = L; off < 64; off <<= 1)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      pg[c] += __shfl_xor(pg[c], off);
      pb[c] += __shfl_xor(pb[c], off);
    }
  if (sub == 0) {
    red[wv][0][li] = pg;
    red[wv][1][li] = pb;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * (d / 4); t += blockDim.x) {
    const int which = t / (d / 4), q = t % (d / 4);
    const f32x4 s = red[0][which][q] + red[1][which][q] + red[2][which][q] + red[3][which][q];
    st4(ws + (int64_t)blockIdx.x * 2 * d + which * d + 4 * q, s);
  }
}

// First pass over the per-workgroup partials: workgroup (x, y) sums partial rows y*C .. y*C + C - 1
// of columns 64x .. 64x + 63 (16 waves, every 16th row each, LDS combine in a fixed order) into
// out[y][2d]; bst_ln_param_kernel then folds the gridDim.y rows.
constexpr int kLnChunk = 64;
__global__ __launch_bounds__(1024) void bst_ln_partial_kernel(const float* __restrict__ ws, int nblocks, int d,
                                                              float* __restrict__ out) {
  __shared__ float red[16][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int k = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * kLnChunk, r1 = min(nblocks, r0 + kLnChunk);
  float s = 0.f;
  if (k < 2 * d)
    for (int r = r0 + wv; r < r1; r += 16) s += ws[(int64_t)r * 2 * d + k];
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && k < 2 * d) {
    float t = 0.f;
    for (int w = 0; w < 16; ++w) t += red[w][lane];
    out[(int64_t)blockIdx.y * 2 * d + k] = t;
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

// float4 form (n % 4 == 0, 16-B aligned): four elements per thread, same per-element hash index.
template <bool BWD>
__global__ __launch_bounds__(256) void bst_leaky_dropout4_kernel(const float* __restrict__ in,
                                                                 const float* __restrict__ f, int64_t n, float slope,
                                                                 uint64_t seed, const int64_t* __restrict__ stream_slot,
                                                                 uint32_t threshold, float scale,
                                                                 float* __restrict__ out) {
  const int64_t i4 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (4 * i4 >= n) return;
  const uint64_t stream = threshold ? (uint64_t)*stream_slot : 0;
  const float s = threshold ? scale : 1.f;
  const f32x4 fv = *reinterpret_cast<const f32x4*>(f + 4 * i4);
  f32x4 iv = {0.f, 0.f, 0.f, 0.f};
  if (BWD) iv = *reinterpret_cast<const f32x4*>(in + 4 * i4);
  f32x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const bool keep = threshold ? dropout_keep(seed, stream, (uint64_t)(4 * i4 + e), threshold) : true;
    if (BWD)
      o[e] = keep ? iv[e] * s * (fv[e] > 0.f ? 1.f : slope) : 0.f;
    else
      o[e] = keep ? (fv[e] > 0.f ? fv[e] : fv[e] * slope) * s : 0.f;
  }
  *reinterpret_cast<f32x4*>(out + 4 * i4) = o;
}

// Pooling, float4 form (d % 4 == 0): workgroup per sample, thread = (4 columns, row group of 256 /
// (d / 4)); row-group partial sums folded in LDS in a fixed order.
__global__ __launch_bounds__(256) void bst_pool_fwd4_kernel(const float* __restrict__ out, int T, int d,
                                                            const int64_t* __restrict__ seq_len, int mean,
                                                            float* __restrict__ row, int64_t ld_row, int col) {
  __shared__ f32x4 red[256];
  const int64_t b = blockIdx.x;
  const int q = d / 4, G = 256 / q;
  const int c = threadIdx.x % q, g = threadIdx.x / q;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (g < G)
    for (int t = g; t < T; t += G) acc += *reinterpret_cast<const f32x4*>(out + (b * T + t) * d + 4 * c);
  red[threadIdx.x] = acc;
  __syncthreads();
  if (threadIdx.x < q) {
    f32x4 sum = red[threadIdx.x];
    for (int k = 1; k < G; ++k) sum += red[k * q + threadIdx.x];
    float* dst = row + b * ld_row + col + 4 * threadIdx.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) dst[e] = mean ? sum[e] / (float)seq_len[b] : sum[e];
  }
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

// float4 slots per thread and operand tile of the persistent attention kernels (0: dh not a
// multiple of 4 -> the one-item kernels).
static int att_slots(int T, int dh) {
  if (dh % 4) return 0;
  const int n = att_pad16(T) * att_pad16(dh) / 4;
  return n <= 256 ? 1 : n <= 512 ? 2 : 4;
}

// Persistent grid: as many workgroups as are resident at once (the runtime's occupancy for this
// kernel, LDS and registers both), or one per item when there are fewer items.
static unsigned att_grid(const void* kernel, int64_t items, size_t lds) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, lds) != hipSuccess || per_cu <= 0)
    per_cu = std::max<int>(1, (int)((160 * 1024) / std::max<size_t>(lds, 1)));
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(items, (int64_t)per_cu * num_cus()));
}

// Dynamic LDS above the 64 KiB default: up to 104 KiB (T = 64, dh = 64 backward).
static void att_set_attrs() {
  for (const void* f : {(const void*)bst_attn_train_fwd_pkernel<1>, (const void*)bst_attn_train_fwd_pkernel<2>,
                        (const void*)bst_attn_train_fwd_pkernel<4>, (const void*)bst_attn_train_bwd_pkernel<1>,
                        (const void*)bst_attn_train_bwd_pkernel<2>, (const void*)bst_attn_train_bwd_pkernel<4>,
                        (const void*)bst_attn_train_fwd_kernel,
                        (const void*)bst_attn_train_bwd_kernel})
    raise_lds_limit(f, 160 * 1024);
}

// Lanes per row of the float4 LayerNorm kernels (0: use the scalar kernels): d % 4 == 0 and every
// row pointer 16-B aligned.
static int ln_lanes(int d, std::initializer_list<const float*> ptrs) {
  if (d % 4 || d > 256) return 0;
  for (const float* p : ptrs)
    if (p && (reinterpret_cast<uintptr_t>(p) & 15)) return 0;
  int L = 8;
  while (4 * L < d) L *= 2;
  return L;
}

static int ln_backward(const float* dy, const float* drow, int64_t ld_row, int col, int T, const int64_t* seq_len,
                       int mean_pool, const float* r, const float* mean, const float* rstd, const float* gamma,
                       int64_t rows, int d, double dropout_p, uint64_t seed, const int64_t* stream_slot, float* dr,
                       float* d_o, float* dgamma, float* dbeta, float* workspace, hipStream_t st, const char* what) {
  const uint32_t thr = dropout_threshold(dropout_p);
  const float scale = (float)(1.0 / (1.0 - dropout_p));
  const int L = ln_lanes(d, {dy, r, gamma, dr, d_o, workspace});
  int blocks;
  if (L) {
    const int64_t groups = (rows + 64 / L - 1) / (64 / L);
    blocks = (int)std::max<int64_t>(1, std::min<int64_t>(kLnBlocks, (groups + 3) / 4));
#define RK_LN_BWD(L_)                                                                                             \
  case L_:                                                                                                        \
    bst_ln_bwd4_kernel<L_><<<blocks, 256, 0, st>>>(dy, drow, ld_row, col, T, seq_len, mean_pool, r, mean, rstd,   \
                                                   gamma, rows, d, seed, stream_slot, thr, scale, dr, d_o,        \
                                                   workspace);                                                    \
    break;
    switch (L) { RK_LN_BWD(8) RK_LN_BWD(16) RK_LN_BWD(32) RK_LN_BWD(64) }
#undef RK_LN_BWD
  } else {
    // the scalar kernel reads dy only: the pooled-row form (drow) exists in the float4 kernels
    if (!dy) return fail(RK_ERR_UNSUPPORTED, "%s: the pooled-row backward needs the float4 path", what);
    blocks = (int)std::max<int64_t>(1, std::min<int64_t>(kLnBlocks, (rows + 3) / 4));
    bst_ln_bwd_kernel<<<blocks, 256, 0, st>>>(dy, r, mean, rstd, gamma, rows, d, seed, stream_slot, thr, scale, dr,
                                              d_o, workspace);
  }
  // two deterministic passes: chunks of kLnChunk partial rows, then the chunk sums
  const int chunks = (blocks + kLnChunk - 1) / kLnChunk;
  float* ws2 = workspace + (int64_t)kLnBlocks * 2 * d;
  bst_ln_partial_kernel<<<dim3(grid_of(2 * d, 64), chunks), 1024, 0, st>>>(workspace, blocks, d, ws2);
  bst_ln_param_kernel<<<grid_of(2 * d, 64), 1024, 0, st>>>(ws2, chunks, d, dgamma, dbeta);
  return check_launch(what);
}

}  // namespace rk

using namespace rk;

RK_API int rk_bst_add_pos(const float* x, const float* pos, int32_t T, int64_t rows, int32_t d, float* xp,
                          void* stream) {
  if (!x || !pos || !xp || T <= 0 || rows < 0 || d <= 0) return fail(RK_ERR_INVALID, "rk_bst_add_pos: bad arguments");
  if (rows == 0) return RK_OK;
  bst_add_pos_kernel<<<grid_of(rows * d), 256, 0, (hipStream_t)stream>>>(x, pos, T, rows, d, xp);
  return check_launch("rk_bst_add_pos");
}

RK_API int rk_bst_gather_pos(const float* table, int64_t rows, int64_t ld_table, const int64_t* idx, int64_t n,
                             int32_t T, int32_t d, const float* pos, float* x, float* xp, void* stream) {
  if (!table || !idx || !pos || !x || !xp || rows <= 0 || n < 0 || T <= 0 || d <= 0 || ld_table < d)
    return fail(RK_ERR_INVALID, "rk_bst_gather_pos: bad arguments");
  if (d % 4 || ld_table % 4 || ((reinterpret_cast<uintptr_t>(table) | reinterpret_cast<uintptr_t>(pos) |
                                 reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(xp)) & 15))
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_gather_pos: needs d %% 4 == 0 and 16-B aligned rows");
  if (n == 0) return RK_OK;
  bst_gather_pos_kernel<<<grid_of(n * (d / 4)), 256, 0, (hipStream_t)stream>>>(table, rows, ld_table, idx, n, T, d,
                                                                              pos, x, xp, device_flags());
  return check_launch("rk_bst_gather_pos");
}

RK_API int rk_bst_attn_train_forward(const float* qkv, int64_t batch, int32_t T, int32_t d, int32_t heads,
                                     const int64_t* seq_len, float* probs, float* ctx, void* stream) {
  if (!qkv || !seq_len || !ctx || batch < 0 || T <= 0 || T > kBstTMax || heads <= 0 || d % heads ||
      d / heads > kBstDhMax)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_attn_train_forward: T <= %d, d %% heads == 0, d/heads <= %d", kBstTMax,
                kBstDhMax);
  if (batch == 0) return RK_OK;
  att_set_attrs();
  const int dh = d / heads;
  const int US = att_slots(T, dh);
  if (!probs && !(US && T % 4 == 0 && d % 4 == 0))
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_attn_train_forward: probs may be NULL only for T %% 4 == 0, dh %% 4 == 0");
  if (US && T % 4 == 0 && d % 4 == 0) {
    const size_t lds = att_lds_bytes(T, dh, false);
#define RK_ATT_FWD(U_)                                                                                          \
  case U_:                                                                                                      \
    bst_attn_train_fwd_pkernel<U_><<<att_grid((const void*)bst_attn_train_fwd_pkernel<U_>, batch * heads, lds), \
                                     256, lds, (hipStream_t)stream>>>(qkv, batch, T, d, heads, seq_len,   \
                                                                            probs, ctx);                        \
    break;
    switch (US) { RK_ATT_FWD(1) RK_ATT_FWD(2) RK_ATT_FWD(4) }
#undef RK_ATT_FWD
    return check_launch("rk_bst_attn_train_forward");
  }
  bst_attn_train_fwd_kernel<<<(unsigned)(batch * heads), 256, att_lds_bytes(T, d / heads, false),
                              (hipStream_t)stream>>>(qkv, batch, T, d, heads,
                                                                                        seq_len, probs, ctx);
  return check_launch("rk_bst_attn_train_forward");
}

RK_API int rk_bst_attn_train_backward(const float* qkv, const float* probs, const float* dctx, int64_t batch,
                                      int32_t T, int32_t d, int32_t heads, float* dqkv, void* stream) {
  if (!qkv || !probs || !dctx || !dqkv || batch < 0 || T <= 0 || T > kBstTMax || heads <= 0 || d % heads ||
      d / heads > kBstDhMax)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_attn_train_backward: T <= %d, d/heads <= %d", kBstTMax, kBstDhMax);
  if (batch == 0) return RK_OK;
  att_set_attrs();
  const int dh = d / heads;
  const int US = att_slots(T, dh);
  if (US && T % 4 == 0 && d % 4 == 0) {
    const size_t lds = att_lds_bytes(T, dh, true);
#define RK_ATT_BWD(U_)                                                                                          \
  case U_:                                                                                                      \
    bst_attn_train_bwd_pkernel<U_><<<att_grid((const void*)bst_attn_train_bwd_pkernel<U_>, batch * heads, lds), \
                                     256, lds, (hipStream_t)stream>>>(qkv, probs, dctx, batch, T, d, heads, dqkv);     \
    break;
    switch (US) { RK_ATT_BWD(1) RK_ATT_BWD(2) RK_ATT_BWD(4) }
#undef RK_ATT_BWD
    return check_launch("rk_bst_attn_train_backward");
  }
  bst_attn_train_bwd_kernel<<<(unsigned)(batch * heads), 256, att_lds_bytes(T, d / heads, true),
                              (hipStream_t)stream>>>(qkv, probs, dctx, batch, T,
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
  const uint32_t thr = dropout_threshold(dropout_p);
  const float scale = (float)(1.0 / (1.0 - dropout_p));
  hipStream_t st = (hipStream_t)stream;
  const int L = ln_lanes(d, {base, o, gamma, beta, r, y});
  if (L) {
    const int64_t groups = (rows + 64 / L - 1) / (64 / L);  // row groups; kLnNR per wave
    const unsigned blocks = (unsigned)std::max<int64_t>(1, std::min<int64_t>((groups + 4 * kLnNR - 1) / (4 * kLnNR),
                                                                            16 * num_cus()));
#define RK_LN_FWD(L_)                                                                                             \
  case L_:                                                                                                        \
    bst_res_dropout_ln_fwd4_kernel<L_><<<blocks, 256, 0, st>>>(base, o, rows, d, seed, stream_slot, thr, scale,   \
                                                               gamma, beta, eps, r, y, mean, rstd);               \
    break;
    switch (L) { RK_LN_FWD(8) RK_LN_FWD(16) RK_LN_FWD(32) RK_LN_FWD(64) }
#undef RK_LN_FWD
  } else {
    bst_res_dropout_ln_fwd_kernel<<<grid_of(rows, 4), 256, 0, st>>>(base, o, rows, d, seed, stream_slot, thr, scale,
                                                                    gamma, beta, eps, r, y, mean, rstd);
  }
  return check_launch("rk_bst_res_dropout_ln_forward");
}

RK_API int64_t rk_bst_ln_backward_workspace_floats(int32_t d) {
  // per-workgroup partials, then the chunk sums of the first reduction pass
  return ((int64_t)kLnBlocks + (kLnBlocks + kLnChunk - 1) / kLnChunk) * 2 * (d > 0 ? d : 0);
}

RK_API int rk_bst_ln_backward(const float* dy, const float* r, const float* mean, const float* rstd,
                              const float* gamma, int64_t rows, int32_t d, double dropout_p, uint64_t seed,
                              const int64_t* stream_slot, float* dr, float* d_o, float* dgamma, float* dbeta,
                              float* workspace, int64_t workspace_floats, void* stream) {
  if (!dy || !r || !mean || !rstd || !gamma || !dr || !dgamma || !dbeta || !workspace || rows < 0 || d <= 0 ||
      d > 256 || !(dropout_p >= 0.0 && dropout_p < 1.0) || (dropout_p > 0.0 && !stream_slot))
    return fail(RK_ERR_INVALID, "rk_bst_ln_backward: bad arguments (d <= 256)");
  if (workspace_floats < rk_bst_ln_backward_workspace_floats(d))
    return fail(RK_ERR_INVALID, "rk_bst_ln_backward: workspace of %lld floats, needs %lld",
                (long long)workspace_floats, (long long)rk_bst_ln_backward_workspace_floats(d));
  return ln_backward(dy, nullptr, 0, 0, 1, nullptr, 0, r, mean, rstd, gamma, rows, d, dropout_p, seed, stream_slot,
                     dr, d_o, dgamma, dbeta, workspace, (hipStream_t)stream, "rk_bst_ln_backward");
}

RK_API int rk_bst_pool_ln_backward(const float* drow, int64_t ld_row, int32_t col, int32_t T,
                                   const int64_t* seq_len, int32_t mean_pool, const float* r, const float* mean,
                                   const float* rstd, const float* gamma, int64_t rows, int32_t d, double dropout_p,
                                   uint64_t seed, const int64_t* stream_slot, float* dr, float* d_o, float* dgamma,
                                   float* dbeta, float* workspace, int64_t workspace_floats, void* stream) {
  if (!drow || !r || !mean || !rstd || !gamma || !dr || !dgamma || !dbeta || !workspace || rows < 0 || T <= 0 ||
      rows % T || d <= 0 || d > 256 || col < 0 || col + d > ld_row || (mean_pool && !seq_len) ||
      !(dropout_p >= 0.0 && dropout_p < 1.0) || (dropout_p > 0.0 && !stream_slot))
    return fail(RK_ERR_INVALID, "rk_bst_pool_ln_backward: bad arguments (d <= 256, rows = batch * T)");
  if (workspace_floats < rk_bst_ln_backward_workspace_floats(d))
    return fail(RK_ERR_INVALID, "rk_bst_pool_ln_backward: workspace of %lld floats, needs %lld",
                (long long)workspace_floats, (long long)rk_bst_ln_backward_workspace_floats(d));
  if (ln_lanes(d, {r, gamma, dr, d_o, workspace}) == 0)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_pool_ln_backward: needs d %% 4 == 0, 16-B aligned rows and workspace");
  return ln_backward(nullptr, drow, ld_row, col, T, seq_len, mean_pool, r, mean, rstd, gamma, rows, d, dropout_p, seed,
                     stream_slot, dr, d_o, dgamma, dbeta, workspace, (hipStream_t)stream, "rk_bst_pool_ln_backward");
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
  if (n % 4 == 0 && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(f) |
                       reinterpret_cast<uintptr_t>(out)) & 15) == 0) {
    if (backward)
      bst_leaky_dropout4_kernel<true><<<grid_of(n / 4), 256, 0, st>>>(in, f, n, slope, seed, stream_slot, thr, scale,
                                                                      out);
    else
      bst_leaky_dropout4_kernel<false><<<grid_of(n / 4), 256, 0, st>>>(in, f, n, slope, seed, stream_slot, thr,
                                                                       scale, out);
    return check_launch("rk_bst_leaky_dropout");
  }
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
  if (d % 4 == 0 && d <= 1024 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
    bst_pool_fwd4_kernel<<<(unsigned)batch, 256, 0, (hipStream_t)stream>>>(out, T, d, seq_len, mean, row, ld_row, col);
    return check_launch("rk_bst_pool");
  }
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
