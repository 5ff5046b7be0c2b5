// Fused BST transformer block(s) + pooling, one workgroup per sample (d_model 128, T <= 64).
// Reference: BSTTransformer.forward bst.py:66-91 and the pooling of BSTModel.forward bst.py:224-241.
//
// A 512-thread workgroup (8 waves) owns one sample.  Its sequence lives in LDS the whole time:
//   Xs  [64][132]  block input x (gathered feed embeddings; later blocks: previous output)
//   Qs  [64][132]  Q, then ctx, then the pre-LN2 sum
//   Ks  [64][132]  K, then out1 (= LN1 output)
//   Vs  [64][132]  V, then the FFN hidden activation
// (row stride 132 floats: conflict-free float4 row reads).  Every projection is a 64 x 128 x 128
// FP32-MFMA GEMM (v_mfma_f32_32x32x2_f32) with the A operand read from LDS (float4 per lane,
// k = 8c + 4*(lane>>5) + e) and the nn.Linear weight rows streamed from L2; the positional
// embedding is added in the A loader of the Q/K projections and in the LN1 residual (it is
// added to queries and keys, not values: bst.py:69-71).  Attention per (head, 32-query tile)
// runs swapped (S^T = K_h Q_h^T: keys in registers, queries on lanes), so the softmax needs only
// a lane-pair exchange and P feeds the P.V MFMA as its B operand straight from the accumulator.
// Masked keys are -inf like bst.py:80; an all-masked row gives NaN exactly as torch's softmax.
#include "common.h"

namespace rk {

constexpr int kBD = 128;        // d_model
constexpr int kBT = 64;         // padded sequence rows
constexpr int kBLD = kBD + 4;   // LDS row stride
constexpr int kBWaves = 8;
constexpr int kBMaxBlocks = 4;

struct BstBlockW {
  const float* pos;  // [max_len, 128]
  const float *wq, *bq, *wk, *bk, *wv, *bv, *wo, *bo, *w1, *b1, *w2, *b2;
  const float *g1, *be1, *g2, *be2;
  float eps1, eps2, slope;
};

struct BstArgs {
  const float* table;
  int64_t rows, ld;
  const int64_t* seq;
  int64_t ld_seq;
  int T;
  const int64_t* seq_len;
  int64_t batch;
  int nblocks;
  BstBlockW blk[kBMaxBlocks];
  float* pool_out;
  int64_t ld_pool;
  int pool_mean;
  uint32_t* flags;
};

typedef float f4 __attribute__((ext_vector_type(4)));

// acc[j] += A[rt*32.., :] . W[ct_j*32.., :]^T over K = 128.  A rows from LDS (+ pos rows from
// global for t < T when ADDPOS), W rows from global; 2-deep register prefetch of W.
template <int NT, bool ADDPOS>
__device__ __forceinline__ void gemm128(const float* __restrict__ A, const float* __restrict__ pos, int T,
                                        const float* const (&W)[NT], f32x16 (&acc)[NT], int rt, int lane) {
  const int l32 = lane & 31, hk = 4 * (lane >> 5);
  const int row = rt * 32 + l32;
  const float* arow = A + row * kBLD + hk;
  const float* prow = (ADDPOS && row < T) ? pos + (int64_t)row * kBD + hk : nullptr;
  const float* wrow[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) wrow[j] = W[j] + (int64_t)l32 * kBD + hk;
  f4 bn[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) bn[j] = *reinterpret_cast<const f4*>(wrow[j]);
#pragma unroll 2
  for (int c = 0; c < kBD / 8; ++c) {
    f4 bc[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) bc[j] = bn[j];
    const int cn = c + 1 < kBD / 8 ? c + 1 : c;
#pragma unroll
    for (int j = 0; j < NT; ++j) bn[j] = *reinterpret_cast<const f4*>(wrow[j] + 8 * cn);
    f4 av = *reinterpret_cast<const f4*>(arow + 8 * c);
    if (ADDPOS) {
      if (prow) av = av + *reinterpret_cast<const f4*>(prow + 8 * c);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = mfma32(av[e], bc[j][e], acc[j]);
  }
}

__device__ __forceinline__ void zero(f32x16& a) {
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = 0.f;
}

// Row LayerNorm of rows [w*8, w*8+8) of S (in place), lane owns columns lane and lane+64.
__device__ __forceinline__ void layernorm_rows(float* S, const float* g, const float* be, float eps, int wave,
                                               int lane) {
  const float g0 = g[lane], g1 = g[lane + 64], b0 = be[lane], b1 = be[lane + 64];
  for (int r = wave * 8; r < wave * 8 + 8; ++r) {
    float* row = S + r * kBLD;
    const float x0 = row[lane], x1 = row[lane + 64];
    const float mean = wave_sum(x0 + x1) * (1.0f / kBD);
    const float d0 = x0 - mean, d1 = x1 - mean;
    const float var = wave_sum(d0 * d0 + d1 * d1) * (1.0f / kBD);
    const float rstd = 1.0f / sqrtf(var + eps);
    row[lane] = d0 * rstd * g0 + b0;
    row[lane + 64] = d1 * rstd * g1 + b1;
  }
}

__global__ __launch_bounds__(512) void bst_block_kernel(BstArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Xs = sm;
  float* Qs = Xs + kBT * kBLD;
  float* Ks = Qs + kBT * kBLD;
  float* Vs = Ks + kBT * kBLD;
  float* red = Vs + kBT * kBLD;  // [8][128] pooling partials

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5, hk = 4 * half;
  const int64_t b = blockIdx.x;
  const int T = a.T;
  const int64_t len = a.seq_len[b];
  const int nvalid = (int)(len < 0 ? 0 : (len > T ? T : len));

  // ---- gather the behaviour sequence: Xs[t] = table[seq[b, t]] (rows >= T are zero)
  for (int i = tid; i < kBT * (kBD / 4); i += 512) {
    const int t = i / (kBD / 4), c = (i % (kBD / 4)) * 4;
    f4 v = {0.f, 0.f, 0.f, 0.f};
    if (t < T) {
      const int64_t r = a.seq[b * a.ld_seq + t];
      if (r >= 0 && r < a.rows)
        v = *reinterpret_cast<const f4*>(a.table + r * a.ld + c);
      else if (c == 0)
        flag_oob(a.flags);
    }
    *reinterpret_cast<f4*>(Xs + t * kBLD + c) = v;
  }
  __syncthreads();

  const float sqrt_dh = 5.65685424949238f;  // math.sqrt(32) -> fp32; scores are divided like bst.py:79

  for (int blk = 0; blk < a.nblocks; ++blk) {
    const BstBlockW& P = a.blk[blk];
    // ---- 1. Q|K (x + pos) and V (x) projections: wave w -> row tile w/4, q/k col tiles
    //         2(w%4), 2(w%4)+1 of the 8 Q|K tiles, and V col tile w%4
    {
      const int rt = wave >> 2, q4 = wave & 3;
      f32x16 acc[2];
      zero(acc[0]);
      zero(acc[1]);
      const int ct0 = 2 * q4, ct1 = 2 * q4 + 1;  // 0..3 -> Q tiles, 4..7 -> K tiles
      const float* W2[2] = {(ct0 < 4 ? P.wq + ct0 * 32 * kBD : P.wk + (ct0 - 4) * 32 * kBD),
                            (ct1 < 4 ? P.wq + ct1 * 32 * kBD : P.wk + (ct1 - 4) * 32 * kBD)};
      gemm128<2, true>(Xs, P.pos, T, W2, acc, rt, lane);
      f32x16 vacc[1];
      zero(vacc[0]);
      const float* W1[1] = {P.wv + q4 * 32 * kBD};
      gemm128<1, false>(Xs, nullptr, T, W1, vacc, rt, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ct = 2 * q4 + j;
        float* dst = ct < 4 ? Qs : Ks;
        const float* bias = ct < 4 ? P.bq : P.bk;
        const int col = (ct & 3) * 32 + l32;
        const float bb = bias[col];
#pragma unroll
        for (int r = 0; r < 16; ++r) dst[(rt * 32 + acc_row(r, lane)) * kBLD + col] = acc[j][r] + bb;
      }
      const int vcol = q4 * 32 + l32;
      const float vb = P.bv[vcol];
#pragma unroll
      for (int r = 0; r < 16; ++r) Vs[(rt * 32 + acc_row(r, lane)) * kBLD + vcol] = vacc[0][r] + vb;
    }
    __syncthreads();

    // ---- 2. attention: wave w -> head w/2, query tile w%2; ctx written over Q_h of that tile
    {
      const int h = wave >> 1, qt = wave & 1, hc = h * 32;
      f32x16 S[2];
#pragma unroll
      for (int kt = 0; kt < 2; ++kt) {
        zero(S[kt]);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const f4 kv = *reinterpret_cast<const f4*>(Ks + (kt * 32 + l32) * kBLD + hc + 8 * c + hk);
          const f4 qv = *reinterpret_cast<const f4*>(Qs + (qt * 32 + l32) * kBLD + hc + 8 * c + hk);
#pragma unroll
          for (int e = 0; e < 4; ++e) S[kt] = mfma32(kv[e], qv[e], S[kt]);
        }
      }
      // scores / sqrt(d_h), keys >= len (and padding rows >= T) -> -inf, softmax over keys
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * 32 + acc_row(r, lane);
          const float s = key < nvalid ? S[kt][r] / sqrt_dh : -INFINITY;
          S[kt][r] = s;
          m = fmaxf(m, s);
        }
      m = fmaxf(m, __shfl_xor(m, 32, kWave));
      float l = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = expf(S[kt][r] - m);
          S[kt][r] = p;
          l += p;
        }
      l += __shfl_xor(l, 32, kWave);
      // ctx^T[d, q] = sum_key V[key, hc + d] * P[key, q]; B operand = the P accumulators
      f32x16 C;
      zero(C);
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 16; ++s) {
          const int key = kt * 32 + (s & 3) + 8 * (s >> 2) + 4 * half;
          C = mfma32(Vs[key * kBLD + hc + l32], S[kt][s], C);
        }
      const float inv_l = 1.0f / l;
#pragma unroll
      for (int r = 0; r < 16; ++r) Qs[(qt * 32 + l32) * kBLD + hc + acc_row(r, lane)] = C[r] * inv_l;
    }
    __syncthreads();

    // ---- 3. out1 = LN1((x + pos) + (ctx . Wo^T + bo)) -> Ks
    {
      const int rt = wave >> 2, ct = wave & 3;
      f32x16 acc[1];
      zero(acc[0]);
      const float* W[1] = {P.wo + ct * 32 * kBD};
      gemm128<1, false>(Qs, nullptr, T, W, acc, rt, lane);
      const int col = ct * 32 + l32;
      const float bb = P.bo[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = rt * 32 + acc_row(r, lane);
        float res = Xs[t * kBLD + col];
        if (t < T) res = res + P.pos[(int64_t)t * kBD + col];
        Ks[t * kBLD + col] = res + (acc[0][r] + bb);
      }
    }
    __syncthreads();
    layernorm_rows(Ks, P.g1, P.be1, P.eps1, wave, lane);
    __syncthreads();

    // ---- 4. f = LeakyReLU(out1 . W1^T + b1) -> Vs
    {
      const int rt = wave >> 2, ct = wave & 3;
      f32x16 acc[1];
      zero(acc[0]);
      const float* W[1] = {P.w1 + ct * 32 * kBD};
      gemm128<1, false>(Ks, nullptr, T, W, acc, rt, lane);
      const int col = ct * 32 + l32;
      const float bb = P.b1[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float z = acc[0][r] + bb;
        Vs[(rt * 32 + acc_row(r, lane)) * kBLD + col] = z > 0.f ? z : z * P.slope;
      }
    }
    __syncthreads();

    // ---- 5. out = LN2(out1 + (f . W2^T + b2)) -> Qs (last block) or Xs (next block's input)
    float* dst = (blk + 1 < a.nblocks) ? Xs : Qs;
    {
      const int rt = wave >> 2, ct = wave & 3;
      f32x16 acc[1];
      zero(acc[0]);
      const float* W[1] = {P.w2 + ct * 32 * kBD};
      gemm128<1, false>(Vs, nullptr, T, W, acc, rt, lane);
      const int col = ct * 32 + l32;
      const float bb = P.b2[col];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int t = rt * 32 + acc_row(r, lane);
        dst[t * kBLD + col] = Ks[t * kBLD + col] + (acc[0][r] + bb);
      }
    }
    __syncthreads();
    layernorm_rows(dst, P.g2, P.be2, P.eps2, wave, lane);
    __syncthreads();
  }

  // ---- pooling over the T real positions (padded positions of the batch included, bst.py:238-241)
  const float* out = Qs;  // the last block's LN2 output
  {
    float s0 = 0.f, s1 = 0.f;
    for (int t = wave * 8; t < wave * 8 + 8; ++t)
      if (t < T) {
        s0 += out[t * kBLD + lane];
        s1 += out[t * kBLD + lane + 64];
      }
    red[wave * kBD + lane] = s0;
    red[wave * kBD + lane + 64] = s1;
  }
  __syncthreads();
  if (tid < kBD) {
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < kBWaves; ++w) s += red[w * kBD + tid];
    if (a.pool_mean) s = s / (float)len;
    a.pool_out[b * a.ld_pool + tid] = s;
  }
}

}  // namespace rk

using namespace rk;

RK_API int rk_bst_forward_blocks(const float* table, int64_t table_rows, int64_t ld_table, const int64_t* seq,
                                 int64_t ld_seq, int32_t T, const int64_t* seq_len, int64_t batch, int32_t d_model,
                                 int32_t heads, int32_t nblocks, const float* const* block_params,
                                 const float* block_scalars, float* pool_out, int64_t ld_pool, int32_t pool_mean,
                                 void* stream) {
  if (d_model != kBD || heads != 4)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_forward_blocks: d_model=%d heads=%d (fused path: 128/4)", d_model, heads);
  if (T <= 0 || T > kBT) return fail(RK_ERR_UNSUPPORTED, "rk_bst_forward_blocks: T=%d outside [1, %d]", T, kBT);
  if (nblocks <= 0 || nblocks > kBMaxBlocks)
    return fail(RK_ERR_UNSUPPORTED, "rk_bst_forward_blocks: %d blocks (max %d)", nblocks, kBMaxBlocks);
  if (!table || !seq || !seq_len || !block_params || !block_scalars || !pool_out || ld_table % 4 ||
      ((uintptr_t)table & 15u) || ld_seq < T || ld_pool < kBD || table_rows <= 0)
    return fail(RK_ERR_INVALID, "rk_bst_forward_blocks: bad arguments");
  BstArgs a = {};
  a.table = table;
  a.rows = table_rows;
  a.ld = ld_table;
  a.seq = seq;
  a.ld_seq = ld_seq;
  a.T = T;
  a.seq_len = seq_len;
  a.batch = batch;
  a.nblocks = nblocks;
  for (int i = 0; i < nblocks; ++i) {
    const float* const* p = block_params + 17 * i;
    BstBlockW& w = a.blk[i];
    w.pos = p[0];
    w.wq = p[1];
    w.bq = p[2];
    w.wk = p[3];
    w.bk = p[4];
    w.wv = p[5];
    w.bv = p[6];
    w.wo = p[7];
    w.bo = p[8];
    w.w1 = p[9];
    w.b1 = p[10];
    w.w2 = p[11];
    w.b2 = p[12];
    w.g1 = p[13];
    w.be1 = p[14];
    w.g2 = p[15];
    w.be2 = p[16];
    for (int k = 0; k < 17; ++k)
      if (!p[k] || ((uintptr_t)p[k] & 15u))
        return fail(RK_ERR_INVALID, "rk_bst_forward_blocks: block %d parameter %d null or misaligned", i, k);
    w.eps1 = block_scalars[3 * i];
    w.eps2 = block_scalars[3 * i + 1];
    w.slope = block_scalars[3 * i + 2];
  }
  a.pool_out = pool_out;
  a.ld_pool = ld_pool;
  a.pool_mean = pool_mean;
  a.flags = device_flags();
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "rk_bst_forward_blocks: negative batch");
  const size_t shm = (size_t)(4 * kBT * kBLD + kBWaves * kBD) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)bst_block_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  bst_block_kernel<<<(unsigned)batch, 512, shm, (hipStream_t)stream>>>(a);
  return check_launch("rk_bst_forward_blocks");
}
