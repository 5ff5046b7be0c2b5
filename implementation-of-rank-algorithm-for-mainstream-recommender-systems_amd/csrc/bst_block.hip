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
constexpr float kLog2eOverSqrtDh = 0.25503486f;  // log2(e) / sqrt(32): softmax scale, d_h = 32

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

// Optional per-phase shader-clock counters (tools/bst_phases.hip builds with RK_BST_PHASES):
// thread 0 adds the cycles since the previous barrier to g_bst_phase[i].
#ifdef RK_BST_PHASES
__device__ unsigned long long g_bst_phase[16];
#define BST_PHASE(i)                                           \
  do {                                                         \
    if (tid == 0) {                                            \
      const unsigned long long now_ = clock64();               \
      atomicAdd(&g_bst_phase[i], now_ - t_phase);              \
      t_phase = now_;                                          \
    }                                                          \
  } while (0)
#else
#define BST_PHASE(i) \
  do {               \
  } while (0)
#endif

// Weight-row stream of NT 32-row W tiles in MFMA B-operand order: lane (n = lane%32, half h)
// holds W[n][32s + 8c + 4h + e] for super-chunk s (32 k = one 128-B line of each W row), chunk c,
// e < 4.  A super-chunk's loads are issued back to back so every line is consumed while in L1;
// super-chunk 0 can be issued before the phase barrier (WStream::start) so its latency overlaps
// the previous phase's epilogue.
template <int NT>
struct WStream {
  const float* wrow[NT];
  f4 bq[2][4][NT];
  __device__ __forceinline__ void start(const float* const (&W)[NT], int lane) {
#pragma unroll
    for (int j = 0; j < NT; ++j) wrow[j] = W[j] + (int64_t)(lane & 31) * kBD + 4 * (lane >> 5);
    issue(0, 0);
  }
  __device__ __forceinline__ void issue(int s, int buf) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c) bq[buf][c][j] = *reinterpret_cast<const f4*>(wrow[j] + 32 * s + 8 * c);
  }
};

// acc[j] += A[rt*32.., :] . W_j[0..32, :]^T over K = 128 (A in LDS, W streamed by `ws`, whose
// super-chunk 0 is already in flight).  Fully unrolled; the next super-chunk is loaded while
// this one feeds the MFMAs, the next A float4 one chunk ahead; sched_barrier keeps the compiler
// from sinking the loads next to their use.
template <int NT>
__device__ __forceinline__ void gemm128(const float* __restrict__ A, WStream<NT>& ws, f32x16 (&acc)[NT], int rt,
                                        int lane) {
  constexpr int NS = kBD / 32;
  const float* arow = A + (rt * 32 + (lane & 31)) * kBLD + 4 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  f4 a_cur = *reinterpret_cast<const f4*>(arow);
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    __builtin_amdgcn_sched_barrier(0);
    if (s + 1 < NS) ws.issue(s + 1, (s + 1) & 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int cc = 4 * s + c;
      f4 a_next = a_cur;
      if (cc + 1 < 4 * NS) a_next = *reinterpret_cast<const f4*>(arow + 8 * (cc + 1));
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[j] = mfma32(a_cur[e], ws.bq[s & 1][c][j][e], acc[j]);
      a_cur = a_next;
    }
  }
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not for its global
// loads, so weight prefetches stay in flight across it (__syncthreads would drain vmcnt).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Sum over the 8 lanes of an aligned lane octet (xor butterfly inside the octet).
__device__ __forceinline__ float octet_sum(float v) {
  v += __shfl_xor(v, 1, kWave);
  v += __shfl_xor(v, 2, kWave);
  v += __shfl_xor(v, 4, kWave);
  return v;
}

// LayerNorm of all 64 rows of S (two-pass mean / biased variance like nn.LayerNorm): thread tid
// owns row tid/8 and columns 4*(tid%8) + 32*q + e (q, e < 4), i.e. each 32-column slice of a row is
// one contiguous 128 B read by the row's 8 lanes.
struct LnCols {
  f4 g[4], b[4];
};
__device__ __forceinline__ LnCols ln_load(const float* g, const float* be, int tid) {
  LnCols p;
  const int c0 = 4 * (tid & 7);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    p.g[q] = *reinterpret_cast<const f4*>(g + c0 + 32 * q);
    p.b[q] = *reinterpret_cast<const f4*>(be + c0 + 32 * q);
  }
  return p;
}
// y = LN(S row).  Output modes: pool != NULL -> pool[wave][col] = sum of y over the wave's 8 rows
// that are < T (the last block feeding the pooling); else S = y, and with `xp` set also
// xp = y + pos[row] (rows < T, zero otherwise): the next block's raw and position-added inputs.
__device__ __forceinline__ void layernorm_rows(float* S, const LnCols& p, float eps, int tid, float* pool, int T,
                                               float* xp, const float* pos) {
  const int r = tid >> 3, c0 = 4 * (tid & 7);
  float* row = S + r * kBLD + c0;
  const bool real = r < T;
  f4 pv[4];
  if (xp) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      pv[q] = real ? *reinterpret_cast<const f4*>(pos + (int64_t)r * kBD + c0 + 32 * q) : z;
    }
  }
  f4 x[4];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    x[q] = *reinterpret_cast<const f4*>(row + 32 * q);
    s += (x[q][0] + x[q][1]) + (x[q][2] + x[q][3]);
  }
  const float mean = octet_sum(s) * (1.0f / kBD);
  float v = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[q][e] -= mean;
      v += x[q][e] * x[q][e];
    }
  const float rstd = 1.0f / sqrtf(octet_sum(v) * (1.0f / kBD) + eps);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = x[q][e] * rstd * p.g[q][e] + p.b[q][e];
    if (!pool) {
      *reinterpret_cast<f4*>(row + 32 * q) = y;
      if (xp) {
        const f4 z = {0.f, 0.f, 0.f, 0.f};
        *reinterpret_cast<f4*>(xp + r * kBLD + c0 + 32 * q) = real ? y + pv[q] : z;
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = real ? y[e] : 0.f;
        t += __shfl_xor(t, 8, kWave);
        t += __shfl_xor(t, 16, kWave);
        t += __shfl_xor(t, 32, kWave);
        y[e] = t;
      }
      if ((tid & 63) < 8) *reinterpret_cast<f4*>(pool + (tid >> 6) * kBD + c0 + 32 * q) = y;
    }
  }
}

__device__ __forceinline__ void zero(f32x16& a) {
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = 0.f;
}

// acc (32x32 tile rt/ct) + bias -> dst rows, optional LeakyReLU / residual.
__device__ __forceinline__ void store_tile(float* dst, const f32x16& acc, const float* bias, int rt, int ct, int lane,
                                           const float* residual = nullptr, float slope = 1.f, bool leaky = false) {
  const int col = ct * 32 + (lane & 31);
  const float bb = bias[col];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int t = rt * 32 + acc_row(r, lane);
    float z = acc[r] + bb;
    if (leaky) z = z > 0.f ? z : z * slope;
    if (residual) z = residual[t * kBLD + col] + z;
    dst[t * kBLD + col] = z;
  }
}

// LDS per sample:  Xs = x + pos (Q/K input and the LN1 residual), Qs = x (V input), then Q / ctx /
// pre-LN2 sum;  Ks = K, then out1;  Vs = V, then the FFN hidden activation.
__global__ __launch_bounds__(512) void bst_block_kernel(BstArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Xs = sm;
  float* Qs = Xs + kBT * kBLD;
  float* Ks = Qs + kBT * kBLD;
  float* Vs = Ks + kBT * kBLD;
  float* red = Vs + kBT * kBLD;  // [8][128] pooling partials

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5, hk = 4 * half;
  const int rt = wave >> 2, q4 = wave & 3;  // GEMM phases: row tile and column tile of this wave
  const int64_t b = blockIdx.x;
  const int T = a.T;
  const int64_t len = a.seq_len[b];
  const int nvalid = (int)(len < 0 ? 0 : (len > T ? T : len));
#ifdef RK_BST_PHASES
  unsigned long long t_phase = clock64();
#endif

  WStream<1> ws1;
  {
    const float* W[1] = {a.blk[0].wv + q4 * 32 * kBD};
    ws1.start(W, lane);
  }
  // ---- gather: Qs[t] = x = table[seq[b, t]], Xs[t] = x + pos[t]  (rows >= T zero)
  for (int i = tid; i < kBT * (kBD / 4); i += 512) {
    const int t = i / (kBD / 4), c = (i % (kBD / 4)) * 4;
    f4 v = {0.f, 0.f, 0.f, 0.f}, vp = v;
    if (t < T) {
      const int64_t r = a.seq[b * a.ld_seq + t];
      const f4 pv = *reinterpret_cast<const f4*>(a.blk[0].pos + (int64_t)t * kBD + c);
      if (r >= 0 && r < a.rows)
        v = *reinterpret_cast<const f4*>(a.table + r * a.ld + c);
      else if (c == 0)
        flag_oob(a.flags);
      vp = v + pv;
    }
    *reinterpret_cast<f4*>(Qs + t * kBLD + c) = v;
    *reinterpret_cast<f4*>(Xs + t * kBLD + c) = vp;
  }
  lds_barrier(); BST_PHASE(0);


  for (int blk = 0; blk < a.nblocks; ++blk) {
    const BstBlockW& P = a.blk[blk];
    // ---- 1a. V = x . Wv^T + bv -> Vs   (wave: row tile rt, column tile q4)
    WStream<2> ws2;
    {
      f32x16 acc[1];
      gemm128<1>(Qs, ws1, acc, rt, lane);
      const int ct0 = 2 * q4, ct1 = 2 * q4 + 1;  // of the 8 Q|K column tiles: 0..3 Q, 4..7 K
      const float* W[2] = {(ct0 < 4 ? P.wq + ct0 * 32 * kBD : P.wk + (ct0 - 4) * 32 * kBD),
                           (ct1 < 4 ? P.wq + ct1 * 32 * kBD : P.wk + (ct1 - 4) * 32 * kBD)};
      ws2.start(W, lane);
      store_tile(Vs, acc[0], P.bv, rt, q4, lane);
    }
    lds_barrier(); BST_PHASE(1);
    // ---- 1b. [Q|K] = (x + pos) . W^T + b -> Qs, Ks   (wave: row tile rt, Q|K tiles 2q4, 2q4+1)
    {
      f32x16 acc[2];
      gemm128<2>(Xs, ws2, acc, rt, lane);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ct = 2 * q4 + j;
        store_tile(ct < 4 ? Qs : Ks, acc[j], ct < 4 ? P.bq : P.bk, rt, ct & 3, lane);
      }
    }
    lds_barrier(); BST_PHASE(2);

    // ---- 2. attention: wave w -> head w/2, query tile w%2; ctx written over Q_h of that tile
    {
      const int h = wave >> 1, qt = wave & 1, hc = h * 32;
      // all operands up front: Q_h (this query tile), K_h and the V_h column this lane feeds
      f4 qv[4], kv[2][4];
      float vv[2][16];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        qv[c] = *reinterpret_cast<const f4*>(Qs + (qt * 32 + l32) * kBLD + hc + 8 * c + hk);
#pragma unroll
        for (int kt = 0; kt < 2; ++kt)
          kv[kt][c] = *reinterpret_cast<const f4*>(Ks + (kt * 32 + l32) * kBLD + hc + 8 * c + hk);
      }
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int s = 0; s < 16; ++s)
          vv[kt][s] = Vs[(kt * 32 + (s & 3) + 8 * (s >> 2) + 4 * half) * kBLD + hc + l32];
      f32x16 S[2];
      zero(S[0]);
      zero(S[1]);
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int kt = 0; kt < 2; ++kt) S[kt] = mfma32(kv[kt][c][e], qv[c][e], S[kt]);
      // softmax over keys of scores / sqrt(d_h), keys >= len (and padding rows >= T) -> -inf
      // (bst.py:79-82): the max is taken on the raw scores (the positive scale commutes with it)
      // and exp((s - m) / sqrt(d_h)) = exp2((s - m) * log2(e) / sqrt(d_h)) on v_exp_f32.  An
      // all-masked row gives m = -inf, (-inf) - (-inf) = NaN, hence NaN like torch.
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = kt * 32 + acc_row(r, lane);
          const float sc = key < nvalid ? S[kt][r] : -INFINITY;
          S[kt][r] = sc;
          m = fmaxf(m, sc);
        }
      m = fmaxf(m, __shfl_xor(m, 32, kWave));
      float l = 0.f;
#pragma unroll
      for (int kt = 0; kt < 2; ++kt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = __builtin_amdgcn_exp2f((S[kt][r] - m) * kLog2eOverSqrtDh);
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
        for (int s = 0; s < 16; ++s) C = mfma32(vv[kt][s], S[kt][s], C);
      const float* W[1] = {P.wo + q4 * 32 * kBD};
      ws1.start(W, lane);
      const float inv_l = 1.0f / l;
#pragma unroll
      for (int r = 0; r < 16; ++r) Qs[(qt * 32 + l32) * kBLD + hc + acc_row(r, lane)] = C[r] * inv_l;
    }
    lds_barrier(); BST_PHASE(3);

    // ---- 3. pre-LN1 = (x + pos) + (ctx . Wo^T + bo) -> Ks;  LN1 in place
    {
      f32x16 acc[1];
      gemm128<1>(Qs, ws1, acc, rt, lane);
      const float* W[1] = {P.w1 + q4 * 32 * kBD};
      ws1.start(W, lane);
      store_tile(Ks, acc[0], P.bo, rt, q4, lane, Xs);
    }
    const LnCols ln1 = ln_load(P.g1, P.be1, tid);
    lds_barrier(); BST_PHASE(4);
    layernorm_rows(Ks, ln1, P.eps1, tid, nullptr, T, nullptr, nullptr);
    lds_barrier(); BST_PHASE(5);

    // ---- 4. f = LeakyReLU(out1 . W1^T + b1) -> Vs
    {
      f32x16 acc[1];
      gemm128<1>(Ks, ws1, acc, rt, lane);
      const float* W[1] = {P.w2 + q4 * 32 * kBD};
      ws1.start(W, lane);
      store_tile(Vs, acc[0], P.b1, rt, q4, lane, nullptr, P.slope, true);
    }
    lds_barrier(); BST_PHASE(6);

    // ---- 5. pre-LN2 = out1 + (f . W2^T + b2) -> Qs;  LN2 -> next block's Qs / Xs, or the pooling
    const bool last = blk + 1 == a.nblocks;
    {
      f32x16 acc[1];
      gemm128<1>(Vs, ws1, acc, rt, lane);
      if (!last) {
        const float* W[1] = {a.blk[blk + 1].wv + q4 * 32 * kBD};
        ws1.start(W, lane);
      }
      store_tile(Qs, acc[0], P.b2, rt, q4, lane, Ks);
    }
    const LnCols ln2 = ln_load(P.g2, P.be2, tid);
    lds_barrier(); BST_PHASE(7);
    // last block: per-wave column sums of the LN2 rows < T (every real position of the batch,
    // padded ones included, bst.py:238-241)
    layernorm_rows(Qs, ln2, P.eps2, tid, last ? red : nullptr, T, last ? nullptr : Xs,
                   last ? nullptr : a.blk[blk + 1].pos);
    lds_barrier(); BST_PHASE(8);
  }
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
