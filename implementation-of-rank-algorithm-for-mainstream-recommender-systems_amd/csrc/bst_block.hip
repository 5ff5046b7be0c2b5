// Fused BST transformer block(s) + pooling, one workgroup per sample (d_model 128, T <= 64).
// Reference: BSTTransformer.forward bst.py:66-91 and the pooling of BSTModel.forward bst.py:224-241.
//
// A persistent 512-thread workgroup (8 waves, one per CU: the LDS below is the occupancy limit)
// walks samples b = blockIdx.x + k * gridDim.x.  A sample's sequence stays in LDS throughout:
//   Xs [64][132]  x + pos         (Q/K projection input and the LN1 residual)
//   Qs [64][132]  x, then Q, ctx, the pre-LN2 sum / LN2 output
//   Ks [64][132]  K, then pre-LN1 / out1
//   Vs [64][132]  V, then the FFN hidden activation
// (row stride 132 floats: conflict-free float4 row reads).  The positional embedding is added to
// queries and keys, not values (bst.py:69-71), so the gather writes both x and x + pos.
//
// Projections (V, Q|K, O, FFN1, FFN2) are 64 x 128 x 128 GEMMs on v_mfma_f32_32x32x2_f32 (exact
// f32; back-to-back dependent accumulation issues at the full 64-cycle rate): wave w owns the
// 32x32 tile (row tile w/4, column tile w%4), A float4s from LDS, the nn.Linear rows streamed from
// L2 in 32-k super-chunks, double buffered, the first one issued before the phase barrier.  Attention per (head, 32-query tile) runs on v_mfma_f32_32x32x2_f32 swapped
// (S^T = K_h Q_h^T: keys in registers, queries on lanes), so the softmax needs one lane-pair
// exchange and P feeds the P.V MFMA as its B operand straight from the accumulator.  Masked keys
// are -inf like bst.py:80; an all-masked row gives NaN exactly as torch's softmax.
#include "common.h"


namespace rk {

constexpr int kBD = 128;       // d_model
constexpr int kBT = 64;        // padded sequence rows
constexpr int kBLD = kBD + 4;  // LDS row stride
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

// Optional per-phase shader-clock counters (tools/bst_phases.hip builds with RK_BST_PHASES).
#ifdef RK_BST_PHASES
__device__ unsigned long long g_bst_phase[16];
__device__ unsigned long long g_bst_wave[10][8];  // [mark][wave]
// cycles since the previous barrier, thread 0, into g_bst_phase[i]
#define BST_PHASE(i)                                            \
  do {                                                          \
    if (lane == 0) {                                            \
      const unsigned long long now_ = clock64();                \
      if (tid == 0) atomicAdd(&g_bst_phase[i], now_ - t_phase); \
      t_phase = now_;                                           \
    }                                                           \
  } while (0)
// cycles from the start of the current phase to this point, per wave
#define BST_MARK(i)                                                            \
  do {                                                                         \
    if (lane == 0) atomicAdd(&g_bst_wave[(i) - 9][wave], clock64() - t_phase); \
  } while (0)
#else
#define BST_PHASE(i) \
  do {               \
  } while (0)
#define BST_MARK(i) \
  do {              \
  } while (0)
#endif

// Weight stream over TT 32-row W tiles in 32x32x2 B-operand order, consumed one tile after the
// other: super-chunk g (tile g/4, k = 32*(g%4) .. +31, one 128-B line of each W row) gives lane
// (n = lane%32, half h) W_tile[n][32*(g%4) + 8c + 4h + e], c < 4, e < 4.  R buffers: start()
// issues the first R-1 super-chunks before the barrier that opens the phase, gemm128() keeps R-1
// in flight.  nn.Linear order (PK false), measured at batch 2048 (tools/bst_phases.hip): 2 buffers
// 328 us, 3 345 us, 4 372 us -- deeper rings cost more in register pressure and VMEM queueing than
// they hide.  PK: the tile stored in that order (rk_bst_pack_block_weight), each load one
// contiguous 1 KiB; there 3 buffers beat 2 in each of three interleaved rounds (279-283 vs
// 282-287 us, profiles/r06/bst_lib_ab.log), at the same 256 VGPRs.
template <int TT, bool PK>
struct WStream {
  static constexpr int R = PK ? 3 : 2;  // super-chunk buffers
  const float* wrow[TT];
  f4 bq[R][4];
  __device__ __forceinline__ void start(const float* const (&W)[TT], int lane) {
#pragma unroll
    for (int j = 0; j < TT; ++j)
      wrow[j] = PK ? W[j] + 4 * lane : W[j] + (int64_t)(lane & 31) * kBD + 4 * (lane >> 5);
#pragma unroll
    for (int g = 0; g + 1 < R; ++g) issue(g);
  }
  __device__ __forceinline__ void issue(int g) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      bq[g % R][c] = *reinterpret_cast<const f4*>(PK ? wrow[g / 4] + 1024 * (g % 4) + 256 * c
                                                     : wrow[g / 4] + 32 * (g % 4) + 8 * c);
  }
};

// acc[j] = A[rt*32.., :] . W_j[0..32, :]^T over K = 128 for the TT tiles of `ws` (its first R - 1
// super-chunks already in flight), A in LDS.  Fully unrolled; super-chunk g + R - 1 is loaded while g feeds
// the MFMAs (one dependent accumulator chain at a time: 32x32x2_f32 accumulates back to back at the
// full 64-cycle issue rate), the next A float4 one chunk ahead; sched_barrier keeps the compiler
// from sinking the loads next to their use.
template <int TT, bool PK>
__device__ __forceinline__ void gemm128(const float* __restrict__ A, WStream<TT, PK>& ws, f32x16 (&acc)[TT], int rt,
                                        int lane) {
  constexpr int NG = TT * (kBD / 32);
  const float* arow = A + (rt * 32 + (lane & 31)) * kBLD + 4 * (lane >> 5);
#pragma unroll
  for (int j = 0; j < TT; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  f4 a_cur = *reinterpret_cast<const f4*>(arow);
  constexpr int R = WStream<TT, PK>::R;
#pragma unroll
  for (int g = 0; g < NG; ++g) {
    __builtin_amdgcn_sched_barrier(0);
    if (g + R - 1 < NG) ws.issue(g + R - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int cc = 4 * (g % 4) + c, cn = (cc + 1) % 16;
      const f4 a_next = g + 1 < NG || c < 3 ? *reinterpret_cast<const f4*>(arow + 8 * cn) : a_cur;
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[g / 4] = mfma32(a_cur[e], ws.bq[g % R][c][e], acc[g / 4]);
      a_cur = a_next;
    }
  }
}

// acc (32x32 tile rt/ct) + bias value of this lane's column (loaded before the GEMM) -> dst rows,
// optional LeakyReLU and residual (residual[t][col] + z, the reference's operand order).
__device__ __forceinline__ void store_tile(float* dst, const f32x16& acc, float bb, int rt, int ct, int lane,
                                           const float* residual = nullptr, float slope = 1.f, bool leaky = false) {
  const int col = ct * 32 + (lane & 31);
  // residual reads all issued before the first store (dst and residual are distinct LDS buffers,
  // which the compiler cannot prove: interleaved, every read would wait for the previous store)
  float res[16];
  if (residual) {
#pragma unroll
    for (int r = 0; r < 16; ++r) res[r] = residual[(rt * 32 + acc_row(r, lane)) * kBLD + col];
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int t = rt * 32 + acc_row(r, lane);
    float z = acc[r] + bb;
    if (leaky) z = z > 0.f ? z : z * slope;
    if (residual) z = res[r] + z;
    dst[t * kBLD + col] = z;
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
// S = LN(S) in place; with `xp` set also xp = LN(S) + pos[row] (rows < T, zero otherwise): the next
// block's raw and position-added inputs.
__device__ __forceinline__ void layernorm_rows(float* S, const LnCols& p, float eps, int tid, int T, float* xp,
                                               const float* pos) {
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
    *reinterpret_cast<f4*>(row + 32 * q) = y;
    if (xp) {
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f4*>(xp + r * kBLD + c0 + 32 * q) = real ? y + pv[q] : z;
    }
  }
}

// Next-sample gather held in registers: thread tid owns rows t = tid/32 + 16k (k < 4), columns
// 4*(tid%32)..+3.  index() loads the ids, rows() the table rows and positions, store() writes x
// and x + pos to LDS at the sample boundary.
struct XGather {
  int64_t idx[4];
  f4 x[4], p[4];
  __device__ __forceinline__ void index(const BstArgs& a, int64_t b, int tid) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = (tid >> 5) + 16 * k;
      idx[k] = t < a.T ? a.seq[b * a.ld_seq + t] : 0;
    }
  }
  __device__ __forceinline__ void rows(const BstArgs& a, int tid) {
    const int c = 4 * (tid & 31);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = (tid >> 5) + 16 * k;
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      x[k] = z;
      p[k] = z;
      if (t < a.T) {
        p[k] = *reinterpret_cast<const f4*>(a.blk[0].pos + (int64_t)t * kBD + c);
        if (idx[k] >= 0 && idx[k] < a.rows)
          x[k] = *reinterpret_cast<const f4*>(a.table + idx[k] * a.ld + c);
        else if (c == 0)
          flag_oob(a.flags);
      }
    }
  }
  __device__ __forceinline__ void store(float* Qs, float* Xs, int T, int tid) const {
    const int c = 4 * (tid & 31);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int t = (tid >> 5) + 16 * k;
      const f4 z = {0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f4*>(Qs + t * kBLD + c) = x[k];
      *reinterpret_cast<f4*>(Xs + t * kBLD + c) = t < T ? x[k] + p[k] : z;
    }
  }
};

__device__ __forceinline__ void zero(f32x16& a) {
#pragma unroll
  for (int r = 0; r < 16; ++r) a[r] = 0.f;
}

template <bool PK>
__global__ __launch_bounds__(512) void bst_block_kernel(BstArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* Xs = sm;
  float* Qs = Xs + kBT * kBLD;
  float* Ks = Qs + kBT * kBLD;
  float* Vs = Ks + kBT * kBLD;
  float* red = Vs + kBT * kBLD;  // [4][128] pooling partials

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5, hk = 4 * half;
  const int rt = wave >> 2, q4 = wave & 3;  // projections: this wave's 32x32 tile (row tile, column tile)
  const int c32 = q4 * 32 + l32;            // this lane's output column in them
  const int T = a.T;
#ifdef RK_BST_PHASES
  unsigned long long t_phase = clock64();
#endif
  int64_t b = blockIdx.x;
  WStream<1, PK> ws1;
  {
    const float* W[1] = {a.blk[0].wv + q4 * 32 * kBD};
    ws1.start(W, lane);
  }
  XGather xg;
  xg.index(a, b, tid);
  xg.rows(a, tid);
  xg.store(Qs, Xs, T, tid);
  lds_barrier(); BST_PHASE(0);

  while (true) {
    const int64_t len = a.seq_len[b];
    const int nvalid = (int)(len < 0 ? 0 : (len > T ? T : len));
    const int64_t next = b + gridDim.x;
    const bool has_next = next < a.batch;
    for (int blk = 0; blk < a.nblocks; ++blk) {
      const BstBlockW& P = a.blk[blk];
      const bool last = blk + 1 == a.nblocks;
      // ---- 1a. V = x . Wv^T + bv -> Vs
      WStream<2, PK> ws2;
      {
        f32x16 acc[1];
        const float bb = P.bv[c32];
        gemm128<1>(Qs, ws1, acc, rt, lane);
        BST_MARK(9);
        const int ct0 = 2 * q4, ct1 = 2 * q4 + 1;  // of the 8 Q|K column tiles: 0..3 Q, 4..7 K
        const float* W[2] = {(ct0 < 4 ? P.wq + ct0 * 32 * kBD : P.wk + (ct0 - 4) * 32 * kBD),
                             (ct1 < 4 ? P.wq + ct1 * 32 * kBD : P.wk + (ct1 - 4) * 32 * kBD)};
        ws2.start(W, lane);
        store_tile(Vs, acc[0], bb, rt, q4, lane);
      }
      BST_MARK(14);
      lds_barrier(); BST_PHASE(1);
      // ---- 1b. [Q|K] = (x + pos) . W^T + b -> Qs, Ks   (wave: row tile rt, Q|K tiles 2q4, 2q4+1)
      {
        f32x16 acc[2];
        float bb[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ct = 2 * q4 + j;
          bb[j] = (ct < 4 ? P.bq : P.bk)[(ct & 3) * 32 + l32];
        }
        gemm128<2>(Xs, ws2, acc, rt, lane);
        BST_MARK(10);
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ct = 2 * q4 + j;
          store_tile(ct < 4 ? Qs : Ks, acc[j], bb[j], rt, ct & 3, lane);
        }
      }
      BST_MARK(15);
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
        // (bst.py:79-82): the max is taken on the raw scores (the positive scale commutes with
        // it) and exp((s - m) / sqrt(d_h)) = exp2((s - m) * log2(e) / sqrt(d_h)) on v_exp_f32.
        // An all-masked row gives m = -inf, (-inf) - (-inf) = NaN, hence NaN like torch.
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
        const float bb = P.bo[c32];
        gemm128<1>(Qs, ws1, acc, rt, lane);
        BST_MARK(11);
        const float* W[1] = {P.w1 + q4 * 32 * kBD};
        ws1.start(W, lane);
        // next sample's ids: issued after this phase's last weight prefetch, because vmcnt waits
        // are in issue order and every weight wait behind a gather load would wait for it too
        if (last && has_next) xg.index(a, next, tid);
        store_tile(Ks, acc[0], bb, rt, q4, lane, Xs);
      }
      const LnCols ln1 = ln_load(P.g1, P.be1, tid);
      BST_MARK(16);
      lds_barrier(); BST_PHASE(4);
      layernorm_rows(Ks, ln1, P.eps1, tid, T, nullptr, nullptr);
      lds_barrier(); BST_PHASE(5);

      // ---- 4. f = LeakyReLU(out1 . W1^T + b1) -> Vs
      {
        f32x16 acc[1];
        const float bb = P.b1[c32];
        gemm128<1>(Ks, ws1, acc, rt, lane);
        BST_MARK(12);
        const float* W[1] = {P.w2 + q4 * 32 * kBD};
        ws1.start(W, lane);
        if (last && has_next) xg.rows(a, tid);  // next sample's rows (same ordering argument)
        store_tile(Vs, acc[0], bb, rt, q4, lane, nullptr, P.slope, true);
      }
      BST_MARK(17);
      lds_barrier(); BST_PHASE(6);

      // ---- 5. pre-LN2 = out1 + (f . W2^T + b2) -> Qs;  LN2 in place (+ next block's x + pos)
      {
        f32x16 acc[1];
        const float bb = P.b2[c32];
        gemm128<1>(Vs, ws1, acc, rt, lane);
        BST_MARK(13);
        if (!last || has_next) {
          const float* W[1] = {(last ? a.blk[0].wv : a.blk[blk + 1].wv) + q4 * 32 * kBD};
          ws1.start(W, lane);
        }
        store_tile(Qs, acc[0], bb, rt, q4, lane, Ks);
      }
      const LnCols ln2 = ln_load(P.g2, P.be2, tid);
      BST_MARK(18);
      lds_barrier(); BST_PHASE(7);
      layernorm_rows(Qs, ln2, P.eps2, tid, T, last ? nullptr : Xs, last ? nullptr : a.blk[blk + 1].pos);
      lds_barrier(); BST_PHASE(8);
    }
    // ---- pooling of the last block's rows < T (every real position of the batch, padded ones
    //      included, bst.py:238-241): column c, row quarter g -> red[g][c], then the 4 partials
    {
      const int c = tid & (kBD - 1), g = tid >> 7;
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int t = 0; t < 16; t += 2) {
        const int r = 16 * g + t;
        if (r < T) s0 += Qs[r * kBLD + c];
        if (r + 1 < T) s1 += Qs[(r + 1) * kBLD + c];
      }
      red[g * kBD + c] = s0 + s1;
    }
    lds_barrier();
    if (tid < kBD) {
      float s = (red[tid] + red[kBD + tid]) + (red[2 * kBD + tid] + red[3 * kBD + tid]);
      if (a.pool_mean) s = s / (float)len;
      a.pool_out[b * a.ld_pool + tid] = s;
    }
    if (!has_next) break;
    b = next;
    xg.store(Qs, Xs, T, tid);
    lds_barrier(); BST_PHASE(0);
  }
}

static int bst_forward_blocks(const float* table, int64_t table_rows, int64_t ld_table, const int64_t* seq,
                              int64_t ld_seq, int32_t T, const int64_t* seq_len, int64_t batch, int32_t d_model,
                              int32_t heads, int32_t nblocks, const float* const* block_params,
                              const float* block_scalars, float* pool_out, int64_t ld_pool, int32_t pool_mean,
                              hipStream_t stream, bool packed, const char* what) {
  if (d_model == 16 && !packed)  // the reference script's own width (bst.py:192): bst_small.hip
    return bst_small_forward(table, table_rows, ld_table, seq, ld_seq, T, seq_len, batch, heads, nblocks, block_params,
                             block_scalars, pool_out, ld_pool, pool_mean, stream);
  if (d_model != kBD || heads != 4)
    return fail(RK_ERR_UNSUPPORTED, "%s: d_model=%d heads=%d (fused paths: 128/4%s)", what, d_model, heads,
                packed ? "" : ", 16/1-8");
  if (T <= 0 || T > kBT) return fail(RK_ERR_UNSUPPORTED, "%s: T=%d outside [1, %d]", what, T, kBT);
  if (nblocks <= 0 || nblocks > kBMaxBlocks)
    return fail(RK_ERR_UNSUPPORTED, "%s: %d blocks (max %d)", what, nblocks, kBMaxBlocks);
  if (!table || !seq || !seq_len || !block_params || !block_scalars || !pool_out || ld_table % 4 ||
      ((uintptr_t)table & 15u) || ld_seq < T || ld_pool < kBD || table_rows <= 0)
    return fail(RK_ERR_INVALID, "%s: bad arguments", what);
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
        return fail(RK_ERR_INVALID, "%s: block %d parameter %d null or misaligned", what, i, k);
    w.eps1 = block_scalars[3 * i];
    w.eps2 = block_scalars[3 * i + 1];
    w.slope = block_scalars[3 * i + 2];
  }
  a.pool_out = pool_out;
  a.ld_pool = ld_pool;
  a.pool_mean = pool_mean;
  a.flags = device_flags();
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "%s: negative batch", what);
  const size_t shm = (size_t)(4 * kBT * kBLD + 4 * kBD) * sizeof(float);
  // one resident workgroup per CU (LDS-bound); each walks samples blockIdx.x + k * gridDim.x
  const int64_t grid = std::min<int64_t>(batch, num_cus());
  auto go = [&](auto kern) {
    raise_lds_limit((const void*)kern, 160 * 1024);
    kern<<<(unsigned)grid, 512, shm, stream>>>(a);
  };
  packed ? go(bst_block_kernel<true>) : go(bst_block_kernel<false>);
  return check_launch(what);
}

// [128 n, 128 k] nn.Linear weight -> the WStream<PK = true> order: float 4096 j + 1024 g + 256 c + 4 l + e
// = W[32 j + l % 32][32 g + 8 c + 4 (l / 32) + e]; thread i moves float4 i
__global__ __launch_bounds__(256) void bst_pack_block_weight_kernel(const float* __restrict__ w, float* __restrict__ out) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // < 4096
  const int l = i & 63, c = (i >> 6) & 3, g = (i >> 8) & 3, j = i >> 10;
  const f4 v = *reinterpret_cast<const f4*>(w + (32 * j + (l & 31)) * kBD + 32 * g + 8 * c + 4 * (l >> 5));
  *reinterpret_cast<f4*>(out + 4 * i) = v;
}

}  // namespace rk

using namespace rk;

RK_API int rk_bst_forward_blocks(const float* table, int64_t table_rows, int64_t ld_table, const int64_t* seq,
                                 int64_t ld_seq, int32_t T, const int64_t* seq_len, int64_t batch, int32_t d_model,
                                 int32_t heads, int32_t nblocks, const float* const* block_params,
                                 const float* block_scalars, float* pool_out, int64_t ld_pool, int32_t pool_mean,
                                 void* stream) {
  return bst_forward_blocks(table, table_rows, ld_table, seq, ld_seq, T, seq_len, batch, d_model, heads, nblocks,
                            block_params, block_scalars, pool_out, ld_pool, pool_mean, (hipStream_t)stream, false,
                            "rk_bst_forward_blocks");
}

RK_API int rk_bst_forward_blocks_packed(const float* table, int64_t table_rows, int64_t ld_table, const int64_t* seq,
                                        int64_t ld_seq, int32_t T, const int64_t* seq_len, int64_t batch,
                                        int32_t d_model, int32_t heads, int32_t nblocks,
                                        const float* const* block_params, const float* block_scalars,
                                        float* pool_out, int64_t ld_pool, int32_t pool_mean, void* stream) {
  return bst_forward_blocks(table, table_rows, ld_table, seq, ld_seq, T, seq_len, batch, d_model, heads, nblocks,
                            block_params, block_scalars, pool_out, ld_pool, pool_mean, (hipStream_t)stream, true,
                            "rk_bst_forward_blocks_packed");
}

RK_API int rk_bst_pack_block_weight(const float* w, float* out, void* stream) {
  if (!w || !out || ((uintptr_t)w & 15u) || ((uintptr_t)out & 15u) || w == out)
    return fail(RK_ERR_INVALID, "rk_bst_pack_block_weight: null, misaligned or in-place operands");
  bst_pack_block_weight_kernel<<<16, 256, 0, (hipStream_t)stream>>>(w, out);
  return check_launch("rk_bst_pack_block_weight");
}
