// Tall-skinny GEMM for the training shapes (BST projections and FFN, DIN attention MLP):
//   C[m, n] (+)= epilogue( sum_k opA(m, k) opB(n, k) ),  M large, N any, reduction K <= 128,
//   opA(m, k) = (A[m, k] + Ap[m % period, k]) * [mask(m, k) > 0]   (addend and mask optional)
//   opB(n, k) = b_trans ? B[k, n] : B[n, k]
// Used by rk_linear (Y = X W^T) and rk_gemm without transposed A (dX = dY W) when M spans many
// workgroups.  The generic kernels stage both operands through LDS per 32-deep step with a barrier
// in between and run at 2 waves/SIMD: at M = 131072, N = K = 128 that is 41-52 TFLOP/s.
//
// Here a workgroup stages its 128-column slice of opB ONCE (the whole reduction, [128][K8 + 4] in
// LDS) and then never synchronises again: each wave walks 32-row slabs of A grid-stride, reading
// its A operand straight from global memory into registers (lane = row, float4 along k — the layout
// v_mfma_f32_32x32x2_f32 consumes, no LDS round trip) with the NEXT slab's loads issued before the
// current slab's 4 x K/2 MFMAs, so the HBM stream overlaps the matrix work.  Exact f32 products in a
// k-ordered fma chain per output (permuted k within a chunk, like the other FP32-MFMA kernels).
#include <cstdlib>

#include "common.h"
#include "train_common.h"

namespace rk {

constexpr int kRowsKMax = 128;  // reduction envelope (all of it resident in registers and LDS)
constexpr int kRowsWaves = 4;

struct RowsArgs {
  const float* A;
  int64_t lda;
  const float* A_mask;
  const float* Ap;
  int aperiod;
  const float* B;
  int64_t ldb;
  int b_trans;
  int64_t M;
  int N;
  int K;
  float* C;
  int64_t ldc;
  int accumulate;
  int c_vec;  // C rows 16-B aligned (float4 stores)
  int b_vec;  // B rows 16-B aligned (float4 staging loads)
  rk_epilogue ep;
  // LN epilogue (rk_linear_res_dropout_ln): C = LayerNorm(base + dropout(A B^T + bias)), N = 128
  const float* ln_bias;
  const float* ln_base;
  const float* ln_gamma;
  const float* ln_beta;
  float ln_eps, ln_scale;
  uint32_t ln_thr;
  uint64_t ln_seed;
  const int64_t* ln_slot;
  float* ln_r;
  float* ln_mean;
  float* ln_rstd;
};

// Linear epilogue handled here: bias and ReLU / LeakyReLU (the training layers); anything else
// (residual, affine, Dice, PReLU) stays on linear_kernel.
__device__ __forceinline__ float rows_act(const RowsArgs& a, float z) {
  if (a.ep.act == RK_ACT_RELU) return z < 0.f ? 0.f : z;  // keeps NaN, like torch.relu
  if (a.ep.act == RK_ACT_LEAKY) return z > 0.f ? z : z * a.ep.slope;
  return z;
}

// A-operand modes: plain, ReLU-masked (opA = A [mask > 0]), periodic addend (opA = A + Ap[m % period]).
enum { kRowsPlain = 0, kRowsMask = 1, kRowsPeriodic = 2 };

// A-operand stream of one wave: chunk (slab s, j) is the float4 of row s*32 + (l & 31) at k = 8j + hk
// (hk = 4 (l >> 5)), the layout v_mfma_f32_32x32x2_f32 consumes; rows past M read row M - 1 (their
// outputs are never stored).  A ring of PD chunks runs PD chunks (PD x 4 NT MFMAs) ahead of the
// MFMAs, across slab boundaries, so the HBM stream overlaps the matrix work without a whole
// second slab in registers.
template <int AM>
struct RowsChunk {
  f32x4 x, aux;  // aux: mask (kRowsMask) or periodic addend (kRowsPeriodic)
};

template <int AM>
__device__ __forceinline__ RowsChunk<AM> rows_fetch(const RowsArgs& a, int64_t s, int j, int l32, int hk) {
  const int64_t m = s * 32 + l32;
  const int64_t mr = m < a.M ? m : a.M - 1;
  RowsChunk<AM> c;
  c.x = *reinterpret_cast<const f32x4*>(a.A + mr * a.lda + hk + 8 * j);
  if (AM == kRowsMask) c.aux = *reinterpret_cast<const f32x4*>(a.A_mask + mr * a.lda + hk + 8 * j);
  if (AM == kRowsPeriodic) c.aux = *reinterpret_cast<const f32x4*>(a.Ap + (mr % a.aperiod) * (int64_t)a.K + hk + 8 * j);
  return c;
}

template <int AM>
__device__ __forceinline__ f32x4 rows_operand(const RowsChunk<AM>& c) {
  f32x4 v = c.x;
  if (AM == kRowsPeriodic) v += c.aux;
  if (AM == kRowsMask) {
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = c.aux[e] > 0.f ? v[e] : 0.f;
  }
  return v;
}

// FAST: every tile's columns lie inside N and C rows are 16-B aligned (the host checks N % (32 NT)),
// so the epilogue is straight-line float4 stores; ACC (plain products only): C += the product, the
// slab's C values prefetched at its top.  Both as template flags, the slab loop has no branches on
// them, and the compiler's vmcnt waits in it stay partial (a branch around the C prefetch made it
// wait for every outstanding load and store at the first MFMA of each slab).
// LN (with EPI, FAST, NT = 4, N = 128: a wave's slab holds whole rows, lane l and l + 32 one half
// each): the BST block's residual LayerNorm (bst.py:84-90, rk_bst_res_dropout_ln_forward) fused into
// the projection's epilogue, so the projection output never goes to HBM and back.
#ifdef RK_ROWS_CLOCK  // timing build only (tools/rows_clock.py): shader vs wall clock per workgroup
constexpr int kRowsClkWG = 4096;
__device__ unsigned long long g_rows_clk[kRowsClkWG][4];  // clock64 start/end, wall start/end
#endif

template <int NK8, int NT, bool EPI, int AM, bool FAST = false, bool ACC = false, bool LN = false>
__global__ __launch_bounds__(256, 2) void gemm_rows_kernel(RowsArgs a) {
#ifdef RK_ROWS_CLOCK
  struct ClkMark {
    unsigned long long c0, w0;
    __device__ ~ClkMark() {
      const unsigned wg = blockIdx.x + gridDim.x * blockIdx.y;
      if (threadIdx.x == 0 && wg < kRowsClkWG) {
        g_rows_clk[wg][0] = c0;
        g_rows_clk[wg][1] = clock64();
        g_rows_clk[wg][2] = w0;
        g_rows_clk[wg][3] = wall_clock64();
      }
    }
  } clk_mark{(unsigned long long)clock64(), (unsigned long long)wall_clock64()};
#endif
  static_assert(!LN || (EPI && FAST && NT == 4), "LN epilogue: whole 128-column rows");
  extern __shared__ __attribute__((aligned(16))) float sB[];
  constexpr int K8 = 8 * NK8, ldb = K8 + 4, BN = 32 * NT;
  constexpr int PD = NK8 < 8 ? NK8 : 8;  // ring depth in chunks (divides NK8)
  const int n0 = blockIdx.y * BN;
  const int bn = min(BN, a.N - n0);
  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, hk = 4 * (lane >> 5);
  const int64_t nslabs = (a.M + 31) / 32;
  const int64_t stride = (int64_t)gridDim.x * kRowsWaves;
  int64_t s = (int64_t)blockIdx.x * kRowsWaves + wave;
  RowsChunk<AM> ring[PD];
  // the wave's first PD A chunks, issued right behind the opB staging loads so that their HBM
  // round trip overlaps the staging (rows past M read row M - 1: safe for a wave with no slab)
  auto prefill = [&]() {
#pragma unroll
    for (int j = 0; j < PD; ++j) ring[j] = rows_fetch<AM>(a, s, j, l32, hk);
  };
  // opB slice [bn][K] -> LDS [BN][K8 + 4], zero-padded.  Every thread issues all of its float4
  // loads (coalesced along the contiguous dim) before the first LDS write: a loop of dependent
  // 4-B load -> store pairs put one L2 round trip per element in front of the first MFMA.
  constexpr int NV = BN * K8 / 4 / 256;  // float4 per thread (BN * K8 is a multiple of 1024)
  f32x4 bvals[NV];
  if (a.b_trans) {  // B is [K][N]: float4 = 4 consecutive n at one k
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + 256 * i, k = idx / (BN / 4), n = 4 * (idx % (BN / 4));
      const float* src = a.B + (int64_t)k * a.ldb + n0 + n;
      if (a.b_vec && n + 3 < bn) {
        bvals[i] = *reinterpret_cast<const f32x4*>(src);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) bvals[i][e] = n + e < bn ? src[e] : 0.f;
      }
    }
    prefill();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + 256 * i, k = idx / (BN / 4), n = 4 * (idx % (BN / 4));
#pragma unroll
      for (int e = 0; e < 4; ++e) sB[(n + e) * ldb + k] = bvals[i][e];
    }
  } else {  // B is [N][K]: float4 = 4 consecutive k of one row
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + 256 * i, n = idx / (K8 / 4), k = 4 * (idx % (K8 / 4));
      const float* src = a.B + (int64_t)(n0 + (n < bn ? n : 0)) * a.ldb + k;
      if (a.b_vec) {
        bvals[i] = *reinterpret_cast<const f32x4*>(src);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) bvals[i][e] = src[e];
      }
      if (n >= bn) bvals[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
    prefill();
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int idx = tid + 256 * i, n = idx / (K8 / 4), k = 4 * (idx % (K8 / 4));
      *reinterpret_cast<f32x4*>(sB + n * ldb + k) = bvals[i];
    }
  }
  float* const sLN = sB + BN * ldb;  // LN: bias, gamma, beta [3][128]
  if (LN && tid < 128) {
    sLN[tid] = a.ln_bias ? a.ln_bias[tid] : 0.f;
    sLN[128 + tid] = a.ln_gamma[tid];
    sLN[256 + tid] = a.ln_beta[tid];
  }
  __syncthreads();

  if (s >= nslabs) return;
  const float* bbase = sB + l32 * ldb + hk;
  // Epilogue operands in registers ahead of use: the bias (per column, the same for every slab)
  // once, and for an accumulating product the slab's C values at the top of the slab, so their
  // round trips overlap the MFMAs instead of sitting, one float4 at a time, behind them.
  const bool cvec = FAST || (a.c_vec && n0 + BN <= a.N);
  f32x4 epi[NT][4];
  if (FAST && EPI) {  // absent bias: zeros, so the epilogue adds unconditionally
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) epi[t][q] = (f32x4){0.f, 0.f, 0.f, 0.f};
  }
  // the activation as one negative-side slope (ReLU 0, LeakyReLU slope, none 1): z > 0 ? z : z ns
  // keeps NaN like torch.relu and gives -0 for a negative ReLU input (+0 in torch: equal in use)
  const float neg_slope = a.ep.act == RK_ACT_RELU ? 0.f : a.ep.act == RK_ACT_LEAKY ? a.ep.slope : 1.f;
  const uint64_t ln_stream = LN && a.ln_thr ? (uint64_t)*a.ln_slot : 0;
  if (EPI && !LN && cvec && a.ep.bias) {
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) epi[t][q] = *reinterpret_cast<const f32x4*>(a.ep.bias + n0 + 32 * t + 8 * q + hk);
  }
  // opB fragments one chunk ahead (PIPE): chunk j + 1's LDS reads are issued before chunk j's MFMAs,
  // so their latency hides under the matrix work instead of opening every chunk; the last chunk
  // reads chunk 0's (the same for every slab) for the next slab.  +4 NT registers: not with LN.
  constexpr bool PIPE = !LN;
  f32x4 bnext[NT];
  auto bload = [&](f32x4* dst, int j) {
#pragma unroll
    for (int t = 0; t < NT; ++t) dst[t] = *reinterpret_cast<const f32x4*>(bbase + 32 * t * ldb + 8 * j);
  };
  if (PIPE) bload(bnext, 0);
  // one 32-row slab (the first one peeled off the loop below, so that the loop is entered in the
  // state its back edge leaves: the waitcnt pass then derives its waits from one state)
  auto slab = [&](const int64_t s) {
    const int64_t sn = s + stride < nslabs ? s + stride : s;  // past the end: re-read (unused)
    if (!EPI && (FAST ? ACC : (cvec && a.accumulate))) {
      const int64_t mr = s * 32 + l32 < a.M ? s * 32 + l32 : a.M - 1;
      const float* crow = a.C + mr * a.ldc + n0 + hk;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) epi[t][q] = *reinterpret_cast<const f32x4*>(crow + 32 * t + 8 * q);
    }
    f32x16 acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
#pragma unroll
    for (int j = 0; j < NK8; ++j) {
      if (LN && j == (NK8 > 4 ? NK8 - 4 : 0)) {
        // the residual rows, 4 chunks before the epilogue (prefetched at the slab top they would be
        // live through the whole reduction and push the kernel past its register budget)
        const int64_t mr = s * 32 + l32 < a.M ? s * 32 + l32 : a.M - 1;
        const float* brow = a.ln_base + mr * a.ldc + hk;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int q = 0; q < 4; ++q) epi[t][q] = *reinterpret_cast<const f32x4*>(brow + 32 * t + 8 * q);
      }
      const f32x4 av = rows_operand<AM>(ring[j % PD]);
      // refill the slot with the chunk PD ahead (this slab's j + PD, else the next slab's)
      ring[j % PD] = j + PD < NK8 ? rows_fetch<AM>(a, s, j + PD, l32, hk)
                                  : rows_fetch<AM>(a, sn, j + PD - NK8, l32, hk);
      f32x4 bv[NT];
      if (PIPE) {
#pragma unroll
        for (int t = 0; t < NT; ++t) bv[t] = bnext[t];
        bload(bnext, (j + 1) % NK8);
      } else {
        bload(bv, j);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] = mfma32(bv[t][e], av[e], acc[t]);  // C^T tile: see below
      // keep each chunk's B fragments and refill in their own step: hoisting every step's LDS reads
      // to the top of the unrolled loop (the scheduler's default) needs 4 NT x NK8 registers
      __builtin_amdgcn_sched_barrier(0);
    }
    // The product is formed transposed (opB as the MFMA A operand), so lane l holds row
    // m = 32 s + (l & 31) and, in registers 4q..4q+3 of tile t, the 4 consecutive columns
    // n = 32 t + 8 q + 4 (l >> 5) + 0..3: one float4 store each, 4 NT stores per slab (the waitcnt
    // pass can still count the ring loads across them; 64 scalar stores overflowed its counter).
    const int64_t m = s * 32 + l32;
    if (LN) {
      // lanes l and l + 32 hold row m (64 columns each) and take the branch together
      if (m < a.M) {
        float sum = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = 32 * t + 8 * q + hk;
            const f32x4 b4 = *reinterpret_cast<const f32x4*>(sLN + n);
            f32x4 r;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              float o = acc[t][4 * q + e] + b4[e];
              if (a.ln_thr)
                o = dropout_keep(a.ln_seed, ln_stream, (uint64_t)m * 128 + n + e, a.ln_thr) ? o * a.ln_scale : 0.f;
              r[e] = epi[t][q][e] + o;
              acc[t][4 * q + e] = r[e];
            }
            sum += (r[0] + r[1]) + (r[2] + r[3]);
            *reinterpret_cast<f32x4*>(a.ln_r + m * a.ldc + n) = r;
            __builtin_amdgcn_sched_barrier(0);  // one float4's hashes at a time (register budget)
          }
        sum += __shfl_xor(sum, 32, kWave);
        const float mean = sum * (1.0f / 128.0f);
        float var = 0.f;
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) var += (acc[t][r] - mean) * (acc[t][r] - mean);
        var += __shfl_xor(var, 32, kWave);
        const float rstd = 1.0f / sqrtf(var * (1.0f / 128.0f) + a.ln_eps);
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int n = 32 * t + 8 * q + hk;
            const f32x4 g4 = *reinterpret_cast<const f32x4*>(sLN + 128 + n);
            const f32x4 be4 = *reinterpret_cast<const f32x4*>(sLN + 256 + n);
            f32x4 yv;
#pragma unroll
            for (int e = 0; e < 4; ++e) yv[e] = (acc[t][4 * q + e] - mean) * rstd * g4[e] + be4[e];
            *reinterpret_cast<f32x4*>(a.C + m * a.ldc + n) = yv;
            __builtin_amdgcn_sched_barrier(0);
          }
        if (hk == 0) {
          a.ln_mean[m] = mean;
          a.ln_rstd[m] = rstd;
        }
      }
    } else if (m < a.M) {
      float* crow = a.C + m * a.ldc;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int n = n0 + 32 * t + 8 * q + hk;
          f32x4 z = {acc[t][4 * q], acc[t][4 * q + 1], acc[t][4 * q + 2], acc[t][4 * q + 3]};
          if (FAST) {
            f32x4* c = reinterpret_cast<f32x4*>(crow + n);
            if (EPI) {
              z += epi[t][q];
#pragma unroll
              for (int e = 0; e < 4; ++e) z[e] = z[e] > 0.f ? z[e] : z[e] * neg_slope;
            } else if (ACC) {
              z += epi[t][q];
            }
            *c = z;
          } else if (cvec) {  // epilogue operands already in registers
            f32x4* c = reinterpret_cast<f32x4*>(crow + n);
            if (EPI) {
              if (a.ep.bias) z += epi[t][q];
#pragma unroll
              for (int e = 0; e < 4; ++e) z[e] = rows_act(a, z[e]);
            } else if (a.accumulate) {
              z += epi[t][q];
            }
            *c = z;
          } else if (a.c_vec && n + 3 < a.N) {
            f32x4* c = reinterpret_cast<f32x4*>(crow + n);
            if (EPI) {
              if (a.ep.bias) z += *reinterpret_cast<const f32x4*>(a.ep.bias + n);
#pragma unroll
              for (int e = 0; e < 4; ++e) z[e] = rows_act(a, z[e]);
            } else if (a.accumulate) {
              z += *c;
            }
            *c = z;
          } else {
#pragma unroll
            for (int e = 0; e < 4; ++e)
              if (n + e < a.N) {
                float* c = crow + n + e;
                float v = z[e];
                if (EPI)
                  v = rows_act(a, a.ep.bias ? v + a.ep.bias[n + e] : v);
                else if (a.accumulate)
                  v = *c + v;
                *c = v;
              }
          }
          __builtin_amdgcn_sched_barrier(0);  // one float4 of epilogue loads live at a time
        }
    }
  };
  slab(s);
  for (s += stride; s < nslabs; s += stride) slab(s);
}

static bool rows_aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Host: true (and launched) when the shape suits the kernel; false leaves the call to the caller's
// generic path.  `ep` null: plain product (accumulate honoured); non-null: linear epilogue.
bool gemm_rows_try(const float* A, int64_t lda, const float* A_mask, const float* Ap, int aperiod, const float* B,
                   int64_t ldb, int b_trans, int64_t M, int N, int K, float* C, int64_t ldc, int accumulate,
                   const rk_epilogue* ep, hipStream_t st) {
  // reduction exactly 32, 64 or 128 deep (no k bounds in the load path)
  if ((K != 32 && K != 64 && K != 128) || (lda & 3) || !rows_aligned16(A) || M <= 0) return false;
  if (A_mask && !rows_aligned16(A_mask)) return false;
  if (Ap && (!rows_aligned16(Ap) || aperiod <= 0)) return false;
  const int64_t nslabs = (M + 31) / 32;
  // at least 4 32-row slabs per CU (M >= 32768 on 256 CUs).  N = K = 128, bias+ReLU / accumulate,
  // against the generic kernels: M = 32768 16.6 / 16.3 us vs 21.9 / 30.1, M = 65536 29.3 / 28.0 us
  // vs 59.4 / 59.5; at M = 16384 the two are even, below that the generic path wins.
  if (nslabs < (int64_t)4 * num_cus()) return false;
  RowsArgs a = {};
  a.A = A;
  a.lda = lda;
  a.A_mask = A_mask;
  a.Ap = Ap;
  a.aperiod = aperiod;
  a.B = B;
  a.ldb = ldb;
  a.b_trans = b_trans;
  a.M = M;
  a.N = N;
  a.K = K;
  a.C = C;
  a.ldc = ldc;
  a.accumulate = accumulate;
  if (ep) a.ep = *ep;
  a.c_vec = (ldc % 4 == 0) && rows_aligned16(C);
  a.b_vec = (ldb % 4 == 0) && rows_aligned16(B);
  const int nk8 = K / 8;
  const int nt = N <= 32 ? 1 : N <= 64 ? 2 : 4;       // 32-column accumulator tiles per workgroup
  const int am = A_mask ? kRowsMask : Ap ? kRowsPeriodic : kRowsPlain;
  if (A_mask && Ap) return false;
  if (ep && (ep->residual || ep->pre_scale || ep->post_scale ||
             (ep->act != RK_ACT_NONE && ep->act != RK_ACT_RELU && ep->act != RK_ACT_LEAKY) ||
             (ep->bias && !rows_aligned16(ep->bias))))
    return false;  // linear_kernel's general epilogue
  if (ep && am == kRowsMask) return false;
  const int ntile = (N + 32 * nt - 1) / (32 * nt);
  if (ntile > 65535) return false;
  const size_t shm = sizeof(float) * (size_t)(32 * nt) * (8 * nk8 + 4);
  const int64_t per_tile = std::min<int64_t>((nslabs + kRowsWaves - 1) / kRowsWaves, (int64_t)2 * num_cus());
  dim3 grid((unsigned)std::max<int64_t>(1, per_tile / ntile), (unsigned)ntile);
  bool done = false;
  auto go = [&](void (*kern)(RowsArgs)) {
    raise_lds_limit((const void*)kern, 80 * 1024);  // > 64 KiB at nt 4, K 128
    kern<<<grid, 256, shm, st>>>(a);
    done = true;
  };
  // FAST (straight-line float4 epilogue) when every tile is whole and C rows are 16-B aligned
  const bool fast = a.c_vec && N % (32 * nt) == 0;
#define RK_ROWS_NT(NK, NT)                                                      \
  if (nk8 == NK && nt == NT) {                                                  \
    if (ep) {                                                                   \
      if (am == kRowsPeriodic)                                                  \
        go(gemm_rows_kernel<NK, NT, true, kRowsPeriodic>);                      \
      else if (fast)                                                            \
        go(gemm_rows_kernel<NK, NT, true, kRowsPlain, true>);                   \
      else                                                                      \
        go(gemm_rows_kernel<NK, NT, true, kRowsPlain>);                         \
    } else {                                                                    \
      if (am == kRowsMask)                                                      \
        go(gemm_rows_kernel<NK, NT, false, kRowsMask>);                         \
      else if (am == kRowsPeriodic)                                             \
        go(gemm_rows_kernel<NK, NT, false, kRowsPeriodic>);                     \
      else if (fast && accumulate)                                              \
        go(gemm_rows_kernel<NK, NT, false, kRowsPlain, true, true>);            \
      else if (fast)                                                            \
        go(gemm_rows_kernel<NK, NT, false, kRowsPlain, true, false>);           \
      else                                                                      \
        go(gemm_rows_kernel<NK, NT, false, kRowsPlain>);                        \
    }                                                                           \
  }
  RK_ROWS_NT(4, 1) RK_ROWS_NT(4, 2) RK_ROWS_NT(4, 4)
  RK_ROWS_NT(8, 1) RK_ROWS_NT(8, 2) RK_ROWS_NT(8, 4)
  RK_ROWS_NT(16, 1) RK_ROWS_NT(16, 2) RK_ROWS_NT(16, 4)
#undef RK_ROWS_NT
  if (!done) return false;
  return true;
}


// C = LayerNorm(base + dropout(A W^T + bias)) for whole 128-wide rows (the BST residual LayerNorm
// after the O projection and after FFN2): false when the shape is not the kernel's.
bool gemm_rows_ln_try(const float* A, int64_t lda, const float* W, int64_t ldw, int64_t M, int K, const float* bias,
                      const float* base, uint32_t thr, float scale, uint64_t seed, const int64_t* slot,
                      const float* gamma, const float* beta, float eps, float* r, float* y, float* mean,
                      float* rstd, hipStream_t st) {
  if ((K != 32 && K != 64 && K != 128) || (lda & 3) || (ldw & 3) || M <= 0) return false;
  for (const void* p : {(const void*)A, (const void*)W, (const void*)base, (const void*)r, (const void*)y})
    if (!rows_aligned16(p)) return false;
  const int64_t nslabs = (M + 31) / 32;  // (any M: one launch instead of two pays at every size)
  RowsArgs a = {};
  a.A = A;
  a.lda = lda;
  a.B = W;
  a.ldb = ldw;
  a.M = M;
  a.N = 128;
  a.K = K;
  a.C = y;
  a.ldc = 128;
  a.c_vec = 1;
  a.b_vec = 1;
  a.ln_bias = bias;
  a.ln_base = base;
  a.ln_gamma = gamma;
  a.ln_beta = beta;
  a.ln_eps = eps;
  a.ln_scale = scale;
  a.ln_thr = thr;
  a.ln_seed = seed;
  a.ln_slot = slot;
  a.ln_r = r;
  a.ln_mean = mean;
  a.ln_rstd = rstd;
  const size_t shm = sizeof(float) * ((size_t)128 * (K + 4) + 3 * 128);
  const int64_t per_tile = std::min<int64_t>((nslabs + kRowsWaves - 1) / kRowsWaves, (int64_t)2 * num_cus());
  dim3 grid((unsigned)std::max<int64_t>(1, per_tile), 1);
  auto go = [&](void (*kern)(RowsArgs)) {
    raise_lds_limit((const void*)kern, 80 * 1024);
    kern<<<grid, 256, shm, st>>>(a);
  };
  if (K == 32)
    go(gemm_rows_kernel<4, 4, true, kRowsPlain, true, false, true>);
  else if (K == 64)
    go(gemm_rows_kernel<8, 4, true, kRowsPlain, true, false, true>);
  else
    go(gemm_rows_kernel<16, 4, true, kRowsPlain, true, false, true>);
  return true;
}

}  // namespace rk

using namespace rk;

RK_API int rk_linear_res_dropout_ln(const float* x, int64_t ldx, int64_t M, int32_t K, const float* w, int64_t ldw,
                                    const float* bias, const float* base, double dropout_p, uint64_t seed,
                                    const int64_t* stream_slot, const float* gamma, const float* beta, float eps,
                                    float* r, float* y, float* mean, float* rstd, void* stream) {
  if (!x || !w || !base || !gamma || !beta || !r || !y || !mean || !rstd || M < 0 || K <= 0 ||
      !(dropout_p >= 0.0 && dropout_p < 1.0) || (dropout_p > 0.0 && !stream_slot))
    return fail(RK_ERR_INVALID, "rk_linear_res_dropout_ln: bad arguments");
  if (M == 0) return RK_OK;
  const uint32_t thr = dropout_threshold(dropout_p);
  const float scale = (float)(1.0 / (1.0 - dropout_p));
  if (!gemm_rows_ln_try(x, ldx, w, ldw, M, K, bias, base, thr, scale, seed, stream_slot, gamma, beta, eps, r, y,
                        mean, rstd, (hipStream_t)stream))
    return fail(RK_ERR_UNSUPPORTED,
                "rk_linear_res_dropout_ln: needs K in {32, 64, 128} and 16-B aligned rows");
  return check_launch("rk_linear_res_dropout_ln");
}

#ifdef RK_ROWS_CLOCK
RK_API int rk_debug_rows_clock(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(rk::g_rows_clk), sizeof(rk::g_rows_clk)) == hipSuccess ? 0 : 1;
}
#endif
