// One wide MLP layer as a 2D-tiled GEMM: y[M, n] = epilogue(x[M, K] . W[n, K]^T) for a layer packed
// by rk_mlp_pack_weight, with the element-wise epilogue of mlp_core.h (bias, residual-free
// BatchNorm affine, activation).  Used for the first DeepFM layer (960 -> 512, deepfm.py:100-112):
// in the fused 16-row tail every CU streams the whole 2 MB weight for 16 rows (~500 MB of L2
// traffic per batch); here a workgroup owns a 64-row x 128-column tile, so the weight traffic
// drops 4x at the same 256 workgroups for batch 4096.
//
// 16 waves: wave w owns column tile w%8 (16 columns) for the 32 rows of half w/8 (two 16-row
// MFMA tiles, v_mfma_f32_16x16x4_f32: every weight float4 feeds 8 MFMAs).  The A tile is staged
// through LDS in K-blocks of up to 256 columns, double buffered: the next block's global loads
// are issued into registers before this block's MFMAs and stored after them.  The weight ring
// (4 chunks of 16 k) streams continuously across the block barriers, which are LDS-only.
#include "mlp_core.h"

namespace rk {

constexpr int kLtRows = 64;   // rows per workgroup
constexpr int kLtCols = 128;  // output columns per workgroup (8 tiles of 16)
constexpr int kLtKB = 256;    // K-block staged in LDS
constexpr int kLtLd = kLtKB + 4;

struct LtArgs {
  const float* x;
  int64_t ldx, M;
  int K, Kp;
  rk_mlp_layer L;
  float* y;
  int64_t ldy;
  int x_vec;
};

__global__ __launch_bounds__(kMlpThreads) void linear_tiled_kernel(LtArgs a) {
  extern __shared__ __attribute__((aligned(16))) float lt_sm[];  // [2][kLtRows * kLtLd]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int64_t m0 = (int64_t)blockIdx.x * kLtRows;
  const int n0 = blockIdx.y * kLtCols;
  const int ct = wave & 7, rh = wave >> 3;
  const int n = n0 + 16 * ct + li;  // this lane's weight row / output column
  const rk_mlp_layer& L = a.L;
  const bool col_live = n < pad64(L.n);

  // weight stream of this lane's row over the whole K (ring of 4 chunks)
  const float* wrow = wfrag(L, col_live ? (n >> 4) : 0, lane);
  const int kchunks = a.Kp / 16;
  f32x4_t ring[kMlpPD];
#pragma unroll
  for (int s = 0; s < kMlpPD; ++s) ring[s] = *reinterpret_cast<const f32x4_t*>(wrow + kFragStep * s);
  const ColEpi ep = col_epi(L, n < L.n ? n : 0);

  // A staging: block b covers columns [256 b, min(256 b + 256, Kp)); thread tid moves float4s
  // i = tid + 1024 j of the 64 x 256 block (4 per thread)
  f32x4_t stage[4];
  auto load_block = [&](int b) {
    const int kb = b * kLtKB, w = min(kLtKB, a.Kp - kb);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + kMlpThreads * j;
      const int r = i / (kLtKB / 4), c = (i % (kLtKB / 4)) * 4;
      f32x4_t v = {0.f, 0.f, 0.f, 0.f};
      const int64_t m = m0 + r;
      if (c < w && m < a.M) {
        const int k = kb + c;
        if (a.x_vec) {
          if (k < a.K) v = *reinterpret_cast<const f32x4_t*>(a.x + m * a.ldx + k);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = k + e < a.K ? a.x[m * a.ldx + k + e] : 0.f;
        }
      }
      stage[j] = v;
    }
  };
  auto store_block = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + kMlpThreads * j;
      const int r = i / (kLtKB / 4), c = (i % (kLtKB / 4)) * 4;
      *reinterpret_cast<f32x4_t*>(lt_sm + buf * kLtRows * kLtLd + r * kLtLd + c) = stage[j];
    }
  };

  const int nblocks = (a.Kp + kLtKB - 1) / kLtKB;
  load_block(0);
  store_block(0);
  mlp_lds_barrier();

  f32x4_t acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  int c = 0;  // global chunk index of the weight stream
  for (int b = 0; b < nblocks; ++b) {
    const int buf = b & 1;
    if (b + 1 < nblocks) load_block(b + 1);
    const int bchunks = min(kLtKB, a.Kp - b * kLtKB) / 16;
    const float* arow = lt_sm + buf * kLtRows * kLtLd + (32 * rh + li) * kLtLd + kq;
    f32x4_t an[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) an[t] = *reinterpret_cast<const f32x4_t*>(arow + 16 * t * kLtLd);
    for (int q0 = 0; q0 < bchunks; q0 += kMlpPD) {
#pragma unroll
      for (int s = 0; s < kMlpPD; ++s) {
        const int q = q0 + s;
        f32x4_t av[2] = {an[0], an[1]};
        const int qa = min(q + 1, bchunks - 1);
#pragma unroll
        for (int t = 0; t < 2; ++t) an[t] = *reinterpret_cast<const f32x4_t*>(arow + 16 * t * kLtLd + 16 * qa);
        const f32x4_t bv = ring[s];  // c is a multiple of kMlpPD
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int t = 0; t < 2; ++t) acc[t] = mfma16(av[t][e], bv[e], acc[t]);
        const int cn = min(c + s + kMlpPD, kchunks - 1);
        ring[s] = *reinterpret_cast<const f32x4_t*>(wrow + kFragStep * cn);
        __builtin_amdgcn_sched_barrier(0);
      }
      c += kMlpPD;
    }
    if (b + 1 < nblocks) {
      store_block(buf ^ 1);
      mlp_lds_barrier();
    }
  }

  // epilogue: bias, BatchNorm affine, activation; rows < M, columns < n
  if (n < L.n) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + 32 * rh + 16 * t + 4 * (lane >> 4) + r;
        if (m < a.M) a.y[m * a.ldy + n] = col_apply(ep, L.act == RK_ACT_DICE, acc[t][r], false, 0.f);
      }
  }
}

}  // namespace rk

using namespace rk;

RK_API int rk_linear_tiled(const float* x, int64_t ldx, int64_t M, int32_t K, const rk_mlp_layer* layer, float* y,
                           int64_t ldy, void* stream) {
  if (!x || !layer || !y || M < 0 || K <= 0 || ldx < K)
    return fail(RK_ERR_INVALID, "rk_linear_tiled: bad arguments (M=%lld K=%d)", (long long)M, K);
  const rk_mlp_layer& L = *layer;
  if (!L.w || L.n <= 0 || L.ldw != pad64(K) || ((uintptr_t)L.w & 15u))
    return fail(RK_ERR_UNSUPPORTED, "rk_linear_tiled: the weight must be packed by rk_mlp_pack_weight (ldw %lld, K %d)",
                (long long)L.ldw, K);
  if (L.residual) return fail(RK_ERR_UNSUPPORTED, "rk_linear_tiled: residual layers are not supported");
  if (L.act == RK_ACT_DICE && (!L.act_scale || !L.act_shift || !L.act_alpha))
    return fail(RK_ERR_INVALID, "rk_linear_tiled: Dice layer incomplete");
  if (L.act == RK_ACT_PRELU && !L.act_alpha) return fail(RK_ERR_INVALID, "rk_linear_tiled: PReLU needs alpha");
  if ((L.pre_scale != nullptr) != (L.pre_shift != nullptr) || (L.post_scale != nullptr) != (L.post_shift != nullptr))
    return fail(RK_ERR_INVALID, "rk_linear_tiled: affine scale/shift must come in pairs");
  if (ldy < L.n) return fail(RK_ERR_INVALID, "rk_linear_tiled: ldy %lld < n %d", (long long)ldy, L.n);
  if (M == 0) return RK_OK;
  LtArgs a = {};
  a.x = x;
  a.ldx = ldx;
  a.M = M;
  a.K = K;
  a.Kp = pad64(K);
  a.L = L;
  a.y = y;
  a.ldy = ldy;
  a.x_vec = (ldx % 4 == 0) && (((uintptr_t)x & 15u) == 0);
  const dim3 grid((unsigned)((M + kLtRows - 1) / kLtRows), (unsigned)((pad64(L.n) + kLtCols - 1) / kLtCols));
  const size_t shm = 2 * kLtRows * kLtLd * sizeof(float);
  raise_lds_limit((const void*)linear_tiled_kernel, (int)shm);
  linear_tiled_kernel<<<grid, kMlpThreads, shm, (hipStream_t)stream>>>(a);
  return check_launch("rk_linear_tiled");
}
