// Fused MLP tail: every hidden layer and the final Linear(N,1)+sigmoid head in one launch.
//
// A workgroup (16 waves, 4 per SIMD) owns 16 rows.  The input tile [16 x K0] is staged in LDS
// once; each layer reads its input from one LDS buffer and writes its activated output to the
// other, so activations never touch HBM.  Layer math is FP32 MFMA v_mfma_f32_16x16x4_f32 (exact
// f32): wave w owns output tiles w and w+16 (16 columns each).  Per 16-deep K chunk a lane reads
// one float4 of its A row from LDS (k = 16c + 4*(lane>>4) + e) and one float4 of its weight row
// per tile from global memory, then issues 4 MFMAs per tile.  Weights are pre-packed
// (rk_mlp_pack_weight: rows padded to 64 columns, K padded to 64, zero fill), so every weight
// load is an unconditional aligned float4 and the chunk count is a multiple of the 4-deep
// register prefetch ring; weights stay L2-resident across the workgroups.  Epilogues (bias,
// BatchNorm folded to scale/shift, ReLU / LeakyReLU / Dice / PReLU, residual) run on the
// accumulators before the LDS write.
//
// Reference tails covered: dcn.py:144-152,175-180; deepfm.py:100-112,143-151;
// din.py:272-285,312-316; bst.py:203-214,245-247; deepcrossing.py:25-42,157-162.
#include "common.h"

namespace rk {

constexpr int kMlpRows = 16;
constexpr int kMlpWaves = 16;
constexpr int kMlpThreads = 64 * kMlpWaves;
constexpr int kMlpPD = 4;     // prefetch depth (chunks)
constexpr int kMlpPad = 64;   // K and N padding of packed weights
constexpr int kMlpMaxN = 512;

typedef float f32x4_t __attribute__((ext_vector_type(4)));

struct MlpArgs {
  rk_mlp_layer L[RK_MLP_MAX_LAYERS];
  int nl;
  rk_epilogue head;
  const float* x;
  int64_t ldx;
  int64_t M;
  int K0;
  int x_vec;
  float* y;
  int64_t ldy;
  int ld0, ld1;  // LDS row strides of the two activation buffers (floats)
  int off1;      // float offset of buffer 1
};

__host__ __device__ constexpr int pad64(int v) { return (v + kMlpPad - 1) / kMlpPad * kMlpPad; }

__device__ __forceinline__ f32x4_t mfma16(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float layer_act(const rk_mlp_layer& L, float z, int n) {
  switch (L.act) {
    case RK_ACT_RELU:
      return z < 0.f ? 0.f : z;
    case RK_ACT_LEAKY:
      return z > 0.f ? z : z * L.slope;
    case RK_ACT_DICE: {
      const float xn = z * L.act_scale[n] + L.act_shift[n];
      const float p = 1.0f / (1.0f + expf(-xn));
      return L.act_alpha[n] * (1.0f - p) * z + p * z;
    }
    case RK_ACT_PRELU: {
      const float a = L.act_alpha[L.act_alpha_len == 1 ? 0 : n];
      return z > 0.f ? z : a * z;
    }
    default:
      return z;
  }
}

// One layer for a wave owning TPW tiles (t = wave + 16*j).
template <int TPW>
__device__ __forceinline__ void mlp_layer(const rk_mlp_layer& L, const float* __restrict__ in, int ldin,
                                          float* __restrict__ out, int ldout, int Kp, int wave, int lane) {
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int kchunks = Kp / 16;  // multiple of kMlpPD
  const int64_t ldw = L.ldw;
  const float* wrow[TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) wrow[j] = L.w + (int64_t)(16 * (wave + kMlpWaves * j) + li) * ldw + kq;

  f32x4_t acc[TPW];
  f32x4_t ring[kMlpPD][TPW];
#pragma unroll
  for (int j = 0; j < TPW; ++j) acc[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < kMlpPD; ++s)
#pragma unroll
    for (int j = 0; j < TPW; ++j) ring[s][j] = *reinterpret_cast<const f32x4_t*>(wrow[j] + 16 * s);

  const float* arow = in + li * ldin + kq;
  for (int c0 = 0; c0 < kchunks; c0 += kMlpPD) {
#pragma unroll
    for (int s = 0; s < kMlpPD; ++s) {
      const int c = c0 + s;
      const f32x4_t av = *reinterpret_cast<const f32x4_t*>(arow + 16 * c);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int j = 0; j < TPW; ++j) acc[j] = mfma16(av[e], ring[s][j][e], acc[j]);
      // refill this slot with chunk c + PD (clamped: the tail re-reads the last chunk, unused)
      const int cn = min(c + kMlpPD, kchunks - 1);
#pragma unroll
      for (int j = 0; j < TPW; ++j) ring[s][j] = *reinterpret_cast<const f32x4_t*>(wrow[j] + 16 * cn);
      // keep the refill here: sinking it to the end of the unrolled body would leave each
      // slot's latency uncovered by the other slots' MFMAs
      __builtin_amdgcn_sched_barrier(0);
    }
  }

#pragma unroll
  for (int j = 0; j < TPW; ++j) {
    const int n = 16 * (wave + kMlpWaves * j) + li;
    const bool real = n < L.n;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = (lane >> 4) * 4 + r;
      float z = 0.f;
      if (real) {
        z = acc[j][r];
        if (L.bias) z += L.bias[n];
        // x + f(x): the previous layer's input still sits in `out` (read-then-write, same lane)
        if (L.residual) z = out[row * ldout + n] + z;
        if (L.pre_scale) z = z * L.pre_scale[n] + L.pre_shift[n];
        z = layer_act(L, z, n);
        if (L.post_scale) z = z * L.post_scale[n] + L.post_shift[n];
      }
      out[row * ldout + n] = z;  // padded columns [n, Np) become the next layer's zero K pad
    }
  }
}

__global__ __launch_bounds__(kMlpThreads) void mlp_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * kMlpRows;
  const int rows = (int)min<int64_t>(kMlpRows, a.M - m0);

  float* const buf0 = sm;
  float* const buf1 = sm + a.off1;
  const int ldb[2] = {a.ld0, a.ld1};

  // ---- stage the input tile, zero-padded to a multiple of 64 columns
  const int K0p = pad64(a.K0);
  if (a.x_vec) {
    const int q = K0p / 4;
    for (int i = tid; i < kMlpRows * q; i += kMlpThreads) {
      const int r = i / q, c = (i % q) * 4;
      f32x4_t v = {0.f, 0.f, 0.f, 0.f};
      if (r < rows && c < a.K0) v = *reinterpret_cast<const f32x4_t*>(a.x + (m0 + r) * a.ldx + c);
      *reinterpret_cast<f32x4_t*>(buf0 + r * a.ld0 + c) = v;
    }
  } else {
    for (int i = tid; i < kMlpRows * K0p; i += kMlpThreads) {
      const int r = i / K0p, c = i % K0p;
      buf0[r * a.ld0 + c] = (r < rows && c < a.K0) ? a.x[(m0 + r) * a.ldx + c] : 0.f;
    }
  }
  __syncthreads();

  int Kp = K0p;
  for (int l = 0; l < a.nl; ++l) {
    const rk_mlp_layer& L = a.L[l];
    const int ntiles = pad64(L.n) / 16;  // multiple of 4
    const float* in = (l & 1) ? buf1 : buf0;
    float* out = (l & 1) ? buf0 : buf1;
    if (wave + kMlpWaves < ntiles) {
      mlp_layer<2>(L, in, ldb[l & 1], out, ldb[(l + 1) & 1], Kp, wave, lane);
    } else if (wave < ntiles) {
      mlp_layer<1>(L, in, ldb[l & 1], out, ldb[(l + 1) & 1], Kp, wave, lane);
    }
    __syncthreads();
    Kp = pad64(L.n);
  }

  // ---- head (one wave per row) or plain output
  const float* fin = (a.nl & 1) ? buf1 : buf0;
  const int ldf = ldb[a.nl & 1];
  const int K = a.nl ? a.L[a.nl - 1].n : a.K0;
  const rk_epilogue& h = a.head;
  if (h.head_w) {
    if (wave < rows) {
      const int r = wave;
      float p = 0.f;
      for (int n = lane; n < K; n += 64) p = fmaf(fin[r * ldf + n], h.head_w[n], p);
      p = wave_sum(p);
      if (lane == 0) {
        const int64_t m = m0 + r;
        float logit = p + h.head_b[0];
        if (h.head_partial) logit = h.head_partial[m] + logit;
        if (h.fm1) {
          if (h.head_aux) h.head_aux[m] = logit;
          logit = h.fm1[m] * h.final_w[0] + h.fm2[m] * h.final_w[1] + logit * h.final_w[2] + h.final_b[0];
        }
        if (h.head_logit) h.head_logit[m] = logit;
        if (h.head_prob) h.head_prob[m] = 1.0f / (1.0f + expf(-logit));
      }
    }
  } else if (a.y) {
    for (int i = tid; i < rows * K; i += kMlpThreads) {
      const int r = i / K, n = i % K;
      a.y[(m0 + r) * a.ldy + n] = fin[r * ldf + n];
    }
  }
}

__global__ void mlp_pack_kernel(const float* __restrict__ w, int64_t ldw, int n, int k, int np, int kp,
                                float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)np * kp) return;
  const int r = (int)(i / kp), c = (int)(i % kp);
  out[i] = (r < n && c < k) ? w[(int64_t)r * ldw + c] : 0.f;
}

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace rk

using namespace rk;

RK_API int rk_mlp_packed_size(int32_t n, int32_t k, int64_t* rows, int64_t* cols) {
  if (n <= 0 || k <= 0 || !rows || !cols) return fail(RK_ERR_INVALID, "rk_mlp_packed_size: bad arguments");
  *rows = pad64(n);
  *cols = pad64(k);
  return RK_OK;
}

RK_API int rk_mlp_pack_weight(const float* w, int64_t ldw, int32_t n, int32_t k, float* out, void* stream) {
  if (!w || !out || n <= 0 || k <= 0 || ldw < k) return fail(RK_ERR_INVALID, "rk_mlp_pack_weight: bad arguments");
  const int np = pad64(n), kp = pad64(k);
  const int64_t total = (int64_t)np * kp;
  mlp_pack_kernel<<<(unsigned)((total + 255) / 256), 256, 0, (hipStream_t)stream>>>(w, ldw, n, k, np, kp, out);
  return check_launch("rk_mlp_pack_weight");
}

RK_API int rk_mlp_forward(const float* x, int64_t ldx, int64_t M, int32_t K0, const rk_mlp_layer* layers,
                          int32_t nlayers, const rk_epilogue* head, float* y, int64_t ldy, void* stream) {
  if (!x || M < 0 || K0 <= 0 || ldx < K0 || nlayers < 0 || nlayers > RK_MLP_MAX_LAYERS || (nlayers && !layers))
    return fail(RK_ERR_INVALID, "rk_mlp_forward: bad arguments (M=%lld K0=%d layers=%d)", (long long)M, K0, nlayers);
  MlpArgs a = {};
  a.nl = nlayers;
  if (head) a.head = *head;
  if (!a.head.head_w && !y) return fail(RK_ERR_INVALID, "rk_mlp_forward: need a head or an output");
  if (a.head.head_w && !a.head.head_b) return fail(RK_ERR_INVALID, "rk_mlp_forward: head needs head_b");
  if (a.head.fm1 && (!a.head.fm2 || !a.head.final_w || !a.head.final_b))
    return fail(RK_ERR_INVALID, "rk_mlp_forward: FM combine incomplete");
  if (pad64(K0) > 1024) return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward: input width %d > 1024", K0);
  int K = K0;
  int need0 = pad64(K0), need1 = kMlpPad;
  for (int l = 0; l < nlayers; ++l) {
    const rk_mlp_layer& L = layers[l];
    if (!L.w || L.n <= 0 || L.n > kMlpMaxN || L.ldw != pad64(K) || !aligned16(L.w))
      return fail(RK_ERR_UNSUPPORTED,
                  "rk_mlp_forward: layer %d (n=%d, ldw=%lld, K=%d) must be packed by rk_mlp_pack_weight, n <= %d", l,
                  L.n, (long long)L.ldw, K, kMlpMaxN);
    if (L.act == RK_ACT_DICE && (!L.act_scale || !L.act_shift || !L.act_alpha))
      return fail(RK_ERR_INVALID, "rk_mlp_forward: Dice layer %d incomplete", l);
    if (L.act == RK_ACT_PRELU && !L.act_alpha) return fail(RK_ERR_INVALID, "rk_mlp_forward: PReLU needs alpha");
    if ((L.pre_scale != nullptr) != (L.pre_shift != nullptr) || (L.post_scale != nullptr) != (L.post_shift != nullptr))
      return fail(RK_ERR_INVALID, "rk_mlp_forward: affine scale/shift must come in pairs");
    if (L.residual && (l == 0 || L.n != (l >= 2 ? layers[l - 2].n : K0)))
      return fail(RK_ERR_INVALID, "rk_mlp_forward: residual layer %d must map back to the width of layer %d's input",
                  l, l - 1);
    a.L[l] = L;
    if ((l + 1) & 1)
      need1 = std::max(need1, pad64(L.n));
    else
      need0 = std::max(need0, pad64(L.n));
    K = L.n;
  }
  // row stride = width + 4 (width is a multiple of 64): conflict-free float4 row reads
  a.ld0 = need0 + 4;
  a.ld1 = need1 + 4;
  a.off1 = kMlpRows * a.ld0;
  const size_t shm = (size_t)kMlpRows * (a.ld0 + a.ld1) * sizeof(float);
  if (shm > 160 * 1024) return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward: widths need %zu B of LDS", shm);
  a.x = x;
  a.ldx = ldx;
  a.M = M;
  a.K0 = K0;
  a.x_vec = (ldx % 4 == 0) && aligned16(x) && (K0 % 4 == 0);
  a.y = y;
  a.ldy = ldy;
  if (M == 0) return RK_OK;
  const int64_t blocks = (M + kMlpRows - 1) / kMlpRows;
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward: M too large");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)mlp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  mlp_kernel<<<(unsigned)blocks, kMlpThreads, shm, (hipStream_t)stream>>>(a);
  return check_launch("rk_mlp_forward");
}
