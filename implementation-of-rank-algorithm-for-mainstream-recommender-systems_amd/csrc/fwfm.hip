// Field-weighted FM forward: FwFM.forward, algorithm/FwFM/fwfm.py:114-139.
//
//   y[b] = sum_f linear_f[idx_f[b]] + sum_{i<j} r_p <E_i[idx_i[b]], E_j[idx_j[b]]> + bias
//   prob[b] = sigmoid(y[b])
// with the pair index p running i-major over i < j (fwfm.py:129-136).
//
// One sample is owned by G lanes; lane q holds VEC consecutive embedding columns
// [q*VEC, q*VEC+VEC) of every field (VEC = 4: one 16-byte load per field and lane; VEC = 1 for
// embedding widths that are not a multiple of 4).  All index loads of a lane are issued first,
// then all row loads, so each lane keeps F row fetches in flight; the F(F-1)/2 pair dots are
// register-only, reduced over the G lanes with cross-lane shuffles.  HBM bytes per sample:
// F x (8 index + 4 dim embedding + 4 linear) + 4 (prob) [+ 4 logit]; the tables (wechat: 188k
// rows x 36 B = 6.8 MB) stay resident in L2 / MALL, so the kernel is latency-bound at small
// batches and index/row-gather bound at large ones.
#include "common.h"

namespace rk {

constexpr int kFwfmMaxFields = 16;

struct FwfmTables {
  rk_segment emb[kFwfmMaxFields];
  rk_segment lin[kFwfmMaxFields];
};

template <int VEC>
struct VecT;
template <>
struct VecT<4> {
  using T = f32x4;
  __device__ static T zero() { return (f32x4){0.f, 0.f, 0.f, 0.f}; }
  __device__ static float dot(const T& a, const T& b) { return a.x * b.x + a.y * b.y + a.z * b.z + a.w * b.w; }
};
template <>
struct VecT<1> {
  using T = float;
  __device__ static T zero() { return 0.f; }
  __device__ static float dot(float a, float b) { return a * b; }
};

template <int G, int VEC>
__global__ __launch_bounds__(64) void fwfm_forward_kernel(FwfmTables t, int F, int dim, int64_t batch,
                                                          const float* __restrict__ field_weight,
                                                          const float* __restrict__ bias, float* __restrict__ logit,
                                                          float* __restrict__ prob, uint32_t* flags) {
  using V = VecT<VEC>;
  using T = typename V::T;
  constexpr int SPW = 64 / G;  // samples per wave
  const int lane = threadIdx.x;
  const int q = lane % G;
  const int64_t b = (int64_t)blockIdx.x * SPW + lane / G;
  const bool live = b < batch;
  const int col = q * VEC;
  const bool has_cols = col < dim;
  const float* rp[kFwfmMaxFields];
  const float* wp[kFwfmMaxFields];
#pragma unroll
  for (int f = 0; f < kFwfmMaxFields; ++f) {
    rp[f] = nullptr;
    wp[f] = nullptr;
    if (f < F && live) {
      const float* r = segment_row(t.emb[f], b, flags);
      rp[f] = has_cols && r ? r + col : nullptr;
      wp[f] = q == 0 ? segment_row(t.lin[f], b, flags) : nullptr;
    }
  }
  T v[kFwfmMaxFields];
  float lin = 0.f;
#pragma unroll
  for (int f = 0; f < kFwfmMaxFields; ++f) {
    v[f] = rp[f] ? *reinterpret_cast<const T*>(rp[f]) : V::zero();
    if (wp[f]) lin += wp[f][0];
  }
  float quad = 0.f;
  int p = 0;
#pragma unroll
  for (int i = 0; i < kFwfmMaxFields; ++i) {
    if (i >= F) break;
#pragma unroll
    for (int j = i + 1; j < kFwfmMaxFields; ++j) {
      if (j >= F) break;
      quad += field_weight[p++] * V::dot(v[i], v[j]);
    }
  }
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) quad += __shfl_xor(quad, o, kWave);
  if (live && q == 0) {
    const float y = lin + quad + bias[0];
    if (logit) logit[b] = y;
    prob[b] = sigmoidf_ref(y);
  }
}

// FwFM backward (training) from dL/dprob (the script's BCELoss on the
// probabilities, fwfm.py:150-156, 245):  dz = dprob * (1 - prob) * prob (torch's sigmoid backward),
//   d_emb[b, i*dim + c] = dz * sum_{j != i} r_{p(i,j)} E_j[c]      (the embedding-row gradients)
//   d_r[p] += dz * <E_i, E_j>,  d_bias += dz,  dz_out[b] = dz      (the linear-table gradient rows)
// Same lane layout as the forward; 4 waves per workgroup, the d_r / d_bias partials are summed in
// LDS and flushed with one float atomic per pair and workgroup.
constexpr int kFwfmMaxPairs = kFwfmMaxFields * (kFwfmMaxFields - 1) / 2;

template <int G, int VEC>
__global__ __launch_bounds__(256) void fwfm_backward_kernel(FwfmTables t, int F, int dim, int64_t batch,
                                                            const float* __restrict__ field_weight,
                                                            const float* __restrict__ prob,
                                                            const float* __restrict__ dprob, float* __restrict__ d_emb,
                                                            int64_t ld_demb, float* __restrict__ dz_out,
                                                            float* __restrict__ d_field_weight,
                                                            float* __restrict__ d_bias, uint32_t* flags) {
  using V = VecT<VEC>;
  using T = typename V::T;
  constexpr int SPW = 64 / G;
  __shared__ float red[kFwfmMaxPairs + 1];
  const int P = F * (F - 1) / 2;
  for (int i = threadIdx.x; i <= P; i += blockDim.x) red[i] = 0.f;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane % G;
  const int64_t b = ((int64_t)blockIdx.x * 4 + wave) * SPW + lane / G;
  const bool live = b < batch;
  const int col = q * VEC;
  const bool has_cols = col < dim;
  const float* rp[kFwfmMaxFields];
#pragma unroll
  for (int f = 0; f < kFwfmMaxFields; ++f) {
    rp[f] = nullptr;
    if (f < F && live) {
      const float* r = segment_row(t.emb[f], b, flags);
      rp[f] = has_cols && r ? r + col : nullptr;
    }
  }
  T v[kFwfmMaxFields];
#pragma unroll
  for (int f = 0; f < kFwfmMaxFields; ++f) v[f] = rp[f] ? *reinterpret_cast<const T*>(rp[f]) : V::zero();
  const float y = live ? prob[b] : 0.f;
  const float dz = live ? dprob[b] * (1.0f - y) * y : 0.f;
  // embedding-row gradients
#pragma unroll
  for (int i = 0; i < kFwfmMaxFields; ++i) {
    if (i >= F) break;
    T acc = V::zero();
#pragma unroll
    for (int j = 0; j < kFwfmMaxFields; ++j) {
      if (j >= F) break;
      if (j == i) continue;
      const int a = i < j ? i : j, c = i < j ? j : i;
      const int p = a * F - a * (a + 1) / 2 + (c - a - 1);  // i-major pair index of (a, c)
      acc = acc + field_weight[p] * v[j];
    }
    if (live && has_cols) *reinterpret_cast<T*>(d_emb + b * ld_demb + (int64_t)i * dim + col) = dz * acc;
  }
  // pair-weight and bias gradients
  int p = 0;
#pragma unroll
  for (int i = 0; i < kFwfmMaxFields; ++i) {
    if (i >= F) break;
#pragma unroll
    for (int j = i + 1; j < kFwfmMaxFields; ++j) {
      if (j >= F) break;
      float s = V::dot(v[i], v[j]);
#pragma unroll
      for (int o = G / 2; o > 0; o >>= 1) s += __shfl_xor(s, o, kWave);
      if (live && q == 0) atomicAdd(&red[p], dz * s);
      ++p;
    }
  }
  if (live && q == 0) {
    atomicAdd(&red[P], dz);
    dz_out[b] = dz;
  }
  __syncthreads();
  for (int i = threadIdx.x; i <= P; i += blockDim.x) atomicAdd(i < P ? d_field_weight + i : d_bias, red[i]);
}


}  // namespace rk

using namespace rk;

RK_API int rk_fwfm_forward(const rk_segment* embeddings, const rk_segment* linear, int32_t num_fields, int32_t dim,
                           int64_t batch, const float* field_weight, const float* bias, float* logit, float* prob,
                           void* stream) {
  if (num_fields < 2 || num_fields > kFwfmMaxFields)
    return fail(RK_ERR_UNSUPPORTED, "rk_fwfm_forward: %d fields (supported 2..%d)", num_fields, kFwfmMaxFields);
  if (!embeddings || !linear || !field_weight || !bias || !prob)
    return fail(RK_ERR_INVALID, "rk_fwfm_forward: null argument");
  if (dim <= 0 || dim > 256) return fail(RK_ERR_UNSUPPORTED, "rk_fwfm_forward: dim %d (supported 1..256)", dim);
  bool vec4 = dim % 4 == 0;
  FwfmTables t;
  for (int f = 0; f < num_fields; ++f) {
    const rk_segment &e = embeddings[f], &l = linear[f];
    if (!e.src || !e.idx || e.rows <= 0 || e.dim != dim || !l.src || !l.idx || l.rows <= 0 || l.dim != 1)
      return fail(RK_ERR_INVALID, "rk_fwfm_forward: field %d tables invalid (embedding dim %d, linear dim %d)", f,
                  e.dim, l.dim);
    vec4 = vec4 && aligned16(e.src) && e.src_ld % 4 == 0;
    t.emb[f] = e;
    t.lin[f] = l;
  }
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "rk_fwfm_forward: negative batch");
  const int vec = vec4 ? 4 : 1;
  int G = 1;
  while (G * vec < dim) G <<= 1;
  if (G > 64) return fail(RK_ERR_UNSUPPORTED, "rk_fwfm_forward: dim %d needs 16-byte aligned rows", dim);
  const int64_t blocks = (batch + 64 / G - 1) / (64 / G);
  hipStream_t st = (hipStream_t)stream;
  uint32_t* fl = device_flags();
#define RK_FWFM_CASE(GG, VV)                                                                                 \
  if (G == GG && vec == VV) {                                                                                \
    fwfm_forward_kernel<GG, VV><<<(unsigned)blocks, 64, 0, st>>>(t, num_fields, dim, batch, field_weight, bias, \
                                                                 logit, prob, fl);                          \
    return check_launch("rk_fwfm_forward");                                                                  \
  }
  RK_FWFM_CASE(1, 4)
  RK_FWFM_CASE(2, 4)
  RK_FWFM_CASE(4, 4)
  RK_FWFM_CASE(8, 4)
  RK_FWFM_CASE(16, 4)
  RK_FWFM_CASE(32, 4)
  RK_FWFM_CASE(64, 4)
  RK_FWFM_CASE(1, 1)
  RK_FWFM_CASE(2, 1)
  RK_FWFM_CASE(4, 1)
  RK_FWFM_CASE(8, 1)
  RK_FWFM_CASE(16, 1)
  RK_FWFM_CASE(32, 1)
  RK_FWFM_CASE(64, 1)
#undef RK_FWFM_CASE
  return fail(RK_ERR_UNSUPPORTED, "rk_fwfm_forward: dim %d", dim);
}

RK_API int rk_fwfm_backward(const rk_segment* embeddings, int32_t num_fields, int32_t dim, int64_t batch,
                            const float* field_weight, const float* prob, const float* dprob, float* d_emb,
                            int64_t ld_demb, float* dz, float* d_field_weight, float* d_bias, void* stream) {
  if (num_fields < 2 || num_fields > kFwfmMaxFields)
    return fail(RK_ERR_UNSUPPORTED, "rk_fwfm_backward: %d fields (supported 2..%d)", num_fields, kFwfmMaxFields);
  if (!embeddings || !field_weight || !prob || !dprob || !d_emb || !dz || !d_field_weight || !d_bias ||
      ld_demb < (int64_t)num_fields * dim)
    return fail(RK_ERR_INVALID, "rk_fwfm_backward: bad arguments");
  if (dim <= 0 || dim > 256) return fail(RK_ERR_UNSUPPORTED, "rk_fwfm_backward: dim %d (supported 1..256)", dim);
  bool vec4 = dim % 4 == 0 && aligned16(d_emb) && ld_demb % 4 == 0;
  FwfmTables t;
  for (int f = 0; f < num_fields; ++f) {
    const rk_segment& e = embeddings[f];
    if (!e.src || !e.idx || e.rows <= 0 || e.dim != dim)
      return fail(RK_ERR_INVALID, "rk_fwfm_backward: field %d table invalid", f);
    vec4 = vec4 && aligned16(e.src) && e.src_ld % 4 == 0;
    t.emb[f] = e;
  }
  hipStream_t st = (hipStream_t)stream;
  const int P = num_fields * (num_fields - 1) / 2;
  if (hipMemsetAsync(d_field_weight, 0, (size_t)P * sizeof(float), st) != hipSuccess ||
      hipMemsetAsync(d_bias, 0, sizeof(float), st) != hipSuccess)
    return fail(RK_ERR_RUNTIME, "rk_fwfm_backward: memset failed");
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "rk_fwfm_backward: negative batch");
  const int vec = vec4 ? 4 : 1;
  int G = 1;
  while (G * vec < dim) G <<= 1;
  if (G > 64) return fail(RK_ERR_UNSUPPORTED, "rk_fwfm_backward: dim %d needs 16-byte aligned rows", dim);
  const int64_t per_block = 4 * (64 / G);
  const int64_t blocks = (batch + per_block - 1) / per_block;
  uint32_t* fl = device_flags();
#define RK_FWFM_CASE(GG, VV)                                                                                   \
  if (G == GG && vec == VV) {                                                                                  \
    fwfm_backward_kernel<GG, VV><<<(unsigned)blocks, 256, 0, st>>>(t, num_fields, dim, batch, field_weight, prob, \
                                                                   dprob, d_emb, ld_demb, dz, d_field_weight,   \
                                                                   d_bias, fl);                                 \
    return check_launch("rk_fwfm_backward");                                                                   \
  }
  RK_FWFM_CASE(1, 4)
  RK_FWFM_CASE(2, 4)
  RK_FWFM_CASE(4, 4)
  RK_FWFM_CASE(8, 4)
  RK_FWFM_CASE(16, 4)
  RK_FWFM_CASE(32, 4)
  RK_FWFM_CASE(64, 4)
  RK_FWFM_CASE(1, 1)
  RK_FWFM_CASE(2, 1)
  RK_FWFM_CASE(4, 1)
  RK_FWFM_CASE(8, 1)
  RK_FWFM_CASE(16, 1)
  RK_FWFM_CASE(32, 1)
  RK_FWFM_CASE(64, 1)
#undef RK_FWFM_CASE
  return fail(RK_ERR_UNSUPPORTED, "rk_fwfm_backward: dim %d", dim);
}
