// BST multi-head self-attention core (reference: BSTTransformer.forward, bst.py:73-84).
//
//   scores = Q_h K_h^T / sqrt(d_h); scores[:, j >= len] = -inf; P = softmax(scores); ctx_h = P V_h
//
// Input is the packed projection buffer qkv [B*T, ld] holding Q | K | V column blocks of
// width d_model (head h uses columns h*d_h .. (h+1)*d_h of each block).  One wave per
// (sample, head): K_h and V_h are staged in LDS, lane = query position, the keys are swept
// with an online softmax.  The mask is either a length per sample (keys j >= len) or an
// explicit [B, T] byte mask (nonzero = padding).  A sample whose keys are all masked yields NaN
// context rows, like torch's softmax over an all -inf row (bst.py:80-82).
#include "common.h"

namespace rk {

template <int DH>
__global__ __launch_bounds__(256) void bst_attention_kernel(const float* __restrict__ qkv, int64_t ld_qkv,
                                                            int64_t batch, int T, int d_model, int heads,
                                                            const int64_t* __restrict__ seq_len,
                                                            const uint8_t* __restrict__ key_mask, int64_t ld_mask,
                                                            float* __restrict__ ctx, int64_t ld_ctx, int waves_per_wg) {
  extern __shared__ __attribute__((aligned(16))) float kv[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t item = (int64_t)blockIdx.x * waves_per_wg + wave;
  const bool live = item < batch * heads;
  float* Ks = kv + (int64_t)wave * 2 * T * DH;
  float* Vs = Ks + (int64_t)T * DH;
  const int64_t b = live ? item / heads : 0;
  const int h = live ? (int)(item % heads) : 0;
  const float* base = qkv + b * T * ld_qkv;

  if (live) {
    for (int i = lane; i < T * DH; i += 64) {
      const int j = i / DH, d = i % DH;
      Ks[i] = base[j * ld_qkv + d_model + h * DH + d];
      Vs[i] = base[j * ld_qkv + 2 * d_model + h * DH + d];
    }
  }
  __syncthreads();
  if (!live) return;

  // keys j >= seq_len[b] are masked (BSTModel's mask, bst.py:228-229); with an explicit
  // key_padding_mask (BSTTransformer.forward, bst.py:79-80) key j is masked where it is nonzero;
  // with neither nothing is masked
  const int64_t len = seq_len ? seq_len[b] : (int64_t)T;
  const int nkeys = (int)(len < 0 ? 0 : (len > T ? T : len));
  const uint8_t* mrow = key_mask ? key_mask + b * ld_mask : nullptr;
  int nvalid = nkeys;
  if (mrow) {
    nvalid = 0;
    for (int j = 0; j < nkeys; ++j) nvalid += mrow[j] == 0;
  }
  const float scale = (float)__builtin_sqrt((double)DH);

  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + lane;
    if (t >= T) continue;
    float q[DH], o[DH];
    const float* qrow = base + (int64_t)t * ld_qkv + h * DH;
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      q[d] = qrow[d];
      o[d] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int j = 0; j < nkeys; ++j) {
      if (mrow && mrow[j]) continue;
      float s = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) s = fmaf(q[d], Ks[j * DH + d], s);
      s = s / scale;
      const float m_new = fmaxf(m, s);
      const float a = expf(m - m_new);
      const float p = expf(s - m_new);
      l = l * a + p;
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] = o[d] * a + p * Vs[j * DH + d];
      m = m_new;
    }
    float* crow = ctx + (b * T + t) * ld_ctx + h * DH;
    const float inv = nvalid > 0 ? 1.0f / l : __builtin_nanf("");
#pragma unroll
    for (int d = 0; d < DH; ++d) crow[d] = nvalid > 0 ? o[d] * inv : inv;
  }
}

}  // namespace rk

using namespace rk;

static int launch_bst_attention(const float* qkv, int64_t ld_qkv, int64_t batch, int32_t T, int32_t d_model,
                                int32_t heads, const int64_t* seq_len, const uint8_t* key_mask, int64_t ld_mask,
                                float* ctx, int64_t ld_ctx, void* stream, const char* who) {
  if (!qkv || !ctx || T <= 0 || d_model <= 0 || heads <= 0 || d_model % heads != 0 || ld_qkv < 3 * d_model ||
      ld_ctx < d_model || batch < 0 || (key_mask && ld_mask < T))
    return fail(RK_ERR_INVALID, "%s: bad arguments (T=%d d=%d heads=%d)", who, T, d_model, heads);
  if (batch == 0) return RK_OK;
  const int dh = d_model / heads;
  const size_t per_wave = (size_t)2 * T * dh * sizeof(float);
  if (per_wave > 160 * 1024) return fail(RK_ERR_UNSUPPORTED, "%s: T*d_h too large for LDS", who);
  int wpg = 4;
  while (wpg > 1 && per_wave * wpg > 64 * 1024) wpg >>= 1;
  const int64_t items = batch * heads;
  const unsigned blocks = (unsigned)((items + wpg - 1) / wpg);
  const size_t shm = per_wave * wpg;
  hipStream_t st = (hipStream_t)stream;
#define RK_BST_CASE(DD)                                                                                       \
  case DD:                                                                                                    \
    if (shm > 64 * 1024) raise_lds_limit((const void*)bst_attention_kernel<DD>, (int)shm);                   \
    bst_attention_kernel<DD><<<blocks, 64 * wpg, shm, st>>>(qkv, ld_qkv, batch, T, d_model, heads, seq_len,   \
                                                           key_mask, ld_mask, ctx, ld_ctx, wpg);              \
    break;
  switch (dh) {
    RK_BST_CASE(1)
    RK_BST_CASE(2)
    RK_BST_CASE(4)
    RK_BST_CASE(8)
    RK_BST_CASE(16)
    RK_BST_CASE(32)
    RK_BST_CASE(64)
    default:
      return fail(RK_ERR_UNSUPPORTED, "%s: head dim %d not in {1,2,4,8,16,32,64}", who, dh);
  }
#undef RK_BST_CASE
  return check_launch(who);
}

RK_API int rk_bst_attention(const float* qkv, int64_t ld_qkv, int64_t batch, int32_t T, int32_t d_model,
                            int32_t heads, const int64_t* seq_len, float* ctx, int64_t ld_ctx, void* stream) {
  if (!seq_len) return fail(RK_ERR_INVALID, "rk_bst_attention: null seq_len");
  return launch_bst_attention(qkv, ld_qkv, batch, T, d_model, heads, seq_len, nullptr, 0, ctx, ld_ctx, stream,
                              "rk_bst_attention");
}

RK_API int rk_bst_attention_masked(const float* qkv, int64_t ld_qkv, int64_t batch, int32_t T, int32_t d_model,
                                   int32_t heads, const uint8_t* key_padding_mask, int64_t ld_mask, float* ctx,
                                   int64_t ld_ctx, void* stream) {
  return launch_bst_attention(qkv, ld_qkv, batch, T, d_model, heads, nullptr, key_padding_mask, ld_mask, ctx,
                              ld_ctx, stream, "rk_bst_attention_masked");
}
