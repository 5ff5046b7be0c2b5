// DIN local-activation attention (reference: din_attention, din.py:42-84).
//
//   cross[t]  = [q, k_t, q - k_t, q * k_t]                     (4H)
//   score[t]  = W3 . relu(W2 . relu(W1 . cross[t] + b1) + b2) + b3
//   softmax:  s = (t < len ? score : -4294967295) / sqrt(H); w = softmax_t(s)
//   else:     w = (t < len ? score : 0)
//   out       = sum_t w[t] * k_t
//
// One wave per sample, the history split in tiles of 32 positions.  The attention MLP
// runs transposed on FP32 MFMA so that no activation ever leaves registers:
//   layer 1: h1^T[j, t] = W1[j, :] . cross[t, :]     A = W1 (LDS), B = cross^T built in
//            registers from the gathered key rows and the query (64 x 32 tile, 2 MFMA tiles)
//   layer 2: h2^T = W2 . h1^T                        B = the layer-1 accumulator as is
//            (register s of a 32x32 accumulator holds row (s&3)+8(s>>2)+4(lane>>5))
//   layer 3: score[t] = sum over the accumulator rows, finished with one lane^32 exchange.
// Softmax runs online across the tiles; the weighted key sum stays lane-local until one
// final half-wave reduction.
#include "common.h"

namespace rk {

constexpr int kDinH1 = 64, kDinH2 = 32;

template <int H>
__global__ __launch_bounds__(256) void din_attention_kernel(
    const float* __restrict__ query, int64_t ld_query, const float* __restrict__ key_table, int64_t key_rows,
    int64_t ld_key, const int64_t* __restrict__ seq, int64_t ld_seq, int64_t ld_kb, int T,
    const int64_t* __restrict__ seq_len,
    int64_t batch, const float* __restrict__ w1, const float* __restrict__ b1, const float* __restrict__ w2,
    const float* __restrict__ b2, const float* __restrict__ w3, const float* __restrict__ b3, int use_softmax,
    float* __restrict__ out, int64_t ld_out, uint32_t* flags) {
  constexpr int K1 = 4 * H;         // layer-1 input width
  constexpr int LD1 = K1 + 4;       // padded LDS rows (conflict-free float4 reads)
  constexpr int LD2 = kDinH1 + 4;
  constexpr int NQ = H / 8;         // float4 chunks of q / k held per lane
  __shared__ __attribute__((aligned(16))) float sW1[kDinH1 * LD1];
  __shared__ __attribute__((aligned(16))) float sW2[kDinH2 * LD2];
  __shared__ float sB1[kDinH1], sB2[kDinH2], sW3[kDinH2];

  for (int i = threadIdx.x; i < kDinH1 * K1; i += 256) sW1[(i / K1) * LD1 + (i % K1)] = w1[i];
  for (int i = threadIdx.x; i < kDinH2 * kDinH1; i += 256) sW2[(i / kDinH1) * LD2 + (i % kDinH1)] = w2[i];
  if (threadIdx.x < kDinH1) sB1[threadIdx.x] = b1[threadIdx.x];
  if (threadIdx.x < kDinH2) {
    sB2[threadIdx.x] = b2[threadIdx.x];
    sW3[threadIdx.x] = w3[threadIdx.x];
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, half = lane >> 5, hk = 4 * half;
  const float bias3 = b3[0];
  const float sqrt_h = (float)__builtin_sqrt((double)H);
  const float pad = -4294967296.0f;  // (-2**32 + 1) rounded to fp32, din.py:74
  const int ntiles = (T + 31) / 32;

  for (int64_t b = (int64_t)blockIdx.x * 4 + wave; b < batch; b += (int64_t)gridDim.x * 4) {
    // query chunks: q[8c + hk + comp]
    f32x4 q[NQ];
    const float* qrow = query + b * ld_query;
#pragma unroll
    for (int c = 0; c < NQ; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) q[c][e] = qrow[8 * c + hk + e];
    const int64_t len = seq_len[b];

    float m_run = -INFINITY, l_run = 0.f;
    f32x4 o[NQ];
#pragma unroll
    for (int c = 0; c < NQ; ++c) o[c] = (f32x4){0.f, 0.f, 0.f, 0.f};

    for (int tt = 0; tt < ntiles; ++tt) {
      asm volatile("" ::: "memory");  // keep the loop-invariant LDS weight reads inside the loop
      const int t = tt * 32 + l32;
      const bool in_seq = t < T;
      f32x4 k[NQ];
      const float* krow = nullptr;
      if (in_seq) {
        if (seq) {  // history gathered from the embedding table
          const int64_t r = seq[b * ld_seq + t];
          if (r >= 0 && r < key_rows)
            krow = key_table + r * ld_key;
          else
            flag_oob(flags);
        } else {  // dense keys [B, T, H]
          krow = key_table + b * ld_kb + (int64_t)t * ld_key;
        }
      }
#pragma unroll
      for (int c = 0; c < NQ; ++c)
        k[c] = krow ? *reinterpret_cast<const f32x4*>(krow + 8 * c + hk) : (f32x4){0.f, 0.f, 0.f, 0.f};

      // ---- layer 1 (transposed): acc1[jt] = W1[jt*32 .. +32, :] . cross^T
      f32x16 acc1[2];
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc1[jt][r] = 0.f;
#pragma unroll
      for (int c8 = 0; c8 < K1 / 8; ++c8) {
        const int seg = (8 * c8) / H, cq = ((8 * c8) % H) / 8;
        f32x4 bv;
        if (seg == 0)
          bv = q[cq];
        else if (seg == 1)
          bv = k[cq];
        else if (seg == 2)
          bv = q[cq] - k[cq];
        else
          bv = q[cq] * k[cq];
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
          const f32x4 av = *reinterpret_cast<const f32x4*>(sW1 + (jt * 32 + l32) * LD1 + 8 * c8 + hk);
#pragma unroll
          for (int e = 0; e < 4; ++e) acc1[jt] = mfma32(av[e], bv[e], acc1[jt]);
        }
      }
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float z = acc1[jt][r] + sB1[jt * 32 + acc_row(r, lane)];
          acc1[jt][r] = z < 0.f ? 0.f : z;
        }

      // ---- layer 2: acc2 = W2 . h1^T, B operand = acc1 registers
      f32x16 acc2;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc2[r] = 0.f;
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const f32x4 av = *reinterpret_cast<const f32x4*>(sW2 + l32 * LD2 + jt * 32 + 8 * u + hk);
#pragma unroll
          for (int v = 0; v < 4; ++v) acc2 = mfma32(av[v], acc1[jt][4 * u + v], acc2);
        }

      // ---- layer 3: score[t]
      float sc = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j2 = acc_row(r, lane);
        float z = acc2[r] + sB2[j2];
        z = z < 0.f ? 0.f : z;
        sc = fmaf(z, sW3[j2], sc);
      }
      sc += __shfl_xor(sc, 32, kWave);
      sc = sc + bias3;

      const bool valid = in_seq && (int64_t)t < len;
      if (use_softmax) {
        const float s = in_seq ? (valid ? sc : pad) / sqrt_h : -INFINITY;
        const float m_tile = wave_max(s);
        const float m_new = fmaxf(m_run, m_tile);
        const float scale_old = expf(m_run - m_new);
        const float p = in_seq ? expf(s - m_new) : 0.f;
        // each position is held by two lanes (halves); count it once
        const float lsum = wave_sum(half == 0 ? p : 0.f);
        l_run = l_run * scale_old + lsum;
        m_run = m_new;
#pragma unroll
        for (int c = 0; c < NQ; ++c) o[c] = o[c] * scale_old + p * k[c];
      } else {
        const float w = valid ? sc : 0.f;
#pragma unroll
        for (int c = 0; c < NQ; ++c) o[c] = o[c] + w * k[c];
      }
    }

    // reduce the lane-local sums over the 32 positions of each half
    const float inv_l = use_softmax ? 1.0f / l_run : 1.0f;
    float* orow = out + b * ld_out;
#pragma unroll
    for (int c = 0; c < NQ; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = half_sum(o[c][e]);
        if (l32 == 4 * c + e) orow[8 * c + hk + e] = use_softmax ? v * inv_l : v;
      }
  }
}

}  // namespace rk

using namespace rk;

static int launch_din_attention(const float* query, int64_t ld_query, const float* key_table, int64_t key_rows,
                                int64_t ld_key, const int64_t* seq, int64_t ld_seq, int64_t ld_kb, int32_t T,
                                const int64_t* seq_len, int64_t batch, int32_t H, const float* w1, const float* b1,
                                const float* w2, const float* b2, const float* w3, const float* b3,
                                int32_t use_softmax, float* out, int64_t ld_out, void* stream, const char* who) {
  if (batch == 0) return RK_OK;
  const int64_t want = (batch + 3) / 4;
  // persistent: W1/W2 are staged in LDS once per workgroup, which then walks many samples
  const unsigned blocks = (unsigned)std::min<int64_t>(want, (int64_t)num_cus() * 2);
  hipStream_t st = (hipStream_t)stream;
  uint32_t* fl = device_flags();
#define RK_DIN_CASE(HH)                                                                                         \
  case HH:                                                                                                      \
    din_attention_kernel<HH><<<blocks, 256, 0, st>>>(query, ld_query, key_table, key_rows, ld_key, seq, ld_seq, \
                                                     ld_kb, T, seq_len, batch, w1, b1, w2, b2, w3, b3,          \
                                                     use_softmax, out, ld_out, fl);                             \
    break;
  switch (H) {
    RK_DIN_CASE(8)
    RK_DIN_CASE(16)
    RK_DIN_CASE(32)
    RK_DIN_CASE(64)
    default:
      return fail(RK_ERR_UNSUPPORTED, "%s: embedding dim %d not in {8,16,32,64}", who, H);
  }
#undef RK_DIN_CASE
  return check_launch(who);
}

RK_API int rk_din_attention(const float* query, int64_t ld_query, const float* key_table, int64_t key_rows,
                            int64_t ld_key, const int64_t* seq, int64_t ld_seq, int32_t T, const int64_t* seq_len,
                            int64_t batch, int32_t H, const float* w1, const float* b1, const float* w2,
                            const float* b2, const float* w3, const float* b3, int32_t use_softmax, float* out,
                            int64_t ld_out, void* stream) {
  if (!query || !key_table || !seq || !seq_len || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !out)
    return fail(RK_ERR_INVALID, "rk_din_attention: null pointer");
  if (T <= 0 || batch < 0 || key_rows <= 0 || ld_seq < T || ld_query < H || ld_out < H || ld_key < H)
    return fail(RK_ERR_INVALID, "rk_din_attention: bad shape T=%d H=%d", T, H);
  if (ld_key % 4 != 0 || ((uintptr_t)key_table & 15u))
    return fail(RK_ERR_UNSUPPORTED, "rk_din_attention: key table rows must be 16-B aligned");
  return launch_din_attention(query, ld_query, key_table, key_rows, ld_key, seq, ld_seq, 0, T, seq_len, batch, H,
                              w1, b1, w2, b2, w3, b3, use_softmax, out, ld_out, stream, "rk_din_attention");
}

RK_API int rk_din_attention_dense(const float* query, int64_t ld_query, const float* keys, int64_t ld_keys_b,
                                  int64_t ld_keys_t, int32_t T, const int64_t* keys_length, int64_t batch,
                                  int32_t H, const float* w1, const float* b1, const float* w2, const float* b2,
                                  const float* w3, const float* b3, int32_t use_softmax, float* out,
                                  int64_t ld_out, void* stream) {
  if (!query || !keys || !keys_length || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !out)
    return fail(RK_ERR_INVALID, "rk_din_attention_dense: null pointer");
  if (T <= 0 || batch < 0 || ld_query < H || ld_out < H || ld_keys_t < H || ld_keys_b < (int64_t)T * ld_keys_t)
    return fail(RK_ERR_INVALID, "rk_din_attention_dense: bad shape T=%d H=%d", T, H);
  if (ld_keys_t % 4 != 0 || ld_keys_b % 4 != 0 || ((uintptr_t)keys & 15u))
    return fail(RK_ERR_UNSUPPORTED, "rk_din_attention_dense: key rows must be 16-B aligned");
  return launch_din_attention(query, ld_query, keys, 0, ld_keys_t, nullptr, 0, ld_keys_b, T, keys_length, batch, H,
                              w1, b1, w2, b2, w3, b3, use_softmax, out, ld_out, stream, "rk_din_attention_dense");
}
