// Fused MLP tail: every hidden layer and the final Linear(N,1)+sigmoid head in one launch
// (machinery in mlp_core.h).  Epilogues (bias, BatchNorm folded to scale/shift, ReLU /
// LeakyReLU / Dice / PReLU, residual) run on the accumulators before the LDS write.
//
// Reference tails covered: dcn.py:144-152,175-180; deepfm.py:100-112,143-151;
// din.py:272-285,312-316; bst.py:203-214,245-247; deepcrossing.py:25-42,157-162.
#include <cstdlib>

#include "mlp_core.h"

namespace rk {

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

// RT row tiles of 16 rows per workgroup: every weight element streamed from L2 serves 16*RT rows
template <int RT>
__global__ __launch_bounds__(kMlpThreads) void mlp_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int ROWS = kMlpRows * RT;
  const int tid = threadIdx.x;
#ifdef RK_MLP_PHASES
  const unsigned long long k_t0 = clock64();
  const unsigned long long w0 = wall_clock64();
  if (tid == 0) {
    atomicMin(&g_mlp_span[0], w0);
    atomicMax(&g_mlp_span[2], w0);  // last workgroup start
  }
#endif
  const int64_t m0 = (int64_t)blockIdx.x * ROWS;
  const int rows = (int)min<int64_t>(ROWS, a.M - m0);
  float* const buf0 = sm;
  float* const buf1 = sm + a.off1;

  // stage the input tile, zero-padded to a multiple of 64 columns (inside mlp_rows: after layer
  // 0's weight prefetch has been issued)
  const int K0p = pad64(a.K0);
  auto stage = [&]() {
    if (a.x_vec) {
      const int q = K0p / 4;
      for (int i = tid; i < ROWS * q; i += kMlpThreads) {
        const int r = i / q, c = (i % q) * 4;
        f32x4_t v = {0.f, 0.f, 0.f, 0.f};
        if (r < rows && c < a.K0) v = *reinterpret_cast<const f32x4_t*>(a.x + (m0 + r) * a.ldx + c);
        *reinterpret_cast<f32x4_t*>(buf0 + r * a.ld0 + c) = v;
      }
    } else {
      for (int i = tid; i < ROWS * K0p; i += kMlpThreads) {
        const int r = i / K0p, c = i % K0p;
        buf0[r * a.ld0 + c] = (r < rows && c < a.K0) ? a.x[(m0 + r) * a.ldx + c] : 0.f;
      }
    }
  };
  mlp_rows<RT>(a.L, a.nl, a.K0, buf0, a.ld0, buf1, a.ld1, m0, rows, a.head, a.y, a.ldy, tid, stage);
  MLP_MARK(3 * RK_MLP_MAX_LAYERS + 1, k_t0);  // whole workgroup (incl. head)
#ifdef RK_MLP_PHASES
  if (tid == 0) {
    const unsigned long long w1 = wall_clock64();
    atomicMax(&g_mlp_span[1], w1);
    atomicMax(&g_mlp_span[3], w1 - w0);  // longest workgroup
    atomicAdd(&g_mlp_span[4], w1 - w0);  // sum of workgroup durations
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (blockIdx.x < 8192) {
      g_mlp_wg[blockIdx.x][0] = hw;
      g_mlp_wg[blockIdx.x][1] = xcc;
      g_mlp_wg[blockIdx.x][2] = (unsigned)(w1 - w0);
      g_mlp_wg[blockIdx.x][3] = (unsigned)(w0 - g_mlp_span[0]);
    }
  }
#endif
}

// Whole DCN eval forward in one launch (DCNModel.forward, dcn.py:161-180): per 16-row tile, wave w
// gathers row m0 + w (dense + category embeddings, dcn.py:163-169) straight into the MLP's LDS
// input buffer while layer 0's weights are already in flight, runs the cross stack on the row in
// registers (x_{l+1} = x0 (x_l . w_l) + b_l + x_l, dcn.py:25-50,171-173) and leaves the cross half of
// output_layer (x_L . W_out[:, :width]) in LDS; then the MLP tail and the head (the dnn half,
// + bias, + the cross partial, sigmoid: dcn.py:175-180) as in mlp_kernel.  Replaces rk_dcn_cross +
// rk_mlp_forward (two launches and an x0 / partial round trip through HBM).
constexpr int kDcnSegs = 8;
constexpr int kDcnPerLane = 4;  // width <= 256

struct DcnArgs {
  MlpArgs m;
  rk_segment segs[kDcnSegs];
  int nseg;
  const float* cross_w;
  const float* cross_b;
  int num_layers;
  const float* cross_head_w;
  uint32_t* flags;
};

__global__ __launch_bounds__(kMlpThreads) void dcn_fused_kernel(DcnArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * kMlpRows;
  const int rows = (int)min<int64_t>(kMlpRows, a.m.M - m0);
  float* const buf0 = sm;
  float* const buf1 = sm + a.m.off1;
  float* const part = buf1 + kMlpRows * a.m.ld1;
  const int width = a.m.K0;
  auto stage = [&]() {
    const int64_t b = m0 + wave;
    const bool live = wave < rows;
    const int K0p = pad64(width);
    float x0[kDcnPerLane], xl[kDcnPerLane];
#pragma unroll
    for (int j = 0; j < kDcnPerLane; ++j) {
      const int c = lane + 64 * j;
      float v = 0.f;
      if (live && c < width) {
        int s = 0;
        for (int t = 1; t < a.nseg; ++t) s = c >= a.segs[t].out_col ? t : s;  // out_col ascending
        const float* row = segment_row(a.segs[s], b, a.flags);
        if (row) v = row[c - a.segs[s].out_col];
      }
      x0[j] = xl[j] = v;
      if (c < K0p) buf0[wave * a.m.ld0 + c] = v;
    }
    for (int l = 0; l < a.num_layers; ++l) {
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < kDcnPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) d = fmaf(xl[j], a.cross_w[(int64_t)l * width + c], d);
      }
      d = wave_sum(d);
#pragma unroll
      for (int j = 0; j < kDcnPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) {
          float t = x0[j] * d;                        // torch.mul(x0, xl_wl)
          t = t + a.cross_b[(int64_t)l * width + c];  // + bl.t()
          xl[j] = t + xl[j];                          // + xl
        }
      }
    }
    float p = 0.f;
#pragma unroll
    for (int j = 0; j < kDcnPerLane; ++j) {
      const int c = lane + 64 * j;
      if (c < width) p = fmaf(xl[j], a.cross_head_w[c], p);
    }
    p = wave_sum(p);
    if (lane == 0) part[wave] = p;
  };
  mlp_rows(a.m.L, a.m.nl, width, buf0, a.m.ld0, buf1, a.m.ld1, m0, rows, a.m.head, nullptr, 0, tid, stage, part);
}

// Fragment-major image (mlp_core.h wfrag): element i of the image is lane (i >> 2) & 63, component
// i & 3 of chunk c of column tile t, i >> 8 = t * kp/16 + c; that lane's value is W[16 t + (lane & 15)]
// [16 c + 4 (lane >> 4) + (i & 3)], zero outside [n, k).
__global__ void mlp_pack_kernel(const float* __restrict__ w, int64_t ldw, int n, int k, int np, int kp,
                                float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)np * kp) return;
  const int e = (int)(i & 3), lane = (int)((i >> 2) & 63);
  const int64_t blk = i >> 8;
  const int kch = kp / 16;
  const int t = (int)(blk / kch), c = (int)(blk % kch);
  const int r = 16 * t + (lane & 15), col = 16 * c + 4 * (lane >> 4) + e;
  out[i] = (r < n && col < k) ? w[(int64_t)r * ldw + col] : 0.f;
}


int mlp_validate(const rk_mlp_layer* layers, int nlayers, int K0, const rk_epilogue& head, int* need0, int* need1,
                 const char* what) {
  if (K0 <= 0 || nlayers < 0 || nlayers > RK_MLP_MAX_LAYERS || (nlayers && !layers))
    return fail(RK_ERR_INVALID, "%s: bad layer stack (K0=%d layers=%d)", what, K0, nlayers);
  if (head.head_w && !head.head_b) return fail(RK_ERR_INVALID, "%s: head needs head_b", what);
  if (head.fm1 && (!head.fm2 || !head.final_w || !head.final_b))
    return fail(RK_ERR_INVALID, "%s: FM combine incomplete", what);
  if (pad64(K0) > 1024) return fail(RK_ERR_UNSUPPORTED, "%s: input width %d > 1024", what, K0);
  int K = K0;
  int n0 = pad64(K0), n1 = kMlpPad;
  for (int l = 0; l < nlayers; ++l) {
    const rk_mlp_layer& L = layers[l];
    if (!L.w || L.n <= 0 || L.n > kMlpMaxN || L.ldw != pad64(K) || !aligned16(L.w))
      return fail(RK_ERR_UNSUPPORTED,
                  "%s: layer %d (n=%d, ldw=%lld, K=%d) must be packed by rk_mlp_pack_weight, n <= %d", what, l, L.n,
                  (long long)L.ldw, K, kMlpMaxN);
    if (L.act == RK_ACT_DICE && (!L.act_scale || !L.act_shift || !L.act_alpha))
      return fail(RK_ERR_INVALID, "%s: Dice layer %d incomplete", what, l);
    if (L.act == RK_ACT_PRELU && !L.act_alpha) return fail(RK_ERR_INVALID, "%s: PReLU needs alpha", what);
    if (L.act < 0 || L.act > RK_ACT_PRELU) return fail(RK_ERR_INVALID, "%s: unknown activation %d", what, L.act);
    if (L.store && L.ld_store < L.n) return fail(RK_ERR_INVALID, "%s: layer %d store ld < n", what, l);
    if ((L.pre_scale != nullptr) != (L.pre_shift != nullptr) || (L.post_scale != nullptr) != (L.post_shift != nullptr))
      return fail(RK_ERR_INVALID, "%s: affine scale/shift must come in pairs", what);
    if (L.residual && (l == 0 || L.n != (l >= 2 ? layers[l - 2].n : K0)))
      return fail(RK_ERR_INVALID, "%s: residual layer %d must map back to the width of layer %d's input", what, l,
                  l - 1);
    if ((l + 1) & 1)
      n1 = std::max(n1, pad64(L.n));
    else
      n0 = std::max(n0, pad64(L.n));
    K = L.n;
  }
  *need0 = n0;
  *need1 = n1;
  return RK_OK;
}

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
  if (!x || M < 0 || ldx < K0) return fail(RK_ERR_INVALID, "rk_mlp_forward: bad input (M=%lld)", (long long)M);
  MlpArgs a = {};
  if (head) a.head = *head;
  if (!a.head.head_w && !y) return fail(RK_ERR_INVALID, "rk_mlp_forward: need a head or an output");
  int need0 = 0, need1 = 0;
  if (int e = mlp_validate(layers, nlayers, K0, a.head, &need0, &need1, "rk_mlp_forward")) return e;
  for (int l = 0; l < nlayers; ++l) a.L[l] = layers[l];
  a.nl = nlayers;
  // row stride = width + 4 (width is a multiple of 64): conflict-free float4 row reads
  a.ld0 = need0 + 4;
  a.ld1 = need1 + 4;
  // rows per workgroup: 16.  32 (two row tiles per wave: half the L2 weight traffic per row)
  // measured slower at batch 4096 — DCN 46.6 vs 52.6 us: half the workgroups, same per-workgroup
  // latency — and is kept as an option (RANKOPS_MLP_ROWS=32) where the buffers fit in LDS.
  const size_t row_bytes = (size_t)(a.ld0 + a.ld1) * sizeof(float);
  int rt = 1;
  if (const char* e = getenv("RANKOPS_MLP_ROWS")) rt = (atoi(e) == 32 && 32 * row_bytes <= 160 * 1024) ? 2 : 1;
  const int rows_per_wg = kMlpRows * rt;
  a.off1 = rows_per_wg * a.ld0;
  const size_t shm = rows_per_wg * row_bytes;
  if (shm > 160 * 1024) return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward: widths need %zu B of LDS", shm);
  a.x = x;
  a.ldx = ldx;
  a.M = M;
  a.K0 = K0;
  a.x_vec = (ldx % 4 == 0) && aligned16(x) && (K0 % 4 == 0);
  a.y = y;
  a.ldy = ldy;
  if (M == 0) return RK_OK;
  const int64_t blocks = (M + rows_per_wg - 1) / rows_per_wg;
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward: M too large");
  raise_lds_limit((const void*)mlp_kernel<1>, 160 * 1024);
  raise_lds_limit((const void*)mlp_kernel<2>, 160 * 1024);
  if (rt == 2)
    mlp_kernel<2><<<(unsigned)blocks, kMlpThreads, shm, (hipStream_t)stream>>>(a);
  else
    mlp_kernel<1><<<(unsigned)blocks, kMlpThreads, shm, (hipStream_t)stream>>>(a);
  return check_launch("rk_mlp_forward");
}

RK_API int rk_dcn_forward(const rk_segment* segs, int32_t nseg, int64_t batch, int32_t width, const float* cross_w,
                          const float* cross_b, int32_t num_layers, const float* cross_head_w,
                          const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head, void* stream) {
  if (!segs || nseg <= 0 || nseg > kDcnSegs || batch < 0 || width <= 0 || width > 64 * kDcnPerLane ||
      num_layers < 0 || (num_layers > 0 && (!cross_w || !cross_b)) || !cross_head_w || !head || !head->head_w)
    return fail(RK_ERR_INVALID, "rk_dcn_forward: bad arguments (nseg %d <= %d, width %d <= %d, head required)", nseg,
                kDcnSegs, width, 64 * kDcnPerLane);
  DcnArgs a = {};
  a.m.head = *head;
  if (a.m.head.head_partial || a.m.head.fm1)
    return fail(RK_ERR_INVALID, "rk_dcn_forward: the cross partial comes from the kernel (no head_partial / fm1)");
  int need0 = 0, need1 = 0;
  if (int e = mlp_validate(layers, nlayers, width, a.m.head, &need0, &need1, "rk_dcn_forward")) return e;
  int prev = -1;
  for (int i = 0; i < nseg; ++i) {
    const rk_segment& g = segs[i];
    if (!g.src || g.dim <= 0 || g.out_col <= prev || g.out_col + g.dim > width || (g.idx && g.rows <= 0))
      return fail(RK_ERR_INVALID, "rk_dcn_forward: segment %d (out_col ascending, inside width)", i);
    prev = g.out_col;
    a.segs[i] = g;
  }
  if (segs[0].out_col != 0) return fail(RK_ERR_INVALID, "rk_dcn_forward: segments must start at column 0");
  for (int l = 0; l < nlayers; ++l) a.m.L[l] = layers[l];
  a.m.nl = nlayers;
  a.m.ld0 = need0 + 4;
  a.m.ld1 = need1 + 4;
  a.m.off1 = kMlpRows * a.m.ld0;
  a.m.M = batch;
  a.m.K0 = width;
  a.nseg = nseg;
  a.cross_w = cross_w;
  a.cross_b = cross_b;
  a.num_layers = num_layers;
  a.cross_head_w = cross_head_w;
  a.flags = device_flags();
  const size_t shm = (size_t)kMlpRows * (a.m.ld0 + a.m.ld1) * sizeof(float) + kMlpRows * sizeof(float);
  if (shm > 160 * 1024) return fail(RK_ERR_UNSUPPORTED, "rk_dcn_forward: widths need %zu B of LDS", shm);
  if (batch == 0) return RK_OK;
  const int64_t blocks = (batch + kMlpRows - 1) / kMlpRows;
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_dcn_forward: batch too large");
  raise_lds_limit((const void*)dcn_fused_kernel, 160 * 1024);
  dcn_fused_kernel<<<(unsigned)blocks, kMlpThreads, shm, (hipStream_t)stream>>>(a);
  return check_launch("rk_dcn_forward");
}
