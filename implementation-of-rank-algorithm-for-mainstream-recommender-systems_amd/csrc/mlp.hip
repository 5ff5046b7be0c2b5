// Fused MLP tail: every hidden layer and the final Linear(N,1)+sigmoid head in one launch
// (machinery in mlp_core.h).  Epilogues (bias, BatchNorm folded to scale/shift, ReLU /
// LeakyReLU / Dice / PReLU, residual) run on the accumulators before the LDS write.
//
// Reference tails covered: dcn.py:144-152,175-180; deepfm.py:100-112,143-151;
// din.py:272-285,312-316; bst.py:203-214,245-247; deepcrossing.py:25-42,157-162.
#include <cstdlib>

#include "mlp_core.h"
#include "mlp_stream.h"

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
  int off_epi;   // streamed plans: float offset of the epilogue-parameter image
};

// RT row tiles of 16 rows per workgroup: every weight element streamed from L2 serves 16*RT rows
template <int RT, bool STORE>
__global__ __launch_bounds__(kMlpThreads) void mlp_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int ROWS = kMlpRows * RT;
  const int tid = threadIdx.x;
#ifdef RK_MLP_PHASES
  const unsigned long long k_t0 = clock64();
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 2);
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
  mlp_rows<RT, STORE>(a.L, a.nl, a.K0, buf0, a.ld0, buf1, a.ld1, m0, rows, a.head, a.y, a.ldy, tid,
                      finish_only(stage));
  MLP_MARK(4 * RK_MLP_MAX_LAYERS + 1, k_t0);  // whole workgroup (incl. head)
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 3);
  MLP_FLUSH(tid);
}

// The generic tail with its input row gathered in the stage (round 5, rk_mlp_forward_gather): wave w
// of the 16-row workgroup reads sample m0 + w's columns straight from the segments (a dense block or
// a table row at the sample's index, rk_concat_gather's column map: the last covering segment wins,
// uncovered columns and out-of-range rows are zero, the latter flagged) into the layer-0 buffer, so
// the [M, width] row never goes through HBM.  DeepCrossing's forward (deepcrossing.py:146-163): the
// residual units and output_layer run on mlp_rows as in mlp_kernel.
constexpr int kMgSegs = 16;
constexpr int kMgCols = 256;
struct MlpGatherArgs {
  MlpArgs m;
  rk_segment segs[kMgSegs];
  uint8_t col_seg[kMgCols], col_off[kMgCols];  // 255: no segment
  uint32_t* flags;
};
static_assert(sizeof(MlpGatherArgs) <= 4096, "kernel arguments beyond 4 KiB");

__global__ __launch_bounds__(kMlpThreads) void mlp_gather_kernel(MlpGatherArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * kMlpRows;
  const int rows = (int)min<int64_t>(kMlpRows, a.m.M - m0);
  float* const buf0 = sm;
  float* const buf1 = sm + a.m.off1;
  const int K0p = pad64(a.m.K0);
  const bool live = wave < rows;
  const int64_t b = m0 + wave;
  // the row's index in every column's segment first (one dependent round trip), the values after
  float v[kMgCols / 64];
  int64_t r[kMgCols / 64];
  int sg[kMgCols / 64];
  auto stage_issue = [&]() {
#pragma unroll
    for (int i = 0; i < kMgCols / 64; ++i) {
      const int c = lane + 64 * i;
      sg[i] = live && c < a.m.K0 ? a.col_seg[c] : 255;
      r[i] = b;
      if (sg[i] != 255) {
        const rk_segment& g = a.segs[sg[i]];
        if (g.idx) {
          r[i] = g.idx[b * g.idx_stride];
          if (r[i] < 0 || r[i] >= g.rows) {
            flag_oob(a.flags);
            r[i] = -1;
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < kMgCols / 64; ++i) {
      v[i] = 0.f;
      if (sg[i] != 255 && r[i] >= 0) {
        const rk_segment& g = a.segs[sg[i]];
        v[i] = g.src[r[i] * g.src_ld + a.col_off[lane + 64 * i]];
      }
    }
  };
  auto stage_store = [&]() {
#pragma unroll
    for (int i = 0; i < kMgCols / 64; ++i) {
      const int c = lane + 64 * i;
      if (c < K0p) buf0[wave * a.m.ld0 + c] = v[i];
    }
  };
  mlp_rows<1, false>(a.m.L, a.m.nl, a.m.K0, buf0, a.m.ld0, buf1, a.m.ld1, m0, rows, a.m.head, a.m.y, a.m.ldy, tid,
                     two_phase(stage_issue, stage_store));
}

// DeepCrossing's forward with every weight in registers (round 6): the residual units
// (deepcrossing.py:25-42: x <- relu(x + W2 relu(W1 x + b1) + b2)) and output_layer over 16 rows per
// workgroup of 16 waves.  mlp_gather_kernel streams each layer's weights through the 8-slot ring
// and fetches the second layer's only after the first layer's MFMAs (an L2 round trip at every
// layer boundary); here the whole image of the workgroup's tiles (50 -> 128 -> 50: 64 KiB, 16 or 48
// VGPRs per wave) is loaded at entry, beside the row gather's index round trip, so the only
// exposed latency is index -> row.  Work split as mlp_rows (wave w owns column tile w of a layer;
// waves without a tile wait at the barrier); the MFMA order, the epilogue (col_apply) and the head
// are mlp_rows', so the outputs are bit-identical to mlp_gather_kernel's.  IT: column tiles of the
// internal layer (internal dim <= 16 IT), U residual units, K0 <= 64 input columns.
constexpr int kDcMaxUnits = 2;
template <int IT, int U>
__global__ __launch_bounds__(kMlpThreads) void dc_forward_kernel(MlpGatherArgs a) {
  static_assert(IT <= kMlpWaves && U <= kDcMaxUnits, "one tile per wave");
  constexpr int KX = 64 + kMlpLdPad, KH = 16 * IT + kMlpLdPad;  // LDS row strides
  __shared__ __attribute__((aligned(16))) float xs[kMlpRows * KX];
  __shared__ __attribute__((aligned(16))) float hs[kMlpRows * KH];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id(), li = lane & 15, kq = 4 * (lane >> 4);
  const int64_t m0 = (int64_t)blockIdx.x * kMlpRows;
  const int rows = (int)min<int64_t>(kMlpRows, a.m.M - m0);
  const bool live = wave < rows;
  const int64_t b = m0 + wave;
  // the row: lane t loads the sample's index in segment t (the descriptor fields picked by selects
  // over constant-index argument reads, as dcn_fused_kernel), while the column -> segment map and
  // the column's source are looked up per lane beside it; then each column takes its segment's index
  // by a cross-lane read and loads its value — index -> value, one dependent round trip after the
  // argument reads instead of map -> descriptor -> index -> value
  const int c = lane;  // K0 <= 64: one column per lane
  const int64_t* ip = a.segs[0].idx;
  int64_t ist = a.segs[0].idx_stride, irows = a.segs[0].rows;
#pragma unroll
  for (int t = 1; t < kMgSegs; ++t)
    if (lane == t) {
      ip = a.segs[t].idx;
      ist = a.segs[t].idx_stride;
      irows = a.segs[t].rows;
    }
  int64_t mine = b;
  if (live && ip) {  // lanes past the segment count read a zeroed slot (idx null): nothing
    mine = ip[b * ist];
    if (mine < 0 || mine >= irows) {
      flag_oob(a.flags);
      mine = -1;
    }
  }
  const int sg = live && c < a.m.K0 ? a.col_seg[c] : 255;
  const float* csrc = nullptr;
  int64_t cld = 0;
  if (sg != 255) {
    csrc = a.segs[sg].src + a.col_off[c];
    cld = a.segs[sg].src_ld;
  }
  const int64_t r = __shfl(mine, sg != 255 ? sg : 0, kWave);
  // every weight fragment of this wave's tiles (fragment-major packed images, mlp_core.h wfrag)
  f32x4_t wa[U][4], wb[U][IT];
  // per-column biases only: dc_plan admits no other epilogue parameter (col_apply reads only the
  // bias of a ReLU layer without affines), so the rest of ColEpi is never live
  float ea[U], eb[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const rk_mlp_layer& LA = a.m.L[2 * u];
    const rk_mlp_layer& LB = a.m.L[2 * u + 1];
    if (wave < IT) {
#pragma unroll
      for (int k = 0; k < 4; ++k) wa[u][k] = *reinterpret_cast<const f32x4_t*>(wfrag(LA, wave, lane) + kFragStep * k);
      const int n = 16 * wave + li;
      ea[u] = col_epi(LA, n < LA.n ? n : 0).bias;
    }
    if (wave < 4) {
#pragma unroll
      for (int k = 0; k < IT; ++k) wb[u][k] = *reinterpret_cast<const f32x4_t*>(wfrag(LB, wave, lane) + kFragStep * k);
      const int n = 16 * wave + li;
      eb[u] = col_epi(LB, n < LB.n ? n : 0).bias;
    }
  }
  const float hw = lane < a.m.K0 ? a.m.head.head_w[lane] : 0.f;
  float v = 0.f;
  if (sg != 255 && r >= 0) v = csrc[r * cld];
  xs[wave * KX + c] = v;  // dead rows and pad columns stage zeros (mlp_rows' zero K pad)
  mlp_lds_barrier();
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const rk_mlp_layer& LA = a.m.L[2 * u];
    const rk_mlp_layer& LB = a.m.L[2 * u + 1];
    if (wave < IT) {  // x [16 x 64] . W1^T -> relu(. + b1) into hs
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      const float* arow = xs + li * KX + kq;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x4_t av = *reinterpret_cast<const f32x4_t*>(arow + 16 * k);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = mfma16(av[e], wa[u][k][e], acc);
      }
      const int n = 16 * wave + li;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = (lane >> 4) * 4 + q;
        const float z = col_apply(LA, ColEpi{ea[u], 1.f, 0.f, 0.f, 0.f, 0.f, 1.f, 0.f}, false, acc[q], false, 0.f);
        hs[row * KH + n] = n < LA.n ? z : 0.f;
      }
    }
    mlp_lds_barrier();
    if (wave < 4) {  // h [16 x 16 IT] . W2^T -> relu(x + . + b2) over x in place
      f32x4_t acc = {0.f, 0.f, 0.f, 0.f};
      const float* arow = hs + li * KH + kq;
#pragma unroll
      for (int k = 0; k < IT; ++k) {
        const f32x4_t av = *reinterpret_cast<const f32x4_t*>(arow + 16 * k);
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = mfma16(av[e], wb[u][k][e], acc);
      }
      const int n = 16 * wave + li;
      float res[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) res[q] = xs[((lane >> 4) * 4 + q) * KX + n];  // read all, then write (same lane)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = (lane >> 4) * 4 + q;
        const float z = col_apply(LB, ColEpi{eb[u], 1.f, 0.f, 0.f, 0.f, 0.f, 1.f, 0.f}, false, acc[q], true, res[q]);
        xs[row * KX + n] = n < LB.n ? z : 0.f;
      }
    }
    mlp_lds_barrier();
  }
  // head: one wave per row (mlp_rows' order: one fmaf per lane, then wave_sum)
  if (live) {
    float p = 0.f;
    if (lane < a.m.K0) p = fmaf(xs[wave * KX + lane], hw, p);
    p = wave_sum(p);
    if (lane == 0) {
      const float logit = p + a.m.head.head_b[0];
      if (a.m.head.head_logit) a.m.head.head_logit[b] = logit;
      if (a.m.head.head_prob) a.m.head.head_prob[b] = 1.0f / (1.0f + expf(-logit));
    }
  }
}

// The layer stacks dc_forward_kernel runs: U <= 2 residual units over K0 <= 64 input columns, each
// (internal <= 128, ReLU, no residual) then (K0 wide, ReLU, residual), bias optional, nothing else
// (no BatchNorm affines, Dice / PReLU, stores); a plain head.  Returns the internal tiles (0: no).
static int dc_plan(const rk_mlp_layer* layers, int nlayers, int K0, const rk_epilogue& h) {
  if (const char* e = getenv("RANKOPS_DC_KERNEL"))
    if (e[0] == '0') return 0;
  if (K0 > 64 || nlayers < 2 || nlayers > 2 * kDcMaxUnits || (nlayers & 1)) return 0;
  if (h.head_partial || h.fm1 || h.head_aux || !h.head_w) return 0;
  const int I = layers[0].n;
  if (I > 128) return 0;
  for (int l = 0; l < nlayers; ++l) {
    const rk_mlp_layer& L = layers[l];
    const bool second = l & 1;
    if (L.act != RK_ACT_RELU || L.store || L.pre_scale || L.post_scale || L.n != (second ? K0 : I) ||
        L.residual != (second ? 1 : 0))
      return 0;
  }
  return I <= 64 ? 4 : 8;
}

// The same tail on a compiled layer plan (mlp_stream.h): one weight stream across the layers.
// RT = 2 (large batches): 32 rows per workgroup, each weight float4 feeding both 16-row tiles.
template <class P, int RT>
__global__ __launch_bounds__(kMlpThreads) void mlp_stream_kernel(MlpArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  constexpr int kRows = kMlpRows * RT;
  const int tid = threadIdx.x;
  const int64_t m0 = (int64_t)blockIdx.x * kRows;
  const int rows = (int)min<int64_t>(kRows, a.M - m0);
  float* const buf0 = sm;
  float* const buf1 = sm + a.off1;
  const int K0p = P::KC0 * 16;
  auto stage = [&]() {
    if (a.x_vec) {
      const int q = K0p / 4;
      for (int i = tid; i < kRows * q; i += kMlpThreads) {
        const int r = i / q, c = (i % q) * 4;
        f32x4_t v = {0.f, 0.f, 0.f, 0.f};
        if (r < rows && c < a.K0) v = *reinterpret_cast<const f32x4_t*>(a.x + (m0 + r) * a.ldx + c);
        *reinterpret_cast<f32x4_t*>(buf0 + r * a.ld0 + c) = v;
      }
    } else {
      for (int i = tid; i < kRows * K0p; i += kMlpThreads) {
        const int r = i / K0p, c = i % K0p;
        buf0[r * a.ld0 + c] = (r < rows && c < a.K0) ? a.x[(m0 + r) * a.ldx + c] : 0.f;
      }
    }
  };
#ifdef RK_MLP_PHASES
  const unsigned long long k_t0 = clock64();
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 2);
#endif
  mlp_stream_rows<P, RK_STREAM_EPI, RT>(a.L, buf0, a.ld0, buf1, a.ld1, sm + a.off_epi, m0, rows, a.head, tid,
                                        finish_only(stage));
  MLP_MARK(4 * RK_MLP_MAX_LAYERS + 1, k_t0);
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 3);
  MLP_FLUSH(tid);
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
constexpr int kDcnPreLayers = 3;  // cross layers whose weights are fetched with the row values

// The gather plan of the stage, with every slot loadable unconditionally: a dense segment (and an
// unused slot) reads its "index" from the device flag word (ignored; the row is the sample), an
// unused slot has out_col past the width, so no column selects it.
struct DcnSeg {
  const float* src;
  const int64_t* idx;  // never null
  int64_t idx_stride;  // 0 for dense / unused slots
  int64_t src_ld;
  int64_t rows;        // bounds of a table; INT64_MAX for dense / unused slots
  int32_t out_col;
  int32_t dense;
};

struct DcnArgs {
  MlpArgs m;
  DcnSeg segs[kDcnSegs];
  int nseg;
  const float* cross_w;
  const float* cross_b;
  int num_layers;
  const float* cross_head_w;
  uint32_t* flags;
};

// NJ = column groups of 64 per lane (1: width <= 64, the DCN wechat row of 50; 4: width <= 256).
// RT = 2 (streamed plan, large batches): 32 rows per workgroup — wave w stages rows m0 + w and
// m0 + 16 + w, each weight-ring slot feeds both 16-row tiles (mlp_stream.h RT), and the side waves
// 8..15 take four cross rows each.  Per-row arithmetic unchanged: bit-identical to RT = 1.
template <int NJ, class P, int RT = 1>
__global__ __launch_bounds__(kMlpThreads) void dcn_fused_kernel(DcnArgs a) {
  static_assert(RT == 1 || (NJ == 1 && !std::is_void_v<P>), "32-row workgroups: streamed plan, width <= 64");
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
#ifdef RK_MLP_PHASES
  const unsigned long long k_t0 = clock64();
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 2);
#endif
  constexpr int kRows = kMlpRows * RT;
  const int64_t m0 = (int64_t)blockIdx.x * kRows;
  const int rows = (int)min<int64_t>(kRows, a.m.M - m0);
  float* const buf0 = sm;
  float* const buf1 = sm + a.m.off1;
  float* const part = buf1 + kRows * a.m.ld1;
  float* const x0s = part + kRows;  // streamed path: the staged rows [16 RT][64], for the side work
  const int width = a.m.K0;
  // Two memory round trips per row instead of one dependent index -> row chain per column: (1) the
  // sample's row index in every segment (wave-uniform loads), (2) the row values of the lane's
  // columns together with the cross weights, the cross biases and the cross half of output_layer.
  // Out-of-range indices read row 0 with the value forced to zero and raise RK_FLAG_INDEX_OOB.
  // stage state carried from issue() (before layer 0's weight prefetch) to the finish
  const int nl = a.num_layers;
  float x0[RT][NJ], xl[NJ], cw[kDcnPreLayers][NJ], cb[kDcnPreLayers][NJ], hw[NJ];
  bool live[RT];
  int64_t bb[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    live[t] = wave + kMlpRows * t < rows;
    bb[t] = live[t] ? m0 + kMlpRows * t + wave : m0;
  }
  // round trip 1: the sample's row in every segment — lane t loads segment t's index (one vector
  // load per wave; 8 scalar loads measured ~2.4 us at kernel start), then every lane reads them
  // back (wave-uniform).  The streamed tail issues it ahead of its weight ring (stage.early()).
  int64_t mine[RT];
  auto stage_index = [&]() {
    const int64_t* ip = a.segs[0].idx;
    int64_t st = a.segs[0].idx_stride;
#pragma unroll
    for (int t = 1; t < kDcnSegs; ++t)
      if (lane == t) ip = a.segs[t].idx, st = a.segs[t].idx_stride;
#pragma unroll
    for (int t = 0; t < RT; ++t) mine[t] = ip[bb[t] * st];
  };
  auto stage_issue = [&]() {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      int64_t rix[kDcnSegs];
#pragma unroll
      for (int t = 0; t < kDcnSegs; ++t) {
        const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)mine[rt], t);
        const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)((uint64_t)mine[rt] >> 32), t);
        rix[t] = (int64_t)(((uint64_t)hi << 32) | lo);
      }
      bool bad = false;
#pragma unroll
      for (int t = 0; t < kDcnSegs; ++t) {
        if (a.segs[t].dense) rix[t] = bb[rt];
        const bool okt = rix[t] >= 0 && rix[t] < a.segs[t].rows;
        bad = bad || !okt;
        rix[t] = okt ? rix[t] : -1;  // -1: zero row (read row 0, value dropped)
      }
      if (bad && live[rt] && lane == 0) flag_oob(a.flags);
      // round trip 2: the lane's row values
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = lane + 64 * j;
        const int cc = min(c, width - 1);
        const float* src = a.segs[0].src;
        int64_t r = rix[0], ld = a.segs[0].src_ld;
        int col = cc;
#pragma unroll
        for (int t = 1; t < kDcnSegs; ++t) {
          const bool sel = cc >= a.segs[t].out_col;  // out_col ascending
          src = sel ? a.segs[t].src : src;
          r = sel ? rix[t] : r;
          ld = sel ? a.segs[t].src_ld : ld;
          col = sel ? cc - a.segs[t].out_col : col;
        }
        const float v = src[(r < 0 ? 0 : r) * ld + col];
        x0[rt][j] = (live[rt] && c < width && r >= 0) ? v : 0.f;
      }
    }
    // ... with the cross weights / biases of the first layers and the cross half of output_layer
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const int cc = min(lane + 64 * j, width - 1);
      // unconditional loads (a clamped layer; with no cross layer, any valid vector): loads under
      // `if (l < nl)` were placed after layer 0's weight ring, and waiting for them drained it
      const float* cwp = nl > 0 ? a.cross_w : a.cross_head_w;
      const float* cbp = nl > 0 ? a.cross_b : a.cross_head_w;
#pragma unroll
      for (int l = 0; l < kDcnPreLayers; ++l) {
        const int64_t o = (int64_t)min(l, max(nl - 1, 0)) * width + cc;
        cw[l][j] = cwp[o];
        cb[l][j] = cbp[o];
      }
      hw[j] = a.cross_head_w[cc];
    }
  };
  auto stage_store = [&]() {
    const int K0p = pad64(width);
#pragma unroll
    for (int t = 0; t < RT; ++t) {
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = lane + 64 * j;
        if (t == 0) xl[j] = x0[0][j];
        if (c < K0p) buf0[(kMlpRows * t + wave) * a.m.ld0 + c] = x0[t][j];
      }
      if constexpr (!std::is_void_v<P>) x0s[(kMlpRows * t + wave) * 64 + lane] = x0[t][0];
    }
  };
  // the cross stack and the cross half of output_layer (generic path, after the stage; the
  // streamed path runs cross_row below as side work instead)
  auto stage_cross = [&]() {
    auto cross = [&](const float* w, const float* bl) {
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (lane + 64 * j < width) d = fmaf(xl[j], w[j], d);
      d = wave_sum_dpp(d);
#pragma unroll
      for (int j = 0; j < NJ; ++j)
        if (lane + 64 * j < width) {
          float t = x0[0][j] * d;  // torch.mul(x0, xl_wl)
          t = t + bl[j];           // + bl.t()
          xl[j] = t + xl[j];       // + xl
        }
    };
    // the first kDcnPreLayers layers straight-line from registers (a runtime loop with loads in it
    // made the compiler close its header with vmcnt(0), draining layer 0's weight ring here)
#pragma unroll
    for (int l = 0; l < kDcnPreLayers; ++l)
      if (l < nl) cross(cw[l], cb[l]);
    for (int l = kDcnPreLayers; l < nl; ++l) {
      float w[NJ], bl[NJ];
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int c = min(lane + 64 * j, width - 1);
        w[j] = a.cross_w[(int64_t)l * width + c];
        bl[j] = a.cross_b[(int64_t)l * width + c];
      }
      cross(w, bl);
    }
    float p = 0.f;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
      if (lane + 64 * j < width) p = fmaf(xl[j], hw[j], p);
    p = wave_sum_dpp(p);
    if (lane == 0) part[wave] = p;
  };
  // streamed path (NJ = 1): the cross stack of staged row s, by any wave (the same arithmetic as
  // stage_cross); the side work of the third layer, whose 8 column tiles leave waves 8..15 idle:
  // wave w takes rows w - 8 and w (and, at RT = 2, those plus 16), off the second layer's critical path
  auto cross_row = [&](int r) {
    const float x0v = x0s[r * 64 + lane];
    float xlv = x0v;
    const bool in = lane < width;
    auto cross1 = [&](float w, float bl) {
      float d = 0.f;
      if (in) d = fmaf(xlv, w, d);
      d = wave_sum_dpp(d);
      if (in) {
        float t = x0v * d;
        t = t + bl;
        xlv = t + xlv;
      }
    };
#pragma unroll
    for (int l = 0; l < kDcnPreLayers; ++l)
      if (l < nl) cross1(cw[l][0], cb[l][0]);
    for (int l = kDcnPreLayers; l < nl; ++l) {
      const int c = min(lane, width - 1);
      cross1(a.cross_w[(int64_t)l * width + c], a.cross_b[(int64_t)l * width + c]);
    }
    float p = 0.f;
    if (in) p = fmaf(xlv, hw[0], p);
    p = wave_sum_dpp(p);
    if (lane == 0) part[r] = p;
  };
  auto side_cross = [&]() {
    if (wave >= kMlpWaves / 2) {
#pragma unroll
      for (int t = 0; t < RT; ++t) {
        cross_row(kMlpRows * t + wave - kMlpWaves / 2);
        cross_row(kMlpRows * t + wave);
      }
    }
  };
  if constexpr (std::is_void_v<P>)
    mlp_rows(a.m.L, a.m.nl, width, buf0, a.m.ld0, buf1, a.m.ld1, m0, rows, a.m.head, nullptr, 0, tid,
             two_phase(
                 [&]() {
                   stage_index();
                   stage_issue();
                 },
                 [&]() {
                   stage_store();
                   stage_cross();
                 }),
             part);
  else
    mlp_stream_rows<P, RK_STREAM_EPI, RT>(a.m.L, buf0, a.m.ld0, buf1, a.m.ld1, sm + a.m.off_epi, m0, rows, a.m.head,
                                          tid, side_at<2>(staged(stage_index, stage_issue, stage_store, side_cross)),
                                          part);
  MLP_MARK(4 * RK_MLP_MAX_LAYERS + 1, k_t0);  // whole workgroup (incl. stage and head)
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 3);
  MLP_FLUSH(tid);
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


int stream_plan_for(const rk_mlp_layer* layers, int nlayers, int K0) {
  if (const char* e = getenv("RANKOPS_MLP_STREAM"))
    if (e[0] == '0') return kStreamNone;
  if (nlayers < 1 || nlayers > 3 || pad64(K0) > 1024) return kStreamNone;
  int nt[3] = {0, 0, 0};
  for (int l = 0; l < nlayers; ++l) {
    if (layers[l].residual || layers[l].store) return kStreamNone;
    nt[l] = pad64(layers[l].n) / 16;
  }
  const int kc0 = pad64(K0) / 16;
  if (nlayers == 3 && nt[0] == 32 && nt[1] == 16 && nt[2] == 8) {
    switch (kc0) {
      case 4: return kStreamK64;
      case 8: return kStreamK128;
      case 12: return kStreamK192;
      case 16: return kStreamK256;
      default: return kStreamNone;
    }
  }
  if (nlayers == 2 && kc0 == 32 && nt[0] == 16 && nt[1] == 8) return kStreamTail512;
  return kStreamNone;
}

int stream_plan_epi_floats(int id) {
  switch (id) {
    case kStreamK64: return StreamPlanK64::epi_floats();
    case kStreamK128: return StreamPlanK128::epi_floats();
    case kStreamK192: return StreamPlanK192::epi_floats();
    case kStreamK256: return StreamPlanK256::epi_floats();
    case kStreamTail512: return StreamPlanTail512::epi_floats();
    default: return 0;
  }
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

// The streamed tail's epilogue-parameter image ([column][8] resolved floats: mlp_stream.h
// StreamEpi, the layout of its LDS image) written to global memory once, for kernels that copy it
// into LDS with LDS-DMA instead of resolving every column's parameters at launch (DIN plans).
struct EpiPackArgs {
  rk_mlp_layer L[RK_MLP_MAX_LAYERS];
  float* out;
};
template <class P>
__global__ __launch_bounds__(kMlpThreads) void mlp_pack_epilogue_kernel(EpiPackArgs a) {
  StreamEpi<P> e;
  e.load(a.L, threadIdx.x);
  e.store(a.out, threadIdx.x);
}

RK_API int rk_mlp_epilogue_image_floats(const rk_mlp_layer* layers, int32_t nlayers, int32_t K0) {
  if (!layers || nlayers <= 0 || nlayers > RK_MLP_MAX_LAYERS || K0 <= 0) return 0;
  return stream_plan_epi_floats(stream_plan_for(layers, nlayers, K0));
}

RK_API int rk_mlp_pack_epilogue(const rk_mlp_layer* layers, int32_t nlayers, int32_t K0, float* out, void* stream) {
  if (!out || ((uintptr_t)out & 15u)) return fail(RK_ERR_INVALID, "rk_mlp_pack_epilogue: output null or misaligned");
  int need0 = 0, need1 = 0;
  const rk_epilogue none = {};
  if (int e = mlp_validate(layers, nlayers, K0, none, &need0, &need1, "rk_mlp_pack_epilogue")) return e;
  EpiPackArgs a = {};
  for (int l = 0; l < nlayers; ++l) a.L[l] = layers[l];
  a.out = out;
  const hipStream_t st = (hipStream_t)stream;
  switch (stream_plan_for(layers, nlayers, K0)) {
    case kStreamK64: mlp_pack_epilogue_kernel<StreamPlanK64><<<1, kMlpThreads, 0, st>>>(a); break;
    case kStreamK128: mlp_pack_epilogue_kernel<StreamPlanK128><<<1, kMlpThreads, 0, st>>>(a); break;
    case kStreamK192: mlp_pack_epilogue_kernel<StreamPlanK192><<<1, kMlpThreads, 0, st>>>(a); break;
    case kStreamK256: mlp_pack_epilogue_kernel<StreamPlanK256><<<1, kMlpThreads, 0, st>>>(a); break;
    case kStreamTail512: mlp_pack_epilogue_kernel<StreamPlanTail512><<<1, kMlpThreads, 0, st>>>(a); break;
    default: return fail(RK_ERR_UNSUPPORTED, "rk_mlp_pack_epilogue: no compiled layer plan for this stack");
  }
  return check_launch("rk_mlp_pack_epilogue");
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
  // row stride = width + kMlpLdPad (width is a multiple of 64): conflict-free float4 row reads
  a.ld0 = need0 + kMlpLdPad;
  a.ld1 = need1 + kMlpLdPad;
  // rows per workgroup: 16.  32 (two row tiles per wave: half the L2 weight traffic per row)
  // measured slower at batch 4096 — DCN 46.6 vs 52.6 us: half the workgroups, same per-workgroup
  // latency — so a compiled plan (the streamed tail) takes 32 only once the batch gives every CU a
  // 32-row workgroup, and mlp_kernel only on request.  RANKOPS_MLP_ROWS=16 / 32 forces either where
  // the buffers fit in LDS.
  const size_t row_bytes = (size_t)(a.ld0 + a.ld1) * sizeof(float);
  const int plan0 = stream_plan_for(layers, nlayers, K0);
  const size_t epi_bytes = plan0 != kStreamNone ? sizeof(float) * stream_plan_epi_floats(plan0) : 0;
  const bool fits32 = 2 * kMlpRows * row_bytes + epi_bytes <= 160 * 1024 - kStreamStaticLds;
  int rt = plan0 != kStreamNone && fits32 && (M + 2 * kMlpRows - 1) / (2 * kMlpRows) >= num_cus() ? 2 : 1;
  if (const char* e = getenv("RANKOPS_MLP_ROWS")) rt = (atoi(e) == 32 && fits32) ? 2 : atoi(e) == 16 ? 1 : rt;
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
  bool store = false;  // hidden activations written out (training); eval compiles the path out
  for (int l = 0; l < nlayers; ++l) store = store || layers[l].store != nullptr;
  auto go = [&](auto kern, size_t bytes) {
    raise_lds_limit((const void*)kern, 160 * 1024);
    kern<<<(unsigned)blocks, kMlpThreads, bytes, (hipStream_t)stream>>>(a);
  };
  // a compiled layer plan: the streamed tail (mlp_stream.h), its epilogue image after the buffers
  const int plan = plan0;
  if (plan != kStreamNone) {
    a.off_epi = (int)(shm / sizeof(float));
    const size_t bytes = shm + sizeof(float) * stream_plan_epi_floats(plan);
    if (bytes <= 160 * 1024 - kStreamStaticLds) {
      auto launch = [&](auto RTI) {
        constexpr int R = decltype(RTI)::value;
        switch (plan) {
          case kStreamK64: go(mlp_stream_kernel<StreamPlanK64, R>, bytes); break;
          case kStreamK128: go(mlp_stream_kernel<StreamPlanK128, R>, bytes); break;
          case kStreamK192: go(mlp_stream_kernel<StreamPlanK192, R>, bytes); break;
          case kStreamK256: go(mlp_stream_kernel<StreamPlanK256, R>, bytes); break;
          default: go(mlp_stream_kernel<StreamPlanTail512, R>, bytes); break;
        }
      };
      if (rt == 2)
        launch(std::integral_constant<int, 2>{});
      else
        launch(std::integral_constant<int, 1>{});
      return check_launch("rk_mlp_forward");
    }
  }
  if (rt == 2)
    store ? go(mlp_kernel<2, true>, shm) : go(mlp_kernel<2, false>, shm);
  else
    store ? go(mlp_kernel<1, true>, shm) : go(mlp_kernel<1, false>, shm);
  return check_launch("rk_mlp_forward");
}

RK_API int rk_mlp_forward_gather(const rk_segment* segs, int32_t nseg, int32_t width, int64_t batch,
                                 const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head, void* stream) {
  if (!segs || nseg <= 0 || nseg > kMgSegs || width <= 0 || width > kMgCols || batch < 0 || !head || !head->head_w)
    return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward_gather: %d segments (<= %d) over %d columns (<= %d), with a head",
                nseg, kMgSegs, width, kMgCols);
  MlpGatherArgs g = {};
  MlpArgs& a = g.m;
  a.head = *head;
  int need0 = 0, need1 = 0;
  if (int e = mlp_validate(layers, nlayers, width, a.head, &need0, &need1, "rk_mlp_forward_gather")) return e;
  for (int l = 0; l < nlayers; ++l) {
    if (layers[l].store) return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward_gather: eval only (layer %d stores)", l);
    a.L[l] = layers[l];
  }
  a.nl = nlayers;
  a.ld0 = need0 + kMlpLdPad;
  a.ld1 = need1 + kMlpLdPad;
  a.off1 = kMlpRows * a.ld0;
  const size_t shm = (size_t)kMlpRows * (a.ld0 + a.ld1) * sizeof(float);
  if (shm > 160 * 1024) return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward_gather: widths need %zu B of LDS", shm);
  a.M = batch;
  a.K0 = width;
  for (int c = 0; c < kMgCols; ++c) {
    g.col_seg[c] = 255;
    g.col_off[c] = 0;
  }
  for (int i = 0; i < nseg; ++i) {
    const rk_segment& sg = segs[i];
    if (!sg.src || sg.dim <= 0 || sg.out_col < 0 || sg.out_col + sg.dim > width || (sg.idx && sg.rows <= 0) ||
        sg.dim > 255)
      return fail(RK_ERR_INVALID, "rk_mlp_forward_gather: segment %d invalid", i);
    g.segs[i] = sg;
    for (int c = sg.out_col; c < sg.out_col + sg.dim; ++c) {  // the last covering segment wins
      g.col_seg[c] = (uint8_t)i;
      g.col_off[c] = (uint8_t)(c - sg.out_col);
    }
  }
  g.flags = device_flags();
  if (!g.flags) return fail(RK_ERR_RUNTIME, "rk_mlp_forward_gather: device not initialised (rk_init)");
  if (batch == 0) return RK_OK;
  const int64_t blocks = (batch + kMlpRows - 1) / kMlpRows;
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_mlp_forward_gather: batch too large");
  if (const int it = dc_plan(layers, nlayers, width, a.head)) {  // DeepCrossing: weights in registers
    auto go = [&](auto kern) { kern<<<(unsigned)blocks, kMlpThreads, 0, (hipStream_t)stream>>>(g); };
    if (it == 4)
      nlayers == 2 ? go(dc_forward_kernel<4, 1>) : go(dc_forward_kernel<4, 2>);
    else
      nlayers == 2 ? go(dc_forward_kernel<8, 1>) : go(dc_forward_kernel<8, 2>);
    return check_launch("rk_mlp_forward_gather");
  }
  raise_lds_limit((const void*)mlp_gather_kernel, 160 * 1024);
  mlp_gather_kernel<<<(unsigned)blocks, kMlpThreads, shm, (hipStream_t)stream>>>(g);
  return check_launch("rk_mlp_forward_gather");
}

#ifdef RK_MLP_PHASES
// Timing build only (tools/dcn_phases.py): copies and clears this module's phase counters.
RK_API int rk_debug_mlp_phases(unsigned long long* marks, int32_t nwg, unsigned* wave_marks) {
  if (nwg < 0 || nwg > kMlpMarkWG) return 1;
  if (hipMemcpyFromSymbol(marks, HIP_SYMBOL(g_mlp_marks), sizeof(g_mlp_marks[0]) * nwg) != hipSuccess) return 1;
  if (wave_marks &&
      hipMemcpyFromSymbol(wave_marks, HIP_SYMBOL(g_mlp_wave_marks), sizeof(g_mlp_wave_marks[0]) * nwg) != hipSuccess)
    return 1;
  return 0;
}
#endif

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
  uint32_t* flags = device_flags();
  if (!flags) return fail(RK_ERR_RUNTIME, "rk_dcn_forward: device not initialised (rk_init)");
  int prev = -1;
  for (int i = 0; i < kDcnSegs; ++i) {
    DcnSeg& d = a.segs[i];
    if (i >= nseg) {  // unused slot: never selected, loads stay inside the flag word
      d = DcnSeg{reinterpret_cast<const float*>(flags), reinterpret_cast<const int64_t*>(flags), 0, 0, INT64_MAX,
                 INT32_MAX, 1};
      continue;
    }
    const rk_segment& g = segs[i];
    if (!g.src || g.dim <= 0 || g.out_col <= prev || g.out_col + g.dim > width || (g.idx && g.rows <= 0))
      return fail(RK_ERR_INVALID, "rk_dcn_forward: segment %d (out_col ascending, inside width)", i);
    prev = g.out_col;
    d.src = g.src;
    d.src_ld = g.src_ld;
    d.out_col = g.out_col;
    if (g.idx) {
      d.idx = g.idx;
      d.idx_stride = g.idx_stride;
      d.rows = g.rows;
      d.dense = 0;
    } else {
      d.idx = reinterpret_cast<const int64_t*>(flags);
      d.idx_stride = 0;
      d.rows = INT64_MAX;
      d.dense = 1;
    }
  }
  if (segs[0].out_col != 0) return fail(RK_ERR_INVALID, "rk_dcn_forward: segments must start at column 0");
  for (int l = 0; l < nlayers; ++l) a.m.L[l] = layers[l];
  a.m.nl = nlayers;
  a.m.ld0 = need0 + kMlpLdPad;
  a.m.ld1 = need1 + kMlpLdPad;
  a.m.M = batch;
  a.m.K0 = width;
  a.nseg = nseg;
  // the stage loads cross weights unconditionally (layer index clamped): any valid pointer will do
  // when there are no cross layers
  a.cross_w = num_layers > 0 ? cross_w : cross_head_w;
  a.cross_b = num_layers > 0 ? cross_b : cross_head_w;
  a.num_layers = num_layers;
  a.cross_head_w = cross_head_w;
  a.flags = flags;
  if (batch == 0) return RK_OK;
  // the wechat row (width <= 64) on a compiled layer plan: the streamed tail, its epilogue image
  // after the cross partials
  int plan = width <= 64 ? stream_plan_for(layers, nlayers, width) : kStreamNone;
  if (plan != kStreamNone && plan != kStreamK64) plan = kStreamNone;
  // 32-row workgroups (streamed plan) once the batch gives every CU one (RANKOPS_DCN_ROW_TILES =
  // 1 / 2 forces either)
  int rt = plan == kStreamK64 && (batch + 2 * kMlpRows - 1) / (2 * kMlpRows) >= num_cus() ? 2 : 1;
  if (const char* e = getenv("RANKOPS_DCN_ROW_TILES"))
    rt = plan == kStreamK64 && atoi(e) == 2 ? 2 : atoi(e) == 1 ? 1 : rt;
  const int rows_wg = kMlpRows * rt;
  a.m.off1 = rows_wg * a.m.ld0;
  size_t shm = (size_t)rows_wg * (a.m.ld0 + a.m.ld1) * sizeof(float) + rows_wg * sizeof(float);
  const size_t x0_bytes = (size_t)rows_wg * 64 * sizeof(float);  // streamed path: x0s
  if (shm > 160 * 1024) return fail(RK_ERR_UNSUPPORTED, "rk_dcn_forward: widths need %zu B of LDS", shm);
  const int64_t blocks = (batch + rows_wg - 1) / rows_wg;
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_dcn_forward: batch too large");
  if (plan != kStreamNone) {
    a.m.off_epi = (int)((shm + x0_bytes) / sizeof(float));
    if (shm + x0_bytes + sizeof(float) * stream_plan_epi_floats(plan) <= 160 * 1024 - kStreamStaticLds)
      shm += x0_bytes + sizeof(float) * stream_plan_epi_floats(plan);
    else
      plan = kStreamNone;
  }
  auto go = [&](auto kern) {
    raise_lds_limit((const void*)kern, 160 * 1024);
    kern<<<(unsigned)blocks, kMlpThreads, shm, (hipStream_t)stream>>>(a);
  };
  if (plan == kStreamK64 && rt == 2)
    go(dcn_fused_kernel<1, StreamPlanK64, 2>);
  else if (plan == kStreamK64)
    go(dcn_fused_kernel<1, StreamPlanK64>);
  else
    width <= 64 ? go(dcn_fused_kernel<1, void>) : go(dcn_fused_kernel<kDcnPerLane, void>);
  return check_launch("rk_dcn_forward");
}
