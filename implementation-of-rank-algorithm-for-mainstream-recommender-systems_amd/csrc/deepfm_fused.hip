// Whole DeepFM eval forward in one launch (DeepFM.forward, deepfm.py:121-151) on the streamed tail
// (mlp_stream.h): per 16-row tile, wave w gathers sample m0 + w's packed rows (rk_fm_pack_table
// layout: the dim second-order values, then the first-order weight) of every field straight into
// the MLP's LDS input row, the three deep layers (Linear + BatchNorm folded + ReLU,
// deepfm.py:100-112) run on one weight stream across the layers, and the head evaluates
// deep_output_layer, final_layer over [fm1, fm2, deep] and the sigmoid (deepfm.py:143-151).
//
// Replaces rk_fm_linear_packed (the gather + FM + first layer as a 64 x 128-tiled GEMM) +
// rk_mlp_forward (the rest of the tail): one launch, no [B, 512] round trip through HBM, no
// K-block barriers (the whole 960-wide row of 16 samples, 61 KB, stays in LDS for layer 0), and
// the FM sums (deepfm.py:122-140) are taken beside layer 0's MFMAs from the staged row instead of
// in the prologue.  The cost: every workgroup streams the whole first-layer weight (1.97 MB) for 16
// rows, from L2 (the 2D tiling streamed a quarter of it for 64 rows).
//
// Gather in three dependent rounds, all issued around layer 0's weight ring: (1) lane f loads the
// sample's index in field f (before the ring); (2) lane f forms the row address, every lane
// fetches its float4s of the row through a cross-lane read of the owning field's address, and lane
// f the first-order weight (after the ring); (3) the LDS store before the barrier that opens
// layer 0.
//
// Large batches (>= 32 rows per CU): RT = 2 row tiles, 32 rows per workgroup (wave w stages samples
// m0 + w and m0 + 16 + w), so each CU streams the weight image once per 32 rows; layer 0 writes its
// output over the input row in place (mlp_stream.h IP0).  Per-row arithmetic and order unchanged:
// bit-identical to RT = 1 (tests/test_gpu_deepfm_fused.py).
#include <cstdlib>
#include <type_traits>

#include "mlp_core.h"
#include "mlp_stream.h"

namespace rk {

constexpr int kDfMaxFields = 32;
// weight-ring loads issued ahead of the 30-field row gather (mlp_stream.h RingEarly): 4 against the
// default 2 measured 54.6 / 55.0 vs 55.6 / 55.9 and 55.8 / 56.5 vs 56.7 / 56.4 us per forward (profiles/r05/ab_early/)
#ifndef RK_DEEPFM_RING_EARLY
#define RK_DEEPFM_RING_EARLY 4
#endif
constexpr int kDfLayers = 3;

struct DfArgs {
  rk_mlp_layer L[kDfLayers];
  rk_epilogue head;
  // per field: packed table (or dense block of packed rows), its index column (a dense field
  // reads the flag word with stride 0 and uses the sample's own row), bounds
  const float* src[kDfMaxFields];
  const int64_t* idx[kDfMaxFields];
  int64_t istride[kDfMaxFields];
  int64_t ld[kDfMaxFields];
  int64_t rows[kDfMaxFields];
  uint32_t dense_mask;
  int F, dim_shift;
  int64_t M;
  int ld0, ld1, off1, off_fm;
  float* fm1;
  float* fm2;
  uint32_t* flags;
};
// rk_deepfm_forward_fo: first-order weight of field f for row index r from fo[f][r * fo_ld[f]] (split
// wire rows: the owner's per-sample partial sum on its first field, nullptr on the others).  A
// separate kernel-argument type, so the packed path's arguments stay as small as before.
struct DfArgsFo : DfArgs {
  const float* fo[kDfMaxFields];
  int64_t fo_ld[kDfMaxFields];
};

// FO: first-order weights from a.fo (rk_deepfm_forward_fo); otherwise from the packed row itself
// (column dim, the address the row's own loads use: no per-field pointer loads)
template <class P, int RT, bool FO>
__global__ __launch_bounds__(kMlpThreads) void deepfm_fused_kernel(std::conditional_t<FO, DfArgsFo, DfArgs> a) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = wave_id();
#ifdef RK_MLP_PHASES
  const unsigned long long k_t0 = clock64();
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 2);
#endif
  constexpr int kRows = kMlpRows * RT;
  const int64_t m0 = (int64_t)blockIdx.x * kRows;
  const int rows = (int)min<int64_t>(kRows, a.M - m0);
  float* const buf0 = sm;
  float* const buf1 = sm + a.off1;
  float* const fm_lds = sm + a.off_fm;  // [fm1 x 16 RT][fm2 x 16 RT]
  const int dim = 1 << a.dim_shift, G = dim >> 2;  // float4 quads per field
  const int nq = a.F * G;                            // float4s of the row
  constexpr int kQ = (P::KC0 * 4 + 63) / 64;         // float4s per lane (the padded row)
  const int f_me = lane < a.F ? lane : 0;

  // per row tile t: the wave's sample m0 + 16 t + wave
  bool live[RT];
  int64_t b[RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) {
    live[t] = wave + kMlpRows * t < rows;
    b[t] = live[t] ? m0 + kMlpRows * t + wave : m0;
  }
  int64_t idx_v[RT];
  f32x4_t v[RT][kQ];
  float fw[RT];
  unsigned long long okmask[RT];
  // round 1: lane f's index in field f
  auto st_index = [&]() {
#pragma unroll
    for (int t = 0; t < RT; ++t) idx_v[t] = a.idx[f_me][b[t] * a.istride[f_me]];
  };
  // round 2: the row address in lane f, the row's float4s (quad q of the row = quad q % G of field
  // q / G) and the first-order weight; loads unconditional from valid addresses, masks applied at
  // the store
  auto st_issue = [&]() {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const int64_t r = (a.dense_mask >> f_me) & 1u ? b[t] : idx_v[t];
      const bool ok = r >= 0 && r < a.rows[f_me];
      const bool bad = lane < a.F && !ok;
      if (live[t] && __builtin_amdgcn_ballot_w64(bad) != 0 && lane == 0) flag_oob(a.flags);
      okmask[t] = __builtin_amdgcn_ballot_w64(ok && live[t] && lane < a.F);
      const int64_t rr = ok ? r : 0;
      const float* p = a.src[f_me] + rr * a.ld[f_me];
      const uint64_t pu = reinterpret_cast<uint64_t>(p);
      const uint32_t plo = (uint32_t)pu, phi = (uint32_t)(pu >> 32);
#pragma unroll
      for (int i = 0; i < kQ; ++i) {
        const int q = lane + 64 * i;
        const int f = min(q >> (a.dim_shift - 2), a.F - 1);
        const uint32_t lo = __shfl(plo, f, kWave), hi = __shfl(phi, f, kWave);
        const float* row = reinterpret_cast<const float*>(((uint64_t)hi << 32) | lo);
        v[t][i] = *reinterpret_cast<const f32x4_t*>(row + 4 * (q & (G - 1)));
      }
      if constexpr (FO) {
        const float* fop = a.fo[f_me];
        fw[t] = fop ? fop[rr * a.fo_ld[f_me]] : 0.f;
      } else {
        fw[t] = p[dim];
      }
    }
  };
  // round 3: the row into buf0 (zeros for padding quads, out-of-range rows and rows past the batch)
  auto st_store = [&]() {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
#pragma unroll
      for (int i = 0; i < kQ; ++i) {
        const int q = lane + 64 * i;
        if (q < P::KC0 * 4) {
          const int f = q >> (a.dim_shift - 2);
          const bool keep = q < nq && ((okmask[t] >> f) & 1ull);
          *reinterpret_cast<f32x4_t*>(buf0 + (kMlpRows * t + wave) * a.ld0 + 4 * q) =
              keep ? v[t][i] : (f32x4_t){0.f, 0.f, 0.f, 0.f};
        }
      }
    }
  };
  // beside layer 0's MFMAs (buf0 is read-only until layer 0's epilogue): fm1 = sum_f w1_f, fm2 =
  // 0.5 sum_d ((sum_f e_fd)^2 - sum_f e_fd^2) over the staged row, as rk_fm_linear_packed
  auto st_fm = [&]() {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const int row = kMlpRows * t + wave;
      f32x4_t s = {0.f, 0.f, 0.f, 0.f}, sq = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < kQ; ++i) {
        const int q = lane + 64 * i;
        if (q < nq) {
          const f32x4_t x = *reinterpret_cast<const f32x4_t*>(buf0 + row * a.ld0 + 4 * q);
          s += x;
          sq += x * x;
        }
      }
      float o = ((okmask[t] >> lane) & 1ull) ? fw[t] : 0.f;  // lanes < F
      // lanes of equal lane % G hold the same dims: sum over lane / G
      for (int x = G; x < 64; x <<= 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[e] += __shfl_xor(s[e], x, kWave);
          sq[e] += __shfl_xor(sq[e], x, kWave);
        }
      }
      float part = (s[0] * s[0] - sq[0]) + (s[1] * s[1] - sq[1]) + (s[2] * s[2] - sq[2]) + (s[3] * s[3] - sq[3]);
      for (int x = G / 2; x > 0; x >>= 1) part += __shfl_xor(part, x, kWave);
      o = wave_sum(o);
      if (lane == 0) {
        const float f2 = 0.5f * part;
        fm_lds[row] = o;
        fm_lds[kRows + row] = f2;
        if (live[t]) {
          a.fm1[b[t]] = o;
          a.fm2[b[t]] = f2;
        }
      }
    }
  };
  mlp_stream_rows<P, RK_STREAM_EPI, RT, (RT > 1)>(a.L, buf0, a.ld0, buf1, a.ld1, nullptr, m0, rows, a.head, tid,
                                    ring_early<RK_DEEPFM_RING_EARLY>(side_at<0>(staged(st_index, st_issue, st_store, st_fm))), nullptr, nullptr,
                                    fm_lds);
  MLP_MARK(4 * RK_MLP_MAX_LAYERS + 1, k_t0);
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 3);
  MLP_FLUSH(tid);
}

}  // namespace rk

using namespace rk;

#ifdef RK_MLP_PHASES
// Timing build only (tools/dcn_phases.py, MODEL=deepfm): this module's phase counters.
RK_API int rk_debug_deepfm_phases(unsigned long long* marks, int32_t nwg, unsigned* wave_marks) {
  if (nwg < 0 || nwg > kMlpMarkWG) return 1;
  if (hipMemcpyFromSymbol(marks, HIP_SYMBOL(g_mlp_marks), sizeof(g_mlp_marks[0]) * nwg) != hipSuccess) return 1;
  if (wave_marks &&
      hipMemcpyFromSymbol(wave_marks, HIP_SYMBOL(g_mlp_wave_marks), sizeof(g_mlp_wave_marks[0]) * nwg) != hipSuccess)
    return 1;
  return 0;
}
#endif

static int deepfm_forward_impl(const rk_segment* fields, const float* const* first, const int64_t* first_ld,
                               int32_t num_fields, int32_t dim, int64_t batch, const rk_mlp_layer* layers,
                               int32_t nlayers, const rk_epilogue* head, float* fm1, float* fm2, void* stream) {
  if (!fields || num_fields <= 0 || num_fields > kDfMaxFields)
    return fail(RK_ERR_UNSUPPORTED, "rk_deepfm_forward: %d fields (max %d)", num_fields, kDfMaxFields);
  if (dim < 4 || dim > 256 || (dim & (dim - 1)))
    return fail(RK_ERR_UNSUPPORTED, "rk_deepfm_forward: dim %d must be a power of two in [4, 256]", dim);
  if (!layers || !head || !head->head_w || !head->head_b || !head->final_w || !head->final_b || !fm1 || !fm2 ||
      batch < 0)
    return fail(RK_ERR_INVALID, "rk_deepfm_forward: bad arguments (head with final_w / final_b, fm1, fm2)");
  const int K0 = num_fields * dim;
  DfArgsFo a = {};
  a.head = *head;
  a.head.fm1 = fm1;  // selects the FM combine; the values come from LDS
  a.head.fm2 = fm2;
  a.head.head_partial = nullptr;
  int need0 = 0, need1 = 0;
  if (int e = mlp_validate(layers, nlayers, K0, a.head, &need0, &need1, "rk_deepfm_forward")) return e;
  // the compiled plan: 960 -> 512 -> 256 -> 128 (configs[1]: 30 fields x 32, hidden [512, 256, 128])
  if (nlayers != kDfLayers || pad64(K0) != StreamPlanK960::KC0 * 16 || stream_plan_for(layers, nlayers, 64) != kStreamK64)
    return fail(RK_ERR_UNSUPPORTED,
                "rk_deepfm_forward: no compiled plan for K0 %d and this layer stack (960 -> 512 -> 256 -> 128)", K0);
  uint32_t* flags = device_flags();
  if (!flags) return fail(RK_ERR_RUNTIME, "rk_deepfm_forward: device not initialised (rk_init)");
  for (int f = 0; f < num_fields; ++f) {
    const rk_segment& s = fields[f];
    if (!s.src || (s.idx && (s.rows <= 0 || s.idx_stride != 1)) || s.dim != dim ||
        s.src_ld < (first ? dim : dim + 1) || s.src_ld % 4 || !aligned16(s.src) || s.out_col != f * dim)
      return fail(RK_ERR_INVALID,
                  "rk_deepfm_forward: field %d is not a packed [rows, >= dim+1] table (unit-stride indices, or "
                  "none: a dense block of packed rows; with separate first-order sources, rows of >= dim) at "
                  "column f*dim",
                  f);
    a.src[f] = s.src;
    a.ld[f] = s.src_ld;
    if (first) {
      if (first[f] && (!first_ld || first_ld[f] < 0))
        return fail(RK_ERR_INVALID, "rk_deepfm_forward_fo: field %d first-order stride", f);
      a.fo[f] = first[f];
      a.fo_ld[f] = first[f] ? first_ld[f] : 0;
    }
    if (s.idx) {
      a.idx[f] = s.idx;
      a.istride[f] = 1;
      a.rows[f] = s.rows;
    } else {
      a.idx[f] = reinterpret_cast<const int64_t*>(flags);
      a.istride[f] = 0;
      a.rows[f] = batch;
      a.dense_mask |= 1u << f;
    }
  }
  for (int l = 0; l < kDfLayers; ++l) a.L[l] = layers[l];
  a.F = num_fields;
  a.dim_shift = __builtin_ctz((unsigned)dim);
  a.M = batch;
  a.fm1 = fm1;
  a.fm2 = fm2;
  a.flags = flags;
  if (batch == 0) return RK_OK;
  // 32-row workgroups once the batch gives every CU at least one (RANKOPS_DEEPFM_ROW_TILES = 1 / 2
  // forces either); layer 0 in place then: buf0 holds the input and layers 0 and 2, buf1 layer 1
  int rt = (batch + 2 * kMlpRows - 1) / (2 * kMlpRows) >= num_cus() ? 2 : 1;
  if (const char* e = getenv("RANKOPS_DEEPFM_ROW_TILES")) rt = atoi(e) == 2 ? 2 : atoi(e) == 1 ? 1 : rt;
  const int rows_wg = kMlpRows * rt;
  int odd = kMlpPad;  // widths of the odd layers (buf1 under IP0)
  for (int l = 1; l < nlayers; l += 2) odd = std::max(odd, pad64(layers[l].n));
  a.ld0 = (rt == 2 ? std::max(need0, need1) : need0) + kMlpLdPad;
  a.ld1 = (rt == 2 ? odd : need1) + kMlpLdPad;
  a.off1 = rows_wg * a.ld0;
  a.off_fm = a.off1 + rows_wg * a.ld1;
  size_t shm = (size_t)(a.off_fm + 2 * rows_wg) * sizeof(float);
  if (rt == 2 && shm > 160 * 1024 - kStreamStaticLds) {  // (the compiled plan fits; other widths fall back)
    rt = 1;
    a.ld0 = need0 + kMlpLdPad;
    a.ld1 = need1 + kMlpLdPad;
    a.off1 = kMlpRows * a.ld0;
    a.off_fm = a.off1 + kMlpRows * a.ld1;
    shm = (size_t)(a.off_fm + 2 * kMlpRows) * sizeof(float);
  }
  if (shm > 160 * 1024 - kStreamStaticLds) return fail(RK_ERR_UNSUPPORTED, "rk_deepfm_forward: widths need %zu B of LDS", shm);
  const int64_t blocks = (batch + kMlpRows * rt - 1) / (kMlpRows * rt);
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_deepfm_forward: batch too large");
  auto go = [&](auto kern, const auto& args) {
    raise_lds_limit((const void*)kern, 160 * 1024);
    kern<<<(unsigned)blocks, kMlpThreads, shm, (hipStream_t)stream>>>(args);
  };
  const DfArgs& base = a;
  if (first)
    rt == 2 ? go(deepfm_fused_kernel<StreamPlanK960, 2, true>, a) : go(deepfm_fused_kernel<StreamPlanK960, 1, true>, a);
  else
    rt == 2 ? go(deepfm_fused_kernel<StreamPlanK960, 2, false>, base)
            : go(deepfm_fused_kernel<StreamPlanK960, 1, false>, base);
  return check_launch("rk_deepfm_forward");
}

RK_API int rk_deepfm_forward(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch,
                             const rk_mlp_layer* layers, int32_t nlayers, const rk_epilogue* head, float* fm1,
                             float* fm2, void* stream) {
  return deepfm_forward_impl(fields, nullptr, nullptr, num_fields, dim, batch, layers, nlayers, head, fm1, fm2,
                             stream);
}

RK_API int rk_deepfm_forward_fo(const rk_segment* fields, const float* const* first, const int64_t* first_ld,
                                int32_t num_fields, int32_t dim, int64_t batch, const rk_mlp_layer* layers,
                                int32_t nlayers, const rk_epilogue* head, float* fm1, float* fm2, void* stream) {
  if (!first) return fail(RK_ERR_INVALID, "rk_deepfm_forward_fo: null first-order source array");
  return deepfm_forward_impl(fields, first, first_ld, num_fields, dim, batch, layers, nlayers, head, fm1, fm2, stream);
}
