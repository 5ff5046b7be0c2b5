// Embedding gather + concat, DCN cross network, DeepFM FM, DIN l2 term, BN folding.
//
// Reference semantics (file:line in the reference snapshot):
//   concat:  nn.Embedding(idx) per field, torch.cat([dense, emb...], 1)    dcn.py:163-169
//   cross:   x_{l+1} = x0 * (x_l @ w_l) + b_l^T + x_l                       dcn.py:47-49
//   FM:      fm1 = sum_f w_f[idx_f]; fm2 = 0.5*sum_d((sum_f e)^2 - sum_f e^2) deepfm.py:122-140
//   l2:      lambda * mean_b ||[cat_emb, target, att]_b||_2                 din.py:318-322
#include <cstdlib>

#include "common.h"

namespace rk {

// ------------------------------------------------------------------------------------
// Generic concat gather: out[b, col] for every column covered by a segment.
// Columns are handled in units of V floats (V = 4 when every segment is 16-B clean).
// ------------------------------------------------------------------------------------
constexpr int kConcatThreads = 256;
constexpr int kConcatMaxUnits = 4096;

template <int V>
__global__ __launch_bounds__(kConcatThreads) void concat_gather_kernel(
    SegTable segs, int nseg, int64_t batch, int width_units, int rows_per_block, float* __restrict__ out,
    int64_t ld_out, uint32_t* flags) {
  __shared__ uint8_t col_seg[kConcatMaxUnits];
  __shared__ uint16_t col_off[kConcatMaxUnits];
  for (int c = threadIdx.x; c < width_units; c += kConcatThreads) {
    uint8_t s_hit = 255;
    uint16_t off = 0;
    for (int s = 0; s < nseg; ++s) {
      const int lo = segs.s[s].out_col / V, hi = (segs.s[s].out_col + segs.s[s].dim) / V;
      if (c >= lo && c < hi) {
        s_hit = (uint8_t)s;
        off = (uint16_t)(c - lo);
      }
    }
    col_seg[c] = s_hit;
    col_off[c] = off;
  }
  __syncthreads();

  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  if (r0 >= batch) return;
  const int rows = (int)min<int64_t>(rows_per_block, batch - r0);
  const int total = rows * width_units;
  for (int e = threadIdx.x; e < total; e += kConcatThreads) {
    const int rr = e / width_units;
    const int c = e - rr * width_units;
    const int s = col_seg[c];
    if (s == 255) continue;
    const int64_t b = r0 + rr;
    const rk_segment& sg = segs.s[s];
    const float* row = segment_row(sg, b, flags);
    float* dst = out + b * ld_out + (int64_t)c * V;
    if constexpr (V == 4) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (row) v = *reinterpret_cast<const f32x4*>(row + (int64_t)col_off[c] * 4);
      *reinterpret_cast<f32x4*>(dst) = v;
    } else {
      *dst = row ? row[col_off[c]] : 0.f;
    }
  }
}

// ------------------------------------------------------------------------------------
// DCN: one wave per sample row; lane c owns column c (width <= 256, 4 columns/lane).
// ------------------------------------------------------------------------------------
constexpr int kCrossMaxPerLane = 4;

__global__ __launch_bounds__(256) void dcn_cross_kernel(SegTable segs, int nseg, int64_t batch, int width,
                                                        const float* __restrict__ cross_w,
                                                        const float* __restrict__ cross_b, int num_layers,
                                                        const float* __restrict__ head_w, float* __restrict__ x0_out,
                                                        int64_t ld_x0, const float* __restrict__ xl_in,
                                                        int64_t ld_xl_in, float* __restrict__ xl_out,
                                                        int64_t ld_xl_out, float* __restrict__ partial,
                                                        uint32_t* flags) {
  const int lane = threadIdx.x & 63;
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int nwaves = (gridDim.x * blockDim.x) >> 6;
  int seg_of[kCrossMaxPerLane], off_of[kCrossMaxPerLane];
#pragma unroll
  for (int j = 0; j < kCrossMaxPerLane; ++j) {
    const int c = lane + 64 * j;
    seg_of[j] = -1;
    off_of[j] = 0;
    for (int s = 0; s < nseg; ++s)
      if (c < width && c >= segs.s[s].out_col && c < segs.s[s].out_col + segs.s[s].dim) {
        seg_of[j] = s;
        off_of[j] = c - segs.s[s].out_col;
      }
  }
  for (int64_t b = wave; b < batch; b += nwaves) {
    float x0[kCrossMaxPerLane], xl[kCrossMaxPerLane];
#pragma unroll
    for (int j = 0; j < kCrossMaxPerLane; ++j) {
      float v = 0.f;
      if (seg_of[j] >= 0) {
        const float* row = segment_row(segs.s[seg_of[j]], b, flags);
        if (row) v = row[off_of[j]];
      }
      x0[j] = v;
      const int c = lane + 64 * j;
      xl[j] = (xl_in && c < width) ? xl_in[b * ld_xl_in + c] : v;
      if (x0_out && c < width) x0_out[b * ld_x0 + c] = v;
    }
    for (int l = 0; l < num_layers; ++l) {
      float d = 0.f;
#pragma unroll
      for (int j = 0; j < kCrossMaxPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) d = fmaf(xl[j], cross_w[(int64_t)l * width + c], d);
      }
      d = wave_sum(d);
#pragma unroll
      for (int j = 0; j < kCrossMaxPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) {
          float t = x0[j] * d;                      // torch.mul(x0, xl_wl)
          t = t + cross_b[(int64_t)l * width + c];  // + bl.t()
          xl[j] = t + xl[j];                        // + xl
        }
      }
    }
    if (xl_out) {
#pragma unroll
      for (int j = 0; j < kCrossMaxPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) xl_out[b * ld_xl_out + c] = xl[j];
      }
    }
    if (partial) {
      float p = 0.f;
#pragma unroll
      for (int j = 0; j < kCrossMaxPerLane; ++j) {
        const int c = lane + 64 * j;
        if (c < width) p = fmaf(xl[j], head_w[c], p);
      }
      p = wave_sum(p);
      if (lane == 0) partial[b] = p;
    }
  }
}

// ------------------------------------------------------------------------------------
// DeepFM FM, sample-major: one wave per sample.  Lane = (field slot j, float4 quad q) with
// G = dim/4 quads and J = 64/G field slots, so one wave-instruction fetches J whole rows and the
// sample's deep-input row (fields in column order) is written as contiguous bytes.  Every index
// load, then every row load of the sample is issued before the first use; sum and sum of squares
// are reduced across field slots by xor-shuffles (no LDS, no barrier), then across quads.
// Measured against a field-major block layout (4 waves x 8 samples, LDS combine): 1.9x faster at
// batch 65536 over 30 x 1e6-row tables (tools/gather_probe.hip).
// ------------------------------------------------------------------------------------
constexpr int kFmMaxFields = 32;
constexpr int kFmjU = 6;  // fields per round of the field-major kernel
// descriptor slots: the field-major kernel's fully unrolled rounds read slots up to the next
// multiple of kFmjU (36); slots past the last field repeat it (filled on the host)
constexpr int kFmSlots = (kFmMaxFields + kFmjU - 1) / kFmjU * kFmjU;
// Per-field descriptors as arrays (one pointer/stride per field), so that every lane's loads of
// its field's descriptor, index and row are branch-free and all issue before the first wait.
struct FmTables {
  const float* src2[kFmSlots];
  const float* src1[kFmSlots];
  const int64_t* idx2[kFmSlots];
  const int64_t* idx1[kFmSlots];
  int64_t istride2[kFmSlots], istride1[kFmSlots];
  int64_t ld2[kFmSlots], ld1[kFmSlots];
  int64_t rows2[kFmSlots], rows1[kFmSlots];
  int32_t col[kFmSlots];
};
static_assert(sizeof(FmTables) + 64 <= 4096, "kernel arguments beyond 4 KiB");

// Slots [F, kFmSlots) repeat field F - 1 (the field-major kernel's rounds past the last field read
// a valid descriptor and discard the values).
inline void fm_fill_slots(FmTables& t, int F) {
  for (int f = F; f < kFmSlots; ++f) {
    t.src2[f] = t.src2[F - 1];
    t.src1[f] = t.src1[F - 1];
    t.idx2[f] = t.idx2[F - 1];
    t.idx1[f] = t.idx1[F - 1];
    t.istride2[f] = t.istride2[F - 1];
    t.istride1[f] = t.istride1[F - 1];
    t.ld2[f] = t.ld2[F - 1];
    t.ld1[f] = t.ld1[F - 1];
    t.rows2[f] = t.rows2[F - 1];
    t.rows1[f] = t.rows1[F - 1];
    t.col[f] = t.col[F - 1];
  }
}

// Modes: kFmTables — embedding tables, any index/row strides; kFmPacked — embedding tables with
// one shared unit-stride index array per field (first- and second-order) and contiguous rows
// (nn.Embedding's layout, DeepFM's call): 5 descriptor words per field instead of 11;
// kFmDense — row b of src (the sharded path's received rows); kFmRowPacked — one packed
// [V, RS] table per field (rk_fm_pack_table: the dim second-order floats, then the first-order
// weight at column dim), one unit-stride index array: the weight shares the row's line pair
// instead of costing a lone 4-B load (and its own 128-B line) in a separate [V, 1] table.
constexpr int kFmTables = 0, kFmPacked = 1, kFmDense = 2, kFmRowPacked = 3;
template <int G, int MODE>  // G = quads per row = dim / 4
__global__ __launch_bounds__(256) void fm_gather_kernel(FmTables t, int F, int64_t batch, float* __restrict__ deep_in,
                                                        int64_t ld_deep, float* __restrict__ fm1,
                                                        float* __restrict__ fm2, uint32_t* flags) {
  constexpr int J = 64 / G;                                // field slots per instruction
  constexpr int NI = (kFmMaxFields + J - 1) / J;           // instructions for the widest sample
  constexpr int CH = NI < 8 ? NI : 8;                      // instructions in flight per chunk
  const int lane = threadIdx.x & 63, q = lane % G, j = lane / G;
  const int64_t b = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (b >= batch) return;
  f32x4 s = {0.f, 0.f, 0.f, 0.f}, sq = {0.f, 0.f, 0.f, 0.f};
  float fo = 0.f;
  bool oob = false;
  const int ni = (F + J - 1) / J;
  for (int c0 = 0; c0 < ni; c0 += CH) {
    int fi[CH];
    bool live[CH];
    int64_t r2[CH], r1[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {  // slots past the last field re-read field F-1 and are masked
      const int f = (c0 + i) * J + j;
      live[i] = f < F;
      fi[i] = live[i] ? f : F - 1;
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if constexpr (MODE == kFmDense) {
        r2[i] = r1[i] = b;
      } else if constexpr (MODE == kFmPacked || MODE == kFmRowPacked) {
        r2[i] = r1[i] = t.idx2[fi[i]][b];
      } else {
        r2[i] = t.idx2[fi[i]][b * t.istride2[fi[i]]];
        r1[i] = t.idx1[fi[i]][b * t.istride1[fi[i]]];
      }
    }
    f32x4 v[CH];
    float w1[CH];
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      constexpr bool kDense = MODE == kFmDense, kPacked = MODE == kFmPacked, kRow = MODE == kFmRowPacked;
      const bool ok2 = kDense || (uint64_t)r2[i] < (uint64_t)t.rows2[fi[i]];
      const bool ok1 = kDense || kPacked || kRow ? ok2 : (uint64_t)r1[i] < (uint64_t)t.rows1[fi[i]];
      oob |= live[i] && !(ok2 && ok1);
      const int64_t ld2 = kPacked ? 4 * G : t.ld2[fi[i]], ld1 = kPacked ? 1 : t.ld1[fi[i]];
      // (nontemporal row loads measured no faster: 143 vs 144 us at batch 65536)
      const float* row = t.src2[fi[i]] + (ok2 ? r2[i] : 0) * ld2;
      v[i] = *reinterpret_cast<const f32x4*>(row + 4 * q);
      if constexpr (kRow)
        w1[i] = row[4 * G];  // the first-order weight sits right after the row's dim floats
      else
        w1[i] = t.src1[fi[i]][(ok1 ? r1[i] : 0) * ld1];
      if (!(live[i] && ok2)) v[i] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (!(live[i] && ok1) || q != 0) w1[i] = 0.f;
    }
#pragma unroll
    for (int i = 0; i < CH; ++i) {
      if (live[i]) *reinterpret_cast<f32x4*>(deep_in + b * ld_deep + t.col[fi[i]] + 4 * q) = v[i];
      s += v[i];
      sq += v[i] * v[i];
      fo += w1[i];
    }
  }
  if (MODE != kFmDense && oob) flag_oob(flags);
#pragma unroll
  for (int o = G; o < 64; o <<= 1) {
    s.x += __shfl_xor(s.x, o, kWave);
    s.y += __shfl_xor(s.y, o, kWave);
    s.z += __shfl_xor(s.z, o, kWave);
    s.w += __shfl_xor(s.w, o, kWave);
    sq.x += __shfl_xor(sq.x, o, kWave);
    sq.y += __shfl_xor(sq.y, o, kWave);
    sq.z += __shfl_xor(sq.z, o, kWave);
    sq.w += __shfl_xor(sq.w, o, kWave);
    fo += __shfl_xor(fo, o, kWave);
  }
  float part = (s.x * s.x - sq.x) + (s.y * s.y - sq.y) + (s.z * s.z - sq.z) + (s.w * s.w - sq.w);
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) part += __shfl_xor(part, o, kWave);
  if (lane == 0) {
    fm2[b] = 0.5f * part;
    fm1[b] = fo;
  }
}

// ------------------------------------------------------------------------------------
// The same gather FIELD-MAJOR (round 6, large batches): a wave owns J = 64 / G samples (lane =
// sample slot j, quad q) and walks the fields in order, U fields' rows in flight per round, the
// next round's indices issued before this round's rows are consumed.  What it buys: on gfx950
// every random access costs one 128-B L2-to-memory request whatever its width (a 4-B first-order
// weight as much as a 128-B row: tools/gather_probe2.hip, profiles/r06/gather_calib), and the
// request rate bounds the gather.  Swept field by field by every resident wave at about the same
// time, field f's first-order table (4 MB at 1e6 rows) is re-read from the on-die caches while the
// field is being swept, instead of costing a request per lookup as in the sample-major walk.
// The deep-input rows go out as nontemporal stores (streamed past L2, which then keeps the
// first-order and index lines).  At batch 65,536 over configs[1]'s tables: 109 us (U = 6) against
// 131 us with ordinary stores and no index prefetch, and 138 us for the sample-major walk.
// Per sample the sums run over the fields in order (a different association from
// fm_gather_kernel's slot-then-shuffle order: the two agree to fp32 rounding, not bit for bit).
// ------------------------------------------------------------------------------------
template <int G, int MODE, int U, bool NTS, bool PF_FIRST = true>
__global__ __launch_bounds__(256) void fm_gather_fmaj_kernel(FmTables t, int F, int64_t batch,
                                                             float* __restrict__ deep_in, int64_t ld_deep,
                                                             float* __restrict__ fm1, float* __restrict__ fm2,
                                                             uint32_t* flags) {
  static_assert(kFmSlots % U == 0, "rounds must tile the descriptor slots");
  constexpr int J = 64 / G;
  constexpr bool kDense = MODE == kFmDense, kPacked = MODE == kFmPacked, kRow = MODE == kFmRowPacked;
  const int lane = threadIdx.x & 63, q = lane % G, j = lane / G;
  const int64_t b = (((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6) * J + j;
  const bool live = b < batch;
  const int64_t bb = live ? b : 0;  // dead slots re-read sample 0 and write nothing
  f32x4 s = {0.f, 0.f, 0.f, 0.f}, sq = {0.f, 0.f, 0.f, 0.f};
  float fo = 0.f;
  bool oob = false;
  int64_t r2[U], r1[U];
  // the rounds are unrolled over every descriptor slot, so each field's descriptor sits at a
  // constant kernel-argument offset (one batch of scalar loads per round, no dependent address
  // arithmetic); rounds past the last field are skipped by a wave-uniform branch
  auto load_idx = [&](int f0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = f0 + u;
      if constexpr (kDense) {
        r2[u] = r1[u] = bb;
      } else if constexpr (kPacked || kRow) {
        r2[u] = r1[u] = t.idx2[f][bb];
      } else {
        r2[u] = t.idx2[f][bb * t.istride2[f]];
        r1[u] = t.idx1[f][bb * t.istride1[f]];
      }
    }
  };
  load_idx(0);
#pragma unroll
  for (int f0 = 0; f0 < kFmSlots; f0 += U) {
    if (f0 >= F) break;
    f32x4 v[U];
    float w1[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int f = f0 + u;
      const bool lf = f < F;
      const bool ok2 = kDense || (uint64_t)r2[u] < (uint64_t)t.rows2[f];
      const bool ok1 = kDense || kPacked || kRow ? ok2 : (uint64_t)r1[u] < (uint64_t)t.rows1[f];
      oob |= live && lf && !(ok2 && ok1);
      const int64_t ld2 = kPacked ? 4 * G : t.ld2[f], ld1 = kPacked ? 1 : t.ld1[f];
      const float* row = t.src2[f] + (ok2 ? r2[u] : 0) * ld2;
      v[u] = *reinterpret_cast<const f32x4*>(row + 4 * q);
      if constexpr (kRow)
        w1[u] = row[4 * G];
      else
        w1[u] = t.src1[f][(ok1 ? r1[u] : 0) * ld1];
      if (!ok2) v[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
      if (!(lf && ok1) || q != 0) w1[u] = 0.f;
    }
    if (PF_FIRST && f0 + U < kFmSlots && f0 + U < F) load_idx(f0 + U);
    // straight-line stores (no branch: a join would make the compiler drain the whole vmcnt queue,
    // the next round's index loads included, behind the stores): a slot past the last field
    // repeats field F - 1 (descriptor, index, value) and rewrites its bytes; a dead sample slot
    // carries sample 0's values and rewrites sample 0's row — identical bytes either way.  The
    // sums take those slots with weight 0.
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row_b = live ? b : 0;
      f32x4* o = reinterpret_cast<f32x4*>(deep_in + row_b * ld_deep + t.col[f0 + u] + 4 * q);
      if constexpr (NTS)
        __builtin_nontemporal_store(v[u], o);
      else
        *o = v[u];
      const float m = f0 + u < F ? 1.f : 0.f;
      s += v[u] * m;
      sq += (v[u] * v[u]) * m;
      fo += w1[u];
    }
    if (!PF_FIRST && f0 + U < kFmSlots && f0 + U < F) load_idx(f0 + U);
  }
  if (!kDense && oob) flag_oob(flags);
  float part = (s.x * s.x - sq.x) + (s.y * s.y - sq.y) + (s.z * s.z - sq.z) + (s.w * s.w - sq.w);
#pragma unroll
  for (int o = 1; o < G; o <<= 1) part += __shfl_xor(part, o, kWave);
  if (live && q == 0) {
    fm2[b] = 0.5f * part;
    fm1[b] = fo;
  }
}

// ------------------------------------------------------------------------------------
// DIN l2 term: scale * mean_r ||x[r, col0:col0+ncols]||_2 — one deterministic workgroup.
// ------------------------------------------------------------------------------------
// Stage 1: block b sums the norms of rows b, b+G, ... (wave-strided, fixed order) into part[b].
constexpr int kL2Blocks = 512;
__global__ __launch_bounds__(256) void row_l2norm_partial_kernel(const float* __restrict__ x, int64_t ld,
                                                                 int64_t rows, int col0, int ncols,
                                                                 float* __restrict__ part) {
  __shared__ float wsum[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float acc = 0.f;
  for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < rows; r += (int64_t)gridDim.x * 4) {
    float ss = 0.f;
    for (int c = lane; c < ncols; c += 64) {
      const float v = x[r * ld + col0 + c];
      ss = fmaf(v, v, ss);
    }
    acc += sqrtf(wave_sum(ss));
  }
  if (lane == 0) wsum[wave] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
}

// Stage 2: one wave adds the block partials in a fixed tree order.
__global__ __launch_bounds__(64) void row_l2norm_final_kernel(const float* __restrict__ part, int nparts,
                                                              int64_t rows, float scale, float* __restrict__ out) {
  float t = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 64) t += part[i];
  t = wave_sum(t);
  if (threadIdx.x == 0) out[0] = scale * (t / (float)rows);
}

// Packed FM table: out[r, 0:dim] = second[r, :], out[r, dim] = first[r, 0], zero pad to ld_out.
// One thread per float4 of the output (ld_out % 4 == 0), a one-off layout pass per weight version.
__global__ __launch_bounds__(256) void fm_pack_table_kernel(const float* __restrict__ second, int64_t ld2,
                                                            const float* __restrict__ first, int64_t ld1,
                                                            int64_t rows, int dim, float* __restrict__ out,
                                                            int64_t ld_out) {
  const int quads = (int)(ld_out / 4);
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows * quads) return;
  const int64_t r = i / quads;
  const int c0 = (int)(i - r * quads) * 4;
  f32x4 v;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = c0 + k;
    v[k] = c < dim ? second[r * ld2 + c] : c == dim ? first[r * ld1] : 0.f;
  }
  *reinterpret_cast<f32x4*>(out + r * ld_out + c0) = v;
}

__global__ void bn_fold_kernel(const float* __restrict__ mean, const float* __restrict__ var,
                               const float* __restrict__ weight, const float* __restrict__ bias, float eps, int n,
                               float* __restrict__ scale, float* __restrict__ shift) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float invstd = 1.0f / sqrtf(var[i] + eps);
  const float a = weight ? invstd * weight[i] : invstd;
  scale[i] = a;
  shift[i] = (bias ? bias[i] : 0.f) - mean[i] * a;
}


int launch_l2_final(const float* part, int n, int64_t rows, float scale, float* out, hipStream_t st) {
  row_l2norm_final_kernel<<<1, 64, 0, st>>>(part, n, rows, scale, out);
  return check_launch("l2 final");
}

static int check_segments(const rk_segment* segs, int nseg, const char* what) {
  if (!segs || nseg <= 0 || nseg > RK_MAX_SEGMENTS) return fail(RK_ERR_INVALID, "%s: bad segment count %d", what, nseg);
  for (int i = 0; i < nseg; ++i) {
    const rk_segment& s = segs[i];
    if (!s.src || s.dim <= 0 || s.out_col < 0)
      return fail(RK_ERR_INVALID, "%s: segment %d invalid (src=%p dim=%d col=%d)", what, i, s.src, s.dim, s.out_col);
    if (s.idx && s.rows <= 0) return fail(RK_ERR_INVALID, "%s: segment %d has no rows", what, i);
  }
  return RK_OK;
}

int launch_fm_gather(const FmTables& t, int mode, int num_fields, int G, int64_t batch, float* deep_in,
                     int64_t ld_deep, float* fm1, float* fm2, hipStream_t st);

}  // namespace rk

using namespace rk;

RK_API int rk_concat_gather(const rk_segment* segs, int32_t nseg, int64_t batch, float* out, int64_t ld_out,
                            void* stream) {
  if (int e = check_segments(segs, nseg, "rk_concat_gather")) return e;
  if (batch < 0 || !out) return fail(RK_ERR_INVALID, "rk_concat_gather: bad batch/out");
  if (batch == 0) return RK_OK;
  SegTable t;
  int width = 0;
  bool vec = aligned16(out) && (ld_out % 4 == 0);
  for (int i = 0; i < nseg; ++i) {
    t.s[i] = segs[i];
    width = std::max(width, segs[i].out_col + segs[i].dim);
    vec = vec && segs[i].dim % 4 == 0 && segs[i].out_col % 4 == 0 && segs[i].src_ld % 4 == 0 && aligned16(segs[i].src);
  }
  if (width > ld_out) return fail(RK_ERR_INVALID, "rk_concat_gather: width %d exceeds ld_out %lld", width, (long long)ld_out);
  const int V = vec ? 4 : 1;
  const int units = (width + V - 1) / V;
  if (units > kConcatMaxUnits) return fail(RK_ERR_UNSUPPORTED, "rk_concat_gather: width %d too large", width);
  // enough blocks to cover every CU several times, each still moving >= ~1 KB
  const int64_t want_blocks = 4 * (int64_t)num_cus();
  int rows_per_block = (int)std::max<int64_t>(1, std::min<int64_t>(4096 / units, (batch + want_blocks - 1) / want_blocks));
  rows_per_block = std::max(rows_per_block, std::max(1, 256 / units));
  const int64_t blocks = (batch + rows_per_block - 1) / rows_per_block;
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_concat_gather: batch too large");
  hipStream_t st = (hipStream_t)stream;
  if (vec)
    concat_gather_kernel<4><<<(unsigned)blocks, kConcatThreads, 0, st>>>(t, nseg, batch, units, rows_per_block, out,
                                                                          ld_out, device_flags());
  else
    concat_gather_kernel<1><<<(unsigned)blocks, kConcatThreads, 0, st>>>(t, nseg, batch, units, rows_per_block, out,
                                                                          ld_out, device_flags());
  return check_launch("rk_concat_gather");
}

RK_API int rk_dcn_cross(const rk_segment* segs, int32_t nseg, int64_t batch, int32_t width, const float* cross_w,
                        const float* cross_b, int32_t num_layers, const float* head_w, float* x0, int64_t ld_x0,
                        const float* xl_in, int64_t ld_xl_in, float* xl_out, int64_t ld_xl_out,
                        float* cross_partial, void* stream) {
  if (int e = check_segments(segs, nseg, "rk_dcn_cross")) return e;
  if (width <= 0 || width > 64 * kCrossMaxPerLane)
    return fail(RK_ERR_UNSUPPORTED, "rk_dcn_cross: width %d outside [1, %d]", width, 64 * kCrossMaxPerLane);
  if (num_layers < 0 || (num_layers > 0 && (!cross_w || !cross_b)) || (x0 && ld_x0 < width) ||
      (xl_in && ld_xl_in < width) || (xl_out && ld_xl_out < width) || (cross_partial && !head_w))
    return fail(RK_ERR_INVALID, "rk_dcn_cross: bad arguments");
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "rk_dcn_cross: negative batch");
  SegTable t;
  for (int i = 0; i < nseg; ++i) t.s[i] = segs[i];
  const int64_t waves = std::min<int64_t>(batch, (int64_t)num_cus() * 32);
  const unsigned blocks = (unsigned)((waves + 3) / 4);
  dcn_cross_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(t, nseg, batch, width, cross_w, cross_b, num_layers,
                                                            head_w, x0, ld_x0, xl_in, ld_xl_in, xl_out, ld_xl_out,
                                                            cross_partial, device_flags());
  return check_launch("rk_dcn_cross");
}

RK_API int rk_fm_gather(const rk_segment* second_order, const rk_segment* first_order, int32_t num_fields,
                        int32_t dim, int64_t batch, float* deep_in, int64_t ld_deep, float* fm1, float* fm2,
                        void* stream) {
  if (num_fields <= 0 || num_fields > kFmMaxFields)
    return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather: %d fields (max %d)", num_fields, kFmMaxFields);
  if (int e = check_segments(second_order, num_fields, "rk_fm_gather(second)")) return e;
  if (int e = check_segments(first_order, num_fields, "rk_fm_gather(first)")) return e;
  if (!deep_in || !fm1 || !fm2 || ld_deep % 4 != 0 || !aligned16(deep_in))
    return fail(RK_ERR_INVALID, "rk_fm_gather: outputs must be non-null, 16-B aligned, ld %% 4 == 0");
  if (dim % 4 != 0 || dim < 4 || dim > 256)
    return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather: dim %d must be a multiple of 4 in [4, 256]", dim);
  const int G = dim / 4;
  if (G & (G - 1)) return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather: dim/4 = %d must be a power of two", G);
  FmTables t;
  int dense = 0;
  for (int f = 0; f < num_fields; ++f) {
    const rk_segment& s = second_order[f];
    const rk_segment& w = first_order[f];
    if (s.dim != dim || s.out_col % 4 || s.src_ld % 4 || !aligned16(s.src) || s.out_col + dim > ld_deep)
      return fail(RK_ERR_INVALID, "rk_fm_gather: field %d layout not 16-B clean", f);
    if (w.dim != 1) return fail(RK_ERR_INVALID, "rk_fm_gather: first-order field %d dim != 1", f);
    dense += (s.idx == nullptr) + (w.idx == nullptr);
    t.src2[f] = s.src;
    t.src1[f] = w.src;
    t.idx2[f] = s.idx;
    t.idx1[f] = w.idx;
    t.istride2[f] = s.idx_stride;
    t.istride1[f] = w.idx_stride;
    t.ld2[f] = s.src_ld;
    t.ld1[f] = w.src_ld;
    t.rows2[f] = s.rows;
    t.rows1[f] = w.rows;
    t.col[f] = s.out_col;
  }
  if (dense != 0 && dense != 2 * num_fields)
    return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather: segments must be all tables or all dense");
  bool packed = dense == 0;
  for (int f = 0; f < num_fields && packed; ++f) {
    const rk_segment& s = second_order[f];
    const rk_segment& w = first_order[f];
    packed = s.idx == w.idx && s.idx_stride == 1 && w.idx_stride == 1 && s.src_ld == dim && w.src_ld == 1;
  }
  if (packed)  // one bounds check per field: the smaller of the two tables
    for (int f = 0; f < num_fields; ++f) t.rows2[f] = std::min(t.rows2[f], t.rows1[f]);
  const int mode = dense ? kFmDense : packed ? kFmPacked : kFmTables;
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "rk_fm_gather: negative batch");
  return launch_fm_gather(t, mode, num_fields, G, batch, deep_in, ld_deep, fm1, fm2, (hipStream_t)stream);
}

RK_API int rk_fm_pack_table(const float* second, int64_t ld_second, const float* first, int64_t ld_first,
                            int64_t rows, int32_t dim, float* out, int64_t ld_out, void* stream) {
  if (!second || !first || !out || rows < 0 || dim <= 0 || ld_second < dim || ld_first < 1 || ld_out < dim + 1 ||
      ld_out % 4 != 0 || !aligned16(out))
    return fail(RK_ERR_INVALID, "rk_fm_pack_table: bad arguments (dim %d, ld_out %lld)", dim, (long long)ld_out);
  if (rows == 0) return RK_OK;
  const int64_t n = rows * (ld_out / 4);
  fm_pack_table_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(second, ld_second, first,
                                                                                    ld_first, rows, dim, out, ld_out);
  return check_launch("rk_fm_pack_table");
}

RK_API int rk_fm_gather_packed(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch,
                               float* deep_in, int64_t ld_deep, float* fm1, float* fm2, void* stream) {
  if (num_fields <= 0 || num_fields > kFmMaxFields)
    return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather_packed: %d fields (max %d)", num_fields, kFmMaxFields);
  if (int e = check_segments(fields, num_fields, "rk_fm_gather_packed")) return e;
  if (!deep_in || !fm1 || !fm2 || ld_deep % 4 != 0 || !aligned16(deep_in))
    return fail(RK_ERR_INVALID, "rk_fm_gather_packed: outputs must be non-null, 16-B aligned, ld %% 4 == 0");
  if (dim % 4 != 0 || dim < 4 || dim > 256 || ((dim / 4) & (dim / 4 - 1)))
    return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather_packed: dim %d must be 4 * a power of two <= 256", dim);
  FmTables t;
  for (int f = 0; f < num_fields; ++f) {
    const rk_segment& s = fields[f];
    if (!s.idx || s.idx_stride != 1 || s.dim != dim || s.src_ld < dim + 1 || s.src_ld % 4 || !aligned16(s.src) ||
        s.out_col % 4 || s.out_col + dim > ld_deep)
      return fail(RK_ERR_INVALID, "rk_fm_gather_packed: field %d is not a unit-stride packed [rows, >= dim+1] table",
                  f);
    t.src2[f] = t.src1[f] = s.src;
    t.idx2[f] = t.idx1[f] = s.idx;
    t.istride2[f] = t.istride1[f] = 1;
    t.ld2[f] = t.ld1[f] = s.src_ld;
    t.rows2[f] = t.rows1[f] = s.rows;
    t.col[f] = s.out_col;
  }
  if (batch <= 0) return batch == 0 ? RK_OK : fail(RK_ERR_INVALID, "rk_fm_gather_packed: negative batch");
  return launch_fm_gather(t, kFmRowPacked, num_fields, dim / 4, batch, deep_in, ld_deep, fm1, fm2,
                          (hipStream_t)stream);
}

namespace rk {
int launch_fm_gather(const FmTables& t0, int mode, int num_fields, int G, int64_t batch, float* deep_in,
                     int64_t ld_deep, float* fm1, float* fm2, hipStream_t st) {
  FmTables t = t0;
  fm_fill_slots(t, num_fields);
  uint32_t* fl = device_flags();
  // field-major from fmaj_min samples (RANKOPS_FM_FMAJ_MIN; 0 = never): at configs[1]'s 4,096 the
  // sample-major form is the faster (more waves, no sweep to share), at 65,536 the field-major one
  const int64_t fmaj_min = [] {
    const char* e = getenv("RANKOPS_FM_FMAJ_MIN");
    return e ? (int64_t)atoll(e) : (int64_t)16384;
  }();
  if (fmaj_min > 0 && batch >= fmaj_min) {
    const int64_t waves = (batch + 64 / G - 1) / (64 / G);
    const int64_t fblocks = (waves + 3) / 4;
    if (fblocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather: batch too large");
    // A/B switch (per call): RANKOPS_FM_FMAJ_VARIANT=1 issues the next round's indices after the
    // stores instead of before them; =2 also drops the nontemporal hint
    const char* ve = getenv("RANKOPS_FM_FMAJ_VARIANT");
    const int variant = ve ? atoi(ve) : 0;
#define RK_FMJ_LAUNCH(GG, MM)                                                                                   \
  do {                                                                                                          \
    if (variant == 1)                                                                                           \
      fm_gather_fmaj_kernel<GG, MM, kFmjU, true, false>                                                         \
          <<<(unsigned)fblocks, 256, 0, st>>>(t, num_fields, batch, deep_in, ld_deep, fm1, fm2, fl);           \
    else if (variant == 2)                                                                                      \
      fm_gather_fmaj_kernel<GG, MM, kFmjU, false, true>                                                         \
          <<<(unsigned)fblocks, 256, 0, st>>>(t, num_fields, batch, deep_in, ld_deep, fm1, fm2, fl);           \
    else                                                                                                        \
      fm_gather_fmaj_kernel<GG, MM, kFmjU, true, true>                                                          \
          <<<(unsigned)fblocks, 256, 0, st>>>(t, num_fields, batch, deep_in, ld_deep, fm1, fm2, fl);           \
  } while (0)
#define RK_FMJ_CASE(GG)          \
  case GG:                       \
    if (mode == kFmDense)        \
      RK_FMJ_LAUNCH(GG, kFmDense); \
    else if (mode == kFmPacked)  \
      RK_FMJ_LAUNCH(GG, kFmPacked); \
    else if (mode == kFmRowPacked) \
      RK_FMJ_LAUNCH(GG, kFmRowPacked); \
    else                         \
      RK_FMJ_LAUNCH(GG, kFmTables); \
    break;
    switch (G) {
      RK_FMJ_CASE(1)
      RK_FMJ_CASE(2)
      RK_FMJ_CASE(4)
      RK_FMJ_CASE(8)
      RK_FMJ_CASE(16)
      RK_FMJ_CASE(32)
      RK_FMJ_CASE(64)
      default:
        return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather: dim %d", 4 * G);
    }
#undef RK_FMJ_CASE
#undef RK_FMJ_LAUNCH
    return check_launch("rk_fm_gather");
  }
  const int64_t blocks = (batch + 3) / 4;  // one wave per sample, 4 waves per workgroup
#define RK_FM_LAUNCH(GG, MM) \
  fm_gather_kernel<GG, MM><<<(unsigned)blocks, 256, 0, st>>>(t, num_fields, batch, deep_in, ld_deep, fm1, fm2, fl)
#define RK_FM_CASE(GG)                                   \
  case GG:                                               \
    if (mode == kFmDense)                                \
      RK_FM_LAUNCH(GG, kFmDense);                        \
    else if (mode == kFmPacked)                          \
      RK_FM_LAUNCH(GG, kFmPacked);                       \
    else if (mode == kFmRowPacked)                       \
      RK_FM_LAUNCH(GG, kFmRowPacked);                    \
    else                                                 \
      RK_FM_LAUNCH(GG, kFmTables);                       \
    break;
  switch (G) {
    RK_FM_CASE(1)
    RK_FM_CASE(2)
    RK_FM_CASE(4)
    RK_FM_CASE(8)
    RK_FM_CASE(16)
    RK_FM_CASE(32)
    RK_FM_CASE(64)
    default:
      return fail(RK_ERR_UNSUPPORTED, "rk_fm_gather: dim %d", 4 * G);
  }
#undef RK_FM_CASE
#undef RK_FM_LAUNCH
  return check_launch("rk_fm_gather");
}
}  // namespace rk

RK_API int rk_row_l2norm_mean(const float* x, int64_t ld, int64_t rows, int32_t col0, int32_t ncols, float scale,
                              float* workspace, float* out_scalar, void* stream) {
  if (!x || !out_scalar || !workspace || rows <= 0 || ncols <= 0 || col0 < 0 || col0 + ncols > ld)
    return fail(RK_ERR_INVALID, "rk_row_l2norm_mean: bad arguments");
  const int blocks = (int)std::min<int64_t>(kL2Blocks, (rows + 3) / 4);
  hipStream_t st = (hipStream_t)stream;
  row_l2norm_partial_kernel<<<blocks, 256, 0, st>>>(x, ld, rows, col0, ncols, workspace);
  row_l2norm_final_kernel<<<1, 64, 0, st>>>(workspace, blocks, rows, scale, out_scalar);
  return check_launch("rk_row_l2norm_mean");
}

RK_API int rk_bn_fold(const float* mean, const float* var, const float* weight, const float* bias, float eps,
                      int32_t n, float* scale, float* shift, void* stream) {
  if (!mean || !var || !scale || !shift || n <= 0) return fail(RK_ERR_INVALID, "rk_bn_fold: bad arguments");
  bn_fold_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(mean, var, weight, bias, eps, n, scale, shift);
  return check_launch("rk_bn_fold");
}
