// The two local steps around ShardedDeepFM's all-to-alls (rankops/sharded.py; the reference's
// DeepFM.forward, deepfm.py:121-151, is single-device — the table-wise sharding over the GPUs of
// one node is this build's own):
//
//  rk_shard_pack_indices  the index all-to-all's send buffer in one launch: the F per-field [B]
//                         int64 index columns of this rank's samples -> int32 blocks [r][b][f_r]
//                         (field slot q of the owner-major field list lands at
//                         B * start_r + b * F_r + j).  Replaces a stack + cat + cast per owner.
//  rk_shard_gather_rows   the row all-to-all's send buffer for one chunk of samples: for every
//                         source rank s and sample b of [b0, b0 + bc), the packed rows
//                         (rk_fm_pack_table layout, RS floats) of this rank's F_me fields at the
//                         int32 indices the source sent, [s][b'][j][RS], flattened over the
//                         output's float4s (kShardU loads in flight per lane).
//
// Both are HBM-bound byte movers: pack 12 B per (sample, field); gather 4 B of index + 2 x RS * 4 B
// per (row, field) (read the packed row, write it to the send buffer).
#include <cstdlib>

#include "common.h"

namespace rk {

constexpr int kShardMaxFields = 32;

struct ShardPackArgs {
  const int64_t* idx[kShardMaxFields];
  int64_t base[kShardMaxFields];  // B * start_r + j
  int32_t stride[kShardMaxFields];  // F_r
  int F;
  int64_t B;
  int32_t* out;
};

__global__ __launch_bounds__(256) void shard_pack_indices_kernel(ShardPackArgs a) {
  const int64_t n = a.B * a.F;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i / a.F;
    const int q = (int)(i - b * a.F);
    // an index outside [0, 2^31) would wrap to a valid row when narrowed: it goes out as -1,
    // which the owner's gather reads as a zero row and flags (RK_FLAG_INDEX_OOB)
    const int64_t v = a.idx[q][b];
    a.out[a.base[q] + b * a.stride[q]] = (v >= 0 && v <= (int64_t)INT32_MAX) ? (int32_t)v : -1;
  }
}

struct ShardGatherArgs {
  const float* src[kShardMaxFields];
  int64_t src_ld[kShardMaxFields], rows[kShardMaxFields];
  int F;       // this rank's fields
  int RS4;     // packed row length in float4s
  const int32_t* idx;  // [P][B_l][F] as received
  int64_t B_l, b0, bc;
  int P;
  float* out;  // [P][bc][F][RS]
  uint32_t* flags;
};

// Flattened over the output's float4s: thread i moves float4s i, i + n/U-stride, ... (kShardU of
// them, all loads issued before any store, so each lane keeps kShardU row reads in flight).  A
// float4 t of the output is (row r = t / per, field j, quad q); its index sits at
// idx[(s * B_l + b0 + r % bc) * F + j] with s = r / bc.  Every lane of a wave works (the old one-
// wave-per-row form left 28 of 64 lanes idle at 4 fields x 9 quads).
constexpr int kShardU = 4;

__global__ __launch_bounds__(256) void shard_gather_rows_kernel(ShardGatherArgs a) {
  const int per = a.F * a.RS4;
  const int64_t n4 = (int64_t)a.P * a.bc * per;
  const int64_t stride = (int64_t)gridDim.x * 256;
  int64_t t0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  f32x4* const out4 = reinterpret_cast<f32x4*>(a.out);
  for (; t0 < n4; t0 += stride * kShardU) {
    int64_t row[kShardU];
    int jj[kShardU], qq[kShardU];
#pragma unroll
    for (int u = 0; u < kShardU; ++u) {
      const int64_t t = t0 + u * stride;
      const int64_t tt = t < n4 ? t : 0;
      const int64_t r = tt / per;
      const int rem = (int)(tt - r * per);
      const int j = rem / a.RS4;
      const int64_t s = r / a.bc, bp = r - s * a.bc;
      jj[u] = j;
      qq[u] = rem - j * a.RS4;
      row[u] = a.idx[(s * a.B_l + a.b0 + bp) * a.F + j];
    }
    f32x4 v[kShardU];
    bool oob = false;
#pragma unroll
    for (int u = 0; u < kShardU; ++u) {
      const int j = jj[u];
      const bool ok = row[u] >= 0 && row[u] < a.rows[j];
      oob |= !ok && t0 + u * stride < n4;
      v[u] = *reinterpret_cast<const f32x4*>(a.src[j] + (ok ? row[u] : 0) * a.src_ld[j] + 4 * qq[u]);
      if (!ok) v[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kShardU; ++u)
      if (t0 + u * stride < n4) out4[t0 + u * stride] = v[u];
    if (oob) flag_oob(a.flags);
  }
}

// The split wire format (round 5): the row exchange carries each field's D second-order floats as
// they are in the nn.Embedding weight ([V, D]: one 128-B line at D = 32, no packed copy of the
// table) and, per (source, sample), ONE first-order value: the sum of this owner's fields' weights
// in field order.  Send block of source s: [b'][j][D] rows, then pad4(bc) partial sums.  The rows
// flattened over float4s (as the packed gather), then one thread per (source, sample) sums the F
// first-order weights in field order.
struct ShardSplitArgs {
  const float* src2[kShardMaxFields];
  const float* src1[kShardMaxFields];
  int64_t ld2[kShardMaxFields], ld1[kShardMaxFields], rows[kShardMaxFields];
  int F, G;            // this rank's fields; float4 quads per row (D / 4)
  const int32_t* idx;  // [P][B_l][F] as received
  int64_t B_l, b0, bc;
  int P;
  float* out;  // per source: [bc][F][D] then pad4(bc) partials
  uint32_t* flags;
};

__global__ __launch_bounds__(256) void shard_gather_split_kernel(ShardSplitArgs a) {
  const int D = 4 * a.G, per = a.F * a.G;
  const int64_t blk = a.bc * a.F * D + ((a.bc + 3) & ~(int64_t)3);  // floats per source block
  const int64_t nrows = (int64_t)a.P * a.bc;                         // (source, sample) rows
  const int64_t n4 = nrows * per;
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  bool oob = false;
  // the second-order rows, flattened over the output's float4s as the packed gather (kShardU loads
  // in flight per lane): float4 t = (row r = t / per, field j, quad q)
  for (int64_t t0 = tid; t0 < n4; t0 += stride * kShardU) {
    int64_t row[kShardU], dst[kShardU];
    int jj[kShardU], qq[kShardU];
#pragma unroll
    for (int u = 0; u < kShardU; ++u) {
      const int64_t t = t0 + u * stride;
      const int64_t tt = t < n4 ? t : 0;
      const int64_t r = tt / per;
      const int rem = (int)(tt - r * per);
      const int j = rem / a.G;
      const int64_t s = r / a.bc, bp = r - s * a.bc;
      jj[u] = j;
      qq[u] = rem - j * a.G;
      dst[u] = s * blk + (bp * a.F + j) * D + 4 * qq[u];
      row[u] = a.idx[(s * a.B_l + a.b0 + bp) * a.F + j];
    }
    f32x4 v[kShardU];
#pragma unroll
    for (int u = 0; u < kShardU; ++u) {
      const int j = jj[u];
      const bool ok = row[u] >= 0 && row[u] < a.rows[j];
      oob |= !ok && t0 + u * stride < n4;
      v[u] = *reinterpret_cast<const f32x4*>(a.src2[j] + (ok ? row[u] : 0) * a.ld2[j] + 4 * qq[u]);
      if (!ok) v[u] = (f32x4){0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int u = 0; u < kShardU; ++u)
      if (t0 + u * stride < n4) *reinterpret_cast<f32x4*>(a.out + dst[u]) = v[u];
  }
  // the first-order partial sums: one thread per (source, sample), the owner's fields in order
  for (int64_t r = tid; r < nrows; r += stride) {
    const int64_t s = r / a.bc, bp = r - s * a.bc;
    const int32_t* ip = a.idx + (s * a.B_l + a.b0 + bp) * a.F;
    float acc = 0.f;
    for (int j = 0; j < a.F; ++j) {
      const int64_t row = ip[j];
      if (row >= 0 && row < a.rows[j]) acc += a.src1[j][row * a.ld1[j]];
    }
    a.out[s * blk + a.bc * a.F * D + bp] = acc;
  }
  if (oob) flag_oob(a.flags);
}

// The same send block with one lane group per (source, sample) (round 5, second form): G = D / 4
// lanes take the quads of that sample's F rows, all F row loads (and, on the group's first lane, the
// F first-order weights) in flight together; grid.y = the source, so no 64-bit divisions by runtime
// sizes.  The first-order sum keeps the field order and skips out-of-range rows, as above.
constexpr int kShardSplitU = 8;  // fields per pass
// NTS: the send-buffer rows go out as nontemporal stores (streamed past L2: each is read once,
// next by the collective), so L2 keeps the index and first-order lines (RANKOPS_SHARD_NTS).
template <int G, bool NTS>
__global__ __launch_bounds__(256) void shard_gather_split_group_kernel(ShardSplitArgs a) {
  constexpr int S = 256 / G, D = 4 * G;
  const int tid = threadIdx.x, q = tid & (G - 1);
  const int64_t bp = (int64_t)blockIdx.x * S + tid / G;
  if (bp >= a.bc) return;  // no barrier below
  const int F = a.F, s = blockIdx.y;
  const int64_t blk = a.bc * F * D + ((a.bc + 3) & ~(int64_t)3);
  float* const out = a.out + s * blk;
  const int32_t* const ip = a.idx + ((int64_t)s * a.B_l + a.b0 + bp) * F;
  float acc = 0.f;
  bool oob = false;
  for (int j0 = 0; j0 < F; j0 += kShardSplitU) {
    int64_t row[kShardSplitU];
#pragma unroll
    for (int u = 0; u < kShardSplitU; ++u) row[u] = j0 + u < F ? ip[j0 + u] : 0;
    f32x4 v[kShardSplitU];
    float w[kShardSplitU];
    bool ok[kShardSplitU];
#pragma unroll
    for (int u = 0; u < kShardSplitU; ++u) {
      const int j = j0 + u;
      ok[u] = false;
      w[u] = 0.f;
      if (j < F) {
        ok[u] = row[u] >= 0 && row[u] < a.rows[j];
        oob |= !ok[u];
        const int64_t r = ok[u] ? row[u] : 0;
        v[u] = *reinterpret_cast<const f32x4*>(a.src2[j] + r * a.ld2[j] + 4 * q);
        if (q == 0) w[u] = a.src1[j][r * a.ld1[j]];
      }
    }
#pragma unroll
    for (int u = 0; u < kShardSplitU; ++u) {
      const int j = j0 + u;
      if (j < F) {
        const f32x4 z = {0.f, 0.f, 0.f, 0.f};
        f32x4* o = reinterpret_cast<f32x4*>(out + (bp * F + j) * D + 4 * q);
        if constexpr (NTS)
          __builtin_nontemporal_store(ok[u] ? v[u] : z, o);
        else
          *o = ok[u] ? v[u] : z;
        if (ok[u]) acc += w[u];
      }
    }
  }
  if (q == 0) out[a.bc * F * D + bp] = acc;
  if (oob) flag_oob(a.flags);
}

}  // namespace rk

using namespace rk;

RK_API int rk_shard_gather_rows_split(const rk_segment* second, const rk_segment* first, int32_t num_fields,
                                      int32_t dim, const int32_t* idx, int32_t num_sources, int64_t source_batch,
                                      int64_t b0, int64_t bc, float* out, void* stream) {
  if (!second || !first || num_fields <= 0 || num_fields > kShardMaxFields || dim < 4 || dim % 4 || !idx || !out ||
      num_sources <= 0 || source_batch < 0 || b0 < 0 || bc < 0 || b0 + bc > source_batch || !aligned16(out))
    return fail(RK_ERR_INVALID, "rk_shard_gather_rows_split: bad arguments (fields %d <= %d, dim %d %% 4 == 0)",
                num_fields, kShardMaxFields, dim);
  ShardSplitArgs a = {};
  for (int j = 0; j < num_fields; ++j) {
    const rk_segment& t2 = second[j];
    const rk_segment& t1 = first[j];
    if (!t2.src || t2.rows <= 0 || t2.src_ld < dim || t2.src_ld % 4 || !aligned16(t2.src) || !t1.src ||
        t1.rows < t2.rows || t1.src_ld < 1)
      return fail(RK_ERR_INVALID, "rk_shard_gather_rows_split: table %d ([rows, >= dim] 16-B aligned, first-order "
                                  "[rows, 1])", j);
    a.src2[j] = t2.src;
    a.ld2[j] = t2.src_ld;
    a.rows[j] = t2.rows;
    a.src1[j] = t1.src;
    a.ld1[j] = t1.src_ld;
  }
  a.F = num_fields;
  a.G = dim / 4;
  a.idx = idx;
  a.B_l = source_batch;
  a.b0 = b0;
  a.bc = bc;
  a.P = num_sources;
  a.out = out;
  a.flags = device_flags();
  if (!a.flags) return fail(RK_ERR_RUNTIME, "rk_shard_gather_rows_split: device not initialised (rk_init)");
  const int64_t nrows = (int64_t)num_sources * bc;
  if (nrows == 0) return RK_OK;
  static const bool flat = [] {  // A/B switch: RANKOPS_SHARD_SPLIT_FLAT=1 keeps the flattened form
    const char* e = getenv("RANKOPS_SHARD_SPLIT_FLAT");
    return e && e[0] == '1';
  }();
  if (!flat && num_sources <= 65535 && (a.G == 4 || a.G == 8 || a.G == 16)) {
    const int S = 256 / a.G;
    const dim3 grid((unsigned)((bc + S - 1) / S), (unsigned)num_sources);
    const char* ne = getenv("RANKOPS_SHARD_NTS");  // per call (A/B)
    const bool nts = !(ne && ne[0] == '0');
    auto go = [&](auto kern) { kern<<<grid, 256, 0, (hipStream_t)stream>>>(a); };
    if (a.G == 8)
      nts ? go(shard_gather_split_group_kernel<8, true>) : go(shard_gather_split_group_kernel<8, false>);
    else if (a.G == 4)
      nts ? go(shard_gather_split_group_kernel<4, true>) : go(shard_gather_split_group_kernel<4, false>);
    else
      nts ? go(shard_gather_split_group_kernel<16, true>) : go(shard_gather_split_group_kernel<16, false>);
    return check_launch("rk_shard_gather_rows_split");
  }
  const int64_t n4 = nrows * num_fields * a.G;
  const unsigned blocks = (unsigned)std::min<int64_t>(
      std::max<int64_t>((n4 + 256 * kShardU - 1) / (256 * kShardU), (nrows + 255) / 256), (int64_t)num_cus() * 32);
  shard_gather_split_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(a);
  return check_launch("rk_shard_gather_rows_split");
}

RK_API int rk_shard_pack_indices(const int64_t* const* idx, const int64_t* base, const int32_t* stride,
                                 int32_t num_fields, int64_t batch, int32_t* out, void* stream) {
  if (!idx || !base || !stride || !out || num_fields <= 0 || num_fields > kShardMaxFields || batch < 0)
    return fail(RK_ERR_INVALID, "rk_shard_pack_indices: bad arguments (%d fields, max %d)", num_fields,
                kShardMaxFields);
  ShardPackArgs a = {};
  for (int q = 0; q < num_fields; ++q) {
    if (!idx[q] || stride[q] <= 0 || base[q] < 0)
      return fail(RK_ERR_INVALID, "rk_shard_pack_indices: field slot %d invalid", q);
    a.idx[q] = idx[q];
    a.base[q] = base[q];
    a.stride[q] = stride[q];
  }
  a.F = num_fields;
  a.B = batch;
  a.out = out;
  if (batch == 0) return RK_OK;
  const int64_t n = batch * num_fields;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, (int64_t)num_cus() * 8);
  shard_pack_indices_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(a);
  return check_launch("rk_shard_pack_indices");
}

RK_API int rk_shard_gather_rows(const rk_segment* tables, int32_t num_fields, int32_t row_floats,
                                const int32_t* idx, int32_t num_sources, int64_t source_batch, int64_t b0,
                                int64_t bc, float* out, void* stream) {
  if (!tables || num_fields <= 0 || num_fields > kShardMaxFields || !idx || !out || num_sources <= 0 ||
      row_floats <= 0 || row_floats % 4 || source_batch < 0 || b0 < 0 || bc < 0 || b0 + bc > source_batch ||
      !aligned16(out))
    return fail(RK_ERR_INVALID, "rk_shard_gather_rows: bad arguments (fields %d <= %d, row_floats %d %% 4 == 0)",
                num_fields, kShardMaxFields, row_floats);
  ShardGatherArgs a = {};
  for (int j = 0; j < num_fields; ++j) {
    const rk_segment& t = tables[j];
    if (!t.src || t.rows <= 0 || t.src_ld < row_floats || t.src_ld % 4 || !aligned16(t.src))
      return fail(RK_ERR_INVALID, "rk_shard_gather_rows: table %d is not a 16-B aligned packed [rows, >= %d] table",
                  j, row_floats);
    a.src[j] = t.src;
    a.src_ld[j] = t.src_ld;
    a.rows[j] = t.rows;
  }
  a.F = num_fields;
  a.RS4 = row_floats / 4;
  a.idx = idx;
  a.B_l = source_batch;
  a.b0 = b0;
  a.bc = bc;
  a.P = num_sources;
  a.out = out;
  a.flags = device_flags();
  if (!a.flags) return fail(RK_ERR_RUNTIME, "rk_shard_gather_rows: device not initialised (rk_init)");
  const int64_t nrows = (int64_t)num_sources * bc;
  if (nrows == 0) return RK_OK;
  const int64_t n4 = nrows * num_fields * a.RS4;
  const unsigned blocks = (unsigned)std::min<int64_t>((n4 + 256 * kShardU - 1) / (256 * kShardU), (int64_t)num_cus() * 32);
  shard_gather_rows_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(a);
  return check_launch("rk_shard_gather_rows");
}
