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
//                         int32 indices the source sent, [s][b'][j][RS].  One wave per output row
//                         (F_me * RS / 4 float4s), indices read once per lane.
//
// Both are HBM-bound byte movers: pack 12 B per (sample, field); gather 4 B of index + 2 x RS * 4 B
// per (row, field) (read the packed row, write it to the send buffer).
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
    a.out[a.base[q] + b * a.stride[q]] = (int32_t)a.idx[q][b];
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

__global__ __launch_bounds__(256) void shard_gather_rows_kernel(ShardGatherArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t nrows = (int64_t)a.P * a.bc;
  const int per = a.F * a.RS4;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < nrows; r += (int64_t)gridDim.x * 4) {
    const int64_t s = r / a.bc, bp = r - s * a.bc;
    const int32_t* ip = a.idx + (s * a.B_l + a.b0 + bp) * a.F;
    f32x4* dst = reinterpret_cast<f32x4*>(a.out + r * a.F * a.RS4 * 4);
    bool oob = false;
    for (int t = lane; t < per; t += 64) {
      const int j = t / a.RS4, q = t - j * a.RS4;
      const int64_t row = ip[j];
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (row >= 0 && row < a.rows[j])
        v = *reinterpret_cast<const f32x4*>(a.src[j] + row * a.src_ld[j] + 4 * q);
      else
        oob = true;
      dst[t] = v;
    }
    if (oob) flag_oob(a.flags);
  }
}

}  // namespace rk

using namespace rk;

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
  const unsigned blocks = (unsigned)std::min<int64_t>((nrows + 3) / 4, (int64_t)num_cus() * 16);
  shard_gather_rows_kernel<<<blocks, 256, 0, (hipStream_t)stream>>>(a);
  return check_launch("rk_shard_gather_rows");
}
