// One wide MLP layer as a 2D-tiled GEMM: y[M, n] = epilogue(x[M, K] . W[n, K]^T) for a layer packed
// by rk_mlp_pack_weight, with the element-wise epilogue of mlp_core.h (bias, residual-free
// BatchNorm affine, activation).  Used for the first DeepFM layer (960 -> 512, deepfm.py:100-112):
// in the fused 16-row tail every CU streams the whole 2 MB weight for 16 rows (~500 MB of L2
// traffic per batch); here a workgroup owns a 64-row x 128-column tile, so the weight traffic
// drops 4x at the same 256 workgroups for batch 4096.
//
// 16 waves: wave w owns column tile w%8 (16 columns) for the 32 rows of half w/8 (two 16-row
// MFMA tiles, v_mfma_f32_16x16x4_f32: every weight float4 feeds 8 MFMAs).  The A tile is staged
// through LDS in K-blocks of up to 256 columns, double buffered: the next block's global loads
// are issued into registers before this block's MFMAs and stored after them.  The weight ring
// (4 chunks of 16 k) streams continuously across the block barriers, which are LDS-only.
#include "mlp_core.h"

namespace rk {

constexpr int kLtRows = 64;   // rows per workgroup
constexpr int kLtCols = 128;  // output columns per workgroup (8 tiles of 16)
constexpr int kLtKB = 256;    // K-block staged in LDS
constexpr int kLtLd = kLtKB + kMlpLdPad;
constexpr int kLtMaxFields = 32;
// Weight ring depth (chunks of 16 k).  Loads retire in order and the compiler's wait for ring slot
// s in the block loop is vmcnt(kLtPD - 1): at a block's start the next block's A loads (issued
// ahead of the refills) must land within kLtPD - 5 chunks.  With 4 the first chunk of every block
// waited for the gather (tools/lt_phases.py: ~22.4k cycles per 16-chunk block against 16.4k of
// MFMA).
constexpr int kLtPD = 8;

struct LtArgs {
  const float* x;
  int64_t ldx, M;
  int K, Kp;
  rk_mlp_layer L;
  float* y;
  int64_t ldy;
  int x_vec;
  int nrt, nct;  // row tiles, column tiles
  int nctg;      // column tiles in the grid: nct, or (FM) at least 4 so that every row has an FM owner
};

// The fused DeepFM front end's A source (rk_fm_linear_packed): row b of A is the concatenation of
// the num_fields packed-table rows idx[f][b] (rk_fm_pack_table layout: dim floats, then the
// first-order weight), and the same pass produces fm1 / fm2 (deepfm.py:122-140) for the rows it
// stages.  A field without an index array (idx null) is a dense block of packed rows, row b at
// src + b * ld: the rows ShardedDeepFM receives from the field's owner rank.
struct LtFm {
  const float* src[kLtMaxFields];
  const int64_t* idx[kLtMaxFields];
  int64_t ld[kLtMaxFields], rows[kLtMaxFields];
  int F, dim_shift;
  float* fm1;
  float* fm2;
  uint32_t* flags;
};

// Tile order: block l works on row tile 8 (l / 8 nct) + l % 8 and column tile (l / 8) % nct, so the
// nct workgroups that stage the same 64 rows are dealt to one XCD (blocks b and b + 8 share one,
// MI355X_MICROARCH.md) and read those rows through one L2.
template <bool FM>
__global__ __launch_bounds__(kMlpThreads) void linear_tiled_kernel(LtArgs a, LtFm fm) {
  // [2][kLtRows * kLtLd] A blocks, then (FM) [F][kLtRows] row pointers
  extern __shared__ __attribute__((aligned(16))) float lt_sm[];
  const int l = blockIdx.x, within = l % (8 * a.nctg);
  const int rt = 8 * (l / (8 * a.nctg)) + within % 8, ctile = within / 8;
  if (rt >= a.nrt) return;  // the whole workgroup, before any barrier
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
#ifdef RK_MLP_PHASES
  const unsigned long long t0 = clock64();
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 2);
#endif
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int64_t m0 = (int64_t)rt * kLtRows;
  const int n0 = ctile * kLtCols;
  const int ct = wave & 7, rh = wave >> 3;
  const int n = n0 + 16 * ct + li;  // this lane's weight row / output column
  const rk_mlp_layer& L = a.L;
  const bool col_live = n < pad64(L.n);

  // FM: the staged rows' indices, issued first (F * 64 <= 2048 entries: at most 2 per thread;
  // entry e = field e / 64, row e % 64, so a wave's loads are one field's 64 contiguous indices)
  constexpr int kIdxPer = kLtMaxFields * kLtRows / kMlpThreads;
  int64_t iv[kIdxPer];
  if constexpr (FM) {
#pragma unroll
    for (int u = 0; u < kIdxPer; ++u) {
      const int e = tid + kMlpThreads * u;
      const int f = __builtin_amdgcn_readfirstlane(e / kLtRows);  // wave-uniform: scalar descriptor loads
      const int64_t m = m0 + e % kLtRows;
      iv[u] = (f < fm.F && m < a.M) ? (fm.idx[f] ? fm.idx[f][m] : m) : -1;
    }
  }

  // weight stream of this wave's column tile over the whole K (ring of kLtPD chunks), as buffer
  // loads: the tile's fragment slab is one wave-uniform descriptor, a lane's address one 32-bit
  // offset (16 lane), the chunk a scalar offset; chunks past the slab read as zeros (bounds check)
  const int kchunks = a.Kp / 16;
  const int wtile = __builtin_amdgcn_readfirstlane(col_live ? (n >> 4) : 0);  // n >> 4 = n0 / 16 + ct
  const __amdgpu_buffer_rsrc_t wsrd = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(L.w + (int64_t)wtile * (L.ldw / 16) * kFragStep), 0, kchunks * kFragStep * (int)sizeof(float),
      0x00020000);
  auto wload = [&](int chunk) {
    return __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(wsrd, 16 * lane,
                                                                              chunk * kFragStep * 4, 0));
  };
  f32x4_t ring[kLtPD];
#pragma unroll
  for (int s = 0; s < kLtPD; ++s) ring[s] = wload(s);
  const ColEpi ep = col_epi(L, n < L.n ? n : 0);

  // FM: the staged rows' row pointers (null past M or out of range: a zero row, as rk_fm_gather)
  const float** s_ptr = reinterpret_cast<const float**>(lt_sm + 2 * kLtRows * kLtLd);
  if constexpr (FM) {
    bool oob = false;
#pragma unroll
    for (int u = 0; u < kIdxPer; ++u) {
      const int e = tid + kMlpThreads * u;
      const int f = __builtin_amdgcn_readfirstlane(e / kLtRows);
      if (f < fm.F) {
        const float* p = nullptr;
        if ((uint64_t)iv[u] < (uint64_t)fm.rows[f])
          p = fm.src[f] + iv[u] * fm.ld[f];
        else if (m0 + e % kLtRows < a.M)
          oob = true;
        s_ptr[e] = p;
      }
    }
    if (oob) flag_oob(fm.flags);
    mlp_lds_barrier();
  }
  MLP_MARK(0, t0);
  // FM sums: workgroup ctile < 4 owns the rows wave + 16 ctile (the grid has >= 4 column tiles);
  // lane holds quad (lane % G) of field (k / dim) for every block, so the field sum is a shuffle
  // over lane / G
  const int G = FM ? (1 << fm.dim_shift) / 4 : 1;
  const bool fm_owner = FM && ctile < 4;
  f32x4_t fs = {0.f, 0.f, 0.f, 0.f}, fq = {0.f, 0.f, 0.f, 0.f};
  float fo = 0.f;

  // A staging: block b covers columns [256 b, min(256 b + 256, Kp)); thread tid moves float4s
  // i = tid + 1024 j of the 64 x 256 block (4 per thread): row wave + 16 j, columns 4 lane ..
  // The loads are unconditional global loads from a valid address (dead ones from a safe row) and
  // the zero masks are applied in store_block: a load under a branch, or a select on its value,
  // made the compiler wait for the gather right after issuing it, and a generic (flat) pointer
  // read from LDS made every later LDS wait of the MFMA loop wait for the gather too.
  typedef const f32x4_t __attribute__((address_space(1)))* g4ptr;
  typedef const float __attribute__((address_space(1)))* gptr;
  f32x4_t stage[4];
  float fw = 0.f;     // (FM) the owned row's first-order weight of this lane's field
  unsigned live = 0;  // bit j: stage[j] is real data
  bool fw_live = false;
  auto load_block = [&](int b) {
    const int kb = b * kLtKB, w = min(kLtKB, a.Kp - kb);
    const int c = 4 * lane, k = kb + c;
    const bool kin = c < w && k < a.K;
    live = 0;
    if constexpr (FM) {
      const int dmask = (1 << fm.dim_shift) - 1, d = k & dmask;
      const float* p[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) p[j] = s_ptr[(kin ? (k >> fm.dim_shift) : 0) * kLtRows + wave + 16 * j];
      const float* safe = fm.src[0];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const bool ok = kin && p[j] != nullptr;
        live |= (unsigned)ok << j;
        stage[j] = *(g4ptr)(ok ? p[j] + d : safe);
      }
      const float* pm = ctile == 0 ? p[0] : ctile == 1 ? p[1] : ctile == 2 ? p[2] : p[3];
      fw_live = fm_owner && kin && pm != nullptr && d + 4 == dmask + 1;
      fw = *(gptr)(fw_live ? pm + dmask + 1 : safe);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int64_t m = m0 + wave + 16 * j;
        const bool ok = kin && m < a.M;
        if (a.x_vec) {
          live |= (unsigned)ok << j;
          stage[j] = *(g4ptr)(ok ? a.x + m * a.ldx + k : a.x);
        } else {  // unaligned rows: scalar loads, zeros written here
          live |= 1u << j;
          f32x4_t v = {0.f, 0.f, 0.f, 0.f};
          if (c < w && m < a.M) {
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = k + e < a.K ? a.x[m * a.ldx + k + e] : 0.f;
          }
          stage[j] = v;
        }
      }
    }
  };
  // (the FM sums are taken here, after the block's MFMAs, not at the loads: summing at the loads
  // made every block wait for its gather before its first MFMA)
  auto store_block = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4_t v = (live >> j) & 1 ? stage[j] : (f32x4_t){0.f, 0.f, 0.f, 0.f};
      *reinterpret_cast<f32x4_t*>(lt_sm + buf * kLtRows * kLtLd + (wave + 16 * j) * kLtLd + 4 * lane) = v;
      if (fm_owner && j == ctile) {
        fs += v;
        fq += v * v;
      }
    }
    if (fm_owner) fo += fw_live ? fw : 0.f;
  };

  const int nblocks = (a.Kp + kLtKB - 1) / kLtKB;
  load_block(0);
  store_block(0);
  mlp_lds_barrier();
  MLP_MARK(1, t0);

  f32x4_t acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  int c = 0;  // global chunk index of the weight stream (a multiple of kLtPD at every block start)
  // One K-block of nc chunks (4, 8, 12 or 16: Kp % 64 == 0) in groups of kLtPD plus a 4-chunk tail.
  auto slot = [&](const float* arow, f32x4_t (&ab)[2][2], int q, int nc, auto SS, auto REFILL) {
    constexpr int S = decltype(SS)::value;  // ring slot = q % kLtPD (c is a multiple of kLtPD)
    const int qa = min(q + 1, nc - 1);
#pragma unroll
    for (int t = 0; t < 2; ++t) ab[(S + 1) & 1][t] = *reinterpret_cast<const f32x4_t*>(arow + 16 * t * kLtLd + 16 * qa);
    __builtin_amdgcn_sched_barrier(0);
    const f32x4_t bv = ring[S];
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = mfma16(ab[S & 1][t][e], bv[e], acc[t]);
    if constexpr (decltype(REFILL)::value) ring[S] = wload(c + q + kLtPD);
    __builtin_amdgcn_sched_barrier(0);
  };
  auto run_block = [&](const float* arow, int nc) {
    // A float4s one chunk ahead in two explicit register sets, the read issued before the chunk's
    // MFMAs (see mlp_core.h mlp_layer)
    f32x4_t ab[2][2];
#pragma unroll
    for (int t = 0; t < 2; ++t) ab[0][t] = *reinterpret_cast<const f32x4_t*>(arow + 16 * t * kLtLd);
    int q0 = 0;
    for (; q0 + kLtPD <= nc; q0 += kLtPD) {
      slot(arow, ab, q0 + 0, nc, std::integral_constant<int, 0>(), std::true_type());
      slot(arow, ab, q0 + 1, nc, std::integral_constant<int, 1>(), std::true_type());
      slot(arow, ab, q0 + 2, nc, std::integral_constant<int, 2>(), std::true_type());
      slot(arow, ab, q0 + 3, nc, std::integral_constant<int, 3>(), std::true_type());
      slot(arow, ab, q0 + 4, nc, std::integral_constant<int, 4>(), std::true_type());
      slot(arow, ab, q0 + 5, nc, std::integral_constant<int, 5>(), std::true_type());
      slot(arow, ab, q0 + 6, nc, std::integral_constant<int, 6>(), std::true_type());
      slot(arow, ab, q0 + 7, nc, std::integral_constant<int, 7>(), std::true_type());
    }
    // nc % 8 == 4: the last block only, so no refills (the ring's load order then stays the same on
    // every path into the group loop, whose waits the compiler derives from the merged paths)
    if (q0 < nc) {
      slot(arow, ab, q0 + 0, nc, std::integral_constant<int, 0>(), std::false_type());
      slot(arow, ab, q0 + 1, nc, std::integral_constant<int, 1>(), std::false_type());
      slot(arow, ab, q0 + 2, nc, std::integral_constant<int, 2>(), std::false_type());
      slot(arow, ab, q0 + 3, nc, std::integral_constant<int, 3>(), std::false_type());
    }
    c += nc;
  };
  for (int b = 0; b < nblocks; ++b) {
    const int buf = b & 1;
    if (b + 1 < nblocks) load_block(b + 1);
    const int bchunks = min(kLtKB, a.Kp - b * kLtKB) / 16;
    run_block(lt_sm + buf * kLtRows * kLtLd + (32 * rh + li) * kLtLd + kq, bchunks);
    if (b < 4) MLP_MARK(2 + 2 * b, t0);
#ifdef RK_MLP_PHASES
    if (lane == 0 && b == 0) s_mlp_wave_marks[1][wave][0] = (unsigned)(clock64() - t0);
    if (lane == 0 && b + 1 == nblocks) s_mlp_wave_marks[0][wave][0] = (unsigned)(clock64() - t0);
#endif
    if (b + 1 < nblocks) {
      store_block(buf ^ 1);
      mlp_lds_barrier();
    }
    if (b < 4) MLP_MARK(3 + 2 * b, t0);
  }

  // epilogue: bias, BatchNorm affine, activation; rows < M, columns < n
  if (n < L.n) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + 32 * rh + 16 * t + 4 * (lane >> 4) + r;
        if (m < a.M) a.y[m * a.ldy + n] = col_apply(L, ep, L.act == RK_ACT_DICE, acc[t][r], false, 0.f);
      }
  }
  MLP_MARK(10, t0);
#ifdef RK_MLP_PHASES
  if (lane == 0) s_mlp_wave_marks[0][wave][1] = (unsigned)(clock64() - t0);
#endif

  // FM outputs: sums over the fields (lanes of equal lane % G), then fm2 = 0.5 sum_d (S_d^2 - Q_d)
  // over the quads (deepfm.py:128-140)
  if constexpr (FM) {
    if (fm_owner) {
      f32x4_t s = fs, q = fq;
      float o = fo;
      for (int x = G; x < 64; x <<= 1) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[e] += __shfl_xor(s[e], x, kWave);
          q[e] += __shfl_xor(q[e], x, kWave);
        }
        o += __shfl_xor(o, x, kWave);
      }
      float part = (s[0] * s[0] - q[0]) + (s[1] * s[1] - q[1]) + (s[2] * s[2] - q[2]) + (s[3] * s[3] - q[3]);
      for (int x = G / 2; x > 0; x >>= 1) {  // the first-order weights sit in the lanes of quad G - 1
        part += __shfl_xor(part, x, kWave);
        o += __shfl_xor(o, x, kWave);
      }
      const int64_t m = m0 + wave + 16 * ctile;
      if (lane == 0 && m < a.M) {
        fm.fm2[m] = 0.5f * part;
        fm.fm1[m] = o;
      }
    }
  }
  MLP_MARK(11, t0);
  MLP_WALL(4 * RK_MLP_MAX_LAYERS + 3);
  MLP_FLUSH(tid);
}

static int check_layer(const rk_mlp_layer& L, int K, int64_t ldy, const char* what) {
  if (!L.w || L.n <= 0 || L.ldw != pad64(K) || ((uintptr_t)L.w & 15u))
    return fail(RK_ERR_UNSUPPORTED, "%s: the weight must be packed by rk_mlp_pack_weight (ldw %lld, K %d)", what,
                (long long)L.ldw, K);
  if (L.residual) return fail(RK_ERR_UNSUPPORTED, "%s: residual layers are not supported", what);
  if (L.act == RK_ACT_DICE && (!L.act_scale || !L.act_shift || !L.act_alpha))
    return fail(RK_ERR_INVALID, "%s: Dice layer incomplete", what);
  if (L.act == RK_ACT_PRELU && !L.act_alpha) return fail(RK_ERR_INVALID, "%s: PReLU needs alpha", what);
  if ((L.pre_scale != nullptr) != (L.pre_shift != nullptr) || (L.post_scale != nullptr) != (L.post_shift != nullptr))
    return fail(RK_ERR_INVALID, "%s: affine scale/shift must come in pairs", what);
  if (ldy < L.n) return fail(RK_ERR_INVALID, "%s: ldy %lld < n %d", what, (long long)ldy, L.n);
  return RK_OK;
}

#ifdef RK_MLP_PHASES
// Timing build only (tools/lt_phases.py): this module's phase counters (marks: 0 prologue, 1 block 0
// staged, 2 + 2b / 3 + 2b block b MFMAs issued / barrier passed, 10 epilogue, 11 end; wave marks
// [0][w] last block issued / epilogue, [1][w][0] block 0 issued).
RK_API int rk_debug_lt_phases(unsigned long long* marks, int32_t nwg, unsigned* wave_marks) {
  if (nwg < 0 || nwg > kMlpMarkWG) return 1;
  if (hipMemcpyFromSymbol(marks, HIP_SYMBOL(g_mlp_marks), sizeof(g_mlp_marks[0]) * nwg) != hipSuccess) return 1;
  if (wave_marks &&
      hipMemcpyFromSymbol(wave_marks, HIP_SYMBOL(g_mlp_wave_marks), sizeof(g_mlp_wave_marks[0]) * nwg) != hipSuccess)
    return 1;
  return 0;
}
#endif

template <bool FM>
static int launch_linear_tiled(LtArgs& a, const LtFm& fm, hipStream_t st, const char* what) {
  a.nrt = (int)((a.M + kLtRows - 1) / kLtRows);
  a.nct = (pad64(a.L.n) + kLtCols - 1) / kLtCols;
  a.nctg = FM ? std::max(a.nct, 4) : a.nct;  // column tiles >= nct only stage rows for their FM sums
  const int64_t blocks = (int64_t)((a.nrt + 7) / 8) * 8 * a.nctg;
  if (blocks > INT32_MAX) return fail(RK_ERR_UNSUPPORTED, "%s: batch too large", what);
  const size_t shm = 2 * kLtRows * kLtLd * sizeof(float) + (FM ? (size_t)fm.F * kLtRows * sizeof(void*) : 0);
  raise_lds_limit((const void*)linear_tiled_kernel<FM>, (int)shm);
  linear_tiled_kernel<FM><<<(unsigned)blocks, kMlpThreads, shm, st>>>(a, fm);
  return check_launch(what);
}

}  // namespace rk

using namespace rk;

RK_API int rk_linear_tiled(const float* x, int64_t ldx, int64_t M, int32_t K, const rk_mlp_layer* layer, float* y,
                           int64_t ldy, void* stream) {
  if (!x || !layer || !y || M < 0 || K <= 0 || ldx < K)
    return fail(RK_ERR_INVALID, "rk_linear_tiled: bad arguments (M=%lld K=%d)", (long long)M, K);
  if (int e = check_layer(*layer, K, ldy, "rk_linear_tiled")) return e;
  if (M == 0) return RK_OK;
  LtArgs a = {};
  a.x = x;
  a.ldx = ldx;
  a.M = M;
  a.K = K;
  a.Kp = pad64(K);
  a.L = *layer;
  a.y = y;
  a.ldy = ldy;
  a.x_vec = (ldx % 4 == 0) && (((uintptr_t)x & 15u) == 0);
  LtFm fm = {};
  return launch_linear_tiled<false>(a, fm, (hipStream_t)stream, "rk_linear_tiled");
}

RK_API int rk_fm_linear_packed(const rk_segment* fields, int32_t num_fields, int32_t dim, int64_t batch,
                               const rk_mlp_layer* layer, float* y, int64_t ldy, float* fm1, float* fm2,
                               void* stream) {
  if (!fields || num_fields <= 0 || num_fields > kLtMaxFields)
    return fail(RK_ERR_UNSUPPORTED, "rk_fm_linear_packed: %d fields (max %d)", num_fields, kLtMaxFields);
  if (dim < 4 || dim > 256 || (dim & (dim - 1)))
    return fail(RK_ERR_UNSUPPORTED, "rk_fm_linear_packed: dim %d must be a power of two in [4, 256]", dim);
  if (!layer || !y || !fm1 || !fm2 || batch < 0)
    return fail(RK_ERR_INVALID, "rk_fm_linear_packed: bad arguments (batch %lld)", (long long)batch);
  const int K = num_fields * dim;
  if (int e = check_layer(*layer, K, ldy, "rk_fm_linear_packed")) return e;
  LtFm fm = {};
  for (int f = 0; f < num_fields; ++f) {
    const rk_segment& s = fields[f];
    if (!s.src || (s.idx && (s.rows <= 0 || s.idx_stride != 1)) || s.dim != dim || s.src_ld < dim + 1 ||
        s.src_ld % 4 || !aligned16(s.src) || s.out_col != f * dim)
      return fail(RK_ERR_INVALID,
                  "rk_fm_linear_packed: field %d is not a packed [rows, >= dim+1] table (unit-stride indices, or "
                  "none: a dense block of packed rows) at column f*dim",
                  f);
    fm.src[f] = s.src;
    fm.idx[f] = s.idx;
    fm.ld[f] = s.src_ld;
    fm.rows[f] = s.idx ? s.rows : batch;  // dense: row b < batch
  }
  fm.F = num_fields;
  fm.dim_shift = __builtin_ctz((unsigned)dim);
  fm.fm1 = fm1;
  fm.fm2 = fm2;
  fm.flags = device_flags();
  if (!fm.flags) return fail(RK_ERR_RUNTIME, "rk_fm_linear_packed: no device flag word");
  if (batch == 0) return RK_OK;
  LtArgs a = {};
  a.M = batch;
  a.K = K;
  a.Kp = pad64(K);
  a.L = *layer;
  a.y = y;
  a.ldy = ldy;
  return launch_linear_tiled<true>(a, fm, (hipStream_t)stream, "rk_fm_linear_packed");
}
