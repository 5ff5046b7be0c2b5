// Whole DIN eval forward in one launch (reference: DIN.forward din.py:294-323 with
// din_attention din.py:42-84, Dice din.py:26-36 and the fcn stack din.py:272-285).
//
// A workgroup of 16 waves owns 16 samples.
//  Phase A (one wave per sample):
//   * gather the sample's feature row [dense | category embeddings | target feed] into LDS
//     (the rk_concat_gather column map, built once per workgroup);
//   * local-activation attention with the first att-MLP layer split algebraically:
//       cross.W1^T = q.(W1a+W1c)^T + k.(W1b-W1c + diag(q) W1d)^T
//     u = q.(W1a+W1c)^T + b1 is a per-sample bias (64 values, one per lane), and the MFMA A
//     operand Weff[j][h] = (W1b-W1c)[j][h] + W1d[j][h]*q[h] is formed on the fly from two LDS
//     rows and the query — layer 1 contracts over H instead of 4H (4x fewer MFMAs than the
//     reference formulation).  Round 4: the history is processed in tiles of 16 positions on
//     v_mfma_f32_16x16x4_f32 (lane = position x key quarter), so a sample pads to a multiple of 16
//     positions, not 32 (T = 50, lengths U[1, 50]: 33 instead of 44 positions per sample); the
//     layer-1 accumulators feed layer 2 as its B operand in place, layer 3, the mask and the
//     (online) softmax and weighted key sum follow per tile;
//   * the attention output goes into the LDS row; the row's l2 norm (din.py:318-322) is taken.
//  Phase B: the fcn tail + output layer + sigmoid over the 16 LDS rows (mlp_stream.h for the
//  compiled [512, 256, 128] plan, mlp_core.h otherwise).
// The l2 term is finished by a one-wave reduction over the per-workgroup partial sums.
#include <cstdlib>
#include <new>

#include "mlp_core.h"
#include "mlp_stream.h"

namespace rk {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void glb_void;

#ifndef RK_DIN_HOIST  // experiment (phase A's layer-1 operand per sample): see the tile loop
#define RK_DIN_HOIST 0
#endif

constexpr int kDinSegs = 32;
constexpr int kDinSegLdsOff = 528;  // bytes past the column map: 256 + 256 map bytes, l2_last int, pad to 16
struct DinSegs {
  rk_segment s[kDinSegs];
};

struct DinArgs {
  DinSegs segs;
  uint8_t col_seg[256], col_off[256];  // column -> (segment, offset) map, built by the host wrapper
  const float* att_image;              // rk_din_pack_attention image (the first DinLds::U floats of LDS)
  int nseg, width, q_col, att_col, l2_col0;
  const float* key_table;
  int64_t key_rows, ld_key;
  const int64_t* seq;
  int64_t ld_seq;
  int T;
  const int64_t* seq_len;
  int64_t batch;
  const float *w1, *b1, *w2, *b2, *w3, *b3;
  int use_softmax;
  int bal_nb;         // balanced assignment: tile-count classes (0 .. ceil(T/32))
  float* l2_part;
  unsigned* l2_count;  // zero between launches: the last workgroup to finish phase A resets it
  float* l2_out;
  float l2_scale;
  uint32_t* flags;
  rk_mlp_layer L[RK_MLP_MAX_LAYERS];
  int nl;
  rk_epilogue head;
  int ld0, ld1;
  int epi_off;  // streamed phase B (mlp_stream.h): float offset of the epilogue-parameter image
  // a plan's launches (rk_din_plan_set_epilogue_image): that image packed in global
  // memory (rk_mlp_pack_epilogue), copied into LDS by LDS-DMA after phase A instead of resolved
  // per column at launch (≈ 1.6 us of the staging: profiles/r04/din_phases_stage*.log)
  const float* epi_image;
};

// LDS carve (floats): [Wk | Wqk | Wq] 3 x 64 x (H+4), W2 32 x 68, b1 64, b2 32, w3 32,
// u 16 x 64, norms 16, then buf0 16 x ld0, buf1 16 x ld1; column map after that (bytes), then the
// segment descriptors, the per-wave prefetch slots and (balanced launches) the assignment area.
template <int H>
struct DinLds {
  static constexpr int LDH = H + 4;
  static constexpr int WK = 0, WQK = WK + 64 * LDH, WQ = WQK + 64 * LDH, W2 = WQ + 64 * LDH;
  static constexpr int B1 = W2 + 32 * 68, B2 = B1 + 64, W3 = B2 + 32, U = W3 + 32, NORM = U + 16 * 64;
  static constexpr int BUF0 = NORM + 16;
};

#ifdef RK_DIN_PHASES  // timing build only (tools/din_phases.py): per-workgroup wall-clock marks
constexpr int kDinPhaseWG = 1024;
// entry, staged, phase A done, phase B done, wave 0 assigned, image copied, classes counted,
// wave 0's row and first keys loaded (tid 0)
__device__ unsigned long long g_din_ts[kDinPhaseWG][8];
__device__ unsigned long long g_din_wave[kDinPhaseWG][16];    // per-wave phase-A cycles (clock64)
// marks are kept in LDS while the kernel runs (a global store mid-kernel joins the vmcnt queue
// every later wait drains) and written out by din_marks_flush() at the end
__shared__ unsigned long long s_din_ts[8];
__shared__ unsigned long long s_din_wave[16];
#define DIN_TS(i)                                \
  do {                                           \
    if (tid == 0) s_din_ts[i] = wall_clock64();  \
  } while (0)
__device__ __forceinline__ void din_marks_flush(int tid) {
  __syncthreads();
  if (blockIdx.x < kDinPhaseWG) {
    if (tid < 8) g_din_ts[blockIdx.x][tid] = s_din_ts[tid];
    if (tid < 16) g_din_wave[blockIdx.x][tid] = s_din_wave[tid];
  }
}
#else
#define DIN_TS(i) \
  do {            \
  } while (0)
#endif

// Balanced assignment (NIT > 0).  The attention cost of a sample is its tile count, and with one
// workgroup per CU the kernel ends with the workgroup whose SIMDs carry the most tiles
// (tools/din_phases.py: phase-A time tracks the 2-tile samples per workgroup, corr 0.91).  The
// workgroups rank their samples by descending tile count (stable in the batch order) and take
// ranks g + G * j, j = 0..15 (G workgroups): each workgroup gets the same mix of long and short
// samples, within one, and wave j gets the j-th longest of its 16.  The ranking is a counting sort
// over the ceil(T/16) + 1 tile classes: per 64-sample block a ballot mask per class in LDS, then
// each wave finds its rank's sample by a prefix over the blocks' popcounts.  NIT == 1 (round 6,
// the default): the ranking runs per 1,024-sample universe, the 64 workgroups of universe j
// serving samples 1024 j ..: one length load per thread instead of the whole batch per
// workgroup (NIT 4 / 8: batch <= 8,192), and any batch size.  The per-universe deal leaves the
// most-loaded SIMD within a tile of the whole-batch one (a simulation at T = 50: 9.01 against 9.00
// tiles) and takes the kernel 40.3 -> 38.5 us at 4,096 (568.6 -> 553.6 us at 65,536 against
// contiguous samples), outputs bit-identical (profiles/r06/din_uni_ab.log).
constexpr int kDinBalMax = 8;  // NIT <= 8: batch <= 8192
constexpr int kDinBalClasses = 17;  // T <= 256 (16-position tiles)

// Inclusive prefix sum over the 64 lanes on the DPP network (no LDS round trips): row_shr 1/2/4/8
// within each 16-lane row, then row_bcast:15 / row_bcast:31 carry the row totals forward.
__device__ __forceinline__ int wave_incl_scan(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return v;
}

// Phase B's layer-0 K-chunks that run before the barrier closing phase A (mlp_stream.h
// PreChunks): the row's columns [0, 16 KS) — dense, category and query columns with the reference's
// layout [dense 16 | category 34 | query H | attention H] — are in LDS before any attention output
// is, so a wave that finishes its sample early accumulates them while the slowest sample is still
// in phase A (the matrix pipe is half idle there), and phase B opens with 8 - KS chunks of layer 0.
template <int H>
constexpr int din_pre_chunks() {
  return (16 + 34 + H) / 16 < 7 ? (16 + 34 + H) / 16 : 7;
}
// balanced launches gather each wave's row inside phase A: the waves count their rows in here
static __shared__ unsigned s_din_rows_ready;
// WAIT: balanced launches only (contiguous ones stage every row before the first barrier); a
// compile-time flag — a runtime member would be read back from scratch behind the weight ring
// DMA: the last four waves may have copied the epilogue image into LDS by LDS-DMA after their
// phase A: the copies retire before the barrier that opens phase B (loads
// retire in order; exactly the RK_STREAM_RING ring loads were issued after them).
template <bool WAIT, bool DMA>
struct DinRowsReady {
  __device__ void issue() const {}
  __device__ void operator()() const {
    if constexpr (DMA) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(RK_STREAM_RING) : "memory");
    if constexpr (WAIT) {
      while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_din_rows_ready, __ATOMIC_RELAXED,
                                                              __HIP_MEMORY_SCOPE_WORKGROUP)) < (unsigned)kMlpWaves)
        __builtin_amdgcn_s_sleep(1);
      asm volatile("" ::: "memory");  // the rows are read after the count
    }
  }
  __device__ void side() const {}
};

// P: the compiled layer plan of phase B (mlp_stream.h), or void for the generic mlp_rows.
// KS: phase B's layer-0 chunks run before the phase-A barrier (streamed plans; 0: none).
template <int H, int NIT, class P, int KS = 0>
__global__ __launch_bounds__(kMlpThreads) void din_forward_kernel(DinArgs a) {
  using Ly = DinLds<H>;
  constexpr int NQ = H / 8;
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* const buf0 = sm + Ly::BUF0;
  float* const buf1 = buf0 + kMlpRows * a.ld0;
  uint8_t* const col_seg = reinterpret_cast<uint8_t*>(buf1 + kMlpRows * a.ld1);
  uint8_t* const col_off = col_seg + 256;
  // the row segments' descriptors, copied to LDS so that the per-column lookups of the row
  // gather read them from LDS instead of the kernel-argument segment (one global round trip less)
  rk_segment* const lsegs = reinterpret_cast<rk_segment*>(col_seg + kDinSegLdsOff);

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5, hk = 4 * half;
  DIN_TS(0);

  // ---- the column map and the row segments' descriptors, issued first: with contiguous samples
  // (NIT == 0) they are in LDS one bare barrier later, and the feature-row gather starts while the
  // attention weights are still in flight
  static_assert(sizeof(rk_segment) % 4 == 0, "segment descriptor of whole words");
  const int seg_words = a.nseg * (int)(sizeof(rk_segment) / 4);
  uint8_t cs_v = 255, co_v = 0;
  int sw_v = 0;
  if (tid < 256) {
    cs_v = a.col_seg[tid];
    co_v = a.col_off[tid];
  }
  if (tid < seg_words) sw_v = reinterpret_cast<const int*>(&a.segs)[tid];

  // ---- per-sample tile counts: a sample needs ceil(min(len, T) / 16) attention tiles of 16
  // positions — positions past its length contribute exactly 0 (plain: masked weight 0; softmax:
  // exp(pad / sqrt(H) - max) underflows to 0) — except with softmax and len <= 0, where every
  // position carries the same pad score and all T count.
  const int64_t m0 = (int64_t)blockIdx.x * kMlpRows;
  const int ntiles_all = (a.T + 15) / 16;
  auto clamp_len = [&](int64_t len) { return len <= 0 ? 0 : (len >= a.T ? a.T : (int)len); };  // 32-bit math
  auto tiles_of = [&](int lc) { return lc ? (lc + 15) >> 4 : (a.use_softmax ? ntiles_all : 0); };
  // LDS after the descriptors: the history indices of positions 0..63 per LDS row ([16][64]), then
  // (NIT > 0) the batch row of each LDS row and the class masks
  int64_t* const kpre0 = reinterpret_cast<int64_t*>(col_seg + kDinSegLdsOff + sizeof(rk_segment) * kDinSegs);
  int64_t* const s_rows = kpre0 + 64 * kMlpRows;
  unsigned long long* const s_mask = reinterpret_cast<unsigned long long*>(s_rows + kMlpRows);  // NIT > 0
  int rows;
  int my_tiles = -1;  // NIT == 0, lanes 0..15: tiles of sample m0 + lane (-1: past the batch)
  int64_t my_len = 0;
  int64_t lv[NIT > 0 ? NIT : 1];  // NIT > 0: lengths of samples u0 + tid + 1024 r (clamped index)
  // NIT == 1: the ranking runs per 1,024-sample universe (samples u0 .. u0 + UB - 1, served by the
  // UG workgroups 64 j ..): one length per thread instead of the whole batch per workgroup
  int u0 = 0, UB = (int)a.batch, UG = (int)gridDim.x, ugl = (int)blockIdx.x;
  if constexpr (NIT == 1) {
    const int j = (int)blockIdx.x / (kMlpThreads / kMlpRows);
    u0 = j * kMlpThreads;
    UB = min(kMlpThreads, (int)(a.batch - u0));
    UG = (UB + kMlpRows - 1) / kMlpRows;
    ugl = (int)blockIdx.x - j * (kMlpThreads / kMlpRows);
  }
  if constexpr (NIT > 0) {
#pragma unroll
    for (int r = 0; r < NIT; ++r) {
      const int64_t i = u0 + tid + kMlpThreads * r;
      lv[r] = a.seq_len[i < a.batch ? i : a.batch - 1];
    }
  } else {
    rows = (int)min<int64_t>(kMlpRows, a.batch - m0);
    if (lane < rows) {
      my_len = a.seq_len[m0 + lane];
      my_tiles = tiles_of(clamp_len(my_len));
    }
  }

  // ---- the split attention weights: with a packed image (rk_din_pack_attention) one round of
  // coalesced float4 loads, all in flight at once, stored to LDS after the row gather is issued
  static_assert(Ly::U % 4 == 0, "image of whole float4s");
  constexpr int kImg4 = Ly::U / 4, kPer = (kImg4 + kMlpThreads - 1) / kMlpThreads;
  f32x4_t v[kPer];
  if (a.att_image) {
#pragma unroll
    for (int r = 0; r < kPer; ++r) {
      const int i = tid + r * kMlpThreads;
      if (i < kImg4) v[r] = reinterpret_cast<const f32x4_t*>(a.att_image)[i];
    }
  }
  // streamed phase B: its epilogue-parameter image rides with the attention image (phase A is long)
  using Epi = std::conditional_t<std::is_void_v<P>, NoStage, StreamEpi<std::conditional_t<std::is_void_v<P>, StreamPlanK128, P>>>;
  Epi epi_img;
  const bool epi_dma = a.epi_image != nullptr;  // copied after phase A instead (see DinArgs)
#ifndef RK_DIN_EXP_NOEPI  // timing experiment only: phase B without its epilogue parameters (wrong outputs)
  if constexpr (!std::is_void_v<P>)
    if (!epi_dma) epi_img.load(a.L, tid);
#endif
  auto image_to_lds = [&]() {
#ifndef RK_DIN_EXP_NOEPI
    if constexpr (!std::is_void_v<P>)
      if (!epi_dma) epi_img.store(sm + a.epi_off, tid);
#endif
    if (a.att_image) {
#pragma unroll
      for (int r = 0; r < kPer; ++r) {
        const int i = tid + r * kMlpThreads;
        if (i < kImg4) reinterpret_cast<f32x4_t*>(sm)[i] = v[r];
      }
    } else {
      for (int i = tid; i < 64 * H; i += kMlpThreads) {
        const int j = i / H, h = i % H;
        const float* r = a.w1 + (int64_t)j * 4 * H;
        sm[Ly::WQ + j * Ly::LDH + h] = r[h] + r[2 * H + h];
        sm[Ly::WK + j * Ly::LDH + h] = r[H + h] - r[2 * H + h];
        sm[Ly::WQK + j * Ly::LDH + h] = r[3 * H + h];
      }
      for (int i = tid; i < 32 * 64; i += kMlpThreads) sm[Ly::W2 + (i / 64) * 68 + (i % 64)] = a.w2[i];
      if (tid < 64) sm[Ly::B1 + tid] = a.b1[tid];
      if (tid < 32) {
        sm[Ly::B2 + tid] = a.b2[tid];
        sm[Ly::W3 + tid] = a.w3[tid];
      }
    }
  };
  if (tid < 256) {
    col_seg[tid] = cs_v;
    col_off[tid] = co_v;
  }
  if (tid < seg_words) reinterpret_cast<int*>(lsegs)[tid] = sw_v;
  uint32_t* flags = a.flags;

  // ---- the feature row of one sample (zero padded to pad64(width)) and its history indices of
  // positions 0..63 (lane = position, the first four tiles): the indices, the row's segment
  // indices, then the row values (two dependent rounds); rowp / kslot: its LDS row and index slot
  const int wp = pad64(a.width);
  constexpr int kColIt = 4;  // width <= 255: at most four 64-column passes
  int64_t kidx = 0;          // history index of position `lane`
  float cval[kColIt];
  auto gather_issue = [&](int64_t bs, bool lv_, int nt_) {
    if (lv_ && lane < 16 * nt_ && lane < a.T) kidx = a.seq[bs * a.ld_seq + lane];
    int64_t cidx[kColIt];
    int cseg[kColIt];
#pragma unroll
    for (int i = 0; i < kColIt; ++i) {
      const int c = lane + 64 * i;
      cseg[i] = (lv_ && c < a.width) ? col_seg[c] : 255;
      cidx[i] = bs;
      if (cseg[i] != 255 && lsegs[cseg[i]].idx) cidx[i] = lsegs[cseg[i]].idx[bs * lsegs[cseg[i]].idx_stride];
    }
#pragma unroll
    for (int i = 0; i < kColIt; ++i) {
      const int c = lane + 64 * i;
      cval[i] = 0.f;
      if (cseg[i] != 255) {
        const rk_segment& g = lsegs[cseg[i]];
        if (g.idx && (cidx[i] < 0 || cidx[i] >= g.rows))
          flag_oob(flags);
        else
          cval[i] = g.src[cidx[i] * g.src_ld + col_off[c]];
      }
    }
  };
  auto gather_store = [&](float* rowp, int64_t* kslot) {
    kslot[lane] = kidx;
#pragma unroll
    for (int i = 0; i < kColIt; ++i) {
      const int c = lane + 64 * i;
      if (c < wp) rowp[c] = cval[i];
    }
  };

  if constexpr (NIT == 0) {
    // wave w gathers sample m0 + w (LDS row w) while the weights stream in: the column map is in
    // LDS after a bare barrier (no wait on the weight loads), the tile counts are in lanes 0..15
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    const int tiles_w = __builtin_amdgcn_readlane(my_tiles, wave);
    gather_issue(m0 + wave, wave < rows, tiles_w);
    image_to_lds();
    gather_store(buf0 + wave * a.ld0, kpre0 + 64 * wave);
  } else {
    image_to_lds();
  }
  DIN_TS(5);
  if constexpr (NIT > 0) {  // class masks of the 64-sample blocks (block 16 r + wave holds sample tid + 1024 r)
    const int nblk = (UB + 63) / 64;
#pragma unroll
    for (int r = 0; r < NIT; ++r) {
      const int cls = tid + kMlpThreads * r < UB ? tiles_of(clamp_len(lv[r])) : -1;
      // class c's mask lands in lane c; lanes 0 .. nb-1 store them
      unsigned long long mk = 0;
#pragma unroll 1
      for (int c = 0; c < a.bal_nb; ++c) {
        const unsigned long long m = __ballot(cls == c);
        mk = lane == c ? m : mk;
      }
      const int blk = 16 * r + wave;
      if (blk < nblk && lane < a.bal_nb) s_mask[blk * a.bal_nb + lane] = mk;
    }
  }
  DIN_TS(6);
  if (KS > 0 && tid == 0) s_din_rows_ready = 0u;
  __syncthreads();
  DIN_TS(1);
#ifdef RK_DIN_PHASES
  const unsigned long long wave_t0 = clock64();
#endif

  // ---- balance the attention work over the SIMDs: waves w, w+4, w+8, w+12 share one SIMD (SIMD
  // w % 4, position w / 4), and the ranks (descending tile count) are dealt to the SIMDs in snake
  // order — position 0 takes ranks 0..3 on SIMDs 0..3, position 1 ranks 4..7 on SIMDs 3..0, and so
  // on: at T = 50 the SIMDs then carry 9/8/9/8 tiles instead of 10/9/8/7 (round 5; rank rho(w)).
  // Every wave computes the same ranking, from scalar reads of lanes 0..15.  (Balanced launches: the
  // ranks are already in descending tile order.)  A sample's LDS row is its rank in the workgroup.
  const int rho = (wave & ~3) | (((wave >> 2) & 1) ? 3 - (wave & 3) : (wave & 3));
  int loc, ntiles;
  int64_t len, b;
  bool live;
  if constexpr (NIT > 0) {
    const int G = UG, B = UB;  // the universe (NIT == 1) or the whole batch (<= 8192): 32-bit index math
    const int p = ugl + G * rho;  // this wave's rank
    rows = min(kMlpRows, (B - ugl + G - 1) / G);
    loc = rho;
    live = p < B;
    int cls = 0;
    b = 0;
    if (live) {
      const int nblk = (B + 63) / 64, bpl = nblk > 64 ? 2 : 1;  // 64-sample blocks per lane (nblk <= 128)
      // lane l's count of each class over its blocks l * bpl .. l * bpl + bpl - 1, prefix-summed
      // over the lanes; the rank's class is found walking the classes in descending order
      const int k0 = p;
      int start = 0, incl = 0, own = 0;
      cls = 0;
      for (int c = a.bal_nb - 1; c >= 0; --c) {
        const int blk = lane * bpl;
        int n = blk < nblk ? __builtin_popcountll(s_mask[blk * a.bal_nb + c]) : 0;
        if (bpl > 1 && blk + 1 < nblk) n += __builtin_popcountll(s_mask[(blk + 1) * a.bal_nb + c]);
        const int sc = wave_incl_scan(n);
        const int tot = __builtin_amdgcn_readlane(sc, 63);
        if (k0 < start + tot || c == 0) {
          cls = c;
          incl = sc;
          own = n;
          break;
        }
        start += tot;
      }
      // the (k0 - start)-th sample of that class in block order: the lane whose prefix passes it ...
      const int k = k0 - start;
      const int L = __builtin_ctzll(__ballot(incl > k));
      int kk = k - __builtin_amdgcn_readlane(incl - own, L);
      // ... then the block within the lane's share, then the bit within the block
      int blk = L * bpl;
      unsigned long long m = s_mask[blk * a.bal_nb + cls];
      if (bpl > 1 && kk >= __builtin_popcountll(m)) {
        kk -= __builtin_popcountll(m);
        m = s_mask[++blk * a.bal_nb + cls];
      }
      const int below = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
      const int pos = __builtin_ctzll(__ballot(((m >> lane) & 1ull) && below == kk));
      b = __builtin_amdgcn_readfirstlane(u0 + 64 * blk + pos);
    }
    ntiles = __builtin_amdgcn_readfirstlane(cls);
    // the length rides with phase A.1's loads (only the tile masks need it) — as a vector load: a
    // scalar one would hold up the lgkmcnt(0) waits of phase A.1's LDS reads
    int bv;
    asm volatile("v_mov_b32 %0, %1" : "=v"(bv) : "s"((int)b));
    len = live ? a.seq_len[bv] : 0;
    if (lane == 0) s_rows[loc] = b;
  } else {
    int rank = 0;
#pragma unroll
    for (int j = 0; j < kMlpRows; ++j) {
      const int tj = __builtin_amdgcn_readlane(my_tiles, j);
      rank += (tj > my_tiles) || (tj == my_tiles && j < lane);
    }
    const unsigned long long pick = __ballot(lane < kMlpRows && rank == rho);
    // wave-uniform values in scalar registers (readfirstlane): the sample's addresses stay scalar
    loc = __builtin_amdgcn_readfirstlane(pick ? __builtin_ctzll(pick) : wave);  // sample in the WG
    ntiles = __builtin_amdgcn_readfirstlane(max(0, __builtin_amdgcn_readlane(my_tiles, loc)));
    len = __shfl(my_len, loc, kWave);
    b = m0 + loc;
    live = loc < rows;
  }
#ifdef RK_DIN_SKIP_A  // timing experiment only (tools/din_phase_time.py): phase B on zero rows
  live = false;
#endif
  DIN_TS(4);
  float* row = buf0 + loc * a.ld0;
  // ---- Phase A on tiles of 16 history positions (v_mfma_f32_16x16x4_f32): lane l holds position
  // p16 = l & 15 of the tile and the key elements h in [HG g, HG g + HG), g = l >> 4, so a tile's 16
  // key rows are one 128-B load round per lane group.  Per tile (64 MFMAs, 128 MFMA-cycles per
  // position as the 32 x 32 form, but a sample pads only to 16 positions: 33 instead of 44
  // positions per sample at T = 50, lengths U[1, 50]):
  //   layer 1  acc1[jt] (j = 16 jt + 4 g + r, position p16) = Weff[j][h] . k[h], K = H: the A operand
  //            Weff = (W1b - W1c) + W1d diag(q) (rows 16 jt + p16, lane group g's h), built per sample
  //   ReLU(+ u[j])  on the accumulators; they are layer 2's B operands as they stand (K-step (jt, r)
  //            takes j = 16 jt + 4 g + r from lane group g)
  //   layer 2  acc2[jt2] (j2 = 16 jt2 + 4 g + r) = W2[j2][j] . h1[j], 16 K-steps
  //   layer 3  the score of each position: ReLU(acc2 + b2) . w3 over the lane's 8 values, summed over
  //            the 4 lane groups
  // then the masked (online) softmax and the weighted key sum o[h] over the tile's positions.
  constexpr int HG = H / 4;
  const int p16 = lane & 15, g = lane >> 4;
  const int64_t* const kslot = kpre0 + 64 * loc;  // indices of positions 0..63 (staged with the row)
  float kk[HG];  // keys of the current tile: position p16, elements HG g + e
  // key row of position t (index r) into kv; positions past T read as zeros, out-of-range rows too
  // (flagged)
  auto load_keys16 = [&](int64_t r, int t, float (&kv)[HG]) {
    const float* krow = nullptr;
    if (t < a.T) {
      if (r >= 0 && r < a.key_rows)
        krow = a.key_table + r * a.ld_key + HG * g;
      else
        flag_oob(flags);
#ifdef RK_DIN_NO_GATHER  // timing experiment only: the keys come from 16 cache-resident rows
      krow = a.key_table + (int64_t)p16 * a.ld_key + HG * g;
#endif
    }
    if constexpr (HG >= 4) {
#pragma unroll
      for (int c = 0; c < HG / 4; ++c) {
        const f32x4_t v4 = krow ? *reinterpret_cast<const f32x4_t*>(krow + 4 * c) : (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) kv[4 * c + e] = v4[e];
      }
    } else {
#pragma unroll
      for (int e = 0; e < HG; ++e) kv[e] = krow ? krow[e] : 0.f;
    }
  };
  auto index_of = [&](int t) -> int64_t { return t < 64 ? kslot[t] : (t < a.T ? a.seq[b * a.ld_seq + t] : 0); };
  // ---- Phase A.1: the first tile's keys.  NIT == 0: the row and the indices are in LDS already
  // (gathered before the barrier above).  NIT > 0: the row, the indices and then the keys for the
  // assigned sample, the row going to LDS while the key rows are still in flight.
  if constexpr (NIT == 0) {
    if (live && ntiles > 0) load_keys16(kslot[p16], p16, kk);
  } else {
    gather_issue(b, live, ntiles);
    const uint32_t lo = __shfl((uint32_t)kidx, p16, kWave), hi = __shfl((uint32_t)((uint64_t)kidx >> 32), p16, kWave);
    if (live && ntiles > 0) load_keys16((int64_t)(((uint64_t)hi << 32) | lo), p16, kk);
    gather_store(row, kpre0 + 64 * loc);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  if constexpr (NIT > 0 && KS > 0) {  // this wave's row is in LDS (its stores completed above)
    if (lane == 0) __hip_atomic_fetch_add(&s_din_rows_ready, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
#ifdef RK_DIN_PHASES
  if (tid == 0) {  // wave 0: its row in LDS and its first tile's keys landed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    s_din_ts[7] = wall_clock64();
  }
#endif

  float norm_part = 0.f;
  if (live) {
    // ---- Phase A.2: per-sample bias u[j] = b1[j] + q . Wq[j]   (lane j)
    {
      float u = sm[Ly::B1 + lane];
      const float* wq = sm + Ly::WQ + lane * Ly::LDH;
      const float* q = row + a.q_col;
#pragma unroll
      for (int h = 0; h < H; ++h) u = fmaf(q[h], wq[h], u);
      sm[Ly::U + wave * 64 + lane] = u;
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    float qv[HG];  // the query elements of lane group g
#pragma unroll
    for (int e = 0; e < HG; ++e) qv[e] = row[a.q_col + HG * g + e];

    const float sqrt_h = (float)__builtin_sqrt((double)H);
    const float pad = -4294967296.0f;  // (-2**32 + 1) rounded to fp32, din.py:74
    const float b3 = a.b3[0];
    float m_run = -INFINITY, l_run = 0.f;
    float o[HG];
#pragma unroll
    for (int e = 0; e < HG; ++e) o[e] = 0.f;
    // RK_DIN_HOIST (experiment, off): layer 1's A operand Weff built once per sample in 32 VGPRs
    // instead of per tile from LDS (118 VGPRs, no spill; half the tile's LDS reads and 32 fewer FMAs
    // per tile) measured flat (42.0 / 42.7 us against 41.8 / 42.7 us per launch,
    // profiles/r04/ab_hoist*.json): phase A is not bound by the operand's LDS reads
#if RK_DIN_HOIST
    float weff[4][HG];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) {
      const float* wk = sm + Ly::WK + (16 * jt + p16) * Ly::LDH + HG * g;
      const float* wqk = sm + Ly::WQK + (16 * jt + p16) * Ly::LDH + HG * g;
#pragma unroll
      for (int e = 0; e < HG; ++e) weff[jt][e] = fmaf(wqk[e], qv[e], wk[e]);
    }
#endif
    for (int tt = 0; tt < ntiles; ++tt) {
      // the weight LDS reads below are loop-invariant (kept in the loop: see RK_DIN_HOIST above)
      asm volatile("" ::: "memory");
      const int t = 16 * tt + p16;
      const bool in_seq = t < a.T;
      // the next tile's keys go out before this tile's MFMAs
      float kn[HG];
      const bool more = tt + 1 < ntiles;
      if (more) load_keys16(index_of(t + 16), t + 16, kn);
      f32x4_t acc1[4];
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) acc1[jt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      // layer 1's A operand, Weff[16 jt + p16][HG g + e] = Wk + Wqk q (rows of the LDS image)
#if RK_DIN_HOIST
#pragma unroll
      for (int e = 0; e < HG; ++e) {
#pragma unroll
        for (int jt = 0; jt < 4; ++jt) acc1[jt] = mfma16(weff[jt][e], kk[e], acc1[jt]);
      }
#else
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const float* wk = sm + Ly::WK + (16 * jt + p16) * Ly::LDH + HG * g;
        const float* wqk = sm + Ly::WQK + (16 * jt + p16) * Ly::LDH + HG * g;
#pragma unroll
        for (int e = 0; e < HG; ++e) acc1[jt] = mfma16(fmaf(wqk[e], qv[e], wk[e]), kk[e], acc1[jt]);
      }
#endif
      // ReLU(layer 1 + u) in place, then layer 2 with the accumulators as its B operands
      f32x4_t acc2[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        const f32x4_t uu = *reinterpret_cast<const f32x4_t*>(sm + Ly::U + wave * 64 + 16 * jt + 4 * g);
        f32x4_t w2[2];
#pragma unroll
        for (int jt2 = 0; jt2 < 2; ++jt2)
          w2[jt2] = *reinterpret_cast<const f32x4_t*>(sm + Ly::W2 + (16 * jt2 + p16) * 68 + 16 * jt + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float z = acc1[jt][r] + uu[r];
          const float h1 = z < 0.f ? 0.f : z;
#pragma unroll
          for (int jt2 = 0; jt2 < 2; ++jt2) acc2[jt2] = mfma16(w2[jt2][r], h1, acc2[jt2]);
        }
      }
      // layer 3: the position's score
      float sc = 0.f;
#pragma unroll
      for (int jt2 = 0; jt2 < 2; ++jt2) {
        const f32x4_t b2v = *reinterpret_cast<const f32x4_t*>(sm + Ly::B2 + 16 * jt2 + 4 * g);
        const f32x4_t w3v = *reinterpret_cast<const f32x4_t*>(sm + Ly::W3 + 16 * jt2 + 4 * g);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float z = acc2[jt2][r] + b2v[r];
          z = z < 0.f ? 0.f : z;
          sc = fmaf(z, w3v[r], sc);
        }
      }
      sc = xor32_sum(xor16_sum(sc));  // bit-identical to the two xor shuffles, no LDS round trip
      sc = sc + b3;

      const bool valid = in_seq && (int64_t)t < len;
      if (a.use_softmax) {
        const float sv = in_seq ? (valid ? sc : pad) / sqrt_h : -INFINITY;
        const float mt = row16_max(sv);
        const float m_new = fmaxf(m_run, mt);
        const float scale_old = expf(m_run - m_new);
        const float p = in_seq ? expf(sv - m_new) : 0.f;
        const float ps = row16_sum(p);
        l_run = l_run * scale_old + ps;
        m_run = m_new;
#pragma unroll
        for (int e = 0; e < HG; ++e) o[e] = o[e] * scale_old + p * kk[e];
      } else {
        const float w = valid ? sc : 0.f;
#pragma unroll
        for (int e = 0; e < HG; ++e) o[e] = o[e] + w * kk[e];
      }
      if (more) {
#pragma unroll
        for (int e = 0; e < HG; ++e) kk[e] = kn[e];
      }
    }
    // the weighted key sum over the positions (the 16 lanes of a group), into the LDS row
    const float inv_l = a.use_softmax ? 1.0f / l_run : 1.0f;
    float mine = 0.f;
#pragma unroll
    for (int e = 0; e < HG; ++e) {
      const float v = row16_sum(o[e]);
      mine = p16 == e ? v : mine;
    }
    if (p16 < HG) row[a.att_col + HG * g + p16] = a.use_softmax ? mine * inv_l : mine;
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    if (a.l2_part) {
      float ss = 0.f;
      for (int c = a.l2_col0 + lane; c < a.width; c += 64) ss = fmaf(row[c], row[c], ss);
      norm_part = sqrtf(wave_sum(ss));
    }
  }
  if (lane == 0) sm[Ly::NORM + wave] = norm_part;
#ifdef RK_DIN_PHASES
  if (lane == 0) s_din_wave[wave] = clock64() - wave_t0;
#endif
  DIN_TS(2);  // (tid 0's own phase A: no workgroup barrier here any more)

  // ---- Phase B: fcn tail + head over the 16 rows.  No barrier in front of it: each wave issues
  // its layer-0 weight ring (mlp_rows' prepare) as soon as its own phase A is done, and mlp_rows'
  // barrier after that prepare closes phase A, so the ring's latency overlaps the wait for the
  // slowest sample instead of opening phase B.
#ifdef RK_DIN_SKIP_B  // timing experiment only (tools/din_phase_time.py)
  return;
#endif
  if constexpr (!std::is_void_v<P>) {
    // the epilogue image by LDS-DMA (1 KiB per wave instruction) from the four waves with the
    // shortest samples (either assignment gives wave j the j-th longest sample of the workgroup),
    // which reach this point first
    constexpr int kBlocks = P::epi_floats() / 256;
    static_assert(P::epi_floats() % 256 == 0, "epilogue image of whole 1 KiB blocks");
    if (epi_dma && wave >= kMlpWaves - 4) {
      for (int k = wave - (kMlpWaves - 4); k < kBlocks; k += 4)
        __builtin_amdgcn_global_load_lds((glb_void*)(a.epi_image + 256 * k + 4 * lane),
                                         (lds_void*)(sm + a.epi_off + 256 * k), 16, 0, 0);
    }
  }
  if constexpr (std::is_void_v<P>)
    mlp_rows(a.L, a.nl, a.width, buf0, a.ld0, buf1, a.ld1, m0, rows, a.head, nullptr, 0, tid, NoStage(), nullptr,
             NIT > 0 ? s_rows : nullptr);
  else
    mlp_stream_rows<P, kEpiLdsCaller>(a.L, buf0, a.ld0, buf1, a.ld1, sm + a.epi_off, m0, rows, a.head, tid,
                                      PreChunks<KS, DinRowsReady<(NIT > 0 && KS > 0), true>>{}, nullptr,
                                      NIT > 0 ? s_rows : nullptr);
  DIN_TS(3);
  // l2 partials: the last workgroup to publish its partial finishes the mean.  Hand-off by atomic
  // read-modify-writes only (round 6): one lane per workgroup publishes its
  // partial with an agent-scope atomic exchange and waits for its return (the exchange is then
  // performed at the location's coherence point), then adds to ONE counter (agent-scope atomic); the
  // workgroup whose add returns n-1 reads every partial with an atomic fetch-add of 0.  Every access
  // of the hand-off is an agent-scope RMW on a single location — coherent across the XCDs (the RMWs
  // of one location are totally ordered at its coherence point) — and the order across locations is
  // by completion: a partial's exchange has returned before its workgroup's add is issued, and the
  // reader issues its partial RMWs after its own add returned n-1.  That is not a C++ happens-before
  // (which would take a release / acquire pair: buffer_wbl2 / buffer_inv, 1.7-3.5 us each on the
  // critical path), but unlike rounds 3-5's sc1 plain stores and loads it does not depend on how a
  // cache treats non-atomic accesses.  The partials are non-negative sums of norms, so adding 0
  // returns them unchanged.
  // tests/test_gpu_din_plan.py checks l2 against the deterministic host-order sum over repeated
  // launches.  (The norms in LDS were ordered before this by mlp_rows' barriers.)
  if (a.l2_part && tid < 64) {
    unsigned prev = 0;
    if (tid == 0) {
      float t = 0.f;
      for (int w = 0; w < kMlpRows; ++w) t += sm[Ly::NORM + w];
      const float old = __hip_atomic_exchange(a.l2_part + blockIdx.x, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      // the counter's add waits for the exchange to return (a use of its result orders it after)
      unsigned one = 1u;
      asm volatile("s_waitcnt vmcnt(0)" : "+v"(one) : "v"(old) : "memory");
      prev = __hip_atomic_fetch_add(a.l2_count, one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev == gridDim.x - 1) {
      float t = 0.f;
      for (int i = tid; i < (int)gridDim.x; i += 64)
        t += __hip_atomic_fetch_add(a.l2_part + i, 0.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      t = wave_sum(t);  // the order of row_l2norm_final_kernel (embedding.hip)
      if (tid == 0) {
        a.l2_out[0] = a.l2_scale * (t / (float)a.batch);
        __hip_atomic_store(a.l2_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
#ifdef RK_DIN_PHASES
  din_marks_flush(tid);
#endif
  MLP_FLUSH(tid);
}

// The LDS image of the split attention weights (see the layout above): WK = W1b - W1c,
// WQK = W1d, WQ = W1a + W1c (rows of H, stride H + 4), W2 (32 x 64, stride 68), b1, b2, w3.
template <int H>
__global__ __launch_bounds__(256) void din_pack_attention_kernel(const float* __restrict__ w1,
                                                                 const float* __restrict__ b1,
                                                                 const float* __restrict__ w2,
                                                                 const float* __restrict__ b2,
                                                                 const float* __restrict__ w3, float* __restrict__ img) {
  using Ly = DinLds<H>;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < Ly::U; i += gridDim.x * blockDim.x) {
    float v = 0.f;
    if (i < Ly::W2) {
      const int which = i / (64 * Ly::LDH), rem = i % (64 * Ly::LDH), j = rem / Ly::LDH, h = rem % Ly::LDH;
      if (h < H) {
        const float* r = w1 + (int64_t)j * 4 * H;
        v = which == 0 ? r[H + h] - r[2 * H + h] : which == 1 ? r[3 * H + h] : r[h] + r[2 * H + h];
      }
    } else if (i < Ly::B1) {
      const int k = i - Ly::W2, j = k / 68, c = k % 68;
      v = c < 64 ? w2[j * 64 + c] : 0.f;
    } else if (i < Ly::B2) {
      v = b1[i - Ly::B1];
    } else if (i < Ly::W3) {
      v = b2[i - Ly::B2];
    } else {
      v = w3[i - Ly::W3];
    }
    img[i] = v;
  }
}

}  // namespace rk

using namespace rk;

RK_API int64_t rk_din_attention_image_floats(int32_t H) {
  switch (H) {
    case 8: return DinLds<8>::U;
    case 16: return DinLds<16>::U;
    case 32: return DinLds<32>::U;
    default: return 0;
  }
}

RK_API int rk_din_pack_attention(const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                                 int32_t H, float* image, void* stream) {
  if (!w1 || !b1 || !w2 || !b2 || !w3 || !image || ((uintptr_t)image & 15u))
    return fail(RK_ERR_INVALID, "rk_din_pack_attention: null or misaligned pointer");
  hipStream_t st = (hipStream_t)stream;
  switch (H) {
    case 8: din_pack_attention_kernel<8><<<8, 256, 0, st>>>(w1, b1, w2, b2, w3, image); break;
    case 16: din_pack_attention_kernel<16><<<16, 256, 0, st>>>(w1, b1, w2, b2, w3, image); break;
    case 32: din_pack_attention_kernel<32><<<36, 256, 0, st>>>(w1, b1, w2, b2, w3, image); break;
    default: return fail(RK_ERR_UNSUPPORTED, "rk_din_pack_attention: embedding dim %d not in {8,16,32}", H);
  }
  return check_launch("rk_din_pack_attention");
}

namespace rk {
// A prepared launch of din_forward_kernel: validated arguments, grid and LDS size.
struct DinPlan {
  DinArgs a;
  int64_t blocks;
  size_t shm;
  int H;
  int nit;     // balanced assignment: seq_len loads per thread (0: contiguous 16-sample blocks)
  int stream;  // phase B on the streamed plan (kStreamK128) or mlp_rows (kStreamNone)
  int pre;     // streamed plan: phase B's layer-0 chunks before the phase-A barrier (din_pre_chunks)
};
}  // namespace rk

static int din_prepare(const rk_segment* row_segs, int32_t nseg, int32_t width, int32_t q_col, int32_t att_col,
                          const float* key_table, int64_t key_rows, int64_t ld_key, const int64_t* seq,
                          int64_t ld_seq, int32_t T, const int64_t* seq_len, int64_t batch, int32_t H,
                          const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                          const float* b3, int32_t use_softmax, const rk_mlp_layer* layers, int32_t nlayers,
                          const rk_epilogue* head, int32_t l2_col0, float l2_scale, float* l2_workspace,
                          float* l2_out, const float* att_image, DinPlan* plan) {
  if (!row_segs || nseg <= 0 || nseg > kDinSegs)
    return fail(RK_ERR_UNSUPPORTED, "rk_din_forward: %d row segments (max %d)", nseg, kDinSegs);
  if (!key_table || !seq || !seq_len || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !head || !head->head_w)
    return fail(RK_ERR_INVALID, "rk_din_forward: null pointer");
  if (H != 8 && H != 16 && H != 32)
    return fail(RK_ERR_UNSUPPORTED, "rk_din_forward: embedding dim %d not in {8,16,32}", H);
  if (width <= 0 || width > 255 || q_col < 0 || q_col + H > width || att_col < 0 || att_col + H > width ||
      T <= 0 || ld_seq < T || key_rows <= 0 || ld_key < H || ld_key % 4 || ((uintptr_t)key_table & 15u))
    return fail(RK_ERR_INVALID, "rk_din_forward: bad row/sequence layout (width=%d T=%d H=%d)", width, T, H);
  if (l2_out && (!l2_workspace || l2_col0 < 0 || l2_col0 >= width || ((uintptr_t)l2_workspace & 3u)))
    return fail(RK_ERR_INVALID, "rk_din_forward: l2 term needs a workspace of ceil(batch/16) + 1 words");
  *plan = DinPlan{};
  DinArgs& a = plan->a;
  plan->H = H;
  for (int s = 0; s < nseg; ++s) {
    const rk_segment& g = row_segs[s];
    if (!g.src || g.dim <= 0 || g.out_col < 0 || g.out_col + g.dim > width || g.dim > 255 || (g.idx && g.rows <= 0))
      return fail(RK_ERR_INVALID, "rk_din_forward: row segment %d invalid", s);
    a.segs.s[s] = g;
  }
  if (att_image && ((uintptr_t)att_image & 15u)) return fail(RK_ERR_INVALID, "rk_din_forward: att_image not 16-B aligned");
  a.att_image = att_image;
  for (int c = 0; c < 256; ++c) {  // column map (rk_concat_gather semantics: the last covering segment wins)
    uint8_t hit = 255, off = 0;
    for (int s = 0; s < nseg && c < width; ++s)
      if (c >= row_segs[s].out_col && c < row_segs[s].out_col + row_segs[s].dim) {
        hit = (uint8_t)s;
        off = (uint8_t)(c - row_segs[s].out_col);
      }
    a.col_seg[c] = hit;
    a.col_off[c] = off;
  }
  a.head = *head;
  int need0 = 0, need1 = 0;
  if (int e = mlp_validate(layers, nlayers, width, a.head, &need0, &need1, "rk_din_forward")) return e;
  for (int l = 0; l < nlayers; ++l) a.L[l] = layers[l];
  a.nl = nlayers;
  a.nseg = nseg;
  a.width = width;
  a.q_col = q_col;
  a.att_col = att_col;
  a.l2_col0 = l2_col0;
  a.key_table = key_table;
  a.key_rows = key_rows;
  a.ld_key = ld_key;
  a.seq = seq;
  a.ld_seq = ld_seq;
  a.T = T;
  a.seq_len = seq_len;
  a.batch = batch;
  a.w1 = w1;
  a.b1 = b1;
  a.w2 = w2;
  a.b2 = b2;
  a.w3 = w3;
  a.b3 = b3;
  a.use_softmax = use_softmax;
  a.l2_part = l2_out ? l2_workspace : nullptr;
  a.l2_count = l2_out ? reinterpret_cast<unsigned*>(l2_workspace + (batch + kMlpRows - 1) / kMlpRows) : nullptr;
  a.l2_out = l2_out;
  a.l2_scale = l2_scale;
  a.flags = device_flags();
  a.ld0 = need0 + kMlpLdPad;
  a.ld1 = need1 + kMlpLdPad;
  static_assert(sizeof(DinArgs) <= 4096, "kernel arguments beyond 4 KiB");
  if (batch < 0) return fail(RK_ERR_INVALID, "rk_din_forward: negative batch");
  plan->blocks = (batch + kMlpRows - 1) / kMlpRows;
  size_t base = 0;
  switch (H) {
    case 8: base = DinLds<8>::BUF0; break;
    case 16: base = DinLds<16>::BUF0; break;
    default: base = DinLds<32>::BUF0; break;
  }
  size_t shm = (base + (size_t)kMlpRows * (a.ld0 + a.ld1)) * sizeof(float) + kDinSegLdsOff +
               sizeof(rk_segment) * kDinSegs + sizeof(int64_t) * 64 * kMlpRows;
  if (shm > 160 * 1024 - kStreamStaticLds) return fail(RK_ERR_UNSUPPORTED, "rk_din_forward: %zu B of LDS needed", shm);
  // balanced assignment (see din_forward_kernel): per 1,024-sample universe at any batch (NIT 1),
  // or (RANKOPS_DIN_UNI=0) over the whole batch up to 8,192 samples (NIT 4 / 8), by default when
  // the histories span three or more 16-position tile counts (T > 32).  Measured
  // (round 3, 32-position tiles, graph replays, batch 4096, lengths uniform in 1..T): T = 128
  // 74.7 -> 68.9 us, T = 256 100.9 -> 91.9 us; round 4 (16-position tiles) at T = 50, kernel averages
  // over two interleaved A/B pairs: 45.18 / 44.22 -> 44.05 / 43.59 us (profiles/r04/ab_bal_*).
  // RANKOPS_DIN_BALANCE=1 / 0 forces it on / off (tests, A/B timing).  Only where its LDS (the
  // batch row of each LDS row and the class masks) still fits: otherwise contiguous samples.
  const char* env = getenv("RANKOPS_DIN_BALANCE");
  a.bal_nb = (T + 15) / 16 + 1;  // tile-count classes 0 .. ceil(T / 16)
  const bool want_bal = env && env[0] ? env[0] != '0' : T > 32;
  const char* uni_env = getenv("RANKOPS_DIN_UNI");  // 0: rank the whole batch (NIT 4 / 8, A/B)
  const bool uni = !(uni_env && uni_env[0] == '0');
  if (want_bal && batch > kMlpRows && (uni || batch <= kDinBalMax * kMlpThreads) && a.bal_nb <= kDinBalClasses) {
    const int64_t ranked = uni ? std::min<int64_t>(batch, kMlpThreads) : batch;
    const size_t extra = sizeof(int64_t) * kMlpRows + sizeof(unsigned long long) * ((ranked + 63) / 64) * a.bal_nb;
    if (shm + extra <= 160 * 1024 - kStreamStaticLds) {
      plan->nit = uni ? 1 : batch <= 4 * kMlpThreads ? 4 : kDinBalMax;
      shm += extra;
    }
  }
  // phase B on the streamed plan (hidden units [512, 256, 128] over a row of <= 128): its
  // epilogue-parameter image goes last, where it still fits
  plan->stream = stream_plan_for(layers, nlayers, width) == kStreamK128 ? kStreamK128 : kStreamNone;
  if (plan->stream != kStreamNone) {
    shm = (shm + 15) / 16 * 16;
    const size_t bytes = sizeof(float) * stream_plan_epi_floats(kStreamK128);
    if (shm + bytes <= 160 * 1024 - kStreamStaticLds) {
      a.epi_off = (int)(shm / sizeof(float));
      shm += bytes;
    } else {
      plan->stream = kStreamNone;
    }
  }
  // the pre-barrier chunks need every column they read outside the attention output (the only
  // columns phase A writes); RANKOPS_DIN_PRE=0 turns them off (A/B timing)
  if (plan->stream != kStreamNone) {
    const int ks = H == 8 ? din_pre_chunks<8>() : H == 16 ? din_pre_chunks<16>() : din_pre_chunks<32>();
    const char* pe = getenv("RANKOPS_DIN_PRE");
    plan->pre = (pe && pe[0] == '0') || att_col < 16 * ks ? 0 : ks;
  }
  plan->shm = shm;
  return RK_OK;
}

static int din_launch(const DinPlan& p, hipStream_t st) {
  if (p.blocks == 0) return RK_OK;
  const unsigned blocks = (unsigned)p.blocks;
  auto go = [&](auto kern) {
    raise_lds_limit((const void*)kern, 160 * 1024);
    kern<<<blocks, kMlpThreads, p.shm, st>>>(p.a);
  };
  if (p.stream == kStreamK128 && p.pre > 0) {
    using S = StreamPlanK128;
    switch (p.H * 16 + p.nit) {
      case 8 * 16: go(din_forward_kernel<8, 0, S, din_pre_chunks<8>()>); break;
      case 8 * 16 + 1: go(din_forward_kernel<8, 1, S, din_pre_chunks<8>()>); break;
      case 8 * 16 + 4: go(din_forward_kernel<8, 4, S, din_pre_chunks<8>()>); break;
      case 8 * 16 + 8: go(din_forward_kernel<8, 8, S, din_pre_chunks<8>()>); break;
      case 16 * 16: go(din_forward_kernel<16, 0, S, din_pre_chunks<16>()>); break;
      case 16 * 16 + 1: go(din_forward_kernel<16, 1, S, din_pre_chunks<16>()>); break;
      case 16 * 16 + 4: go(din_forward_kernel<16, 4, S, din_pre_chunks<16>()>); break;
      case 16 * 16 + 8: go(din_forward_kernel<16, 8, S, din_pre_chunks<16>()>); break;
      case 32 * 16: go(din_forward_kernel<32, 0, S, din_pre_chunks<32>()>); break;
      case 32 * 16 + 1: go(din_forward_kernel<32, 1, S, din_pre_chunks<32>()>); break;
      case 32 * 16 + 4: go(din_forward_kernel<32, 4, S, din_pre_chunks<32>()>); break;
      default: go(din_forward_kernel<32, 8, S, din_pre_chunks<32>()>); break;
    }
    return check_launch("rk_din_forward");
  }
  if (p.stream == kStreamK128) {
    using S = StreamPlanK128;
    switch (p.H * 16 + p.nit) {
      case 8 * 16: go(din_forward_kernel<8, 0, S>); break;
      case 8 * 16 + 1: go(din_forward_kernel<8, 1, S>); break;
      case 8 * 16 + 4: go(din_forward_kernel<8, 4, S>); break;
      case 8 * 16 + 8: go(din_forward_kernel<8, 8, S>); break;
      case 16 * 16: go(din_forward_kernel<16, 0, S>); break;
      case 16 * 16 + 1: go(din_forward_kernel<16, 1, S>); break;
      case 16 * 16 + 4: go(din_forward_kernel<16, 4, S>); break;
      case 16 * 16 + 8: go(din_forward_kernel<16, 8, S>); break;
      case 32 * 16: go(din_forward_kernel<32, 0, S>); break;
      case 32 * 16 + 1: go(din_forward_kernel<32, 1, S>); break;
      case 32 * 16 + 4: go(din_forward_kernel<32, 4, S>); break;
      default: go(din_forward_kernel<32, 8, S>); break;
    }
    return check_launch("rk_din_forward");
  }
  switch (p.H * 16 + p.nit) {
    case 8 * 16: go(din_forward_kernel<8, 0, void>); break;
    case 8 * 16 + 1: go(din_forward_kernel<8, 1, void>); break;
    case 8 * 16 + 4: go(din_forward_kernel<8, 4, void>); break;
    case 8 * 16 + 8: go(din_forward_kernel<8, 8, void>); break;
    case 16 * 16: go(din_forward_kernel<16, 0, void>); break;
    case 16 * 16 + 1: go(din_forward_kernel<16, 1, void>); break;
    case 16 * 16 + 4: go(din_forward_kernel<16, 4, void>); break;
    case 16 * 16 + 8: go(din_forward_kernel<16, 8, void>); break;
    case 32 * 16: go(din_forward_kernel<32, 0, void>); break;
    case 32 * 16 + 1: go(din_forward_kernel<32, 1, void>); break;
    case 32 * 16 + 4: go(din_forward_kernel<32, 4, void>); break;
    default: go(din_forward_kernel<32, 8, void>); break;
  }
  return check_launch("rk_din_forward");
}

#define RK_DIN_ARG_NAMES                                                                                          \
  row_segs, nseg, width, q_col, att_col, key_table, key_rows, ld_key, seq, ld_seq, T, seq_len, batch, H, w1, b1, \
      w2, b2, w3, b3, use_softmax, layers, nlayers, head, l2_col0, l2_scale, l2_workspace, l2_out, att_image

RK_API int rk_din_forward(const rk_segment* row_segs, int32_t nseg, int32_t width, int32_t q_col, int32_t att_col,
                          const float* key_table, int64_t key_rows, int64_t ld_key, const int64_t* seq,
                          int64_t ld_seq, int32_t T, const int64_t* seq_len, int64_t batch, int32_t H,
                          const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                          const float* b3, int32_t use_softmax, const rk_mlp_layer* layers, int32_t nlayers,
                          const rk_epilogue* head, int32_t l2_col0, float l2_scale, float* l2_workspace,
                          float* l2_out, const float* att_image, void* stream) {
  DinPlan p;
  if (int e = din_prepare(RK_DIN_ARG_NAMES, &p)) return e;
  return din_launch(p, (hipStream_t)stream);
}

RK_API int rk_din_forward_ex(const rk_segment* row_segs, int32_t nseg, int32_t width, int32_t q_col, int32_t att_col,
                             const float* key_table, int64_t key_rows, int64_t ld_key, const int64_t* seq,
                             int64_t ld_seq, int32_t T, const int64_t* seq_len, int64_t batch, int32_t H,
                             const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                             const float* b3, int32_t use_softmax, const rk_mlp_layer* layers, int32_t nlayers,
                             const rk_epilogue* head, int32_t l2_col0, float l2_scale, float* l2_workspace,
                             float* l2_out, const float* att_image, const float* epi_image, void* stream) {
  if (epi_image && ((uintptr_t)epi_image & 15u)) return fail(RK_ERR_INVALID, "rk_din_forward_ex: misaligned epi_image");
  DinPlan p;
  if (int e = din_prepare(RK_DIN_ARG_NAMES, &p)) return e;
  if (p.stream == kStreamK128) p.a.epi_image = epi_image;  // (other phase-B paths resolve at launch)
  return din_launch(p, (hipStream_t)stream);
}

RK_API int rk_din_forward_plan(const rk_segment* row_segs, int32_t nseg, int32_t width, int32_t q_col, int32_t att_col,
                          const float* key_table, int64_t key_rows, int64_t ld_key, const int64_t* seq,
                          int64_t ld_seq, int32_t T, const int64_t* seq_len, int64_t batch, int32_t H,
                          const float* w1, const float* b1, const float* w2, const float* b2, const float* w3,
                          const float* b3, int32_t use_softmax, const rk_mlp_layer* layers, int32_t nlayers,
                          const rk_epilogue* head, int32_t l2_col0, float l2_scale, float* l2_workspace,
                          float* l2_out, const float* att_image, void** plan_out) {
  if (!plan_out) return fail(RK_ERR_INVALID, "rk_din_forward_plan: null plan_out");
  *plan_out = nullptr;
  DinPlan* p = new (std::nothrow) DinPlan;
  if (!p) return fail(RK_ERR_RUNTIME, "rk_din_forward_plan: out of host memory");
  if (int e = din_prepare(RK_DIN_ARG_NAMES, p)) {
    delete p;
    return e;
  }
  *plan_out = p;
  return RK_OK;
}

RK_API int rk_din_plan_launch(const void* plan, void* stream) {
  if (!plan) return fail(RK_ERR_INVALID, "rk_din_plan_launch: null plan");
  return din_launch(*static_cast<const DinPlan*>(plan), (hipStream_t)stream);
}

RK_API void rk_din_plan_destroy(void* plan) { delete static_cast<DinPlan*>(plan); }

RK_API int rk_din_plan_set_epilogue_image(void* plan, const float* image) {
  if (!plan) return fail(RK_ERR_INVALID, "rk_din_plan_set_epilogue_image: null plan");
  DinPlan& p = *static_cast<DinPlan*>(plan);
  if (image && ((uintptr_t)image & 15u)) return fail(RK_ERR_INVALID, "rk_din_plan_set_epilogue_image: misaligned image");
  if (image && p.stream != kStreamK128)
    return fail(RK_ERR_UNSUPPORTED, "rk_din_plan_set_epilogue_image: the plan has no streamed phase B");
  p.a.epi_image = image;
  return RK_OK;
}

#ifdef RK_DIN_PHASES
RK_API int rk_debug_din_phases(unsigned long long* ts, unsigned long long* waves, unsigned long long* mlp) {
  if (hipMemcpyFromSymbol(ts, HIP_SYMBOL(g_din_ts), sizeof(g_din_ts)) != hipSuccess) return 1;
  if (hipMemcpyFromSymbol(waves, HIP_SYMBOL(g_din_wave), sizeof(g_din_wave)) != hipSuccess) return 1;
#ifdef RK_MLP_PHASES
  if (hipMemcpyFromSymbol(mlp, HIP_SYMBOL(g_mlp_marks), sizeof(g_mlp_marks[0]) * kDinPhaseWG) != hipSuccess) return 1;
#else
  (void)mlp;
#endif
  return 0;
}
#endif
