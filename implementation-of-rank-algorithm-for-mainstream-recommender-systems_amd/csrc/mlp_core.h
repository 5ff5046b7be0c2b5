// Fused-MLP machinery shared by rk_mlp_forward (mlp.hip) and the fused DIN forward (din_fused.hip).
//
// 16 rows (x RT row tiles) per workgroup of 16 waves (4 per SIMD).  Activations live in two LDS
// buffers; each layer reads one and writes the other.  Layer math is FP32 MFMA
// v_mfma_f32_16x16x4_f32 (exact f32): wave w owns output tiles w and w+16 (16 columns each).  Per
// 16-deep K chunk a lane reads one float4 of its A row from LDS (k = 16c + 4*(lane>>4) + e, one
// chunk ahead) and one float4 of its weight row per tile from global memory (a 4-deep register
// ring), then issues 4 MFMAs per tile.  Weights are pre-packed (rk_mlp_pack_weight: rows padded
// to 64 columns, K padded to 64, zero fill), so every weight load is an unconditional aligned
// float4.  Each layer's weight ring and per-column epilogue parameters are issued before the
// barrier that closes the previous layer (LayerPipe::prepare + an LDS-only barrier), and the
// epilogue parameters sit in registers: read after the LDS stores they were re-fetched per
// element behind the whole weight-load queue (tools/mlp_phases.hip: DeepFM layer-0 epilogue
// 38k -> 8k cycles; DIN 48.8 -> 51.4 M samples/s).
#pragma once

#include <type_traits>

#include "common.h"

namespace rk {

#ifndef RK_MLP_EPI_PRIO
#define RK_MLP_EPI_PRIO 1
#endif
// Lockstep within a layer: every kMlpSyncChunks K-chunks all waves meet at a barrier.  Without it
// the SIMD's matrix pipe serves its 4 waves oldest-first: in DCN's 512 -> 256 layer wave w
// finished its MFMAs at 10.2k / 13.5k / 17.6k / 21.5k cycles for w = 0..3 / 4..7 / 8..11 /
// 12..15 (tools/dcn_phases.py), and the last wave of each SIMD, running alone, could not cover
// the L2 latency of its weight ring with its own 8 chunks of MFMAs.
#ifndef RK_MLP_SYNC
#define RK_MLP_SYNC 1
#endif
// RK_MLP_EARLY_RING=1: the next layer's weight ring goes out right after a wave's last MFMA of the
// current layer, ahead of its epilogue (the epilogue parameters after it).  Measured no gain (DIN
// kernel 51.1 -> 51.9-53.0 us, DCN / DeepFM within noise: profiles/r03/NOTES.md), so off.
#ifndef RK_MLP_EARLY_RING
#define RK_MLP_EARLY_RING 0
#endif
// RK_MLP_UNIFORM_PREP=1: one prepare() code path for both layer shapes (LayerPipe::prepare_any).
// Measured DCN 130.2 -> 128.4 M, DIN / DeepFM within noise (profiles/r03/NOTES.md), so off.
// RK_MLP_EP_LANES16=1: epilogue parameters fetched by lanes 0..15 only and broadcast in the
// epilogue (ep_bcast).  Measured DCN 130.4 -> 127.8 M, DIN / DeepFM -1 % (profiles/r03/NOTES.md): off.
#ifndef RK_MLP_EP_LANES16
#define RK_MLP_EP_LANES16 0
#endif
#ifndef RK_MLP_UNIFORM_PREP
#define RK_MLP_UNIFORM_PREP 0
#endif

constexpr int kMlpRows = 16;
constexpr int kMlpWaves = 16;
constexpr int kMlpThreads = 64 * kMlpWaves;
constexpr int kMlpPD = 4;    // prefetch depth (chunks)
constexpr int kMlpSyncChunks = 8;  // RK_MLP_SYNC barrier interval (K-chunks of 16)

// A bare s_barrier: no wait on this wave's memory counters (the weight ring stays in flight).
__device__ __forceinline__ void mlp_sync_barrier() { asm volatile("s_barrier"); }

constexpr int kMlpPad = 64;  // K and N padding of packed weights
// LDS activation row stride = width (a multiple of 64) + kMlpLdPad floats.  The A operand read
// (lane: row lane & 15, float4 4 (lane >> 4) of the chunk) as ds_read_b128 is served in the lane
// groups {0-3,12-15,20-27}, {4-11,16-19,28-31} (+32) (MI355X_MICROARCH.md, LDS): a pad of 4 puts
// lanes 12 and 27 on one 16-B slot (2-way, 8 LDS cycles per read), a pad of 8 is conflict-free (4).
constexpr int kMlpLdPad = 8;
constexpr int kMlpMaxN = 512;

typedef float f32x4_t __attribute__((ext_vector_type(4)));

__host__ __device__ constexpr int pad64(int v) { return (v + kMlpPad - 1) / kMlpPad * kMlpPad; }

// Packed weights are fragment-major (rk_mlp_pack_weight): the float4 a lane of column tile t
// feeds to the 4 MFMAs of K-chunk c (16 k) sits at wfrag(L, t, lane) + kFragStep * c, so a wave's
// chunk load is one contiguous, fully coalesced 1 KiB (8 whole cache lines) rather than sixteen
// half lines of sixteen weight rows.  ldw is pad64(K), the image holds pad64(n) x pad64(K) floats.
constexpr int kFragStep = 256;
__device__ __forceinline__ const float* wfrag(const rk_mlp_layer& L, int tile, int lane) {
  return L.w + (int64_t)tile * (L.ldw / 16) * kFragStep + 4 * lane;
}

__device__ __forceinline__ f32x4_t mfma16(float a, float b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Per-column epilogue parameters of one output column, loaded into registers before the MFMA
// loop: read in the epilogue they would be re-fetched after every LDS store (the compiler cannot
// prove the generic output pointer does not alias them), each fetch waiting on the whole vmcnt
// queue of weight loads.  The loads are unconditional (an absent vector reads the always-valid
// weight image instead) and the raw values are resolved against the layer's flags only in the
// epilogue: loads under `p ? p[n] : default` became scalar branches whose join the compiler
// closed with a full vmcnt(0), draining the next layer's whole weight ring inside prepare().
struct ColEpi {
  float bias, pre_s, pre_b, act_s, act_b, alpha, post_s, post_b;
};

__device__ __forceinline__ ColEpi col_epi(const rk_mlp_layer& L, int n) {
  // L.w holds at least 64 x 64 floats and n < 512: any index read from it is in bounds
  auto ld = [&](const float* p, int i) { return (p ? p : L.w)[i]; };
  ColEpi e;
  e.bias = ld(L.bias, n);
  e.pre_s = ld(L.pre_scale, n);
  e.pre_b = ld(L.pre_scale ? L.pre_shift : nullptr, n);
  e.post_s = ld(L.post_scale, n);
  e.post_b = ld(L.post_scale ? L.post_shift : nullptr, n);
  const bool dice = L.act == RK_ACT_DICE;
  e.act_s = ld(dice ? L.act_scale : nullptr, n);
  e.act_b = ld(dice ? L.act_shift : nullptr, n);
  e.alpha = ld(dice || L.act == RK_ACT_PRELU ? L.act_alpha : nullptr, dice || L.act_alpha_len != 1 ? n : 0);
  return e;
}

// Dice on one element, a*(1-p)*z + p*z with p = sigmoid(z*s + b) (din.py:26-36, BN folded into s, b);
// the contraction is spelled out so every epilogue that uses it rounds the same way.
__device__ __forceinline__ float dice_apply(float z, float s, float b, float a) {
  const float p = sigmoid_fast(__builtin_fmaf(z, s, b));
  return __builtin_fmaf(p, z, (a * (1.0f - p)) * z);
}

// The element-wise epilogue in the reference's order (bias, residual, pre-BN, activation,
// post-BN); `dice` and `has_res` are wave-uniform.  Absent affine parts are the identity (z * 1 + 0
// is exact), and the piecewise-linear activations one negative-side slope `neg` (ReLU 0,
// LeakyReLU slope, PReLU alpha, none 1), so the code is straight-line apart from Dice.  ReLU of a
// negative value gives -0 here (z * 0), equal to torch.relu's +0 in every later use; NaN stays NaN
// as in torch.relu.
__device__ __forceinline__ float col_apply(const rk_mlp_layer& L, const ColEpi& e, bool dice, float z, bool has_res,
                                           float res) {
  z += L.bias ? e.bias : 0.f;
  if (has_res) z = res + z;
  z = z * (L.pre_scale ? e.pre_s : 1.f) + (L.pre_scale ? e.pre_b : 0.f);
  if (dice) {
    z = dice_apply(z, e.act_s, e.act_b, e.alpha);
  } else {
    const float neg = L.act == RK_ACT_RELU ? 0.f : L.act == RK_ACT_LEAKY ? L.slope : L.act == RK_ACT_PRELU ? e.alpha : 1.f;
    z = z > 0.f ? z : z * neg;
  }
  return z * (L.post_scale ? e.post_s : 1.f) + (L.post_scale ? e.post_b : 0.f);
}

// Optional per-workgroup phase marks (timing builds with RK_MLP_PHASES: tools/dcn_phases.py,
// tools/din_phases.py).  Wave 0 keeps clock64() deltas in LDS (no memory traffic while the kernel
// runs: global atomics here used to stall every later vmcnt wait of the wave); the kernel's last
// step copies them to g_mlp_marks[workgroup]:
//   [4l + {0,1,2,3}]  cycles from layer l's start to: MFMA loop issued, epilogue stored, the next
//                     layer's prepare issued, barrier passed
//   [4L]              mlp_rows prologue (input staged, layer 0 weights in flight)
//   [4L + 1]          whole workgroup (kernel entry to end), [4L + 2 / 3] wall clock at entry / end
#ifdef RK_MLP_PHASES
constexpr int kMlpMarks = 4 * RK_MLP_MAX_LAYERS + 4;
constexpr int kMlpMarkWG = 8192;
__device__ unsigned long long g_mlp_marks[kMlpMarkWG][kMlpMarks];
__shared__ unsigned long long s_mlp_marks[kMlpMarks];
// per wave, layers 0..3: cycles from the layer's start to its MFMA loop issued / epilogue stored
__device__ unsigned g_mlp_wave_marks[kMlpMarkWG][4][16][2];
__shared__ unsigned s_mlp_wave_marks[4][16][2];
#define MLP_MARK(i, t0)                                   \
  do {                                                    \
    if (tid == 0) s_mlp_marks[i] = clock64() - (t0);      \
  } while (0)
#define MLP_WALL(i)                                       \
  do {                                                    \
    if (tid == 0) s_mlp_marks[i] = wall_clock64();        \
  } while (0)
__device__ __forceinline__ void mlp_marks_flush(int tid) {
  __syncthreads();
  if (tid < kMlpMarks && blockIdx.x < kMlpMarkWG) g_mlp_marks[blockIdx.x][tid] = s_mlp_marks[tid];
  if (tid < 4 * 16 * 2 && blockIdx.x < kMlpMarkWG)
    (&g_mlp_wave_marks[blockIdx.x][0][0][0])[tid] = (&s_mlp_wave_marks[0][0][0])[tid];
}
#define MLP_FLUSH(tid) mlp_marks_flush(tid)
#else
#define MLP_MARK(i, t0) \
  do {                  \
  } while (0)
#define MLP_WALL(i) \
  do {              \
  } while (0)
#define MLP_FLUSH(tid) \
  do {                 \
  } while (0)
#endif

// Weight ring and per-column epilogue parameters of one layer for a wave owning TPW column tiles
// (t = wave + 16*j).  prepare() issues the first PD weight chunks and the parameter loads; it runs
// before the barrier that closes the previous layer, so that latency overlaps the previous
// layer's tail instead of opening this one.  One register set serves both layer shapes: chunk s of
// tile j sits in ring[s * TPW + j], so a one-tile layer (n <= 256) runs 8 chunks ahead instead of 4
// (at 4 waves per SIMD, 4 chunks of one tile were ~2k cycles of cover against the L2 latency of
// 256 CUs streaming the same weights: tools/mlp_phases.hip layer 1 waited ~9k cycles at its barrier).
constexpr int kMlpRing = 8;  // f32x4 ring slots per lane

struct LayerPipe {
  const float* wrow[2];
  f32x4_t ring[kMlpRing];
  ColEpi ep[2];
  template <int TPW, int PD>
  __device__ __forceinline__ void prepare(const rk_mlp_layer& L, int kchunks, int wave, int lane) {
    prepare_ring<TPW, PD>(L, kchunks, wave, lane);
    prepare_ep<TPW>(L, wave, lane);
  }
  // The two halves of prepare(): the weight ring may go out as soon as the previous layer's last
  // MFMA is issued (its last ring cycle issues no refill, so the registers and wrow are free); the
  // epilogue parameters only after that layer's epilogue has consumed ep.
  template <int TPW, int PD>
  __device__ __forceinline__ void prepare_ring(const rk_mlp_layer& L, int kchunks, int wave, int lane) {
    static_assert(TPW * PD <= kMlpRing, "ring overflow");
#pragma unroll
    for (int j = 0; j < TPW; ++j) wrow[j] = wfrag(L, wave + kMlpWaves * j, lane);
    // issue the ring in consumption order (slot-major): the MFMA loop's vmcnt waits assume that
    // ring register k is the k-th outstanding load; a reordered prepare (the scheduler groups
    // loads by base address) makes every wait of the loop that follows it conservative.  The ring
    // goes first: nothing is outstanding in front of it, so reloading the ring registers costs no
    // wait; the epilogue parameters behind it are consumed only after the whole loop.
#pragma unroll
    for (int s = 0; s < PD; ++s)
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        ring[s * TPW + j] = *reinterpret_cast<const f32x4_t*>(wrow[j] + kFragStep * min(s, kchunks - 1));
        __builtin_amdgcn_sched_barrier(0);
      }
  }
  // Both layer shapes in one code path (`two`: the wave owns two column tiles): slot k holds chunk
  // k >> 1 of tile k & 1 (two tiles) or chunk k (one tile), the order the two mlp_layer variants
  // consume.  With a prepare per variant the ring values met at a join after it, and the compiler
  // copied them into one register set there — copies that wait for each load to land, i.e. a full
  // vmcnt(0) drain of the ring right after issuing it, before the layer barrier.
  __device__ __forceinline__ void prepare_any(const rk_mlp_layer& L, int kchunks, bool two, int wave, int lane) {
    wrow[0] = wfrag(L, wave, lane);
    wrow[1] = wfrag(L, wave + kMlpWaves, lane);  // dereferenced only when two
#pragma unroll
    for (int k = 0; k < kMlpRing; ++k) {
      const float* p = two ? wrow[k & 1] + kFragStep * min(k >> 1, kchunks - 1) : wrow[0] + kFragStep * min(k, kchunks - 1);
      ring[k] = *reinterpret_cast<const f32x4_t*>(p);
      __builtin_amdgcn_sched_barrier(0);
    }
    const int li = lane & 15;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = 16 * (wave + kMlpWaves * j) + li;
      ep[j] = col_epi(L, n < L.n ? n : 0);
    }
  }
  template <int TPW>
  __device__ __forceinline__ void prepare_ep(const rk_mlp_layer& L, int wave, int lane) {
    const int li = lane & 15;
#if RK_MLP_EP_LANES16
    // the 4 lane groups of a column tile need the same 16 columns: only lanes 0..15 fetch them
    // (a quarter of the address/data work in the shared TA path, which every wave's prepare
    // otherwise saturates at the layer boundary), the epilogue broadcasts them (ep_bcast)
    if (lane < 16)
#endif
#pragma unroll
      for (int j = 0; j < TPW; ++j) {
        const int n = 16 * (wave + kMlpWaves * j) + li;
        ep[j] = col_epi(L, n < L.n ? n : 0);
      }
  }
};

// Lanes 0..15's epilogue parameters to every lane of the column tile (ds_bpermute; in the
// epilogue, where waiting for the loads is free).
__device__ __forceinline__ ColEpi ep_bcast(const ColEpi& e, int lane) {
#if RK_MLP_EP_LANES16
  const int src = lane & 15;
  ColEpi o;
  o.bias = __shfl(e.bias, src, 64);
  o.pre_s = __shfl(e.pre_s, src, 64);
  o.pre_b = __shfl(e.pre_b, src, 64);
  o.act_s = __shfl(e.act_s, src, 64);
  o.act_b = __shfl(e.act_b, src, 64);
  o.alpha = __shfl(e.alpha, src, 64);
  o.post_s = __shfl(e.post_s, src, 64);
  o.post_b = __shfl(e.post_b, src, 64);
  return o;
#else
  (void)lane;
  return e;
#endif
}

// One layer (weights already in flight in P) over RT row tiles of 16 rows: each weight float4
// feeds RT x 4 MFMAs.  kchunks = Kp / 16 (a multiple of 4).
// `next` runs right after the last MFMA is issued (mlp_rows: the next layer's weight ring).
template <int TPW, int RT, int PD, bool STORE, class Next>
__device__ __forceinline__ void mlp_layer(LayerPipe& P, const rk_mlp_layer& L, const float* __restrict__ in,
                                          int ldin, float* __restrict__ out, int ldout, int Kp, int wave, int lane,
                                          int64_t m0, int rows, Next next, int dbg_mark = 0,
                                          unsigned long long dbg_t0 = 0) {
  const int li = lane & 15, kq = 4 * (lane >> 4);
  const int kchunks = Kp / 16;
  f32x4_t acc[TPW][RT];
#pragma unroll
  for (int j = 0; j < TPW; ++j)
#pragma unroll
    for (int t = 0; t < RT; ++t) acc[j][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const float* arow = in + li * ldin + kq;
  // A float4s run one chunk ahead of their MFMAs in two explicit register sets (slot s reads set
  // s & 1 and loads chunk c + 1 into the other; PD is even, so the parity of a chunk is the parity
  // of its slot).  With one set the copy av = an was coalesced away and the next chunk's
  // ds_read_b128 had to wait for this chunk's MFMAs to read their operands: every slot then
  // opened with the full LDS latency exposed.
  f32x4_t ab[2][RT];
#pragma unroll
  for (int t = 0; t < RT; ++t) ab[0][t] = *reinterpret_cast<const f32x4_t*>(arow + 16 * t * ldin);
  // One ring cycle (PD chunks starting at c0); REFILL loads chunk c + PD into the slot just used.
  // The last cycle issues no refill: a load past the end would still be in flight at the
  // epilogue, and the next layer's prepare() (which reloads the same ring registers) would have
  // to drain it with a full vmcnt(0) — the 4-7k-cycle "epilogue" of the round-2 phase counters.
  auto cycle = [&](int c0, int nslots, auto refill) {
#pragma unroll
    for (int s = 0; s < PD; ++s) {
      if (s < nslots) {  // nslots == PD except the last cycle of a reduction that is not a multiple of PD
        const int c = c0 + s;
        const int cA = min(c + 1, kchunks - 1);
#pragma unroll
        for (int t = 0; t < RT; ++t)
          ab[(s + 1) & 1][t] = *reinterpret_cast<const f32x4_t*>(arow + 16 * t * ldin + 16 * cA);
        __builtin_amdgcn_sched_barrier(0);  // the read goes out before this slot's MFMAs
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int j = 0; j < TPW; ++j)
#pragma unroll
            for (int t = 0; t < RT; ++t) acc[j][t] = mfma16(ab[s & 1][t][e], P.ring[s * TPW + j][e], acc[j][t]);
        if constexpr (decltype(refill)::value) {
          const int cn = min(c + PD, kchunks - 1);  // clamped only when kchunks % PD != 0
#pragma unroll
          for (int j = 0; j < TPW; ++j)
            P.ring[s * TPW + j] = *reinterpret_cast<const f32x4_t*>(P.wrow[j] + kFragStep * cn);
        }
      }
      // keep the refill here: sinking it to the end of the unrolled body would leave each
      // slot's latency uncovered by the other slots' MFMAs
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  int c0 = 0;
  for (; c0 + PD < kchunks; c0 += PD) {
    cycle(c0, PD, std::true_type{});
#if RK_MLP_SYNC
    if ((c0 + PD) % kMlpSyncChunks == 0) mlp_sync_barrier();
#endif
  }
  if (kchunks - c0 == PD) {
    cycle(c0, PD, std::false_type{});
  } else {
    cycle(c0, kchunks - c0, std::false_type{});
    // the slots this short cycle left unused still hold clamped loads: drain them here, so the
    // state after this layer is the same on both paths (no pending ring load for the next
    // prepare() to wait behind)
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0) only (lgkmcnt / expcnt at their maximum)
  }
  next();

#ifdef RK_MLP_PHASES
  if (wave == 0 && lane == 0) s_mlp_marks[dbg_mark] = clock64() - dbg_t0;
  if (lane == 0 && dbg_mark / 4 < 4) s_mlp_wave_marks[dbg_mark / 4][wave][0] = (unsigned)(clock64() - dbg_t0);
#endif
#if RK_MLP_EPI_PRIO
  // this wave's MFMAs are all issued: its epilogue and the next layer's prepare are on the
  // layer boundary's critical path, so let them win issue arbitration against the waves of the
  // SIMD still in their MFMA loops (reset to 0 after the barrier)
  __builtin_amdgcn_s_setprio(2);
#endif
  float* const store = STORE ? L.store : nullptr;  // eval kernels compile the store path out
  const int64_t ld_store = L.ld_store;
  // The two wave-uniform switches (Dice, residual) are taken once for the whole epilogue: inside
  // the unrolled element loop the compiler kept them as per-element scalar branches around exec-
  // masked blocks (~25 instructions per element); specialised, each element is straight-line VALU
  // and the pad columns a select.
  auto epilogue = [&](auto DICE, auto RES) {
#pragma unroll
    for (int j = 0; j < TPW; ++j) {
      const int n = 16 * (wave + kMlpWaves * j) + li;
      const bool real = n < L.n;
      const ColEpi ep = ep_bcast(P.ep[j], lane);
      // x + f(x): the previous layer's input still sits in `out` (read all, then write: same lane)
      float res[RT][4];
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) res[t][r] = RES ? out[(16 * t + (lane >> 4) * 4 + r) * ldout + n] : 0.f;
#pragma unroll
      for (int t = 0; t < RT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * t + (lane >> 4) * 4 + r;
          const float v = col_apply(L, ep, DICE, acc[j][t][r], RES, res[t][r]);
          const float z = real ? v : 0.f;
          out[row * ldout + n] = z;  // padded columns [n, Np) become the next layer's zero K pad
          if constexpr (STORE)
            if (store && real && row < rows) store[(m0 + row) * ld_store + n] = z;
        }
    }
  };
  const bool dice = L.act == RK_ACT_DICE;
  if (L.residual != 0) {
    if (dice)
      epilogue(std::true_type{}, std::true_type{});
    else
      epilogue(std::false_type{}, std::true_type{});
  } else {
    if (dice)
      epilogue(std::true_type{}, std::false_type{});
    else
      epilogue(std::false_type{}, std::false_type{});
  }
#ifdef RK_MLP_PHASES
  if (lane == 0 && dbg_mark / 4 < 4) s_mlp_wave_marks[dbg_mark / 4][wave][1] = (unsigned)(clock64() - dbg_t0);
#endif
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS ops, not for its global
// loads, so the next layer's weight prefetch stays in flight across it.
__device__ __forceinline__ void mlp_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Runs layers[0..nl) on the 16*RT rows staged (zero-padded to pad64(K0) columns) in buf0, then
// the head (one wave per row) or a plain copy of the last activation to y.  Must be called by
// all kMlpThreads threads of the workgroup.
// The stage fills buf0 in two calls around layer 0's weight prefetch: stage.issue() runs first
// (the gather's own loads go out ahead of the 8 ring loads per wave, which would otherwise queue
// in front of them in the CU's memory pipeline), stage() after it (the rest, then a barrier).
// side(): optional work the streamed tail (mlp_stream.h) runs inside its second layer, after the
// MFMAs of an early chunk are issued — stage work no layer needs before the head (DCN's cross
// network) then fills the wave's idle issue slots beside the matrix pipe instead of the prologue.
struct NoStage {
  __device__ void issue() const {}
  __device__ void operator()() const {}
  __device__ void side() const {}
};
template <class I, class F>
struct TwoPhaseStage {
  I i;
  F f;
  __device__ void issue() { i(); }
  __device__ void operator()() { f(); }
  __device__ void side() {}
};
// early() (streamed tail only, kEarly): the stage's first, independent loads (DCN: the sample's
// indices) go out before the weight ring, whose issue then overlaps their latency; issue() (the
// dependent loads) follows the ring.
template <class E, class I, class F, class S>
struct StagedStage {
  static constexpr bool kEarly = true;
  E e;
  I i;
  F f;
  S s;
  __device__ void early() { e(); }
  __device__ void issue() { i(); }
  __device__ void operator()() { f(); }
  __device__ void side() { s(); }
};
template <class E, class I, class F, class S>
__device__ __forceinline__ StagedStage<E, I, F, S> staged(E e, I i, F f, S s) {
  return StagedStage<E, I, F, S>{e, i, f, s};
}
template <class T, class = void>
struct stage_has_early : std::false_type {};
template <class T>
struct stage_has_early<T, std::void_t<decltype(T::kEarly)>> : std::true_type {};
// The layer a stage's side work runs beside (mlp_stream.h), when the stage names one: SideAt<L, S>
// (DeepFM's FM sums read the staged input row, which stays in LDS only through layer 0).
template <class T, class = void>
struct stage_side_layer {
  static constexpr int value = -1;
};
template <class T>
struct stage_side_layer<T, std::void_t<decltype(T::kSideLayer)>> {
  static constexpr int value = T::kSideLayer;
};
// Layer-0 K-chunks the streamed tail (mlp_stream.h) runs before the barrier that opens layer 0,
// after stage() (PreChunks<KS, S>): the stage guarantees that input columns [0, 16 KS) of every row
// are in LDS by then (DIN: the feature and query columns, before the slowest sample's attention).
template <class T, class = void>
struct stage_pre_chunks {
  static constexpr int value = 0;
};
template <class T>
struct stage_pre_chunks<T, std::void_t<decltype(T::kPreChunks)>> {
  static constexpr int value = T::kPreChunks;
};
template <int KS, class S>
struct PreChunks : S {
  static constexpr int kPreChunks = KS;
};
// Ring loads a kEarly stage lets out ahead of its dependent loads (mlp_stream.h), when the stage
// names a count: RingEarly<N, S> (DeepFM's 30-field row gather: 4; default RK_STREAM_RING_EARLY).
template <class T, class = void>
struct stage_ring_early {
  static constexpr int value = -1;
};
template <class T>
struct stage_ring_early<T, std::void_t<decltype(T::kRingEarly)>> {
  static constexpr int value = T::kRingEarly;
};
template <int N, class S>
struct RingEarly : S {
  static constexpr int kRingEarly = N;
};
template <int N, class S>
__device__ __forceinline__ RingEarly<N, S> ring_early(S s) {
  return RingEarly<N, S>{s};
}
template <int L, class S>
struct SideAt : S {
  static constexpr int kSideLayer = L;
};
template <int L, class S>
__device__ __forceinline__ SideAt<L, S> side_at(S s) {
  return SideAt<L, S>{s};
}
template <class I, class F>
__device__ __forceinline__ TwoPhaseStage<I, F> two_phase(I i, F f) {
  return TwoPhaseStage<I, F>{i, f};
}
template <class F>
__device__ __forceinline__ auto finish_only(F f) {
  return two_phase([] {}, f);
}

// `lds_partial` (optional): per-row head partials the stage left in LDS (DCN's cross half of
// output_layer), used instead of h.head_partial.  `row_ids` (optional, LDS): the batch row of each
// of the `rows` LDS rows for the head outputs, instead of m0 + r (DIN's balanced assignment).
template <int RT = 1, bool STORE = false, class Stage = NoStage>
__device__ __forceinline__ void mlp_rows(const rk_mlp_layer* __restrict__ layers, int nl, int K0, float* buf0,
                                         int ld0, float* buf1, int ld1, int64_t m0, int rows,
                                         const rk_epilogue& h, float* y, int64_t ldy, int tid,
                                         Stage stage = Stage(), const float* lds_partial = nullptr,
                                         const int64_t* row_ids = nullptr) {
  // wave index as an SGPR: the per-wave tile / variant choices become scalar branches
  const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  LayerPipe pipe;
  // Ring discipline shared by every layer variant: 8 loads in flight, ring register k is always the
  // k-th outstanding load (two-tile layers: 4 chunks x 2 tiles, one-tile layers: 8 chunks), so
  // the loop after any prepare() gets the same vmcnt waits.  (A 4-deep one-tile variant used to
  // merge into the 8-deep loop's entry and cut every one of its waits from vmcnt(7) to vmcnt(3).)
  auto prepare = [&](int l) {
    const int nt = pad64(layers[l].n) / 16;  // multiple of 4
    const int kch = pad64(l ? layers[l - 1].n : K0) / 16;
#if RK_MLP_UNIFORM_PREP
    if (wave < nt) pipe.prepare_any(layers[l], kch, wave + kMlpWaves < nt, wave, lane);
#else
    if (wave + kMlpWaves < nt)
      pipe.prepare<2, 4>(layers[l], kch, wave, lane);
    else if (wave < nt)
      pipe.prepare<1, 8>(layers[l], kch, wave, lane);
#endif
  };
#if RK_MLP_EARLY_RING
  auto prepare_ring = [&](int l) {
    const int nt = pad64(layers[l].n) / 16;
    const int kch = pad64(layers[l - 1].n) / 16;
    if (wave + kMlpWaves < nt)
      pipe.prepare_ring<2, 4>(layers[l], kch, wave, lane);
    else if (wave < nt)
      pipe.prepare_ring<1, 8>(layers[l], kch, wave, lane);
  };
  auto prepare_ep = [&](int l) {
    const int nt = pad64(layers[l].n) / 16;
    if (wave + kMlpWaves < nt)
      pipe.prepare_ep<2>(layers[l], wave, lane);
    else if (wave < nt)
      pipe.prepare_ep<1>(layers[l], wave, lane);
  };
#endif
  // The head's operands (head_w for this lane's columns, this wave's row scalars) are loaded while
  // the last layer runs: fetched after the final barrier they put two dependent L2 round trips
  // (~10k cycles at 256 busy CUs, tools/mlp_phases.hip) between the last MFMA and the logits.
  const int Kh = nl ? layers[nl - 1].n : K0;
  const bool hpre = h.head_w != nullptr && Kh <= 128;
  float hw[2] = {0.f, 0.f};
  float hp = 0.f;
  auto head_prefetch = [&]() {
    if (!hpre) return;
#pragma unroll
    for (int c = 0; c < 2; ++c)
      if (lane + 64 * c < Kh) hw[c] = h.head_w[lane + 64 * c];
    if (wave < rows && h.head_partial && !lds_partial) hp = h.head_partial[row_ids ? row_ids[wave] : m0 + wave];
  };
#ifdef RK_MLP_PHASES
  const unsigned long long t_start = clock64();
#endif
  stage.issue();
  __builtin_amdgcn_sched_barrier(0);  // the stage's loads stay ahead of the weight ring
  if (nl > 0) prepare(0);
  if (nl <= 1) head_prefetch();
  MLP_MARK(4 * RK_MLP_MAX_LAYERS - 4, t_start);  // (timing builds: the last layer's slots, unused here)
  stage();
  mlp_lds_barrier();
  MLP_MARK(4 * RK_MLP_MAX_LAYERS, t_start);  // prologue: input staged, layer 0 weights in flight
  int Kp = pad64(K0);
  for (int l = 0; l < nl; ++l) {
    const unsigned long long t0 =
#ifdef RK_MLP_PHASES
        clock64();
#else
        0;
#endif
    const rk_mlp_layer& L = layers[l];
    const int ntiles = pad64(L.n) / 16;
    const float* in = (l & 1) ? buf1 : buf0;
    float* out = (l & 1) ? buf0 : buf1;
    const int ldin = (l & 1) ? ld1 : ld0, ldout = (l & 1) ? ld0 : ld1;
#if RK_MLP_EARLY_RING
    auto next = [&] {
      if (l + 1 < nl) prepare_ring(l + 1);
    };
#else
    auto next = [] {};
#endif
    if (wave + kMlpWaves < ntiles) {
      mlp_layer<2, RT, 4, STORE>(pipe, L, in, ldin, out, ldout, Kp, wave, lane, m0, rows, next, 4 * l, t0);
    } else if (wave < ntiles) {
      mlp_layer<1, RT, 8, STORE>(pipe, L, in, ldin, out, ldout, Kp, wave, lane, m0, rows, next, 4 * l, t0);
    } else {
#if RK_MLP_SYNC
      // no tile in this layer: take part in the active waves' lockstep barriers
      for (int i = 0; i < (Kp / 16 - 1) / kMlpSyncChunks; ++i) mlp_sync_barrier();
#endif
      next();
    }
    MLP_MARK(4 * l + 1, t0);
#if RK_MLP_EARLY_RING
    if (l + 1 < nl) prepare_ep(l + 1);
#else
    if (l + 1 < nl) prepare(l + 1);
#endif
    if (l + 2 == nl) head_prefetch();
    MLP_MARK(4 * l + 2, t0);
    mlp_lds_barrier();
#if RK_MLP_EPI_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
    MLP_MARK(4 * l + 3, t0);
    Kp = pad64(L.n);
  }
  const float* fin = (nl & 1) ? buf1 : buf0;
  const int ldf = (nl & 1) ? ld1 : ld0;
  const int K = nl ? layers[nl - 1].n : K0;
  if (h.head_w) {
    for (int r = wave; r < rows; r += kMlpWaves) {
      const bool pre = hpre && r == wave;  // operands prefetched for the wave's first row
      float p = 0.f;
      if (pre) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
          if (lane + 64 * c < K) p = fmaf(fin[r * ldf + lane + 64 * c], hw[c], p);
      } else {
        for (int n = lane; n < K; n += 64) p = fmaf(fin[r * ldf + n], h.head_w[n], p);
      }
      p = wave_sum(p);
      if (lane == 0) {
        const int64_t m = row_ids ? row_ids[r] : m0 + r;
        float logit = p + h.head_b[0];
        if (lds_partial)
          logit = lds_partial[r] + logit;
        else if (h.head_partial)
          logit = (pre ? hp : h.head_partial[m]) + logit;
        if (h.fm1) {
          if (h.head_aux) h.head_aux[m] = logit;
          logit = h.fm1[m] * h.final_w[0] + h.fm2[m] * h.final_w[1] + logit * h.final_w[2] + h.final_b[0];
        }
        if (h.head_logit) h.head_logit[m] = logit;
        if (h.head_prob) h.head_prob[m] = 1.0f / (1.0f + expf(-logit));
      }
    }
  } else if (y) {
    for (int i = tid; i < rows * K; i += kMlpThreads) {
      const int r = i / K, n = i % K;
      y[(row_ids ? row_ids[r] : m0 + r) * ldy + n] = fin[r * ldf + n];
    }
  }
}

// Host: validates a layer stack for mlp_rows and returns the two LDS buffer widths (floats,
// multiples of 64) needed by an input of width K0.
int mlp_validate(const rk_mlp_layer* layers, int nlayers, int K0, const rk_epilogue& head, int* need0, int* need1,
                 const char* what);

}  // namespace rk
