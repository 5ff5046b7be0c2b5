// Streamed fused-MLP tail for fixed layer plans (round 4): mlp_rows (mlp_core.h) restructured so
// that the weight stream of a wave never stops at a layer boundary.
//
// Same work split as mlp_rows — 16 rows per workgroup of 16 waves, wave w owns the 16-column
// tiles w and w + 16 of every layer, v_mfma_f32_16x16x4_f32 over fragment-major packed weights
// (rk_mlp_pack_weight), activations ping-ponging between two LDS buffers — with three changes:
//  * The layer plan (K0 chunks, column tiles per layer) is a template parameter and the whole
//    layer sequence is unrolled.  Each wave's weight loads of ALL layers form one sequence, and
//    the R-slot register ring runs over it continuously: consuming a slot of layer l's last chunks
//    refills it with layer l+1's first chunks.  mlp_rows stopped refilling in a layer's last ring
//    cycle and issued the next layer's whole ring (128 KiB per CU) after the epilogue, behind the
//    TA: 1.6-4.4k cycles per boundary (profiles/r03/phases_epi_pf1.log) on the critical path.
//    With one definition of every ring register per point of the unrolled sequence, the compiler
//    sees the exact vmcnt of every use (the r03 attempt to spread the ring inside the generic loop
//    spilled because the ring reached the next layer from two definitions).
//  * The per-column epilogue parameters of every layer are resolved once per workgroup into an
//    LDS image ([Np][8] floats per layer) in the prologue, so the vector memory queue holds only
//    weight loads (ring register k is always the k-th outstanding load) and no parameter VGPRs
//    are live across a layer.
//  * Waves that own no tile of a layer (the 128-wide last layer: waves 8..15) are a separate
//    unrolled class; their stream simply ends earlier.
// Accumulation order, epilogue arithmetic (col_apply) and the head are those of mlp_rows, so the
// outputs are bit-identical to it (tests/test_gpu_mlp_stream.py).
//
// RT = 2 (large batches: DeepFM at 65,536 rows): 32 rows per workgroup, every weight float4 feeds
// two MFMAs (one per 16-row tile, as mlp_rows' RT), so a CU streams the weight image once per 32
// rows instead of 16; the accumulation order of a row is unchanged (bit-identical to RT = 1).
// IP0: layer 0 writes its output over its own input in buf0 after a workgroup barrier (32 rows of
// a 960-wide input and of the 512-wide layer 0 output do not fit in LDS side by side); the later
// layers ping-pong buf0 -> buf1 -> buf0.
//
// Eval only (no activation stores), no residual layers: everything else stays on mlp_rows.
#pragma once

#include <type_traits>
#include <utility>

#include "mlp_core.h"

namespace rk {

// weight-ring slots per wave (f32x4 each); 12 measured 1-2 % slower (profiles/r04/ab_r12*.json)
#ifndef RK_STREAM_RING
#define RK_STREAM_RING 8
#endif
// epilogue parameters of the rk_mlp_forward / DCN streamed tails (StreamEpiMode below)
#ifndef RK_STREAM_EPI
#define RK_STREAM_EPI 2
#endif
// experiment: single-tile layers accumulate odd K-steps into a second register set (two
// independent MFMA chains per wave), summed before the epilogue — not bit-identical to mlp_rows.
// A compute-and-stream probe gains 12 % from two chains (tools/stream_probe.hip,
// profiles/r04/stream_probe3.log), but this form makes hipcc spill ~400 VGPRs (DCN 3x slower,
// profiles/r04/ab_split_*.json), and alternating the chains per K-chunk instead is within noise
// (ab_split2_*.json).  Off.
#ifndef RK_STREAM_SPLITACC
#define RK_STREAM_SPLITACC 0
#endif
// Layer hand-off by per-tile ready flags instead of a workgroup barrier: after its epilogue a wave
// sets the bits of its output tiles in an LDS word (rk_stream_ready[l]); a wave of layer l+1 waits
// for bit c only before it reads K-chunk c (= layer l's tile c).  The matrix pipe serves a SIMD's
// waves oldest-first, so waves 0-3 finish a layer first and, with a barrier, idled through the
// younger waves' last MFMAs and epilogues (DCN 512->256 boundary: waves 0-3 done at 4.9k, barrier
// at 7.4k cycles, tools/dcn_phases.py); with the flags they start the next layer's chunks in the
// order the older waves produce them.  The accumulation order is unchanged (bit-identical to
// mlp_rows).  The barrier before the head stays.  Measured no gain (DIN 88.1 / 88.0 M against
// 89.3 / 89.9 M with the barrier, DCN and DeepFM within noise: profiles/r04/ab_flags_*.json): the
// lockstep barriers 8 chunks into the next layer pull the early waves back, so off.
#ifndef RK_STREAM_FLAGS
#define RK_STREAM_FLAGS 0
#endif
// Weight-stream loads with the nontemporal hint (experiment): every weight element is read once
// per CU, so its L1 line is never reused; the memory-pipe counters show the CU's TCP stalled on
// pending requests 32-43 % of the kernel (profiles/r04/ta).
#ifndef RK_STREAM_NT
#define RK_STREAM_NT 0
#endif
// Ring refills in groups: a layer's chunks refill their slots RK_STREAM_REFILL_GROUP loads at a time
// (the loads of max(1, GROUP / T) consecutive chunks back to back after the last of them's MFMAs)
// instead of T loads after every chunk: the same loads, issued in bursts.  The layout probe
// (tools/stream_layout_probe.hip, a 1-KiB load per 4 MFMAs) runs 19.6 / 18.7 / 18.1 / 20.9 µs
// refilling 1 / 2 / 4 / 8 at a time; 1 is the round-4 order.
#ifndef RK_STREAM_REFILL_GROUP
#define RK_STREAM_REFILL_GROUP 4
#endif
// Ring loads issued ahead of a kEarly stage's dependent loads (the rest right after them).  A/B
// over two interleaved runs (profiles/r04/ab_re*.json): DCN 176.0 / 179.8 M with the whole ring
// ahead (8), 181.0 / 183.0 M at 2, 181.4 / 179.5 at 0, 179.0 / 180.6 at 4; DeepFM within noise.
#ifndef RK_STREAM_RING_EARLY
#define RK_STREAM_RING_EARLY 2
#endif
// LDS that the streamed tail adds to its kernel beyond the caller's carve (the ready words); host
// LDS budgets leave room for it
constexpr int kStreamStaticLds = 64;
#if RK_STREAM_FLAGS
static __shared__ unsigned rk_stream_ready[RK_MLP_MAX_LAYERS];
#endif

template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// KC0: 16-deep K chunks of the input (pad64(K0) / 16); NT: 16-column tiles of each layer
// (pad64(n_l) / 16, at most 32).  Layer l > 0 contracts over the previous layer's tiles.
template <int KC0_, int... NT_>
struct StreamPlan {
  static constexpr int NL = sizeof...(NT_);
  static constexpr int KC0 = KC0_;
  static constexpr int nt(int l) {
    constexpr int v[] = {NT_...};
    return v[l];
  }
  static constexpr int kc(int l) { return l == 0 ? KC0 : nt(l - 1); }
  // column tiles of layer l owned by wave w (tiles w, w + 16)
  static constexpr int tpw(int l, int w) { return w < nt(l) ? (nt(l) - 1 - w) / 16 + 1 : 0; }
  // first load of layer l in wave w's stream, and the stream's length
  static constexpr int base(int l, int w) {
    int b = 0;
    for (int i = 0; i < l; ++i) b += tpw(i, w) * kc(i);
    return b;
  }
  static constexpr int layer_of(int g, int w) {
    int l = 0;
    while (l + 1 < NL && base(l + 1, w) <= g) ++l;
    return l;
  }
  static constexpr bool same_class(int a, int b) {
    for (int l = 0; l < NL; ++l)
      if (tpw(l, a) != tpw(l, b)) return false;
    return true;
  }
  // the lowest wave with the same tile counts in every layer (waves are dispatched by class)
  static constexpr int rep(int w) {
    int r = 0;
    while (!same_class(r, w)) ++r;
    return r;
  }
  // LDS epilogue-parameter image: [Np_l][8] floats per layer
  static constexpr int epi_off(int l) {
    int o = 0;
    for (int i = 0; i < l; ++i) o += 16 * nt(i) * 8;
    return o;
  }
  static constexpr int epi_floats() { return epi_off(NL); }
  static constexpr int epi_cols() { return epi_off(NL) / 8; }
  static_assert(NL >= 1 && NL <= RK_MLP_MAX_LAYERS, "layer count");
  static_assert(epi_off(NL) / 8 <= 2 * kMlpThreads, "epilogue image: two columns per thread at most");
};

// col_epi's raw values resolved against the layer's flags: absent affine parts become the identity
// (col_apply adds 0 / scales by 1 for them too, so the arithmetic is the same), and the non-Dice
// activations one negative-side slope in the alpha slot.
__device__ __forceinline__ ColEpi resolve_epi(const rk_mlp_layer& L, ColEpi r) {
  r.bias = L.bias ? r.bias : 0.f;
  r.pre_s = L.pre_scale ? r.pre_s : 1.f;
  r.pre_b = L.pre_scale ? r.pre_b : 0.f;
  r.post_s = L.post_scale ? r.post_s : 1.f;
  r.post_b = L.post_scale ? r.post_b : 0.f;
  if (L.act != RK_ACT_DICE)
    r.alpha = L.act == RK_ACT_RELU ? 0.f : L.act == RK_ACT_LEAKY ? L.slope : L.act == RK_ACT_PRELU ? r.alpha : 1.f;
  return r;
}

// col_apply on resolved parameters (bias, pre affine, activation, post affine).
template <bool DICE>
__device__ __forceinline__ float apply_epi(const ColEpi& e, float z) {
  z = z + e.bias;
  z = z * e.pre_s + e.pre_b;
  if constexpr (DICE)
    z = dice_apply(z, e.act_s, e.act_b, e.alpha);
  else
    z = z > 0.f ? z : z * e.alpha;
  return z * e.post_s + e.post_b;
}

// Where a streamed tail finds its per-column epilogue parameters.
enum StreamEpiMode {
  kEpiLdsHere = 0,    // LDS image, loaded and stored by mlp_stream_rows in its prologue
  kEpiLdsCaller = 1,  // LDS image stored by the caller before the barrier that opens layer 0 (DIN)
  kEpiRegs = 2,       // registers: layer 0's after the ring in the prologue, layer l+1's after layer l's epilogue
};

// The epilogue-parameter image, in two halves: load() issues the (unconditional) loads of at most
// two columns per thread into registers, store() writes them to LDS.  Column i of the image is
// layer l's column i - cols(<l); values are col_epi's (absent vectors read as any valid float and
// are resolved by col_apply against the layer's flags, exactly as mlp_rows does).
template <class P>
struct StreamEpi {
  ColEpi e[2];
  static constexpr int kCols = (P::epi_cols() + kMlpThreads - 1) / kMlpThreads;  // per thread, 1 or 2
  __device__ __forceinline__ void load(const rk_mlp_layer* __restrict__ layers, int tid) {
#pragma unroll
    for (int k = 0; k < kCols; ++k) {
      const int i = tid + kMlpThreads * k;
      // the thread's layer by selects over the (scalar) layer table: loads under a per-layer
      // branch would close their joins with vmcnt(0)
      int l = 0;
#pragma unroll
      for (int q = 1; q < P::NL; ++q) l = i >= P::epi_off(q) / 8 ? q : l;
      rk_mlp_layer L = layers[0];
#pragma unroll
      for (int q = 1; q < P::NL; ++q)
        if (l == q) L = layers[q];
      const int n = i - P::epi_off(l) / 8;
      e[k] = resolve_epi(L, col_epi(L, n < L.n ? n : 0));
    }
  }
  __device__ __forceinline__ void store(float* __restrict__ img, int tid) const {
#pragma unroll
    for (int k = 0; k < kCols; ++k) {
      const int i = tid + kMlpThreads * k;
      if (i < P::epi_cols()) {
        f32x4_t* d = reinterpret_cast<f32x4_t*>(img + 8 * i);
        d[0] = (f32x4_t){e[k].bias, e[k].pre_s, e[k].pre_b, e[k].act_s};
        d[1] = (f32x4_t){e[k].act_b, e[k].alpha, e[k].post_s, e[k].post_b};
      }
    }
  }
};

// Chunk of the side layer at which wave position k (0..3 on its SIMD) runs stage.side(), and the
// positions that run it at chunk c.
constexpr int side_chunk(int KC, int k) {
  const int step = KC / 4 > 0 ? KC / 4 : 1;
  const int c = (KC > 2 ? 2 : KC - 1) + step * k;
  return c < KC - 1 ? c : KC - 1;
}
constexpr int side_first_pos(int KC, int c) {
  for (int k = 0; k < 4; ++k)
    if (side_chunk(KC, k) == c) return k;
  return 4;
}
constexpr int side_last_pos(int KC, int c) {
  for (int k = 3; k >= 0; --k)
    if (side_chunk(KC, k) == c) return k;
  return -1;
}

// One wave class W (P::rep(W) == W) of the streamed tail.  `epi` is the LDS parameter image
// (stored before the barrier that opens layer 0); `stage` as in mlp_rows (issue() before the ring,
// operator() after it, before that barrier).  EPI: StreamEpiMode.
template <class P, int W, int EPI, int RT, bool IP0, class Stage>
__device__ __forceinline__ void mlp_stream_class(const rk_mlp_layer* __restrict__ layers, float* buf0, int ld0,
                                                 float* buf1, int ld1, float* epi, int64_t m0, int rows,
                                                 const rk_epilogue& h, int tid, int wave, Stage& stage,
                                                 const float* lds_partial, const int64_t* row_ids,
                                                 const float* lds_fm) {
  constexpr int R = RK_STREAM_RING;
  constexpr int NL = P::NL;
  constexpr int TOT = P::base(NL, W);
  const int lane = tid & 63, li = lane & 15, kq = 4 * (lane >> 4);
  f32x4_t ring[R];

  // load g of the stream: layer l, chunk c of tile j (consumption order: chunk-major)
  auto issue = [&](auto G) {
    constexpr int g = G;
    if constexpr (g < TOT) {
      constexpr int l = P::layer_of(g, W);
      constexpr int T = P::tpw(l, W);
      constexpr int i = g - P::base(l, W), c = i / T, j = i % T;
      const rk_mlp_layer& L = layers[l];
      const float* p = L.w + ((int64_t)(wave + kMlpWaves * j) * (L.ldw / 16) + c) * kFragStep;
#if RK_STREAM_NT
      ring[g % R] = __builtin_nontemporal_load(reinterpret_cast<const f32x4_t*>(p + 4 * lane));
#else
      ring[g % R] = *reinterpret_cast<const f32x4_t*>(p + 4 * lane);
#endif
    }
  };

  const int Kh = layers[NL - 1].n;
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
  StreamEpi<P> ep_stage;
  constexpr bool kEarly = stage_has_early<Stage>::value;
  // the layer whose MFMAs the stage's side work runs beside: the stage's choice, else the second
  constexpr int kSideL = stage_side_layer<Stage>::value >= 0 ? stage_side_layer<Stage>::value : (NL > 1 ? 1 : 0);
  // kEpiRegs: the parameters of the wave's columns of one layer (tiles j = 0, 1)
  ColEpi epr[2];
  auto load_epr = [&](auto LI) {
    constexpr int l = LI;
    if constexpr (l < NL) {
      const rk_mlp_layer& L = layers[l];
#pragma unroll
      for (int j = 0; j < P::tpw(l, W); ++j) {
        const int n = 16 * (wave + kMlpWaves * j) + li;
        epr[j] = col_epi(L, n < L.n ? n : 0);
      }
    }
  };
  if constexpr (kEarly) {
    stage.early();
    __builtin_amdgcn_sched_barrier(0);
  } else {
    stage.issue();
    if constexpr (EPI == kEpiLdsHere) ep_stage.load(layers, tid);
    __builtin_amdgcn_sched_barrier(0);  // the stage's and the parameters' loads stay ahead of the ring
  }
  // kEarly stages: only the first R0 ring loads go out before the stage's dependent loads (DCN /
  // DeepFM: the row gather), so those queue behind R0 KiB per wave in the CU's memory pipe instead
  // of the whole ring (16 waves x 8 KiB); the rest of the ring follows them
  constexpr int kRE = stage_ring_early<Stage>::value >= 0 ? stage_ring_early<Stage>::value : RK_STREAM_RING_EARLY;
  constexpr int R0 = kEarly ? (kRE < R ? kRE : R) : R;
  static_for<0, R0>([&](auto G) {
    issue(G);
    __builtin_amdgcn_sched_barrier(0);
  });
  if constexpr (kEarly) {
    stage.issue();
    if constexpr (EPI == kEpiLdsHere) ep_stage.load(layers, tid);
    __builtin_amdgcn_sched_barrier(0);
    static_for<R0, R>([&](auto G) {
      issue(G);
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  // layer 0's parameters behind the ring (needed only at its epilogue)
  if constexpr (EPI == kEpiRegs) load_epr(std::integral_constant<int, 0>{});
  if constexpr (NL == 1) head_prefetch();
  MLP_MARK(4 * RK_MLP_MAX_LAYERS - 4, t_start);  // (timing builds) ring issued
  stage();
  // layer 0's first KS K-chunks before the barrier (PreChunks: their input columns are staged
  // already), accumulated in order into the accumulators layer 0 continues from — bit-identical
  constexpr int KS = stage_pre_chunks<Stage>::value;
  constexpr int T0 = P::tpw(0, W);
  static_assert(KS == 0 || (KS < kMlpSyncChunks && KS < P::kc(0) && kSideL != 0 && !(RK_STREAM_SPLITACC && T0 == 1) &&
                            RT == 1 && !IP0),
                "pre-barrier chunks: no lockstep barrier or side work among them");
  static_assert(RT == 1 || RT == 2, "one or two 16-row tiles");
  f32x4_t acc0[T0 > 0 ? T0 : 1];
  if constexpr (KS > 0 && T0 > 0) {
#pragma unroll
    for (int j = 0; j < T0; ++j) acc0[j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const float* arow = buf0 + li * ld0 + kq;
    f32x4_t ab[2];
    ab[0] = *reinterpret_cast<const f32x4_t*>(arow);
    static_for<0, KS>([&](auto CI) {
      constexpr int c = CI;
      if constexpr (c + 1 < KS) ab[(c + 1) & 1] = *reinterpret_cast<const f32x4_t*>(arow + 16 * (c + 1));
      __builtin_amdgcn_sched_barrier(0);
      static_for<0, 4>([&](auto EI) {
        constexpr int e = EI;
        static_for<0, T0>([&](auto JI) {
          constexpr int j = JI;
          acc0[j] = mfma16(ab[c & 1][e], ring[(c * T0 + j) % R][e], acc0[j]);
        });
      });
      static_for<0, T0>([&](auto JI) {
        constexpr int j = JI;
        issue(std::integral_constant<int, c * T0 + j + R>{});
      });
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  if constexpr (EPI == kEpiLdsHere) ep_stage.store(epi, tid);
#if RK_STREAM_FLAGS
  if (tid < NL) rk_stream_ready[tid] = 0u;  // read only after the barrier below
#endif
  mlp_lds_barrier();
  MLP_MARK(4 * RK_MLP_MAX_LAYERS, t_start);  // prologue done

  static_for<0, NL>([&](auto LI) {
    constexpr int l = LI;
    constexpr int T = P::tpw(l, W), KC = P::kc(l), B0 = P::base(l, W);
#ifdef RK_MLP_PHASES
    const unsigned long long t0 = clock64();
#endif
    const rk_mlp_layer& L = layers[l];
    // lockstep barriers, except in a layer the stage chose for side work that leaves waves without
    // a tile: those waves do the side work instead, and a barrier would make the others wait for it
    constexpr bool kSync = !(stage_side_layer<Stage>::value == l && P::nt(l) < kMlpWaves);
    // IP0: layer 0 in place in buf0, then the ping-pong one step behind
    constexpr bool kIn1 = IP0 ? (l > 0 && !(l & 1)) : (l & 1);
    constexpr bool kOut1 = IP0 ? (l & 1) : !(l & 1);
    const float* in = kIn1 ? buf1 : buf0;
    float* out = kOut1 ? buf1 : buf0;
    const int ldin = kIn1 ? ld1 : ld0, ldout = kOut1 ? ld1 : ld0;
    if constexpr (T == 0) {
      if constexpr (l == kSideL) stage.side();  // (no tile here: the side work all the same)
#if RK_MLP_SYNC
      // no tile in this layer: take part in the active waves' lockstep barriers
      if constexpr (kSync)
        static_for<0, (KC - 1) / kMlpSyncChunks>([&](auto) { mlp_sync_barrier(); });
#endif
      if constexpr (IP0 && l == 0) mlp_lds_barrier();
    } else {
      constexpr int CB = l == 0 ? KS : 0;  // first chunk of this section (layer 0: after the pre-chunks)
      f32x4_t acc[T][RT];
#pragma unroll
      for (int j = 0; j < T; ++j) {
#pragma unroll
        for (int t = 0; t < RT; ++t) {
          if constexpr (CB > 0)
            acc[j][t] = acc0[j];
          else
            acc[j][t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        }
      }
      constexpr bool kSplit = RK_STREAM_SPLITACC && T == 1 && RT == 1;
      f32x4_t acc_odd = {0.f, 0.f, 0.f, 0.f};
      const float* arow = in + li * ldin + kq;
      // layer l > 0, flag hand-off: K-chunk c is layer l-1's output tile c; `ready` caches the bits
      // seen set (wave-uniform), the LDS word is re-read only for a chunk not seen yet
      unsigned ready = 0u;
      auto wait_chunk = [&](int c) {
#if RK_STREAM_FLAGS
        if constexpr (l > 0) {
          if (!((ready >> c) & 1u)) {
            do {
              ready = __builtin_amdgcn_readfirstlane(
                  __hip_atomic_load(&rk_stream_ready[l - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            } while (!((ready >> c) & 1u));
            asm volatile("" ::: "memory");  // the chunk's activation reads stay behind the flag
          }
        }
#endif
      };
      // A float4s one chunk ahead in two register sets (see mlp_layer)
      f32x4_t ab[2][RT];
      wait_chunk(CB);
#pragma unroll
      for (int t = 0; t < RT; ++t) ab[CB & 1][t] = *reinterpret_cast<const f32x4_t*>(arow + 16 * t * ldin + 16 * CB);
      static_for<CB, KC>([&](auto CI) {
        constexpr int c = CI;
        if constexpr (c + 1 < KC) {
          wait_chunk(c + 1);
#pragma unroll
          for (int t = 0; t < RT; ++t)
            ab[(c + 1) & 1][t] = *reinterpret_cast<const f32x4_t*>(arow + 16 * t * ldin + 16 * (c + 1));
        }
        __builtin_amdgcn_sched_barrier(0);  // the read goes out before this chunk's MFMAs
        static_for<0, 4>([&](auto EI) {
          constexpr int e = EI;
          static_for<0, T>([&](auto JI) {
            constexpr int j = JI;
            static_for<0, RT>([&](auto TI) {
              constexpr int t = TI;
              if constexpr (kSplit && (e & 1))
                acc_odd = mfma16(ab[c & 1][t][e], ring[(B0 + c * T + j) % R][e], acc_odd);
              else
                acc[j][t] = mfma16(ab[c & 1][t][e], ring[(B0 + c * T + j) % R][e], acc[j][t]);
            });
          });
        });
        // refill the slots just read with the stream's next loads (past this layer: the next
        // layer's first chunks), CG chunks' loads at a time
        {
          constexpr int CG = RK_STREAM_REFILL_GROUP / T > 1 ? RK_STREAM_REFILL_GROUP / T : 1;
          if constexpr ((c - CB + 1) % CG == 0 || c + 1 == KC) {
            constexpr int c0 = c - (c - CB) % CG;
            static_for<c0 * T, (c + 1) * T>([&](auto GI) {
              constexpr int g = GI;
              issue(std::integral_constant<int, B0 + g + R>{});
            });
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        // the stage's side work, once, beside the MFMAs of layer kSideL (default: the second),
        // staggered over the SIMD's four waves (wave w sits at position w / 4 of SIMD w % 4): wave
        // position k at chunk side_chunk(k), one per lockstep window when the layer has 32 chunks, so
        // three of a SIMD's waves keep the matrix pipe fed while the fourth waits on the side work's
        // cross-lane reductions (all four at one chunk left the pipe idle for that latency)
        if constexpr (l == kSideL) {
          constexpr int kFirst = side_first_pos(KC, c), kLast = side_last_pos(KC, c);
          if constexpr (kFirst <= kLast) {
            const int pos = wave >> 2;
            if (pos >= kFirst && pos <= kLast) stage.side();
            __builtin_amdgcn_sched_barrier(0);
          }
        }
#if RK_MLP_SYNC
        if constexpr (kSync && (c + 1) % kMlpSyncChunks == 0 && c + 1 < KC) mlp_sync_barrier();
#endif
      });
      if constexpr (kSplit) acc[0][0] += acc_odd;
      if constexpr (IP0 && l == 0) mlp_lds_barrier();  // every wave's layer-0 reads of buf0 are done
      MLP_MARK(4 * l, t0);
#ifdef RK_MLP_PHASES
      if (lane == 0 && l < 4) s_mlp_wave_marks[l][wave][0] = (unsigned)(clock64() - t0);
#endif
#if RK_MLP_EPI_PRIO
      __builtin_amdgcn_s_setprio(2);
#endif
      const float* img = epi + P::epi_off(l);
      auto epilogue = [&](auto DICE) {
#pragma unroll
        for (int j = 0; j < T; ++j) {
          const int n = 16 * (wave + kMlpWaves * j) + li;
          const bool real = n < L.n;
          ColEpi e;
          if constexpr (EPI == kEpiRegs) {
            e = resolve_epi(L, epr[j]);
          } else {
            const f32x4_t p0 = *reinterpret_cast<const f32x4_t*>(img + 8 * n);
            const f32x4_t p1 = *reinterpret_cast<const f32x4_t*>(img + 8 * n + 4);
            e.bias = p0[0];
            e.pre_s = p0[1];
            e.pre_b = p0[2];
            e.act_s = p0[3];
            e.act_b = p1[0];
            e.alpha = p1[1];
            e.post_s = p1[2];
            e.post_b = p1[3];
          }
#pragma unroll
          for (int t = 0; t < RT; ++t) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int row = 16 * t + (lane >> 4) * 4 + r;
              const float z = apply_epi<decltype(DICE)::value>(e, acc[j][t][r]);
              out[row * ldout + n] = real ? z : 0.f;  // padded columns: the next layer's zero K pad
            }
          }
        }
      };
      if (L.act == RK_ACT_DICE)
        epilogue(std::true_type{});
      else
        epilogue(std::false_type{});
#if RK_STREAM_FLAGS
      if constexpr (l + 1 < NL) {
        // this wave's output tiles are in LDS (its own LDS ops complete in order): publish them
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        unsigned bits = 0u;
#pragma unroll
        for (int j = 0; j < T; ++j) bits |= 1u << (wave + kMlpWaves * j);
        if (lane == 0) __hip_atomic_fetch_or(&rk_stream_ready[l], bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
#endif
#ifdef RK_MLP_PHASES
      if (lane == 0 && l < 4) s_mlp_wave_marks[l][wave][1] = (unsigned)(clock64() - t0);
#endif
    }
    MLP_MARK(4 * l + 1, t0);
    // the next layer's parameters (this layer's are consumed): in flight across the barrier, behind
    // that layer's first ring loads
    if constexpr (EPI == kEpiRegs) load_epr(std::integral_constant<int, l + 1>{});
    if constexpr (l + 2 == NL) head_prefetch();
    MLP_MARK(4 * l + 2, t0);
    if constexpr (!RK_STREAM_FLAGS || l + 1 == NL) mlp_lds_barrier();  // (flags: only before the head)
    MLP_MARK(4 * l + 3, t0);
#if RK_MLP_EPI_PRIO
    if constexpr (T > 0) __builtin_amdgcn_s_setprio(0);
#endif
  });

  // head: one wave per row, as mlp_rows
  constexpr bool kFin1 = IP0 ? ((NL - 1) & 1) : (NL & 1);
  const float* fin = kFin1 ? buf1 : buf0;
  const int ldf = kFin1 ? ld1 : ld0;
  const int K = Kh;
  if (h.head_w) {
    for (int r = wave; r < rows; r += kMlpWaves) {
      const bool pre = hpre && r == wave;
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
          const float f1 = lds_fm ? lds_fm[r] : h.fm1[m], f2 = lds_fm ? lds_fm[kMlpRows * RT + r] : h.fm2[m];
          logit = f1 * h.final_w[0] + f2 * h.final_w[1] + logit * h.final_w[2] + h.final_b[0];
        }
        if (h.head_logit) h.head_logit[m] = logit;
        if (h.head_prob) h.head_prob[m] = 1.0f / (1.0f + expf(-logit));
      }
    }
  }
}

// Entry point: dispatches the calling wave to its class's unrolled body.  Must be called by all
// kMlpThreads threads.  `epi`: P::epi_floats() floats of LDS (16-B aligned).  RT row tiles of 16
// (rows <= 16 RT; lds_fm: [fm1 x 16 RT][fm2 x 16 RT]); IP0: layer 0 in place (see the top).
template <class P, int EPI = kEpiRegs, int RT = 1, bool IP0 = false, class Stage = NoStage>
__device__ __forceinline__ void mlp_stream_rows(const rk_mlp_layer* __restrict__ layers, float* buf0, int ld0,
                                                float* buf1, int ld1, float* epi, int64_t m0, int rows,
                                                const rk_epilogue& h, int tid, Stage stage = Stage(),
                                                const float* lds_partial = nullptr,
                                                const int64_t* row_ids = nullptr, const float* lds_fm = nullptr) {
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  static_for<0, kMlpWaves>([&](auto WI) {
    constexpr int w = WI;
    if constexpr (P::rep(w) == w) {
      bool mine = true;  // is the calling wave in class w?
#pragma unroll
      for (int l = 0; l < P::NL; ++l) mine = mine && P::tpw(l, wave) == P::tpw(l, w);
      if (mine)
        mlp_stream_class<P, w, EPI, RT, IP0>(layers, buf0, ld0, buf1, ld1, epi, m0, rows, h, tid, wave, stage,
                                         lds_partial, row_ids, lds_fm);
    }
  });
}

// Plans compiled into the library (hidden units [512, 256, 128], the reference's default for
// DCN / DIN / BST / DeepFM): by the input's K chunks.  DeepFM's tail after its tiled first layer
// is [256, 128] over K0 = 512.
using StreamPlanK64 = StreamPlan<4, 32, 16, 8>;    // DCN (width 50)
using StreamPlanK80 = StreamPlan<5, 32, 16, 8>;    // BST d 16 DNN (16 + 34 + 16 = 66; K chunks past 80 all zero)
using StreamPlanK128 = StreamPlan<8, 32, 16, 8>;   // DIN (16 + 34 + 2H <= 128)
using StreamPlanK192 = StreamPlan<12, 32, 16, 8>;  // BST DNN (16 + 34 + d = 178 at d 128)
using StreamPlanK256 = StreamPlan<16, 32, 16, 8>;
using StreamPlanTail512 = StreamPlan<32, 16, 8>;   // DeepFM: 512 -> 256 -> 128
using StreamPlanK960 = StreamPlan<60, 32, 16, 8>;  // DeepFM whole (30 fields x 32: deepfm_fused.hip)

// Host: the compiled plan matching a layer stack (0: none — use mlp_rows).  Eval only: no
// activation stores, no residual layers.  RANKOPS_MLP_STREAM=0 disables the streamed path.
enum StreamPlanId { kStreamNone = 0, kStreamK64, kStreamK128, kStreamK192, kStreamK256, kStreamTail512 };
int stream_plan_for(const rk_mlp_layer* layers, int nlayers, int K0);
int stream_plan_epi_floats(int id);

}  // namespace rk
