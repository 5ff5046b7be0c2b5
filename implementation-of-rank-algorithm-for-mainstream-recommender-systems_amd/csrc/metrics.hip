// Evaluation metrics on the device: what the reference's evaluate() computes
// on the host after copying every batch back (dcn.py:214-239; the same in din/bst/deepfm/afm/
// deepcrossing): the mean over batches of BCEWithLogitsLoss, accuracy_score(labels,
// np.round(preds)) and sklearn's roc_auc_score(labels, preds).
//
// rk_eval_batch accumulates one batch into accum (3 x 8 bytes): [0] double, sum over batches of the
// batch's mean loss — loss_kind 0: BCEWithLogitsLoss on the logits (dcn/bst/deepcrossing), 1: BCELoss
// on the probabilities, logs clamped at -100 like torch (din/deepfm/afm/fwfm) — plus *extra when
// given (DIN's per-batch l2_reg, din.py:380); [1] uint64, the number of rint(p) == label (np.round is
// round-half-even, like rintf); [2] uint64, the number of batches.
// rk_auc: exact ROC AUC = Mann-Whitney U / (P N) with ties credited 1/2 — the trapezoidal area
// sklearn's roc_curve + auc give — from integer counts: (score, label) pairs radix-sorted,
// reduced by equal score into (positives, negatives) per distinct score, negatives
// exclusive-scanned, 2U = sum_g pos_g * (2 neg_before_g + neg_g) in int64, one double division.
// NaN scores or a single class give NaN (sklearn raises).  rocPRIM device primitives do the
// sort / reduce-by-key / scan; the pair and reduction kernels are ours.
#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_reduce_by_key.hpp>
#include <rocprim/device/device_scan.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "common.h"

namespace rk {

struct PosNeg {
  long long pos, neg;
  __host__ __device__ PosNeg operator+(const PosNeg& o) const { return {pos + o.pos, neg + o.neg}; }
};

struct LabelToPN {
  __host__ __device__ PosNeg operator()(float y) const { return y > 0.5f ? PosNeg{1, 0} : PosNeg{0, 1}; }
};

struct PlusPN {
  __host__ __device__ PosNeg operator()(const PosNeg& a, const PosNeg& b) const { return a + b; }
};

// neg of group g, or 0 past the number of groups (read from device memory)
struct GroupNeg {
  const PosNeg* agg;
  const unsigned* ngroups;
  __host__ __device__ long long operator()(unsigned g) const { return g < *ngroups ? agg[g].neg : 0ll; }
};

template <int KIND>
__global__ void eval_batch_kernel(const float* __restrict__ logits, const float* __restrict__ probs,
                                  const float* __restrict__ labels, int64_t n, const float* __restrict__ extra,
                                  double* __restrict__ acc) {
  double loss = 0.0;
  unsigned long long correct = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float p = probs[i], y = labels[i];
    if (KIND == 0) {
      // BCEWithLogits: max(x, 0) - x y + log1p(exp(-|x|))
      const float x = logits[i];
      loss += (double)(fmaxf(x, 0.f) - x * y + log1pf(expf(-fabsf(x))));
    } else {
      // BCELoss: -(y max(log p, -100) + (1 - y) max(log(1 - p), -100))
      loss -= (double)(y * fmaxf(logf(p), -100.f) + (1.f - y) * fmaxf(log1pf(-p), -100.f));
    }
    correct += rintf(p) == y;
  }
  for (int o = 32; o > 0; o >>= 1) {
    loss += __shfl_down(loss, o, kWave);
    correct += __shfl_down(correct, o, kWave);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(&acc[0], loss / (double)n);  // this batch's mean, summed over batches
    if (extra && blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&acc[0], (double)*extra);
    atomicAdd(reinterpret_cast<unsigned long long*>(&acc[1]), correct);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(reinterpret_cast<unsigned long long*>(&acc[2]), 1ull);
}

__global__ void auc_final_kernel(const PosNeg* __restrict__ agg, const long long* __restrict__ neg_before,
                                 const unsigned* __restrict__ ngroups, const float* __restrict__ sorted_keys,
                                 int64_t n, double* __restrict__ out) {
  __shared__ long long s2u[4], sp[4], sn[4];
  const unsigned G = *ngroups;
  long long two_u = 0, P = 0, N = 0;
  for (unsigned g = threadIdx.x; g < G; g += blockDim.x) {
    const PosNeg a = agg[g];
    two_u += a.pos * (2 * neg_before[g] + a.neg);
    P += a.pos;
    N += a.neg;
  }
  for (int o = 32; o > 0; o >>= 1) {
    two_u += __shfl_down(two_u, o, kWave);
    P += __shfl_down(P, o, kWave);
    N += __shfl_down(N, o, kWave);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    s2u[w] = two_u;
    sp[w] = P;
    sn[w] = N;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long t = 0, p = 0, q = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) {
      t += s2u[i];
      p += sp[i];
      q += sn[i];
    }
    // radix sort places NaN keys (either sign) at the ends; any NaN -> NaN like sklearn's error
    const bool has_nan = n > 0 && (isnan(sorted_keys[0]) || isnan(sorted_keys[n - 1]));
    *out = (has_nan || p == 0 || q == 0) ? __builtin_nan("") : (double)t / (2.0 * (double)p * (double)q);
  }
}

struct AucPlan {
  size_t sort_bytes, rbk_bytes, scan_bytes, total;
  size_t off_keys, off_vals, off_ukeys, off_agg, off_cnt, off_nb, off_tmp;
};

static AucPlan auc_plan(int64_t n) {
  AucPlan p{};
  const unsigned un = (unsigned)n;
  float* fk = nullptr;
  (void)rocprim::radix_sort_pairs(nullptr, p.sort_bytes, fk, fk, fk, fk, un);
  auto vin = rocprim::make_transform_iterator(fk, LabelToPN());
  (void)rocprim::reduce_by_key(nullptr, p.rbk_bytes, fk, vin, un, fk, (PosNeg*)nullptr, (unsigned*)nullptr, PlusPN());
  auto sin = rocprim::make_transform_iterator(rocprim::counting_iterator<unsigned>(0), GroupNeg{nullptr, nullptr});
  (void)rocprim::exclusive_scan(nullptr, p.scan_bytes, sin, (long long*)nullptr, 0ll, (size_t)un,
                                rocprim::plus<long long>());
  auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
  size_t o = 0;
  p.off_keys = o;
  o += al(n * sizeof(float));
  p.off_vals = o;
  o += al(n * sizeof(float));
  p.off_ukeys = o;
  o += al(n * sizeof(float));
  p.off_agg = o;
  o += al(n * sizeof(PosNeg));
  p.off_cnt = o;
  o += al(sizeof(unsigned));
  p.off_nb = o;
  o += al(n * sizeof(long long));
  p.off_tmp = o;
  o += al(std::max(p.sort_bytes, std::max(p.rbk_bytes, p.scan_bytes)));
  p.total = o;
  return p;
}

}  // namespace rk

using namespace rk;

RK_API int rk_auc_workspace_size(int64_t n, int64_t* bytes) {
  if (n < 0 || n > (int64_t)UINT32_MAX || !bytes) return fail(RK_ERR_INVALID, "rk_auc_workspace_size: bad n");
  *bytes = (int64_t)auc_plan(std::max<int64_t>(n, 1)).total;
  return RK_OK;
}

RK_API int rk_auc(const float* scores, const float* labels, int64_t n, void* workspace, int64_t ws_bytes,
                  double* out, void* stream) {
  if (!scores || !labels || !workspace || !out || n <= 0 || n > (int64_t)UINT32_MAX)
    return fail(RK_ERR_INVALID, "rk_auc: bad arguments (n=%lld)", (long long)n);
  const AucPlan p = auc_plan(n);
  if (ws_bytes < (int64_t)p.total)
    return fail(RK_ERR_INVALID, "rk_auc: workspace %lld < %zu bytes", (long long)ws_bytes, p.total);
  hipStream_t st = (hipStream_t)stream;
  char* ws = static_cast<char*>(workspace);
  float* keys = reinterpret_cast<float*>(ws + p.off_keys);
  float* vals = reinterpret_cast<float*>(ws + p.off_vals);
  float* ukeys = reinterpret_cast<float*>(ws + p.off_ukeys);
  PosNeg* agg = reinterpret_cast<PosNeg*>(ws + p.off_agg);
  unsigned* cnt = reinterpret_cast<unsigned*>(ws + p.off_cnt);
  long long* nb = reinterpret_cast<long long*>(ws + p.off_nb);
  void* tmp = ws + p.off_tmp;
  const unsigned un = (unsigned)n;
  size_t b = p.sort_bytes;
  if (rocprim::radix_sort_pairs(tmp, b, scores, keys, labels, vals, un, 0, 32, st) != hipSuccess)
    return fail(RK_ERR_RUNTIME, "rk_auc: radix sort failed");
  b = p.rbk_bytes;
  if (rocprim::reduce_by_key(tmp, b, keys, rocprim::make_transform_iterator(vals, LabelToPN()), un, ukeys, agg, cnt,
                             PlusPN(), rocprim::equal_to<float>(), st) != hipSuccess)
    return fail(RK_ERR_RUNTIME, "rk_auc: reduce_by_key failed");
  b = p.scan_bytes;
  auto sin = rocprim::make_transform_iterator(rocprim::counting_iterator<unsigned>(0), GroupNeg{agg, cnt});
  if (rocprim::exclusive_scan(tmp, b, sin, nb, 0ll, (size_t)un, rocprim::plus<long long>(), st) != hipSuccess)
    return fail(RK_ERR_RUNTIME, "rk_auc: scan failed");
  auc_final_kernel<<<1, 256, 0, st>>>(agg, nb, cnt, keys, n, out);
  return check_launch("rk_auc");
}

RK_API int rk_eval_batch(const float* logits, const float* probs, const float* labels, int64_t n, int loss_kind,
                         const float* extra, void* accum_, void* stream) {
  double* accum = static_cast<double*>(accum_);
  if (!probs || !labels || !accum || n <= 0 || (loss_kind != 0 && loss_kind != 1) || (loss_kind == 0 && !logits))
    return fail(RK_ERR_INVALID, "rk_eval_batch: bad arguments (n=%lld, loss_kind=%d)", (long long)n, loss_kind);
  const int64_t blocks = std::min<int64_t>((n + 255) / 256, 4 * num_cus());
  if (loss_kind == 0)
    eval_batch_kernel<0><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(logits, probs, labels, n, extra, accum);
  else
    eval_batch_kernel<1><<<(unsigned)blocks, 256, 0, (hipStream_t)stream>>>(logits, probs, labels, n, extra, accum);
  return check_launch("rk_eval_batch");
}
