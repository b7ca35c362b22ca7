// Fused KGE training step for gfx950 -- element-wise model family.
//
// One reference batch step (KGEModel.__run_single_batch, BaseModel.py:293-330)
// runs as stream-ordered kernels:
//
//   K0  constrain   full-table row renormalisation of ent_emb when the model's
//                   _constraint_loss assigns it (TransE.py:171-172,
//                   DistMult.py:162-163).
//   KS  score       8-wave workgroups, `wpp` waves per positive. In-register
//                   Philox negative draws (ns_strategy.py:39-64 in the layout
//                   of BaseModel.py:332-408); each wave streams its slots'
//                   rows in register batches (gather -> forward -> ONE
//                   transposed multi-reduction per batch -> loss weight ->
//                   backward), with SANS's softmax folded in online (loss.py
//                   :174-182), so every sampled row is read exactly once. The
//                   positive's own rows are reduced on chip; every negative
//                   leaves one (alpha, value) coefficient and its destination
//                   key, filed straight into that destination's list (one
//                   int atomic per key). The last workgroup reduces the
//                   loss and the per-variable gradient norms (clip_by_norm,
//                   BaseModel.py:327) in a fixed order.
//   KU  update      destination-major, one wave per entity / relation row:
//                   its keys in ascending code order (bit-reproducible sums,
//                   no float atomics), each negative's row gradient re-derived
//                   from ONE frozen context row + its coefficient, the
//                   positives' own row gradients added, clip scale and SGD
//                   (BaseModel.py:328, keras SGD ResourceScatterAdd) applied
//                   with ONE read-modify-write per touched row.
#include <algorithm>

#include "kge_proj.h"

namespace kge {

// ------------------------------------------------------------ K0 constrain
// kind 0: normalized_embeddings(p=2) -> X / pow(sum X^2, 1/2) * value
// kind 1: clip_constraint(p=2)       -> rows with norm >= value rescaled
// Each wave owns 4 rows and issues all their loads before reducing.
__global__ __launch_bounds__(256) void constrain_rows_kernel(float* __restrict__ t, int64_t rows,
                                                              int32_t cols, int64_t ld, int kind,
                                                              float value, StepCtl* ctl, uint32_t sig,
                                                              int32_t* status) {
  if (ctl && ws_refused(ctl, sig, status, nullptr)) return;   // launched by a step: guarded
  constexpr int RPW = 4;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / KGE_WAVE);
  const bool v4 = (cols % 4 == 0) && (ld % 4 == 0) && (((uintptr_t)t & 15) == 0) && cols <= 4 * KGE_WAVE;
  for (int64_t r0 = ((int64_t)blockIdx.x * (blockDim.x / KGE_WAVE) + wave_id()) * RPW; r0 < rows;
       r0 += nw * RPW) {
    if (v4) {
      float4 x[RPW];
      float s[RPW];
      const int e0 = lane_id() * 4;
#pragma unroll
      for (int u = 0; u < RPW; ++u) {
        x[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (r0 + u < rows && e0 < cols) x[u] = *reinterpret_cast<const float4*>(t + (r0 + u) * ld + e0);
      }
#pragma unroll
      for (int u = 0; u < RPW; ++u) s[u] = x[u].x * x[u].x + x[u].y * x[u].y + x[u].z * x[u].z + x[u].w * x[u].w;
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
#pragma unroll
        for (int u = 0; u < RPW; ++u) s[u] += __shfl_xor(s[u], o, KGE_WAVE);
      }
#pragma unroll
      for (int u = 0; u < RPW; ++u) {
        if (r0 + u >= rows || e0 >= cols) continue;
        const float n = sqrtf(s[u]);
        float4 y = x[u];
        if (kind == 0) {
          y.x = y.x / n * value; y.y = y.y / n * value; y.z = y.z / n * value; y.w = y.w / n * value;
        } else if (!(n < value)) {
          const float d = fmaxf(n, 1e-9f);
          y.x = y.x / d * value; y.y = y.y / d * value; y.z = y.z / d * value; y.w = y.w / d * value;
        } else {
          continue;
        }
        *reinterpret_cast<float4*>(t + (r0 + u) * ld + e0) = y;
      }
    } else {
      for (int u = 0; u < RPW && r0 + u < rows; ++u) {
        float* row = t + (r0 + u) * ld;
        float s = 0.f;
        for (int e = lane_id(); e < cols; e += KGE_WAVE) s += row[e] * row[e];
        s = wave_sum(s);
        const float n = sqrtf(s);
        if (kind == 0) {
          for (int e = lane_id(); e < cols; e += KGE_WAVE) row[e] = row[e] / n * value;
        } else if (!(n < value)) {
          const float d = fmaxf(n, 1e-9f);
          for (int e = lane_id(); e < cols; e += KGE_WAVE) row[e] = row[e] / d * value;
        }
      }
    }
  }
}

// ------------------------------------------------------------ apply
// var += -lr * clip(g) (keras SGD) or keras Adam over every element
// (kge_hip.h kge_apply_desc). A contiguous table (ld == cols) is one flat
// float4 stream (no per-element row division); a strided one goes a wave per
// row, float4 lanes when the row allows.
__device__ __forceinline__ void apply_one(const ApplyArgs& a, float cs, float& w, float g, float& m, float& v) {
  const float gv = g * cs;
  if (!a.adam) {
    w = w + gv * (-a.lr);
  } else {
    m = a.b1 * m + (1.f - a.b1) * gv;
    v = a.b2 * v + (1.f - a.b2) * (gv * gv);
    w = w - a.lr_t * m / (sqrtf(v) + a.eps);
  }
}
__device__ __forceinline__ void apply4(const ApplyArgs& a, float cs, float* w, const float* g, float* m, float* v) {
  float4 W = *reinterpret_cast<const float4*>(w);
  const float4 G = *reinterpret_cast<const float4*>(g);
  float4 Mv = make_float4(0.f, 0.f, 0.f, 0.f), Vv = Mv;
  if (a.adam) {
    Mv = *reinterpret_cast<const float4*>(m);
    Vv = *reinterpret_cast<const float4*>(v);
  }
  apply_one(a, cs, W.x, G.x, Mv.x, Vv.x);
  apply_one(a, cs, W.y, G.y, Mv.y, Vv.y);
  apply_one(a, cs, W.z, G.z, Mv.z, Vv.z);
  apply_one(a, cs, W.w, G.w, Mv.w, Vv.w);
  *reinterpret_cast<float4*>(w) = W;
  if (a.adam) {
    *reinterpret_cast<float4*>(m) = Mv;
    *reinterpret_cast<float4*>(v) = Vv;
  }
}

__device__ __forceinline__ void apply_body(const ApplyArgs& a, int flat4, int64_t blk, int64_t nblk) {
  if (a.ctl && ws_refused(a.ctl, a.sig, a.status, nullptr)) return;
  if (a.abort && *a.abort != 0.f) return;
  const float cs = a.clip / fmaxf(sqrtf(*a.norm2), a.clip);
  float dm = 0.f, dv = 0.f;
  if (flat4) {
    const int64_t n4 = a.rows * (int64_t)a.cols / 4;
    for (int64_t q = blk * blockDim.x + threadIdx.x; q < n4; q += nblk * blockDim.x)
      apply4(a, cs, a.w + 4 * q, a.g + 4 * q, a.adam ? a.m + 4 * q : nullptr, a.adam ? a.v + 4 * q : nullptr);
    return;
  }
  const bool v4 = a.cols % 4 == 0 && a.ld % 4 == 0 && ((uintptr_t)a.w % 16) == 0 && ((uintptr_t)a.g % 16) == 0 &&
                  (!a.adam || (((uintptr_t)a.m % 16) == 0 && ((uintptr_t)a.v % 16) == 0));
  const int64_t nw = nblk * (blockDim.x / KGE_WAVE);
  for (int64_t r = blk * (blockDim.x / KGE_WAVE) + wave_id(); r < a.rows; r += nw) {
    float* wr = a.w + r * a.ld;
    const int64_t go = r * (int64_t)a.cols;
    if (v4) {
      for (int c = 4 * lane_id(); c < a.cols; c += 4 * KGE_WAVE)
        apply4(a, cs, wr + c, a.g + go + c, a.adam ? a.m + go + c : nullptr, a.adam ? a.v + go + c : nullptr);
    } else {
      for (int c = lane_id(); c < a.cols; c += KGE_WAVE)
        apply_one(a, cs, wr[c], a.g[go + c], a.adam ? a.m[go + c] : dm, a.adam ? a.v[go + c] : dv);
    }
  }
}

struct ApplyMany {
  ApplyArgs a[kMaxApply];
  int32_t flat4[kMaxApply];
  uint32_t first[kMaxApply + 1];   // variable v owns blocks [first[v], first[v + 1])
  int32_t n;
};

__global__ __launch_bounds__(256) void apply_kernel(ApplyMany M) {
  const uint32_t b = blockIdx.x;
  int v = 0;
  while (v + 1 < M.n && b >= M.first[v + 1]) ++v;
  apply_body(M.a[v], M.flat4[v], (int64_t)(b - M.first[v]), (int64_t)(M.first[v + 1] - M.first[v]));
}

void launch_apply_many(const ApplyArgs* a, int n, hipStream_t st) {
  ApplyMany M{};
  uint32_t nb = 0;
  int k = 0;
  for (int i = 0; i < n && i < kMaxApply; ++i) {
    const int64_t total = a[i].rows * (int64_t)a[i].cols;
    if (total == 0) continue;
    const bool flat4 = a[i].ld == a[i].cols && total % 4 == 0 && ((uintptr_t)a[i].w % 16) == 0 &&
                       ((uintptr_t)a[i].g % 16) == 0 &&
                       (!a[i].adam || (((uintptr_t)a[i].m % 16) == 0 && ((uintptr_t)a[i].v % 16) == 0));
    const int64_t work = flat4 ? (total / 4 + 255) / 256 : (a[i].rows + 3) / 4;
    M.a[k] = a[i];
    M.flat4[k] = flat4 ? 1 : 0;
    M.first[k] = nb;
    nb += (uint32_t)std::min<int64_t>(std::max<int64_t>(work, 1), 8192);
    ++k;
  }
  if (k == 0) return;
  M.first[k] = nb;
  M.n = k;
  hipLaunchKernelGGL(apply_kernel, dim3(nb), dim3(256), 0, st, M);
}

void launch_apply(const ApplyArgs& a, hipStream_t st) { launch_apply_many(&a, 1, st); }

kge_status launch_step_elementwise(const StepArgs& A, const StepGeom& G, int model, int sk,
                                   hipStream_t st, hipEvent_t const* ev) {
#ifdef KGE_ONLY_ONE
  // quick-iteration builds (tools/phase_prof.py): the bench's C2 instance only
  if (model == KGE_MODEL_TRANSE && G.vec == 4 && G.nc == 1 && sk == SK_P2 && A.side_mode == KGE_SIDE_HT)
    return launch_family<TransE, 4, 1, SK_P2>(A, G, st, ev);
  return KGE_EUNSUPPORTED;
#else
  switch (model) {
    case KGE_MODEL_TRANSE: return launch_transe(A, G, sk, st, ev);
    case KGE_MODEL_DISTMULT: return launch_distmult(A, G, st, ev);
    case KGE_MODEL_ROTATE: return launch_rotate(A, G, sk, st, ev);
    default: return KGE_EUNSUPPORTED;
  }
#endif
}

#ifdef KGE_ONLY_ONE
// single-instance builds (tools/phase_prof.py, tools/variants.py): the other families are stubs
kge_status launch_step_proj(const StepArgs&, const StepGeom&, const PjPlan&, int, hipStream_t, hipEvent_t const*) {
  return KGE_EUNSUPPORTED;
}
kge_status launch_rank(const RankArgs&, int, int, int, hipStream_t) { return KGE_EUNSUPPORTED; }
kge_status launch_step_rescal(const StepArgs&, const StepGeom&, const RelArgs&, float, float*, hipStream_t,
                              hipEvent_t const*) {
  return KGE_EUNSUPPORTED;
}
#endif


}  // namespace kge

#ifdef KGE_PHASE_PROF
// profiling builds: read / reset the per-phase tick counters
extern "C" int kge_prof_read(unsigned long long* out, int n) {
  if (n > 64) n = 64;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(kge::g_kge_prof), n * sizeof(unsigned long long)) != hipSuccess) return 1;
  unsigned long long z[64] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(kge::g_kge_prof), z, sizeof(z)) != hipSuccess;
}
#endif
