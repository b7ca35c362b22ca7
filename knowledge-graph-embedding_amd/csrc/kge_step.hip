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
// Each wave owns 4 rows and issues all their loads before reducing. A second
// table (t2, may be null) is constrained in the same launch (TransR / TransD
// clip ent_emb and rel_emb: one launch, not two).
__device__ __forceinline__ void constrain_table(float* __restrict__ t, int64_t rows, int32_t cols, int64_t ld,
                                                int kind, float value) {
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

__global__ __launch_bounds__(256) void constrain_rows_kernel(float* __restrict__ t, int64_t rows,
                                                              int32_t cols, int64_t ld, int kind,
                                                              float value, StepCtl* ctl, uint32_t sig,
                                                              int32_t* status, float* __restrict__ t2,
                                                              int64_t rows2, int32_t cols2, int64_t ld2) {
  if (ctl && ws_refused(ctl, sig, status, nullptr)) return;   // launched by a step: guarded
  constrain_table(t, rows, cols, ld, kind, value);
  if (t2) constrain_table(t2, rows2, cols2, ld2, kind, value);
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

// ------------------------------------------------------------ owner merge update
// The update pass of the owner merge (KGE_FLAG_OWNER_MERGE | PHASE_UPDATE,
// StepArgs::seg_merge): this rank's positives' own row gradients (gpos rows,
// owner_merge_kernel) summed per destination -- head / tail entity rows
// (own rows: the clip-scaled SGD step; fetched rows >= remote_from: the raw
// gradient in place) and relation rows (raw gradient into grel) -- as a
// segmented sum over the n = 3 B keys (destination << 32 | code), code = 4 i
// + c (c: 0 head, 1 tail, 2 relation):
//   M1  plan     the split-step phase gate (workgroup 0), grel zero-filled,
//                and every key (written by the merge, seg_raw) placed at its
//                rank (#smaller keys: the keys are distinct) -- all n keys
//                staged in each workgroup's LDS, a wave per 4 keys, no sort
//                passes;
//   M2  chunks   a wave per CH (4-8) consecutive sorted keys, every gradient row and
//                destination row of the chunk requested at once; each run of
//                one destination that starts and ends in the chunk is summed
//                (ascending code) and applied; a run entering from the
//                previous chunk leaves a head partial, one leaving into the
//                next chunk a tail partial;
//   M3  combine  the wave of the chunk where a chunk-spanning run starts
//                finds the run's last chunk (64 chunks tested per step), adds
//                its tail partial and the following chunks' head partials in
//                chunk order (8 in flight), and applies the sum.
// A Zipf-hot destination (hundreds of keys at C5) is summed by many waves,
// not one chain (the update kernel / rel_rank / rel_seg / long_rows sequence
// this replaces took ~80 us per step there). Same values every run.
__global__ __launch_bounds__(256) void merge_plan_kernel(StepArgs A, float* zero, int64_t nz) {
  __shared__ unsigned long long s_k[kSegMaxKeys];
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nz; q += (int64_t)gridDim.x * blockDim.x)
    zero[q] = 0.f;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // the phase gate (phase_gate_kernel, kge_abi.hip), vector loads first
    const uint32_t s = __hip_atomic_load(&A.ctl->plan_sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t p = __hip_atomic_load(&A.ctl->score_pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (p != 0u) __hip_atomic_store(&A.ctl->score_pending, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s != A.sig || p != A.sig) {
      if (s == 0u || s == A.sig)
        __hip_atomic_store(&A.ctl->plan_sig, kPoisonedSig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      set_status(A.status, KGE_EWORKSPACE);
    }
  }
  // another plan's workspace: nothing of it is touched (this plan's own
  // refused pass may still rank its keys: the chunk kernels refuse it)
  if (ws_refused(A.ctl, A.sig, A.status, nullptr)) return;
  // the keys the merge left (seg_raw, in positive order), staged whole; each
  // wave ranks 4 of them, its lanes sweeping n / 64 keys each
  const int n = 3 * (int)A.B;
  if ((int64_t)blockIdx.x * 16 >= n) return;
  for (int j = threadIdx.x; j < n; j += blockDim.x) s_k[j] = A.seg_raw[j];
  __syncthreads();
  const int lane = lane_id();
  const int me0 = (int)blockIdx.x * 16 + wave_id() * 4;
  unsigned long long k[4];
  int rank[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    k[q] = me0 + q < n ? s_k[me0 + q] : 0ull;
    rank[q] = 0;
  }
  for (int j = lane; j < n; j += KGE_WAVE) {   // one LDS read, four compares
    const unsigned long long x = s_k[j];
#pragma unroll
    for (int q = 0; q < 4; ++q) rank[q] += x < k[q];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) rank[q] += __shfl_xor(rank[q], o, KGE_WAVE);
    if (lane == q && me0 + q < n) A.seg_keys[rank[q]] = k[q];
  }
}

// the apply of one destination's summed row g (this lane's columns 4 lane +
// 256 u); y: the destination row as loaded with the chunk (own entity rows)
template <int JM>
__device__ __forceinline__ void seg_apply(const StepArgs& A, int64_t dest, const float4 (&g)[JM],
                                          const float4 (&y)[JM], float sce) {
  const int lane = lane_id();
  if (dest < A.ent.rows) {
    float* row = A.ent.row_w(dest);
    const bool raw = dest >= A.remote_from;
#pragma unroll
    for (int u = 0; u < JM; ++u) {
      const int c = 4 * lane + 256 * u;
      const float v[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
      const float w[4] = {y[u].x, y[u].y, y[u].z, y[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c + e < A.ent.cols) row[c + e] = raw ? v[e] : w[e] + v[e] * sce;
    }
  } else {
    const int64_t r = dest - A.ent.rows;
    float scr = A.ctl->scale[A.sc_rel_idx];
    if (A.scale_from_norm2) scr = -A.lr * (A.clip_norm / fmaxf(sqrtf(A.norm2_out[A.sc_rel_idx]), A.clip_norm));
#pragma unroll
    for (int u = 0; u < JM; ++u) {
      const int c = 4 * lane + 256 * u;
      const float v[4] = {g[u].x, g[u].y, g[u].z, g[u].w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (c + e >= A.rel_gcols) break;
        if (A.rel_grad || A.grad_mode) A.grel[r * (int64_t)A.rel_gcols + c + e] = v[e];
        else { float* wp = A.rel.row_w(r) + c + e; *wp = *wp + v[e] * scr; }
      }
    }
  }
}

__device__ __forceinline__ float seg_scale_ent(const StepArgs& A) {
  float sc = A.ctl->scale[A.sc_ent_idx];
  if (A.scale_from_norm2) sc = -A.lr * (A.clip_norm / fmaxf(sqrtf(A.norm2_out[A.sc_ent_idx]), A.clip_norm));
  return sc;
}

// key's gradient row (gpos [B, 3, gcols]: head, relation, tail) and its
// destination row (own entity rows only; else entity row 0, unused)
template <int JM>
__device__ __forceinline__ void seg_load(const StepArgs& A, unsigned long long key, float4 (&x)[JM],
                                         float4 (&y)[JM]) {
  const int lane = lane_id();
  const uint32_t code = (uint32_t)key;
  const int64_t dest = (int64_t)(key >> 32);
  const uint32_t c = code & 3u;
  const int v = c == 0u ? 0 : c == 1u ? 2 : 1;
  const int cols = v == 1 ? A.rel_gcols : A.ent.cols;
  const float* g = A.gpos + (int64_t)(code >> 2) * 3 * A.gcols + (int64_t)v * A.gcols;
  const float* w = A.ent.row(dest < A.ent.rows && dest < A.remote_from ? dest : 0);
#pragma unroll
  for (int u = 0; u < JM; ++u) {
    const int cc = 4 * lane + 256 * u;
    x[u] = cc < cols ? *reinterpret_cast<const float4*>(g + cc) : make_float4(0.f, 0.f, 0.f, 0.f);
    y[u] = cc < A.ent.cols ? *reinterpret_cast<const float4*>(w + cc) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int JM>
constexpr int seg_chunk() { return JM == 1 ? 8 : 4; }   // keys per chunk (a wave each)

template <int JM>
__global__ __launch_bounds__(256) void merge_chunk_kernel(StepArgs A) {
  constexpr int CH = seg_chunk<JM>();
  if (ws_refused(A.ctl, A.sig, A.status, nullptr)) return;
  if (A.abort_flag && *A.abort_flag != 0.f) return;
  const int n = 3 * (int)A.B;
  const int nch = (n + CH - 1) / CH;
  const int k = (int)blockIdx.x * 4 + wave_id();
  if (k >= nch) return;
  const int lane = lane_id();
  const int j0 = k * CH, cnt = min(CH, n - j0);
  // the chunk's keys (lanes 0..CH-1) and its neighbours' (lane 62: previous, 63: next)
  unsigned long long kv = ~0ull;
  if (lane < cnt) kv = A.seg_keys[j0 + lane];
  else if (lane == 62 && j0 > 0) kv = A.seg_keys[j0 - 1];
  else if (lane == 63 && j0 + cnt < n) kv = A.seg_keys[j0 + cnt];
  auto key_at = [&](int l) { return (unsigned long long)__shfl((long long)kv, l, KGE_WAVE); };
  const int64_t dprev = j0 > 0 ? (int64_t)(key_at(62) >> 32) : -1;
  const int64_t dnext = j0 + cnt < n ? (int64_t)(key_at(63) >> 32) : -1;
  // every row of the chunk in flight at once
  float4 x[CH][JM], y[CH][JM];
  int64_t dst[CH];
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    const unsigned long long kt = key_at(min(t, cnt - 1));
    dst[t] = (int64_t)(kt >> 32);
    seg_load<JM>(A, kt, x[t], y[t]);
  }
  const float sce = seg_scale_ent(A);
  float4 acc[JM];
#pragma unroll
  for (int u = 0; u < JM; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  bool first = true;   // the current run starts at the chunk's first key
#pragma unroll
  for (int t = 0; t < CH; ++t) {
    if (t < cnt) {
#pragma unroll
      for (int u = 0; u < JM; ++u) {
        acc[u].x += x[t][u].x; acc[u].y += x[t][u].y; acc[u].z += x[t][u].z; acc[u].w += x[t][u].w;
      }
      const bool last = t == cnt - 1 || dst[t + 1 < CH ? t + 1 : t] != dst[t];
      if (last) {   // (uniform)
        const bool from_prev = first && dst[t] == dprev;
        const bool to_next = t == cnt - 1 && dst[t] == dnext;
        if (!from_prev && !to_next) {
          seg_apply<JM>(A, dst[t], acc, y[t], sce);
        } else {   // head partial (entered from the previous chunk), else tail partial
          float* pr = A.seg_part + (int64_t)(2 * k + (from_prev ? 0 : 1)) * A.gcols;
#pragma unroll
          for (int u = 0; u < JM; ++u) {
            const int c = 4 * lane + 256 * u;
            if (c < A.gcols) *reinterpret_cast<float4*>(pr + c) = acc[u];
          }
        }
#pragma unroll
        for (int u = 0; u < JM; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        first = false;
      }
    }
  }
}

template <int JM>
__global__ __launch_bounds__(256) void merge_combine_kernel(StepArgs A) {
  constexpr int CH = seg_chunk<JM>();
  if (ws_refused(A.ctl, A.sig, A.status, nullptr)) return;
  if (A.abort_flag && *A.abort_flag != 0.f) return;
  const int n = 3 * (int)A.B;
  const int nch = (n + CH - 1) / CH;
  const int k = (int)blockIdx.x * 4 + wave_id();
  if (k >= nch - 1) return;   // (the last chunk's runs cannot leave it)
  const int lane = lane_id();
  const int j0 = k * CH;
  // this chunk's keys (lanes 0..CH-1), the one before it (lane 62), the next chunk's first (63)
  unsigned long long kv = ~0ull;
  if (lane < CH) kv = A.seg_keys[j0 + lane];
  else if (lane == 62 && j0 > 0) kv = A.seg_keys[j0 - 1];
  else if (lane == 63) kv = A.seg_keys[j0 + CH];
  const int64_t dk = (int64_t)(kv >> 32);
  const int64_t dlast = __shfl(dk, CH - 1, KGE_WAVE);
  if (__shfl(dk, 63, KGE_WAVE) != dlast) return;   // no run leaves this chunk
  // the leaving run starts here unless it also entered (then an earlier chunk owns it)
  const uint64_t same = __ballot(lane < CH && dk == dlast);
  if (same == ((1ull << CH) - 1ull) && j0 > 0 && __shfl(dk, 62, KGE_WAVE) == dlast) return;
  // the run's last chunk: the first m > k it does not go through (lanes test
  // 64 chunks at a time: chunk m full, its last key and the next chunk's
  // first key still the run's destination)
  int mend = nch - 1;
  for (int m0 = k + 1; m0 < nch; m0 += KGE_WAVE) {
    const int m = m0 + lane;
    bool through = false;
    if (m < nch - 1) {
      const int jm = m * CH;
      through = (int64_t)(A.seg_keys[jm + CH - 1] >> 32) == dlast && (int64_t)(A.seg_keys[jm + CH] >> 32) == dlast;
    }
    const uint64_t stop = __ballot(m < nch && !through);
    if (stop) { mend = m0 + __builtin_ctzll(stop); break; }
  }
  float4 acc[JM], y[JM];
  const float* pr = A.seg_part + (int64_t)(2 * k + 1) * A.gcols;
  const float* w = A.ent.row(dlast < A.ent.rows && dlast < A.remote_from ? dlast : 0);
#pragma unroll
  for (int u = 0; u < JM; ++u) {
    const int c = 4 * lane + 256 * u;
    acc[u] = c < A.gcols ? *reinterpret_cast<const float4*>(pr + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    y[u] = c < A.ent.cols ? *reinterpret_cast<const float4*>(w + c) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // the head partials of chunks k + 1 .. mend in chunk order, 8 in flight
  for (int m0 = k + 1; m0 <= mend; m0 += 8) {
    float4 x[8][JM];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float* hp = A.seg_part + (int64_t)(2 * min(m0 + t, mend)) * A.gcols;
#pragma unroll
      for (int u = 0; u < JM; ++u) {
        const int c = 4 * lane + 256 * u;
        x[t][u] = c < A.gcols ? *reinterpret_cast<const float4*>(hp + c) : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int t = 0; t < 8; ++t)
      if (m0 + t <= mend) {
#pragma unroll
        for (int u = 0; u < JM; ++u) {
          acc[u].x += x[t][u].x; acc[u].y += x[t][u].y; acc[u].z += x[t][u].z; acc[u].w += x[t][u].w;
        }
      }
  }
  seg_apply<JM>(A, dlast, acc, y, seg_scale_ent(A));
}

template <int JM>
static void launch_merge_chunks(const StepArgs& A, int n, hipStream_t st) {
  const int nch = (n + seg_chunk<JM>() - 1) / seg_chunk<JM>();
  const unsigned g = (unsigned)((nch + 3) / 4);
  hipLaunchKernelGGL(merge_chunk_kernel<JM>, dim3(g), dim3(256), 0, st, A);
  hipLaunchKernelGGL(merge_combine_kernel<JM>, dim3(g), dim3(256), 0, st, A);
}

void launch_merge_segsum(const StepArgs& A, hipStream_t st) {
  const int64_t nz = (A.rel_grad || A.grad_mode) ? A.rel.rows * (int64_t)A.rel_gcols : 0;
  const int n = 3 * (int)A.B;
  const int64_t blocks = std::max<int64_t>({(int64_t)1, (n + 15) / 16, std::min<int64_t>((nz + 1023) / 1024, 256)});
  hipLaunchKernelGGL(merge_plan_kernel, dim3((unsigned)blocks), dim3(256), 0, st, A, A.grel, nz);
  const int w = std::max<int>(A.ent.cols, A.rel_gcols);
  if (w <= 256) launch_merge_chunks<1>(A, n, st);
  else if (w <= 512) launch_merge_chunks<2>(A, n, st);
  else launch_merge_chunks<4>(A, n, st);
}

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
