// Owner-side scoring for the multi-GPU step (KGE/sharded.py "owner" mode;
// the reference is single-device, BaseModel.py:19-21, so SURVEY.md 8(e) is
// the spec). Instead of fetching every negative's row to the positive's rank,
// each rank scores all ranks' positives against the negatives IT owns and
// sends back one record per positive; the positive's rank merges them.
//
//   owner score   score_kernel<..., OWN = true> (kge_step_impl.h)
//   merge         owner_merge_kernel (here): per positive of this rank, the
//                 records of every owner -> the reference's per-positive
//                 quantities (BaseModel.py:320-327): softmax over all K
//                 negatives (loss.py:174-182), loss, clip-norm partials, the
//                 positive's h / r / t row gradients, destination keys
//   owner update  owner_coef_kernel (here) turns each owned negative's
//                 (R, ties) into its coefficient with the positive's global
//                 softmax state, then the update kernel applies them
#pragma once
#include "kge_step_impl.h"

namespace kge {

constexpr int kMergeWaves = 4;   // merge kernel: one wave per positive

// One wave per positive i of this rank: its context, score and own gradient
// (as the score kernel computes them), then the G owners' records merged the
// way the score kernel merges its waves -- Ms = max_o Ms_o, F_o = exp(Ms_o -
// Ms) (SANS), Z = sum F_o Z_o, every accumulator and norm partial scaled by
// F_o / Z -- so the result is the single-device step's up to float order.
template <template <int, int, int> class Model, int VEC, int NC, int SK>
__global__ __launch_bounds__(kMergeWaves * KGE_WAVE) void owner_merge_kernel(StepArgs A) {
  using M = Model<VEC, NC, SK>;
  using F = Frag<VEC, NC>;
  constexpr int FL = KGE_WAVE * VEC * NC;
  __shared__ float s_img[kMergeWaves][3 * FL];
  __shared__ float s_part[kMergeWaves][8];
  __shared__ int s_last;
  if (ws_refused(A.ctl, A.sig, A.status, A.loss_out)) return;
  const int lane = lane_id(), wv = wave_id(), tid = threadIdx.x;
  const int64_t i = (int64_t)blockIdx.x * kMergeWaves + wv;
  const bool active = i < A.B;
  const int G = A.own_G;
  int err = 0;
  float lossi = 0.f, n[4] = {0.f, 0.f, 0.f, 0.f};
  int64_t ph = 0, pr = 0, pt = 0;
  if (active) {
    ph = load_idx(A.pos, i * 3 + 0, A.i64);
    pr = load_idx(A.pos, i * 3 + 1, A.i64);
    pt = load_idx(A.pos, i * 3 + 2, A.i64);
    ph = ent_row(A, ph, &err);
    if (pr < 0 || pr >= A.rel.rows) { err = KGE_ERANGE; pr = 0; }
    pt = ent_row(A, pt, &err);
    const MP mp{A.limit, false, nullptr};
    typename M::Ctx ctx;
    M::load_ctx(ctx, A.ent, A.rel, ph, pr, pt, mp);
    float Rp, tp = 1.f, sp, lpp = 0.f;
    F pH, pR, pT;
    pH.zero(); pR.zero(); pT.zero();
    float pn[4] = {0.f, 0.f, 0.f, 0.f};
    {
      F a, b, E0;
      E0.zero();
      M::fwd(ctx, KIND_POS, E0, a, b);
      Rp = lane_reduce<5, SK == SK_PINF>(score_partial<SK, M::CPLX>(a, b, A.p));
      if (SK == SK_PINF) tp = lane_reduce<5, false>(tie_partial<M::CPLX>(a, Rp));
      sp = score_value<SK>(Rp, A.pw, &lpp, A.p);
      if (A.train) M::bwd(ctx, KIND_POS, E0, a, b, 1.f, SK == SK_PGEN ? A.p : Rp, pH, pR, pT, pn, mp);
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) pn[v] = wave_sum(pn[v]);
    // the owners' record headers (every lane reads the same words)
    const bool sans = A.loss_kind == KGE_LOSS_SANS;
    auto rec = [&](int o) { return A.own_rec + ((int64_t)o * A.B + i) * (int64_t)A.rec_cols; };
    float Ms = -INFINITY;
    for (int o = 0; o < G; ++o) Ms = fmaxf(Ms, rec(o)[0]);
    float Z = 0.f, cw = 0.f;
    for (int o = 0; o < G; ++o) {
      const float* h = rec(o);
      const float fo = !sans ? 1.f : (h[0] == -INFINITY ? 0.f : expf(h[0] - Ms));
      Z += h[1] * fo;
      cw += h[3];
    }
    const float invZ = sans ? (Z > 0.f ? 1.f / Z : 0.f) : 1.f;
    float lossp, cp;
    switch (A.loss_kind) {
      case KGE_LOSS_HINGE:
        lossp = 0.f;
        cp = -cw;
        if (A.Keff == 0) lossp = NAN;   // sum([]) / 0 (loss.py:81-82)
        break;
      case KGE_LOSS_LOGISTIC: lossp = 0.f; cp = -cw; break;
      case KGE_LOSS_BCE:
        lossp = -log_sigmoid(sp) * A.inv_b;
        cp = -sigmoid(-sp) * A.inv_b;
        break;
      case KGE_LOSS_SANS:
        lossp = -log_sigmoid(sp + A.margin) * A.inv_b;
        cp = -sigmoid(-(sp + A.margin)) * A.inv_b;
        break;
      default:
        lossp = (sp - 1.f) * (sp - 1.f) * 0.5f * A.inv_b;
        cp = (sp - 1.f) * A.inv_b;
        break;
    }
    const float ap = score_alpha<SK>(cp, Rp, lpp, tp, A.pw, A.p);
    float wl;   // weight of the negatives' summed loss terms (loss.py)
    switch (A.loss_kind) {
      case KGE_LOSS_HINGE: wl = A.inv_bk; break;
      case KGE_LOSS_LOGISTIC: wl = 1.f; break;
      case KGE_LOSS_SANS: case KGE_LOSS_BCE: wl = -A.inv_b; break;
      default: wl = 0.5f * A.inv_b; break;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) n[v] = ap * ap * pn[v];
    float lneg = 0.f;
    F gH, gR, gT;
    if (A.train) {
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) { gH.v[q] = ap * pH.v[q]; gR.v[q] = ap * pR.v[q]; gT.v[q] = ap * pT.v[q]; }
    }
    for (int o = 0; o < G; ++o) {
      const float* h = rec(o);
      const float fo = (!sans ? 1.f : (h[0] == -INFINITY ? 0.f : expf(h[0] - Ms))) * invZ;
      lneg += (sans ? fo : 1.f) * h[2];
#pragma unroll
      for (int v = 0; v < 4; ++v) n[v] += fo * fo * h[4 + v];
      if (A.train) {
        F x, y;
        load_row(x, h + kRecHead, FL);
#pragma unroll
        for (int q = 0; q < VEC * NC; ++q) gH.v[q] += fo * x.v[q];
        if constexpr (rec_img<M>::n == 2) {   // r accumulator = h - t (TransE, kge_models.h)
          load_row(y, h + kRecHead + FL, FL);
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) {
            gR.v[q] += fo * (x.v[q] - y.v[q]);
            gT.v[q] += fo * y.v[q];
          }
        } else {
          load_row(y, h + kRecHead + FL, FL);
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) gR.v[q] += fo * y.v[q];
          load_row(y, h + kRecHead + 2 * FL, FL);
#pragma unroll
          for (int q = 0; q < VEC * NC; ++q) gT.v[q] += fo * y.v[q];
        }
      }
    }
    float rsq = 0.f;
    if (A.rel_reg != 0.f) {   // DistMult: lambda * mean_i ||r_i||^2 (DistMult.py:164-165), its own slice
      F Rr;
      load_row(Rr, A.rel.row(pr), A.rel.cols);
      rsq = wave_sum(sq_partial(Rr));
      const float gsc = A.rel_reg * A.inv_b;
      lossp += rsq * gsc;
      n[1] += 4.f * gsc * gsc * rsq;
    }
    lossi = lossp + wl * lneg;
    if (A.train) {
      float* img = s_img[wv];
#pragma unroll
      for (int q = 0; q < VEC * NC; ++q) {
        const int e = (q / VEC * KGE_WAVE + lane) * VEC + q % VEC;
        img[e] = gH.v[q];
        img[FL + e] = gR.v[q];
        img[2 * FL + e] = gT.v[q];
      }
    }
    if (lane == 0) {
      if (A.own_stats_out) {
        float4 st = make_float4(Ms, invZ, sp, 0.f);
        *reinterpret_cast<float4*>(A.own_stats_out + 4 * i) = st;
      }
      if (A.pos_score_out) A.pos_score_out[i] = sp;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (A.train) {
      // the positive's row gradients where the update kernel reads them
      // (gpos [B, 3, gcols]; RotatE's phase gradient of element k at float 2k)
      const float* img = s_img[wv];
      for (int v = 0; v < 3; ++v) {
        const int cols = v == 1 ? A.rel_gcols : A.ent.cols;
        for (int k = lane; k < cols; k += KGE_WAVE) {
          const int src = (v == 1 && A.rel_half) ? 2 * k : k;
          float s = img[v * FL + src];
          if (v == 1 && A.rel_reg != 0.f) s += (A.rel_reg * A.inv_b) * (2.f * A.rel.row(pr)[k]);
          A.gpos[i * 3 * (int64_t)A.gcols + v * (int64_t)A.gcols + k] = s;
        }
      }
      if (A.seg_merge) {   // the segmented update pass's keys: (destination << 32 | 4 i + c)
        if (lane < 3) {
          const int64_t dest = lane == 0 ? ph : lane == 1 ? pt : A.ent.rows + pr;
          A.seg_raw[3 * i + lane] = ((unsigned long long)dest << 32) | (unsigned long long)(4u * (uint32_t)i + lane);
        }
      } else if (lane < 3 && (A.rel_dests || lane != 2)) {
        const int64_t dest = lane == 0 ? ph : lane == 1 ? pt : A.ent.rows + pr;
        bin_key(A, dest, A.nkeyneg + (((uint32_t)i) << 2) + (uint32_t)lane);
      }
    }
  }
  if (err) set_status(A.status, err);
  if (lane == 0) {
    s_part[wv][0] = lossi;
#pragma unroll
    for (int v = 0; v < 4; ++v) s_part[wv][1 + v] = n[v];
  }
  __syncthreads();
  // workgroup partials in wave order; the last workgroup reduces them in
  // workgroup order (this rank's loss and norm^2 shares; the caller
  // all-reduces them) and hands the overflow list length to the update pass
  if (tid == 0) {
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < kMergeWaves; ++w)
#pragma unroll
      for (int k = 0; k < 5; ++k) acc[k] += s_part[w][k];
#pragma unroll
    for (int k = 0; k < 5; ++k)
      __hip_atomic_store(&A.part[(int64_t)blockIdx.x * 8 + k], acc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t prev = __hip_atomic_fetch_add(&A.ctl->score_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (uint32_t)(gridDim.x - 1);
  }
  __syncthreads();
  if (s_last && wv == 0) {
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = lane; w < (int)gridDim.x; w += KGE_WAVE) {
#pragma unroll
      for (int k = 0; k < 5; ++k)
        acc[k] += __hip_atomic_load(&A.part[(int64_t)w * 8 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int k = 0; k < 5; ++k) acc[k] = wave_sum(acc[k]);
    if (lane == 0) {
      A.loss_out[0] = acc[0];
      A.ctl->loss = acc[0];
#pragma unroll
      for (int v = 0; v < 4; ++v)
        if (A.norm2_out) A.norm2_out[v] = acc[1 + v];
      A.ctl->score_ticket = 0u;
      A.ctl->ovf_len = __hip_atomic_exchange(&A.ctl->ovf_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      A.ctl->lng_count = 0u;   // the update pass's deferred long destinations
      A.ctl->score_pending = A.sig;   // (the merge is always a PHASE_SCORE call: the phase gate's token)
      if (A.own_flags_out) {   // the step's flags for the caller's all-reduce, zeroed for the next step
        const float x = A.own_flags_in ? A.own_flags_in[0] : 0.f, o = A.own_flags_in ? A.own_flags_in[1] : 0.f;
        A.own_flags_out[0] = x;
        A.own_flags_out[1] = o;
        A.own_flags_out[2] = x + o;
        if (A.own_flags_in) { A.own_flags_in[0] = 0.f; A.own_flags_in[1] = 0.f; }
      }
    }
  }
}

// The split step's phase gate, one thread (phase_gate_kernel, kge_abi.hip):
// the score pass's token read and cleared; a missing / foreign one poisons
// the workspace (every guarded kernel after it refuses) and sets the status.
// Vector (atomic) loads, and the reset only after p is known: plain loads of
// these uniform words become scalar loads, which the reset's vector store
// may overtake (it would read its own 0).
__device__ __forceinline__ void phase_gate_check(StepCtl* ctl, uint32_t sig, int32_t* status) {
  const uint32_t s = __hip_atomic_load(&ctl->plan_sig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t p = __hip_atomic_load(&ctl->score_pending, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (p != 0u) __hip_atomic_store(&ctl->score_pending, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (s != sig || p != sig) {
    // (s is another plan's: its kernels refuse the workspace anyway; 0: the
    // update pass would claim a fresh workspace and run on empty lists)
    if (s == 0u || s == sig) __hip_atomic_store(&ctl->plan_sig, kPoisonedSig, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    set_status(status, KGE_EWORKSPACE);
  }
}

// Each owned negative's coefficient from its (R, ties) and its positive's
// global softmax state: the score kernel's finalise pass (neg_coef,
// score_alpha) with (Ms, 1/Z, s_pos) from the merge. The owner update pass's
// first launch, so it carries the phase gate (thread 0 of block 0). The
// other threads may still compute coefficients for a refused pass: they
// write only workspace scratch, and the update kernel after this launch
// refuses the poisoned workspace.
template <int SK>
__global__ __launch_bounds__(256) void owner_coef_kernel(StepArgs A) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    phase_gate_check(A.ctl, A.sig, A.status);
    if (A.own_sticky && A.own_flags_out) {   // (every training step, aborted ones included)
      A.own_sticky[0] = fmaxf(A.own_sticky[0], A.own_flags_out[0]);
      A.own_sticky[1] = fmaxf(A.own_sticky[1], A.own_flags_out[1]);
    }
  }
  if (ws_refused(A.ctl, A.sig, A.status, nullptr)) return;
  if (A.abort_flag && *A.abort_flag != 0.f) return;
  const uint32_t n = min(A.ctl->own_len, A.own_cap);
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
    const uint32_t code = A.own_codes[k];
    const float4 st = *reinterpret_cast<const float4*>(A.own_stats + 4 * (int64_t)(code >> A.kshift));
    const float2 raw = A.coef[code];
    float lp;
    const float s = score_value<SK>(raw.x, A.pw, &lp, A.p);
    const float c = neg_coef(A, s, st.z, st.x, st.y);
    A.coef[code] = make_float2(score_alpha<SK>(c, raw.x, lp, raw.y, A.pw, A.p), SK == SK_PGEN ? A.p : raw.x);
  }
}

template <template <int, int, int> class Model, int VEC, int NC, int SK>
kge_status launch_owner_family(const StepArgs& A, const StepGeom& G, int phase, hipStream_t st) {
  switch (phase) {
    case 0:   // owner score
      if (A.side_mode == KGE_SIDE_HT)
        hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK, KGE_SIDE_HT, true>), dim3(G.nWG), dim3(kStepThreads),
                           G.lds_score, st, A);
      else if (A.side_mode == KGE_SIDE_H)
        hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK, KGE_SIDE_H, true>), dim3(G.nWG), dim3(kStepThreads),
                           G.lds_score, st, A);
      else
        hipLaunchKernelGGL((score_kernel<Model, VEC, NC, SK, KGE_SIDE_T, true>), dim3(G.nWG), dim3(kStepThreads),
                           G.lds_score, st, A);
      return KGE_OK;
    case 1: {   // owner coefficients (the update kernel follows)
      const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(((int64_t)A.own_cap + 255) / 256, 2048));
      hipLaunchKernelGGL((owner_coef_kernel<SK>), dim3((unsigned)blocks), dim3(256), 0, st, A);
      return KGE_OK;
    }
    default:   // merge
      hipLaunchKernelGGL((owner_merge_kernel<Model, VEC, NC, SK>), dim3((unsigned)((A.B + kMergeWaves - 1) / kMergeWaves)),
                         dim3(kMergeWaves * KGE_WAVE), 0, st, A);
      return KGE_OK;
  }
}

// per-family dispatch over the fragment geometry (kge_owner_<family>.hip)
kge_status launch_owner_transe(const StepArgs& A, const StepGeom& G, int sk, int phase, hipStream_t st);
kge_status launch_owner_other(const StepArgs& A, const StepGeom& G, int model, int sk, int phase, hipStream_t st);

}  // namespace kge
