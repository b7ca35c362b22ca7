// Projection-family step (TransH / TransD): update passes, TransH's dense
// constraint-gradient kernel and the launch sequence. The score kernel
// instances live in kge_proj_transh.hip / kge_proj_transd.hip.
#include <cstdio>
#include <cstdlib>

#include "kge_proj.h"

namespace kge {

kge_status launch_proj_transh(const StepArgs& A, const StepGeom& G, const PjArgs& P, int sk, hipStream_t st);
kge_status launch_proj_transd(const StepArgs& A, const StepGeom& G, const PjArgs& P, int sk, hipStream_t st);

// TransH _constraint_loss terms (TransH.py:200-211) with `constraint`:
//   lambda * ( sum_e [||e||^2 - 1]_+  +  sum_r [(w_r . r / ||r||)^2 - 1e-18]_+ )
// Their gradients reach every row, so TF's gradients of ent_emb, rel_emb and
// rel_hyper are dense tensors (the lookups' slices summed in). One wave per
// row adds the term's gradient to the summed-slice gradient the update passes
// wrote, and reduces the dense norm^2 of each variable (clip_by_norm of the
// dense tensor) and the term's loss. Fixed grid, fixed row order per wave,
// the last workgroup reduces the partials in workgroup order.
__global__ __launch_bounds__(256) void transh_dense_kernel(StepArgs A, PjPlan J) {
  __shared__ float s_w[4][4];
  __shared__ int s_last;
  if (ws_refused(A.ctl, A.sig, A.status, A.loss_out)) return;
  const int lane = lane_id(), wv = wave_id();
  const int64_t E = A.ent.rows, R = A.rel.rows;
  const int d = A.ent.cols;
  const float lam = J.lam;
  const int64_t nw = (int64_t)gridDim.x * 4;
  float n[3] = {0.f, 0.f, 0.f}, loss = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 4 + wv; row < E + R; row += nw) {
    if (row < E) {
      // soft_constraint (constraint.py:34-67, p = 2, value = 1)
      const float* e = A.ent.row(row);
      float* g = J.gdense[0] + row * (int64_t)d;
      float s = 0.f;
      for (int c = lane; c < d; c += KGE_WAVE) s += e[c] * e[c];
      s = lane_reduce<5, false>(s);
      const float nrm = sqrtf(s);
      const float q = nrm * nrm - 1.f;
      const float coef = q >= 0.f ? 2.f * lam : 0.f;
      if (lane == 0) loss += fmaxf(q, 0.f);
      if (!J.grads) continue;
      for (int c = lane; c < d; c += KGE_WAVE) {
        const float v = g[c] + coef * e[c];
        g[c] = v;
        n[0] += v * v;
      }
    } else {
      // orthogonality: u = (w . r) / ||r||, term [u^2 - 1e-18]_+
      const int64_t r = row - E;
      const float* w = J.P.raux.row(r);
      const float* rv = A.rel.row(r);
      float* gr = J.gdense[1] + r * (int64_t)d;
      float* gw = J.gdense[2] + r * (int64_t)d;
      float dot = 0.f, rr = 0.f;
      for (int c = lane; c < d; c += KGE_WAVE) {
        dot += w[c] * rv[c];
        rr += rv[c] * rv[c];
      }
      dot = lane_reduce<5, false>(dot);
      rr = lane_reduce<5, false>(rr);
      const float nr = sqrtf(rr);
      const float u = dot / nr;
      const float q = u * u - 1e-18f;
      const float c0 = q >= 0.f ? lam * 2.f * u : 0.f;
      if (lane == 0) loss += fmaxf(q, 0.f);
      if (!J.grads) continue;
      // d u / d w = r / ||r|| ; d u / d r = w / ||r|| - (w . r) r / ||r||^3
      const float a = c0 / nr, b = c0 * dot / (nr * nr * nr);
      for (int c = lane; c < d; c += KGE_WAVE) {
        const float vr = gr[c] + (a * w[c] - b * rv[c]);
        const float vw = gw[c] + a * rv[c];
        gr[c] = vr;
        gw[c] = vw;
        n[1] += vr * vr;
        n[2] += vw * vw;
      }
    }
  }
  float v4[4] = {n[0], n[1], n[2], loss};
#pragma unroll
  for (int k = 0; k < 4; ++k) v4[k] = lane_reduce<5, false>(v4[k]);
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 4; ++k) s_w[wv][k] = v4[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < 4; ++w) {
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] += s_w[w][k];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      __hip_atomic_store(&J.dpart[(int64_t)blockIdx.x * 4 + k], acc[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t prev = __hip_atomic_fetch_add(&A.ctl->reg_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == gridDim.x - 1;
  }
  __syncthreads();
  if (s_last && wv == 0) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int w = lane; w < (int)gridDim.x; w += KGE_WAVE) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc[k] += __hip_atomic_load(&J.dpart[(int64_t)w * 4 + k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] = lane_reduce<5, false>(acc[k]);
    if (lane == 0) {
      const float reg = lam * acc[3];
      A.loss_out[0] += reg;
      if (A.loss_accum) A.loss_accum[0] += reg;
      A.ctl->loss += reg;
      if (J.grads) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          A.ctl->dn2[k] = acc[k];
          if (A.norm2_out) A.norm2_out[k] = acc[k];
        }
      }
      A.ctl->reg_ticket = 0u;
    }
  }
}

template <int VEC, int NC>
static void upd_mat(const StepArgs& A, unsigned grid, hipStream_t st) {
  if (A.compact)
    hipLaunchKernelGGL((update_kernel<Materialised, VEC, NC, SK_DOT, 1, true>), dim3(grid), dim3(kUpdThreads), 0, st, A);
  else
    hipLaunchKernelGGL((update_kernel<Materialised, VEC, NC, SK_DOT>), dim3(grid), dim3(kUpdThreads), 0, st, A);
}
static void launch_update_mat_pj(const StepArgs& A, int vec, int nc, unsigned grid, hipStream_t st) {
  if (grid == 0) return;
  if (vec == 4) { if (nc == 1) upd_mat<4, 1>(A, grid, st); else upd_mat<4, 2>(A, grid, st); }
  else if (vec == 2) { if (nc == 1) upd_mat<2, 1>(A, grid, st); else upd_mat<2, 2>(A, grid, st); }
  else { if (nc == 1) upd_mat<1, 1>(A, grid, st); else upd_mat<1, 2>(A, grid, st); }
}

static void dbg_sync(hipStream_t st, const char* what) {
  static const bool on = getenv("KGE_DEBUG_SYNC") != nullptr;
  if (!on) return;
  fprintf(stderr, "[kge] launched %s ...", what);
  const hipError_t e = hipStreamSynchronize(st);
  fprintf(stderr, " done (%s)\n", hipGetErrorString(e));
}

kge_status launch_step_proj(const StepArgs& A, const StepGeom& G, const PjPlan& J, int sk, hipStream_t st,
                            hipEvent_t const* ev) {
  dbg_sync(st, "pre");
  const kge_status s = J.td ? launch_proj_transd(A, G, J.P, sk, st) : launch_proj_transh(A, G, J.P, sk, st);
  dbg_sync(st, "proj_kernel");
  if (s != KGE_OK) return s;
  if (ev) (void)hipEventRecord(ev[2], st);
  if (!A.train) {   // validation: the regulariser's loss only
    if (J.dense) hipLaunchKernelGGL(transh_dense_kernel, dim3(kPjDenseWGs), dim3(256), 0, st, A, J);
    return KGE_OK;
  }
  const bool gm = A.grad_mode || J.dense;   // passes write summed gradients
  // aux-table pass first: it leaves the destination counters for the main pass
  StepArgs B2 = A;
  B2.keep_cnt = true;
  B2.grad_mode = gm;
  B2.gpos = J.P.gpos2;
  B2.gpe = J.P.gpos2;
  B2.rel = J.raux_tab;
  B2.sc_rel_idx = 2;
  B2.grel = J.dense ? J.gdense[2] : A.grad_mode ? A.grel_aux : nullptr;
  unsigned grid2;
  if (J.td) {
    B2.ent = J.eaux_tab;
    B2.gneg = J.P.gnegp;
    B2.sc_ent_idx = 3;
    B2.gent = A.grad_mode ? A.gent_aux : nullptr;
    grid2 = (unsigned)G.gridU;
  } else {
    // rel_hyper only: the relation destinations come first in the full
    // (non-compact) mapping, so a grid of R waves visits exactly them;
    // compact: their leaders are positives' keys, the first 3B positions
    B2.rel_only = true;
    if (A.compact) {
      const int64_t waves = (A.npos3 + kUpdKeysPerWave - 1) / kUpdKeysPerWave;
      grid2 = (unsigned)((waves + kUpdWaves - 1) / kUpdWaves);
    } else {
      grid2 = (unsigned)((A.rel.rows + kUpdWaves - 1) / kUpdWaves);
    }
  }
  launch_update_mat_pj(B2, G.vec, G.nc, grid2, st);
  dbg_sync(st, "pass B");
  StepArgs A1 = A;
  A1.grad_mode = gm;
  if (J.dense) {
    A1.gent = J.gdense[0];
    A1.grel = J.gdense[1];
  }
  launch_update_mat_pj(A1, G.vec, G.nc, (unsigned)G.gridU, st);
  dbg_sync(st, "pass A");
  if (J.dense) {
    hipLaunchKernelGGL(transh_dense_kernel, dim3(kPjDenseWGs), dim3(256), 0, st, A, J);
    dbg_sync(st, "dense");
    if (!A.grad_mode) {
      const TabView tabs[3] = {A.ent, A.rel, J.raux_tab};
      for (int v = 0; v < 3; ++v) {
        ApplyArgs a{};
        a.w = tabs[v].p; a.rows = tabs[v].rows; a.cols = tabs[v].cols; a.ld = tabs[v].ld;
        a.g = J.gdense[v]; a.norm2 = &A.ctl->dn2[v]; a.lr = A.lr; a.clip = A.clip_norm;
        a.ctl = A.ctl; a.sig = A.sig; a.status = A.status;
        launch_apply(a, st);
        dbg_sync(st, "apply");
      }
    }
  }
  return KGE_OK;
}

}  // namespace kge
