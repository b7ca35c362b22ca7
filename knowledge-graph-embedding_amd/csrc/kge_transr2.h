// TransR step kernel, two positives per CU (transr2_kernel), and the fp32
// MFMA helpers it shares with transr_kernel (kge_transr.hip). Instantiated
// per score kind by kge_transr2_*.hip (launch_transr2<SK>), so the kinds
// compile in parallel.
#pragma once
#include "kge_step_impl.h"

namespace kge {

using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

constexpr int kTrQ = (kTrMaxSlots + kTrWaves - 1) / kTrWaves;   // slots per wave
constexpr int kTrKV = kTrMaxDim / KGE_WAVE;                     // projected-row floats per lane
constexpr int kTrKS3 = ((kTrMaxSlots + 1 + 15) / 16) * 4;       // GEMM3 k-steps (K + 2 slot rows, 16-padded)

// element gradient of the score wrt a = x - y (Lp kinds): score_grad's rule
template <int SK>
__device__ __forceinline__ float lp_elem_grad(float a, float alpha, float M) {
  if (SK == SK_P2) return alpha * a;
  float s = a > 0.f ? alpha : (a < 0.f ? -alpha : 0.f);
  if (SK == SK_PGEN) return a != 0.f ? s * powf(fabsf(a), M - 1.f) : 0.f;   // M carries p
  if (SK == SK_PINF && fabsf(a) != M) s = 0.f;
  return s;
}

// all-lane sum / max over the wave (permlane + DPP tree, kge_common.h)
__device__ __forceinline__ float wsum(float x) { return lane_reduce<5, false>(x); }
__device__ __forceinline__ float wmax(float x) { return lane_reduce<5, true>(x); }

// Two 16x16 output tiles sharing one B column (bf, in registers) over NC
// 16-wide k chunks, straight-line. The k order inside a chunk is permuted so
// each lane's four A values are adjacent: MFMA step u of chunk c gives lane
// group g = l >> 4 the index k = 16c + 4g + u (bf is loaded in the same
// order), so A comes from LDS as ONE ds_read_b128 per tile per chunk. p0 / p1
// point at row (l & 15) of each tile plus 4g; pad columns of A and bf are zero.
template <int NC>
__device__ __forceinline__ void mfma_pair_b128(f32x4& a0, f32x4& a1, const float* p0, const float* p1,
                                               const float (&bf)[4 * NC]) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const float4 x0 = *reinterpret_cast<const float4*>(p0 + 16 * c);
    const float4 x1 = *reinterpret_cast<const float4*>(p1 + 16 * c);
    a0 = mfma16(x0.x, bf[4 * c + 0], a0);
    a1 = mfma16(x1.x, bf[4 * c + 0], a1);
    a0 = mfma16(x0.y, bf[4 * c + 1], a0);
    a1 = mfma16(x1.y, bf[4 * c + 1], a1);
    a0 = mfma16(x0.z, bf[4 * c + 2], a0);
    a1 = mfma16(x1.z, bf[4 * c + 2], a1);
    a0 = mfma16(x0.w, bf[4 * c + 3], a0);
    a1 = mfma16(x1.w, bf[4 * c + 3], a1);
  }
}

// One 16x16 tile (the odd last row tile of a GEMM): the same k order, the
// chunk's four steps split over two accumulator chains (added at the end) so
// the 40-cycle dependent MFMA latency stays under the 32-cycle issue interval
template <int NC>
__device__ __forceinline__ void mfma_one_b128(f32x4& a0, const float* p0, const float (&bf)[4 * NC]) {
  f32x4 b0 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const float4 x0 = *reinterpret_cast<const float4*>(p0 + 16 * c);
    a0 = mfma16(x0.x, bf[4 * c + 0], a0);
    b0 = mfma16(x0.y, bf[4 * c + 1], b0);
    a0 = mfma16(x0.z, bf[4 * c + 2], a0);
    b0 = mfma16(x0.w, bf[4 * c + 3], b0);
  }
  a0 += b0;
}

// ============================================================ two positives per CU
// The same three products in <= 128 VGPRs and ~78 KB of LDS, so two
// workgroups share a CU and one's VALU phases run under the other's MFMA
// (transr_kernel: 144 KB, 197 VGPRs -> one workgroup per CU).
//
// P = X M_r never goes to LDS. Wave role w owns P's column tiles w and w + 8
// over every row tile, in MFMA accumulator layout: lane l holds column
// l & 15 of rows 4 (l >> 4) .. + 3 of each 16-row tile. Per-row quantities
// (norms, scores, the clip-backward dots) are 16-lane reductions of each tile,
// one partial per wave role in LDS, summed in role order by one thread per
// row. Column quantities (the relation gradient, the summed h / t slices) stay
// in the wave that owns the column. The entity slices S' are kept in the same
// register layout. Over X's buffer go first the positive-side slices
// (re-derived from P) for GEMM2's norm pass, then S' for GEMM2 and GEMM3.
// Rows of the MFMA tiles: the K negatives (row q = negative q). The positive's
// h and t rows are not in the tiles (they would cost a fifth 16-row tile for 2
// rows at K = 64): their projections, back-projections and the rank-2 part of
// dM are matrix-vector products on the VALU, riding on the M_r columns the
// MFMA products already hold in registers. Per-row scalars have two more
// slots: HR = the h row, TR = the t row, which also carries the positive's
// score (its "slot").
struct Tr2Lds {
  int NC, W, LX, NR16, NRR;
  int R, xht, red, ph, pt, rr, sh, st, qh, qt;
  int pn, pinv, xx, xh, xt, sS, sR, sT, sA, dx, dy, ids, misc, total_floats;
};
__host__ __device__ inline Tr2Lds tr2_lds(int d, int k, int K) {
  Tr2Lds L;
  L.NC = tr_nc(d, k);
  L.W = 16 * L.NC;
  L.LX = L.W + 4;
  L.NR16 = (K + 15) & ~15;
  if (L.NR16 == 0) L.NR16 = 16;
  L.NRR = L.NR16 + 2;            // + HR, TR
  int o = 0;
  L.R = o; o += L.NR16 * L.LX;   // X (through GEMM1), then the Q rows, then S' rows
  L.xht = o; o += 2 * L.LX;      // the positive's h, t entity rows
  L.red = o; o += 2 * kTrWaves * L.NRR;   // row reductions: [2][wave role][row]
  int* v[] = {&L.ph, &L.pt, &L.rr, &L.sh, &L.st, &L.qh, &L.qt};   // rows of k floats
  for (int* p : v) { *p = o; o += L.LX; }
  int* f[] = {&L.pn, &L.pinv, &L.xx, &L.xh, &L.xt, &L.sS, &L.sR, &L.sT, &L.sA, &L.dx, &L.dy};
  for (int* p : f) { *p = o; o += L.NRR; }
  L.ids = o; o += (K + 3) & ~3;
  L.misc = o; o += 64;
  L.total_floats = o;
  return L;
}

// the 16-lane sums (or maxima) of four rows' partials x[j] (rows 16 rt + 4 (l >> 4) + j)
// -> dst[row] (lanes with l & 3 == 0 write)
template <bool MAX>
__device__ __forceinline__ void tr2_tile_out(const float (&x)[4], int rt, float* dst) {
  const int lane = lane_id();
  const float s = multi_reduce<4, MAX, 3>(x);
  if ((lane & 3) == 0) dst[rt * 16 + 4 * (lane >> 4) + ((lane & 15) >> 2)] = s;
}
// sum over the four 16-lane groups (lane bits 5, 4): every lane the same bits
__device__ __forceinline__ float tr2_col_sum(float v) {
  float a, b;
  half_swap<5>(v, v, a, b);
  v = a + b;
  half_swap<4>(v, v, a, b);
  return a + b;
}

// NRT: the row-tile count, 1..5 (straight-line row loops; a runtime count
// made the row loops' guards real branches, and the products spilled)
template <int SK, int NC, int NRT>
__global__ __launch_bounds__(kTrThreads) __attribute__((amdgpu_waves_per_eu(4))) void transr2_kernel(StepArgs A, TrArgs T) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  __shared__ float s_w[kTrWaves][4];
  __shared__ int s_last;
  if (ws_refused(A.ctl, A.sig, A.status, A.loss_out)) return;
  const int d = T.d, k = T.k, K = A.Keff;
  const Tr2Lds L = tr2_lds(d, k, K);
  constexpr int W = 16 * NC;
  const int LX = L.LX, NR16 = 16 * NRT, nrt = NRT, nct = (k + 15) >> 4;
  const int NRR = NR16 + 2, HR = NR16, TR = NR16 + 1;
  float* X = sm + L.R;
  float* XH = sm + L.xht;        // [0] h row, [1] t row
  float* red = sm + L.red;
  float* phs = sm + L.ph;
  float* pts = sm + L.pt;
  float* rrs = sm + L.rr;
  float* shs = sm + L.sh;        // summed h slices (k)
  float* sts = sm + L.st;        // summed t slices
  float* qhs = sm + L.qh;        // the positive's own h slice
  float* qts = sm + L.qt;        // the positive's own t slice
  float* pn = sm + L.pn;
  float* pinv = sm + L.pinv;     // 1 / norm of the rows the clip divides, else 1
  float* xx = sm + L.xx;
  float* xh = sm + L.xh;
  float* xt = sm + L.xt;
  float* sS = sm + L.sS;
  float* sR = sm + L.sR;
  float* sT = sm + L.sT;
  float* sA = sm + L.sA;
  float* sdx = sm + L.dx;
  float* sdy = sm + L.dy;
  int32_t* ids = reinterpret_cast<int32_t*>(sm + L.ids);
  float* misc = sm + L.misc;

  KGE_PROF_INIT();
  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  const int g4 = 4 * (lane >> 4), c16 = lane & 15;
  const bool g0 = lane < 16;     // (the positive's values are counted in lane group 0 only)
  const int64_t i = blockIdx.x;
  int err = 0;
  int64_t ph = load_idx(A.pos, i * 3 + 0, A.i64);
  int64_t pr = load_idx(A.pos, i * 3 + 1, A.i64);
  int64_t pt = load_idx(A.pos, i * 3 + 2, A.i64);
  ph = ent_row(A, ph, &err);
  if (pr < 0 || pr >= A.rel.rows) { err = KGE_ERANGE; pr = 0; }
  pt = ent_row(A, pt, &err);
  for (int j = tid; j < K; j += kTrThreads) ids[j] = slot_entity(A, i, j, &err);
  __syncthreads();
  // row -> triple kind (TR carries the positive; HR and pad rows none)
  auto rkind = [&](int row) -> int {
    return row < K ? slot_kind(A.side_mode, row) : row == TR ? KIND_POS : -1;
  };

  KGE_PROF(32);
  // ---- gather X (the negatives; pad rows and columns zero) and the h, t rows:
  // a wave's rows (row = wave + 8 u) all in flight at once
  {
    constexpr int GU = (16 * NRT + 2 + kTrWaves - 1) / kTrWaves;   // rows per wave
    float v[GU][kTrKV];
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int row = wv + u * kTrWaves;
      const float* src = row < K ? A.ent.row(ids[row]) : row == NR16 ? A.ent.row(ph)
                       : row == NR16 + 1 ? A.ent.row(pt) : nullptr;
#pragma unroll
      for (int c4 = 0; c4 < kTrKV; ++c4) {
        const int c = lane + KGE_WAVE * c4;
        v[u][c4] = (src && c < d) ? src[c] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < GU; ++u) {
      const int row = wv + u * kTrWaves;
      if (row >= NR16 + 2) break;
      float* dst = row < NR16 ? X + row * LX : XH + (row - NR16) * LX;
#pragma unroll
      for (int c4 = 0; c4 < kTrKV; ++c4) {
        const int c = lane + KGE_WAVE * c4;
        if (c < W) dst[c] = v[u][c4];
      }
    }
  }
  __syncthreads();
  KGE_PROF(33);
  // row statistics for the rel_proj slice norms: ||x||^2, x.h, x.t (rows K.. NR16: zero)
  for (int row = wv; row < NRR; row += kTrWaves) {
    const float* xr = row < NR16 ? X + row * LX : XH + (row - NR16) * LX;
    float a = 0.f, b = 0.f, c2 = 0.f;
    for (int c = lane; c < d; c += KGE_WAVE) {
      const float x = xr[c];
      a += x * x;
      b += XH[c] * x;
      c2 += XH[LX + c] * x;
    }
    a = wsum(a);
    b = wsum(b);
    c2 = wsum(c2);
    if (lane == 0) { xx[row] = a; xh[row] = b; xt[row] = c2; }
  }

  // wave role: P column tiles w0 and w0 + 8. The two workgroups resident on a
  // CU shift their roles by two waves against each other, so the roles holding
  // a second tile fall on different SIMDs. On an XCD (blockIdx mod 8) the
  // local index j = blockIdx / 8 goes round-robin over 32 CUs (pair j, j + 32)
  // or fills a CU first (pair 2c, 2c + 1): bit 0 of j ^ (j >> 5) differs in both.
  const int jx = (int)(blockIdx.x >> 3);
  const int w0 = (wv - 2 * ((jx ^ (jx >> 5)) & 1)) & (kTrWaves - 1);
  const bool has0 = w0 < nct, has1 = w0 + 8 < nct;
  const int colu[2] = {16 * w0 + c16, 16 * (w0 + 8) + c16};
  auto has = [&](int u) { return u == 0 ? has0 : has1; };
  auto live = [&](int u) { return has(u) && colu[u] < k; };

  // ---- GEMM1: P = X M_r, this role's column tiles, every row tile (in pairs);
  // the h / t projections from the same M_r column (VALU, group partials summed)
  const float* Mr = T.proj.row(pr);
  f32x4 P[2][5];
  float phv[2] = {0.f, 0.f}, ptv[2] = {0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 2; ++u)
#pragma unroll
    for (int rt = 0; rt < 5; ++rt) P[u][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (!has(u)) continue;
    const int col = colu[u];
    float bf[4 * NC];
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int kk = 16 * c + g4 + q;
        bf[4 * c + q] = (kk < d && col < k) ? Mr[(int64_t)kk * k + col] : 0.f;
      }
#pragma unroll
    for (int rt = 0; rt < 5; rt += 2) {
      if (rt >= nrt) break;
      const float* x0 = X + (rt * 16 + c16) * LX + g4;
      if (rt + 1 < 5 && rt + 1 < nrt) mfma_pair_b128<NC>(P[u][rt], P[u][rt + 1 < 5 ? rt + 1 : rt], x0, x0 + 16 * LX, bf);
      else mfma_one_b128<NC>(P[u][rt], x0, bf);
    }
    float sh_ = 0.f, st_ = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const float4 a = *reinterpret_cast<const float4*>(XH + 16 * c + g4);
      const float4 b = *reinterpret_cast<const float4*>(XH + LX + 16 * c + g4);
      sh_ += a.x * bf[4 * c] + a.y * bf[4 * c + 1] + a.z * bf[4 * c + 2] + a.w * bf[4 * c + 3];
      st_ += b.x * bf[4 * c] + b.y * bf[4 * c + 1] + b.z * bf[4 * c + 2] + b.w * bf[4 * c + 3];
    }
    phv[u] = tr2_col_sum(sh_);
    ptv[u] = tr2_col_sum(st_);
  }
  KGE_PROF(34);

  // ---- clip the projected rows (TransR.py:187-189, constraint.py:94-99)
#pragma unroll
  for (int rt = 0; rt < 5; ++rt) {
    if (rt >= nrt) break;
    float x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (has(u)) x[j] += P[u][rt][j] * P[u][rt][j];
    }
    tr2_tile_out<false>(x, rt, red + w0 * NRR);
  }
  {
    float a = 0.f, b = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (has(u) && g0) { a += phv[u] * phv[u]; b += ptv[u] * ptv[u]; }
    a = lane_reduce<3, false>(a);
    b = lane_reduce<3, false>(b);
    if (lane == 0) { red[w0 * NRR + HR] = a; red[w0 * NRR + TR] = b; }
  }
  __syncthreads();
  if (tid < NRR) {
    float s = 0.f;
    for (int w = 0; w < kTrWaves; ++w)
      if (w < nct) s += red[w * NRR + tid];
    const float n = sqrtf(s);
    pn[tid] = n;
    pinv[tid] = (T.clip && !(n < 1.f)) ? 1.f / fmaxf(n, 1e-9f) : 1.f;
  }
  __syncthreads();
#pragma unroll
  for (int rt = 0; rt < 5; ++rt) {
    if (rt >= nrt) break;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float inv = pinv[rt * 16 + g4 + j];   // (1 when the row is not clipped)
#pragma unroll
      for (int u = 0; u < 2; ++u) P[u][rt][j] *= inv;
    }
  }
  {
    const float ih = pinv[HR], it = pinv[TR];
#pragma unroll
    for (int u = 0; u < 2; ++u) { phv[u] *= ih; ptv[u] *= it; }
  }
  // the projected h, t and r (this role's columns) to LDS, re-read after the
  // products that need the registers
  if (g0) {
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (has(u)) {
        phs[colu[u]] = phv[u];
        pts[colu[u]] = ptv[u];
        rrs[colu[u]] = colu[u] < k ? A.rel.row(pr)[colu[u]] : 0.f;
      }
  }
  // (no barrier: phv / ptv are already in every lane -- tr2_col_sum gives
  // them the same bits -- and the LDS copies are read after later barriers)
  float rr[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) rr[u] = (has(u) && colu[u] < k) ? A.rel.row(pr)[colu[u]] : 0.f;
  auto load_rows = [&]() {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      phv[u] = has(u) ? phs[colu[u]] : 0.f;
      ptv[u] = has(u) ? pts[colu[u]] : 0.f;
      rr[u] = has(u) ? rrs[colu[u]] : 0.f;
    }
  };
  // element (row, column tile u): projected x / y rows; scored x = xp + r, y = yp
  // (p = the row's own projected value; the positive's own row is t)
  auto xyp = [&](int u, float p, bool own_y, float& xp, float& yp) {
    xp = own_y ? phv[u] : p;
    yp = own_y ? p : ptv[u];
  };
  auto score_part = [&](float x, float y, float part) {
    if (SK == SK_DOT) return part + x * y;
    const float ma = fabsf(x - y);
    return SK == SK_P2 ? part + ma * ma : SK == SK_P1 ? part + ma
         : SK == SK_PGEN ? part + powf(ma, A.p) : fmaxf(part, ma);
  };

  KGE_PROF(35);
  // ---- scores: s(x, y) per row
#pragma unroll
  for (int rt = 0; rt < 5; ++rt) {
    if (rt >= nrt) break;
    float x4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int kind = rkind(rt * 16 + g4 + j);
      float part = 0.f;
      if (kind >= 0) {
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (!live(u)) continue;
          float xp, yp;
          xyp(u, P[u][rt][j], kind != KIND_HC, xp, yp);
          part = score_part(xp + rr[u], yp, part);
        }
      }
      x4[j] = part;
    }
    tr2_tile_out<SK == SK_PINF>(x4, rt, red + w0 * NRR);
  }
  {
    float part = 0.f;
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (live(u) && g0) part = score_part(phv[u] + rr[u], ptv[u], part);
    part = lane_reduce<3, SK == SK_PINF>(part);
    if (lane == 0) red[w0 * NRR + TR] = part;
  }
  __syncthreads();
  if (tid < NRR) {
    float R = 0.f;
    for (int w = 0; w < kTrWaves; ++w)
      if (w < nct) R = SK == SK_PINF ? fmaxf(R, red[w * NRR + tid]) : R + red[w * NRR + tid];
    sR[tid] = R;
    if (SK != SK_PINF) {
      float lp;
      sS[tid] = score_value<SK>(R, A.pw, &lp, A.p);
      sT[tid] = 1.f;
    }
  }
  __syncthreads();
  if (SK == SK_PINF) {   // ties of the maximum (TF reduce_max splits the gradient evenly)
#pragma unroll
    for (int rt = 0; rt < 5; ++rt) {
      if (rt >= nrt) break;
      float x4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = rt * 16 + g4 + j;
        const int kind = rkind(row);
        float tq = 0.f;
        if (kind >= 0) {
          const float M = sR[row];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            if (!live(u)) continue;
            float xp, yp;
            xyp(u, P[u][rt][j], kind != KIND_HC, xp, yp);
            if (fabsf(xp + rr[u] - yp) == M) tq += 1.f;
          }
        }
        x4[j] = tq;
      }
      tr2_tile_out<false>(x4, rt, red + w0 * NRR);
    }
    {
      float tq = 0.f;
      const float M = sR[TR];
#pragma unroll
      for (int u = 0; u < 2; ++u)
        if (live(u) && g0 && fabsf(phv[u] + rr[u] - ptv[u]) == M) tq += 1.f;
      tq = lane_reduce<3, false>(tq);
      if (lane == 0) red[w0 * NRR + TR] = tq;
    }
    __syncthreads();
    if (tid < NRR) {
      float t = 0.f;
      for (int w = 0; w < kTrWaves; ++w)
        if (w < nct) t += red[w * NRR + tid];
      sT[tid] = t;
      float lp;
      sS[tid] = score_value<SK>(sR[tid], A.pw, &lp, A.p);
    }
    __syncthreads();
  }

  KGE_PROF(36);
  // ---- loss and dL/ds per triple (one wave, IEEE transcendentals)
  if (wv == 0) {
    const float sp = sS[TR];
    const bool sans = A.loss_kind == KGE_LOSS_SANS;
    float Ms = -INFINITY;
    if (sans)
      for (int q = lane; q < K; q += KGE_WAVE) Ms = fmaxf(Ms, A.temperature * sS[q]);
    Ms = wmax(Ms);
    float Z = 0.f;
    if (sans)
      for (int q = lane; q < K; q += KGE_WAVE) Z += expf(A.temperature * sS[q] - Ms);
    Z = wsum(Z);
    const float invZ = sans ? (Z > 0.f ? 1.f / Z : 0.f) : 1.f;
    float lneg = 0.f, csum = 0.f;
    for (int q = lane; q < K; q += KGE_WAVE) {
      const float s = sS[q];
      float lp;
      score_value<SK>(sR[q], A.pw, &lp, A.p);
      const float c = neg_coef(A, s, sp, Ms, invZ);
      sA[q] = score_alpha<SK>(c, sR[q], lp, sT[q], A.pw, A.p);
      csum += c;
      switch (A.loss_kind) {
        case KGE_LOSS_HINGE: lneg += fmaxf(A.margin + s - sp, 0.f); break;
        case KGE_LOSS_LOGISTIC: lneg += logf(1.f + expf(s - sp)); break;
        case KGE_LOSS_BCE: lneg += log_sigmoid(-s); break;
        case KGE_LOSS_SANS: lneg += expf(A.temperature * s - Ms) * invZ * log_sigmoid(-s - A.margin); break;
        default: lneg += s * s; break;
      }
    }
    lneg = wsum(lneg);
    csum = wsum(csum);
    if (lane == 0) {
      float lossp, cp;
      switch (A.loss_kind) {
        case KGE_LOSS_HINGE: lossp = lneg * A.inv_bk; cp = -csum; if (K == 0) lossp = NAN; break;
        case KGE_LOSS_LOGISTIC: lossp = lneg; cp = -csum; break;
        case KGE_LOSS_BCE: lossp = -(log_sigmoid(sp) + lneg) * A.inv_b; cp = -sigmoid(-sp) * A.inv_b; break;
        case KGE_LOSS_SANS:
          lossp = -(log_sigmoid(sp + A.margin) + lneg) * A.inv_b;
          cp = -sigmoid(-(sp + A.margin)) * A.inv_b;
          break;
        default: lossp = ((sp - 1.f) * (sp - 1.f) + lneg) * 0.5f * A.inv_b; cp = (sp - 1.f) * A.inv_b; break;
      }
      float lpp;
      score_value<SK>(sR[TR], A.pw, &lpp, A.p);
      sA[TR] = score_alpha<SK>(cp, sR[TR], lpp, sT[TR], A.pw, A.p);
      misc[0] = lossp;
      if (A.pos_score_out) A.pos_score_out[i] = sp;
    }
  }
  if (A.neg_score_out)
    for (int q = tid; q < K; q += kTrThreads) A.neg_score_out[i * K + q] = sS[q];
  __syncthreads();

  KGE_PROF(37);
  float n_ent = 0.f, n_rel = 0.f, n_proj = 0.f;
  if (A.train) {
    auto grads = [&](float x, float y, float alpha, float Mx, float& gx, float& gy) {
      if (SK == SK_DOT) {
        gx = alpha * y;
        gy = alpha * x;
      } else {
        gx = lp_elem_grad<SK>(x - y, alpha, Mx);
        gy = -gx;
      }
    };
    // ---- pass A: raw slice gradients; per row x . g_x, y . g_y; the relation gradient
    float rs[2] = {0.f, 0.f};
#pragma unroll
    for (int rt = 0; rt < 5; ++rt) {
      if (rt >= nrt) break;
      float vx[4], vy[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = rt * 16 + g4 + j;
        const int kind = rkind(row);
        vx[j] = vy[j] = 0.f;
        if (kind >= 0) {
          const float alpha = sA[row], Mx = SK == SK_PGEN ? A.p : sR[row];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            if (!live(u)) continue;
            float xp, yp, gx, gy;
            xyp(u, P[u][rt][j], kind != KIND_HC, xp, yp);
            grads(xp + rr[u], yp, alpha, Mx, gx, gy);
            n_rel += gx * gx;
            rs[u] += gx;                 // the r-lookup slice is d s / d x
            vx[j] += gx * xp;
            vy[j] += gy * yp;
          }
        }
      }
      tr2_tile_out<false>(vx, rt, red + w0 * NRR);
      tr2_tile_out<false>(vy, rt, red + (kTrWaves + w0) * NRR);
    }
    {   // the positive: x = h + r, y = t
      const float alpha = sA[TR], Mx = SK == SK_PGEN ? A.p : sR[TR];
      float vx = 0.f, vy = 0.f;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        if (!live(u) || !g0) continue;
        float gx, gy;
        grads(phv[u] + rr[u], ptv[u], alpha, Mx, gx, gy);
        n_rel += gx * gx;
        rs[u] += gx;
        vx += gx * phv[u];
        vy += gy * ptv[u];
      }
      vx = lane_reduce<3, false>(vx);
      vy = lane_reduce<3, false>(vy);
      if (lane == 0) { red[w0 * NRR + TR] = vx; red[(kTrWaves + w0) * NRR + TR] = vy; }
    }
    __syncthreads();
    if (tid < NRR) {
      float a = 0.f, b = 0.f;
      for (int w = 0; w < kTrWaves; ++w)
        if (w < nct) { a += red[w * NRR + tid]; b += red[(kTrWaves + w) * NRR + tid]; }
      sdx[tid] = a;
      sdy[tid] = b;
    }
    __syncthreads();
    // the slices back through clip_constraint: Gx (x side), Gy (y side); E = the
    // row's own entity slice, Q = its positive-side slice (for the positive's row
    // TR: E = the t slice, Q = the h slice)
    auto slices = [&](int u, float p, int row, int kind, float& E, float& Q, float& Gx, float& Gy) {
      const bool own_y = kind != KIND_HC;
      const int xr = own_y ? HR : row, yr = own_y ? row : TR;
      float xp, yp, gx, gy;
      xyp(u, p, own_y, xp, yp);
      grads(xp + rr[u], yp, sA[row], SK == SK_PGEN ? A.p : sR[row], gx, gy);
      Gx = (T.clip && !(pn[xr] < 1.f)) ? (gx - sdx[row] * xp) * pinv[xr] : gx;
      Gy = (T.clip && !(pn[yr] < 1.f)) ? (gy - sdy[row] * yp) * pinv[yr] : gy;
      E = own_y ? Gy : Gx;
      Q = own_y ? Gx : Gy;
    };
    // ---- pass B: the slices; S' (this role's columns, accumulator layout) = the
    // negatives' entity slices; the summed h / t slices per column; the rel_proj
    // slice norms ||x_x (x) Gx + x_y (x) Gy||^2 summed element by element
    // (per-row scalars times per-element squares: no row reduction)
    f32x4 SP[2][5];
    float sh[2] = {0.f, 0.f}, st[2] = {0.f, 0.f};
    auto nproj = [&](int row, int kind, float Gx, float Gy) {
      const bool own_y = kind != KIND_HC;
      const float hx = xx[own_y ? HR : row], tx = xx[own_y ? row : TR];
      const float htx = kind == KIND_TC ? xh[row] : kind == KIND_HC ? xt[row] : xh[TR];
      return hx * (Gx * Gx) + tx * (Gy * Gy) + 2.f * htx * (Gx * Gy);
    };
    // The Q rows (negative q's positive-side slice, GEMM2's norm pass) go to
    // LDS as they are computed, over X (dead since GEMM1, several barriers
    // ago): rows without a triple and columns past k as zeros
#pragma unroll
    for (int rt = 0; rt < 5; ++rt) {
#pragma unroll
      for (int u = 0; u < 2; ++u) SP[u][rt] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (rt >= nrt) continue;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = rt * 16 + g4 + j;
        const int kind = rkind(row);
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          if (!has(u)) continue;
          float Q = 0.f;
          if (kind >= 0 && colu[u] < k) {
            float E, Gx, Gy;
            slices(u, P[u][rt][j], row, kind, E, Q, Gx, Gy);
            n_proj += nproj(row, kind, Gx, Gy);
            if (kind != KIND_HC) sh[u] += Q; else st[u] += Q;
            SP[u][rt][j] = E;
          }
          X[row * LX + colu[u]] = Q;
        }
      }
    }
    float qh[2] = {0.f, 0.f}, qt[2] = {0.f, 0.f};
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!live(u) || !g0) continue;
      float E, Q, Gx, Gy;
      slices(u, ptv[u], TR, KIND_POS, E, Q, Gx, Gy);
      n_proj += nproj(TR, KIND_POS, Gx, Gy);
      qh[u] = Q;
      qt[u] = E;
      sh[u] += Q;
      st[u] += E;
    }
    float* gp = A.gpos + i * 3 * (int64_t)A.gcols;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      rs[u] = tr2_col_sum(rs[u]);
      sh[u] = tr2_col_sum(sh[u]);
      st[u] = tr2_col_sum(st[u]);
      if (g0 && has(u)) {
        const bool lv = colu[u] < k;
        if (lv) gp[A.gcols + colu[u]] = rs[u];
        shs[colu[u]] = lv ? sh[u] : 0.f;
        sts[colu[u]] = lv ? st[u] : 0.f;
        qhs[colu[u]] = lv ? qh[u] : 0.f;
        qts[colu[u]] = lv ? qt[u] : 0.f;
      }
    }
    if (tid < W - 16 * nct) {   // (the row vectors' columns past P's tiles)
      const int c = 16 * nct + tid;
      shs[c] = sts[c] = qhs[c] = qts[c] = 0.f;
    }

    KGE_PROF(38);
    // (no barrier: X is dead since GEMM1, several barriers ago; the row vectors
    // written above are read by GEMM2, after the barrier that ends the staging)
    KGE_PROF(39);
    load_rows();
    // (the Q rows were written by pass B)
    {   // (columns past P's tiles: zero, as the S' rows below)
      const int c0 = 16 * nct, wpad = W - c0;
      for (int e = tid; e < NR16 * wpad; e += kTrThreads) X[(e / wpad) * LX + c0 + e % wpad] = 0.f;
    }
    __syncthreads();
    KGE_PROF(44);
    // ---- GEMM2: Y = S M_r^T over the staged rows; job = one 16-column tile of
    // Y (d) over every row tile, M_r^T's column streamed chunk by chunk (two
    // chunks ahead). Two k-vectors ride on the same column (VALU): NORMS = false:
    // S' rows -> gneg[code] (+ norms), the summed h / t slices -> the positive's
    // gradient rows; NORMS = true: ||.||^2 of the Q rows and of the positive's
    // own h / t slices.
    auto gemm2 = [&](auto norms, auto vec4) {
      constexpr bool NORMS = decltype(norms)::value, V4 = decltype(vec4)::value;
      const float* va = NORMS ? qhs : shs;
      const float* vb = NORMS ? qts : sts;
      const int nctd = (d + 15) / 16;
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int mt = w0 + 8 * u;
        if (mt >= nctd) continue;
        const int col = mt * 16 + c16;
        const float* mrow = Mr + (int64_t)(col < d ? col : d - 1) * k;
        // raw loads into a ring three chunks deep; the bounds mask is applied at
        // use (a select right after the load would wait for it)
        auto ldb = [&](int c, float (&b)[4]) {
          const int kk = 16 * c + g4;
          if (V4) {
            const float4 m4 = *reinterpret_cast<const float4*>(mrow + (kk < k ? kk : 0));
            b[0] = m4.x;
            b[1] = m4.y;
            b[2] = m4.z;
            b[3] = m4.w;
          } else {
#pragma unroll
            for (int q = 0; q < 4; ++q) b[q] = mrow[kk + q < k ? kk + q : 0];
          }
        };
        f32x4 acc[5];
#pragma unroll
        for (int rt = 0; rt < 5; ++rt) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
        float ya = 0.f, yb = 0.f;
        float bq[3][4];
        ldb(0, bq[0]);
        if (NC > 1) ldb(1, bq[1]);
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          if (c + 2 < NC) ldb(c + 2, bq[(c + 2) % 3]);
          float4 xa[5];
#pragma unroll
          for (int rt = 0; rt < 5; ++rt)
            if (rt < nrt) xa[rt] = *reinterpret_cast<const float4*>(X + (rt * 16 + c16) * LX + 16 * c + g4);
          const float4 a4 = *reinterpret_cast<const float4*>(va + 16 * c + g4);
          const float4 b4 = *reinterpret_cast<const float4*>(vb + 16 * c + g4);
          // (keep the prefetch two chunks ahead: the occupancy-bound scheduler
          // would otherwise sink each load to its first use)
          __builtin_amdgcn_sched_barrier(0);
          float b[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) b[q] = (16 * c + g4 + q < k && col < d) ? bq[c % 3][q] : 0.f;
          // k step outer, row tile inner: consecutive MFMAs are independent chains
#pragma unroll
          for (int rt = 0; rt < 5; ++rt)
            if (rt < nrt) acc[rt] = mfma16(xa[rt].x, b[0], acc[rt]);
#pragma unroll
          for (int rt = 0; rt < 5; ++rt)
            if (rt < nrt) acc[rt] = mfma16(xa[rt].y, b[1], acc[rt]);
#pragma unroll
          for (int rt = 0; rt < 5; ++rt)
            if (rt < nrt) acc[rt] = mfma16(xa[rt].z, b[2], acc[rt]);
#pragma unroll
          for (int rt = 0; rt < 5; ++rt)
            if (rt < nrt) acc[rt] = mfma16(xa[rt].w, b[3], acc[rt]);
          ya += a4.x * b[0] + a4.y * b[1] + a4.z * b[2] + a4.w * b[3];
          yb += b4.x * b[0] + b4.y * b[1] + b4.z * b[2] + b4.w * b[3];
        }
        ya = tr2_col_sum(ya);
        yb = tr2_col_sum(yb);
        if (col >= d) continue;
        if (g0) {
          if (NORMS) {
            n_ent += ya * ya + yb * yb;
          } else {
            gp[col] = ya;
            gp[2 * A.gcols + col] = yb;
          }
        }
#pragma unroll
        for (int rt = 0; rt < 5; ++rt) {
          if (rt >= nrt) break;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int row = rt * 16 + g4 + q;
            const float v = acc[rt][q];
            if (row < K) {
              n_ent += v * v;
              if (!NORMS) A.gneg[(int64_t)(((uint32_t)i << A.kshift) | (uint32_t)row) * d + col] = v;
            }
          }
        }
      }
    };
    const bool mv4 = (k & 3) == 0 && (T.proj.ld & 3) == 0 && ((uintptr_t)T.proj.p & 15) == 0;
    if (mv4) gemm2(std::true_type{}, std::true_type{});
    else gemm2(std::true_type{}, std::false_type{});
    __syncthreads();   // Q consumed: S' rows over it
    KGE_PROF(40);
    // ---- S' rows to LDS (columns past k and past P's tiles zero)
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (!has(u)) continue;
#pragma unroll
      for (int rt = 0; rt < 5; ++rt) {
        if (rt >= nrt) break;
#pragma unroll
        for (int j = 0; j < 4; ++j) X[(rt * 16 + g4 + j) * LX + colu[u]] = SP[u][rt][j];
      }
    }
    __syncthreads();

    if (mv4) gemm2(std::false_type{}, std::true_type{});
    else gemm2(std::false_type{}, std::false_type{});
    KGE_PROF(43);
    // ---- GEMM3: dM_i = X^T S' + x_h^T (sum of h slices) + x_t^T (sum of t slices)
    // (S' rows in LDS, X re-read from the table: L2; the rank-2 part in the
    // epilogue); job = 16-row tile of dM (its A column in registers) x a pair of
    // column tiles
    {
      auto gemm3 = [&](auto n3c) {
        constexpr int N3 = decltype(n3c)::value;
        const int nrt3 = (d + 15) / 16, nkc = N3 ? N3 : nrt;
        float* dm = T.dmpart + i * (int64_t)d * k;
        const int npc = (nct + 1) / 2, nj = nrt3 * npc;
        const int jb = wv * nj / kTrWaves, je = (wv + 1) * nj / kTrWaves;
        int cur = -1;
        float af[kTrKS3];
        for (int jo = jb; jo < je; ++jo) {
          const int rt = jo / npc, ct = (jo - rt * npc) * 2;
          const int ci = rt * 16 + c16;
          if (rt != cur) {
            cur = rt;
            const int cic = ci < d ? ci : d - 1;
#pragma unroll
            for (int ks = 0; ks < kTrKS3; ++ks) {
              const int kk = ks * 4 + (lane >> 4);
              const float v = A.ent.row(ids[kk < K ? kk : 0])[cic];
              af[ks] = (kk < K && ci < d) ? v : 0.f;
            }
          }
          const int ct1 = ct + 1 < nct ? ct + 1 : ct;
          const bool pair = ct1 != ct;
          f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
          const float* b0 = X + (lane >> 4) * LX + ct * 16 + c16;
          const float* b1 = X + (lane >> 4) * LX + ct1 * 16 + c16;
#pragma unroll
          for (int c = 0; c < kTrKS3 / 4; ++c) {
            if (c < nkc) {
              float y0[4], y1[4];
#pragma unroll
              for (int q = 0; q < 4; ++q) {
                y0[q] = b0[(c * 4 + q) * 4 * LX];
                y1[q] = b1[(c * 4 + q) * 4 * LX];
              }
              if (pair) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  a0 = mfma16(af[c * 4 + q], y0[q], a0);
                  a1 = mfma16(af[c * 4 + q], y1[q], a1);
                }
              } else {   // the odd last column tile alone: two chains, added below
                a0 = mfma16(af[c * 4 + 0], y0[0], a0);
                a1 = mfma16(af[c * 4 + 1], y0[1], a1);
                a0 = mfma16(af[c * 4 + 2], y0[2], a0);
                a1 = mfma16(af[c * 4 + 3], y0[3], a1);
              }
            }
          }
          if (!pair) a0 += a1;
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            if (h == 1 && !pair) break;
            const int col = (h ? ct1 : ct) * 16 + c16;
            if (col >= k) continue;
            const float sgh = shs[col], sgt = sts[col];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int row = rt * 16 + g4 + q;
              if (row < d) dm[(int64_t)row * k + col] = (h ? a1 : a0)[q] + XH[row] * sgh + XH[LX + row] * sgt;
            }
          }
        }
      };
      if (NRT) gemm3(std::integral_constant<int, NRT>{});   // (straight-line chunk loop)
      else gemm3(std::integral_constant<int, 0>{});
    }
    KGE_PROF(41);
    // ---- destination keys for the update pass
    for (int q = tid; q < K; q += kTrThreads) bin_key(A, ids[q], ((uint32_t)i << A.kshift) | (uint32_t)q);
    if (tid < 3) {
      const int64_t dest = tid == 0 ? ph : tid == 1 ? pt : A.ent.rows + pr;
      bin_key(A, dest, A.nkeyneg + ((uint32_t)i << 2) + (uint32_t)tid);
    }
  }
  if (err) set_status(A.status, err);
  KGE_PROF(42);

  // ---- partials: loss, ||g||^2 per variable (0 ent, 1 rel_emb, 2 rel_proj);
  // the last workgroup reduces them in a fixed order
  n_ent = wsum(n_ent);
  n_rel = wsum(n_rel);
  n_proj = wsum(n_proj);
  if (lane == 0) { s_w[wv][0] = n_ent; s_w[wv][1] = n_rel; s_w[wv][2] = n_proj; }
  __syncthreads();
  if (tid == 0) {
    float acc[5] = {misc[0], 0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < kTrWaves; ++w) {
      acc[1] += s_w[w][0];
      acc[2] += s_w[w][1];
      acc[3] += s_w[w][2];
    }
#pragma unroll
    for (int c = 0; c < 5; ++c)
      __hip_atomic_store(&A.part[(int64_t)blockIdx.x * 8 + c], acc[c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_s_waitcnt(0);
    const uint32_t prev = __hip_atomic_fetch_add(&A.ctl->score_ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = prev == (uint32_t)(gridDim.x - 1);
  }
  __syncthreads();
  if (s_last && wv == 0) {
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = lane; w < (int)gridDim.x; w += KGE_WAVE) {
#pragma unroll
      for (int c = 0; c < 5; ++c)
        acc[c] += __hip_atomic_load(&A.part[(int64_t)w * 8 + c], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int c = 0; c < 5; ++c) acc[c] = wsum(acc[c]);
    if (lane == 0) {
      A.loss_out[0] = acc[0];
      if (A.loss_accum) A.loss_accum[0] += acc[0];
      A.ctl->loss = acc[0];
      A.ctl->score_ticket = 0u;
      A.ctl->ovf_len = __hip_atomic_exchange(&A.ctl->ovf_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        A.ctl->scale[v] = -A.lr * (A.clip_norm / fmaxf(sqrtf(acc[1 + v]), A.clip_norm));
        if (A.norm2_out) A.norm2_out[v] = acc[1 + v];
      }
    }
  }
}

template <int SK>
void launch_transr2(const StepArgs& A, const TrArgs& T, hipStream_t st) {
  const dim3 grid((unsigned)A.B), blk(kTrThreads);
  const Tr2Lds L = tr2_lds(T.d, T.k, A.Keff);
  const size_t lds = (size_t)L.total_floats * 4;
  auto go = [&](auto nrt) {
    constexpr int R = decltype(nrt)::value;
    switch (L.NC) {
      case 4: hipLaunchKernelGGL((transr2_kernel<SK, 4, R>), grid, blk, lds, st, A, T); break;
      case 8: hipLaunchKernelGGL((transr2_kernel<SK, 8, R>), grid, blk, lds, st, A, T); break;
      case 13: hipLaunchKernelGGL((transr2_kernel<SK, 13, R>), grid, blk, lds, st, A, T); break;
      default: hipLaunchKernelGGL((transr2_kernel<SK, 16, R>), grid, blk, lds, st, A, T); break;
    }
  };
  switch (L.NR16 >> 4) {   // (K <= kTrMaxSlots - 1: at most five row tiles)
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 3: go(std::integral_constant<int, 3>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    default: go(std::integral_constant<int, 5>{}); break;
  }
}

}  // namespace kge
