// KS, pipelined form (score_pipe_kernel): the score pass of
// KGEModel.__run_single_batch (BaseModel.py:316-327) for the element-wise
// models whose row fits one fragment chunk (TransE, d <= 256) -- the same
// arithmetic as score_kernel (kge_step_impl.h), organised so that a
// positive's non-streaming work runs under the next positive's row stream.
//
// score_kernel gives each workgroup nP positives at once; all 512 workgroups
// of C2 are resident together, stream together, and then all spend ~20 us
// per workgroup in phases that read nothing (the merge barrier's wait for
// the slowest wave, softmax merge, coefficients, key filing, partials).
// Here one 16-wave workgroup per CU walks its run of positives in order, and
// EVERY wave streams a share (SW <= 64 slots) of EVERY positive:
//
//   for n in 0 .. np-1:
//     S(n)   stream the wave's slots of positive n (gather, forward, one
//            transposed reduction per row batch, SANS softmax online,
//            backward into the wave's accumulators) -- score_kernel's loop
//     the next positive's context rows and draws issued
//     state(n) -> LDS buffer n % 2, one arrival on an LDS counter
//     T(n-1) the previous positive's tail, by every wave for its own share:
//            merged softmax state (every wave merges the 16 headers itself),
//            its slots' coefficients, loss terms and destination keys, its
//            1/16 of the positive's row gradients (gpos), the designated
//            wave's positive keys
//   T(np-1)
//
// A wave waits only when another wave of its workgroup is a whole positive
// behind (buffer (n-1) % 2's arrivals before T(n-1); its tails of n-2 done
// before it overwrites buffer n % 2). Per-wave partials (loss, clip norms)
// are summed in wave order, then across workgroups by the last one, so the
// step stays bit-reproducible run to run (test_fused_step_deterministic).
#pragma once
// (included by kge_step_impl.h inside namespace kge)

constexpr int kPipeWaves = 16;
constexpr int kPipeThreads = kPipeWaves * KGE_WAVE;
constexpr int kPipeMaxSW = KGE_WAVE;   // slots per wave per positive: one lane each in the tail

// LDS layout (bytes): per buffer b in {0, 1} (positive n uses n % 2)
//   img  [2][NW][NI][cols]  the waves' accumulator images
//   hdr  [2][NW][8]         Mrun, Z, hinge / logistic weight sum, norm^2 x4, -
//   ph   [2][16]            the positive's Rp, ties, s, lp, own norm^2 x4, |r|^2
//   posg [2][3][cols]       its own gradient rows at unit alpha
//   gr, gt [2][Keff]        per slot: reduced value, ties (read back by the slot's own wave only)
//   pos  [np][3] int64      the run's triples (table rows)
//   cnt  [4] u32            per buffer: arrivals, tails done (monotonic within the
//                           launch; a counter per buffer, since one wave may be a
//                           positive ahead of another: a single arrival count would
//                           let its two arrivals stand in for a slower wave's one)
//   red  [NW][8]            per-wave partials at the end
struct PipeLds {
  int img, hdr, ph, posg, gr, gt, pos, cnt, red, total;
};
__host__ __device__ inline PipeLds pipe_lds(int cols, int NI, int Keff, int ppw) {
  PipeLds L;
  int o = 0;
  L.img = o;  o += lds_align16(2 * kPipeWaves * NI * cols * 4);
  L.hdr = o;  o += lds_align16(2 * kPipeWaves * 8 * 4);
  L.ph = o;   o += lds_align16(2 * 16 * 4);
  L.posg = o; o += lds_align16(2 * 3 * cols * 4);
  L.gr = o;   o += lds_align16(2 * Keff * 4);
  L.gt = o;   o += lds_align16(2 * Keff * 4);
  L.pos = o;  o += lds_align16(ppw * 3 * 8);
  L.cnt = o;  o += 16;
  L.red = o;  o += lds_align16(kPipeWaves * 8 * 4);
  L.total = o;
  return L;
}

template <class M, class = void> struct pipe_ok { static constexpr bool v = false; };
template <class M> struct pipe_ok<M, std::void_t<decltype(M::PIPE)>> { static constexpr bool v = M::PIPE; };

__device__ __forceinline__ void pipe_wait(const uint32_t* c, uint32_t target) {
  while (__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < target) __builtin_amdgcn_s_sleep(1);
}
__device__ __forceinline__ void pipe_signal(uint32_t* c) {
  // (every lane's LDS stores of this wave precede the release)
  if (lane_id() == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <template <int, int, int> class Model, int VEC, int SK, int SIDE>
__global__ __launch_bounds__(kPipeThreads) __attribute__((amdgpu_waves_per_eu(KGE_SCORE_WPE)))
void score_pipe_kernel(StepArgs A) {
  using M = Model<VEC, 1, SK>;
  using F = Frag<VEC, 1>;
  constexpr int NW = kPipeWaves;
  constexpr int NI = rec_img<M>::n;   // 2: h, t images (r = h - t); 3: h, r, t
  constexpr int ROWS = KGE_STREAM_ROWS > 1 ? KGE_STREAM_ROWS : 2;
  constexpr int SH = ROWS == 16 ? 2 : ROWS == 8 ? 3 : ROWS == 4 ? 4 : 5;
  constexpr int LPR = 1 << SH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ int s_last;

  const int cols = A.ent.cols, Keff = A.Keff, SW = A.pipe_sw, ppw = A.pipe_ppw;
  const PipeLds L = pipe_lds(cols, NI, Keff, ppw);
  float* s_img = reinterpret_cast<float*>(smem + L.img);
  float* s_hdr = reinterpret_cast<float*>(smem + L.hdr);
  float* s_ph = reinterpret_cast<float*>(smem + L.ph);
  float* s_posg = reinterpret_cast<float*>(smem + L.posg);
  float* s_gr = reinterpret_cast<float*>(smem + L.gr);
  float* s_gt = reinterpret_cast<float*>(smem + L.gt);
  int64_t* s_pos = reinterpret_cast<int64_t*>(smem + L.pos);
  uint32_t* s_cnt = reinterpret_cast<uint32_t*>(smem + L.cnt);
  float* s_red = reinterpret_cast<float*>(smem + L.red);

  if (ws_refused(A.ctl, A.sig, A.status, A.loss_out)) return;
  const int tid = threadIdx.x, lane = lane_id(), wv = wave_id();
  int err = 0;
  const int64_t p0 = (int64_t)blockIdx.x * ppw;
  const int np = (int)min<int64_t>((int64_t)ppw, A.B - p0);

  // the run's triples as table rows, once
  for (int e = tid; e < 3 * np; e += kPipeThreads) {
    int64_t x = load_idx(A.pos, (p0 + e / 3) * 3 + e % 3, A.i64);
    if (e % 3 == 1) { if (x < 0 || x >= A.rel.rows) { err = KGE_ERANGE; x = 0; } }
    else x = ent_row(A, x, &err);
    s_pos[e] = x;
  }
  if (tid < 4) s_cnt[tid] = 0u;
  __syncthreads();

  const int jbeg = min(Keff, wv * SW), jend = min(Keff, jbeg + SW);
  const int lrow = lane >> SH;
  const bool lead = (lane & (LPR - 1)) == 0;
  constexpr bool RAW = M::NRM_FROM_R;
  const bool lane_in = lane * VEC < cols;
  // this wave's loss weight for its negatives' summed loss terms (loss.py)
  float wl;
  switch (A.loss_kind) {
    case KGE_LOSS_HINGE: wl = A.inv_bk; break;
    case KGE_LOSS_LOGISTIC: wl = 1.f; break;
    case KGE_LOSS_SANS: case KGE_LOSS_BCE: wl = -A.inv_b; break;
    default: wl = 0.5f * A.inv_b; break;
  }
  float part_loss = 0.f, part_n[4] = {0.f, 0.f, 0.f, 0.f};

  // ---- per positive: draws (lane l: slot jbeg + l) and context rows
  auto draw = [&](int n) -> int32_t {
    const int j = jbeg + lane;
    return j < jend ? slot_entity(A, p0 + n, j, &err) : 0;
  };
  typename M::Ctx ctx;
  const MP mp{A.limit, A.fuse_norm, nullptr};
  auto load_ctx_raw = [&](int n) {   // (M::ctx_finish completes it)
    M::load_ctx_raw(ctx, A.ent, A.rel, s_pos[3 * n], s_pos[3 * n + 1], s_pos[3 * n + 2]);
  };
  int32_t idv = np > 0 ? draw(0) : 0;   // the current positive's slot ids (one per lane)
  int32_t idp = 0;                       // the previous positive's (its tail files their keys)
  if (np > 0) {
    load_ctx_raw(0);
    M::ctx_finish(ctx, mp);
  }

  // ---- the tail of positive m (buffer m % 2), this wave's share
  auto tail = [&](int m) {
    const int b = m & 1;
    const int64_t i = p0 + m;
    pipe_wait(&s_cnt[b], (uint32_t)(NW * (m / 2 + 1)));   // every wave's state(m) is in
    // merged softmax state of the positive (every wave merges the headers itself)
    const float* hd = s_hdr + b * NW * 8;
    const float* ph = s_ph + b * 16;
    const bool sans = A.loss_kind == KGE_LOSS_SANS;
    const float hM = lane < NW ? hd[lane * 8] : -INFINITY;
    const float Ms = wave_max(hM);
    const float fl = lane < NW ? (!sans ? 1.f : (hM == -INFINITY ? 0.f : expf(hM - Ms))) : 0.f;
    const float Z = wave_sum(lane < NW ? hd[lane * 8 + 1] * fl : 0.f);
    const float cw = wave_sum(lane < NW ? hd[lane * 8 + 3] : 0.f);
    const float invZ = sans ? (Z > 0.f ? 1.f / Z : 0.f) : 1.f;
    const float Rpv = ph[0], tpv = ph[1], spv = ph[2], lppv = ph[3];
    float lossp, cp;
    switch (A.loss_kind) {
      case KGE_LOSS_HINGE: lossp = 0.f; cp = -cw; if (Keff == 0) lossp = NAN; break;   // (loss.py:81-82)
      case KGE_LOSS_LOGISTIC: lossp = 0.f; cp = -cw; break;
      case KGE_LOSS_BCE: lossp = -log_sigmoid(spv) * A.inv_b; cp = -sigmoid(-spv) * A.inv_b; break;
      case KGE_LOSS_SANS:
        lossp = -log_sigmoid(spv + A.margin) * A.inv_b;
        cp = -sigmoid(-(spv + A.margin)) * A.inv_b;
        break;
      default:
        lossp = (spv - 1.f) * (spv - 1.f) * 0.5f * A.inv_b;
        cp = (spv - 1.f) * A.inv_b;
        break;
    }
    const float ap = score_alpha<SK>(cp, Rpv, lppv, tpv, A.pw, A.p);
    // this wave's slots: loss terms, coefficient, score, destination key
    float lfin = 0.f;
    {
      const int j = jbeg + lane;
      if (j < jend) {
        const float* gr = s_gr + b * Keff;
        const float* gt = s_gt + b * Keff;
        const float R = gr[j];
        float lp;
        const float s = score_value<SK>(R, A.pw, &lp, A.p);
        switch (A.loss_kind) {
          case KGE_LOSS_HINGE: lfin = fmaxf(A.margin + s - spv, 0.f); break;
          case KGE_LOSS_LOGISTIC: lfin = logf(1.f + expf(s - spv)); break;
          case KGE_LOSS_BCE: lfin = log_sigmoid(-s); break;
          case KGE_LOSS_SANS: lfin = expf(A.temperature * s - Ms) * invZ * log_sigmoid(-s - A.margin); break;
          default: lfin = s * s; break;
        }
        if (A.neg_score_out) A.neg_score_out[i * Keff + j] = s;
        if (A.train) {
          const float c = neg_coef(A, s, spv, Ms, invZ);
          const uint32_t code = ((uint32_t)i << A.kshift) | (uint32_t)j;
          A.coef[code] = make_float2(score_alpha<SK>(c, R, lp, gt[j], A.pw, A.p), SK == SK_PGEN ? A.p : R);
          bin_key(A, idp, code);
        }
      }
    }
    part_loss += wl * wave_sum(lfin);
    // this wave's share of the positive's row gradients [3, cols] (gpos)
    if (A.train) {
      const int tot = 3 * A.gcols;
      const int per = (tot + NW - 1) / NW;
      const int e = wv * per + lane;
      if (lane < per && e < tot) {
        const int v = e / A.gcols, k = e - v * A.gcols;
        const int vc = v == 1 ? A.rel_gcols : cols;
        if (k < vc) {
          const float* img = s_img + b * NW * NI * cols;
          float s = ap * s_posg[(b * 3 + v) * cols + k];
          for (int w = 0; w < NW; ++w) {
            const float fw = bcast(fl, w) * invZ;   // (header w's softmax factor, lane w's)
            const float* iw = img + w * NI * cols;
            float x;
            if constexpr (NI == 2) x = v == 0 ? iw[k] : v == 2 ? iw[cols + k] : iw[k] - iw[cols + k];
            else x = iw[v * cols + k];
            s += fw * x;
          }
          if (v == 1 && A.rel_reg != 0.f)
            s += (A.rel_reg * A.inv_b) * (2.f * A.rel.row(s_pos[3 * m + 1])[k]);
          A.gpos[i * 3 * (int64_t)A.gcols + v * (int64_t)A.gcols + k] = s;
        }
      }
    }
    // the designated wave: the positive's own loss, clip-norm terms and keys
    if (wv == m % NW) {
      float n[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float hv = lane < NW ? hd[lane * 8 + 4 + v] * (fl * invZ) * (fl * invZ) : 0.f;
        n[v] = ap * ap * ph[4 + v] + wave_sum(hv);
      }
      float lpos = lossp;
      if (A.rel_reg != 0.f) {   // DistMult: lambda * mean_i ||r_i||^2, its own IndexedSlices block
        const float gsc = A.rel_reg * A.inv_b;
        lpos += ph[8] * gsc;
        n[1] += 4.f * gsc * gsc * ph[8];
      }
      part_loss += lpos;
#pragma unroll
      for (int v = 0; v < 4; ++v) part_n[v] += n[v];
      if (A.train && lane < 3 && (A.rel_dests || lane != 2)) {
        const int64_t dest = lane == 0 ? s_pos[3 * m] : lane == 1 ? s_pos[3 * m + 2] : A.ent.rows + s_pos[3 * m + 1];
        bin_key(A, dest, A.nkeyneg + (((uint32_t)i) << 2) + (uint32_t)lane);
      }
    }
    pipe_signal(&s_cnt[2 + b]);
  };

  for (int n = 0; n <= np; ++n) {
    if (n == np) {   // (one tail call site: the last positive's tail)
      if (np > 0) tail(np - 1);
      break;
    }
    const int b = n & 1;
    const int64_t i = p0 + n;
    float* gR = s_gr + b * Keff;
    float* gT = s_gt + b * Keff;
    // the positive's score, in every wave (hinge / logistic weights need it)
    float Rp, tp = 1.f, sp, lpp = 0.f;
    {
      F a, bb, E0;
      E0.zero();
      M::fwd(ctx, KIND_POS, E0, a, bb);
      Rp = lane_reduce<5, SK == SK_PINF>(score_partial<SK, M::CPLX>(a, bb, A.p));
      if (SK == SK_PINF) tp = lane_reduce<5, false>(tie_partial<M::CPLX>(a, Rp));
      sp = score_value<SK>(Rp, A.pw, &lpp, A.p);
    }
    float Mrun = -INFINITY, Zs = 0.f, csum = 0.f;
    float nrm[4] = {0.f, 0.f, 0.f, 0.f};
    F accH, accR, accT;
    accH.zero(); accR.zero(); accT.zero();
    // ---- S(n): score_kernel's stream over [jbeg, jend) (every row's load
    // issued before any is used; rows past the range repeat the last one)
    auto stream = [&](auto lkc) {
      constexpr int LK = decltype(lkc)::value;
      const int lk = LK >= 0 ? LK : A.loss_kind;
      for (int j0 = jbeg; j0 < jend; j0 += ROWS) {
        const int nrow = min(ROWS, jend - j0);
        const int jo = j0 - jbeg;
        F E[ROWS];
#pragma unroll
        for (int u = 0; u < ROWS; ++u) {
          const float* row = A.ent.row(__builtin_amdgcn_readlane(idv, jo + min(u, nrow - 1)));
          if (RAW) load_row_raw(E[u], row, cols);
          else load_row(E[u], row, cols);
        }
        if (A.fuse_norm) {
          float sq[ROWS];
#pragma unroll
          for (int u = 0; u < ROWS; ++u) sq[u] = (!RAW || lane_in) ? norm_partial(E[u]) : 0.f;
          const float inv = inv_norm(multi_reduce<ROWS, false>(sq));
#pragma unroll
          for (int u = 0; u < ROWS; ++u) scale_row(E[u], bcast(inv, u << SH));
        }
        F a[ROWS], bb[ROWS];
        float part[ROWS];
        static_for<ROWS>([&](auto uc) {
          constexpr int u = decltype(uc)::value;
          M::template fwdk<kind_at<SIDE>(u)>(ctx, E[u], a[u], bb[u]);
          float pu;
          if constexpr (M::FAST_STREAM) pu = M::template fast_partial<SK>(a[u], bb[u]);
          else pu = score_partial<SK, M::CPLX>(a[u], bb[u], A.p);
          part[u] = (u < nrow && (!RAW || lane_in)) ? pu : 0.f;
        });
        const float Rl = multi_reduce<ROWS, SK == SK_PINF>(part);
        float tl = 1.f;
        if constexpr (SK == SK_PINF) {
          float tq[ROWS];
#pragma unroll
          for (int u = 0; u < ROWS; ++u) tq[u] = u < nrow ? tie_partial<M::CPLX>(a[u], bcast(Rl, u << SH)) : 0.f;
          tl = multi_reduce<ROWS, false>(tq);
        }
        const int j = j0 + lrow;
        const bool valid = lrow < nrow;
        float lp;
        const float s = score_value_fast<SK>(Rl, A.pw, &lp, A.p);
        float c = 0.f;
        switch (lk) {
          case KGE_LOSS_HINGE: {
            float lpi;
            const float si = score_value<SK>(Rl, A.pw, &lpi, A.p);
            c = (A.margin + si - sp >= 0.f) ? A.inv_bk : 0.f;
            if (valid && lead) csum += c;
          } break;
          case KGE_LOSS_LOGISTIC: {
            const float ex = fast_exp(s - sp);
            c = ex * __builtin_amdgcn_rcpf(1.f + ex);
            if (valid && lead) csum += c;
          } break;
          case KGE_LOSS_BCE:
            c = fast_sigmoid(s) * A.inv_b;
            break;
          case KGE_LOSS_SANS: {
            const float z = valid ? A.temperature * s : -INFINITY;
            const float Mn = fmaxf(Mrun, lane_reduce<5, true>(z));
            if (Mn > Mrun) {   // wave-uniform: rescale everything accumulated so far
              const float sc = (Mrun == -INFINITY) ? 0.f : fast_exp(Mrun - Mn);
              const float sc2 = sc * sc;
#pragma unroll
              for (int q = 0; q < VEC; ++q) { accH.v[q] *= sc; accR.v[q] *= sc; accT.v[q] *= sc; }
#pragma unroll
              for (int v = 0; v < 4; ++v) nrm[v] *= sc2;
              Zs *= sc;
              Mrun = Mn;
            }
            const float e = valid ? fast_exp(z - Mrun) : 0.f;
            c = e * fast_sigmoid(s + A.margin) * A.inv_b;
            if (valid && lead) Zs += e;
          } break;
          default:  // SQERR
            c = s * A.inv_b;
            break;
        }
        const float al = valid ? score_alpha_fast<SK>(c, Rl, lp, tl, A.pw, A.p) : 0.f;
        if (valid && lead) {
          gR[j] = Rl;
          gT[j] = tl;
          if (M::NRM_FROM_R) {
            const float n2 = al * al * Rl;
            nrm[0] += 2.f * n2;
            nrm[1] += n2;
          }
        }
        static_for<ROWS>([&](auto uc) {
          constexpr int u = decltype(uc)::value;
          const float alu = bcast(al, u << SH);
          const float Mu = SK == SK_PINF ? bcast(Rl, u << SH) : SK == SK_PGEN ? A.p : 0.f;
          M::template bwdk<kind_at<SIDE>(u)>(ctx, E[u], a[u], bb[u], alu, Mu, accH, accR, accT, nrm, mp);
        });
      }
    };
    if (A.loss_kind == KGE_LOSS_SANS) stream(std::integral_constant<int, KGE_LOSS_SANS>{});
    else stream(std::integral_constant<int, -1>{});
    M::finish(accH, accR, accT);

    // ---- state(n) -> buffer b, once every tail of n - 2 has read it
    if (n >= 2) pipe_wait(&s_cnt[2 + b], (uint32_t)(NW * (n / 2)));   // every tail of n - 2 is done
    {
      const float Zw = wave_sum(Zs), cw = wave_sum(csum);
      float nw[4];
#pragma unroll
      for (int v = 0; v < 4; ++v) nw[v] = wave_sum(nrm[v]);
      float* hd = s_hdr + (b * NW + wv) * 8;
      if (lane == 0) {
        hd[0] = Mrun; hd[1] = Zw; hd[2] = 0.f; hd[3] = cw;
        hd[4] = nw[0]; hd[5] = nw[1]; hd[6] = nw[2]; hd[7] = nw[3];
      }
      if (A.train && lane_in) {
        float* img = s_img + (b * NW + wv) * NI * cols;
        const int e0 = lane * VEC;
#pragma unroll
        for (int q = 0; q < VEC; ++q) {
          if (NI == 2) {
            img[e0 + q] = accH.v[q];
            img[cols + e0 + q] = accT.v[q];
          } else {
            img[e0 + q] = accH.v[q];
            img[cols + e0 + q] = accR.v[q];
            img[2 * cols + e0 + q] = accT.v[q];
          }
        }
      }
    }
    // the designated wave: the positive's own gradient at unit alpha, its
    // context rows for the update kernel, its score
    if (wv == n % NW) {
      F pH, pR, pT;
      float pn[4] = {0.f, 0.f, 0.f, 0.f};
      pH.zero(); pR.zero(); pT.zero();
      if (A.train) {
        F a, bb, E0;
        E0.zero();
        M::fwd(ctx, KIND_POS, E0, a, bb);
        M::bwd(ctx, KIND_POS, E0, a, bb, 1.f, SK == SK_PGEN ? A.p : Rp, pH, pR, pT, pn, mp);
        M::write_snap(ctx, A.snap + i * (M::NSNAP * (int64_t)A.snap_cols), A.snap_cols);
        if (lane_in) {
          float* pg = s_posg + b * 3 * cols;
          const int e0 = lane * VEC;
#pragma unroll
          for (int q = 0; q < VEC; ++q) {
            pg[e0 + q] = pH.v[q];
            pg[cols + e0 + q] = pR.v[q];
            pg[2 * cols + e0 + q] = pT.v[q];
          }
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) pn[v] = wave_sum(pn[v]);
      float rsq = 0.f;
      if (A.rel_reg != 0.f) {
        F Rr;
        load_row(Rr, A.rel.row(s_pos[3 * n + 1]), A.rel.cols);
        rsq = wave_sum(sq_partial(Rr));
      }
      if (lane == 0) {
        float* ph = s_ph + b * 16;
        ph[0] = Rp; ph[1] = tp; ph[2] = sp; ph[3] = lpp;
        ph[4] = pn[0]; ph[5] = pn[1]; ph[6] = pn[2]; ph[7] = pn[3]; ph[8] = rsq;
        if (A.pos_score_out) A.pos_score_out[i] = sp;
      }
    }
    pipe_signal(&s_cnt[b]);
    // the next positive's draws and context rows in flight under the tail
    const int32_t id_n = idv;
    if (n + 1 < np) {
      idv = draw(n + 1);
      load_ctx_raw(n + 1);
    }
    if (n >= 1) tail(n - 1);   // (its keys: idp, the ids of n - 1)
    idp = id_n;
    if (n + 1 < np) M::ctx_finish(ctx, mp);
  }
  if (err) set_status(A.status, err);

  // ---- workgroup partials in wave order; the last workgroup reduces them
  // in workgroup order and publishes the clip scales and the loss
  if (lane == 0) {
    s_red[wv * 8 + 0] = part_loss;
#pragma unroll
    for (int v = 0; v < 4; ++v) s_red[wv * 8 + 1 + v] = part_n[v];
  }
  __syncthreads();
  if (tid == 0) {
    float acc[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
    for (int w = 0; w < NW; ++w)
#pragma unroll
      for (int k = 0; k < 5; ++k) acc[k] += s_red[w * 8 + k];
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
      if (A.loss_accum) A.loss_accum[0] += acc[0];
      A.ctl->loss = acc[0];
      A.ctl->score_ticket = 0u;
      A.ctl->ovf_len = __hip_atomic_exchange(&A.ctl->ovf_count, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&A.ctl->score_pending, A.mark_pending ? A.sig : 0u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        A.ctl->scale[v] = -A.lr * (A.clip_norm / fmaxf(sqrtf(acc[1 + v]), A.clip_norm));
        if (A.norm2_out) A.norm2_out[v] = acc[1 + v];
      }
    }
  }
}
