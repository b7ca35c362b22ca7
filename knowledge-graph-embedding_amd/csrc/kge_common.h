// Device-side building blocks shared by the KGE kernels (gfx950 / CDNA4).
//
//  * Philox4x32-10 counter-based generator + the TF UniformDistribution
//    mapping (bits % range) used by the negative samplers.
//  * wave64 reductions.
//  * Row fragments: a table row of `cols` floats is spread over the 64 lanes
//    of ONE wave, lane l holding elements [(c*64 + l)*VEC, +VEC) for chunk
//    c < NC; VEC = 4 gives one 16-byte load per lane per chunk, i.e. a whole
//    800-byte row (d = 200) per wave-instruction.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/kge_hip.h"

#define KGE_WAVE 64

namespace kge {

// ---------------------------------------------------------------- Philox
struct PhiloxKey { uint32_t k0, k1; };

__device__ __forceinline__ uint4 philox4x32_10(uint4 c, PhiloxKey k) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    if (r) { k.k0 += 0x9E3779B9u; k.k1 += 0xBB67AE85u; }
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = make_uint4(hi1 ^ c.y ^ k.k0, lo1, hi0 ^ c.w ^ k.k1, lo0);
  }
  return c;
}

// Draw n of counter plane `plane`: uniform integer in [0, range).
// int32 ids: 4 draws per Philox block (bits = word q, 32-bit modulo);
// int64 ids: 2 draws per block (bits = w[2q] | w[2q+1] << 32, 64-bit modulo).
__device__ __forceinline__ uint64_t philox_draw(PhiloxKey key, uint64_t plane, uint64_t n,
                                                bool i64, uint64_t range) {
  const uint64_t per = i64 ? 2 : 4;
  const uint64_t b = n / per;
  const uint32_t q = (uint32_t)(n % per);
  const uint4 w = philox4x32_10(make_uint4((uint32_t)b, (uint32_t)(b >> 32),
                                           (uint32_t)plane, (uint32_t)(plane >> 32)), key);
  if (i64) {
    const uint64_t bits = q == 0 ? ((uint64_t)w.x | ((uint64_t)w.y << 32))
                                 : ((uint64_t)w.z | ((uint64_t)w.w << 32));
    return bits % range;
  }
  const uint32_t bits = q == 0 ? w.x : q == 1 ? w.y : q == 2 ? w.z : w.w;
  return (uint64_t)(bits % (uint32_t)range);
}

// Sampler view shared by the standalone sampler and the fused step.
struct SamplerView {
  int32_t kind;
  bool i64;
  PhiloxKey key;
  uint64_t offset;
  int64_t n_entities;
  const void* pool;
  const int32_t* ent_type;
  const int32_t* type_offsets;
  const int32_t* type_members;
  const int32_t* pos_in_type;
};

__host__ inline SamplerView make_sampler_view(const kge_sampler_desc& s) {
  SamplerView v;
  v.kind = s.kind;
  v.i64 = s.idx_dtype == KGE_IDX_I64;
  v.key.k0 = (uint32_t)s.seed;
  v.key.k1 = (uint32_t)(s.seed >> 32);
  v.offset = s.offset;
  v.n_entities = s.n_entities;
  v.pool = s.pool;
  v.ent_type = s.ent_type;
  v.type_offsets = s.type_offsets;
  v.type_members = s.type_members;
  v.pos_in_type = s.pos_in_type;
  return v;
}

__device__ __forceinline__ int64_t load_idx(const void* p, int64_t i, bool i64) {
  return i64 ? ((const int64_t*)p)[i] : (int64_t)((const int32_t*)p)[i];
}
__device__ __forceinline__ void store_idx(void* p, int64_t i, int64_t v, bool i64) {
  if (i64) ((int64_t*)p)[i] = v; else ((int32_t*)p)[i] = (int32_t)v;
}

// One negative entity for reference entity `x` (the entity being replaced),
// draw n of plane `plane`. Returns -1 and sets *err for a singleton type
// (np.random.choice on an empty pool raises, utils.py:11-16).
__device__ __forceinline__ int64_t sample_entity(const SamplerView& s, uint64_t plane, uint64_t n,
                                                 int64_t x, int* err) {
  if (s.kind == KGE_SAMPLER_UNIFORM) {
    const uint64_t k = philox_draw(s.key, plane, n, s.i64, (uint64_t)s.n_entities);
    return s.pool ? load_idx(s.pool, (int64_t)k, s.i64) : (int64_t)k;
  }
  // typed: uniform over type2inds[ind2type[x]] minus x (utils.py:12-14)
  const int32_t ty = s.ent_type[x];
  const int32_t beg = s.type_offsets[ty], cnt = s.type_offsets[ty + 1] - beg;
  if (cnt <= 1) { *err = KGE_EINVAL; return -1; }
  uint64_t k = philox_draw(s.key, plane, n, s.i64, (uint64_t)(cnt - 1));
  if ((int64_t)k >= s.pos_in_type[x]) ++k;
  return s.type_members[beg + k];
}

// ---------------------------------------------------------------- waves
__device__ __forceinline__ int lane_id() { return threadIdx.x & (KGE_WAVE - 1); }
// wave index as a scalar (SGPR): everything derived from it stays wave-uniform,
// so per-wave bounds compile to scalar branches, not exec-mask divergence
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x / KGE_WAVE); }

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, KGE_WAVE);
  return x;
}
__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, KGE_WAVE));
  return x;
}

// ------------------------------------------------------------ cross-lane
// Lane pairings used by the reductions. Bits 5 and 4 go through the gfx950
// half-exchange instructions (v_permlane32_swap / v_permlane16_swap); bits
// 3..0 through DPP: row_mirror (l ^ 15), row_half_mirror (l ^ 7),
// quad_perm [2,3,0,1] (l ^ 2), quad_perm [1,0,3,2] (l ^ 1). Each pairing
// flips lane bit B, and together they span all 64 lanes.
template <int B> struct PairCtl;
template <> struct PairCtl<3> { static constexpr int v = 0x140; };
template <> struct PairCtl<2> { static constexpr int v = 0x141; };
template <> struct PairCtl<1> { static constexpr int v = 0x4E; };
template <> struct PairCtl<0> { static constexpr int v = 0xB1; };

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
template <bool MAX>
__device__ __forceinline__ float comb(float a, float b) { return MAX ? fmaxf(a, b) : a + b; }

// half exchange across lane bit B (5 or 4): lo = a with the high side's a
// moved in, hi = b with the low side's b moved in (v_permlane{32,16}_swap)
template <int B>
__device__ __forceinline__ void half_swap(float a, float b, float& lo, float& hi) {
  const unsigned ua = __builtin_bit_cast(unsigned, a), ub = __builtin_bit_cast(unsigned, b);
  if constexpr (B == 5) {
    const auto r = __builtin_amdgcn_permlane32_swap(ua, ub, false, false);
    lo = __builtin_bit_cast(float, (unsigned)r[0]);
    hi = __builtin_bit_cast(float, (unsigned)r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(ua, ub, false, false);
    lo = __builtin_bit_cast(float, (unsigned)r[0]);
    hi = __builtin_bit_cast(float, (unsigned)r[1]);
  }
}

// all-lane reduction of one value over lane bits [0, B]
template <int B, bool MAX>
__device__ __forceinline__ float lane_reduce(float v) {
  if constexpr (B < 0) {
    return v;
  } else {
    if constexpr (B >= 4) {
      float x, y;
      half_swap<B>(v, v, x, y);
      v = comb<MAX>(x, y);
    } else {
      v = comb<MAX>(v, dpp_mov<PairCtl<B>::v>(v));
    }
    return lane_reduce<B - 1, MAX>(v);
  }
}

// Transposed multi-reduction: N per-lane partials (N a power of two <= 64)
// -> lane l holds the wave-wide reduction of value (l >> (6 - log2 N)).
// Each step halves the list: a lane keeps one half, sends the other to its
// partner and adds what it receives, so N values cost N - 1 + (6 - log2 N)
// exchanges instead of 6 N.
template <int N, bool MAX, int B = 5>
__device__ __forceinline__ float multi_reduce(const float (&x)[N]) {
  if constexpr (N == 1) {
    return lane_reduce<B, MAX>(x[0]);
  } else {
    constexpr int H = N / 2;
    float y[H];
    if constexpr (B >= 4) {
#pragma unroll
      for (int k = 0; k < H; ++k) {
        float lo, hi;
        half_swap<B>(x[k], x[H + k], lo, hi);
        y[k] = comb<MAX>(lo, hi);
      }
    } else {
      const bool up = (lane_id() >> B) & 1;
#pragma unroll
      for (int k = 0; k < H; ++k) {
        const float keep = up ? x[H + k] : x[k];
        const float send = up ? x[k] : x[H + k];
        y[k] = comb<MAX>(keep, dpp_mov<PairCtl<B>::v>(send));
      }
    }
    return multi_reduce<H, MAX, B - 1>(y);
  }
}

// ---------------------------------------------------------------- fragments
template <int VEC, int NC>
struct Frag {
  float v[VEC * NC];
  __device__ __forceinline__ void zero() {
#pragma unroll
    for (int i = 0; i < VEC * NC; ++i) v[i] = 0.f;
  }
};

// element index of v[c*VEC + q] on this lane
template <int VEC>
__device__ __forceinline__ int frag_elem(int c, int q) { return (c * KGE_WAVE + lane_id()) * VEC + q; }

// Branch-free: lanes past the row's end load its first element group (same
// cache lines, no extra traffic) and zero the value, so a row load is one
// vector-memory instruction per chunk with no exec-mask branches. cols >= VEC.
template <int VEC, int NC>
__device__ __forceinline__ void load_row(Frag<VEC, NC>& f, const float* __restrict__ row, int cols) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e0 = (c * KGE_WAVE + lane_id()) * VEC;
    const bool in = e0 < cols;
    const int e = in ? e0 : 0;
    if (VEC == 4) {
      const float4 x = *reinterpret_cast<const float4*>(row + e);
      f.v[c * 4 + 0] = in ? x.x : 0.f; f.v[c * 4 + 1] = in ? x.y : 0.f;
      f.v[c * 4 + 2] = in ? x.z : 0.f; f.v[c * 4 + 3] = in ? x.w : 0.f;
    } else if (VEC == 2) {
      const float2 x = *reinterpret_cast<const float2*>(row + e);
      f.v[c * 2 + 0] = in ? x.x : 0.f; f.v[c * 2 + 1] = in ? x.y : 0.f;
    } else {
      const float x = row[e];
      f.v[c] = in ? x : 0.f;
    }
  }
}

// Unmasked: lanes past the row's end load its first element group and keep
// it (callers mask what they reduce). cols >= VEC.
template <int VEC, int NC>
__device__ __forceinline__ void load_row_raw(Frag<VEC, NC>& f, const float* __restrict__ row, int cols) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e0 = (c * KGE_WAVE + lane_id()) * VEC;
    const int e = e0 < cols ? e0 : 0;
    if (VEC == 4) {
      const float4 x = *reinterpret_cast<const float4*>(row + e);
      f.v[c * 4 + 0] = x.x; f.v[c * 4 + 1] = x.y; f.v[c * 4 + 2] = x.z; f.v[c * 4 + 3] = x.w;
    } else if (VEC == 2) {
      const float2 x = *reinterpret_cast<const float2*>(row + e);
      f.v[c * 2 + 0] = x.x; f.v[c * 2 + 1] = x.y;
    } else {
      f.v[c] = row[e];
    }
  }
}

template <int VEC, int NC>
__device__ __forceinline__ void store_row(const Frag<VEC, NC>& f, float* __restrict__ row, int cols) {
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e0 = (c * KGE_WAVE + lane_id()) * VEC;
    if (e0 >= cols) continue;
    if (VEC == 4) {
      *reinterpret_cast<float4*>(row + e0) =
          make_float4(f.v[c * 4 + 0], f.v[c * 4 + 1], f.v[c * 4 + 2], f.v[c * 4 + 3]);
    } else if (VEC == 2) {
      *reinterpret_cast<float2*>(row + e0) = make_float2(f.v[c * 2 + 0], f.v[c * 2 + 1]);
    } else {
      row[e0] = f.v[c];
    }
  }
}

// Half-width load: element (c*64+l)*VEC/2 + q of a row with cols/2 ... used by
// RotatE to fetch the phase row so that phase k sits beside complex element k
// (re, im interleaved in the entity fragment).
template <int VEC, int NC>
__device__ __forceinline__ void load_row_half(float (&h)[(VEC / 2 > 0 ? VEC / 2 : 1) * NC],
                                              const float* __restrict__ row, int cols_half) {
  constexpr int HV = VEC / 2 > 0 ? VEC / 2 : 1;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e0 = (c * KGE_WAVE + lane_id()) * HV;
    if (HV == 2) {
      float2 x = make_float2(0.f, 0.f);
      if (e0 < cols_half) x = *reinterpret_cast<const float2*>(row + e0);
      h[c * 2 + 0] = x.x; h[c * 2 + 1] = x.y;
    } else {
      h[c] = e0 < cols_half ? row[e0] : 0.f;
    }
  }
}

template <int VEC, int NC>
__device__ __forceinline__ void store_row_half(const float (&h)[(VEC / 2 > 0 ? VEC / 2 : 1) * NC],
                                               float* __restrict__ row, int cols_half) {
  constexpr int HV = VEC / 2 > 0 ? VEC / 2 : 1;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const int e0 = (c * KGE_WAVE + lane_id()) * HV;
    if (e0 >= cols_half) continue;
    if (HV == 2) *reinterpret_cast<float2*>(row + e0) = make_float2(h[c * 2 + 0], h[c * 2 + 1]);
    else row[e0] = h[c];
  }
}

// Phase profiling (profiling builds only, -DKGE_PHASE_PROF): thread 0 of each
// workgroup adds the wall-clock ticks of each phase to a device counter.
#ifdef KGE_PHASE_PROF
#define KGE_PROF_INIT() unsigned long long kge_prof_t_ = threadIdx.x == 0 ? wall_clock64() : 0ull
#define KGE_PROF(k)                                                   \
  do {                                                                \
    if (threadIdx.x == 0) {                                           \
      const unsigned long long kge_prof_n_ = wall_clock64();          \
      atomicAdd(&g_kge_prof[(k)], kge_prof_n_ - kge_prof_t_);         \
      kge_prof_t_ = kge_prof_n_;                                      \
    }                                                                 \
  } while (0)
#else
#define KGE_PROF_INIT() do {} while (0)
#define KGE_PROF(k) do {} while (0)
#endif

// Row normalisation of the fused constraint (TransE.py:171-172,
// DistMult.py:162-163: X / pow(sum |X|^2, 1/2) * 1): the per-lane partial is
// rounded op by op (no contraction) and reduced with lane_reduce's tree, the
// same tree multi_reduce uses, so every kernel that normalises a row gets the
// same bits. Lanes past the row's end must hold zeros.
template <int VEC, int NC>
__device__ __forceinline__ float norm_partial(const Frag<VEC, NC>& f) {
#pragma clang fp contract(off)
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VEC * NC; ++i) s = s + f.v[i] * f.v[i];
  return s;
}
__device__ __forceinline__ float inv_norm(float sumsq) { return 1.f / sqrtf(sumsq); }
template <int VEC, int NC>
__device__ __forceinline__ void scale_row(Frag<VEC, NC>& f, float k) {
#pragma clang fp contract(off)
#pragma unroll
  for (int i = 0; i < VEC * NC; ++i) f.v[i] = f.v[i] * k;
}
template <int VEC, int NC>
__device__ __forceinline__ void normalize_row(Frag<VEC, NC>& f) {
  scale_row(f, inv_norm(lane_reduce<5, false>(norm_partial(f))));
}

__device__ __forceinline__ void set_status(int32_t* status, int code) {
  if (status) atomicCAS(status, 0, code);
}

}  // namespace kge
