// Multi-GPU sparse row exchange (KGE/sharded.py), device side.
//
// Entity row e lives on rank e mod G at local row e div G. A rank's step
// needs the rows of its batch's ids; the ones another rank owns travel in
// fixed-capacity blocks (cap rows per owner), so every collective of the step
// has static sizes and nothing waits on the host (no counts read back, no
// sort). A rank's extended entity table is [its owned rows | G blocks of cap
// fetched rows]; the step runs on it directly, updates owned rows in place and
// writes the fetched rows' raw gradients back over them (KGE_FLAG_PHASE_UPDATE
// remote_rows_from), which then travel back to their owners.
//
//   kge_exchange_plan   the step's id occurrences -> extended-table rows:
//                       own ids straight to their shard row; the others
//                       de-duplicated in a hash table (one 64-bit CAS per new
//                       id, slot = (id + 1) << 32 | (position + 1)), each new
//                       id taking the next position of its owner's block
//   kge_exchange_rows   owner side: gather the requested rows into the send
//                       blocks; apply one source's gradient rows (SGD) or add
//                       them into a dense gradient (Adam)
//
// Block positions follow atomic arrival order, so which fetched row lands
// where varies from run to run; nothing summed depends on it (the update
// kernel sums a row's keys in code order; owners apply sources in rank order).
#include <algorithm>

#include "kge_step.h"

namespace kge {
namespace {

__device__ __forceinline__ uint32_t xhash(uint64_t id, uint64_t mask) {
  return (uint32_t)(((id * 0x9E3779B97F4A7C15ull) >> 29) & mask);
}

// every id occurrence: own ids need nothing; the others are inserted once.
// A new id's block position comes from its owner's counter; the counts are
// first summed per workgroup in LDS (one global atomic per owner per
// workgroup pass, not one per id: a single counter taking every id of a step
// serialises ~10^5 atomics on one address)
constexpr int kAggOwners = 64;

__global__ __launch_bounds__(256) void exch_insert_kernel(kge_exchange_desc d, int64_t n) {
  __shared__ int s_cnt[kAggOwners];
  __shared__ int s_base[kAggOwners];
  // the next call's zero state (zero_next), grid-stride
  if (d.zero_next) {
    uint32_t* z = reinterpret_cast<uint32_t*>(d.zero_next);
    const int64_t nw = d.zero_next_bytes / 4;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nw; q += (int64_t)gridDim.x * blockDim.x)
      z[q] = 0u;
  }
  const bool i64 = d.idx_dtype == KGE_IDX_I64;
  const uint64_t mask = (uint64_t)d.hslots - 1;
  const bool agg = d.world <= kAggOwners;
  const int tid = (int)threadIdx.x;
  for (int64_t q0 = (int64_t)blockIdx.x * blockDim.x; q0 < n; q0 += (int64_t)gridDim.x * blockDim.x) {
    const int64_t q = q0 + tid;   // (block-uniform trip count: the barriers below)
    if (agg) {
      if (tid < d.world) s_cnt[tid] = 0;
      __syncthreads();
    }
    bool fresh = false;
    int o = 0, lpos = 0;
    uint32_t h = 0;
    int64_t e = -1;
    unsigned long long key = 0;
    if (q < n) {
      if (q < 2 * d.batch) e = load_idx(d.pos, (q % d.batch) * 3 + (q < d.batch ? 0 : 2), i64);
      else e = load_idx(d.neg, q - 2 * d.batch, i64);
      if (e >= 0 && e < d.n_entities) {   // (bad ids are reported by the remap pass)
        o = (int)(e % d.world);
        if (o != d.rank || d.loopback) {
          key = (unsigned long long)(e + 1) << 32;
          h = xhash((uint64_t)e, mask);
          for (;;) {   // the table has >= 2 slots per occurrence: a free slot is always found
            const unsigned long long cur = atomicCAS(&d.htab[h], 0ull, key);
            if (cur == 0ull) {
              fresh = true;
              break;
            }
            if ((cur & 0xFFFFFFFF00000000ull) == key) break;
            h = (uint32_t)((h + 1) & mask);
          }
        }
      }
    }
    if (fresh) lpos = agg ? atomicAdd(&s_cnt[o], 1) : atomicAdd(&d.req_cnt[o], 1);
    if (agg) {
      __syncthreads();
      if (tid < d.world && s_cnt[tid] != 0) s_base[tid] = atomicAdd(&d.req_cnt[tid], s_cnt[tid]);
      __syncthreads();
      if (fresh) lpos += s_base[o];
    }
    if (fresh) {
      if (lpos < d.cap) store_idx(d.req_ids, (int64_t)o * d.cap + lpos, e, i64);
      atomicExch(&d.htab[h], key | (unsigned long long)(uint32_t)(lpos + 1));
    }
    if (agg) __syncthreads();   // (s_cnt / s_base reused by the next pass)
  }
}

// every occurrence -> its row of the extended table (positives' r copied)
__global__ __launch_bounds__(256) void exch_remap_kernel(kge_exchange_desc d, int64_t n) {
  const bool i64 = d.idx_dtype == KGE_IDX_I64;
  const uint64_t mask = (uint64_t)d.hslots - 1;
  int err = 0;
  bool over = false;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const bool is_pos = q < 2 * d.batch;
    const int64_t i = q % d.batch;
    int64_t e = is_pos ? load_idx(d.pos, i * 3 + (q < d.batch ? 0 : 2), i64) : load_idx(d.neg, q - 2 * d.batch, i64);
    int64_t row = d.local_rows;   // (a bad id / a full block: a row of the blocks, the step is void)
    if (e < 0 || e >= d.n_entities) {
      err = KGE_ERANGE;
      over = true;
    } else {
      const int o = (int)(e % d.world);
      if (o == d.rank && !d.loopback) {
        row = e / d.world;
      } else {
        const unsigned long long key = (unsigned long long)(e + 1) << 32;
        uint32_t h = xhash((uint64_t)e, mask);
        unsigned long long cur;
        while (((cur = d.htab[h]) & 0xFFFFFFFF00000000ull) != key) h = (uint32_t)((h + 1) & mask);
        const int64_t pos = (int64_t)(uint32_t)cur - 1;
        if (pos >= d.cap) over = true;
        else row += (int64_t)o * d.cap + pos;
      }
    }
    if (is_pos) {
      store_idx(d.pos_out, i * 3 + (q < d.batch ? 0 : 2), row, i64);
      if (q < d.batch) store_idx(d.pos_out, i * 3 + 1, load_idx(d.pos, i * 3 + 1, i64), i64);
    } else {
      store_idx(d.neg_out, q - 2 * d.batch, row, i64);
    }
  }
  if (err) set_status(d.status, err);
  if (over && d.err_flag) d.err_flag[0] = 1.f;
}

// POS mode: one wave per (positive, h / t), the row copied float4-wide when the strides allow
__global__ __launch_bounds__(256) void exch_pos_rows_kernel(kge_exchange_rows_desc d) {
  const bool i64 = d.idx_dtype == KGE_IDX_I64;
  const int64_t w = (int64_t)blockIdx.x * (blockDim.x / KGE_WAVE) + wave_id();
  if (w >= 2 * d.cap) return;
  const int64_t i = w >> 1;
  const int64_t r = load_idx(d.ids, 3 * i + 2 * (w & 1), i64);
  if (r < 0 || r >= d.shard.rows) {
    if (lane_id() == 0) set_status(d.status, KGE_ERANGE);
    return;
  }
  const float* src = d.shard.data + r * d.shard.ld;
  float* dst = d.rows + w * d.rows_ld;
  const int cols = (int)d.shard.cols;
  const bool v4 = cols % 4 == 0 && d.shard.ld % 4 == 0 && d.rows_ld % 4 == 0 &&
                  ((uintptr_t)d.shard.data % 16) == 0 && ((uintptr_t)d.rows % 16) == 0;
  if (v4) {
    for (int c = 4 * lane_id(); c < cols; c += 4 * KGE_WAVE)
      *reinterpret_cast<float4*>(dst + c) = *reinterpret_cast<const float4*>(src + c);
  } else {
    for (int c = lane_id(); c < cols; c += KGE_WAVE) dst[c] = src[c];
  }
}

// owner side: one wave per (block, position); float4 rows when the strides allow
__global__ __launch_bounds__(256) void exch_rows_kernel(kge_exchange_rows_desc d, int32_t b0, int32_t nb) {
  if ((d.mode == KGE_XROWS_SGD || d.mode == KGE_XROWS_ACCUM) && d.abort_flag && *d.abort_flag != 0.f) return;
  const bool i64 = d.idx_dtype == KGE_IDX_I64;
  const int64_t per = d.cap;
  const int64_t nw = (int64_t)gridDim.x * (blockDim.x / KGE_WAVE);
  float cs = 0.f;
  if (d.mode == KGE_XROWS_SGD) cs = -d.lr * (d.clip_norm / fmaxf(sqrtf(*d.norm2), d.clip_norm));
  const int cols = (int)d.shard.cols;
  const bool v4 = cols % 4 == 0 && d.shard.ld % 4 == 0 && d.rows_ld % 4 == 0 &&
                  ((uintptr_t)d.shard.data % 16) == 0 && ((uintptr_t)d.rows % 16) == 0 &&
                  (d.mode != KGE_XROWS_ACCUM || ((uintptr_t)d.acc % 16) == 0);
  for (int64_t w = (int64_t)blockIdx.x * (blockDim.x / KGE_WAVE) + wave_id(); w < (int64_t)nb * per; w += nw) {
    const int s = b0 + (int)(w / per);
    const int64_t q = w % per;
    if (q >= d.cnt[s]) continue;
    const int64_t slot = (int64_t)s * per + q;
    const int64_t e = load_idx(d.ids, slot, i64);
    if (e < 0 || e % d.world != d.rank || e / d.world >= d.shard.rows) {
      if (lane_id() == 0) set_status(d.status, KGE_ERANGE);
      continue;
    }
    float* sr = d.shard.data + (e / d.world) * d.shard.ld;
    float* rr = d.rows + slot * d.rows_ld;
    float* ar = d.mode == KGE_XROWS_ACCUM ? d.acc + (e / d.world) * (int64_t)cols : nullptr;
    if (v4) {
      for (int c = 4 * lane_id(); c < cols; c += 4 * KGE_WAVE) {
        if (d.mode == KGE_XROWS_GATHER) {
          *reinterpret_cast<float4*>(rr + c) = *reinterpret_cast<const float4*>(sr + c);
        } else if (d.mode == KGE_XROWS_SGD) {
          float4 x = *reinterpret_cast<const float4*>(sr + c);
          const float4 g = *reinterpret_cast<const float4*>(rr + c);
          x.x = x.x + g.x * cs; x.y = x.y + g.y * cs; x.z = x.z + g.z * cs; x.w = x.w + g.w * cs;
          *reinterpret_cast<float4*>(sr + c) = x;
        } else {
          float4 x = *reinterpret_cast<const float4*>(ar + c);
          const float4 g = *reinterpret_cast<const float4*>(rr + c);
          x.x += g.x; x.y += g.y; x.z += g.z; x.w += g.w;
          *reinterpret_cast<float4*>(ar + c) = x;
        }
      }
    } else {
      for (int c = lane_id(); c < cols; c += KGE_WAVE) {
        if (d.mode == KGE_XROWS_GATHER) rr[c] = sr[c];
        else if (d.mode == KGE_XROWS_SGD) sr[c] = sr[c] + rr[c] * cs;
        else ar[c] += rr[c];
      }
    }
  }
}

kge_status xfail(const char* msg) {
  kge_set_error(msg);
  return KGE_EINVAL;
}

}  // namespace
}  // namespace kge

using namespace kge;

extern "C" {

kge_status kge_exchange_plan(const kge_exchange_desc* d, void* stream) {
  if (!d) return xfail("null descriptor");
  if (d->abi_version != KGE_ABI_VERSION) return xfail("kge_exchange_plan: abi_version mismatch");
  if (d->idx_dtype != KGE_IDX_I32 && d->idx_dtype != KGE_IDX_I64) return xfail("kge_exchange_plan: bad idx_dtype");
  if (d->world < 1 || d->rank < 0 || d->rank >= d->world) return xfail("kge_exchange_plan: bad world / rank");
  if (d->batch < 0 || d->n_neg < 0 || d->cap <= 0 || d->local_rows < 0) return xfail("kge_exchange_plan: bad sizes");
  if (d->n_entities <= 0 || d->n_entities > (int64_t)0xFFFFFFFE) return xfail("kge_exchange_plan: n_entities out of range");
  const int64_t n = 2 * d->batch + d->n_neg;
  if (d->zero_next && (d->zero_next_bytes < 0 || d->zero_next_bytes % 4 != 0 || ((uintptr_t)d->zero_next % 4) != 0))
    return xfail("kge_exchange_plan: zero_next must be 4-byte aligned, a multiple of 4 bytes");
  if (n == 0) {
    if (d->zero_next && d->zero_next_bytes > 0) {
      const hipError_t e = hipMemsetAsync(d->zero_next, 0, (size_t)d->zero_next_bytes, (hipStream_t)stream);
      if (e != hipSuccess) { kge_set_error(hipGetErrorString(e)); return KGE_EHIP; }
    }
    return KGE_OK;
  }
  if (d->hslots < 2 * n || (d->hslots & (d->hslots - 1)) != 0)
    return xfail("kge_exchange_plan: hslots must be a power of two >= 2 x occurrences");
  if (!d->pos || (d->n_neg && !d->neg) || !d->pos_out || (d->n_neg && !d->neg_out) || !d->htab || !d->req_ids ||
      !d->req_cnt)
    return xfail("kge_exchange_plan: null array");
  hipStream_t st = (hipStream_t)stream;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(exch_insert_kernel, dim3(blocks), dim3(256), 0, st, *d, n);
  hipLaunchKernelGGL(exch_remap_kernel, dim3(blocks), dim3(256), 0, st, *d, n);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    kge_set_error(hipGetErrorString(e));
    return KGE_EHIP;
  }
  return KGE_OK;
}

kge_status kge_exchange_rows(const kge_exchange_rows_desc* d, void* stream) {
  if (!d) return xfail("null descriptor");
  if (d->mode != KGE_XROWS_GATHER && d->mode != KGE_XROWS_SGD && d->mode != KGE_XROWS_ACCUM &&
      d->mode != KGE_XROWS_POS)
    return xfail("kge_exchange_rows: bad mode");
  if (d->mode == KGE_XROWS_POS) {
    if (d->idx_dtype != KGE_IDX_I32 && d->idx_dtype != KGE_IDX_I64) return xfail("kge_exchange_rows: bad idx_dtype");
    if (d->cap < 0 || !d->ids || !d->rows || !d->shard.data || d->shard.cols <= 0 || d->shard.ld < d->shard.cols ||
        d->rows_ld < d->shard.cols)
      return xfail("kge_exchange_rows: POS needs ids, rows, a shard and rows_ld >= its columns");
    if (d->cap == 0) return KGE_OK;
    const unsigned blocks = (unsigned)((2 * d->cap + 3) / 4);
    hipLaunchKernelGGL(exch_pos_rows_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *d);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
      kge_set_error(hipGetErrorString(e));
      return KGE_EHIP;
    }
    return KGE_OK;
  }
  if (d->idx_dtype != KGE_IDX_I32 && d->idx_dtype != KGE_IDX_I64) return xfail("kge_exchange_rows: bad idx_dtype");
  if (d->world < 1 || d->rank < 0 || d->rank >= d->world || d->cap <= 0) return xfail("kge_exchange_rows: bad sizes");
  if (!d->shard.data || d->shard.cols <= 0 || d->shard.ld < d->shard.cols || d->rows_ld < d->shard.cols)
    return xfail("kge_exchange_rows: bad shard / row stride");
  if (!d->ids || !d->cnt || !d->rows) return xfail("kge_exchange_rows: null array");
  if (d->mode == KGE_XROWS_SGD && (!d->norm2 || !(d->clip_norm > 0.f)))
    return xfail("kge_exchange_rows: SGD needs norm2 and clip_norm > 0");
  if (d->mode == KGE_XROWS_ACCUM && !d->acc) return xfail("kge_exchange_rows: ACCUM needs acc");
  int32_t b0 = d->source, nb = 1;
  if (d->source < 0) {
    if (d->mode != KGE_XROWS_GATHER) return xfail("kge_exchange_rows: SGD / ACCUM take one source block");
    b0 = 0;
    nb = d->world;
  } else if (d->source >= d->world) {
    return xfail("kge_exchange_rows: source out of range");
  }
  const int64_t waves = (int64_t)nb * d->cap;
  const unsigned blocks = (unsigned)std::min<int64_t>((waves + 3) / 4, 16384);
  hipLaunchKernelGGL(exch_rows_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *d, b0, nb);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    kge_set_error(hipGetErrorString(e));
    return KGE_EHIP;
  }
  return KGE_OK;
}

}  // extern "C"
