// Deterministic ordered scatter-add: out[key[i]] = sum of val[i] over the entries of each key,
// added in increasing entry index i.  The deterministic-order mode of the backward passes whose
// fast path scatters with float atomics (rasterizer, shading): SURVEY.md §5 "race detection".
//
//   1. the caller writes one key per entry (keys >= M are dropped);
//   2. detsum_sort: a stable LSD radix sort of (key, entry index) over the key's significant bits
//      (rocPRIM through hipCUB: one library sort, no float work) -- each key's entries end up
//      contiguous and in entry order;
//   3. the caller writes the C components of each entry at its SORTED position (it knows the
//      entry index there, so per-entry values are computed once, already in segment order), or
//      fills them in entry order and calls detsum_gather;
//   4. detsum_reduce: each key's segment is summed in chunks of `chunk` entries (sequentially
//      inside a chunk), then the chunk sums sequentially.  chunk <= 0 sums every segment in one
//      sequential pass: exactly the order of a serial loop over the entries, as the CPU oracle's
//      (PyTorch3D's CPU) backward accumulates.  Either way the result depends only on the
//      entries, never on timing.
//   5. detsum_reduce_chain: a long entry range in batches (bounded workspace): the first batch
//      sums from 0, every later one continues each key's sequential chain from the previous
//      batches' total -- bitwise one serial loop over all the entries.
#include <cstdlib>

#include <hipcub/hipcub.hpp>

#include "pr_common.h"

namespace pr {
namespace {

constexpr size_t kAlign = 256;
size_t up(size_t b) { return (b + kAlign - 1) / kAlign * kAlign; }

int key_bits(int64_t M) {  // bits of the largest key that can occur (M = dropped)
  int b = 1;
  while (b < 32 && (uint64_t)M >> b) ++b;
  return b;
}

size_t sort_temp_bytes(int64_t n, int end_bit) {
  size_t t = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, t, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                         (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, end_bit) != hipSuccess)
    return 0;
  return t;
}

__global__ void iota_kernel(uint32_t* idx, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    idx[i] = (uint32_t)i;
}

// segment bounds of every key present: start = first sorted position, end = one past the last
__global__ void bounds_kernel(const uint32_t* keys, int64_t n, int64_t M, uint32_t* start, uint32_t* end) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    if (k >= (uint64_t)M) continue;
    if (i == 0 || keys[i - 1] != k) start[k] = (uint32_t)i;
    if (i == n - 1 || keys[i + 1] != k) end[k] = (uint32_t)(i + 1);
  }
}

__global__ void gather_kernel(const uint32_t* keys_sorted, const uint32_t* idx_sorted, const float* vals,
                              float* vals_sorted, int64_t n, int64_t M, int C) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (keys_sorted[i] >= (uint64_t)M) continue;
    const int64_t src = (int64_t)idx_sorted[i] * C;
    for (int c = 0; c < C; ++c) vals_sorted[i * C + c] = vals[src + c];
  }
}

// sequential sum of vals[(s..e) * C + c] for c < C (C <= 9), 8 entries of loads in flight
template <int C>
PR_DEV void seq_sum(const float* vals, int64_t s, int64_t e, float acc[C]) {
  int64_t j = s;
  for (; j + 8 <= e; j += 8) {
    float x[8][C];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < C; ++c) x[u][c] = vals[(j + u) * C + c];
#pragma unroll
    for (int u = 0; u < 8; ++u)
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] += x[u][c];
  }
  for (; j < e; ++j)
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] += vals[j * C + c];
}

// pass 1: the head of each chunk sums its chunk into its own sorted position (init: the chain
// continues from out[k] -- detsum_reduce_chain; one chunk per key then)
template <int C>
__global__ void chunk_kernel(const uint32_t* keys, const uint32_t* start, const uint32_t* end, float* vals,
                             int64_t n, int64_t M, int64_t chunk, const float* init) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = keys[i];
    if (k >= (uint64_t)M) continue;
    const int64_t s = start[k], e = end[k];
    if ((i - s) % chunk != 0) continue;
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = init ? init[(int64_t)k * C + c] : 0.f;
    seq_sum<C>(vals, i, i + chunk < e ? i + chunk : e, acc);
#pragma unroll
    for (int c = 0; c < C; ++c) vals[i * C + c] = acc[c];
  }
}

// pass 2: per key, its chunk sums in order (one chunk: the plain sequential sum of pass 1)
// (accumulate: 0 out = sum, 1 out += sum, 2 chained -- the single chunk already started from out;
// keys without entries keep out)
template <int C>
__global__ void segment_kernel(const uint32_t* start, const uint32_t* end, const float* vals, float* out, int64_t M,
                               int64_t chunk, int accumulate) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < M; k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t s = start[k], e = end[k];
    if (accumulate == 2) {
      if (s < e)
#pragma unroll
        for (int c = 0; c < C; ++c) out[k * C + c] = vals[s * C + c];
      continue;
    }
    float acc[C];
#pragma unroll
    for (int c = 0; c < C; ++c) acc[c] = 0.f;
    int64_t j = s;
    for (; j + 4 * chunk <= e; j += 4 * chunk) {  // 4 chunk sums in flight
      float x[4][C];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c) x[u][c] = vals[(j + u * chunk) * C + c];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int c = 0; c < C; ++c) acc[c] += x[u][c];
    }
    for (; j < e; j += chunk)
#pragma unroll
      for (int c = 0; c < C; ++c) acc[c] += vals[j * C + c];
#pragma unroll
    for (int c = 0; c < C; ++c) out[k * C + c] = accumulate ? out[k * C + c] + acc[c] : acc[c];
  }
}

int blocks(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + kThreads - 1) / kThreads, 16384)); }

}  // namespace

size_t detsum_workspace(int64_t n, int64_t M, int C) {
  if (n <= 0 || M <= 0) return 0;
  return 4 * up((size_t)n * 4) + 2 * up((size_t)n * C * 4) + 2 * up((size_t)M * 4) +
         up(sort_temp_bytes(n, key_bits(M)));
}

int detsum_layout(void* ws, size_t bytes, int64_t n, int64_t M, int C, DetSum& d) {
  d = DetSum{};
  d.n = n; d.M = M; d.C = C;
  if (n <= 0 || M <= 0) return PR_OK;
  if (n > (int64_t)INT32_MAX || M >= (int64_t)UINT32_MAX || C < 1 || C > 9)
    return set_error(PR_ERR_ARG, "deterministic scatter: too many entries / keys, or C outside 1..9");
  if (!ws || bytes < detsum_workspace(n, M, C))
    return set_error(PR_ERR_WORKSPACE, "deterministic scatter: workspace too small");
  char* p = reinterpret_cast<char*>(ws);
  auto take = [&](size_t b) { char* q = p; p += up(b); return q; };
  d.keys = reinterpret_cast<uint32_t*>(take((size_t)n * 4));
  d.keys_sorted = reinterpret_cast<uint32_t*>(take((size_t)n * 4));
  d.idx = reinterpret_cast<uint32_t*>(take((size_t)n * 4));
  d.idx_sorted = reinterpret_cast<uint32_t*>(take((size_t)n * 4));
  d.vals = reinterpret_cast<float*>(take((size_t)n * C * 4));
  d.vals_sorted = reinterpret_cast<float*>(take((size_t)n * C * 4));
  d.start = reinterpret_cast<uint32_t*>(take((size_t)M * 4));
  d.end = reinterpret_cast<uint32_t*>(take((size_t)M * 4));
  d.end_bit = key_bits(M);
  d.temp_bytes = sort_temp_bytes(n, d.end_bit);
  d.temp = take(d.temp_bytes);
  return PR_OK;
}

int detsum_sort(const DetSum& d, hipStream_t st) {
  if (d.n <= 0) return PR_OK;
  iota_kernel<<<blocks(d.n), kThreads, 0, st>>>(d.idx, d.n);
  if (int e = check_launch("detsum_iota")) return e;
  size_t tb = d.temp_bytes;
  if (hipcub::DeviceRadixSort::SortPairs(d.temp, tb, d.keys, d.keys_sorted, d.idx, d.idx_sorted, (int)d.n, 0,
                                         d.end_bit, st) != hipSuccess)
    return set_error(PR_ERR_HIP, "deterministic scatter: radix sort failed");
  return check_launch("detsum_sort");
}

int detsum_gather(const DetSum& d, hipStream_t st) {
  if (d.n <= 0) return PR_OK;
  gather_kernel<<<blocks(d.n), kThreads, 0, st>>>(d.keys_sorted, d.idx_sorted, d.vals, d.vals_sorted, d.n, d.M,
                                                  d.C);
  return check_launch("detsum_gather");
}

namespace {
int reduce_impl(const DetSum& d, float* out, int64_t chunk, int mode, hipStream_t st) {
  if (d.M <= 0) return PR_OK;
  if (d.n <= 0) {
    if (mode == 0 && hipMemsetAsync(out, 0, (size_t)d.M * d.C * 4, st) != hipSuccess)
      return set_error(PR_ERR_HIP, "deterministic scatter: memset failed");
    return PR_OK;
  }
  if (chunk <= 0) chunk = d.n;
  const float* init = mode == 2 ? out : nullptr;
  if (hipMemsetAsync(d.start, 0, (size_t)d.M * 4, st) != hipSuccess ||
      hipMemsetAsync(d.end, 0, (size_t)d.M * 4, st) != hipSuccess)
    return set_error(PR_ERR_HIP, "deterministic scatter: memset failed");
  bounds_kernel<<<blocks(d.n), kThreads, 0, st>>>(d.keys_sorted, d.n, d.M, d.start, d.end);
  if (int e = check_launch("detsum_bounds")) return e;
  switch (d.C) {
#define PR_DETSUM_C(CC)                                                                                      \
  case CC:                                                                                                   \
    chunk_kernel<CC><<<blocks(d.n), kThreads, 0, st>>>(d.keys_sorted, d.start, d.end, d.vals_sorted, d.n,    \
                                                       d.M, chunk, init);                                    \
    if (int e = check_launch("detsum_chunk")) return e;                                                      \
    segment_kernel<CC><<<blocks(d.M), kThreads, 0, st>>>(d.start, d.end, d.vals_sorted, out, d.M, chunk,     \
                                                         mode);                                              \
    break;
    PR_DETSUM_C(1) PR_DETSUM_C(3) PR_DETSUM_C(6) PR_DETSUM_C(9)
#undef PR_DETSUM_C
    default:
      return set_error(PR_ERR_ARG, "deterministic scatter: C must be 1, 3, 6 or 9");
  }
  return check_launch("detsum_segment");
}
}  // namespace

int64_t det_batch() {
  const char* e = getenv("PR_DET_BATCH");
  const long long v = e ? atoll(e) : 0;
  return v > 0 ? (int64_t)v : (int64_t(1) << 24);
}

int detsum_reduce(const DetSum& d, float* out, int64_t chunk, bool accumulate, hipStream_t st) {
  return reduce_impl(d, out, chunk, accumulate ? 1 : 0, st);
}

int detsum_reduce_chain(const DetSum& d, float* out, bool first, hipStream_t st) {
  return reduce_impl(d, out, 0, first ? 0 : 2, st);
}

}  // namespace pr
