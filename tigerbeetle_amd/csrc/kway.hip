// kway.hip — the scan path's k-way merge, data-parallel.
//
// The reference (src/lsm/k_way_merge.zig:8-205, KWayMergeIteratorType) pops
// the k sorted streams through a binary heap; among equal keys the stream
// with precedence wins (`ordered`, :197-203) and `pop` discards every later
// value whose key equals the last one popped (:91-107). With the precedence
// of the reference's own tests (stream_precedence(a, b) = a > b, :239-244:
// higher streams win) the output is a pure function of each element:
//
//   value (s, i) is emitted  iff  it is the first of its key's run in stream s
//                                 and no stream s' > s holds that key;
//   its output position      =    sum over streams s' of the emitted values of
//                                 s' whose key comes before it (direction order).
//
// Kernels: emit flags (binary searches in the higher streams) -> exclusive scan
// of the flags (hipCUB) -> scatter (one binary search per stream). Each
// element is read once per kernel plus O(k log n) key probes; the scatter
// moves each emitted value once (16-byte copies).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "keys.h"

namespace tbc {

template <int KIND, bool DESC, int KL = KeyLimbs<KIND>::value>
__device__ __forceinline__ bool before(const Key<KL> &a, const Key<KL> &b) {
    return DESC ? key_lt(b, a) : key_lt(a, b);
}

// First index j of stream [v, v + n) whose key is not before `k`.
template <int KIND, bool DESC, int KL = KeyLimbs<KIND>::value>
__device__ __forceinline__ uint32_t kway_lower_bound(const uint8_t *v, uint32_t n, uint32_t vs, uint32_t ts,
                                                     const Key<KL> &k) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (before<KIND, DESC>(load_key<KIND>(v + (size_t)mid * vs, ts), k)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

__device__ __forceinline__ uint32_t stream_of(const uint32_t *pre, uint32_t k, uint32_t g) {
    uint32_t s = 0;
    while (s + 1 < k && gld<uint32_t>(pre + s + 1) <= g) s++;
    return s;
}

template <int KIND, bool DESC>
__global__ __launch_bounds__(256) void k_kway_flags(const uint64_t *ptr, const uint32_t *pre, uint32_t k, uint32_t n,
                                                    uint32_t vs, uint32_t ts, uint32_t *flags) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g > n) return;
    if (g == n) { // the scan's total lands in flags[n]'s slot
        gst<uint32_t>(flags + n, 0u);
        return;
    }
    const uint32_t s = stream_of(pre, k, g);
    const uint32_t i = g - gld<uint32_t>(pre + s);
    const uint8_t *v = (const uint8_t *)gld<uint64_t>(ptr + s);
    const auto key = load_key<KIND>(v + (size_t)i * vs, ts);
    bool emit = i == 0 || !key_eq(load_key<KIND>(v + (size_t)(i - 1) * vs, ts), key);
    for (uint32_t t = s + 1; emit && t < k; t++) {
        const uint32_t base = gld<uint32_t>(pre + t), len = gld<uint32_t>(pre + t + 1) - base;
        const uint8_t *w = (const uint8_t *)gld<uint64_t>(ptr + t);
        const uint32_t j = kway_lower_bound<KIND, DESC>(w, len, vs, ts, key);
        if (j < len && key_eq(load_key<KIND>(w + (size_t)j * vs, ts), key)) emit = false;
    }
    gst<uint32_t>(flags + g, emit ? 1u : 0u);
}

template <int KIND, bool DESC>
__global__ __launch_bounds__(256) void k_kway_scatter(const uint64_t *ptr, const uint32_t *pre, uint32_t k, uint32_t n,
                                                      uint32_t vs, uint32_t ts, const uint32_t *flags,
                                                      const uint32_t *scan, uint8_t *out) {
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= n || !gld<uint32_t>(flags + g)) return;
    const uint32_t s = stream_of(pre, k, g);
    const uint32_t i = g - gld<uint32_t>(pre + s);
    const uint8_t *v = (const uint8_t *)gld<uint64_t>(ptr + s) + (size_t)i * vs;
    const auto key = load_key<KIND>(v, ts);
    uint32_t pos = 0;
    for (uint32_t t = 0; t < k; t++) {
        const uint32_t base = gld<uint32_t>(pre + t), len = gld<uint32_t>(pre + t + 1) - base;
        const uint32_t j = t == s ? i : kway_lower_bound<KIND, DESC>((const uint8_t *)gld<uint64_t>(ptr + t), len, vs, ts, key);
        pos += gld<uint32_t>(scan + base + j) - gld<uint32_t>(scan + base);
    }
    uint8_t *d = out + (size_t)pos * vs;
    for (uint32_t o = 0; o < vs; o += 16) { // 16-byte moves (value sizes are multiples of 16)
        const uint64_t lo = gld<uint64_t>(v + o), hi = gld<uint64_t>(v + o + 8);
        gst<uint64_t>(d + o, lo);
        gst<uint64_t>(d + o + 8, hi);
    }
}

template <int KIND, bool DESC>
static int launch_kway_t(const uint64_t *ptr, const uint32_t *pre, uint32_t k, uint32_t n, uint32_t vs, uint32_t ts,
                         uint32_t *flags, uint32_t *scan, void *cub_tmp, size_t cub_bytes, uint8_t *out, hipStream_t s) {
    const uint32_t grid1 = (n + 1 + 255) / 256, grid2 = (n + 255) / 256;
    hipLaunchKernelGGL((k_kway_flags<KIND, DESC>), dim3(grid1), dim3(256), 0, s, ptr, pre, k, n, vs, ts, flags);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipcub::DeviceScan::ExclusiveSum(cub_tmp, cub_bytes, flags, scan, (int)n + 1, s) != hipSuccess) return -1;
    if (n) {
        hipLaunchKernelGGL((k_kway_scatter<KIND, DESC>), dim3(grid2), dim3(256), 0, s, ptr, pre, k, n, vs, ts, flags,
                           scan, out);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

size_t kway_scan_tmp_bytes(uint32_t n) {
    size_t bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n + 1);
    return bytes;
}

int launch_kway(uint32_t key_kind, bool descending, const uint64_t *ptr, const uint32_t *pre, uint32_t k, uint32_t n,
                uint32_t vs, uint32_t ts, uint32_t *flags, uint32_t *scan, void *cub_tmp, size_t cub_bytes,
                uint8_t *out, void *stream) {
    hipStream_t s = (hipStream_t)stream;
#define TBC_KWAY(KIND)                                                                                    \
    return descending ? launch_kway_t<KIND, true>(ptr, pre, k, n, vs, ts, flags, scan, cub_tmp, cub_bytes, out, s) \
                      : launch_kway_t<KIND, false>(ptr, pre, k, n, vs, ts, flags, scan, cub_tmp, cub_bytes, out, s)
    switch (key_kind) {
    case kKeyTimestamp: TBC_KWAY(kKeyTimestamp);
    case kKeyIdU128: TBC_KWAY(kKeyIdU128);
    case kKeyCompositeU64: TBC_KWAY(kKeyCompositeU64);
    case kKeyCompositeU128: TBC_KWAY(kKeyCompositeU128);
    default: return -1;
    }
#undef TBC_KWAY
}

} // namespace tbc
