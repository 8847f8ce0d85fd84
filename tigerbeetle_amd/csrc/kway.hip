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
// of the flags (hipCUB) -> scatter (one binary search per stream), both
// searching only a per-tile window of each other stream. Each
// element is read once per kernel plus O(k log n) key probes; the scatter
// moves each emitted value once (16-byte copies).
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "keys.h"
#include "tbc.h"

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

constexpr uint32_t kKwayTile = 256;

// Workgroups take 256 consecutive values of ONE stream (tiles never straddle
// streams). The lower bounds of any key of the tile in another stream t lie
// between those of the tile's first and last keys, so lanes 0..k-1 search
// those two once and every thread then searches only that window (usually a
// few hundred values, cache-resident) instead of the whole stream.
struct KwayTile {
    uint32_t s, i0, n_s;
};

__device__ __forceinline__ KwayTile kway_tile(const uint32_t *pre, const uint32_t *tile_pre, uint32_t k) {
    KwayTile t{0, 0, 0};
    while (t.s + 1 < k && gld<uint32_t>(tile_pre + t.s + 1) <= blockIdx.x) t.s++;
    t.i0 = (blockIdx.x - gld<uint32_t>(tile_pre + t.s)) * kKwayTile;
    t.n_s = gld<uint32_t>(pre + t.s + 1) - gld<uint32_t>(pre + t.s);
    return t;
}

template <int KIND, bool DESC>
__device__ __forceinline__ void kway_windows(const uint64_t *ptr, const uint32_t *pre, uint32_t k, uint32_t vs,
                                             uint32_t ts, const KwayTile &tl, uint32_t *lo, uint32_t *hi) {
    const uint32_t t = threadIdx.x;
    if (t < k && t != tl.s) {
        const uint8_t *v = (const uint8_t *)gld<uint64_t>(ptr + tl.s);
        const uint32_t last = min(tl.i0 + kKwayTile, tl.n_s) - 1;
        const uint8_t *w = (const uint8_t *)gld<uint64_t>(ptr + t);
        const uint32_t len = gld<uint32_t>(pre + t + 1) - gld<uint32_t>(pre + t);
        lo[t] = kway_lower_bound<KIND, DESC>(w, len, vs, ts, load_key<KIND>(v + (size_t)tl.i0 * vs, ts));
        hi[t] = kway_lower_bound<KIND, DESC>(w, len, vs, ts, load_key<KIND>(v + (size_t)last * vs, ts));
    }
    __syncthreads();
}

// lower bound of `key` in stream t, known to lie in [lo, hi].
template <int KIND, bool DESC, int KL = KeyLimbs<KIND>::value>
__device__ __forceinline__ uint32_t kway_window_search(const uint8_t *w, uint32_t lo, uint32_t hi, uint32_t vs,
                                                       uint32_t ts, const Key<KL> &key) {
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (before<KIND, DESC>(load_key<KIND>(w + (size_t)mid * vs, ts), key)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Lower bounds of `key` in every stream u < KMAX (u != skip) at once: one
// bisection step per stream per round, so a thread has up to k independent
// probes in flight instead of k dependent searches (k <= KMAX only).
constexpr int kKwayLockstep = 16;

template <int KIND, bool DESC, int KMAX, int KL = KeyLimbs<KIND>::value>
__device__ __forceinline__ void kway_lockstep(const uint64_t *ptr, uint32_t k, uint32_t vs, uint32_t ts,
                                              const uint32_t *wlo, const uint32_t *whi, uint32_t rounds,
                                              uint32_t from, uint32_t skip, const Key<KL> &key,
                                              uint32_t (&j)[KMAX], const uint8_t *(&w)[KMAX]) {
    uint32_t hi[KMAX];
#pragma unroll
    for (int u = 0; u < KMAX; u++) {
        const bool on = (uint32_t)u < k && (uint32_t)u >= from && (uint32_t)u != skip;
        j[u] = on ? wlo[u] : 0;
        hi[u] = on ? whi[u] : 0;
        w[u] = (uint32_t)u < k ? (const uint8_t *)gld<uint64_t>(ptr + u) : nullptr;
    }
    for (uint32_t r = 0; r < rounds; r++) {
#pragma unroll
        for (int u = 0; u < KMAX; u++) {
            if (j[u] < hi[u]) {
                const uint32_t mid = (j[u] + hi[u]) >> 1;
                if (before<KIND, DESC>(load_key<KIND>(w[u] + (size_t)mid * vs, ts), key)) j[u] = mid + 1;
                else hi[u] = mid;
            }
        }
    }
}

__device__ __forceinline__ uint32_t bisect_rounds(uint32_t width) {
    return 32 - __builtin_clz(width | 1); // ceil(log2(width + 1))
}

template <int KIND, bool DESC, int KMAX, int KL = KeyLimbs<KIND>::value>
__device__ __forceinline__ bool kway_emit_lockstep(const uint64_t *ptr, const uint32_t *pre, uint32_t k, uint32_t vs,
                                                   uint32_t ts, const uint32_t *lo, const uint32_t *hi, uint32_t s,
                                                   const Key<KL> &key, bool emit) {
    uint32_t j[KMAX];
    const uint8_t *w[KMAX];
    uint32_t rounds = 0;
    for (uint32_t u = s + 1; u < k; u++) rounds = max(rounds, bisect_rounds(hi[u] - lo[u]));
    kway_lockstep<KIND, DESC, KMAX>(ptr, k, vs, ts, lo, hi, rounds, s + 1, s, key, j, w);
#pragma unroll
    for (int u = 0; u < KMAX; u++) {
        if ((uint32_t)u > s && (uint32_t)u < k) {
            const uint32_t len = gld<uint32_t>(pre + u + 1) - gld<uint32_t>(pre + u);
            if (j[u] < len && key_eq(load_key<KIND>(w[u] + (size_t)j[u] * vs, ts), key)) emit = false;
        }
    }
    return emit;
}

template <int KIND, bool DESC, int KMAX, int KL = KeyLimbs<KIND>::value>
__device__ __forceinline__ uint32_t kway_pos_lockstep(const uint64_t *ptr, const uint32_t *pre, uint32_t k,
                                                      uint32_t vs, uint32_t ts, const uint32_t *lo,
                                                      const uint32_t *hi, uint32_t s, uint32_t i, const Key<KL> &key,
                                                      const uint32_t *scan) {
    uint32_t j[KMAX];
    const uint8_t *w[KMAX];
    uint32_t rounds = 0;
    for (uint32_t u = 0; u < k; u++)
        if (u != s) rounds = max(rounds, bisect_rounds(hi[u] - lo[u]));
    kway_lockstep<KIND, DESC, KMAX>(ptr, k, vs, ts, lo, hi, rounds, 0, s, key, j, w);
    uint32_t pos = 0;
#pragma unroll
    for (int u = 0; u < KMAX; u++) {
        if ((uint32_t)u < k) {
            const uint32_t base = gld<uint32_t>(pre + u);
            const uint32_t jj = (uint32_t)u == s ? i : j[u];
            pos += gld<uint32_t>(scan + base + jj) - gld<uint32_t>(scan + base);
        }
    }
    return pos;
}

template <int KIND, bool DESC, bool LS>
__global__ __launch_bounds__(256) void k_kway_flags(const uint64_t *ptr, const uint32_t *pre, const uint32_t *tile_pre,
                                                    uint32_t k, uint32_t n, uint32_t vs, uint32_t ts, uint32_t *flags) {
    __shared__ uint32_t lo[TBC_KWAY_STREAMS_MAX], hi[TBC_KWAY_STREAMS_MAX];
    const KwayTile tl = kway_tile(pre, tile_pre, k);
    kway_windows<KIND, DESC>(ptr, pre, k, vs, ts, tl, lo, hi);
    const uint32_t i = tl.i0 + threadIdx.x;
    if (blockIdx.x == 0 && threadIdx.x == 0) gst<uint32_t>(flags + n, 0u); // the scan's total lands there
    if (i >= tl.n_s) return;
    const uint8_t *v = (const uint8_t *)gld<uint64_t>(ptr + tl.s);
    const auto key = load_key<KIND>(v + (size_t)i * vs, ts);
    bool emit = i == 0 || !key_eq(load_key<KIND>(v + (size_t)(i - 1) * vs, ts), key);
    if (LS) { // 9..16 streams (a separate instantiation: its registers do not cost the others occupancy)
        gst<uint32_t>(flags + gld<uint32_t>(pre + tl.s) + i,
                      kway_emit_lockstep<KIND, DESC, kKwayLockstep>(ptr, pre, k, vs, ts, lo, hi, tl.s, key, emit)
                          ? 1u : 0u);
        return;
    }
    for (uint32_t t = tl.s + 1; emit && t < k; t++) {
        const uint32_t len = gld<uint32_t>(pre + t + 1) - gld<uint32_t>(pre + t);
        const uint8_t *w = (const uint8_t *)gld<uint64_t>(ptr + t);
        const uint32_t j = kway_window_search<KIND, DESC>(w, lo[t], hi[t], vs, ts, key);
        if (j < len && key_eq(load_key<KIND>(w + (size_t)j * vs, ts), key)) emit = false;
    }
    gst<uint32_t>(flags + gld<uint32_t>(pre + tl.s) + i, emit ? 1u : 0u);
}

template <int KIND, bool DESC, bool LS>
__global__ __launch_bounds__(256) void k_kway_scatter(const uint64_t *ptr, const uint32_t *pre, const uint32_t *tile_pre,
                                                      uint32_t k, uint32_t vs, uint32_t ts, const uint32_t *flags,
                                                      const uint32_t *scan, uint8_t *out) {
    __shared__ uint32_t lo[TBC_KWAY_STREAMS_MAX], hi[TBC_KWAY_STREAMS_MAX];
    const KwayTile tl = kway_tile(pre, tile_pre, k);
    kway_windows<KIND, DESC>(ptr, pre, k, vs, ts, tl, lo, hi);
    const uint32_t i = tl.i0 + threadIdx.x;
    if (i >= tl.n_s || !gld<uint32_t>(flags + gld<uint32_t>(pre + tl.s) + i)) return;
    const uint8_t *v = (const uint8_t *)gld<uint64_t>(ptr + tl.s) + (size_t)i * vs;
    const auto key = load_key<KIND>(v, ts);
    uint32_t pos = 0;
    if (LS) {
        pos = kway_pos_lockstep<KIND, DESC, kKwayLockstep>(ptr, pre, k, vs, ts, lo, hi, tl.s, i, key, scan);
    } else {
    for (uint32_t t = 0; t < k; t++) {
        const uint32_t base = gld<uint32_t>(pre + t);
        const uint32_t j = t == tl.s ? i
                                     : kway_window_search<KIND, DESC>((const uint8_t *)gld<uint64_t>(ptr + t), lo[t],
                                                                      hi[t], vs, ts, key);
        pos += gld<uint32_t>(scan + base + j) - gld<uint32_t>(scan + base);
    }
    }
    uint8_t *d = out + (size_t)pos * vs;
    for (uint32_t o = 0; o < vs; o += 16) { // 16-byte moves (value sizes are multiples of 16)
        const uint64_t a = gld<uint64_t>(v + o), b = gld<uint64_t>(v + o + 8);
        gst<uint64_t>(d + o, a);
        gst<uint64_t>(d + o + 8, b);
    }
}

template <int KIND, bool DESC, bool LS>
static int launch_kway_t3(const uint64_t *ptr, const uint32_t *pre, const uint32_t *tile_pre, uint32_t tiles, uint32_t k,
                         uint32_t n, uint32_t vs, uint32_t ts, uint32_t *flags, uint32_t *scan, void *cub_tmp,
                         size_t cub_bytes, uint8_t *out, hipStream_t s) {
    hipLaunchKernelGGL((k_kway_flags<KIND, DESC, LS>), dim3(tiles), dim3(kKwayTile), 0, s, ptr, pre, tile_pre, k, n, vs, ts,
                       flags);
    if (hipGetLastError() != hipSuccess) return -1;
    if (hipcub::DeviceScan::ExclusiveSum(cub_tmp, cub_bytes, flags, scan, (int)n + 1, s) != hipSuccess) return -1;
    hipLaunchKernelGGL((k_kway_scatter<KIND, DESC, LS>), dim3(tiles), dim3(kKwayTile), 0, s, ptr, pre, tile_pre, k, vs, ts,
                       flags, scan, out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

template <int KIND, bool DESC>
static int launch_kway_t(const uint64_t *ptr, const uint32_t *pre, const uint32_t *tile_pre, uint32_t tiles, uint32_t k,
                         uint32_t n, uint32_t vs, uint32_t ts, uint32_t *flags, uint32_t *scan, void *cub_tmp,
                         size_t cub_bytes, uint8_t *out, hipStream_t s) {
    // Few streams: dependent searches with early exit measured faster (8
    // streams); 9..16 streams: lockstep bisection (16: 13.6 -> 8.3 ms).
    if (k > 8 && k <= (uint32_t)kKwayLockstep)
        return launch_kway_t3<KIND, DESC, true>(ptr, pre, tile_pre, tiles, k, n, vs, ts, flags, scan, cub_tmp,
                                                cub_bytes, out, s);
    return launch_kway_t3<KIND, DESC, false>(ptr, pre, tile_pre, tiles, k, n, vs, ts, flags, scan, cub_tmp, cub_bytes,
                                             out, s);
}

size_t kway_scan_tmp_bytes(uint32_t n) {
    size_t bytes = 0;
    hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr, (int)n + 1);
    return bytes;
}

int launch_kway(uint32_t key_kind, bool descending, const uint64_t *ptr, const uint32_t *pre, const uint32_t *tile_pre,
                uint32_t tiles, uint32_t k, uint32_t n, uint32_t vs, uint32_t ts, uint32_t *flags, uint32_t *scan,
                void *cub_tmp, size_t cub_bytes, uint8_t *out, void *stream) {
    hipStream_t s = (hipStream_t)stream;
#define TBC_KWAY(KIND)                                                                                    \
    return descending ? launch_kway_t<KIND, true>(ptr, pre, tile_pre, tiles, k, n, vs, ts, flags, scan, cub_tmp, cub_bytes, out, s) \
                      : launch_kway_t<KIND, false>(ptr, pre, tile_pre, tiles, k, n, vs, ts, flags, scan, cub_tmp, cub_bytes, out, s)
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
