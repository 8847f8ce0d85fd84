// kway.hip — the scan path's k-way merge, data-parallel.
//
// The reference (src/lsm/k_way_merge.zig:8-205, KWayMergeIteratorType) pops
// the k sorted streams through a binary heap; among equal keys the stream
// with precedence wins (`ordered`, :197-203) and `pop` discards every later
// value whose key equals the last one popped (:91-107). With the precedence
// of the reference's own tests (stream_precedence(a, b) = a > b, :239-244:
// higher streams win), take the merged order "key, then higher stream first,
// then position in the stream": the reference emits exactly the values whose
// key differs from the previous value's in that order.
//
// That rule composes: merging two already-merged groups of streams (the
// higher group first on equal keys) and emitting on a key change gives the
// merge of all their streams. So k streams are merged as a pairwise tree,
// ceil(log2 k) levels, every pair of a level in the same launches:
//   k_kpair_partition  merge-path split of every 2,048-position tile;
//   k_kpair_tile       per tile: the keys of both sides in LDS, each thread
//                      merges 8 positions and sets their side and emit bits,
//                      and the tile's emitted count;
//   k_kpair_scan       per pair: tile offsets, and the pair's output count
//                      (on the device: the next level reads it there);
//   k_kpair_scatter    the emitted values, 16 bytes per lane.
// Each level reads every value once for keys and once for the copy and
// writes its output once; nothing waits on the host (the final count is
// copied back with the rest, tbc_kway_poll).
#include <hip/hip_runtime.h>

#include "keys.h"
#include "tbc.h"

namespace tbc {

constexpr uint32_t kPairTile = 2048;
constexpr uint32_t kPairThreads = 256;
constexpr uint32_t kPairPer = kPairTile / kPairThreads;      // 8 positions per thread
constexpr uint32_t kPairWords = kPairTile / 64;              // mask words per kind per tile

// One 2-way merge of a level: A is the higher-precedence side (first on
// equal keys), B the lower; counts live on the device (a previous level's
// output counts).
struct KPair {
    const uint8_t *a, *b;
    const uint32_t *na, *nb; // device counts
    uint8_t *out;
    uint32_t *n_out;         // device: emitted values
    uint32_t tile_base;      // first tile of the pair (tiles_cap tiles)
    uint32_t split_base;     // first split slot (tiles_cap + 1 slots)
    uint32_t tiles_cap;      // tiles of the pair's capacity (its counts are an upper bound)
    uint32_t pad;
};

template <int KIND, bool DESC, int KL = KeyLimbs<KIND>::value>
__device__ __forceinline__ bool kbefore(const Key<KL> &x, const Key<KL> &y) {
    return DESC ? key_lt(y, x) : key_lt(x, y);
}
template <int KIND, bool DESC, int KL = KeyLimbs<KIND>::value>
__device__ __forceinline__ bool kle(const Key<KL> &x, const Key<KL> &y) {
    return !kbefore<KIND, DESC>(y, x);
}

template <bool SPLITS>
__device__ __forceinline__ uint32_t pair_of(const KPair *pairs, uint32_t npairs, uint32_t g) {
    uint32_t lo = 0, hi = npairs - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if ((SPLITS ? pairs[mid].split_base : pairs[mid].tile_base) <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// splits[tile_base + t] = number of A values among the first t * kPairTile
// merged positions (A first on equal keys), for t = 0 .. tiles_cap.
template <int KIND, bool DESC>
__global__ __launch_bounds__(256) void k_kpair_partition(const KPair *pairs, uint32_t npairs, uint32_t total,
                                                         uint32_t vs, uint32_t ts, uint32_t *splits) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x;
    if (g >= total) return;
    const KPair P = pairs[pair_of<true>(pairs, npairs, g)];
    const uint32_t t = g - P.split_base; // 0 .. tiles_cap
    const uint32_t na = *P.na, nb = *P.nb, n = na + nb;
    const uint32_t d = t * kPairTile < n ? t * kPairTile : n;
    uint32_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (kle<KIND, DESC>(load_key<KIND>(P.a + (size_t)mid * vs, ts), load_key<KIND>(P.b + (size_t)(d - 1 - mid) * vs, ts)))
            lo = mid + 1;
        else
            hi = mid;
    }
    splits[g] = lo;
}

template <int KL> struct PairShared {
    uint64_t key[KL][kPairTile + 2];
    uint32_t wave_sums[kPairThreads / 64];
};

template <int KIND, bool DESC>
__global__ __launch_bounds__(kPairThreads) void k_kpair_tile(const KPair *pairs, uint32_t npairs, uint32_t vs,
                                                             uint32_t ts, const uint32_t *splits, uint64_t *masks,
                                                             uint32_t *tile_cnt) {
    constexpr int KL = KeyLimbs<KIND>::value;
    __shared__ PairShared<KL> sh;
    const uint32_t g = blockIdx.x, tid = threadIdx.x;
    const KPair P = pairs[pair_of<false>(pairs, npairs, g)];
    const uint32_t t = g - P.tile_base;
    const uint32_t na = *P.na, nb = *P.nb, n = na + nb;
    const uint32_t d0 = t * kPairTile;
    if (d0 >= n) { // beyond the pair's actual merge (its counts were only known on the device)
        if (tid == 0) tile_cnt[g] = 0;
        return;
    }
    const uint32_t d1 = d0 + kPairTile < n ? d0 + kPairTile : n;
    const uint32_t sb = P.split_base + t; // split slot of this tile's first boundary
    const uint32_t i0 = splits[sb], i1 = splits[sb + 1];
    const uint32_t j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t ea = i1 - i0, eb = j1 - j0;
    // LDS: A[i0 .. i1) at [0, ea), B[j0 .. j1) at [ea, ea + eb), the previous merged key at kPairTile + 1.
    // Every entry's key loaded before any is stored (a load whose use sat in
    // the same loop iteration was waited for there: kPairPer round trips in
    // sequence); entries past the tile re-read its last one.
    Key<KL> kr[kPairPer];
#pragma unroll
    for (uint32_t r = 0; r < kPairPer; r++) {
        const uint32_t e0 = tid + r * kPairThreads, e = e0 < ea + eb ? e0 : ea + eb - 1;
        const uint8_t *v = e < ea ? P.a + (size_t)(i0 + e) * vs : P.b + (size_t)(j0 + e - ea) * vs;
        kr[r] = load_key<KIND>(v, ts);
    }
#pragma unroll
    for (uint32_t r = 0; r < kPairPer; r++) {
        const uint32_t e = tid + r * kPairThreads;
        if (e < ea + eb)
#pragma unroll
            for (int l = 0; l < KL; l++) sh.key[l][e] = kr[r].l[l];
    }
    if (tid == 0) {
        // The merged predecessor of position d0 is the later of A[i0-1] and
        // B[j0-1]; only its key matters: the larger one (in merge order).
        Key<KL> pk;
        bool have = false;
        if (i0 > 0) pk = load_key<KIND>(P.a + (size_t)(i0 - 1) * vs, ts), have = true;
        if (j0 > 0) {
            const auto kb = load_key<KIND>(P.b + (size_t)(j0 - 1) * vs, ts);
            if (!have || kbefore<KIND, DESC>(pk, kb)) pk = kb;
            have = true;
        }
        const uint64_t flag = have ? 1u : 0u;
#pragma unroll
        for (int l = 0; l < KL; l++) sh.key[l][kPairTile + 1] = have ? pk.l[l] : 0;
        sh.key[0][kPairTile] = flag; // slot kPairTile holds "has a predecessor"
    }
    __syncthreads();
    auto key_at = [&](uint32_t e) {
        Key<KL> k;
#pragma unroll
        for (int l = 0; l < KL; l++) k.l[l] = sh.key[l][e];
        return k;
    };
    // This thread's positions [d, d + kPairPer) of the tile: merge-path search in LDS.
    const uint32_t tot = ea + eb;
    const uint32_t d = kPairPer * tid < tot ? kPairPer * tid : tot;
    uint32_t a, b;
    {
        uint32_t lo = d > eb ? d - eb : 0, hi = d < ea ? d : ea;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (kle<KIND, DESC>(key_at(mid), key_at(ea + d - 1 - mid))) lo = mid + 1;
            else hi = mid;
        }
        a = lo;
        b = d - lo;
    }
    // Key of the merged position before d.
    bool have_prev;
    Key<KL> prev;
    if (d == 0) {
        have_prev = sh.key[0][kPairTile] != 0;
        prev = key_at(kPairTile + 1);
    } else {
        have_prev = true;
        if (a == 0) prev = key_at(ea + b - 1);
        else if (b == 0) prev = key_at(a - 1);
        else {
            const auto ka = key_at(a - 1), kb = key_at(ea + b - 1);
            prev = kbefore<KIND, DESC>(ka, kb) ? kb : ka;
        }
    }
    uint32_t ebits = 0, abits = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPairPer; k++) {
        if (d + k >= tot) continue;
        const bool take_a = a < ea && (b >= eb || kle<KIND, DESC>(key_at(a), key_at(ea + b)));
        const auto kk = take_a ? key_at(a) : key_at(ea + b);
        const bool emit = !have_prev || !key_eq(kk, prev);
        ebits |= (emit ? 1u : 0u) << k;
        abits |= (take_a ? 1u : 0u) << k;
        if (take_a) a++;
        else b++;
        prev = kk;
        have_prev = true;
    }
    constexpr uint32_t kThreadsPerWord = 64 / kPairPer;
    const uint32_t shb = kPairPer * (tid % kThreadsPerWord);
    uint64_t ew = (uint64_t)ebits << shb, aw = (uint64_t)abits << shb;
    for (uint32_t o = 1; o < kThreadsPerWord; o <<= 1) {
        ew |= __shfl_xor(ew, o, 64);
        aw |= __shfl_xor(aw, o, 64);
    }
    uint64_t *m = masks + (size_t)g * (2 * kPairWords);
    if (tid % kThreadsPerWord == 0) {
        m[tid / kThreadsPerWord] = ew;
        m[kPairWords + tid / kThreadsPerWord] = aw;
    }
    uint32_t sum = __builtin_popcount(ebits);
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if ((tid & 63) == 0) sh.wave_sums[tid >> 6] = sum;
    __syncthreads();
    if (tid == 0) tile_cnt[g] = sh.wave_sums[0] + sh.wave_sums[1] + sh.wave_sums[2] + sh.wave_sums[3];
}

// Per pair (one workgroup): exclusive scan of its tiles' counts into
// tile_off, the pair's output count into *n_out.
constexpr uint32_t kPairScanThreads = 1024;
__global__ __launch_bounds__(kPairScanThreads) void k_kpair_scan(const KPair *pairs, const uint32_t *tile_cnt,
                                                                 uint32_t *tile_off) {
    __shared__ uint32_t wsum[kPairScanThreads / 64];
    __shared__ uint32_t carry;
    const KPair P = pairs[blockIdx.x];
    const uint32_t first = P.tile_base;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < P.tiles_cap; base += kPairScanThreads) {
        const uint32_t t = base + tid;
        const uint32_t c = t < P.tiles_cap ? tile_cnt[first + t] : 0u;
        uint32_t incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += y;
        }
        if (lane == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        uint32_t off = carry;
        for (uint32_t w = 0; w < (tid >> 6); w++) off += wsum[w];
        if (t < P.tiles_cap) tile_off[first + t] = off + incl - c;
        __syncthreads();
        if (tid == kPairScanThreads - 1) carry = off + incl;
        __syncthreads();
    }
    if (tid == 0) *P.n_out = carry;
}

__global__ __launch_bounds__(kPairThreads) void k_kpair_scatter(const KPair *pairs, uint32_t npairs, uint32_t vs,
                                                                const uint32_t *splits, const uint64_t *masks,
                                                                const uint32_t *tile_off) {
    __shared__ uint32_t s_pre[3][kPairWords + 1]; // emitted, A taken, B taken before word w
    __shared__ uint64_t s_src[4][64], s_dst[4][64];
    const uint32_t g = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const KPair P = pairs[pair_of<false>(pairs, npairs, g)];
    const uint32_t t = g - P.tile_base;
    const uint32_t na = *P.na, nb = *P.nb, n = na + nb;
    const uint32_t d0 = t * kPairTile;
    if (d0 >= n) return;
    const uint32_t i0 = splits[P.split_base + t], j0 = d0 - i0;
    const uint64_t *m = masks + (size_t)g * (2 * kPairWords);
    auto valid_of = [&](uint32_t w) -> uint64_t {
        const uint32_t pos0 = d0 + 64 * w;
        return pos0 >= n ? 0ull : (n - pos0 >= 64 ? ~0ull : ((1ull << (n - pos0)) - 1));
    };
    if (tid < kPairWords) {
        const uint64_t em = m[tid], am = m[kPairWords + tid];
        s_pre[0][tid + 1] = __builtin_popcountll(em);
        s_pre[1][tid + 1] = __builtin_popcountll(am);
        s_pre[2][tid + 1] = __builtin_popcountll(valid_of(tid) & ~am);
    }
    __syncthreads();
    if (tid < 3) {
        uint32_t acc = 0;
        s_pre[tid][0] = 0;
        for (uint32_t w = 1; w <= kPairWords; w++) {
            acc += s_pre[tid][w];
            s_pre[tid][w] = acc;
        }
    }
    __syncthreads();
    const uint32_t out0 = tile_off[g];
    const uint32_t cpv = vs >> 4;
    const uint64_t lt = (1ull << lane) - 1;
    for (uint32_t w = wv; w < kPairWords; w += 4) {
        if (d0 + 64 * w >= n) break;
        const uint64_t em = m[w], am = m[kPairWords + w];
        const uint32_t ns = __builtin_popcountll(em);
        if (ns == 0) continue;
        const uint64_t valid = valid_of(w);
        if ((em >> lane) & 1) {
            const uint32_t r = __builtin_popcountll(em & lt);
            const bool from_a = (am >> lane) & 1;
            const uint8_t *src = from_a ? P.a + (size_t)(i0 + s_pre[1][w] + __builtin_popcountll(am & lt)) * vs
                                        : P.b + (size_t)(j0 + s_pre[2][w] + __builtin_popcountll(valid & ~am & lt)) * vs;
            s_src[wv][r] = (uint64_t)(uintptr_t)src;
            s_dst[wv][r] = (uint64_t)(uintptr_t)(P.out + (size_t)(out0 + s_pre[0][w] + r) * vs);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const uint32_t total = ns * cpv;
        for (uint32_t c0 = 0; c0 < total; c0 += 64 * 4) {
            u32x4 v[4];
#pragma unroll
            for (uint32_t u = 0; u < 4; u++) {
                const uint32_t c = c0 + lane + 64 * u < total ? c0 + lane + 64 * u : total - 1; // loads unconditional
                v[u] = gld<u32x4>((const uint8_t *)(uintptr_t)s_src[wv][c / cpv] + 16 * (c % cpv));
            }
#pragma unroll
            for (uint32_t u = 0; u < 4; u++) {
                const uint32_t c = c0 + lane + 64 * u;
                if (c < total) gst<u32x4>((uint8_t *)(uintptr_t)s_dst[wv][c / cpv] + 16 * (c % cpv), v[u]);
            }
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    }
}

// Every level's launches for `npairs` pairs whose descriptors are on the
// device; split slots: tiles_cap + 1 per pair; tiles: tiles_cap per pair.
template <int KIND, bool DESC>
static int launch_level_t(const KPair *d_pairs, uint32_t npairs, uint32_t slots, uint32_t tiles, uint32_t vs,
                          uint32_t ts, uint32_t *splits, uint64_t *masks, uint32_t *tile_cnt, uint32_t *tile_off,
                          hipStream_t s) {
    hipLaunchKernelGGL((k_kpair_partition<KIND, DESC>), dim3((slots + 255) / 256), dim3(256), 0, s, d_pairs, npairs,
                       slots, vs, ts, splits);
    hipLaunchKernelGGL((k_kpair_tile<KIND, DESC>), dim3(tiles), dim3(kPairThreads), 0, s, d_pairs, npairs, vs, ts,
                       (const uint32_t *)splits, masks, tile_cnt);
    hipLaunchKernelGGL(k_kpair_scan, dim3(npairs), dim3(kPairScanThreads), 0, s, d_pairs, (const uint32_t *)tile_cnt,
                       tile_off);
    hipLaunchKernelGGL(k_kpair_scatter, dim3(tiles), dim3(kPairThreads), 0, s, d_pairs, npairs, vs,
                       (const uint32_t *)splits, (const uint64_t *)masks, (const uint32_t *)tile_off);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_kway_level(uint32_t key_kind, bool descending, const void *d_pairs, uint32_t npairs, uint32_t slots,
                      uint32_t tiles, uint32_t vs, uint32_t ts, uint32_t *splits, uint64_t *masks, uint32_t *tile_cnt,
                      uint32_t *tile_off, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    const KPair *P = (const KPair *)d_pairs;
#define TBC_KWAY(KIND)                                                                                             \
    return descending ? launch_level_t<KIND, true>(P, npairs, slots, tiles, vs, ts, splits, masks, tile_cnt, tile_off, s) \
                      : launch_level_t<KIND, false>(P, npairs, slots, tiles, vs, ts, splits, masks, tile_cnt, tile_off, s)
    switch (key_kind) {
    case kKeyTimestamp: TBC_KWAY(kKeyTimestamp);
    case kKeyIdU128: TBC_KWAY(kKeyIdU128);
    case kKeyCompositeU64: TBC_KWAY(kKeyCompositeU64);
    case kKeyCompositeU128: TBC_KWAY(kKeyCompositeU128);
    default: return -1;
    }
#undef TBC_KWAY
}

uint32_t kway_pair_tile() { return kPairTile; }
uint32_t kway_pair_bytes() { return sizeof(KPair); }

} // namespace tbc
