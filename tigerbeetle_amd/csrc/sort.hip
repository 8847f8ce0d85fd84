// sort.hip — TableMemory.sort (src/lsm/table_memory.zig:140-154) on gfx950.
//
// The reference sorts the mutable table's Values with std.mem.sort (Zig 0.11
// stable block sort) by key_from_value, only when puts arrived out of order
// (table_memory.zig:83-87). Stability is load-bearing: fill_immutable_values
// keeps the LAST of a run of equal keys (compaction.zig:519-522).
//
// A batch of memtables (every tree's at the bar end) is sorted by one
// enqueued launch sequence that never waits on the host:
//
//   k_sort_extract  per tile of 2,048 items: key limbs (limb-major) and item
//                   indices, a copy of the values (the gather's source),
//                   OR/AND of the keys, per-table sortedness, and the 8-bit
//                   digit histograms of every pass, per table;
//   k_sort_plan     per table: which passes move anything (a digit that is
//                   constant over the batch cannot reorder), each pass's
//                   source buffer, and every digit's start in its table;
//   k_sort_pass x P one launch per potential pass (P = 8 per key limb); an
//                   inactive pass returns at once. Onesweep: each tile ranks
//                   its items by digit (wave match ballots + per-wave counts:
//                   stable), publishes its digit counts, looks back over the
//                   tiles before it in its table for their prefix (decoupled
//                   look-back, one 32-bit flag|count word per tile and digit),
//                   and writes the tile out through LDS so each digit's run
//                   is contiguous;
//   k_sort_gather   values[i] = copy[idx[i]] for tables that were unsorted.
//
// Tiles never straddle tables, so a table's passes are independent of the
// others' (a segmented sort with no table digit). Tables whose puts arrived
// in order are left untouched (table_memory.zig:141).
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "tbc_internal.h"

namespace tbc {

constexpr uint32_t kSortThreads = 256;
constexpr uint32_t kSortWaves = kSortThreads / 64;
constexpr uint32_t kSortRounds = 8;
constexpr uint32_t kSortTile = kSortThreads * kSortRounds; // 2,048 items
constexpr uint32_t kRadix = 256;
constexpr uint32_t kMaxLimbs = 3;
constexpr uint32_t kMaxPasses = 8 * kMaxLimbs;

// Look-back words: flag in the top two bits, count below (counts < 2^30).
constexpr uint32_t kFlagAggregate = 1u << 30;
constexpr uint32_t kFlagPrefix = 2u << 30;
constexpr uint32_t kCountMask = (1u << 30) - 1;

struct SortSeg {
    uint8_t *values;
    uint8_t *copy; // n * vs bytes: the table as put, the gather's source
    uint32_t n, vs, ts_off, kind;
    uint32_t item_base, tile_base, tiles, unsorted;
};

struct SortPlan {
    uint64_t key_or[kMaxLimbs], key_and[kMaxLimbs];
    uint32_t active[kMaxPasses]; // pass moves items
    uint32_t src[kMaxPasses];    // ping-pong buffer the pass reads
    uint32_t final_buf;          // buffer holding the sorted indices
    uint32_t kl;                 // key limbs of the batch
    uint32_t any_unsorted;
};

__device__ __forceinline__ void key_of(uint32_t kind, const uint8_t *v, uint32_t ts_off, uint64_t k[3]) {
    k[1] = k[2] = 0;
    switch (kind) {
    case kKeyTimestamp: k[0] = gld<uint64_t>(v + ts_off) & ~kTombstoneBit; break;
    case kKeyIdU128: k[0] = gld<uint64_t>(v); k[1] = gld<uint64_t>(v + 8); break;
    case kKeyCompositeU64: k[0] = gld<uint64_t>(v + 8) & ~kTombstoneBit; k[1] = gld<uint64_t>(v); break;
    default: k[0] = gld<uint64_t>(v + 16) & ~kTombstoneBit; k[1] = gld<uint64_t>(v); k[2] = gld<uint64_t>(v + 8); break;
    }
}

// hist layout: [segment][pass][digit] u32.
__device__ __forceinline__ uint32_t *seg_hist(uint32_t *hist, uint32_t s) { return hist + (size_t)s * kMaxPasses * kRadix; }

// --------------------------------------------------------------------------
// Extract: one workgroup per tile.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kSortThreads) void k_sort_extract(SortSeg *segs, const uint32_t *tile_seg, uint32_t kl,
                                                               uint32_t N, uint64_t *keys, uint32_t *idx,
                                                               SortPlan *plan, uint32_t *hist) {
    __shared__ uint32_t s_hist[kMaxPasses * kRadix];
    __shared__ uint64_t s_or[kMaxLimbs][kSortWaves], s_and[kMaxLimbs][kSortWaves];
    __shared__ uint32_t s_uns;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t sg = tile_seg[blockIdx.x];
    const SortSeg S = segs[sg];
    const uint32_t lt = blockIdx.x - S.tile_base;
    for (uint32_t i = tid; i < 8 * kl * kRadix; i += kSortThreads) s_hist[i] = 0;
    if (tid == 0) s_uns = 0;
    __syncthreads();
    uint64_t o[kMaxLimbs] = {0, 0, 0}, a[kMaxLimbs] = {~0ull, ~0ull, ~0ull};
    uint32_t uns = 0;
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint32_t li = lt * kSortTile + r * kSortThreads + tid;
        if (lt * kSortTile + r * kSortThreads >= S.n) break; // wave-uniform (whole row past the end)
        const bool in = li < S.n;
        const uint32_t i = S.item_base + li;
        uint64_t k[3] = {0, 0, 0}, kn[3];
        if (in) key_of(S.kind, S.values + (size_t)li * S.vs, S.ts_off, k);
        // The next item's key comes from the next lane; lane 63 reads its neighbour.
        for (uint32_t l = 0; l < 3; l++) kn[l] = __shfl_down(k[l], 1, 64);
        if (lane == 63 && li + 1 < S.n) key_of(S.kind, S.values + (size_t)(li + 1) * S.vs, S.ts_off, kn);
        if (!in) continue;
        for (uint32_t q = 0; q < S.vs; q += 16)
            gst<u32x4>(S.copy + (size_t)li * S.vs + q, gld<u32x4>(S.values + (size_t)li * S.vs + q));
        for (uint32_t l = 0; l < kl; l++) {
            keys[(size_t)l * N + i] = k[l];
            o[l] |= k[l];
            a[l] &= k[l];
            for (uint32_t b = 0; b < 8; b++) atomicAdd(&s_hist[(8 * l + b) * kRadix + ((k[l] >> (8 * b)) & 255)], 1u);
        }
        idx[i] = i;
        if (li + 1 < S.n) {
            bool gt = false, decided = false;
            for (int l = (int)kl - 1; l >= 0 && !decided; l--) {
                if (k[l] != kn[l]) {
                    gt = k[l] > kn[l];
                    decided = true;
                }
            }
            uns |= gt ? 1u : 0u;
        }
    }
    for (uint32_t l = 0; l < kMaxLimbs; l++) {
        for (int off = 32; off > 0; off >>= 1) {
            o[l] |= __shfl_xor(o[l], off, 64);
            a[l] &= __shfl_xor(a[l], off, 64);
        }
        if (lane == 0) {
            s_or[l][wave] = o[l];
            s_and[l][wave] = a[l];
        }
    }
    if (uns) atomicOr(&s_uns, 1u);
    __syncthreads();
    uint32_t *h = seg_hist(hist, sg);
    for (uint32_t i = tid; i < 8 * kl * kRadix; i += kSortThreads)
        if (s_hist[i]) atomicAdd(&h[i], s_hist[i]);
    if (tid < kl) {
        uint64_t oo = 0, aa = ~0ull;
        for (uint32_t w = 0; w < kSortWaves; w++) {
            oo |= s_or[tid][w];
            aa &= s_and[tid][w];
        }
        atomicOr((unsigned long long *)&plan->key_or[tid], (unsigned long long)oo);
        atomicAnd((unsigned long long *)&plan->key_and[tid], (unsigned long long)aa);
    }
    if (tid == 0 && s_uns) {
        atomicOr(&segs[sg].unsorted, 1u);
        atomicOr(&plan->any_unsorted, 1u);
    }
}

// --------------------------------------------------------------------------
// Plan: one workgroup per table (block 0 also fills the batch-wide plan).
// bins[segment][pass][digit] = the digit's first item in the global item
// space (table base + exclusive prefix of the table's histogram).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kRadix) void k_sort_plan(const SortSeg *segs, SortPlan *plan, const uint32_t *hist,
                                                      uint32_t *bins) {
    const uint32_t s = blockIdx.x, d = threadIdx.x, lane = d & 63, wave = d >> 6;
    __shared__ uint32_t wsum[kRadix / 64];
    const uint32_t kl = plan->kl;
    if (s == 0 && d == 0) {
        uint32_t buf = 0;
        for (uint32_t p = 0; p < kMaxPasses; p++) {
            const uint32_t l = p >> 3;
            const bool act = l < kl && plan->any_unsorted &&
                             (((plan->key_or[l] ^ plan->key_and[l]) >> (8 * (p & 7))) & 255) != 0;
            plan->active[p] = act ? 1u : 0u;
            plan->src[p] = buf;
            if (act) buf ^= 1u;
        }
        plan->final_buf = buf;
    }
    const uint32_t *h = hist + (size_t)s * kMaxPasses * kRadix;
    uint32_t *out = bins + (size_t)s * kMaxPasses * kRadix;
    for (uint32_t p = 0; p < 8 * kl; p++) {
        const uint32_t c = h[p * kRadix + d];
        uint32_t incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += y;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (uint32_t w = 0; w < wave; w++) off += wsum[w];
        out[p * kRadix + d] = segs[s].item_base + off + incl - c;
        __syncthreads();
    }
}

// --------------------------------------------------------------------------
// One onesweep pass (digit = byte `p & 7` of limb `p >> 3`).
// --------------------------------------------------------------------------
__device__ __forceinline__ uint32_t lb_load(const uint32_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint32_t *p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <uint32_t KL>
__global__ __launch_bounds__(kSortThreads) void k_sort_pass(const SortSeg *segs, const uint32_t *tile_seg,
                                                            const SortPlan *plan, uint32_t p, uint32_t ntiles,
                                                            uint32_t N, uint64_t *keys0, uint64_t *keys1,
                                                            uint32_t *idx0, uint32_t *idx1, const uint32_t *bins,
                                                            uint32_t *status, uint32_t *tile_counter) {
    if (!plan->active[p]) return; // uniform: a constant digit cannot reorder anything
    __shared__ uint32_t s_tile;
    __shared__ uint32_t s_wcnt[kSortWaves][kRadix]; // per wave: running, then total counts
    __shared__ uint32_t s_start[kRadix];            // local start of each digit in the tile
    __shared__ uint32_t s_excl[kRadix];             // items of the digit in the table's earlier tiles
    __shared__ uint64_t s_key[KL][kSortTile];
    __shared__ uint32_t s_idx[kSortTile];
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // Dynamic tile ids in arrival order: every tile a workgroup looks back on
    // was taken by a workgroup that is running or done (forward progress).
    if (tid == 0) s_tile = atomicAdd(&tile_counter[p], 1u);
    for (uint32_t i = tid; i < kSortWaves * kRadix; i += kSortThreads) (&s_wcnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t t = s_tile;
    if (t >= ntiles) return;
    const uint32_t sg = tile_seg[t];
    const SortSeg S = segs[sg];
    if (!S.unsorted) return; // tables put in order are left as they are
    const uint32_t lt = t - S.tile_base;
    const uint32_t base = S.item_base + lt * kSortTile;
    const uint32_t m = (S.n - lt * kSortTile) < kSortTile ? (S.n - lt * kSortTile) : kSortTile;
    const uint32_t limb = p >> 3, shift = 8 * (p & 7);
    const uint32_t live = plan->kl - limb; // limbs [limb, kl) still move with the items
    const uint64_t *ksrc = plan->src[p] ? keys1 : keys0;
    uint64_t *kdst = plan->src[p] ? keys0 : keys1;
    const uint32_t *isrc = plan->src[p] ? idx1 : idx0;
    uint32_t *idst = plan->src[p] ? idx0 : idx1;

    // Wave w owns items [512 w, 512 w + 512) of the tile, 64 per round in
    // lane order: stable rank = (earlier waves) + (earlier rounds of this
    // wave, counted in s_wcnt) + (earlier lanes with the same digit).
    const uint64_t lt_mask = (1ull << lane) - 1;
    uint32_t rank[kSortRounds], dig[kSortRounds];
    uint64_t k[kSortRounds][KL];
    uint32_t ix[kSortRounds];
#pragma unroll
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint32_t e = wave * (64 * kSortRounds) + r * 64 + lane;
        const bool in = e < m;
#pragma unroll
        for (uint32_t l = 0; l < KL; l++)
            k[r][l] = in && l < live ? gld<uint64_t>(ksrc + (size_t)(limb + l) * N + base + e) : 0ull;
        ix[r] = in ? gld<uint32_t>(isrc + base + e) : 0u;
        const uint32_t d = in ? (uint32_t)(k[r][0] >> shift) & 255u : 0u;
        dig[r] = d;
        uint64_t peers = __ballot(in);
#pragma unroll
        for (uint32_t b = 0; b < 8; b++) {
            const uint64_t bal = __ballot((d >> b) & 1u);
            peers &= ((d >> b) & 1u) ? bal : ~bal;
        }
        const uint32_t before = __builtin_popcountll(peers & lt_mask);
        const uint32_t prior = in ? s_wcnt[wave][d] : 0u;
        __builtin_amdgcn_wave_barrier();
        if (in && before == 0) s_wcnt[wave][d] = prior + (uint32_t)__builtin_popcountll(peers);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        rank[r] = prior + before;
    }
    __syncthreads();
    // Per digit (thread d): counts of the tile, exclusive prefix over waves,
    // and the tile-local start (exclusive scan over digits).
    const uint32_t d = tid;
    uint32_t cnt = 0, wpre[kSortWaves];
#pragma unroll
    for (uint32_t w = 0; w < kSortWaves; w++) {
        wpre[w] = cnt;
        cnt += s_wcnt[w][d];
    }
    {
        uint32_t incl = cnt;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += y;
        }
        __shared__ uint32_t s_wsum[kSortWaves];
        if (lane == 63) s_wsum[wave] = incl;
        __syncthreads();
        uint32_t off = 0;
        for (uint32_t w = 0; w < wave; w++) off += s_wsum[w];
        s_start[d] = off + incl - cnt;
    }
    __syncthreads();
#pragma unroll
    for (uint32_t w = 0; w < kSortWaves; w++) s_wcnt[w][d] = wpre[w]; // becomes the wave's offset
    // Decoupled look-back over the table's earlier tiles, one digit per thread.
    uint32_t *st = status + (size_t)p * ntiles * kRadix;
    uint32_t excl = 0;
    if (lt == 0) {
        lb_store(&st[(size_t)t * kRadix + d], kFlagPrefix | cnt);
    } else {
        lb_store(&st[(size_t)t * kRadix + d], kFlagAggregate | cnt);
        uint32_t pred = t - 1;
        for (uint32_t spins = 0;;) {
            const uint32_t v = lb_load(&st[(size_t)pred * kRadix + d]);
            if ((v & ~kCountMask) == 0) { // not published yet
                if (++spins > (1u << 26)) break; // bounded (a broken invariant, not a hang)
                __builtin_amdgcn_s_sleep(1);
                continue;
            }
            excl += v & kCountMask;
            if ((v & ~kCountMask) == kFlagPrefix || pred == S.tile_base) break;
            pred--;
        }
        lb_store(&st[(size_t)t * kRadix + d], kFlagPrefix | (excl + cnt));
    }
    s_excl[d] = excl;
    __syncthreads();
    // Items into LDS at their tile-local sorted position.
#pragma unroll
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint32_t e = wave * (64 * kSortRounds) + r * 64 + lane;
        if (e < m) {
            const uint32_t pos = s_start[dig[r]] + s_wcnt[wave][dig[r]] + rank[r];
#pragma unroll
            for (uint32_t l = 0; l < KL; l++) s_key[l][pos] = k[r][l];
            s_idx[pos] = ix[r];
        }
    }
    __syncthreads();
    // Out in that order: each digit's run lands contiguously.
    const uint32_t *bin = bins + ((size_t)sg * kMaxPasses + p) * kRadix;
    for (uint32_t j = tid; j < m; j += kSortThreads) {
        const uint32_t dj = (uint32_t)(s_key[0][j] >> shift) & 255u;
        const uint32_t dst = bin[dj] + s_excl[dj] + (j - s_start[dj]);
#pragma unroll
        for (uint32_t l = 0; l < KL; l++)
            if (l < live) gst<uint64_t>(kdst + (size_t)(limb + l) * N + dst, s_key[l][j]);
        gst<uint32_t>(idst + dst, s_idx[j]);
    }
}

// values[i] = copy[idx[i]] (table-local), 16 bytes per lane; sorted tables
// are left alone.
__global__ __launch_bounds__(256) void k_sort_gather(const SortSeg *segs, const uint32_t *tile_seg,
                                                     const SortPlan *plan, const uint32_t *idx0,
                                                     const uint32_t *idx1) {
    const SortSeg S = segs[tile_seg[blockIdx.x]];
    if (!S.unsorted) return;
    const uint32_t *idx = plan->final_buf ? idx1 : idx0;
    const uint32_t lt = blockIdx.x - S.tile_base;
    const uint32_t first = lt * kSortTile;
    const uint32_t m = (S.n - first) < kSortTile ? (S.n - first) : kSortTile;
    const uint32_t cpv = S.vs >> 4;
    for (uint32_t c = threadIdx.x; c < m * cpv; c += 256) {
        const uint32_t e = c / cpv, part = c % cpv;
        const uint32_t src = gld<uint32_t>(idx + S.item_base + first + e) - S.item_base;
        gst<u32x4>(S.values + (size_t)(first + e) * S.vs + 16 * part,
                   gld<u32x4>(S.copy + (size_t)src * S.vs + 16 * part));
    }
}

static uint32_t key_limbs(uint32_t kind) { return kind == kKeyTimestamp ? 1 : kind == kKeyCompositeU128 ? 3 : 2; }

static uint64_t tiles_of(uint32_t n) { return (n + kSortTile - 1) / kSortTile; }
static uint64_t align256(uint64_t x) { return (x + 255) / 256 * 256; }

// Scratch layout (sort_scratch_bytes must match launch_sort_batch).
struct SortScratch {
    uint64_t plan, segs, tile_seg, keys, idx, hist, bins, status, counters, copies, total;
};

static SortScratch scratch_layout(const SortItem *items, uint32_t count) {
    uint64_t N = 0, tiles = 0, vals = 0, nseg = 0, kl = 1;
    for (uint32_t j = 0; j < count; j++) {
        if (items[j].n < 2) continue;
        N += items[j].n;
        tiles += tiles_of(items[j].n);
        vals += align256((uint64_t)items[j].n * items[j].value_size);
        nseg++;
        kl = kl > key_limbs(items[j].key_kind) ? kl : key_limbs(items[j].key_kind);
    }
    SortScratch s;
    uint64_t o = 0;
    s.plan = o;
    o += align256(sizeof(SortPlan));
    s.segs = o;
    o += align256(sizeof(SortSeg) * count);
    s.tile_seg = o;
    o += align256(4 * tiles);
    s.keys = o;
    o += 2 * align256(8 * N * kl);
    s.idx = o;
    o += 2 * align256(4 * N);
    s.hist = o;
    o += align256(4ull * nseg * kMaxPasses * kRadix);
    s.bins = o;
    o += align256(4ull * nseg * kMaxPasses * kRadix);
    s.status = o;
    o += align256(4ull * 8 * kl * tiles * kRadix);
    s.counters = o;
    o += align256(4ull * kMaxPasses);
    s.copies = o;
    o += vals;
    s.total = o;
    return s;
}

uint64_t sort_scratch_bytes(const SortItem *items, uint32_t count) { return scratch_layout(items, count).total; }

// Everything is enqueued on `stream`; the host never waits. The plan, table
// descriptors and tile map go through the caller's pinned staging (`host`,
// at least sort_host_bytes) which must stay untouched until the stream has
// passed this batch.
uint64_t sort_host_bytes(const SortItem *items, uint32_t count) {
    const SortScratch s = scratch_layout(items, count);
    return s.keys; // plan + segs + tile map
}

int launch_sort_batch(const SortItem *items, uint32_t count, void *scratch, uint64_t scratch_bytes, void *host,
                      void *stream) {
    const SortScratch L = scratch_layout(items, count);
    if (scratch_bytes < L.total) return -1;
    hipStream_t s = (hipStream_t)stream;
    uint8_t *base = (uint8_t *)scratch, *hbase = (uint8_t *)host;
    SortPlan *hplan = (SortPlan *)(hbase + L.plan);
    SortSeg *hsegs = (SortSeg *)(hbase + L.segs);
    uint32_t *htile = (uint32_t *)(hbase + L.tile_seg);
    uint32_t N = 0, kl = 1, nseg = 0, ntiles = 0;
    uint64_t copy_off = L.copies;
    for (uint32_t j = 0; j < count; j++) {
        const SortItem &it = items[j];
        if (it.n < 2) continue;
        SortSeg g{};
        g.values = (uint8_t *)it.values;
        g.copy = base + copy_off;
        copy_off += align256((uint64_t)it.n * it.value_size);
        g.n = it.n;
        g.vs = it.value_size;
        g.ts_off = it.timestamp_offset;
        g.kind = it.key_kind;
        g.item_base = N;
        g.tile_base = ntiles;
        g.tiles = (uint32_t)tiles_of(it.n);
        for (uint32_t t = 0; t < g.tiles; t++) htile[ntiles + t] = nseg;
        ntiles += g.tiles;
        N += it.n;
        kl = kl > key_limbs(it.key_kind) ? kl : key_limbs(it.key_kind);
        hsegs[nseg++] = g;
    }
    if (!nseg) return 0;
    memset(hplan, 0, sizeof(SortPlan));
    for (uint32_t l = 0; l < kMaxLimbs; l++) hplan->key_and[l] = ~0ull;
    hplan->kl = kl;
    SortPlan *plan = (SortPlan *)(base + L.plan);
    SortSeg *d_segs = (SortSeg *)(base + L.segs);
    uint32_t *d_tile = (uint32_t *)(base + L.tile_seg);
    uint64_t *keys0 = (uint64_t *)(base + L.keys), *keys1 = (uint64_t *)(base + L.keys + align256(8ull * N * kl));
    uint32_t *idx0 = (uint32_t *)(base + L.idx), *idx1 = (uint32_t *)(base + L.idx + align256(4ull * N));
    uint32_t *hist = (uint32_t *)(base + L.hist), *bins = (uint32_t *)(base + L.bins);
    uint32_t *status = (uint32_t *)(base + L.status), *counters = (uint32_t *)(base + L.counters);
    // Histograms, look-back words and tile counters start at zero.
    if (hipMemcpyAsync(base, hbase, L.keys, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(hist, 0, L.copies - L.hist, s) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_sort_extract, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile, kl, N, keys0, idx0,
                       plan, hist);
    hipLaunchKernelGGL(k_sort_plan, dim3(nseg), dim3(kRadix), 0, s, d_segs, plan, hist, bins);
    for (uint32_t p = 0; p < 8 * kl; p++) {
        switch (kl - (p >> 3)) { // limbs still moving in this pass
        case 1:
            hipLaunchKernelGGL(k_sort_pass<1>, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile, plan, p, ntiles,
                               N, keys0, keys1, idx0, idx1, bins, status, counters);
            break;
        case 2:
            hipLaunchKernelGGL(k_sort_pass<2>, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile, plan, p, ntiles,
                               N, keys0, keys1, idx0, idx1, bins, status, counters);
            break;
        default:
            hipLaunchKernelGGL(k_sort_pass<3>, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile, plan, p, ntiles,
                               N, keys0, keys1, idx0, idx1, bins, status, counters);
            break;
        }
    }
    hipLaunchKernelGGL(k_sort_gather, dim3(ntiles), dim3(256), 0, s, d_segs, d_tile, plan, idx0, idx1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace tbc
