// sort.hip — TableMemory.sort (src/lsm/table_memory.zig:140-154) on gfx950.
//
// The reference sorts the mutable table's Values with std.mem.sort (Zig 0.11
// stable block sort) by key_from_value, only when puts arrived out of order
// (table_memory.zig:83-87). Stability is load-bearing: fill_immutable_values
// keeps the LAST of a run of equal keys (compaction.zig:519-522).
//
// A batch of memtables (every tree's at the bar end) is sorted by ONE
// launch sequence (segmented: tiles never straddle memtables).
// Here: a stable LSD radix sort of (key limbs, original index) items with
// 4-bit digits, skipping every digit that is constant across the table (one
// probe pass computes OR/AND of all keys and the sortedness flag), then one
// gather of the Values by original index. Per pass:
//   hist    — per-tile digit counts (16 bins x tiles, digit-major);
//   scan    — exclusive scan of the [table][digit][tile] counts (chunk sums,
//             their scan, chunk rescans: three short coalesced launches);
//   scatter — each tile is staged through LDS so every thread owns 8
//             consecutive items, per-thread digit counts are scanned across
//             the tile in digit-major order, and items are written to
//             (tile offset of digit) + (rank among earlier same-digit items):
//             stable by construction.
#include <hip/hip_runtime.h>

#include <vector>

#include "tbc_internal.h"

namespace tbc {

constexpr uint32_t kSortThreads = 256;
constexpr uint32_t kSortPer = 8;
constexpr uint32_t kSortTile = kSortThreads * kSortPer; // 2048 items per tile
constexpr uint32_t kDigitBits = 4;
constexpr uint32_t kBins = 1u << kDigitBits;

struct SortProbe {
    uint64_t or_[4];
    uint64_t and_[4];
};
// Workgroups fold their OR/AND into one of kProbeBuckets probes (one hot
// address per limb serialised thousands of atomics in L2); the host folds
// the buckets.
constexpr uint32_t kProbeBuckets = 64;

// One memtable of the batch. Items of all segments live in one global item
// space (segment s at [item_base, item_base + n)); tiles never straddle a
// segment, so every tile knows its segment and the digit-major histograms of
// a segment are contiguous: ONE exclusive scan over [segment][digit][tile]
// yields global, segment-grouped destinations (a segmented stable sort with
// no segment digit).
struct SortSeg {
    uint8_t *values;
    uint8_t *scratch; // n * vs bytes: the unsorted table, the gather's source
    uint32_t n, vs, ts_off, kind;
    uint32_t item_base, tile_base, tiles, unsorted;
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

// One workgroup per tile: extract keys (limb-major, global item positions)
// and item indices; OR/AND of all keys; per-segment sortedness
// (table_memory.zig:83-87 tracks it on put; here it is recomputed).
__global__ __launch_bounds__(256) void k_sort_extract(SortSeg *segs, const uint32_t *tile_seg, uint32_t kl,
                                                      uint32_t N, uint64_t *keys, uint32_t *idx, SortProbe *probe) {
    __shared__ uint64_t s_or[3][4], s_and[3][4];
    __shared__ uint32_t s_uns;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t sg = tile_seg[blockIdx.x];
    const SortSeg S = segs[sg];
    const uint32_t lt = blockIdx.x - S.tile_base;
    if (tid == 0) s_uns = 0;
    uint64_t o[3] = {0, 0, 0}, a[3] = {~0ull, ~0ull, ~0ull};
    uint32_t uns = 0;
    for (uint32_t r = 0; r < kSortPer; r++) {
        const uint32_t li = lt * kSortTile + r * kSortThreads + tid;
        if (lt * kSortTile + r * kSortThreads >= S.n) break; // wave-uniform (whole row past the end)
        const bool in = li < S.n;
        const uint32_t i = S.item_base + li;
        uint64_t k[3] = {0, 0, 0}, kn[3];
        if (in) key_of(S.kind, S.values + (size_t)li * S.vs, S.ts_off, k);
        // The next item's key comes from the next lane (one value read per
        // item); lane 63 reads its neighbour itself.
        for (uint32_t l = 0; l < 3; l++) kn[l] = __shfl_down(k[l], 1, 64);
        if (lane == 63 && li + 1 < S.n) key_of(S.kind, S.values + (size_t)(li + 1) * S.vs, S.ts_off, kn);
        if (!in) continue;
        // Stage the value in the table's scratch (the gather reads from there
        // and writes the table in place: no copy-back pass).
        for (uint32_t q = 0; q < S.vs; q += 16)
            gst<u32x4>(S.scratch + (size_t)li * S.vs + q, gld<u32x4>(S.values + (size_t)li * S.vs + q));
        for (uint32_t l = 0; l < kl; l++) {
            keys[(size_t)l * N + i] = k[l];
            o[l] |= k[l];
            a[l] &= k[l];
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
    for (uint32_t l = 0; l < 3; l++) {
        for (int off = 32; off > 0; off >>= 1) {
            o[l] |= __shfl_xor(o[l], off, 64);
            a[l] &= __shfl_xor(a[l], off, 64);
        }
        if (lane == 0) {
            s_or[l][wave] = o[l];
            s_and[l][wave] = a[l];
        }
    }
    __syncthreads();
    if (uns) atomicOr(&s_uns, 1u);
    __syncthreads();
    if (tid == 0) {
        for (uint32_t l = 0; l < kl; l++) {
            uint64_t oo = 0, aa = ~0ull;
            for (int w = 0; w < 4; w++) {
                oo |= s_or[l][w];
                aa &= s_and[l][w];
            }
            SortProbe *pb = probe + (blockIdx.x % kProbeBuckets);
            atomicOr((unsigned long long *)&pb->or_[l], (unsigned long long)oo);
            atomicAnd((unsigned long long *)&pb->and_[l], (unsigned long long)aa);
        }
        if (s_uns) atomicOr(&segs[sg].unsorted, 1u);
    }
}

__device__ __forceinline__ uint32_t hist_slot(const SortSeg &S, uint32_t d, uint32_t lt) {
    return S.tile_base * kBins + d * S.tiles + lt;
}

__global__ __launch_bounds__(kSortThreads) void k_sort_hist(const SortSeg *segs, const uint32_t *tile_seg,
                                                            const uint64_t *keys, uint32_t N, uint32_t limb,
                                                            uint32_t shift, uint32_t *hist) {
    __shared__ uint32_t cnt[kBins];
    const uint32_t tid = threadIdx.x;
    const SortSeg S = segs[tile_seg[blockIdx.x]];
    const uint32_t lt = blockIdx.x - S.tile_base;
    if (tid < kBins) cnt[tid] = 0;
    __syncthreads();
    for (uint32_t r = 0; r < kSortPer; r++) {
        const uint32_t li = lt * kSortTile + r * kSortThreads + tid;
        if (li < S.n) {
            const uint32_t i = S.item_base + li;
            atomicAdd(&cnt[(uint32_t)(gld<uint64_t>(keys + (size_t)limb * N + i) >> shift) & (kBins - 1)], 1u);
        }
    }
    __syncthreads();
    if (tid < kBins) hist[hist_slot(S, tid, lt)] = cnt[tid];
}

// Exclusive scan of the m histogram entries in place, in three short
// launches (all loads coalesced): per-chunk sums, a scan of the chunk sums,
// then every chunk rescanned with its offset. kScanChunk entries per chunk.
constexpr uint32_t kScanChunk = 2048;

__device__ __forceinline__ uint32_t block_excl_scan_256(uint32_t v, uint32_t *wsum, uint32_t &total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t incl = v;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63) wsum[wave] = incl;
    __syncthreads();
    uint32_t off = 0;
    total = 0;
    for (uint32_t w = 0; w < 4; w++) {
        off += w < wave ? wsum[w] : 0u;
        total += wsum[w];
    }
    __syncthreads();
    return off + incl - v;
}

__global__ __launch_bounds__(256) void k_scan_reduce(const uint32_t *hist, uint32_t m, uint32_t *chunk_sums) {
    __shared__ uint32_t wsum[4];
    const uint32_t base = blockIdx.x * kScanChunk;
    uint32_t sum = 0;
    for (uint32_t k = threadIdx.x; k < kScanChunk; k += 256)
        sum += base + k < m ? hist[base + k] : 0u;
    uint32_t total;
    block_excl_scan_256(sum, wsum, total);
    if (threadIdx.x == 0) chunk_sums[blockIdx.x] = total;
}

// One workgroup: exclusive scan of the chunk sums in place.
__global__ __launch_bounds__(256) void k_scan_top(uint32_t *chunk_sums, uint32_t chunks) {
    __shared__ uint32_t wsum[4];
    uint32_t carry = 0;
    for (uint32_t b = 0; b < chunks; b += 256) {
        const uint32_t i = b + threadIdx.x;
        const uint32_t v = i < chunks ? chunk_sums[i] : 0u;
        uint32_t total;
        const uint32_t ex = block_excl_scan_256(v, wsum, total);
        if (i < chunks) chunk_sums[i] = carry + ex;
        carry += total;
    }
}

// Each thread owns 8 consecutive entries of the chunk (loaded as 2 x 16 B).
__global__ __launch_bounds__(256) void k_scan_apply(uint32_t *hist, uint32_t m, const uint32_t *chunk_sums) {
    __shared__ uint32_t wsum[4];
    const uint32_t base = blockIdx.x * kScanChunk + threadIdx.x * 8;
    uint32_t v[8], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        v[k] = base + k < m ? hist[base + k] : 0u;
        sum += v[k];
    }
    uint32_t total;
    uint32_t run = chunk_sums[blockIdx.x] + block_excl_scan_256(sum, wsum, total);
#pragma unroll
    for (uint32_t k = 0; k < 8; k++) {
        if (base + k < m) hist[base + k] = run;
        run += v[k];
    }
}

template <int KL>
__global__ __launch_bounds__(kSortThreads) void k_sort_scatter(const SortSeg *segs, const uint32_t *tile_seg,
                                                               const uint64_t *keys_in, const uint32_t *idx_in,
                                                               uint64_t *keys_out, uint32_t *idx_out, uint32_t N,
                                                               uint32_t limb, uint32_t shift, const uint32_t *hist) {
    __shared__ uint64_t s_key[KL][kSortTile];
    __shared__ uint32_t s_idx[kSortTile];
    __shared__ uint32_t s_cnt[kBins][kSortThreads + 1]; // digit-major per-thread counts
    __shared__ uint32_t s_tot[kBins], s_dstart[kBins], s_gbase[kBins];
    __shared__ uint16_t s_perm[kSortTile]; // tile position in digit order -> item
    const uint32_t tid = threadIdx.x;
    const SortSeg S = segs[tile_seg[blockIdx.x]];
    const uint32_t lt = blockIdx.x - S.tile_base;
    const uint32_t base = S.item_base + lt * kSortTile;
    const uint32_t m = (S.n - lt * kSortTile) < kSortTile ? (S.n - lt * kSortTile) : kSortTile;
    // Coalesced load into LDS.
    for (uint32_t r = 0; r < kSortPer; r++) {
        const uint32_t e = r * kSortThreads + tid;
        if (e < m) {
#pragma unroll
            for (int l = 0; l < KL; l++) s_key[l][e] = gld<uint64_t>(keys_in + (size_t)(limb + l) * N + base + e);
            s_idx[e] = gld<uint32_t>(idx_in + base + e);
        }
    }
    __syncthreads();
    // Thread tid owns items [tid*8, tid*8+8) in order.
    uint32_t dig[kSortPer];
    uint32_t c[kBins];
#pragma unroll
    for (uint32_t d = 0; d < kBins; d++) c[d] = 0;
#pragma unroll
    for (uint32_t k = 0; k < kSortPer; k++) {
        const uint32_t e = tid * kSortPer + k;
        dig[k] = e < m ? (uint32_t)(s_key[0][e] >> shift) & (kBins - 1) : kBins; // kBins = none
#pragma unroll
        for (uint32_t d = 0; d < kBins; d++) c[d] += dig[k] == d ? 1u : 0u;
    }
#pragma unroll
    for (uint32_t d = 0; d < kBins; d++) s_cnt[d][tid] = c[d];
    __syncthreads();
    // Per digit, exclusive scan across threads (one wave per digit group).
    {
        const uint32_t wave = tid >> 6, lane = tid & 63;
        for (uint32_t d = wave; d < kBins; d += kSortThreads / 64) {
            uint32_t carry = 0;
            for (uint32_t b0 = 0; b0 < kSortThreads; b0 += 64) {
                const uint32_t v = s_cnt[d][b0 + lane];
                uint32_t incl = v;
                for (int o = 1; o < 64; o <<= 1) {
                    uint32_t y = __shfl_up(incl, o, 64);
                    if (lane >= (uint32_t)o) incl += y;
                }
                s_cnt[d][b0 + lane] = carry + incl - v;
                carry += __shfl(incl, 63, 64);
            }
            if (lane == 0) s_tot[d] = carry;
        }
    }
    __syncthreads();
    if (tid < kBins) s_gbase[tid] = hist[hist_slot(S, tid, lt)];
    if (tid == 0) {
        uint32_t acc = 0;
        for (uint32_t d = 0; d < kBins; d++) {
            s_dstart[d] = acc;
            acc += s_tot[d];
        }
    }
    __syncthreads();
    // Rank every item inside the tile in digit order (stable: thread order,
    // then item order within the thread) ...
    uint32_t run[kBins];
#pragma unroll
    for (uint32_t d = 0; d < kBins; d++) run[d] = s_dstart[d] + s_cnt[d][tid];
#pragma unroll
    for (uint32_t k = 0; k < kSortPer; k++) {
        if (dig[k] < kBins) {
            uint32_t loc = 0;
#pragma unroll
            for (uint32_t d = 0; d < kBins; d++)
                if (dig[k] == d) loc = run[d]++;
            s_perm[loc] = (uint16_t)(tid * kSortPer + k);
        }
    }
    __syncthreads();
    // ... then write the tile out in that order: consecutive threads write
    // consecutive destinations inside each digit's run (coalesced).
    for (uint32_t i = tid; i < m; i += kSortThreads) {
        const uint32_t e = s_perm[i];
        const uint32_t d = (uint32_t)(s_key[0][e] >> shift) & (kBins - 1);
        const uint32_t dst = s_gbase[d] + (i - s_dstart[d]);
#pragma unroll
        for (int l = 0; l < KL; l++) gst<uint64_t>(keys_out + (size_t)(limb + l) * N + dst, s_key[l][e]);
        gst<uint32_t>(idx_out + dst, s_idx[e]);
    }
}

// values[i] = scratch[idx[i]] (segment-local; scratch holds the unsorted
// table), 16 bytes per lane; sorted tables are left alone.
__global__ __launch_bounds__(256) void k_sort_gather(const SortSeg *segs, const uint32_t *tile_seg,
                                                     const uint32_t *idx) {
    const SortSeg S = segs[tile_seg[blockIdx.x]];
    if (!S.unsorted) return;
    const uint32_t lt = blockIdx.x - S.tile_base;
    const uint32_t first = lt * kSortTile;
    const uint32_t m = (S.n - first) < kSortTile ? (S.n - first) : kSortTile;
    const uint32_t cpv = S.vs >> 4;
    for (uint32_t c = threadIdx.x; c < m * cpv; c += 256) {
        const uint32_t e = c / cpv, part = c % cpv;
        const uint32_t src = gld<uint32_t>(idx + S.item_base + first + e) - S.item_base;
        gst<u32x4>(S.values + (size_t)(first + e) * S.vs + 16 * part,
                   gld<u32x4>(S.scratch + (size_t)src * S.vs + 16 * part));
    }
}

static uint32_t key_limbs(uint32_t kind) {
    return kind == kKeyTimestamp ? 1 : kind == kKeyCompositeU128 ? 3 : 2;
}

static uint64_t tiles_of(uint32_t n) { return (n + kSortTile - 1) / kSortTile; }

uint64_t sort_scratch_bytes(const SortItem *items, uint32_t count) {
    uint64_t N = 0, tiles = 0, vals = 0;
    for (uint32_t j = 0; j < count; j++) {
        if (items[j].n < 2) continue;
        N += items[j].n;
        tiles += tiles_of(items[j].n);
        vals += ((uint64_t)items[j].n * items[j].value_size + 255) / 256 * 256;
    }
    return sizeof(SortProbe) * kProbeBuckets           // probes
           + ((uint64_t)sizeof(SortSeg) * count + 255) / 256 * 256
           + (4 * tiles + 255) / 256 * 256              // tile -> segment
           + 2 * ((N * 3 * 8) + (N * 4 + 255) / 256 * 256) // two item buffers
           + (4 * kBins * tiles + 255) / 256 * 256      // histogram
           + (4 * (kBins * tiles / kScanChunk + 1) + 255) / 256 * 256 // scan chunk sums
           + vals;                                      // gathered values
}

int launch_sort_batch(const SortItem *items, uint32_t count, void *scratch, uint64_t scratch_bytes, void *stream) {
    if (scratch_bytes < sort_scratch_bytes(items, count)) return -1;
    hipStream_t s = (hipStream_t)stream;
    // Host plan: segments (n >= 2), tile bases, widest key.
    std::vector<SortSeg> segs;
    std::vector<uint32_t> tile_seg;
    uint32_t N = 0, kl = 1;
    for (uint32_t j = 0; j < count; j++) {
        const SortItem &it = items[j];
        if (it.n < 2) continue;
        SortSeg g{};
        g.values = (uint8_t *)it.values;
        g.n = it.n;
        g.vs = it.value_size;
        g.ts_off = it.timestamp_offset;
        g.kind = it.key_kind;
        g.item_base = N;
        g.tile_base = (uint32_t)tile_seg.size();
        g.tiles = (uint32_t)tiles_of(it.n);
        for (uint32_t t = 0; t < g.tiles; t++) tile_seg.push_back((uint32_t)segs.size());
        N += it.n;
        kl = kl > key_limbs(it.key_kind) ? kl : key_limbs(it.key_kind);
        segs.push_back(g);
    }
    if (segs.empty()) return 0;
    const uint32_t nseg = (uint32_t)segs.size(), ntiles = (uint32_t)tile_seg.size();
    uint8_t *p = (uint8_t *)scratch;
    SortProbe *probe = (SortProbe *)p;
    p += sizeof(SortProbe) * kProbeBuckets;
    SortSeg *d_segs = (SortSeg *)p;
    p += ((uint64_t)sizeof(SortSeg) * count + 255) / 256 * 256;
    uint32_t *d_tile_seg = (uint32_t *)p;
    p += (4ull * ntiles + 255) / 256 * 256;
    uint64_t *keys[2];
    uint32_t *idx[2];
    for (int b = 0; b < 2; b++) {
        keys[b] = (uint64_t *)p;
        p += (uint64_t)N * 3 * 8;
        idx[b] = (uint32_t *)p;
        p += ((uint64_t)N * 4 + 255) / 256 * 256;
    }
    uint32_t *hist = (uint32_t *)p;
    p += ((uint64_t)4 * kBins * ntiles + 255) / 256 * 256;
    uint32_t *chunk_sums = (uint32_t *)p;
    p += ((uint64_t)4 * (kBins * ntiles / kScanChunk + 1) + 255) / 256 * 256;
    for (SortSeg &g : segs) {
        g.scratch = p;
        p += ((uint64_t)g.n * g.vs + 255) / 256 * 256;
    }

    // The plan is staged through static host memory owned by the caller's
    // stream order: copy it synchronously with the probe read below.
    std::vector<SortProbe> init(kProbeBuckets);
    for (SortProbe &pr : init)
        for (int l = 0; l < 4; l++) pr.or_[l] = 0, pr.and_[l] = ~0ull;
    if (hipMemcpyAsync(probe, init.data(), sizeof(SortProbe) * kProbeBuckets, hipMemcpyHostToDevice, s) !=
            hipSuccess ||
        hipMemcpyAsync(d_segs, segs.data(), sizeof(SortSeg) * nseg, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_tile_seg, tile_seg.data(), 4ull * ntiles, hipMemcpyHostToDevice, s) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_sort_extract, dim3(ntiles), dim3(256), 0, s, d_segs, d_tile_seg, kl, N, keys[0], idx[0],
                       probe);
    // The digit plan needs the probe on the host (one small synchronous read
    // per batch, not per memtable).
    std::vector<SortProbe> buckets(kProbeBuckets);
    std::vector<SortSeg> hsegs(nseg);
    if (hipMemcpyAsync(buckets.data(), probe, sizeof(SortProbe) * kProbeBuckets, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipMemcpyAsync(hsegs.data(), d_segs, sizeof(SortSeg) * nseg, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return -1;
    SortProbe host = buckets[0];
    for (const SortProbe &pr : buckets)
        for (int l = 0; l < 4; l++) host.or_[l] |= pr.or_[l], host.and_[l] &= pr.and_[l];
    bool any = false;
    for (const SortSeg &g : hsegs) any |= g.unsorted != 0;
    if (!any) return 0; // table_memory.zig:141: already sorted, no-op
    int cur = 0;
    // LSD passes carry only the limbs still to be sorted on: limbs below the
    // current one are final, limbs above the highest varying one are constant.
    uint32_t hi = 0;
    for (uint32_t limb = 0; limb < kl; limb++)
        if (host.or_[limb] ^ host.and_[limb]) hi = limb + 1;
    for (uint32_t limb = 0; limb < hi; limb++) {
        const uint64_t varies = host.or_[limb] ^ host.and_[limb];
        const uint32_t live = hi - limb; // limbs [limb, hi) move with the items
        for (uint32_t shift = 0; shift < 64; shift += kDigitBits) {
            if (((varies >> shift) & (kBins - 1)) == 0) continue; // constant digit: order unchanged
            hipLaunchKernelGGL(k_sort_hist, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile_seg, keys[cur],
                               N, limb, shift, hist);
            const uint32_t m = kBins * ntiles, chunks = (m + kScanChunk - 1) / kScanChunk;
            hipLaunchKernelGGL(k_scan_reduce, dim3(chunks), dim3(256), 0, s, hist, m, chunk_sums);
            hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(256), 0, s, chunk_sums, chunks);
            hipLaunchKernelGGL(k_scan_apply, dim3(chunks), dim3(256), 0, s, hist, m, chunk_sums);
            switch (live) {
            case 1:
                hipLaunchKernelGGL(k_sort_scatter<1>, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile_seg,
                                   keys[cur], idx[cur], keys[cur ^ 1], idx[cur ^ 1], N, limb, shift, hist);
                break;
            case 2:
                hipLaunchKernelGGL(k_sort_scatter<2>, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile_seg,
                                   keys[cur], idx[cur], keys[cur ^ 1], idx[cur ^ 1], N, limb, shift, hist);
                break;
            default:
                hipLaunchKernelGGL(k_sort_scatter<3>, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile_seg,
                                   keys[cur], idx[cur], keys[cur ^ 1], idx[cur ^ 1], N, limb, shift, hist);
                break;
            }
            cur ^= 1;
        }
    }
    hipLaunchKernelGGL(k_sort_gather, dim3(ntiles), dim3(256), 0, s, d_segs, d_tile_seg, idx[cur]);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace tbc
