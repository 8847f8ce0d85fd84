// sort.hip — TableMemory.sort (src/lsm/table_memory.zig:140-154) on gfx950.
//
// The reference sorts the mutable table's Values with std.mem.sort (Zig 0.11
// stable block sort) by key_from_value, only when puts arrived out of order
// (table_memory.zig:83-87). Stability is load-bearing: fill_immutable_values
// keeps the LAST of a run of equal keys (compaction.zig:519-522).
//
// A batch of memtables (every tree's at the bar end) is sorted by one
// enqueued launch sequence that never waits on the host. Items are sorted
// as (packed key, index) pairs by a stable LSD radix sort with 8-bit digits:
//
//   k_sort_extract  per tile of 2,048 items: a copy of the values (the
//                   gather's source), OR/AND of every key limb, and whether
//                   the table is out of order at all;
//   k_sort_layout   per table: the key bytes that vary over the table, in
//                   significance order; the rest cannot decide any order, so
//                   the packed key (those bytes only, 8 per limb) orders the
//                   table exactly as its key does (config 3's composite u128
//                   keys: 24 key bytes, 6 varying -> one 64-bit limb);
//   k_sort_pack     per tile: packed keys + indices, the digit histograms of
//                   every packed byte, and which low-order prefixes of the
//                   packed key the table is already in order on;
//   k_sort_plan     per table: LSD passes run from the least significant
//                   byte up, so the bytes of a prefix the table is already
//                   in order on (a secondary index put in timestamp order)
//                   cannot change the stable order and are skipped; each
//                   remaining pass's source buffer; every digit's start;
//   k_sort_pass x P one launch per potential pass (P = 8 per key limb of the
//                   batch's widest key), persistent workgroups; a pass no
//                   table needs returns at once. Onesweep: each tile ranks
//                   its items by digit (wave match ballots + per-wave counts:
//                   stable), publishes its digit counts, looks back over the
//                   tiles before it in its table for their prefix (decoupled
//                   look-back), and writes the tile out through LDS so each
//                   digit's run is contiguous; a table's last pass moves
//                   the values themselves (values[i] = copy[idx[i]]).
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
constexpr uint32_t kTopBytes = 4;   // truncated sorts keep at least this many top bytes
constexpr uint32_t kRunMax = 64;    // longest run of equal top bytes k_sort_fixup orders
constexpr uint32_t kDirectPasses = 6; // passes with a launch each; the rest share k_sort_pass_rest

// Look-back words (64-bit): the pass launch's epoch in the top half (words
// of earlier launches read as "not published", so the buffer is zeroed once,
// never per pass), the flag in bits 31:30, the count below (< 2^30).
constexpr uint64_t kFlagAggregate = 1ull << 30;
constexpr uint64_t kFlagPrefix = 2ull << 30;
constexpr uint64_t kCountMask = (1ull << 30) - 1;

struct SortSeg {
    uint64_t key_or[kMaxLimbs], key_and[kMaxLimbs]; // over the table (extract)
    uint8_t *values;
    uint8_t *copy; // n * vs bytes: the table as put, the gather's source
    uint32_t n, vs, ts_off, kind;
    uint32_t kl; // key limbs of the table's key kind
    uint32_t item_base, tile_base, tiles;
    uint32_t unsorted;  // some adjacent pair is out of key order (extract)
    uint32_t nbytes;    // varying key bytes = packed key bytes (layout)
    uint32_t viol;      // bit b: out of order on packed bytes [0, b] (pack)
    uint32_t active;    // bit p: pass p moves this table's items (plan)
    uint32_t src_bits;  // bit p: pass p reads buffer 1
    uint32_t final_buf; // buffer the last pass would have written
    uint32_t skip;      // packed bytes [0, skip): the table is in order on them
    uint32_t top;       // truncated: passes cover only packed bytes [top, nbytes) (0: not truncated)
    uint32_t overflow;  // truncated and a run of equal top bytes too long to fix up: rescued
    uint32_t nact;      // passes of the table: pass q sorts on packed byte act[q]
    uint8_t byte_src[kMaxPasses]; // packed byte j = key byte byte_src[j] (limb * 8 + byte)
    uint8_t act[kMaxPasses];
};

struct SortBatch {
    uint32_t active; // passes some table needs
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

// hist / bins layout: [segment][pass][digit] u32.
__device__ __forceinline__ uint32_t *seg_hist(uint32_t *hist, uint32_t s) { return hist + (size_t)s * kMaxPasses * kRadix; }

// The key and the next item's key (the next lane's; lane 63 loads its
// neighbour, which may sit in the next tile) of every lane of a row.
__device__ __forceinline__ void row_keys(const SortSeg &S, uint32_t li, bool in, uint64_t k[3], uint64_t kn[3]) {
    k[0] = k[1] = k[2] = 0;
    if (in) key_of(S.kind, S.values + (size_t)li * S.vs, S.ts_off, k);
    for (uint32_t l = 0; l < 3; l++) kn[l] = __shfl_down(k[l], 1, 64);
    if ((threadIdx.x & 63) == 63 && li + 1 < S.n) key_of(S.kind, S.values + (size_t)(li + 1) * S.vs, S.ts_off, kn);
}

// --------------------------------------------------------------------------
// Extract: one workgroup per tile.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kSortThreads) void k_sort_extract(SortSeg *segs, const uint32_t *tile_seg) {
    __shared__ uint64_t s_or[kMaxLimbs][kSortWaves], s_and[kMaxLimbs][kSortWaves];
    __shared__ uint32_t s_uns;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t sg = tile_seg[blockIdx.x];
    const SortSeg S = segs[sg];
    const uint32_t lt = blockIdx.x - S.tile_base;
    if (tid == 0) s_uns = 0;
    __syncthreads();
    uint64_t o[kMaxLimbs] = {0, 0, 0}, a[kMaxLimbs] = {~0ull, ~0ull, ~0ull};
    uint32_t uns = 0;
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint32_t li = lt * kSortTile + r * kSortThreads + tid;
        if (lt * kSortTile + r * kSortThreads >= S.n) break; // wave-uniform (whole row past the end)
        const bool in = li < S.n;
        uint64_t k[3], kn[3];
        row_keys(S, li, in, k, kn);
        if (!in) continue;
        for (uint32_t b = 0; b < S.vs; b += 128) { // up to 8 loads in flight before their stores
            u32x4 v[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
                if (b + 16 * q < S.vs) v[q] = gld<u32x4>(S.values + (size_t)li * S.vs + b + 16 * q);
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
                if (b + 16 * q < S.vs) gst<u32x4>(S.copy + (size_t)li * S.vs + b + 16 * q, v[q]);
        }
        for (uint32_t l = 0; l < S.kl; l++) {
            o[l] |= k[l];
            a[l] &= k[l];
        }
        if (li + 1 < S.n) {
            int cmp = 0;
            for (uint32_t l = 0; l < S.kl; l++)
                if (k[l] != kn[l]) cmp = k[l] > kn[l] ? 1 : -1;
            uns |= cmp > 0 ? 1u : 0u;
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
    if (tid < S.kl) {
        uint64_t oo = 0, aa = ~0ull;
        for (uint32_t w = 0; w < kSortWaves; w++) {
            oo |= s_or[tid][w];
            aa &= s_and[tid][w];
        }
        atomicOr((unsigned long long *)&segs[sg].key_or[tid], (unsigned long long)oo);
        atomicAnd((unsigned long long *)&segs[sg].key_and[tid], (unsigned long long)aa);
    }
    if (tid == 0 && s_uns) atomicOr(&segs[sg].unsorted, 1u);
}

// Layout: one thread per table — its varying key bytes, least significant first.
__global__ __launch_bounds__(64) void k_sort_layout(SortSeg *segs, uint32_t nseg) {
    const uint32_t s = blockIdx.x * 64 + threadIdx.x;
    if (s >= nseg) return;
    SortSeg &S = segs[s];
    uint32_t nb = 0;
    if (S.unsorted)
        for (uint32_t l = 0; l < S.kl; l++)
            for (uint32_t b = 0; b < 8; b++)
                if (((S.key_or[l] ^ S.key_and[l]) >> (8 * b)) & 255) S.byte_src[nb++] = (uint8_t)(8 * l + b);
    S.nbytes = nb;
}

__device__ __forceinline__ void pack_key(const uint8_t *map, uint32_t nb, const uint64_t k[3], uint64_t pk[3]) {
    pk[0] = pk[1] = pk[2] = 0;
    for (uint32_t j = 0; j < nb; j++) {
        const uint32_t src = map[j];
        pk[j >> 3] |= ((k[src >> 3] >> (8 * (src & 7))) & 255ull) << (8 * (j & 7));
    }
}

// One wave's 64 digits into an LDS histogram row: a digit shared by the
// whole row (a slowly varying key byte) is one add; otherwise the lanes
// with equal digits (8 ballots) add once through their first lane.
__device__ __forceinline__ void hist_add(uint32_t *row, uint32_t d, bool in) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t act = __ballot(in);
    if (!act) return;
    const uint32_t first = __builtin_ctzll(act);
    const uint32_t d0 = (uint32_t)__builtin_amdgcn_readlane((int)d, (int)first);
    if (!__ballot(in && d != d0)) {
        if (lane == first) atomicAdd(&row[d0], (uint32_t)__builtin_popcountll(act));
        return;
    }
    uint64_t peers = act;
#pragma unroll
    for (uint32_t b = 0; b < 8; b++) {
        const uint64_t bal = __ballot((d >> b) & 1u);
        peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    if (in && !(peers & ((1ull << lane) - 1))) atomicAdd(&row[d], (uint32_t)__builtin_popcountll(peers));
}

// Pack: one workgroup per tile of an unsorted table.
__global__ __launch_bounds__(kSortThreads) void k_sort_pack(SortSeg *segs, const uint32_t *tile_seg, uint32_t N,
                                                            uint64_t *keys, uint32_t *idx, uint32_t *hist) {
    __shared__ uint32_t s_hist[kMaxPasses][kRadix];
    __shared__ uint32_t s_viol;
    const uint32_t tid = threadIdx.x;
    const uint32_t sg = tile_seg[blockIdx.x];
    const SortSeg S = segs[sg];
    const uint32_t nb = S.nbytes;
    if (!nb) return; // uniform: a sorted table
    __shared__ uint8_t s_map[kMaxPasses]; // the byte map is read per item: LDS, not scratch
    const uint32_t pl = (nb + 7) >> 3;
    for (uint32_t j = 0; j < nb; j++) s_hist[j][tid] = 0;
    if (tid < kMaxPasses) s_map[tid] = segs[sg].byte_src[tid];
    if (tid == 0) s_viol = 0;
    __syncthreads();
    const uint32_t lt = blockIdx.x - S.tile_base;
    uint32_t viol = 0;
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint32_t li = lt * kSortTile + r * kSortThreads + tid;
        if (lt * kSortTile + r * kSortThreads >= S.n) break; // uniform
        const bool in = li < S.n;
        uint64_t k[3], kn[3], pk[3], pn[3];
        row_keys(S, li, in, k, kn);
        pack_key(s_map, nb, k, pk);
        const uint32_t i = S.item_base + li;
        if (in) {
            for (uint32_t l = 0; l < pl; l++) keys[(size_t)l * N + i] = pk[l];
            idx[i] = i;
        }
        for (uint32_t j = 0; j < nb; j++) hist_add(s_hist[j], (uint32_t)(pk[j >> 3] >> (8 * (j & 7))) & 255u, in);
        if (in && li + 1 < S.n) {
            pack_key(s_map, nb, kn, pn);
            int cmp = 0; // order of (item, next) on packed bytes [0, j]
            for (uint32_t j = 0; j < nb; j++) {
                const uint32_t x = (uint32_t)(pk[j >> 3] >> (8 * (j & 7))) & 255u;
                const uint32_t y = (uint32_t)(pn[j >> 3] >> (8 * (j & 7))) & 255u;
                if (x != y) cmp = x > y ? 1 : -1;
                if (cmp > 0) viol |= 1u << j;
            }
        }
    }
    if (viol) atomicOr(&s_viol, viol);
    __syncthreads();
    uint32_t *h = seg_hist(hist, sg);
    for (uint32_t j = 0; j < nb; j++)
        if (s_hist[j][tid]) atomicAdd(&h[j * kRadix + tid], s_hist[j][tid]);
    if (tid == 0 && s_viol) atomicOr(&segs[sg].viol, s_viol);
}

// Plan: one workgroup per table. Passes [skip, nbytes) run, where the table
// is already in order on packed bytes [0, skip) (the largest such prefix);
// then the digit starts of those passes.
__global__ __launch_bounds__(kRadix) void k_sort_plan(SortSeg *segs, SortBatch *batch, const uint32_t *hist,
                                                      uint32_t *bins) {
    const uint32_t s = blockIdx.x, d = threadIdx.x, lane = d & 63, wave = d >> 6;
    __shared__ uint32_t wsum[kRadix / 64];
    SortSeg &S = segs[s];
    const uint32_t nb = S.nbytes;
    uint32_t skip = 0;
    for (uint32_t j = 1; j < nb; j++)
        if (!((S.viol >> (j - 1)) & 1u)) skip = j;
    // Many varying bytes (random u64/u128 fields): sort on the top bytes
    // only (at least kTopBytes, 10 bits beyond log2 n) and let k_sort_fixup
    // order each run of equal top bytes by the full key -- when the top
    // bytes' histograms predict short runs: n x prod(largest digit share)
    // <= 1 if the bytes were independent. Clustered keys (config 3's Zipf
    // accounts) keep every pass; a misprediction costs k_sort_rescue.
    const uint32_t *h = hist + (size_t)s * kMaxPasses * kRadix;
    const uint32_t log2n = 32 - __builtin_clz(S.n | 1);
    const uint32_t top_bytes = (log2n + 10 + 7) / 8 > kTopBytes ? (log2n + 10 + 7) / 8 : kTopBytes;
    uint32_t first = skip;
    if (nb - skip > top_bytes) {
        __shared__ uint32_t wmax[kRadix / 64];
        float est = (float)S.n;
        for (uint32_t b = nb - top_bytes; b < nb; b++) {
            uint32_t mx = h[b * kRadix + d];
            for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
            if (lane == 0) wmax[wave] = mx;
            __syncthreads();
            mx = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
            __syncthreads();
            est *= (float)mx / (float)S.n;
        }
        if (est <= 1.0f) first = nb - top_bytes;
    }
    uint32_t active = 0;
    for (uint32_t p = first; p < nb; p++) active |= 1u << p;
    __syncthreads(); // every thread has read viol before thread 0 writes the plan
    if (d == 0) {
        S.active = active;
        S.nact = nb - first;
        for (uint32_t q = 0; q < nb - first; q++) S.act[q] = (uint8_t)(first + q);
        S.final_buf = (nb - first) & 1u;
        S.skip = skip;
        S.top = first > skip ? first : 0;
        if (nb > first) atomicOr(&batch->active, (1u << (nb - first)) - 1u); // pass q runs if some table has > q
    }
    uint32_t *out = bins + (size_t)s * kMaxPasses * kRadix;
    for (uint32_t m = active; m; m &= m - 1) {
        const uint32_t p = __builtin_ctz(m);
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
        out[p * kRadix + d] = S.item_base + off + incl - c;
        __syncthreads();
    }
}

// --------------------------------------------------------------------------
// One onesweep pass (digit = packed byte p: byte p & 7 of packed limb p >> 3).
// --------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Persistent workgroups take tiles in arrival order (dynamic ids): every
// tile one looks back on was taken by a workgroup that is running or done.
// The tile is reordered through LDS one key limb at a time (16 KiB), so the
// workgroup's LDS does not grow with the key width (5 workgroups per CU).
// A table's last pass moves the values themselves (values[dst] =
// copy[index]) instead of keys and indices: the gather is fused into it.
struct PassShared {
    uint32_t tile;
    uint32_t wcnt[kSortWaves][kRadix]; // per wave: running, then total counts
    uint32_t start[kRadix];            // local start of each digit in the tile
    uint32_t excl[kRadix];             // items of the digit in the table's earlier tiles
    uint32_t wsum[kSortWaves];
    uint64_t key[kSortTile];           // one limb at a time
    uint32_t idx[kSortTile];
    uint8_t dig[kSortTile];
};

// Pass p over the tiles taken from tile_counter[p] (ticket order), until
// they run out. `done` (the rest kernel only): every finished tile adds one
// to done[p] after an agent-scope release, and before its first tile of pass
// p a workgroup waits for done[p - 1] == ntiles and acquires (the pass reads
// what every tile of the previous pass wrote, on any XCD).
__device__ __forceinline__ void sort_pass_tiles(PassShared &sh, const SortSeg *segs, const uint32_t *tile_seg,
                                                const uint32_t *tile_order, uint32_t p, uint32_t ntiles, uint32_t N,
                                                uint64_t *keys0, uint64_t *keys1, uint32_t *idx0, uint32_t *idx1,
                                                const uint32_t *bins, uint64_t *status, uint32_t epoch,
                                                uint32_t *tile_counter, uint32_t *done) {
    constexpr uint32_t R = kSortRounds;
    auto &s_tile = sh.tile;
    auto &s_wcnt = sh.wcnt;
    auto &s_start = sh.start;
    auto &s_excl = sh.excl;
    auto &s_wsum = sh.wsum;
    auto &s_key = sh.key;
    auto &s_idx = sh.idx;
    auto &s_dig = sh.dig;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t ep = (uint64_t)epoch << 32;
    const uint64_t lt_mask = (1ull << lane) - 1;
    // The first pass of the rest kernel follows a kernel boundary: nothing to wait for.
    bool waited = done == nullptr || p == kDirectPasses;
    for (bool first = true;; first = false) {
        // Every wave releases its own stores of the previous tile (at agent
        // scope: waits for them and writes the XCD's L2 back) before the
        // tile is counted as done.
        if (!first && done) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads(); // the previous tile's LDS readers are done
        if (!first && done && tid == 0)
            __hip_atomic_fetch_add(&done[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (tid == 0) s_tile = atomicAdd(&tile_counter[p], 1u);
        for (uint32_t i = tid; i < kSortWaves * kRadix; i += kSortThreads) (&s_wcnt[0][0])[i] = 0;
        __syncthreads();
        if (s_tile >= ntiles) return;
        if (!waited) { // rest kernel: every tile of pass p - 1 is complete and visible
            if (tid == 0) {
                for (uint32_t spins = 0; __hip_atomic_load(&done[p - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                                             ntiles;) {
                    if (++spins > (1u << 26)) break; // bounded (a broken invariant, not a hang)
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            __syncthreads();
            waited = true;
        }
        const uint32_t t = tile_order[s_tile];
        const uint32_t sg = tile_seg[t];
        const SortSeg &S = segs[sg];
        const uint32_t nact = S.nact;
        if (p >= nact) continue; // uniform: the table's passes are done (or it is in order)
        const bool last = p + 1 == nact && S.top == 0; // truncated tables finish in k_sort_fixup
        const uint32_t pb = S.act[p];                   // this pass's packed byte for the table
        const uint32_t limb = pb >> 3, shift = 8 * (pb & 7);
        const uint32_t lt = t - S.tile_base;
        const uint32_t base = S.item_base + lt * kSortTile;
        const uint32_t m = (S.n - lt * kSortTile) < kSortTile ? (S.n - lt * kSortTile) : kSortTile;
        const uint32_t live = ((S.nbytes + 7) >> 3) - limb; // packed limbs [limb, ..) still move
        const bool from1 = (p & 1u) != 0; // passes alternate buffers, the first reads buffer 0
        const uint64_t *ksrc = from1 ? keys1 : keys0;
        uint64_t *kdst = from1 ? keys0 : keys1;
        const uint32_t *isrc = from1 ? idx1 : idx0;
        uint32_t *idst = from1 ? idx0 : idx1;

        // Wave w owns items [512 w, 512 w + 512) of the tile, 64 per round in
        // lane order: stable rank = (earlier waves) + (earlier rounds of this
        // wave, counted in s_wcnt) + (earlier lanes with the same digit).
        uint32_t rank[R], dig[R], ix[R];
        uint64_t k[R][kMaxLimbs];
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t e = wave * (64 * R) + r * 64 + lane;
            const bool in = e < m;
#pragma unroll
            for (uint32_t l = 0; l < kMaxLimbs; l++)
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
        // Per digit (thread d): counts of the tile, exclusive prefix over
        // waves, and the tile-local start (exclusive scan over digits).
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
        uint32_t excl = 0;
        if (lt == 0) {
            lb_store(&status[(size_t)t * kRadix + d], ep | kFlagPrefix | cnt);
        } else {
            lb_store(&status[(size_t)t * kRadix + d], ep | kFlagAggregate | cnt);
            // Tiles in flight together all publish their aggregates at about
            // the same time, so a walk can be long: read a window of kLook
            // predecessors per round trip, nearest first.
            constexpr uint32_t kLook = 8;
            uint32_t pred = t - 1;
            for (uint32_t spins = 0;;) {
                uint64_t v[kLook];
#pragma unroll
                for (uint32_t w = 0; w < kLook; w++)
                    v[w] = pred >= S.tile_base + w ? lb_load(&status[(size_t)(pred - w) * kRadix + d]) : 0ull;
                bool done = false, stall = false;
#pragma unroll
                for (uint32_t w = 0; w < kLook; w++) {
                    if (done || stall) continue;
                    if ((v[w] >> 32) != epoch || !(v[w] & (3ull << 30))) { // not published by this pass yet
                        stall = true;
                        pred -= w;
                        continue;
                    }
                    excl += (uint32_t)(v[w] & kCountMask);
                    if ((v[w] & (3ull << 30)) == kFlagPrefix || pred - w == S.tile_base) done = true;
                }
                if (done) break;
                if (stall) {
                    if (++spins > (1u << 24)) break; // bounded (a broken invariant, not a hang)
                    __builtin_amdgcn_s_sleep(1);
                } else {
                    pred -= kLook;
                }
            }
            lb_store(&status[(size_t)t * kRadix + d], ep | kFlagPrefix | (excl + cnt));
        }
        s_excl[d] = excl;
        __syncthreads();
        // Tile-local sorted position of every item; indices and digits into LDS.
        uint32_t pos[R];
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t e = wave * (64 * R) + r * 64 + lane;
            pos[r] = s_start[dig[r]] + s_wcnt[wave][dig[r]] + rank[r];
            if (e < m) {
                s_idx[pos[r]] = ix[r];
                s_dig[pos[r]] = (uint8_t)dig[r];
            }
        }
        __syncthreads();
        // Destination of sorted position j = tid + 256 q: each digit's run
        // lands contiguously.
        const uint32_t *bin = bins + ((size_t)sg * kMaxPasses + pb) * kRadix;
        uint32_t dst[R];
#pragma unroll
        for (uint32_t q = 0; q < R; q++) {
            const uint32_t j = tid + kSortThreads * q;
            const uint32_t dj = j < m ? s_dig[j] : 0u;
            dst[q] = bin[dj] + s_excl[dj] + (j - s_start[dj]);
        }
        if (last) {
            // values[dst] = copy[index]: 16 bytes per lane, a lane group per value.
            const uint32_t cpv = S.vs >> 4, vpr = kSortThreads / cpv; // values per row of the workgroup
            for (uint32_t j0 = 0; j0 < m; j0 += vpr) {
                const uint32_t j = j0 + tid / cpv, part = tid % cpv;
                if (j < m) {
                    const uint32_t dj = s_dig[j];
                    const uint32_t to = bin[dj] + s_excl[dj] + (j - s_start[dj]) - S.item_base;
                    const uint32_t from = s_idx[j] - S.item_base;
                    gst<u32x4>(S.values + (size_t)to * S.vs + 16 * part,
                               gld<u32x4>(S.copy + (size_t)from * S.vs + 16 * part));
                }
            }
            continue;
        }
#pragma unroll
        for (uint32_t q = 0; q < R; q++) {
            const uint32_t j = tid + kSortThreads * q;
            if (j < m) gst<uint32_t>(idst + dst[q], s_idx[j]);
        }
#pragma unroll
        for (uint32_t l = 0; l < kMaxLimbs; l++) { // unrolled: k[r][l] stays in registers
            if (l >= live) break;
            __syncthreads(); // the previous limb's readers are done
#pragma unroll
            for (uint32_t r = 0; r < R; r++) {
                const uint32_t e = wave * (64 * R) + r * 64 + lane;
                if (e < m) s_key[pos[r]] = k[r][l];
            }
            __syncthreads();
#pragma unroll
            for (uint32_t q = 0; q < R; q++) {
                const uint32_t j = tid + kSortThreads * q;
                if (j < m) gst<uint64_t>(kdst + (size_t)(limb + l) * N + dst[q], s_key[j]);
            }
        }
    }
}

// One launch per pass below kDirectPasses: the kernel boundary orders the
// passes. A pass no table needs returns at once.
__global__ __launch_bounds__(kSortThreads) void k_sort_pass(const SortSeg *segs, const SortBatch *batch,
                                                            const uint32_t *tile_seg, const uint32_t *tile_order,
                                                            uint32_t p, uint32_t ntiles,
                                                            uint32_t N, uint64_t *keys0, uint64_t *keys1,
                                                            uint32_t *idx0, uint32_t *idx1, const uint32_t *bins,
                                                            uint64_t *status, uint32_t epoch,
                                                            uint32_t *tile_counter) {
    __shared__ PassShared sh;
    if (!((batch->active >> p) & 1u)) return; // uniform: no table has this many passes
    sort_pass_tiles(sh, segs, tile_seg, tile_order, p, ntiles, N, keys0, keys1, idx0, idx1, bins, status, epoch,
                    tile_counter, nullptr);
}

// Passes [kDirectPasses, kMaxPasses) in ONE launch (most batches need none:
// a truncated sort keeps at least 4 bytes, an in-order prefix is skipped):
// workgroups take pass p's tiles after pass p - 1's tickets ran out, so a
// tile only ever waits on tiles already taken by running workgroups (no
// grid barrier, no residency assumption), and the completion counters with
// agent-scope release/acquire order the passes across XCDs. Each pass takes
// a fresh look-back epoch.
__global__ __launch_bounds__(kSortThreads) void k_sort_pass_rest(const SortSeg *segs, const SortBatch *batch,
                                                                 const uint32_t *tile_seg, const uint32_t *tile_order,
                                                                 uint32_t ntiles, uint32_t N, uint64_t *keys0,
                                                                 uint64_t *keys1, uint32_t *idx0, uint32_t *idx1,
                                                                 const uint32_t *bins, uint64_t *status,
                                                                 uint32_t epoch0, uint32_t *tile_counter,
                                                                 uint32_t *done) {
    __shared__ PassShared sh;
    for (uint32_t p = kDirectPasses; p < kMaxPasses; p++) {
        if (!((batch->active >> p) & 1u)) return; // passes run as a prefix: none beyond either
        sort_pass_tiles(sh, segs, tile_seg, tile_order, p, ntiles, N, keys0, keys1, idx0, idx1, bins, status,
                        epoch0 + (p - kDirectPasses), tile_counter, done);
    }
}

// --------------------------------------------------------------------------
// Truncated tables: the passes ordered the items by their top packed bytes
// (stable); each run of equal top bytes is put in full-key order here (ties
// by put order, i.e. by item index: stability), and every value is written.
// One thread per sorted position; keys are re-read from the put-order copy.
// A run longer than kRunMax marks the table for k_sort_rescue.
// --------------------------------------------------------------------------
__device__ __forceinline__ void packed_of(const SortSeg &S, const uint8_t *map, uint32_t item, uint64_t pk[3]) {
    uint64_t k[3];
    key_of(S.kind, S.copy + (size_t)item * S.vs, S.ts_off, k);
    pack_key(map, S.nbytes, k, pk);
}

__device__ __forceinline__ bool top_eq(const uint64_t a[3], const uint64_t b[3], uint32_t top) {
    // packed bytes [top, 24): limbs above top's limb whole, top's limb from byte top % 8
    const uint32_t l0 = top >> 3, sh = 8 * (top & 7);
    if ((a[l0] >> sh) != (b[l0] >> sh)) return false;
    for (uint32_t l = l0 + 1; l < 3; l++)
        if (a[l] != b[l]) return false;
    return true;
}

__device__ __forceinline__ bool key_before(const uint64_t a[3], uint32_t ia, const uint64_t b[3], uint32_t ib) {
    for (int l = 2; l >= 0; l--)
        if (a[l] != b[l]) return a[l] < b[l];
    return ia < ib;
}

__global__ __launch_bounds__(256) void k_sort_fixup(SortSeg *segs, const uint32_t *tile_seg, const uint32_t *idx0,
                                                    const uint32_t *idx1) {
    __shared__ uint8_t s_map[kMaxPasses];
    const uint32_t sg = tile_seg[blockIdx.x];
    const SortSeg S = segs[sg];
    if (!S.top) return; // uniform: not truncated
    if (threadIdx.x < kMaxPasses) s_map[threadIdx.x] = segs[sg].byte_src[threadIdx.x];
    __syncthreads();
    const uint32_t *idx = (S.final_buf ? idx1 : idx0) + S.item_base; // table-local sorted order
    const uint32_t first = (blockIdx.x - S.tile_base) * kSortTile;
    for (uint32_t r = 0; r < kSortRounds; r++) {
        const uint32_t i = first + r * kSortThreads + threadIdx.x;
        if (i >= S.n) break;
        const uint32_t me = idx[i] - S.item_base;
        uint64_t pk[3];
        packed_of(S, s_map, me, pk);
        // run bounds [lo, hi) of equal top bytes around i
        uint32_t lo = i, hi = i + 1;
        bool too_long = false;
        while (lo > 0) {
            uint64_t q[3];
            packed_of(S, s_map, idx[lo - 1] - S.item_base, q);
            if (!top_eq(q, pk, S.top)) break;
            if (i - --lo >= kRunMax) { too_long = true; break; }
        }
        while (!too_long && hi < S.n) {
            uint64_t q[3];
            packed_of(S, s_map, idx[hi] - S.item_base, q);
            if (!top_eq(q, pk, S.top)) break;
            if (++hi - lo > kRunMax) too_long = true;
        }
        if (too_long) {
            atomicOr(&segs[sg].overflow, 1u);
            continue;
        }
        uint32_t rank = 0;
        for (uint32_t j = lo; j < hi; j++) {
            if (j == i) continue;
            const uint32_t other = idx[j] - S.item_base;
            uint64_t q[3];
            packed_of(S, s_map, other, q);
            rank += key_before(q, other, pk, me) ? 1u : 0u;
        }
        const uint32_t to = lo + rank;
        for (uint32_t b = 0; b < S.vs; b += 16)
            gst<u32x4>(S.values + (size_t)to * S.vs + b, gld<u32x4>(S.copy + (size_t)me * S.vs + b));
    }
}

// A truncated table whose top bytes left a run too long to fix up (rare:
// keys clustered in their top bytes): one workgroup sorts it again, all its
// varying bytes, LSD from the put-order copy, stable (ranks by wave match
// ballots within 256-item chunks in order), then writes every value. Slow
// but correct; the common case never launches work here.
__global__ __launch_bounds__(256) void k_sort_rescue(SortSeg *segs, uint32_t N, uint64_t *keys0, uint64_t *keys1,
                                                     uint32_t *idx0, uint32_t *idx1) {
    __shared__ uint8_t s_map[kMaxPasses];
    __shared__ uint32_t s_off[kRadix];
    __shared__ uint32_t s_wc[4][kRadix];
    __shared__ uint32_t s_wsum[4];
    const SortSeg S = segs[blockIdx.x];
    if (!S.overflow) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < kMaxPasses) s_map[tid] = segs[blockIdx.x].byte_src[tid];
    __syncthreads();
    const uint32_t nb = S.nbytes, pl = (nb + 7) >> 3, base = S.item_base;
    for (uint32_t i = tid; i < S.n; i += 256) {
        uint64_t pk[3];
        packed_of(S, s_map, i, pk);
        for (uint32_t l = 0; l < pl; l++) keys0[(size_t)l * N + base + i] = pk[l];
        idx0[base + i] = i;
    }
    __syncthreads();
    uint64_t *ks = keys0, *kd = keys1;
    uint32_t *is = idx0, *id = idx1;
    const uint64_t lt = (1ull << lane) - 1;
    for (uint32_t p = S.skip; p < nb; p++) {
        const uint32_t limb = p >> 3, sh = 8 * (p & 7);
        s_off[tid] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < S.n; i += 256)
            atomicAdd(&s_off[(uint32_t)(ks[(size_t)limb * N + base + i] >> sh) & 255u], 1u);
        __syncthreads();
        { // exclusive scan of the histogram (thread = digit)
            const uint32_t c = s_off[tid];
            uint32_t incl = c;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (lane >= (uint32_t)o) incl += y;
            }
            if (lane == 63) s_wsum[wave] = incl;
            __syncthreads();
            uint32_t off = 0;
            for (uint32_t w = 0; w < wave; w++) off += s_wsum[w];
            s_off[tid] = off + incl - c;
        }
        __syncthreads();
        for (uint32_t c0 = 0; c0 < S.n; c0 += 256) {
            const uint32_t i = c0 + tid;
            const bool in = i < S.n;
            const uint32_t d = in ? (uint32_t)(ks[(size_t)limb * N + base + i] >> sh) & 255u : 0u;
            for (uint32_t w = 0; w < 4; w++) s_wc[w][tid] = 0;
            __syncthreads();
            uint64_t peers = __ballot(in);
            for (uint32_t b = 0; b < 8; b++) {
                const uint64_t bal = __ballot((d >> b) & 1u);
                peers &= ((d >> b) & 1u) ? bal : ~bal;
            }
            if (in && !(peers & lt)) s_wc[wave][d] = __builtin_popcountll(peers);
            __syncthreads();
            if (in) {
                uint32_t pos = s_off[d] + __builtin_popcountll(peers & lt);
                for (uint32_t w = 0; w < wave; w++) pos += s_wc[w][d];
                for (uint32_t l = limb; l < pl; l++) kd[(size_t)l * N + base + pos] = ks[(size_t)l * N + base + i];
                id[base + pos] = is[base + i];
            }
            __syncthreads();
            s_off[tid] += s_wc[0][tid] + s_wc[1][tid] + s_wc[2][tid] + s_wc[3][tid];
            __syncthreads();
        }
        uint64_t *tk = ks;
        ks = kd;
        kd = tk;
        uint32_t *ti = is;
        is = id;
        id = ti;
        __syncthreads();
    }
    for (uint32_t i = tid; i < S.n; i += 256) {
        const uint32_t from = is[base + i];
        for (uint32_t b = 0; b < S.vs; b += 16)
            gst<u32x4>(S.values + (size_t)i * S.vs + b, gld<u32x4>(S.copy + (size_t)from * S.vs + b));
    }
}

static uint32_t key_limbs(uint32_t kind) { return kind == kKeyTimestamp ? 1 : kind == kKeyCompositeU128 ? 3 : 2; }

static uint64_t tiles_of(uint32_t n) { return (n + kSortTile - 1) / kSortTile; }
static uint64_t align256(uint64_t x) { return (x + 255) / 256 * 256; }

// Scratch layout (sort_scratch_bytes must match launch_sort_batch). The
// look-back words live in their own buffer (sort_status_words): epochs are
// only unique there.
struct SortScratch {
    uint64_t segs, tile_seg, tile_order, hist, counters, batch, bins, keys, idx, copies, total;
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
    s.segs = o;
    o += align256(sizeof(SortSeg) * count);
    s.tile_seg = o;
    o += align256(4 * tiles);
    s.tile_order = o;
    o += align256(4 * tiles);
    s.hist = o; // zeroed per batch: hist, counters, batch
    o += align256(4ull * nseg * kMaxPasses * kRadix);
    s.counters = o; // per pass: tile tickets, then (rest kernel) completed tiles
    o += align256(8ull * kMaxPasses);
    s.batch = o;
    o += align256(sizeof(SortBatch));
    s.bins = o;
    o += align256(4ull * nseg * kMaxPasses * kRadix);
    s.keys = o;
    o += 2 * align256(8 * N * kl);
    s.idx = o;
    o += 2 * align256(4 * N);
    s.copies = o;
    o += vals;
    s.total = o;
    return s;
}

uint64_t sort_scratch_bytes(const SortItem *items, uint32_t count) { return scratch_layout(items, count).total; }

uint64_t sort_status_words(const SortItem *items, uint32_t count) {
    uint64_t tiles = 0;
    for (uint32_t j = 0; j < count; j++)
        if (items[j].n >= 2) tiles += tiles_of(items[j].n);
    return tiles * kRadix;
}

// Everything is enqueued on `stream`; the host never waits. The table
// descriptors and tile map go through the caller's pinned staging (`host`,
// at least sort_host_bytes) which must stay untouched until the stream has
// passed this batch. `status` (sort_status_words, zeroed once when
// allocated) is reused by every pass: each pass launch takes a fresh epoch.
uint64_t sort_host_bytes(const SortItem *items, uint32_t count) {
    const SortScratch s = scratch_layout(items, count);
    return s.hist; // segs + tile map
}

int launch_sort_batch(const SortItem *items, uint32_t count, void *scratch, uint64_t scratch_bytes, uint64_t *status,
                      uint64_t status_words, uint32_t *epoch, void *host, void *stream) {
    const SortScratch L = scratch_layout(items, count);
    if (scratch_bytes < L.total || status_words < sort_status_words(items, count)) return -1;
    hipStream_t s = (hipStream_t)stream;
    uint8_t *base = (uint8_t *)scratch, *hbase = (uint8_t *)host;
    SortSeg *hsegs = (SortSeg *)(hbase + L.segs);
    uint32_t *htile = (uint32_t *)(hbase + L.tile_seg);
    uint32_t N = 0, nseg = 0, ntiles = 0;
    uint32_t max_kl = 0;
    uint64_t copy_off = L.copies;
    for (uint32_t j = 0; j < count; j++) {
        const SortItem &it = items[j];
        if (it.n < 2) continue;
        SortSeg g{};
        for (uint32_t l = 0; l < kMaxLimbs; l++) g.key_and[l] = ~0ull;
        g.values = (uint8_t *)it.values;
        g.copy = base + copy_off;
        copy_off += align256((uint64_t)it.n * it.value_size);
        g.n = it.n;
        g.vs = it.value_size;
        g.ts_off = it.timestamp_offset;
        g.kind = it.key_kind;
        g.kl = key_limbs(it.key_kind);
        g.item_base = N;
        g.tile_base = ntiles;
        g.tiles = (uint32_t)tiles_of(it.n);
        for (uint32_t t = 0; t < g.tiles; t++) htile[ntiles + t] = nseg;
        ntiles += g.tiles;
        N += it.n;
        max_kl = max_kl > g.kl ? max_kl : g.kl;
        hsegs[nseg++] = g;
    }
    if (!nseg) return 0;
    // Pass tile order: round-robin over the tables (local tile 0 of every
    // table, then local tile 1, ...). A table's tiles are still taken in
    // order (the look-back's progress guarantee), but fewer of one table's
    // tiles are in flight together, so a tile's look-back walk to the nearest
    // inclusive prefix is shorter.
    {
        uint32_t *horder = (uint32_t *)(hbase + L.tile_order), o = 0;
        for (uint32_t lt = 0; o < ntiles; lt++)
            for (uint32_t g = 0; g < nseg; g++)
                if (lt < hsegs[g].tiles) horder[o++] = hsegs[g].tile_base + lt;
    }
    SortSeg *d_segs = (SortSeg *)(base + L.segs);
    uint32_t *d_tile = (uint32_t *)(base + L.tile_seg);
    const uint32_t *d_order = (const uint32_t *)(base + L.tile_order);
    const uint64_t klw = align256(8ull * N * max_kl);
    uint64_t *keys0 = (uint64_t *)(base + L.keys), *keys1 = (uint64_t *)(base + L.keys + klw);
    uint32_t *idx0 = (uint32_t *)(base + L.idx), *idx1 = (uint32_t *)(base + L.idx + align256(4ull * N));
    uint32_t *hist = (uint32_t *)(base + L.hist), *bins = (uint32_t *)(base + L.bins);
    uint32_t *counters = (uint32_t *)(base + L.counters);
    SortBatch *d_batch = (SortBatch *)(base + L.batch);
    if (hipMemcpyAsync(base, hbase, L.hist, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemsetAsync(hist, 0, L.bins - L.hist, s) != hipSuccess)
        return -1;
    hipLaunchKernelGGL(k_sort_extract, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile);
    hipLaunchKernelGGL(k_sort_layout, dim3((nseg + 63) / 64), dim3(64), 0, s, d_segs, nseg);
    hipLaunchKernelGGL(k_sort_pack, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile, N, keys0, idx0, hist);
    hipLaunchKernelGGL(k_sort_plan, dim3(nseg), dim3(kRadix), 0, s, d_segs, d_batch, hist, bins);
    // Persistent: as many workgroups as are resident at once (VGPRs allow
    // three per CU): more would only start after the tiles run out, and an
    // idle pass (no table has that many bytes) costs its launch alone.
    static uint32_t resident = 0;
    if (!resident) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sort_pass, kSortThreads, 0) != hipSuccess ||
            hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1)
            return -1;
        resident = (uint32_t)(per_cu * cus);
    }
    const uint32_t pgrid = ntiles < resident ? ntiles : resident;
    const uint32_t passes = 8 * max_kl;
    for (uint32_t p = 0; p < passes && p < kDirectPasses; p++) {
        if (*epoch == 0) *epoch = 1; // 0 is the zeroed buffer's
        hipLaunchKernelGGL(k_sort_pass, dim3(pgrid), dim3(kSortThreads), 0, s, d_segs, d_batch, d_tile, d_order, p,
                           ntiles, N, keys0, keys1, idx0, idx1, bins, status, (*epoch)++, counters);
    }
    if (passes > kDirectPasses) {
        if (*epoch == 0 || *epoch + kMaxPasses < *epoch) *epoch = 1; // a fresh epoch per pass, none 0
        hipLaunchKernelGGL(k_sort_pass_rest, dim3(pgrid), dim3(kSortThreads), 0, s, d_segs, d_batch, d_tile, d_order,
                           ntiles, N, keys0, keys1, idx0, idx1, bins, status, *epoch, counters,
                           counters + kMaxPasses);
        *epoch += kMaxPasses;
    }
    hipLaunchKernelGGL(k_sort_fixup, dim3(ntiles), dim3(256), 0, s, d_segs, (const uint32_t *)d_tile,
                       (const uint32_t *)idx0, (const uint32_t *)idx1);
    hipLaunchKernelGGL(k_sort_rescue, dim3(nseg), dim3(256), 0, s, d_segs, N, keys0, keys1, idx0, idx1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace tbc
