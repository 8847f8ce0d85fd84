// sort.hip — TableMemory.sort (src/lsm/table_memory.zig:140-154) on gfx950.
//
// The reference sorts the mutable table's Values with std.mem.sort (Zig 0.11
// stable block sort) by key_from_value, only when puts arrived out of order
// (table_memory.zig:83-87). Stability is load-bearing: fill_immutable_values
// keeps the LAST of a run of equal keys (compaction.zig:519-522).
//
// A batch of memtables (every tree's at the bar end) is sorted by one
// enqueued launch sequence that never waits on the host. Every item is ONE
// 64-bit word: the key bits that vary over its table (packed), above the
// item's index in the table. The words are distinct, so any order of them is
// the stable order of the keys; a stable LSD radix sort with 8-bit digits
// over the packed bits moves 8 bytes per item per pass:
//
//   k_sort_extract  per tile of 4,096 items: a copy of the values (the
//                   gather's source), OR/AND of every key limb, and whether
//                   the table is out of order at all;
//   k_sort_layout   per table: the key bits that vary over the table as at
//                   most 8 runs of bits, most significant first (the others
//                   cannot decide any order), and the index width; config 3's
//                   composite u128 keys (account id, timestamp) pack into
//                   ~34 bits above an 18-bit index;
//   k_sort_pack     per tile: the words, the digit histograms of every packed
//                   digit, and which low-order digit prefixes the table is
//                   already in order on;
//   k_sort_plan     per table: LSD passes run from the least significant
//                   digit up, so the digits of a prefix the table is already
//                   in order on (a secondary index put in timestamp order)
//                   cannot change the stable order and are skipped; each
//                   remaining pass's digit; every digit's start;
//   k_sort_pass x P a workgroup per tile (persistent workgroups taking tickets
//                   when the tiles outnumber the resident workgroups); a pass
//                   no table needs returns at once. Onesweep: each tile ranks its items by
//                   digit (wave match ballots + per-wave counts: stable),
//                   publishes its digit counts, looks back over the tiles
//                   before it in its table for their prefix (decoupled
//                   look-back), and writes the tile out through LDS so each
//                   digit's run is contiguous;
//   k_sort_finish   values[i] = copy[index of sorted word i] (a gather with
//                   every workgroup's loads in flight, apart from the passes'
//                   register and LDS footprint).
//
// Tiles never straddle tables, so a table's passes are independent of the
// others' (a segmented sort with no table digit). Tables whose puts arrived
// in order are left untouched (table_memory.zig:141). Keys wider than the
// word holds are sorted on their top bits and each run of equal top bits is
// ordered by the full key (k_sort_finish; k_sort_rescue if a run is long).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <vector>

#include "tbc_internal.h"

namespace tbc {

constexpr uint32_t kSortThreads = 256;
constexpr uint32_t kSortWaves = kSortThreads / 64;
constexpr uint32_t kSortRounds = 16;
constexpr uint32_t kSortTile = kSortThreads * kSortRounds; // 4,096 items
constexpr uint32_t kRadix = 256;
constexpr uint32_t kMaxLimbs = 3;
constexpr uint32_t kMaxPasses = 8;  // 8-bit digits of a 64-bit word
constexpr uint32_t kMaxBytes = 8 * kMaxLimbs;
constexpr uint32_t kMaxRuns = 8;    // bit runs of a packed key
constexpr uint32_t kTopDigits = 4;  // truncated sorts keep at least this many top digits
constexpr uint32_t kRunMax = 64;    // longest run of equal top bits k_sort_finish orders
constexpr uint32_t kDirectPasses = 6; // passes with a launch each; the rest share k_sort_pass_rest

// Look-back words (64-bit): the pass launch's epoch in the top half (words
// of earlier launches read as "not published", so the buffer is zeroed once,
// never per pass), the flag in bits 31:30, the count below (< 2^30).
constexpr uint64_t kFlagAggregate = 1ull << 30;
constexpr uint64_t kFlagPrefix = 2ull << 30;
constexpr uint64_t kCountMask = (1ull << 30) - 1;

struct SortSeg {
    uint64_t key_or[kMaxLimbs], key_and[kMaxLimbs]; // over the table (extract)
    uint8_t *values;     // where the sorted table goes
    uint8_t *copy;       // n * vs bytes: the table as put, the gather's source
    const uint8_t *src;  // the table as put, for extract and pack (values in place, copy out of place)
    uint32_t oop;        // out of place: values is written, never read; copy is the caller's input
    uint32_t n, vs, ts_off, kind;
    uint32_t kl; // key limbs of the table's key kind
    uint32_t item_base, tile_base, tiles;
    uint32_t unsorted;  // some adjacent pair is out of key order (extract)
    uint32_t ib;        // index bits: word = packed key << ib | index (layout)
    uint32_t kbits;     // packed key bits (<= 64 - ib)
    uint32_t trunc;     // the key varies in more bits than the word holds: its lowest were dropped
    uint32_t ndig;      // 8-bit digits of the packed key (0: in order, untouched)
    uint32_t nruns;
    uint32_t run[kMaxRuns]; // limb | source bit << 8 | width << 16 | packed bit << 24
    uint32_t nbytes;    // varying key bytes (k_sort_rescue's full sort)
    uint32_t viol;      // bit j: out of order on packed digits [0, j] (pack)
    uint32_t active;    // bit p: pass p moves this table's items (plan)
    uint32_t final_buf; // buffer the last pass wrote
    uint32_t skip;      // digits [0, skip): the table is in order on them
    uint32_t top;       // fixup compares packed digits [top, ndig)
    uint32_t fix;       // runs of equal sorted bits are ordered by k_sort_finish
    uint32_t overflow;  // such a run too long to fix up: rescued
    uint32_t nact;      // passes of the table: pass q sorts on digit act[q]
    uint8_t byte_src[kMaxBytes]; // rescue: packed byte j = key byte byte_src[j] (limb * 8 + byte)
    uint8_t act[kMaxPasses];
};

struct SortBatch {
    uint32_t active; // passes some table needs
    uint32_t broken; // a pass hit a wait bound (a broken invariant): k_sort_rescue re-sorts every moved table
};

// key_from_value by kind (keys.h load_key), in two halves: key_raw issues
// the loads (three words, unconditionally: every offset lies inside a value
// of >= 16 bytes) and key_fix forms the limbs. Any use of a loaded word next
// to its load -- a branch by kind that masked it, a select against a default
// -- made the wave wait for that load right there, so a row "prefetched"
// this way was not in flight while the previous row was packed.
struct KeyRaw {
    uint64_t w[3];
};
__device__ __forceinline__ KeyRaw key_raw(uint32_t kind, const uint8_t *v, uint32_t ts_off) {
    const uint32_t o0 = kind == kKeyTimestamp ? ts_off : kind == kKeyIdU128 ? 0u : kind == kKeyCompositeU64 ? 8u : 16u;
    const uint32_t o1 = kind == kKeyIdU128 ? 8u : 0u;
    KeyRaw r;
    r.w[0] = gld<uint64_t>(v + o0);
    r.w[1] = gld<uint64_t>(v + o1);
    r.w[2] = gld<uint64_t>(v + 8);
    return r;
}
__device__ __forceinline__ void key_fix(uint32_t kind, const KeyRaw &r, uint64_t k[3]) {
    k[0] = kind == kKeyIdU128 ? r.w[0] : r.w[0] & ~kTombstoneBit;
    k[1] = kind == kKeyTimestamp ? 0ull : r.w[1];
    k[2] = kind == kKeyCompositeU128 ? r.w[2] : 0ull;
}
__device__ __forceinline__ void key_of(uint32_t kind, const uint8_t *v, uint32_t ts_off, uint64_t k[3]) {
    key_fix(kind, key_raw(kind, v, ts_off), k);
}

__host__ __device__ __forceinline__ uint64_t low_mask(uint32_t bits) { return bits >= 64 ? ~0ull : (1ull << bits) - 1; }

// The packed key: every run's bits at its packed position. The runs are
// uniform and sit in registers, every run unrolled (round 3, one box: from
// LDS per item, config 3's pack 68 us; from registers, 61).
__device__ __forceinline__ uint64_t pack_bits(const uint32_t (&runs)[kMaxRuns], uint32_t nr, const uint64_t k[3]) {
    uint64_t p = 0;
#pragma unroll
    for (uint32_t r = 0; r < kMaxRuns; r++) {
        if (r >= nr) break;
        const uint32_t d = runs[r], limb = d & 3, src = (d >> 8) & 63, w = (d >> 16) & 127, at = d >> 24;
        const uint64_t x = limb == 0 ? k[0] : limb == 1 ? k[1] : k[2];
        p |= ((x >> src) & low_mask(w)) << at;
    }
    return p;
}

// hist / bins layout: [segment][pass][digit] u32.
__device__ __forceinline__ uint32_t *seg_hist(uint32_t *hist, uint32_t s) { return hist + (size_t)s * kMaxPasses * kRadix; }

// The key and the next item's key (the next lane's; lane 63 loads its
// neighbour, which may sit in the next tile) of every lane of a row.
// row_issue issues both loads (indices clamped into the table: a lane past
// the end re-reads the last item, and callers use only lanes inside it);
// row_form makes the keys and the neighbours once they are in.
struct RowRaw {
    KeyRaw k, kx;
};
__device__ __forceinline__ RowRaw row_issue(const SortSeg &S, uint32_t li) {
    const uint32_t n = S.n, i0 = li < n ? li : n - 1;
    const uint32_t i1 = ((threadIdx.x & 63) == 63 && li + 1 < n) ? li + 1 : i0;
    RowRaw r;
    r.k = key_raw(S.kind, S.src + (size_t)i0 * S.vs, S.ts_off);
    r.kx = key_raw(S.kind, S.src + (size_t)i1 * S.vs, S.ts_off);
    return r;
}
__device__ __forceinline__ void row_form(const SortSeg &S, uint32_t li, const RowRaw &r, uint64_t k[3],
                                         uint64_t kn[3]) {
    uint64_t kx[3];
    key_fix(S.kind, r.k, k);
    key_fix(S.kind, r.kx, kx);
    for (uint32_t l = 0; l < 3; l++) kn[l] = __shfl_down(k[l], 1, 64);
    if ((threadIdx.x & 63) == 63 && li + 1 < S.n)
        for (uint32_t l = 0; l < 3; l++) kn[l] = kx[l];
}
// In place (extract's copying path): the keys of a row used at once, only
// lane 63 loading its neighbour.
__device__ __forceinline__ void row_keys(const SortSeg &S, uint32_t li, uint64_t k[3], uint64_t kn[3]) {
    uint64_t kx[3] = {0, 0, 0};
    k[0] = k[1] = k[2] = 0;
    if (li < S.n) key_of(S.kind, S.src + (size_t)li * S.vs, S.ts_off, k);
    if ((threadIdx.x & 63) == 63 && li + 1 < S.n) key_of(S.kind, S.src + (size_t)(li + 1) * S.vs, S.ts_off, kx);
    for (uint32_t l = 0; l < 3; l++) kn[l] = __shfl_down(k[l], 1, 64);
    if ((threadIdx.x & 63) == 63 && li + 1 < S.n)
        for (uint32_t l = 0; l < 3; l++) kn[l] = kx[l];
}

// --------------------------------------------------------------------------
// Extract: one workgroup per tile.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(kSortThreads) void k_sort_extract(SortSeg *segs, const uint32_t *tile_seg) {
    __shared__ uint64_t s_or[kMaxLimbs][kSortWaves], s_and[kMaxLimbs][kSortWaves];
    __shared__ uint32_t s_uns;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint32_t sg = tile_seg[blockIdx.x];
    const SortSeg S = segs[sg]; // a copy: the stores below may not alias it
    const uint32_t n = S.n, vs = S.vs, kl = S.kl;
    const uint32_t lt = blockIdx.x - S.tile_base;
    if (tid == 0) s_uns = 0;
    __syncthreads();
    uint64_t o[kMaxLimbs] = {0, 0, 0}, a[kMaxLimbs] = {~0ull, ~0ull, ~0ull};
    uint32_t uns = 0;
    // Out of place, the caller's input is the gather's source: keys only,
    // the next row's loaded while a row is folded in (as k_sort_pack).
    const uint32_t left = n - lt * kSortTile; // > 0: the tile is in the table
    const uint32_t rows = left >= kSortTile ? kSortRounds : (left + kSortThreads - 1) / kSortThreads;
    if (S.oop) {
        RowRaw cur = row_issue(S, lt * kSortTile + tid);
        for (uint32_t r = 0; r < rows; r++) {
            const uint32_t li = lt * kSortTile + r * kSortThreads + tid;
            const RowRaw nxt = row_issue(S, r + 1 < rows ? li + kSortThreads : li); // the last row re-reads itself
            uint64_t k[3], kn[3];
            row_form(S, li, cur, k, kn);
            if (li < n) {
                for (uint32_t l = 0; l < kl; l++) {
                    o[l] |= k[l];
                    a[l] &= k[l];
                }
                if (li + 1 < n) {
                    int cmp = 0;
                    for (uint32_t l = 0; l < kl; l++)
                        if (k[l] != kn[l]) cmp = k[l] > kn[l] ? 1 : -1;
                    uns |= cmp > 0 ? 1u : 0u;
                }
            }
            cur = nxt;
        }
    }
    for (uint32_t r = 0; !S.oop && r < rows; r++) {
        const uint32_t li = lt * kSortTile + r * kSortThreads + tid;
        const bool in = li < n;
        // The row's first 128 bytes of every value are loaded with its keys
        // (one round trip), then stored; longer values loop.
        u32x4 v[8];
        if (in) {
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
                if (16 * q < vs) v[q] = gld<u32x4>(S.values + (size_t)li * vs + 16 * q);
        }
        uint64_t k[3], kn[3];
        row_keys(S, li, k, kn);
        if (!in) continue;
#pragma unroll
        for (uint32_t q = 0; q < 8; q++)
            if (16 * q < vs) gst<u32x4>(S.copy + (size_t)li * vs + 16 * q, v[q]);
        for (uint32_t b = 128; b < vs; b += 128) { // up to 8 loads in flight before their stores
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
                if (b + 16 * q < vs) v[q] = gld<u32x4>(S.values + (size_t)li * vs + b + 16 * q);
#pragma unroll
            for (uint32_t q = 0; q < 8; q++)
                if (b + 16 * q < vs) gst<u32x4>(S.copy + (size_t)li * vs + b + 16 * q, v[q]);
        }
        for (uint32_t l = 0; l < kl; l++) {
            o[l] |= k[l];
            a[l] &= k[l];
        }
        if (li + 1 < n) {
            int cmp = 0;
            for (uint32_t l = 0; l < kl; l++)
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
    if (tid < kl) {
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

// Layout: one workgroup (its first thread) per table. The varying bits of every limb, most
// significant limb and bit first, as runs of consecutive bits; while there
// are more than kMaxRuns, the two same-limb runs with the smallest gap merge
// (the constant bits between them are kept: they cannot decide any order).
// The word holds 64 - ib key bits: beyond that, the lowest are dropped
// (trunc) and k_sort_finish orders the resulting runs of equal words.
__global__ __launch_bounds__(64) void k_sort_layout(SortSeg *segs) {
    __shared__ uint8_t rl[kMaxLimbs * 32], rs[kMaxLimbs * 32], rw[kMaxLimbs * 32]; // LDS, not scratch
    if (threadIdx.x) return;
    SortSeg &S = segs[blockIdx.x];
    S.nbytes = S.ndig = S.nruns = 0;
    if (!S.unsorted) return;
    // The fields read below, once: S is written as it is filled in, so every
    // read after a write to it was a fresh load waited for alone.
    const uint32_t kl = S.kl, n = S.n;
    uint64_t vary[kMaxLimbs];
    for (uint32_t l = 0; l < kMaxLimbs; l++) vary[l] = l < kl ? S.key_or[l] ^ S.key_and[l] : 0;
    uint32_t nb = 0;
    for (uint32_t l = 0; l < kl; l++)
        for (uint32_t b = 0; b < 8; b++)
            if ((vary[l] >> (8 * b)) & 255) S.byte_src[nb++] = (uint8_t)(8 * l + b);
    S.nbytes = nb;
    // Runs (limb, lowest bit, width), most significant first.
    uint32_t nr = 0;
    for (int l = (int)kl - 1; l >= 0; l--) {
        uint64_t m = vary[l];
        while (m) {
            const uint32_t hi = 63 - __builtin_clzll(m);
            const uint64_t gaps = ~m & low_mask(hi + 1); // clear bits at or below hi
            const uint32_t lo = gaps ? 64 - __builtin_clzll(gaps) : 0;
            rl[nr] = (uint8_t)l;
            rs[nr] = (uint8_t)lo;
            rw[nr] = (uint8_t)(hi - lo + 1);
            nr++;
            m &= low_mask(lo);
        }
    }
    while (nr > kMaxRuns) {
        uint32_t best = 0, gap = ~0u;
        for (uint32_t r = 0; r + 1 < nr; r++)
            if (rl[r] == rl[r + 1] && rs[r] - (rs[r + 1] + rw[r + 1]) < gap) {
                gap = rs[r] - (rs[r + 1] + rw[r + 1]);
                best = r;
            }
        if (gap == ~0u) break; // cannot happen with <= 3 limbs (some limb has 3 runs)
        rw[best] = (uint8_t)(rs[best] + rw[best] - rs[best + 1]);
        rs[best] = rs[best + 1];
        for (uint32_t r = best + 1; r + 1 < nr; r++) {
            rl[r] = rl[r + 1];
            rs[r] = rs[r + 1];
            rw[r] = rw[r + 1];
        }
        nr--;
    }
    const uint32_t ib = 32 - __builtin_clz(n - 1); // n >= 2
    uint32_t v = 0;
    for (uint32_t r = 0; r < nr; r++) v += rw[r];
    uint32_t trunc = 0;
    while (v > 64 - ib) { // drop the lowest bits
        trunc = 1;
        const uint32_t cut = v - (64 - ib);
        if (rw[nr - 1] <= cut) {
            v -= rw[--nr];
        } else {
            rs[nr - 1] = (uint8_t)(rs[nr - 1] + cut);
            rw[nr - 1] = (uint8_t)(rw[nr - 1] - cut);
            v -= cut;
        }
    }
    uint32_t at = v;
    for (uint32_t r = 0; r < nr; r++) {
        at -= rw[r];
        S.run[r] = rl[r] | (uint32_t)rs[r] << 8 | (uint32_t)rw[r] << 16 | at << 24;
    }
    S.trunc = trunc;
    S.nruns = nr;
    S.ib = ib;
    S.kbits = v;
    S.ndig = (v + 7) / 8;
}

// One wave's 64 digits into an LDS histogram row: a digit shared by the
// whole row (a slowly varying key byte) is one add; otherwise every lane adds
// its own (the LDS serialises equal addresses). Round 3, one box: grouping
// equal digits first by 8 match ballots (one add per distinct digit) cost
// more VALU than it saved -- config 3's pack 100 -> 67 us without it.
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
    if (in) atomicAdd(&row[d], 1u);
}

// Pack: one workgroup per tile of an unsorted table.
__global__ __launch_bounds__(kSortThreads) void k_sort_pack(SortSeg *segs, const uint32_t *tile_seg,
                                                            uint64_t *words, uint32_t *hist) {
    __shared__ uint32_t s_hist[kMaxPasses][kRadix];
    __shared__ uint32_t s_viol;
    const uint32_t tid = threadIdx.x;
    const uint32_t sg = tile_seg[blockIdx.x];
    const SortSeg S = segs[sg]; // a copy: the stores below may not alias it
    const uint32_t nd = S.ndig, nr = S.nruns, ib = S.ib, n = S.n;
    if (!nd) return; // uniform: a sorted table
    for (uint32_t j = 0; j < nd; j++) s_hist[j][tid] = 0;
    uint32_t runs[kMaxRuns]; // constant indices only (registers; S.run[tid] would put S in scratch)
#pragma unroll
    for (uint32_t r = 0; r < kMaxRuns; r++) runs[r] = segs[sg].run[r];
    if (tid == 0) s_viol = 0;
    __syncthreads();
    const uint32_t lt = blockIdx.x - S.tile_base;
    uint32_t viol = 0;
    const uint32_t left = n - lt * kSortTile; // > 0: the tile is in the table
    const uint32_t rows = left >= kSortTile ? kSortRounds : (left + kSortThreads - 1) / kSortThreads;
    // The next row's keys load while a row is packed (round 3, one box, with
    // S out of scratch: config 3's pack 119 -> 100 us; two rows ahead: 98).
    RowRaw cur = row_issue(S, lt * kSortTile + tid);
    for (uint32_t r = 0; r < rows; r++) {
        const uint32_t li = lt * kSortTile + r * kSortThreads + tid;
        const bool in = li < n;
        const RowRaw nxt = row_issue(S, r + 1 < rows ? li + kSortThreads : li); // the last row re-reads itself
        uint64_t k[3], kn[3];
        row_form(S, li, cur, k, kn);
        const uint64_t p = pack_bits(runs, nr, k);
        if (in) gst<uint64_t>(words + S.item_base + li, p << ib | li);
        for (uint32_t j = 0; j < nd; j++) hist_add(s_hist[j], (uint32_t)(p >> (8 * j)) & 255u, in);
        if (in && li + 1 < n) {
            const uint64_t q = pack_bits(runs, nr, kn);
            for (uint32_t j = 0; j < nd; j++) { // out of order on digits [0, j]: the low 8(j+1) bits
                const uint64_t m = low_mask(8 * (j + 1));
                if ((p & m) > (q & m)) viol |= 1u << j;
            }
        }
        cur = nxt;
    }
    if (viol) atomicOr(&s_viol, viol);
    __syncthreads();
    uint32_t *h = seg_hist(hist, sg);
    for (uint32_t j = 0; j < nd; j++)
        if (s_hist[j][tid]) atomicAdd(&h[j * kRadix + tid], s_hist[j][tid]);
    if (tid == 0 && s_viol) atomicOr(&segs[sg].viol, s_viol);
}

// Plan: one workgroup per table. Passes [skip, ndig) run, where the table
// is already in order on digits [0, skip) (the largest such prefix); then
// the digit starts of those passes.
__global__ __launch_bounds__(kRadix) void k_sort_plan(SortSeg *segs, SortBatch *batch, const uint32_t *hist,
                                                      uint32_t *bins) {
    const uint32_t s = blockIdx.x, d = threadIdx.x, lane = d & 63, wave = d >> 6;
    __shared__ uint32_t wsum[kRadix / 64];
    SortSeg &S = segs[s];
    const uint32_t nd = S.ndig;
    uint32_t skip = 0;
    for (uint32_t j = 1; j < nd; j++)
        if (!((S.viol >> (j - 1)) & 1u)) skip = j;
    // Many varying digits (random u64/u128 fields): sort on the top digits
    // only (at least kTopDigits, 10 bits beyond log2 n) and let k_sort_finish
    // order each run of equal top digits by the full key -- when the top
    // digits' histograms predict short runs: n x prod(largest digit share)
    // <= 1 if the digits were independent. Clustered keys (config 3's Zipf
    // accounts) keep every pass; a misprediction costs k_sort_rescue.
    const uint32_t *h = hist + (size_t)s * kMaxPasses * kRadix;
    const uint32_t log2n = 32 - __builtin_clz(S.n | 1);
    const uint32_t top_digits = (log2n + 10 + 7) / 8 > kTopDigits ? (log2n + 10 + 7) / 8 : kTopDigits;
    uint32_t first = skip;
    if (nd - skip > top_digits) {
        __shared__ uint32_t wmax[kRadix / 64];
        float est = (float)S.n;
        for (uint32_t b = nd - top_digits; b < nd; b++) {
            uint32_t mx = h[b * kRadix + d];
            for (int o = 32; o > 0; o >>= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
            if (lane == 0) wmax[wave] = mx;
            __syncthreads();
            mx = max(max(wmax[0], wmax[1]), max(wmax[2], wmax[3]));
            __syncthreads();
            est *= (float)mx / (float)S.n;
        }
        if (est <= 1.0f) first = nd - top_digits;
    }
    uint32_t active = 0;
    for (uint32_t p = first; p < nd; p++) active |= 1u << p;
    __syncthreads(); // every thread has read viol before thread 0 writes the plan
    if (d == 0) {
        S.active = active;
        S.nact = nd - first;
        for (uint32_t q = 0; q < nd - first; q++) S.act[q] = (uint8_t)(first + q);
        S.final_buf = (nd - first) & 1u;
        S.skip = skip;
        S.top = first > skip ? first : 0;
        S.fix = (first > skip || S.trunc) ? 1u : 0u;
        if (nd > first) atomicOr(&batch->active, (1u << (nd - first)) - 1u); // pass q runs if some table has > q
    }
    uint32_t *out = bins + (size_t)s * kMaxPasses * kRadix;
    const uint32_t item_base = S.item_base; // read once: the stores below may alias S
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
        out[p * kRadix + d] = item_base + off + incl - c;
        __syncthreads();
    }
}

// --------------------------------------------------------------------------
// One onesweep pass (digit = packed digit act[p] of the table's words).
// --------------------------------------------------------------------------
__device__ __forceinline__ uint64_t lb_load(const uint64_t *p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(uint64_t *p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Persistent workgroups take tiles in ticket order when they are free: every
// tile one looks back on was taken by a workgroup that is running or done.
// (Taking the next ticket one tile ahead, to hide its round trip, measured
// slower: config 3's passes 58 vs 44 us, as a reserved tile's successors
// wait on it for a whole tile.)
struct PassShared {
    uint32_t next;
    uint32_t wcnt[kSortWaves][kRadix]; // per wave: running, then total counts
    uint32_t start[kRadix];            // local start of each digit in the tile
    uint32_t off[kRadix];              // destination of the digit's tile-local position 0 (mod 2^32)
    uint32_t wsum[kSortWaves];
    uint64_t word[kSortTile];
    uint8_t dig[kSortTile];
};

// Pass p over the tiles taken from tile_counter[p] (ticket order), until
// they run out. `done` (the rest kernel only): every finished tile adds one
// to done[p] after an agent-scope release, and before its first tile of pass
// p a workgroup waits for done[p - 1] == ntiles and acquires (the pass reads
// what every tile of the previous pass wrote, on any XCD).
__device__ __forceinline__ void sort_pass_tiles(PassShared &sh, const SortSeg *segs, const uint32_t *tile_seg,
                                                const uint32_t *tile_order, uint32_t p, uint32_t ntiles,
                                                uint64_t *words0, uint64_t *words1, const uint32_t *bins,
                                                uint64_t *status, uint32_t epoch, uint32_t *tile_counter,
                                                uint32_t *done, SortBatch *batch) {
    constexpr uint32_t R = kSortRounds;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const uint64_t ep = (uint64_t)epoch << 32;
    const uint64_t lt_mask = (1ull << lane) - 1;
    // The first pass of the rest kernel follows a kernel boundary: nothing to wait for.
    bool waited = done == nullptr || p == kDirectPasses;
    const bool from1 = (p & 1u) != 0; // passes alternate buffers, the first reads buffer 0
    const uint64_t *src = from1 ? words1 : words0;
    uint64_t *dstw = from1 ? words0 : words1;
    for (bool first = true;; first = false) {
        // Every wave releases its own stores of the previous tile (at agent
        // scope: waits for them and writes the XCD's L2 back) before the
        // tile is counted as done.
        if (!first && done) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads(); // the previous tile's LDS readers are done; sh.next is written
        if (!first && done && tid == 0)
            __hip_atomic_fetch_add(&done[p], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // Null counter (one tile per workgroup): the tile is the workgroup's
        // index. Workgroups are dispatched in index order on each XCD, so the
        // lowest undispatched tile's XCD only holds tiles below it, which
        // wait only on tiles further below: they finish and it is dispatched
        // (other kernels' workgroups on its CUs, e.g. chains on a tail
        // stream, never wait on this sort, so they leave too). HIP does not
        // promise that dispatch order; were it broken, a look-back wait
        // would reach its bound (2^24 sleeps, below) and mark the batch
        // broken, and k_sort_rescue re-sorts its tables: slower, still in
        // order, never a hang. TBC_SORT_TICKETS=1 keeps the tickets always.
        // (Config 1's passes 30.2 -> 24.9 us: the ticket's device-scope
        // atomic, one per tile on one word, cost ~5 us per pass.)
        if (tid == 0) sh.next = tile_counter ? atomicAdd(&tile_counter[p], 1u) : (first ? blockIdx.x : ntiles);
        __syncthreads();
        const uint32_t tile = sh.next;
        if (tile >= ntiles) return; // uniform
        for (uint32_t i = tid; i < kSortWaves * kRadix; i += kSortThreads) (&sh.wcnt[0][0])[i] = 0;
        __syncthreads(); // every thread has read sh.next
        if (!waited) { // rest kernel: every tile of pass p - 1 is complete and visible
            if (tid == 0) {
                for (uint32_t spins = 0; __hip_atomic_load(&done[p - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                                             ntiles;) {
                    if (++spins > (1u << 26)) { // bounded: a broken invariant, reported, not a hang
                        atomicOr(&batch->broken, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            }
            __syncthreads();
            waited = true;
        }
        const uint32_t t = tile_order[tile];
        const uint32_t sg = tile_seg[t];
        const SortSeg &S = segs[sg];
        const uint32_t nact = S.nact;
        if (p >= nact) continue; // uniform: the table's passes are done (or it is in order)
        const uint32_t pd = S.act[p];              // this pass's digit for the table
        const uint32_t shift = S.ib + 8 * pd;
        const uint32_t lt = t - S.tile_base;
        const uint32_t base = S.item_base + lt * kSortTile;
        const uint32_t m = (S.n - lt * kSortTile) < kSortTile ? (S.n - lt * kSortTile) : kSortTile;
        const uint32_t bin_d = bins[((size_t)sg * kMaxPasses + pd) * kRadix + tid]; // thread = digit (below)

        // Wave w owns items [1024 w, 1024 w + 1024) of the tile, 64 per round
        // in lane order: stable rank = (earlier waves) + (earlier rounds of
        // this wave, counted in wcnt) + (earlier lanes with the same digit).
        uint32_t rd[R]; // rank << 8 | digit
        uint64_t w[R];
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t e = wave * (64 * R) + r * 64 + lane;
            w[r] = e < m ? gld<uint64_t>(src + base + e) : 0ull;
        }
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t e = wave * (64 * R) + r * 64 + lane;
            const bool in = e < m;
            const uint32_t d = in ? (uint32_t)(w[r] >> shift) & 255u : 0u;
            uint64_t peers = __ballot(in);
#pragma unroll
            for (uint32_t b = 0; b < 8; b++) {
                const uint64_t bal = __ballot((d >> b) & 1u);
                peers &= ((d >> b) & 1u) ? bal : ~bal;
            }
            const uint32_t before = __builtin_popcountll(peers & lt_mask);
            const uint32_t prior = in ? sh.wcnt[wave][d] : 0u;
            __builtin_amdgcn_wave_barrier();
            if (in && before == 0) sh.wcnt[wave][d] = prior + (uint32_t)__builtin_popcountll(peers);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            rd[r] = (prior + before) << 8 | d;
        }
        __syncthreads();
        // Per digit (thread d): counts of the tile, exclusive prefix over
        // waves, and the tile-local start (exclusive scan over digits).
        const uint32_t d = tid;
        uint32_t cnt = 0, wpre[kSortWaves];
#pragma unroll
        for (uint32_t v = 0; v < kSortWaves; v++) {
            wpre[v] = cnt;
            cnt += sh.wcnt[v][d];
        }
        {
            uint32_t incl = cnt;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, 64);
                if (lane >= (uint32_t)o) incl += y;
            }
            if (lane == 63) sh.wsum[wave] = incl;
            __syncthreads();
            uint32_t off = 0;
            for (uint32_t v = 0; v < wave; v++) off += sh.wsum[v];
            sh.start[d] = off + incl - cnt;
        }
        __syncthreads();
#pragma unroll
        for (uint32_t v = 0; v < kSortWaves; v++) sh.wcnt[v][d] = wpre[v]; // becomes the wave's offset
        __syncthreads(); // every digit's wave offsets are in place
        // Tile-local sorted position of every item; words and digits into LDS.
#pragma unroll
        for (uint32_t r = 0; r < R; r++) {
            const uint32_t e = wave * (64 * R) + r * 64 + lane;
            if (e < m) {
                const uint32_t dg = rd[r] & 255u;
                const uint32_t pos = sh.start[dg] + sh.wcnt[wave][dg] + (rd[r] >> 8);
                sh.word[pos] = w[r];
                sh.dig[pos] = (uint8_t)dg;
            }
        }
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
                for (uint32_t i = 0; i < kLook; i++)
                    v[i] = pred >= S.tile_base + i ? lb_load(&status[(size_t)(pred - i) * kRadix + d]) : 0ull;
                bool fin = false, stall = false;
#pragma unroll
                for (uint32_t i = 0; i < kLook; i++) {
                    if (fin || stall) continue;
                    if ((v[i] >> 32) != epoch || !(v[i] & (3ull << 30))) { // not published by this pass yet
                        stall = true;
                        pred -= i;
                        continue;
                    }
                    excl += (uint32_t)(v[i] & kCountMask);
                    if ((v[i] & (3ull << 30)) == kFlagPrefix || pred - i == S.tile_base) fin = true;
                }
                if (fin) break;
                if (stall) {
                    if (++spins > (1u << 24)) { // bounded: a broken invariant, reported, not a hang
                        atomicOr(&batch->broken, 1u);
                        break;
                    }
                    __builtin_amdgcn_s_sleep(1);
                } else {
                    pred -= kLook;
                }
            }
            lb_store(&status[(size_t)t * kRadix + d], ep | kFlagPrefix | (excl + cnt));
        }
        sh.off[d] = bin_d + excl - sh.start[d];
        __syncthreads(); // every digit's destination is in place
        // Sorted position j (digit dj) goes to off[dj] + j: each digit's run
        // lands contiguously.
#pragma unroll 4
        for (uint32_t q = 0; q < R; q++) {
            const uint32_t j = tid + kSortThreads * q;
            if (j < m) gst<uint64_t>(dstw + sh.off[sh.dig[j]] + j, sh.word[j]);
        }
    }
}

// One launch per pass below kDirectPasses: the kernel boundary orders the
// passes. A pass no table needs returns at once.
__global__ __launch_bounds__(kSortThreads, 3) void k_sort_pass(const SortSeg *segs, SortBatch *batch,
                                                            const uint32_t *tile_seg, const uint32_t *tile_order,
                                                            uint32_t p, uint32_t ntiles, uint64_t *words0,
                                                            uint64_t *words1, const uint32_t *bins, uint64_t *status,
                                                            uint32_t epoch, uint32_t *tile_counter) {
    __shared__ PassShared sh;
    if (!((batch->active >> p) & 1u)) return; // uniform: no table has this many passes
    sort_pass_tiles(sh, segs, tile_seg, tile_order, p, ntiles, words0, words1, bins, status, epoch, tile_counter,
                    nullptr, batch);
}

// Passes [kDirectPasses, kMaxPasses) in ONE launch (most batches need none:
// a truncated sort keeps at least 4 digits, an in-order prefix is skipped):
// workgroups take pass p's tiles after pass p - 1's tickets ran out, so a
// tile only ever waits on tiles already taken by running workgroups (no
// grid barrier, no residency assumption), and the completion counters with
// agent-scope release/acquire order the passes across XCDs. Each pass takes
// a fresh look-back epoch.
__global__ __launch_bounds__(kSortThreads, 3) void k_sort_pass_rest(const SortSeg *segs, SortBatch *batch,
                                                                 const uint32_t *tile_seg, const uint32_t *tile_order,
                                                                 uint32_t ntiles, uint64_t *words0, uint64_t *words1,
                                                                 const uint32_t *bins, uint64_t *status,
                                                                 uint32_t epoch0, uint32_t *tile_counter,
                                                                 uint32_t *done) {
    __shared__ PassShared sh;
    for (uint32_t p = kDirectPasses; p < kMaxPasses; p++) {
        if (!((batch->active >> p) & 1u)) return; // passes run as a prefix: none beyond either
        sort_pass_tiles(sh, segs, tile_seg, tile_order, p, ntiles, words0, words1, bins, status,
                        epoch0 + (p - kDirectPasses), tile_counter, done, batch);
        // Its last tile's stores are released and counted before the next pass.
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
    }
}

// --------------------------------------------------------------------------
// Finish: every sorted table's values from its sorted words, 1,024 sorted
// positions per workgroup. Exact tables gather: values[i] = copy[index of
// word i] (reads at random, writes in order; eight values' loads in flight
// per lane before their stores). Fixed-up tables (truncated words, or passes
// on the top digits only): the passes ordered the words by their digits
// [top, ndig) (stable); each run of equal such digits is put in full-key order
// (ties by put order, i.e. by item index: stability), one thread per sorted
// position, runs found on the sorted words, keys re-read from the put-order
// copy; a run longer than kRunMax marks the table for k_sort_rescue.
// --------------------------------------------------------------------------
constexpr uint32_t kFinishItems = 1024;

__device__ __forceinline__ bool key_before(const uint64_t a[3], uint32_t ia, const uint64_t b[3], uint32_t ib) {
    for (int l = 2; l >= 0; l--)
        if (a[l] != b[l]) return a[l] < b[l];
    return ia < ib;
}

// One value of C 16-byte chunks: every load issued before the first store.
template <uint32_t C> __device__ __forceinline__ void copy_value(uint8_t *dst, const uint8_t *src) {
    u32x4 v[C];
#pragma unroll
    for (uint32_t c = 0; c < C; c++) v[c] = gld<u32x4>(src + 16 * c);
#pragma unroll
    for (uint32_t c = 0; c < C; c++) gst<u32x4>(dst + 16 * c, v[c]);
}

// One value of vs bytes (a power of two >= 16; uniform across the wave).
__device__ __forceinline__ void copy_any(uint8_t *dst, const uint8_t *src, uint32_t vs) {
    switch (vs >> 4) {
    case 1: copy_value<1>(dst, src); break;
    case 2: copy_value<2>(dst, src); break;
    case 4: copy_value<4>(dst, src); break;
    case 8: copy_value<8>(dst, src); break;
    default: // 256 bytes and up
        for (uint32_t b = 0; b < vs; b += 256) copy_value<16>(dst + b, src + b);
        break;
    }
}

__global__ __launch_bounds__(256) void k_sort_finish(SortSeg *segs, const uint32_t *tile_seg, const uint64_t *words0,
                                                     const uint64_t *words1) {
    const uint32_t tile = blockIdx.x / (kSortTile / kFinishItems);
    const uint32_t sg = tile_seg[tile];
    const SortSeg S = segs[sg];
    const uint32_t n = S.n, vs = S.vs, tid = threadIdx.x;
    const uint32_t first = (tile - S.tile_base) * kSortTile + (blockIdx.x % (kSortTile / kFinishItems)) * kFinishItems;
    if (!S.nact) { // uniform: in order; in place untouched, out of place copied as is
        if (!S.oop || first >= n) return;
        const uint32_t last = first + kFinishItems < n ? first + kFinishItems : n;
        const uint32_t chunks = (last - first) * (vs >> 4);
        const uint8_t *src = S.copy + (size_t)first * vs;
        uint8_t *dst = S.values + (size_t)first * vs;
        for (uint32_t c0 = 0; c0 < chunks; c0 += 8 * 256) { // eight loads in flight per lane, then their stores
            u32x4 v[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t c = c0 + q * 256 + tid;
                v[q] = gld<u32x4>(src + 16 * (size_t)(c < chunks ? c : chunks - 1));
            }
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t c = c0 + q * 256 + tid;
                if (c < chunks) gst<u32x4>(dst + 16 * (size_t)c, v[q]);
            }
        }
        return;
    }
    const uint64_t *wv = (S.final_buf ? words1 : words0) + S.item_base; // the table's sorted words
    const uint64_t imask = low_mask(S.ib);
    if (first >= n) return;
    const uint32_t last = first + kFinishItems < n ? first + kFinishItems : n;
    if (!S.fix) {
        const uint32_t cpv = vs >> 4, vpr = 256 / cpv; // values per row of the workgroup
        const uint32_t jl = tid / cpv, part = tid % cpv;
        if (jl >= vpr) return;
        for (uint32_t j0 = first; j0 < last; j0 += 8 * vpr) {
            // Loads issued unconditionally (indices clamped into the range),
            // so that all eight words, then all eight values, are in flight
            // together: loads behind a branch each ended in their own wait.
            uint32_t from[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t j = j0 + q * vpr + jl;
                from[q] = (uint32_t)(wv[j < last ? j : last - 1] & imask);
            }
            u32x4 v[8];
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) v[q] = gld<u32x4>(S.copy + (size_t)from[q] * vs + 16 * part);
#pragma unroll
            for (uint32_t q = 0; q < 8; q++) {
                const uint32_t j = j0 + q * vpr + jl;
                if (j < last) gst<u32x4>(S.values + (size_t)j * vs + 16 * part, v[q]);
            }
        }
        return;
    }
    const uint32_t sh = S.ib + 8 * S.top;
    for (uint32_t i = first + tid; i < last; i += 256) {
        // The word and both neighbours at once: most runs of equal top
        // digits are one item long (the plan predicted so), and such an item
        // is copied straight to its place, every chunk's load before a store.
        const uint64_t wi = wv[i], ti = wi >> sh;
        const uint64_t wp = wv[i > 0 ? i - 1 : i], wn = wv[i + 1 < n ? i + 1 : i];
        if ((i == 0 || (wp >> sh) != ti) && (i + 1 >= n || (wn >> sh) != ti)) {
            copy_any(S.values + (size_t)i * vs, S.copy + (size_t)(uint32_t)(wi & imask) * vs, vs);
            continue;
        }
        // run bounds [lo, hi) of equal top digits around i
        uint32_t lo = i, hi = i + 1;
        while (lo > 0 && (wv[lo - 1] >> sh) == ti && i - lo < kRunMax) lo--;
        while (hi < n && (wv[hi] >> sh) == ti && hi - lo <= kRunMax) hi++;
        if (hi - lo > kRunMax) {
            atomicOr(&segs[sg].overflow, 1u);
            continue;
        }
        const uint32_t me = (uint32_t)(wi & imask);
        uint64_t k[3];
        key_of(S.kind, S.copy + (size_t)me * vs, S.ts_off, k);
        uint32_t rank = 0;
        for (uint32_t j = lo; j < hi; j++) {
            if (j == i) continue;
            const uint32_t other = (uint32_t)(wv[j] & imask);
            uint64_t q[3];
            key_of(S.kind, S.copy + (size_t)other * vs, S.ts_off, q);
            rank += key_before(q, other, k, me) ? 1u : 0u;
        }
        const uint32_t to = lo + rank;
        copy_any(S.values + (size_t)to * vs, S.copy + (size_t)me * vs, vs);
    }
}

// A fixed-up table whose top bits left a run too long to fix up (rare: keys
// clustered in their top bits): one workgroup sorts it again, all its
// varying bytes, LSD from the put-order copy, stable (ranks by wave match
// ballots within 256-item chunks in order), then writes every value. Slow
// but correct; the common case never launches work here. Packed keys of up
// to three limbs (`keys`, N words per limb) and indices (`idx`) are its own.
__device__ __forceinline__ void pack_bytes(const uint8_t *map, uint32_t nb, const uint64_t k[3], uint64_t pk[3]) {
    pk[0] = pk[1] = pk[2] = 0;
    for (uint32_t j = 0; j < nb; j++) {
        const uint32_t src = map[j];
        pk[j >> 3] |= ((k[src >> 3] >> (8 * (src & 7))) & 255ull) << (8 * (j & 7));
    }
}

__global__ __launch_bounds__(256) void k_sort_rescue(SortSeg *segs, const SortBatch *batch, uint32_t N,
                                                     uint64_t *keys0, uint64_t *keys1, uint32_t *idx0, uint32_t *idx1) {
    __shared__ uint8_t s_map[kMaxBytes];
    __shared__ uint32_t s_off[kRadix];
    __shared__ uint32_t s_wc[4][kRadix];
    __shared__ uint32_t s_wsum[4];
    const SortSeg S = segs[blockIdx.x];
    // A pass that hit a wait bound (SortBatch.broken) may have left any moved
    // table's words incomplete: every such table is sorted again from its
    // put-order copy, so a broken invariant costs time, never order.
    const bool broken = *(volatile const uint32_t *)&batch->broken != 0 && S.nact;
    if (!S.overflow && !broken) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid < kMaxBytes) s_map[tid] = segs[blockIdx.x].byte_src[tid];
    __syncthreads();
    const uint32_t nb = S.nbytes, pl = (nb + 7) >> 3, base = S.item_base;
    for (uint32_t i = tid; i < S.n; i += 256) {
        uint64_t k[3], pk[3];
        key_of(S.kind, S.copy + (size_t)i * S.vs, S.ts_off, k);
        pack_bytes(s_map, nb, k, pk);
        for (uint32_t l = 0; l < pl; l++) keys0[(size_t)l * N + base + i] = pk[l];
        idx0[base + i] = i;
    }
    __syncthreads();
    uint64_t *ks = keys0, *kd = keys1;
    uint32_t *is = idx0, *id = idx1;
    const uint64_t lt = (1ull << lane) - 1;
    for (uint32_t p = 0; p < nb; p++) {
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
// only unique there. `words` (two buffers of N) are the passes'; the rescue
// keys (two buffers of N per key limb) and indices are k_sort_rescue's.
struct SortScratch {
    uint64_t segs, tile_seg, tile_order, hist, counters, batch, bins, words, keys, idx, copies, total;
};

static SortScratch scratch_layout(const SortItem *items, uint32_t count) {
    uint64_t N = 0, tiles = 0, vals = 0, nseg = 0, kl = 1;
    for (uint32_t j = 0; j < count; j++) {
        if (items[j].n < 2) continue;
        N += items[j].n;
        tiles += tiles_of(items[j].n);
        if (!items[j].out) vals += align256((uint64_t)items[j].n * items[j].value_size);
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
    s.words = o;
    o += 2 * align256(8 * N);
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
    if (scratch_bytes < L.total || status_words < sort_status_words(items, count)) return -2;
    hipStream_t s = (hipStream_t)stream;
    uint8_t *base = (uint8_t *)scratch, *hbase = (uint8_t *)host;
    SortSeg *hsegs = (SortSeg *)(hbase + L.segs);
    uint32_t *htile = (uint32_t *)(hbase + L.tile_seg);
    uint32_t N = 0, nseg = 0, ntiles = 0;
    uint32_t max_kl = 0, max_pass = 0;
    uint64_t copy_off = L.copies;
    for (uint32_t j = 0; j < count; j++) {
        const SortItem &it = items[j];
        if (it.n < 2) {
            if (it.n == 1 && it.out && hipMemcpyAsync(it.out, it.values, it.value_size, hipMemcpyDeviceToDevice, s) != hipSuccess)
                return -3;
            continue;
        }
        SortSeg g{};
        for (uint32_t l = 0; l < kMaxLimbs; l++) g.key_and[l] = ~0ull;
        g.src = (const uint8_t *)it.values;
        if (it.out) { // out of place: the input is the gather's source, no copy
            g.values = (uint8_t *)it.out;
            g.copy = (uint8_t *)it.values;
            g.oop = 1;
        } else {
            g.values = (uint8_t *)it.values;
            g.copy = base + copy_off;
            copy_off += align256((uint64_t)it.n * it.value_size);
        }
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
        // The most passes the table's words can need: its key bits, at most
        // 64 minus the index bits, in 8-bit digits.
        const uint32_t ib = 32 - __builtin_clz(it.n - 1);
        const uint32_t kb = 64 * g.kl < 64 - ib ? 64 * g.kl : 64 - ib;
        max_pass = max_pass > (kb + 7) / 8 ? max_pass : (kb + 7) / 8;
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
    uint64_t *words0 = (uint64_t *)(base + L.words), *words1 = (uint64_t *)(base + L.words + align256(8ull * N));
    const uint64_t klw = align256(8ull * N * max_kl);
    uint64_t *keys0 = (uint64_t *)(base + L.keys), *keys1 = (uint64_t *)(base + L.keys + klw);
    uint32_t *idx0 = (uint32_t *)(base + L.idx), *idx1 = (uint32_t *)(base + L.idx + align256(4ull * N));
    uint32_t *hist = (uint32_t *)(base + L.hist), *bins = (uint32_t *)(base + L.bins);
    uint32_t *counters = (uint32_t *)(base + L.counters);
    SortBatch *d_batch = (SortBatch *)(base + L.batch);
    // Descriptors up and the histograms, counters and batch words zeroed, one launch.
    if (launch_upload(base, hbase, L.hist, s, hist, L.bins - L.hist) != 0) return -4;
    hipLaunchKernelGGL(k_sort_extract, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile);
    hipLaunchKernelGGL(k_sort_layout, dim3(nseg), dim3(64), 0, s, d_segs);
    hipLaunchKernelGGL(k_sort_pack, dim3(ntiles), dim3(kSortThreads), 0, s, d_segs, d_tile, words0, hist);
    hipLaunchKernelGGL(k_sort_plan, dim3(nseg), dim3(kRadix), 0, s, d_segs, d_batch, hist, bins);
    // Persistent: as many workgroups as are resident at once: more would
    // only start after the tiles run out, and an idle pass (no table has
    // that many digits) costs its launch alone.
    static uint32_t resident = 0;
    if (!resident) {
        int per_cu = 0, dev = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_sort_pass, kSortThreads, 0) != hipSuccess ||
            hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || per_cu < 1)
            return -5;
        resident = (uint32_t)(per_cu * cus);
    }
    const uint32_t pgrid = ntiles < resident ? ntiles : resident;
    const uint32_t passes = max_pass < kMaxPasses ? max_pass : kMaxPasses;
    // Tickets only when some workgroup takes more than one tile (TBC_SORT_TICKETS=1: always, A/B).
    static const bool ordered = getenv("TBC_SORT_TICKETS") == nullptr;
    for (uint32_t p = 0; p < passes && p < kDirectPasses; p++) {
        if (*epoch == 0) *epoch = 1; // 0 is the zeroed buffer's
        hipLaunchKernelGGL(k_sort_pass, dim3(pgrid), dim3(kSortThreads), 0, s, d_segs, d_batch, d_tile, d_order, p,
                           ntiles, words0, words1, bins, status, (*epoch)++,
                           ordered && pgrid == ntiles ? nullptr : counters);
    }
    if (passes > kDirectPasses) {
        if (*epoch == 0 || *epoch + kMaxPasses < *epoch) *epoch = 1; // a fresh epoch per pass, none 0
        hipLaunchKernelGGL(k_sort_pass_rest, dim3(pgrid), dim3(kSortThreads), 0, s, d_segs, d_batch, d_tile, d_order,
                           ntiles, words0, words1, bins, status, *epoch, counters, counters + kMaxPasses);
        *epoch += kMaxPasses;
    }
    hipLaunchKernelGGL(k_sort_finish, dim3(ntiles * (kSortTile / kFinishItems)), dim3(256), 0, s, d_segs,
                       (const uint32_t *)d_tile, (const uint64_t *)words0, (const uint64_t *)words1);
    hipLaunchKernelGGL(k_sort_rescue, dim3(nseg), dim3(256), 0, s, d_segs, (const SortBatch *)d_batch, N, keys0,
                       keys1, idx0, idx1);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

} // namespace tbc
