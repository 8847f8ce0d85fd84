// merge.hip — the 2-way newest-wins merge of one compaction, data-parallel.
//
// The reference (src/lsm/compaction.zig:483-559, 647-804) walks A (the
// immutable table memory, deduplicated by fill_immutable_values, or a disk
// table) and B (the overlapping level-B tables, concatenated) with one CPU
// loop. Its result depends only on the merged order, so it is restated as a
// pure function of each element and its merge-order neighbours:
//
//   merged order: A before B on equal keys (A-first tie break);
//   A[i] survives dedup   iff it is the last of its run of equal keys and
//                          (general, or the run length is odd: pairs cancel
//                          from the left, compaction.zig:508-523);
//   A[i] is written       iff it survives dedup and not (drop_tombstones and
//                          tombstone) and not (secondary_index and B has the
//                          key) (compaction.zig:764-796, 724-736);
//   B[j] is written       iff A has no dedup survivor with the same key
//                          (B tombstones are never dropped, :775-779).
//
// Kernels: merge-path split per tile boundary -> per tile: survivor and side
// bit masks plus the survivor count (tiles independent) -> per job: scan of
// the counts into tile output offsets and the output shape. k_data_blocks
// then assembles each output block from the masks (producer waves) while its
// AEGIS chain checksums it (aegis.hip).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>

#include "tbc_internal.h"
#include "keys.h"

namespace tbc {

__device__ __forceinline__ uint32_t load_tomb(const uint8_t *v, uint32_t ts_off) {
    return (uint32_t)(ld64(v + ts_off) >> 63);
}

// Segment containing element idx: the largest s with seg_pre[s] <= idx.
__device__ __forceinline__ uint32_t seg_search(const Stream &s, uint32_t idx) {
    if (s.uniform) {
        const uint32_t q = idx / s.uniform;
        return q < s.nseg ? q : s.nseg - 1;
    }
    uint32_t lo = 0, hi = s.nseg - 1;
    while (lo < hi) {
        uint32_t mid = (lo + hi + 1) >> 1;
        if (gld<uint32_t>(s.seg_pre + mid) <= idx) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ const uint8_t *elem_ptr(const Stream &s, uint32_t seg, uint32_t idx, uint32_t vs) {
    return (const uint8_t *)gld<uint64_t>(s.seg_ptr + seg) + (size_t)(idx - gld<uint32_t>(s.seg_pre + seg)) * vs;
}

// --------------------------------------------------------------------------
// Merge-path partition: for every tile boundary d = t * merge_tile, the number
// i of A elements among the first d merged elements, plus the segments that
// hold A[max(i-1, 0)] and B[min(d-i, nb-1)] (where the tile starts reading).
// --------------------------------------------------------------------------
// All key kinds of a batch in ONE launch (the split's job picks the key
// loader): a batch mixing trees paid one latency-bound launch per kind.
// One thread per split: a binary search (~21 dependent probes).
template <int KIND>
__device__ __forceinline__ uint32_t merge_path_split(const JobDesc &j, uint32_t d) {
    const uint32_t na = j.a.n, nb = j.b.n;
    uint32_t lo = d > nb ? d - nb : 0;
    uint32_t hi = d < na ? d : na;
    const uint32_t vs = j.value_size, ts = j.timestamp_offset;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t ib = d - 1 - mid;
        const uint8_t *pa = elem_ptr(j.a, seg_search(j.a, mid), mid, vs);
        const uint8_t *pb = elem_ptr(j.b, seg_search(j.b, ib), ib, vs);
        if (key_le(load_key<KIND>(pa, ts), load_key<KIND>(pb, ts))) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// One wave per split: a 64-ary merge-path search (each round, the 64 lanes
// probe 64 evenly spaced candidates and a ballot keeps the interval between
// the last true and the first false), 4 dependent rounds for 2^24 values
// instead of ~24 single-lane probes.
template <int KIND>
__device__ __forceinline__ uint32_t merge_path_split_wave(const JobDesc &j, uint32_t d) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t nb = j.b.n, vs = j.value_size, ts = j.timestamp_offset;
    uint32_t lo = d > nb ? d - nb : 0, hi = d < j.a.n ? d : j.a.n; // answer in [lo, hi]
    while (lo < hi) {
        const uint32_t span = hi - lo;
        // candidate i: "A[i] sorts before B[d - 1 - i]" holds for i < answer
        const uint32_t i = span <= 64 ? lo + lane : lo + (uint32_t)(((uint64_t)span * lane) >> 6);
        bool pred = false;
        if (i < hi) {
            const uint8_t *pa = elem_ptr(j.a, seg_search(j.a, i), i, vs);
            const uint8_t *pb = elem_ptr(j.b, seg_search(j.b, d - 1 - i), d - 1 - i, vs);
            pred = key_le(load_key<KIND>(pa, ts), load_key<KIND>(pb, ts));
        }
        const uint64_t t = __ballot(pred && i < hi);
        const uint32_t c = __builtin_popcountll(t); // predicates hold on a prefix of the lanes
        if (span <= 64) return lo + c;
        const uint32_t last_true = c ? lo + (uint32_t)(((uint64_t)span * (c - 1)) >> 6) : lo;
        const uint32_t first_false = c < 64 ? lo + (uint32_t)(((uint64_t)span * c) >> 6) : hi;
        lo = c ? last_true + 1 : lo;
        hi = first_false;
    }
    return lo;
}

// A batch with few splits (config 1's half-bars: a few thousand) searches
// one split per wave, 4 dependent rounds instead of ~21 (k_partition_all
// ~50 -> ~36 us per batch); with many splits (configs 2-5: tens of
// thousands) the 64 probes per round cost more bandwidth than the rounds
// save (config 2's k_partition_unique 49 -> 135 us), so one thread per split.
// The mask merges' partitions switch at 12,288 splits (config 1's
// partitions 2.45 -> 2.16 ms per step; at 32,768 config 5's grew 192 -> 500
// us), the unique merges' at 4,096.
constexpr uint32_t kWaveSplitsMax = 4096;
constexpr uint32_t kWaveSplitsMaxMask = 12288;
static uint32_t wave_splits_max() { return kWaveSplitsMaxMask; }

template <int KIND, bool Wave>
__device__ __forceinline__ uint32_t split_at(const JobDesc &j, uint32_t d) {
    if constexpr (Wave) return merge_path_split_wave<KIND>(j, d);
    else return merge_path_split<KIND>(j, d);
}

template <bool Wave>
__device__ __forceinline__ uint32_t split_index() {
    return Wave ? blockIdx.x * 4 + (threadIdx.x >> 6) : blockIdx.x * 256 + threadIdx.x;
}

template <bool Wave>
__global__ __launch_bounds__(256) void k_partition_all(const JobDesc *jobs, int njobs, uint32_t nsplits,
                                                       SplitDesc *splits, const JobResultDev *res, uint32_t phase) {
    const uint32_t gsplit = split_index<Wave>();
    if (gsplit >= nsplits) return; // wave-uniform
    const int ji = find_job(jobs, njobs, gsplit, [](const JobDesc &d) { return d.split_base; });
    const JobDesc &j = jobs[ji];
    if (phase_skips(j, res, phase)) return;
    const uint32_t t = gsplit - j.split_base;
    const uint32_t na = j.a.n, nb = j.b.n, n = na + nb;
    const uint32_t d = (uint64_t)t * j.merge_tile < n ? t * j.merge_tile : n;
    uint32_t lo;
    switch (j.key_kind) {
    case kKeyTimestamp: lo = split_at<kKeyTimestamp, Wave>(j, d); break;
    case kKeyIdU128: lo = split_at<kKeyIdU128, Wave>(j, d); break;
    case kKeyCompositeU64: lo = split_at<kKeyCompositeU64, Wave>(j, d); break;
    default: lo = split_at<kKeyCompositeU128, Wave>(j, d); break;
    }
    // The segments the tile starting here reads, resolved for k_merge_tile:
    // two value pointers and three prefix counts per side, their loads
    // issued together (clamped into the tables, then masked).
    auto fill = [](const Stream &st, uint32_t seg, uint64_t *ptr, uint32_t *pre) {
        const uint32_t ns = st.nseg;
        if (!ns) {
            ptr[0] = ptr[1] = 0;
            pre[0] = pre[1] = pre[2] = 0xffffffffu;
            return;
        }
        uint64_t p[2];
        uint32_t q[3];
        for (uint32_t k = 0; k < 2; k++) p[k] = gld<uint64_t>(st.seg_ptr + (seg + k < ns ? seg + k : ns - 1));
        for (uint32_t k = 0; k < 3; k++) q[k] = gld<uint32_t>(st.seg_pre + (seg + k <= ns ? seg + k : ns));
        for (uint32_t k = 0; k < 2; k++) ptr[k] = seg + k < ns ? p[k] : 0;
        for (uint32_t k = 0; k < 3; k++) pre[k] = seg + k <= ns ? q[k] : 0xffffffffu;
    };
    const uint32_t jb = d - lo;
    if constexpr (Wave) { // lane 0 resolves side A, lane 1 side B, at once
        const uint32_t lane = threadIdx.x & 63;
        if (lane > 1) return;
        const bool bside = lane == 1;
        const Stream &st = bside ? j.b : j.a;
        const uint32_t cnt = bside ? nb : na, idx = bside ? (jb < nb ? jb : nb - 1) : (lo > 0 ? lo - 1 : 0);
        const uint32_t seg = cnt ? seg_search(st, idx) : 0;
        uint64_t ptr[2];
        uint32_t pre[3];
        fill(st, seg, ptr, pre);
        SplitSeg &g = j.split_segs[t];
        for (uint32_t k = 0; k < 2; k++) (bside ? g.b_ptr : g.a_ptr)[k] = ptr[k];
        for (uint32_t k = 0; k < 3; k++) (bside ? g.b_pre : g.a_pre)[k] = pre[k];
        const uint32_t seg_b = (uint32_t)__shfl((int)seg, 1, 64);
        if (!bside) splits[gsplit] = SplitDesc{lo, seg, seg_b, 0};
        return;
    }
    SplitDesc s;
    s.i = lo;
    s.seg_a = na ? seg_search(j.a, lo > 0 ? lo - 1 : 0) : 0;
    s.seg_b = nb ? seg_search(j.b, jb < nb ? jb : nb - 1) : 0;
    s.pad = 0;
    splits[gsplit] = s;
    SplitSeg g;
    fill(j.a, s.seg_a, g.a_ptr, g.a_pre);
    fill(j.b, s.seg_b, g.b_ptr, g.b_pre);
    j.split_segs[t] = g;
}

// Speculated jobs (TBC_COMPACTION_UNIQUE_KEYS): with every value surviving,
// data block k holds merged positions [k * vcm, (k + 1) * vcm); its producer
// starts from the merge-path split at k * vcm. The thread of block 0 also
// writes the job's speculative results (write_blocks' shape for n values,
// compaction.zig:806-850); a broken speculation has them rewritten by the
// recomputation's k_tile_scan.
__global__ __launch_bounds__(256) void k_partition_blocks(const JobDesc *jobs, int njobs, uint32_t total,
                                                          SplitDesc *bsplits, JobResultDev *res) {
    const uint32_t m = blockIdx.x * 4 + (threadIdx.x >> 6);
    if (m >= total) return;
    const int ji = find_job(jobs, njobs, m, [](const JobDesc &d) { return d.dblock_base; });
    const JobDesc &j = jobs[ji];
    const uint32_t k = m - j.dblock_base;
    if (!j.unique || k >= j.dblock_max) return;
    const uint32_t na = j.a.n, nb = j.b.n;
    const uint32_t d = k * j.vcm;
    uint32_t lo;
    switch (j.key_kind) {
    case kKeyTimestamp: lo = merge_path_split_wave<kKeyTimestamp>(j, d); break;
    case kKeyIdU128: lo = merge_path_split_wave<kKeyIdU128>(j, d); break;
    case kKeyCompositeU64: lo = merge_path_split_wave<kKeyCompositeU64>(j, d); break;
    default: lo = merge_path_split_wave<kKeyCompositeU128>(j, d); break;
    }
    if ((threadIdx.x & 63) != 0) return;
    SplitDesc s;
    s.i = lo;
    s.seg_a = na ? seg_search(j.a, lo > 0 ? lo - 1 : 0) : 0;
    const uint32_t jb = d - lo;
    s.seg_b = nb ? seg_search(j.b, jb < nb ? jb : nb - 1) : 0;
    // Segment of B[jb - 1] (the value before the block on the B side).
    s.pad = nb && jb > 0 ? seg_search(j.b, jb - 1 < nb ? jb - 1 : nb - 1) : 0;
    bsplits[m] = s;
    if (k == 0) {
        JobResultDev &r = res[j.job_index];
        const uint64_t n = (uint64_t)na + nb;
        r.value_count = n;
        r.data_block_count = j.dblock_max;
        r.table_count = j.table_max;
        r.block_count = j.dblock_max + j.table_max;
        r.spec = kSpecHeld;
    }
}

int launch_partition_blocks(const JobDesc *d_jobs, int njobs, uint32_t total_dblocks, SplitDesc *d_bsplits,
                            JobResultDev *d_results, void *stream) {
    if (!total_dblocks) return 0;
    hipLaunchKernelGGL(k_partition_blocks, dim3((total_dblocks + 3) / 4), dim3(256), 0, (hipStream_t)stream,
                       d_jobs, njobs, total_dblocks, d_bsplits, d_results);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// --------------------------------------------------------------------------
// Pipelined speculated batches (engine.hip submit_impl, round 4): a
// TBC_COMPACTION_UNIQUE_KEYS job's bodies merged tile by tile on the engine
// stream, HBM-bound, while earlier batches' AEGIS chains run on tail streams.
// If no key repeats and no tombstone is dropped, every value survives
// (compaction.zig:483-559 dedup and :757-798 merge keep it), so merged
// position g lands at data block g / vcm, slot g % vcm: A[i] at
// (i - ia0) + |{B in the tile < A[i]}|, B[j] at (j - jb0) + |{A in the tile
// <= B[j]}| (A first on equal keys). The speculation holds iff no output key
// equals its merged predecessor's: an A key equal to its lower bound in B
// (the tile's B range, or the first B after it), an A key equal to the A
// before it, a B key equal to the B before it; and no A tombstone when
// tombstones are dropped. A broken job is marked (JobResultDev.spec) and
// recomputed through the merge path by the batch's phase 1.
// --------------------------------------------------------------------------
// UniqueSplit.below / .above of the boundary after A[0, i) and B[0, jb).
template <int KIND>
__device__ __forceinline__ void split_bounds(const JobDesc &j, uint32_t i, uint32_t jb, UniqueSplit &s) {
    constexpr int KL = KeyLimbs<KIND>::value;
    const uint32_t vs = j.value_size, ts = j.timestamp_offset;
    auto key_at = [&](const Stream &st, uint32_t idx) {
        return load_key<KIND>(elem_ptr(st, seg_search(st, idx), idx, vs), ts);
    };
    Key<KL> lo, hi;
    bool have_lo = false, have_hi = false;
    if (i > 0) {
        lo = key_at(j.a, i - 1);
        have_lo = true;
    }
    if (jb > 0) {
        const Key<KL> k = key_at(j.b, jb - 1);
        if (!have_lo || key_lt(k, lo)) lo = k;
        have_lo = true;
    }
    if (i < j.a.n) {
        hi = key_at(j.a, i);
        have_hi = true;
    }
    if (jb < j.b.n) {
        const Key<KL> k = key_at(j.b, jb);
        if (!have_hi || key_lt(hi, k)) hi = k;
        have_hi = true;
    }
#pragma unroll
    for (int l = 0; l < 3; l++) {
        s.below[l] = l < KL && have_lo ? lo.l[l] : 0ull;
        s.above[l] = l < KL ? (have_hi ? hi.l[l] : ~0ull) : 0ull;
    }
}

template <bool Wave>
__global__ __launch_bounds__(256) void k_partition_unique(const JobDesc *jobs, int njobs, uint32_t nsplits,
                                                          UniqueSplit *usplits, JobResultDev *res) {
    const uint32_t g = split_index<Wave>();
    if (g >= nsplits) return;
    const int ji = find_job(jobs, njobs, g, [](const JobDesc &d) { return d.usplit_base; });
    const JobDesc &j = jobs[ji];
    if (!j.unique || g - j.usplit_base > j.utile_count) return;
    const uint32_t t = g - j.usplit_base;
    const uint32_t na = j.a.n, nb = j.b.n, n = na + nb;
    const uint32_t d = (uint64_t)t * kUniqueTile < n ? t * kUniqueTile : n;
    uint32_t lo;
    switch (j.key_kind) {
    case kKeyTimestamp: lo = split_at<kKeyTimestamp, Wave>(j, d); break;
    case kKeyIdU128: lo = split_at<kKeyIdU128, Wave>(j, d); break;
    case kKeyCompositeU64: lo = split_at<kKeyCompositeU64, Wave>(j, d); break;
    default: lo = split_at<kKeyCompositeU128, Wave>(j, d); break;
    }
    if (Wave && (threadIdx.x & 63) != 0) return;
    UniqueSplit s;
    s.i = lo;
    s.pad = 0;
    const uint32_t jb = d - lo;
    s.seg_a = na ? seg_search(j.a, lo > 0 ? lo - 1 : 0) : 0;
    s.seg_b = nb ? seg_search(j.b, jb > 0 ? jb - 1 : 0) : 0;
    s.a_ptr = na ? gld<uint64_t>(j.a.seg_ptr + s.seg_a) : 0;
    s.a_lo = na ? gld<uint32_t>(j.a.seg_pre + s.seg_a) : 0;
    s.a_hi = na ? gld<uint32_t>(j.a.seg_pre + s.seg_a + 1) : 0;
    s.b_ptr = nb ? gld<uint64_t>(j.b.seg_ptr + s.seg_b) : 0;
    s.b_lo = nb ? gld<uint32_t>(j.b.seg_pre + s.seg_b) : 0;
    s.b_hi = nb ? gld<uint32_t>(j.b.seg_pre + s.seg_b + 1) : 0;
    switch (j.key_kind) {
    case kKeyTimestamp: split_bounds<kKeyTimestamp>(j, lo, jb, s); break;
    case kKeyIdU128: split_bounds<kKeyIdU128>(j, lo, jb, s); break;
    case kKeyCompositeU64: split_bounds<kKeyCompositeU64>(j, lo, jb, s); break;
    default: split_bounds<kKeyCompositeU128>(j, lo, jb, s); break;
    }
    usplits[g] = s;
    if (t == 0) { // speculative results (write_blocks' shape for n values, compaction.zig:806-850)
        JobResultDev &r = res[j.job_index];
        r.value_count = n;
        r.data_block_count = j.dblock_max;
        r.table_count = j.table_max;
        r.block_count = j.dblock_max + j.table_max;
        r.spec = kSpecHeld;
    }
}

// LDS of a k_merge_unique workgroup: the tile's broken flag, then a 32-bit
// window of every entry's key (entries [0, na + 1) = A[ia0 - 1 .. ia1),
// [na + 1, na + nb + 3) = B[jb0 - 1 .. jb1]): the key's 32 bits right below
// the leading bits every key of the tile shares (UniqueSplit.below/.above),
// so keys compare by their windows and, when those are equal, in full from
// the values (global, L2-hot: the tile has just read them). 8.2 KiB for
// 2,048 positions whatever the key width (round 5 kept the top 64 bits:
// 16.4 KiB), so TWO workgroups fit beside an AEGIS chain workgroup's 136 KiB
// of a CU's 160.
constexpr uint32_t kUniqueRow = kUniqueTile + 3;
static inline uint32_t unique_lds_bytes() { return 16 + kUniqueRow * 4; }

// Leading bits common to the keys `lo` <= `hi` (most significant limb last).
template <int KL> __device__ __forceinline__ uint32_t common_prefix(const uint64_t *lo, const uint64_t *hi) {
    uint32_t p = 0;
#pragma unroll
    for (int l = KL - 1; l >= 0; l--) {
        const uint64_t x = lo[l] ^ hi[l];
        if (x) return p + (uint32_t)__builtin_clzll(x);
        p += 64;
    }
    return p;
}

// Bits [p, p + 32) of the key counted from its most significant bit (zeros
// past its least significant one). For keys sharing their first p bits the
// windows order as the keys do, up to ties.
template <int KL> __device__ __forceinline__ uint32_t key_window(const Key<KL> &k, uint32_t p) {
    const uint32_t t = p >> 6, sh = p & 63;
    uint64_t top = 0;
#pragma unroll
    for (int l = 0; l < KL; l++) {
        if ((uint32_t)(KL - 1 - l) == t) top |= k.l[l] << sh;
        if (sh && (uint32_t)(KL - 2 - l) == t) top |= k.l[l] >> (64 - sh);
    }
    return (uint32_t)(top >> 32);
}

// Element idx of a stream whose split resolved segment [lo, hi) at ptr: in
// that segment, or (a tile crossing an input block boundary) found by walking
// the segment table forward from it.
__device__ __forceinline__ const uint8_t *unique_elem(const Stream &st, uint32_t seg, uint64_t ptr, uint32_t lo,
                                                      uint32_t hi, uint32_t idx, uint32_t vs) {
    if (idx < hi || seg + 1 >= st.nseg) return (const uint8_t *)(uintptr_t)ptr + (size_t)(idx - lo) * vs;
    SegCursor c;
    c.init(st, seg + 1);
    return c.elem(idx, vs);
}

// Byte offset of key limb l in a value (keys.h load_key's order).
template <int KIND> __device__ __forceinline__ uint32_t key_limb_off(int l, uint32_t ts) {
    if constexpr (KIND == kKeyTimestamp) return ts;
    else if constexpr (KIND == kKeyIdU128) return 8u * l;
    else if constexpr (KIND == kKeyCompositeU64) return l == 0 ? 8u : 0u;
    else return l == 0 ? 16u : 8u * (l - 1);
}

// The 8-byte word at byte `off` (< 32, a multiple of 8) of a value whose first
// 32 bytes are v0, v1.
__device__ __forceinline__ uint64_t word_of(const u32x4 &v0, const u32x4 &v1, uint32_t off) {
    const u32x4 &v = off < 16 ? v0 : v1;
    return (off & 8) ? ((uint64_t)v.w << 32 | v.z) : ((uint64_t)v.y << 32 | v.x);
}

// One tile, kUniqueTile / kUniqueThreads merged elements per thread (tile
// order: its A elements, then its B elements; thread i owns elements i, i +
// 512, ...). Each value's first 32 bytes and key are loaded together before
// the barrier, so their HBM latency overlaps the ranking; pointers come from
// the split's resolved segments (a tile spans one or two input blocks).
// Wide (values over 32 bytes: the object trees): no value bytes held across
// the barrier (keys read apart); each stored value's chunks are loaded
// together, one element at a time. A launch of its own, so the narrow
// kernel keeps its registers.
template <int KIND, bool Wide>
__device__ __forceinline__ void merge_unique_tile(uint8_t *lds, const JobDesc &j, uint32_t t,
                                                  const UniqueSplit *usplits, JobResultDev *res) {
    constexpr int KL = KeyLimbs<KIND>::value;
    constexpr uint32_t T = kUniqueTile, NT = kUniqueThreads, E = T / NT;
    static_assert(T == E * NT, "whole elements per thread");
    uint32_t &s_bad = *(uint32_t *)lds;
    uint32_t *s_win = (uint32_t *)(lds + 16);
    const uint32_t tid = threadIdx.x;
    const uint32_t na_all = j.a.n, nb_all = j.b.n, n = na_all + nb_all;
    const uint32_t d0 = t * T, d1 = d0 + T < n ? d0 + T : n;
    const UniqueSplit s0 = usplits[j.usplit_base + t];
    const uint32_t ia0 = s0.i, ia1 = usplits[j.usplit_base + t + 1].i;
    const uint32_t jb0 = d0 - ia0, jb1 = d1 - ia1;
    const uint32_t na = ia1 - ia0, nb = jb1 - jb0, m = na + nb;
    const uint32_t vs = j.value_size, ts = j.timestamp_offset;
    const bool drop = j.drop_tombstones != 0;
    const uint32_t eb = na + 1; // entry of B[jb0 - 1]
    constexpr uint32_t kMaxOff = KIND == kKeyTimestamp ? 0u : (KIND == kKeyCompositeU128 ? 16u : 8u);
    const uint32_t reg_bytes = vs < 32 ? vs : 32u;
    const bool in_regs = !Wide && (KIND == kKeyTimestamp ? ts : (kMaxOff > ts ? kMaxOff : ts)) + 8 <= reg_bytes;
    if (tid == 0) s_bad = 0;
    // The job's fields the stores below need, read once: the output stores
    // could alias the descriptor, so every use after one re-read it.
    const Stream sa = j.a, sb = j.b;
    const uint32_t dbcm = j.dbcm, bsize = j.block_size;
    uint8_t *const grid_base = j.grid_base, *const out_blocks = j.out_blocks;
    const uint64_t *const addresses = j.addresses;
    auto elem_a = [&](uint32_t i) { return unique_elem(sa, s0.seg_a, s0.a_ptr, s0.a_lo, s0.a_hi, i, vs); };
    auto elem_b = [&](uint32_t i) { return unique_elem(sb, s0.seg_b, s0.b_ptr, s0.b_lo, s0.b_hi, i, vs); };
    // Entry e's full key (A entries 0..na, B entries eb..eb+nb+1), from the input.
    auto full_key = [&](uint32_t e) {
        const uint8_t *p = e < eb ? elem_a(ia0 - 1 + e) : elem_b(jb0 - 1 + (e - eb));
        return load_key<KIND>(p, ts);
    };
    // This thread's elements: their values' first 32 bytes into registers
    // (their keys are taken from there when they lie in them).
    const uint8_t *src[E];
    u32x4 v0[E], v1[E];
    Key<KL> kw[Wide ? E : 1]; // Wide: every element's key, loaded together below
    auto key_of = [&](uint32_t q) {
        Key<KL> k;
        if constexpr (Wide) {
            k = kw[q];
        } else if (in_regs) {
#pragma unroll
            for (int l = 0; l < KL; l++) {
                k.l[l] = word_of(v0[q], v1[q], key_limb_off<KIND>(l, ts));
                if (l == 0 && KIND != kKeyIdU128) k.l[l] &= ~kTombstoneBit;
            }
        } else {
            k = load_key<KIND>(src[q], ts);
        }
        return k;
    };
    // Every element's pointer first (a tile crossing an input block walks
    // the segment table), then every value load: a load whose address waits
    // on a pointer load waited on all loads before it too, so loads issued
    // element by element went out one round trip at a time.
#pragma unroll
    for (uint32_t q = 0; q < E; q++) {
        const uint32_t e = tid + q * NT;
        const bool is_a = e < na;
        src[q] = e < m ? (is_a ? elem_a(ia0 + e) : elem_b(jb0 + (e - na))) : nullptr;
    }
#pragma unroll
    for (uint32_t q = 0; q < E; q++) {
        v0[q] = v1[q] = u32x4{0, 0, 0, 0};
        if (!Wide && src[q]) {
            v0[q] = gld<u32x4>(src[q]);
            if (vs >= 32) v1[q] = gld<u32x4>(src[q] + 16);
        }
    }
    if constexpr (Wide) { // keys loaded together (each read next to its use waited for it alone)
        const uint8_t *fb = src[0] ? src[0] : (const uint8_t *)(uintptr_t)(s0.a_ptr ? s0.a_ptr : s0.b_ptr);
#pragma unroll
        for (uint32_t q = 0; q < E; q++) kw[q] = load_key<KIND>(src[q] ? src[q] : fb, ts);
    }
    // The leading bits every key the tile compares shares (uniform: from
    // the tile's two boundaries, scalar loads).
    const uint32_t pre = common_prefix<KL>(s0.below, usplits[j.usplit_base + t + 1].above);
    uint32_t win[E];
#pragma unroll
    for (uint32_t q = 0; q < E; q++) {
        const uint32_t e = tid + q * NT;
        win[q] = e < m ? key_window(key_of(q), pre) : 0u;
        if (e < m) s_win[e < na ? 1 + e : e + 2] = win[q];
    }
    // The boundary entries: A[ia0 - 1], B[jb0 - 1], B[jb1] (absent: never compared).
    if (tid < 3) {
        const bool bside = tid != 0;
        const Stream &st = bside ? sb : sa;
        const int64_t bi = tid == 0 ? (int64_t)ia0 - 1 : tid == 1 ? (int64_t)jb0 - 1 : (int64_t)jb1;
        const uint32_t e = tid == 0 ? 0u : tid == 1 ? eb : eb + nb + 1;
        uint32_t w = ~0u;
        if (bi >= 0 && bi < (int64_t)st.n)
            w = key_window(load_key<KIND>(bside ? elem_b((uint32_t)bi) : elem_a((uint32_t)bi), ts), pre);
        s_win[e] = w;
    }
    __syncthreads();
    // Order of entry e against key k (window wk): -1 below, 0 equal, 1
    // above; by the windows, and (rarely) in full when they are equal.
    auto cmp = [&](uint32_t e, const Key<KL> &k, uint32_t wk) -> int {
        const uint32_t h = s_win[e];
        if (h != wk) return h < wk ? -1 : 1;
        const Key<KL> f = full_key(e);
        return key_lt(f, k) ? -1 : (key_eq(f, k) ? 0 : 1);
    };
    bool bad = false;
    const uint32_t vcm = j.vcm;
#pragma unroll
    for (uint32_t q = 0; q < E; q++) {
        const uint32_t e = tid + q * NT;
        if (e >= m) continue;
        const Key<KL> k = key_of(q);
        const uint32_t wk = win[q];
        uint32_t pos;
        if (e < na) {
            // |{B in the tile < k}|: lower bound over entries [eb + 1, eb + 1 + nb).
            uint32_t lo = 0, hi = nb;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (cmp(eb + 1 + mid, k, wk) < 0) lo = mid + 1;
                else hi = mid;
            }
            pos = e + lo;
            // The B at the lower bound (inside the tile, or the first after it).
            const bool b_there = lo < nb || jb1 < nb_all;
            bad |= b_there && cmp(eb + 1 + lo, k, wk) == 0;
            bad |= (ia0 + e > 0) && cmp(e, k, wk) == 0;
            bad |= drop && (in_regs ? (word_of(v0[q], v1[q], ts) >> 63) != 0 : load_tomb(src[q], ts) != 0);
        } else {
            const uint32_t b = e - na;
            // |{A in the tile <= k}|: upper bound over entries [1, 1 + na).
            uint32_t lo = 0, hi = na;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (cmp(1 + mid, k, wk) <= 0) lo = mid + 1;
                else hi = mid;
            }
            pos = b + lo;
            bad |= (jb0 + b > 0) && cmp(eb + b, k, wk) == 0;
        }
        const uint32_t g = d0 + pos;
        const uint32_t kb = g / vcm, slot = data_block_slot(kb, dbcm);
        uint8_t *blk = grid_base ? grid_base + (size_t)(gld<uint64_t>(addresses + slot) - 1) * bsize
                                 : out_blocks + (size_t)slot * bsize; // block_ptr
        uint8_t *dst = blk + kHeaderSize + (size_t)(g - kb * vcm) * vs;
        if constexpr (Wide) {
            asm volatile("" ::: "memory"); // one element's chunks live at a time
            constexpr uint32_t kChunks = 8;   // 128 bytes
            u32x4 r[kChunks];
#pragma unroll
            for (uint32_t c = 0; c < kChunks; c++)
                if (16 * c < vs) r[c] = gld<u32x4>(src[q] + 16 * c);
#pragma unroll
            for (uint32_t c = 0; c < kChunks; c++)
                if (16 * c < vs) gst<u32x4>(dst + 16 * c, r[c]);
            for (uint32_t c = 16 * kChunks; c < vs; c += 16) gst<u32x4>(dst + c, gld<u32x4>(src[q] + c));
        } else {
            gst<u32x4>(dst, v0[q]);
            if (vs >= 32) gst<u32x4>(dst + 16, v1[q]);
            for (uint32_t c = 32; c < vs; c += 16) gst<u32x4>(dst + c, gld<u32x4>(src[q] + c));
        }
    }
    if (__any(bad) && (tid & 63) == 0) atomicOr(&s_bad, 1u);
    __syncthreads();
    if (tid == 0 && s_bad) {
        __hip_atomic_store(&res[j.job_index].spec, kSpecBroken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(j.spec_any, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// One tile per workgroup, the tiles [first, first + gridDim.x) of one key
// kind (a batch's jobs are grouped by kind, so each kind's tiles are
// contiguous; a launch per kind keeps each kernel's registers its own).
// Wide: the tiles of jobs whose values exceed 32 bytes (the other launch
// takes the rest). At most 80 VGPRs (6 waves per SIMD): two workgroups fit
// beside a chain workgroup (82 VGPRs, 2 waves per SIMD) on one CU.
template <int KIND, bool Wide>
__global__ __launch_bounds__(kUniqueThreads) __attribute__((amdgpu_waves_per_eu(6))) void k_merge_unique(
    const JobDesc *jobs, int njobs, uint32_t first, const UniqueSplit *usplits, JobResultDev *res) {
    extern __shared__ __attribute__((aligned(16))) uint8_t unique_lds[];
    const uint32_t g = first + blockIdx.x;
    const int ji = find_job(jobs, njobs, g, [](const JobDesc &d) { return d.utile_base; });
    const JobDesc &j = jobs[ji];
    if (!j.unique || g - j.utile_base >= j.utile_count || (j.value_size > 32) != Wide) return; // uniform
    merge_unique_tile<KIND, Wide>(unique_lds, j, g - j.utile_base, usplits, res);
}

int launch_merge_unique(const JobDesc *d_jobs, const JobDesc *h_jobs, int njobs, SplitDesc *d_usplits,
                        JobResultDev *d_results, uint32_t *d_ticket, void *stream, void (*mark)(void *, const char *),
                        void *mark_ctx, void *part_stream, void *part_done) {
    hipStream_t s = (hipStream_t)part_stream ? (hipStream_t)part_stream : (hipStream_t)stream;
    // The partition may run ahead on another stream (the batch's descriptors
    // were uploaded there): the merge, and whatever follows on `stream`, wait.
    auto join = [&]() {
        if (s == (hipStream_t)stream) return true;
        const bool ok = hipEventRecord((hipEvent_t)part_done, s) == hipSuccess &&
                        hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)part_done, 0) == hipSuccess;
        s = (hipStream_t)stream;
        return ok;
    };
    uint32_t nsplits = 0, ntiles = 0;
    if (njobs) {
        const JobDesc &l = h_jobs[njobs - 1];
        nsplits = l.usplit_base + (l.unique ? l.utile_count + 1 : 0);
        ntiles = l.utile_base + l.utile_count;
    }
    if (!nsplits || !ntiles) return join() ? 0 : -1;
    if (nsplits <= kWaveSplitsMax)
        hipLaunchKernelGGL(k_partition_unique<true>, dim3((nsplits + 3) / 4), dim3(256), 0, s, d_jobs, njobs, nsplits,
                       (UniqueSplit *)d_usplits, d_results);
    else
        hipLaunchKernelGGL(k_partition_unique<false>, dim3((nsplits + 255) / 256), dim3(256), 0, s, d_jobs, njobs, nsplits,
                       (UniqueSplit *)d_usplits, d_results);
    if (hipGetLastError() != hipSuccess) return -1;
    if (!join()) return -1;
    if (mark) mark(mark_ctx, "partition_unique");
    (void)d_ticket;
    // One launch per key kind and width (jobs are grouped by key kind).
    for (int i = 0; i < njobs;) {
        int k = i;
        while (k + 1 < njobs && h_jobs[k + 1].key_kind == h_jobs[i].key_kind) k++;
        const uint32_t t0 = h_jobs[i].utile_base, t1 = h_jobs[k].utile_base + h_jobs[k].utile_count;
        bool narrow = false, wide = false;
        for (int q = i; q <= k; q++)
            if (h_jobs[q].unique) (h_jobs[q].value_size > 32 ? wide : narrow) = true;
        for (int w = 0; w < 2 && t1 > t0; w++) {
            if (!(w ? wide : narrow)) continue;
            const dim3 grid(t1 - t0), block(kUniqueThreads);
            const uint32_t lds = unique_lds_bytes();
#define TBC_MU(K)                                                                                                      \
    do {                                                                                                               \
        if (w)                                                                                                         \
            hipLaunchKernelGGL((k_merge_unique<K, true>), grid, block, lds, s, d_jobs, njobs, t0,                     \
                               (const UniqueSplit *)d_usplits, d_results);                                             \
        else                                                                                                           \
            hipLaunchKernelGGL((k_merge_unique<K, false>), grid, block, lds, s, d_jobs, njobs, t0,                    \
                               (const UniqueSplit *)d_usplits, d_results);                                             \
    } while (0)
            switch (h_jobs[i].key_kind) {
            case kKeyTimestamp: TBC_MU(kKeyTimestamp); break;
            case kKeyIdU128: TBC_MU(kKeyIdU128); break;
            case kKeyCompositeU64: TBC_MU(kKeyCompositeU64); break;
            default: TBC_MU(kKeyCompositeU128); break;
            }
#undef TBC_MU
        }
        i = k + 1;
    }
    if (hipGetLastError() != hipSuccess) return -1;
    if (mark) mark(mark_ctx, "merge_unique");
    return 0;
}

// --------------------------------------------------------------------------
// One pass per tile (merged positions [d0, d1)): load keys, decide each
// position's side (A or B) and whether it survives, and publish them as two
// bit masks per 64 positions plus the tile's survivor count. Tiles are
// independent (no look-back, any order); k_tile_scan turns the counts into
// output offsets, and the producer waves of k_data_blocks walk the masks to
// assemble each output block's body.
// --------------------------------------------------------------------------
constexpr uint32_t kMaskWords = kMergeTile / 64; // per mask kind per tile

template <int KL> struct TileShared {
    uint64_t key[KL][kMergeTile + 3]; // A[i0-1 .. i1] then B[j0 .. j1]
    uint8_t tomb[kMergeTile + 4];
    uint32_t wave_sums[kMergeThreads / 64];
};

template <int KIND>
__device__ __forceinline__ void merge_tile(const JobDesc *jobs, const TileRef *order, uint32_t order_offset,
                                           const SplitDesc *splits, uint64_t *status, uint64_t *masks,
                                           const JobResultDev *res, uint32_t phase, uint32_t slot) {
    constexpr int KL = KeyLimbs<KIND>::value;
    __shared__ TileShared<KL> sh;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    const TileRef ref = order[order_offset + slot];
    const JobDesc &j = jobs[ref.job];
    if (phase_skips(j, res, phase)) return;
    const uint32_t t = ref.tile;
    const uint32_t na_all = j.a.n, nb_all = j.b.n, n = na_all + nb_all;
    const uint32_t d0 = t * kMergeTile;
    const uint32_t d1 = (d0 + kMergeTile) < n ? d0 + kMergeTile : n;
    const SplitDesc s0 = splits[j.split_base + t];
    const uint32_t i0 = s0.i, i1 = splits[j.split_base + t + 1].i;
    const uint32_t j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t na = i1 - i0, nb = j1 - j0;
    const uint32_t vs = j.value_size, ts = j.timestamp_offset;
    const bool immutable = j.a_immutable != 0;
    const bool secondary = j.usage == 1;
    const bool drop = j.drop_tombstones != 0;

    // The segments around the tile, resolved by the partition (no segment
    // table round trip and no barrier before the key loads).
    const SplitSeg sg = j.split_segs[t];

    // Load keys: entries [0, ea) = A[i0-1 .. i1], entries [ea, ea+eb) = B[j0 .. j1].
    const uint32_t ea = na + 2, eb = nb + 1;
    constexpr uint32_t kPerLoad = (kMergeTile + 3 + kMergeThreads - 1) / kMergeThreads;
    const uint8_t *ptrs[kPerLoad];
#pragma unroll
    for (uint32_t r = 0; r < kPerLoad; r++) {
        const uint32_t e = tid + r * kMergeThreads;
        const uint8_t *p = nullptr;
        if (e < ea + eb) {
            const bool is_a = e < ea;
            const Stream &s = is_a ? j.a : j.b;
            const int64_t idx = is_a ? (int64_t)i0 - 1 + e : (int64_t)j0 + (e - ea);
            if (idx >= 0 && idx < (int64_t)s.n) {
                const uint32_t x = (uint32_t)idx;
                const uint64_t *ptr = is_a ? sg.a_ptr : sg.b_ptr;
                const uint32_t *pre = is_a ? sg.a_pre : sg.b_pre;
                if (x < pre[1]) p = (const uint8_t *)ptr[0] + (size_t)(x - pre[0]) * vs;
                else if (x < pre[2]) p = (const uint8_t *)ptr[1] + (size_t)(x - pre[1]) * vs;
                else p = elem_ptr(s, seg_search(s, x), x, vs); // blocks under 2,051 values: the table
            }
        }
        ptrs[r] = p;
    }
    // Every entry's loads are issued before any is waited for: loads behind
    // a branch each ended in their own wait (one HBM round trip per entry,
    // kPerLoad in sequence); an absent entry reads a value the tile has.
    // (a stand-in: the first value of a side the tile reads, one exists)
    const uint8_t *any = (const uint8_t *)(sg.a_ptr[0] ? sg.a_ptr[0] : sg.b_ptr[0]);
    Key<KL> kr[kPerLoad];
    uint32_t tr[kPerLoad];
#pragma unroll
    for (uint32_t r = 0; r < kPerLoad; r++) {
        const uint8_t *p = ptrs[r] ? ptrs[r] : any;
        kr[r] = load_key<KIND>(p, ts);
        tr[r] = load_tomb(p, ts);
    }
#pragma unroll
    for (uint32_t r = 0; r < kPerLoad; r++) {
        const uint32_t e = tid + r * kMergeThreads;
        if (e >= ea + eb) continue;
#pragma unroll
        for (int l = 0; l < KL; l++) sh.key[l][e] = ptrs[r] ? kr[r].l[l] : ~0ull;
        if (e < ea) sh.tomb[e] = ptrs[r] ? (uint8_t)tr[r] : (uint8_t)0;
    }
    __syncthreads();

    auto entry_key = [&](uint32_t e) {
        Key<KL> k;
#pragma unroll
        for (int l = 0; l < KL; l++) k.l[l] = sh.key[l][e];
        return k;
    };
    // Length of the run of equal keys ending at A[ia] (secondary-index dedup).
    auto run_len = [&](uint32_t ia) {
        const Key<KL> k = entry_key(ia - i0 + 1);
        uint32_t len = 1;
        int64_t idx = (int64_t)ia - 1;
        while (idx >= 0) {
            Key<KL> kk;
            if (idx >= (int64_t)i0 - 1) {
                kk = entry_key((uint32_t)(idx - ((int64_t)i0 - 1)));
            } else {
                const uint8_t *p = elem_ptr(j.a, seg_search(j.a, (uint32_t)idx), (uint32_t)idx, vs);
                kk = load_key<KIND>(p, ts);
            }
            if (!key_eq(kk, k)) break;
            len++;
            idx--;
        }
        return len;
    };

    // Each thread owns merged positions [kPer*tid, kPer*tid + kPer): one
    // merge-path search in LDS for its start, then a sequential merge (A
    // first on equal keys) applying the survivor rules to each element.
    constexpr uint32_t kPer = kMergeTile / kMergeThreads;
    static_assert(64 % kPer == 0 && kPer <= 32, "a mask word covers whole threads");
    const uint32_t total_pos = na + nb;
    const uint32_t d = kPer * tid < total_pos ? kPer * tid : total_pos;
    uint32_t a, b;
    {
        uint32_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (key_le(entry_key(1 + mid), entry_key(ea + d - 1 - mid))) lo = mid + 1;
            else hi = mid;
        }
        a = lo;
        b = d - lo;
    }
    uint32_t sbits = 0, abits = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        if (d + k >= total_pos) continue;
        const bool take_a = a < na && (b >= nb || key_le(entry_key(1 + a), entry_key(ea + b)));
        bool surv;
        if (take_a) {
            // A element ia = i0 + a at entry a + 1; B[b] (entry ea + b) is the next B.
            const uint32_t ia = i0 + a, e = a + 1;
            const Key<KL> ka = entry_key(e);
            bool dedup = true;
            if (immutable) {
                const bool next_eq = (ia + 1 < na_all) && key_eq(entry_key(e + 1), ka);
                dedup = !next_eq;
                if (dedup && secondary) dedup = (run_len(ia) & 1) != 0;
            }
            const bool b_valid = b < nb || j1 < nb_all;
            const bool eq_b = b_valid && key_eq(entry_key(ea + b), ka);
            surv = dedup && !(drop && sh.tomb[e]) && !(secondary && eq_b);
            abits |= 1u << k;
            a++;
        } else {
            // B element jb = j0 + b at entry ea + b; the previous A (global
            // index i0 + a - 1) is entry a.
            const uint32_t e = ea + b;
            const Key<KL> kb = entry_key(e);
            bool a_exists = (i0 + a) >= 1 && key_eq(entry_key(a), kb);
            if (a_exists && immutable && secondary) a_exists = (run_len(i0 + a - 1) & 1) != 0;
            surv = !a_exists;
            b++;
        }
        sbits |= (surv ? 1u : 0u) << k;
    }
    // Mask word q (positions 64q..64q+63) is the OR of the bit groups of
    // threads q*64/kPer .. (q+1)*64/kPer - 1, all in one wave.
    constexpr uint32_t kThreadsPerWord = 64 / kPer;
    const uint32_t sh_bits = kPer * (tid % kThreadsPerWord);
    uint64_t sw = (uint64_t)sbits << sh_bits, aw = (uint64_t)abits << sh_bits;
    for (uint32_t o = 1; o < kThreadsPerWord; o <<= 1) {
        sw |= __shfl_xor(sw, o, 64);
        aw |= __shfl_xor(aw, o, 64);
    }
    uint64_t *m = masks + (size_t)(j.tile_base + t) * (2 * kMaskWords);
    if (tid % kThreadsPerWord == 0) {
        gst<uint64_t>(m + tid / kThreadsPerWord, sw);
        gst<uint64_t>(m + kMaskWords + tid / kThreadsPerWord, aw);
    }
    uint32_t sum = __builtin_popcount(sbits);
    for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o, 64);
    if (lane == 0) sh.wave_sums[tid >> 6] = sum;
    __syncthreads();
    uint32_t cnt = 0;
    for (uint32_t w = 0; w < kMergeThreads / 64; w++) cnt += sh.wave_sums[w];
    if (tid == 0) gst<uint64_t>(status + j.tile_base + t, (uint64_t)cnt);
}

// One merge tile per workgroup.
template <int KIND>
__global__ __launch_bounds__(kMergeThreads) void k_merge_tile(const JobDesc *jobs, const TileRef *order,
                                                              uint32_t order_offset, const SplitDesc *splits,
                                                              uint64_t *status, uint64_t *masks,
                                                              const JobResultDev *res, uint32_t phase) {
    merge_tile<KIND>(jobs, order, order_offset, splits, status, masks, res, phase, blockIdx.x);
}

// The recomputation phase of a speculating batch: a small grid strides over
// the tiles (most leave at once, all of them while no speculation broke).
template <int KIND>
__global__ __launch_bounds__(kMergeThreads) void k_merge_tile_redo(const JobDesc *jobs, const TileRef *order,
                                                                   uint32_t order_offset, const SplitDesc *splits,
                                                                   uint64_t *status, uint64_t *masks,
                                                                   const JobResultDev *res, uint32_t ntiles) {
    if (*(volatile const uint32_t *)jobs[0].spec_any == 0) return;
    for (uint32_t slot = blockIdx.x; slot < ntiles; slot += gridDim.x) {
        merge_tile<KIND>(jobs, order, order_offset, splits, status, masks, res, 1u, slot);
        __syncthreads();
    }
}

// Per job (one workgroup): exclusive scan of the tile survivor counts into
// status[t] = count | offset << 32, the output shape (write_blocks,
// compaction.zig:806-850: full data blocks except the last, full tables
// except the last), and for every data block k the tile holding its first
// value (block_tile[dblock_base + k]).
constexpr uint32_t kScanThreads = 1024;

__global__ __launch_bounds__(kScanThreads) void k_tile_scan(const JobDesc *jobs, uint64_t *status,
                                                           uint32_t *block_tile, JobResultDev *res, uint32_t phase) {
    __shared__ uint32_t wsum[kScanThreads / 64];
    __shared__ uint64_t carry;
    const JobDesc &j = jobs[blockIdx.x];
    if (phase_skips(j, res, phase)) return;
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    uint64_t *st = status + j.tile_base;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < j.tile_count; base += kScanThreads) {
        const uint32_t t = base + tid;
        const uint32_t c = t < j.tile_count ? (uint32_t)gld<uint64_t>(st + t) : 0u;
        uint32_t incl = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += y;
        }
        if (lane == 63) wsum[tid >> 6] = incl;
        __syncthreads();
        uint32_t woff = 0;
        for (uint32_t w = 0; w < (tid >> 6); w++) woff += wsum[w];
        const uint64_t off = carry + woff + incl - c;
        if (t < j.tile_count) {
            gst<uint64_t>(st + t, (uint64_t)c | (off << 32));
            // Data blocks whose first value lies in this tile.
            if (c) {
                uint64_t k = (off + j.vcm - 1) / j.vcm;
                for (; k * j.vcm < off + c; k++) gst<uint32_t>(block_tile + j.dblock_base + k, t);
            }
        }
        __syncthreads();
        if (tid == kScanThreads - 1) carry = off + c;
        __syncthreads();
    }
    if (tid == 0) {
        const uint64_t total = carry;
        const uint32_t db = (uint32_t)((total + j.vcm - 1) / j.vcm);
        const uint32_t tables = (db + j.dbcm - 1) / j.dbcm;
        JobResultDev &r = res[j.job_index];
        r.value_count = total;
        r.data_block_count = db;
        r.table_count = tables;
        r.block_count = db + tables;
    }
}

template <int KIND>
static int launch_kind(uint32_t phase, const JobDesc *d_jobs, const JobDesc *h_jobs, int first, int count,
                       SplitDesc *d_splits, uint64_t *d_status, uint64_t *d_masks, const TileRef *d_order,
                       const JobResultDev *d_res, hipStream_t s) {
    const JobDesc &f = h_jobs[first];
    const JobDesc &l = h_jobs[first + count - 1];
    const uint32_t split_off = f.split_base;
    const uint32_t nsplits = l.split_base + l.tile_count + 1 - split_off;
    const uint32_t tile_off = f.tile_base;
    const uint32_t ntiles = l.tile_base + l.tile_count - tile_off;
    (void)split_off;
    (void)nsplits;
    // Jobs of this kind that the phase runs (host-known: speculated or not).
    bool any = false;
    for (int k = first; k < first + count; k++) any |= phase == 0 ? !h_jobs[k].unique : h_jobs[k].unique != 0;
    if (!any) return 0;
    // The recomputation leaves at once while no speculation broke, but every
    // workgroup needs a CU with room for its tile's LDS first: beside the
    // chain workgroups of earlier batches few CUs have it, so a grid of 1,024
    // waited up to 0.3 ms for slots (config 2, round 6 trace); 64 workgroups
    // striding over the tiles when a speculation did break.
    if (ntiles && phase)
        hipLaunchKernelGGL((k_merge_tile_redo<KIND>), dim3(std::min<uint32_t>(ntiles, 64)), dim3(kMergeThreads), 0,
                           s, d_jobs, d_order, tile_off, (const SplitDesc *)d_splits, d_status, d_masks, d_res, ntiles);
    else if (ntiles)
        hipLaunchKernelGGL((k_merge_tile<KIND>), dim3(ntiles), dim3(kMergeThreads), 0, s, d_jobs, d_order, tile_off,
                           (const SplitDesc *)d_splits, d_status, d_masks, d_res, phase);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Jobs must be grouped by key kind (contiguous runs) by the caller. d_status
// holds one u64 per tile, d_masks 2 * kMergeTile / 64 u64 per tile,
// d_block_tile one u32 per data block (upper bound); results start zeroed.
int launch_merge(const JobDesc *d_jobs, const JobDesc *h_jobs, int njobs, SplitDesc *d_splits,
                 uint64_t *d_status, uint64_t *d_masks, uint32_t *d_block_tile, const TileRef *d_order,
                 JobResultDev *d_results, void *stream, void (*mark)(void *, const char *), void *mark_ctx,
                 uint32_t phase) {
    hipStream_t s = (hipStream_t)stream;
    bool any = false;
    for (int k = 0; k < njobs; k++) any |= phase == 0 ? !h_jobs[k].unique : h_jobs[k].unique != 0;
    if (!any) return 0;
    auto for_each_kind = [&](auto fn) {
        int first = 0;
        while (first < njobs) {
            int last = first;
            while (last + 1 < njobs && h_jobs[last + 1].key_kind == h_jobs[first].key_kind) last++;
            if (fn(h_jobs[first].key_kind, first, last - first + 1)) return -1;
            first = last + 1;
        }
        return 0;
    };
    auto run = [&](uint32_t ph) {
        return for_each_kind([&](uint32_t kind, int first, int count) {
            switch (kind) {
            case kKeyTimestamp: return launch_kind<kKeyTimestamp>(ph, d_jobs, h_jobs, first, count, d_splits, d_status, d_masks, d_order, d_results, s);
            case kKeyIdU128: return launch_kind<kKeyIdU128>(ph, d_jobs, h_jobs, first, count, d_splits, d_status, d_masks, d_order, d_results, s);
            case kKeyCompositeU64: return launch_kind<kKeyCompositeU64>(ph, d_jobs, h_jobs, first, count, d_splits, d_status, d_masks, d_order, d_results, s);
            default: return launch_kind<kKeyCompositeU128>(ph, d_jobs, h_jobs, first, count, d_splits, d_status, d_masks, d_order, d_results, s);
            }
        });
    };
    {
        const JobDesc &l = h_jobs[njobs - 1];
        const uint32_t nsplits = l.split_base + l.tile_count + 1;
        if (nsplits <= wave_splits_max())
            hipLaunchKernelGGL(k_partition_all<true>, dim3((nsplits + 3) / 4), dim3(256), 0, s, d_jobs, njobs, nsplits,
                           d_splits, (const JobResultDev *)d_results, phase);
        else
            hipLaunchKernelGGL(k_partition_all<false>, dim3((nsplits + 255) / 256), dim3(256), 0, s, d_jobs, njobs, nsplits,
                           d_splits, (const JobResultDev *)d_results, phase);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mark) mark(mark_ctx, phase ? "recompute_partition" : "merge_partition");
    if (run(phase)) return -1;
    hipLaunchKernelGGL(k_tile_scan, dim3(njobs), dim3(kScanThreads), 0, s, d_jobs, d_status, d_block_tile,
                       d_results, phase);
    if (hipGetLastError() != hipSuccess) return -1;
    if (mark) mark(mark_ctx, phase ? "recompute_merge" : "merge");
    return 0;
}

} // namespace tbc
