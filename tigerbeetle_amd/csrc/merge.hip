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
// Kernels: merge-path split per tile boundary -> per-tile survivor count ->
// per-job exclusive scan (also yields data-block / table counts) -> per-tile
// write of survivors straight into their output data-block slots.
#include <hip/hip_runtime.h>

#include "tbc_internal.h"

namespace tbc {

template <int KIND> struct KeyLimbs { static constexpr int value = KIND == kKeyTimestamp ? 1 : KIND == kKeyCompositeU128 ? 3 : 2; };

template <int KL> struct Key {
    uint64_t l[KL];
};

template <int KL> __device__ __forceinline__ bool key_eq(const Key<KL> &a, const Key<KL> &b) {
    bool e = true;
#pragma unroll
    for (int i = 0; i < KL; i++) e &= a.l[i] == b.l[i];
    return e;
}

// a <= b (unsigned, most significant limb last)
template <int KL> __device__ __forceinline__ bool key_le(const Key<KL> &a, const Key<KL> &b) {
#pragma unroll
    for (int i = KL - 1; i > 0; i--)
        if (a.l[i] != b.l[i]) return a.l[i] < b.l[i];
    return a.l[0] <= b.l[0];
}

template <int KL> __device__ __forceinline__ bool key_lt(const Key<KL> &a, const Key<KL> &b) {
#pragma unroll
    for (int i = KL - 1; i > 0; i--)
        if (a.l[i] != b.l[i]) return a.l[i] < b.l[i];
    return a.l[0] < b.l[0];
}

__device__ __forceinline__ uint64_t ld64(const uint8_t *p) { return gld<uint64_t>(p); }

// key_from_value (composite_key.zig:48-50, groove.zig:27-29, 59-61).
template <int KIND>
__device__ __forceinline__ Key<KeyLimbs<KIND>::value> load_key(const uint8_t *v, uint32_t ts_off) {
    Key<KeyLimbs<KIND>::value> k;
    if constexpr (KIND == kKeyTimestamp) {
        k.l[0] = ld64(v + ts_off) & ~kTombstoneBit;
    } else if constexpr (KIND == kKeyIdU128) {
        k.l[0] = ld64(v);
        k.l[1] = ld64(v + 8);
    } else if constexpr (KIND == kKeyCompositeU64) {
        k.l[0] = ld64(v + 8) & ~kTombstoneBit;
        k.l[1] = ld64(v);
    } else {
        k.l[0] = ld64(v + 16) & ~kTombstoneBit;
        k.l[1] = ld64(v);
        k.l[2] = ld64(v + 8);
    }
    return k;
}

__device__ __forceinline__ uint32_t load_tomb(const uint8_t *v, uint32_t ts_off) {
    return (uint32_t)(ld64(v + ts_off) >> 63);
}

// Segment containing element idx: the largest s with seg_pre[s] <= idx.
__device__ __forceinline__ uint32_t seg_search(const Stream &s, uint32_t idx) {
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
// Merge-path partition: for every tile boundary d = t * kMergeTile, the number
// of A elements among the first d merged elements.
// --------------------------------------------------------------------------
template <int KIND>
__global__ __launch_bounds__(256) void k_partition(const JobDesc *jobs, int njobs, uint32_t split_offset,
                                                   uint32_t nsplits, uint32_t *splits) {
    const uint32_t gid = blockIdx.x * 256 + threadIdx.x;
    if (gid >= nsplits) return;
    const uint32_t gsplit = split_offset + gid;
    const int ji = find_job(jobs, njobs, gsplit, [](const JobDesc &d) { return d.split_base; });
    const JobDesc &j = jobs[ji];
    const uint32_t t = gsplit - j.split_base;
    const uint32_t na = j.a.n, nb = j.b.n, n = na + nb;
    const uint32_t d = (uint64_t)t * kMergeTile < n ? t * kMergeTile : n;
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
    splits[gsplit] = lo;
}

// --------------------------------------------------------------------------
// Tile kernel: survivors of merged positions [d0, d1). COUNT: per-tile
// survivor count. WRITE: copy survivors to their output slots.
// --------------------------------------------------------------------------
template <int KL> struct TileShared {
    uint64_t key[KL][kMergeTile + 3]; // A[i0-1 .. i1] then B[j0 .. j1]
    const uint8_t *ptr[kMergeTile + 3];
    uint8_t tomb[kMergeTile + 2];
    uint32_t pos[kMergeTile];  // merged position -> entry (0xffffffff = dropped)
    uint32_t out[kMergeTile];  // output order -> entry
    uint32_t wave_sums[kMergeThreads / 64];
    uint32_t seg_a, seg_b, count;
};

template <int KIND, bool WRITE>
__global__ __launch_bounds__(kMergeThreads) void k_merge_tile(const JobDesc *jobs, int njobs, uint32_t tile_offset,
                                                              const uint32_t *splits, uint32_t *tile_counts) {
    constexpr int KL = KeyLimbs<KIND>::value;
    __shared__ TileShared<KL> sh;
    const uint32_t tid = threadIdx.x;
    const uint32_t gtile = tile_offset + blockIdx.x;
    const int ji = find_job(jobs, njobs, gtile, [](const JobDesc &d) { return d.tile_base; });
    const JobDesc &j = jobs[ji];
    const uint32_t t = gtile - j.tile_base;
    const uint32_t na_all = j.a.n, nb_all = j.b.n, n = na_all + nb_all;
    const uint32_t d0 = t * kMergeTile;
    const uint32_t d1 = (d0 + kMergeTile) < n ? d0 + kMergeTile : n;
    const uint32_t i0 = splits[j.split_base + t], i1 = splits[j.split_base + t + 1];
    const uint32_t j0 = d0 - i0, j1 = d1 - i1;
    const uint32_t na = i1 - i0, nb = j1 - j0;
    const uint32_t vs = j.value_size, ts = j.timestamp_offset;
    const bool immutable = j.a_immutable != 0;
    const bool secondary = j.usage == 1;
    const bool drop = j.drop_tombstones != 0;

    if (tid == 0) {
        sh.seg_a = na_all ? seg_search(j.a, i0 > 0 ? i0 - 1 : 0) : 0;
        sh.seg_b = nb_all ? seg_search(j.b, j0 < nb_all ? j0 : (nb_all ? nb_all - 1 : 0)) : 0;
    }
    __syncthreads();

    // Load keys: entries [0, na+2) = A[i0-1 .. i1], entries [na+2, na+2+nb+1) = B[j0 .. j1].
    const uint32_t ea = na + 2, eb = nb + 1;
    for (uint32_t e = tid; e < ea + eb; e += kMergeThreads) {
        const bool is_a = e < ea;
        const Stream &s = is_a ? j.a : j.b;
        const int64_t idx = is_a ? (int64_t)i0 - 1 + e : (int64_t)j0 + (e - ea);
        const bool valid = idx >= 0 && idx < (int64_t)s.n;
        Key<KL> k;
#pragma unroll
        for (int l = 0; l < KL; l++) k.l[l] = ~0ull;
        const uint8_t *p = nullptr;
        uint32_t tb = 0;
        if (valid) {
            uint32_t seg = is_a ? sh.seg_a : sh.seg_b;
            while (seg + 1 < s.nseg && gld<uint32_t>(s.seg_pre + seg + 1) <= (uint32_t)idx) seg++;
            p = elem_ptr(s, seg, (uint32_t)idx, vs);
            k = load_key<KIND>(p, ts);
            if (is_a) tb = load_tomb(p, ts);
        }
#pragma unroll
        for (int l = 0; l < KL; l++) sh.key[l][e] = k.l[l];
        if (WRITE) sh.ptr[e] = p;
        if (is_a) sh.tomb[e] = (uint8_t)tb;
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

    uint32_t local = 0;
    for (uint32_t q = tid; q < na + nb; q += kMergeThreads) {
        uint32_t pos, entry;
        bool surv;
        if (q < na) {
            // A element ia = i0 + q at entry q + 1.
            const uint32_t ia = i0 + q;
            entry = q + 1;
            const Key<KL> ka = entry_key(entry);
            // lower_bound over in-tile B entries: count of B < ka.
            uint32_t lo = 0, hi = nb;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (key_lt(entry_key(ea + mid), ka)) lo = mid + 1;
                else hi = mid;
            }
            pos = q + lo;
            bool dedup = true;
            if (immutable) {
                const bool next_eq = (ia + 1 < na_all) && key_eq(entry_key(entry + 1), ka);
                dedup = !next_eq;
                if (dedup && secondary) dedup = (run_len(ia) & 1) != 0;
            }
            const bool b_valid = lo < nb || j1 < nb_all;
            const bool eq_b = b_valid && key_eq(entry_key(ea + lo), ka);
            surv = dedup && !(drop && sh.tomb[entry]) && !(secondary && eq_b);
        } else {
            // B element jb = j0 + qb at entry ea + qb.
            const uint32_t qb = q - na;
            entry = ea + qb;
            const Key<KL> kb = entry_key(entry);
            // upper_bound over in-tile A entries [1, na]: count of A <= kb.
            uint32_t lo = 0, hi = na;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (key_le(entry_key(1 + mid), kb)) lo = mid + 1;
                else hi = mid;
            }
            pos = qb + lo;
            // Previous A (global index i0 + lo - 1) is entry lo.
            const bool prev_valid = (i0 + lo) >= 1;
            bool a_exists = prev_valid && key_eq(entry_key(lo), kb);
            if (a_exists && immutable && secondary) a_exists = (run_len(i0 + lo - 1) & 1) != 0;
            surv = !a_exists;
            entry |= 0x80000000u;
        }
        local += surv ? 1u : 0u;
        if (WRITE) sh.pos[pos] = surv ? entry : 0xffffffffu;
    }

    if (!WRITE) {
        // Block reduction of survivor counts.
        uint32_t v = local;
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        if ((tid & 63) == 0) sh.wave_sums[tid >> 6] = v;
        __syncthreads();
        if (tid == 0) {
            uint32_t s = 0;
            for (uint32_t w = 0; w < kMergeThreads / 64; w++) s += sh.wave_sums[w];
            tile_counts[gtile] = s;
        }
        return;
    }

    __syncthreads();
    // Exclusive scan of survivor flags in merged order; each thread owns 4
    // consecutive positions.
    const uint32_t total_pos = na + nb;
    constexpr uint32_t kPer = kMergeTile / kMergeThreads;
    uint32_t f[kPer];
    uint32_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        const uint32_t pidx = tid * kPer + k;
        f[k] = (pidx < total_pos && sh.pos[pidx] != 0xffffffffu) ? 1u : 0u;
        sum += f[k];
    }
    // Wave inclusive scan.
    const uint32_t lane = tid & 63;
    uint32_t incl = sum;
    for (int o = 1; o < 64; o <<= 1) {
        uint32_t y = __shfl_up(incl, o, 64);
        if (lane >= (uint32_t)o) incl += y;
    }
    if (lane == 63) sh.wave_sums[tid >> 6] = incl;
    __syncthreads();
    uint32_t wave_off = 0;
    for (uint32_t w = 0; w < (tid >> 6); w++) wave_off += sh.wave_sums[w];
    if (tid == kMergeThreads - 1) sh.count = wave_off + incl;
    uint32_t o = wave_off + incl - sum;
#pragma unroll
    for (uint32_t k = 0; k < kPer; k++) {
        const uint32_t pidx = tid * kPer + k;
        if (f[k]) sh.out[o++] = sh.pos[pidx];
    }
    __syncthreads();

    // Copy survivors, 16 bytes per lane, to data block k = g / vcm, slot
    // k + k / dbcm (table.zig:306-384 block order, compaction.zig:819-835 acquire order).
    const uint32_t cnt = sh.count;
    const uint64_t g0 = tile_counts[gtile];
    const uint32_t cpv = vs >> 4;
    const uint32_t cpv_shift = __builtin_ctz(cpv);
    const uint32_t vcm = j.vcm;
    const uint32_t k_start = (uint32_t)(g0 / vcm);
    const uint32_t o_start = (uint32_t)(g0 - (uint64_t)k_start * vcm);
    for (uint32_t c = tid; c < cnt * cpv; c += kMergeThreads) {
        const uint32_t v = c >> cpv_shift, part = c & (cpv - 1);
        const uint32_t e = sh.out[v] & 0x7fffffffu;
        const u32x4 val = gld<u32x4>(sh.ptr[e] + 16 * part);
        const uint32_t rel = o_start + v;
        const uint32_t kb = k_start + rel / vcm;
        const uint32_t ob = rel - (kb - k_start) * vcm;
        uint8_t *dst = j.out_blocks + (size_t)data_block_slot(kb, j.dbcm) * j.block_size + kHeaderSize +
                       (size_t)ob * vs + 16 * part;
        gst<u32x4>(dst, val);
    }
}

// Per-job exclusive scan of tile counts; derives the output shape
// (write_blocks, compaction.zig:806-850: full data blocks except the last,
// full tables except the last).
__global__ __launch_bounds__(256) void k_merge_scan(const JobDesc *jobs, uint32_t *tile_counts, JobResultDev *res) {
    __shared__ uint32_t wave_sums[4];
    __shared__ uint64_t carry;
    const JobDesc &j = jobs[blockIdx.x];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (tid == 0) carry = 0;
    __syncthreads();
    for (uint32_t base = 0; base < j.tile_count; base += 256) {
        const uint32_t i = base + tid;
        const uint32_t v = i < j.tile_count ? tile_counts[j.tile_base + i] : 0;
        uint32_t incl = v;
        for (int o = 1; o < 64; o <<= 1) {
            uint32_t y = __shfl_up(incl, o, 64);
            if (lane >= (uint32_t)o) incl += y;
        }
        if (lane == 63) wave_sums[tid >> 6] = incl;
        __syncthreads();
        uint32_t woff = 0;
        for (uint32_t w = 0; w < (tid >> 6); w++) woff += wave_sums[w];
        const uint64_t c0 = carry;
        if (i < j.tile_count) tile_counts[j.tile_base + i] = (uint32_t)(c0 + woff + incl - v);
        __syncthreads();
        if (tid == 255) carry = c0 + woff + incl;
        __syncthreads();
    }
    if (tid == 0) {
        const uint64_t total = carry;
        const uint32_t db = (uint32_t)((total + j.vcm - 1) / j.vcm);
        const uint32_t tables = (db + j.dbcm - 1) / j.dbcm;
        JobResultDev r;
        r.value_count = total;
        r.data_block_count = db;
        r.table_count = tables;
        r.block_count = db + tables;
        r.status = 0;
        r.invariant = 0;
        r.pad = 0;
        res[j.job_index] = r;
    }
}

template <int KIND>
static int launch_kind(int phase, const JobDesc *d_jobs, const JobDesc *h_jobs, int first, int count,
                       uint32_t *d_splits, uint32_t *d_tile_counts, hipStream_t s) {
    const JobDesc &f = h_jobs[first];
    const JobDesc &l = h_jobs[first + count - 1];
    const uint32_t split_off = f.split_base;
    const uint32_t nsplits = l.split_base + l.tile_count + 1 - split_off;
    const uint32_t tile_off = f.tile_base;
    const uint32_t ntiles = l.tile_base + l.tile_count - tile_off;
    if (phase == 0)
        hipLaunchKernelGGL(k_partition<KIND>, dim3((nsplits + 255) / 256), dim3(256), 0, s, d_jobs + first, count,
                           split_off, nsplits, d_splits);
    else if (phase == 1 && ntiles)
        hipLaunchKernelGGL((k_merge_tile<KIND, false>), dim3(ntiles), dim3(kMergeThreads), 0, s, d_jobs + first,
                           count, tile_off, (const uint32_t *)d_splits, d_tile_counts);
    else if (phase == 2 && ntiles)
        hipLaunchKernelGGL((k_merge_tile<KIND, true>), dim3(ntiles), dim3(kMergeThreads), 0, s, d_jobs + first,
                           count, tile_off, (const uint32_t *)d_splits, d_tile_counts);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Jobs must be grouped by key kind (contiguous runs) by the caller.
int launch_merge(const JobDesc *d_jobs, const JobDesc *h_jobs, int njobs, uint32_t total_tiles,
                 uint32_t total_splits, uint32_t *d_splits, uint32_t *d_tile_counts, JobResultDev *d_results,
                 void *stream, void (*mark)(void *, const char *), void *mark_ctx) {
    (void)total_tiles;
    (void)total_splits;
    hipStream_t s = (hipStream_t)stream;
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
    auto phase = [&](int ph) {
        return for_each_kind([&](uint32_t kind, int first, int count) {
            switch (kind) {
            case kKeyTimestamp: return launch_kind<kKeyTimestamp>(ph, d_jobs, h_jobs, first, count, d_splits, d_tile_counts, s);
            case kKeyIdU128: return launch_kind<kKeyIdU128>(ph, d_jobs, h_jobs, first, count, d_splits, d_tile_counts, s);
            case kKeyCompositeU64: return launch_kind<kKeyCompositeU64>(ph, d_jobs, h_jobs, first, count, d_splits, d_tile_counts, s);
            default: return launch_kind<kKeyCompositeU128>(ph, d_jobs, h_jobs, first, count, d_splits, d_tile_counts, s);
            }
        });
    };
    if (phase(0)) return -1;
    if (mark) mark(mark_ctx, "merge_partition");
    if (phase(1)) return -1;
    if (mark) mark(mark_ctx, "merge_count");
    hipLaunchKernelGGL(k_merge_scan, dim3(njobs), dim3(256), 0, s, d_jobs, d_tile_counts, d_results);
    if (hipGetLastError() != hipSuccess) return -1;
    if (mark) mark(mark_ctx, "merge_scan");
    int rc = phase(2);
    if (mark) mark(mark_ctx, "merge_write");
    return rc;
}

} // namespace tbc
