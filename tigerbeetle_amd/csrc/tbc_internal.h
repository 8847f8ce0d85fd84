// tbc_internal.h — device/host shared definitions of the compaction engine.
//
// Layout of one batch in device memory (all in the engine's static arena):
//   JobDesc[count]          per-compaction descriptor (tree layout, streams, bases)
//   u64 seg_ptr[...]        per-stream segment value pointers
//   u32 seg_pre[...]        per-stream segment prefix counts (nseg + 1 each)
//   u64 addresses[...]      acquire-order block addresses per job
//   SplitDesc splits[...]   merge-path A-splits at every tile boundary (tiles + 1 per job)
//   u64 status[...]         per tile: survivor count | output offset << 32
//   u32 block_tile[...]     per data block (upper bound): tile of its first value
//   JobResultDev[count]     device results (copied to pinned host memory at the end)
//   u8  table_infos[...]    128-byte ManifestNode.TableInfo per output table
// plus the engine's mask buffer (grown on demand, outside the arena):
//   u64 masks[tiles][2][kMergeTile / 64]   survivor bits, then from-A bits
#pragma once

#include <stddef.h>
#include <stdint.h>

namespace tbc {

constexpr uint32_t kHeaderSize = 256;  // @sizeOf(vsr.Header) (message_header.zig:68)
constexpr uint32_t kSectorSize = 4096; // constants.sector_size (constants.zig:418)
constexpr uint32_t kTableInfoSize = 128;
constexpr uint64_t kTombstoneBit = 1ull << 63;

// Merge tile: merged-sequence positions handled by one workgroup. Fixed:
// the block producers load a tile's 2 x 32 mask words one per lane of a wave
// (aegis.hip produce_body), so other sizes are not supported builds.
constexpr uint32_t kMergeTile = 2048;
static_assert(2 * (kMergeTile / 64) == 64, "one mask word per lane");
constexpr uint32_t kMergeThreads = kMergeTile / 4;

enum KeyKind : uint32_t { kKeyTimestamp = 0, kKeyIdU128 = 1, kKeyCompositeU64 = 2, kKeyCompositeU128 = 3 };

struct Stream {
    const uint64_t *seg_ptr; // device pointer of each segment's first value
    const uint32_t *seg_pre; // prefix counts, nseg + 1 entries
    uint32_t nseg;
    uint32_t n; // total values
    // Nonzero when every segment but the last holds exactly this many values
    // (full data blocks: one disk table, or tables of whole blocks): the
    // segment of an element is then a division, not a binary search.
    uint32_t uniform;
    uint32_t pad;
};

struct JobDesc {
    // Tree layout (table.zig:107-129, schema.zig:119-157).
    uint32_t key_kind, usage, value_size, timestamp_offset;
    uint32_t key_size, vcm, dbcm, index_size;
    uint32_t idx_checksums_off, idx_keys_min_off, idx_keys_max_off, idx_addresses_off;
    uint32_t block_size;
    uint16_t tree_id;
    uint8_t a_immutable, drop_tombstones;
    uint8_t level_b;
    uint8_t unique; // TBC_COMPACTION_UNIQUE_KEYS held by the batch's plan (latency regime): blocks by speculation
    uint8_t pad0[2];
    uint64_t cluster_lo, cluster_hi, snapshot_min;
    Stream a, b;
    const uint64_t *addresses;
    uint32_t address_count;
    uint32_t merge_tile; // merged positions per merge tile (kMergeTile)
    uint8_t *out_blocks;
    // Batch bases (global grid indices).
    uint32_t tile_base, tile_count;      // merge tiles
    uint32_t split_base;                 // tile_count + 1 splits
    uint32_t dblock_base, dblock_max;    // data blocks (upper bound), batch-wide numbering
    uint32_t table_base, table_max;      // index-block groups (upper bound)
    uint32_t info_base;                  // first TableInfo slot in the batch's info buffer
    uint32_t job_index;
    // TBC_COMPACTION_GRID: output block `slot` lives at grid_base + (addresses[slot] - 1) * block_size.
    uint8_t *grid_base;
    // Speculating batches: the number of broken speculations (one word of the
    // batch's zeroed scratch); phase-1 kernels leave at once while it is 0.
    uint32_t *spec_any;
    // Pipelined speculated batches (merge.hip k_merge_unique): the job's
    // tiles of kUniqueTile merged positions, batch-wide numbering, and their
    // utile_count + 1 merge-path splits (0 tiles for a job not speculated).
    uint32_t utile_base, utile_count, usplit_base, pad1;
    // Key-range split of one job (split.py). VALUES_ONLY with
    // out_offset: survivor o lands at the job's merged output position
    // out_offset + o (its global data block and slot). Seal jobs
    // (tbc_compaction_seal, seal = 1): bodies are already in place; data
    // blocks [block_lo, block_lo + dblock_max) are finished and their index
    // entries written into their tables' index block slots, and the index
    // blocks of tables [table_lo, table_lo + table_max) are sealed from the
    // entries found there.
    uint64_t out_offset;
    uint32_t block_lo, table_lo;
    uint32_t seal, pad2;
    // Mask-merge tiles (merge.hip k_merge_tile): the input segments around
    // each tile boundary, resolved by the partition (tile_count + 1 of them).
    struct SplitSeg *split_segs;
};

// The input segments a mask-merge tile reads, resolved by the partition at
// its first boundary: for each side, the segment holding its first entry
// (A[i - 1], or A[0]; B[j], or B's last) and the next one — pointers and
// prefix counts (pre[2] = the end of the second) — so a tile computes its
// entries' addresses without a segment-table round trip (entries past the
// second segment, only with blocks under 2,051 values, search the table).
struct SplitSeg {
    uint64_t a_ptr[2], b_ptr[2];
    uint32_t a_pre[3], b_pre[3];
};

// Merged positions per tile of k_merge_unique (four per thread): the most
// significant 64 bits of the tile's keys (plus three neighbours) take 16.4
// KiB of LDS, so a workgroup fits beside a chain workgroup's 136 KiB of a
// CU's 160.
constexpr uint32_t kUniqueTile = 2048; // 1,024 x 256 threads measured no faster beside 8-wave tails (round 5)
constexpr uint32_t kUniqueThreads = 512;

struct SplitDesc {
    uint32_t i;     // A elements before the tile boundary (merge path)
    uint32_t seg_a; // segment of A[max(i-1, 0)]
    uint32_t seg_b; // segment of B[min(d-i, nb-1)]
    uint32_t pad;
};

// A k_merge_unique tile boundary: the merge-path split plus the input
// segment each side's first element lies in, resolved (pointer and element
// range), so a tile's loads start without walking the segment tables; and
// two keys around it: `below` = the smaller of A[i - 1], B[j - 1] that exist
// (zero if neither) and `above` = the larger of A[i], B[j] that exist (all
// ones if neither). Merge path orders everything before a boundary before
// everything after it, so every key a tile compares (its own and its three
// neighbour entries) lies in [below of its first boundary, above of its
// last]: they share those two keys' leading bits (merge.hip k_merge_unique).
// Six SplitDesc slots of the batch scratch.
struct UniqueSplit {
    uint32_t i;            // A elements before the boundary
    uint32_t seg_a, seg_b; // segments of A[max(i-1, 0)] and B[max(d-i-1, 0)]
    uint32_t pad;
    uint64_t a_ptr, b_ptr; // their first elements
    uint32_t a_lo, a_hi;   // element range [lo, hi) of segment seg_a
    uint32_t b_lo, b_hi;
    uint64_t below[3], above[3]; // keys, least significant limb first
};
static_assert(sizeof(UniqueSplit) == 6 * sizeof(SplitDesc), "six split slots");

// One entry of the batch's tile order: tiles of the jobs of one key kind,
// interleaved round-robin (job index into the batch's JobDesc array, tile).
struct TileRef {
    uint32_t job;
    uint32_t tile;
};

struct JobResultDev {
    uint64_t value_count;
    uint32_t data_block_count;
    uint32_t table_count;
    uint32_t block_count;
    uint32_t status;
    uint32_t invariant;   // nonzero if an input broke a reference invariant
    uint32_t block_error; // nonzero if a grid input block failed its checks (tbc_block_check code)
    uint32_t spec;        // unique-keys speculation: 0 none, 1 held, 2 broken (recomputed by the merge path)
    uint32_t pad;
};

constexpr uint32_t kSpecNone = 0, kSpecHeld = 1, kSpecBroken = 2;
// Launch phases of a batch with speculated jobs: phase 0 runs every
// non-speculated job (and the speculative block phase), phase 1 only the
// speculated jobs whose speculation broke.
__device__ __forceinline__ bool phase_skips(const JobDesc &j, const JobResultDev *res, uint32_t phase) {
    if (phase == 0) return j.unique != 0;
    return !j.unique || *(volatile const uint32_t *)j.spec_any == 0 ||
           *(volatile const uint32_t *)&res[j.job_index].spec != kSpecBroken;
}

// One grid input block of a batch (TBC_COMPACTION_GRID): the cache-hit checks
// of read_block_from_cache (grid.zig:802-841) plus the header fields the
// compaction relies on, and for blocks staged from storage the full
// read_block_validate (grid.zig:1059-1084).
struct InputCheck {
    uint64_t ptr;         // device pointer of the block
    uint64_t address;
    uint64_t checksum[2]; // expected header checksum
    uint32_t value_count; // data block: its values; index block: the table's data blocks
    uint32_t job;         // JobResultDev index
    uint32_t kind;        // schema.zig BlockType: 5 data, 4 index
    uint32_t pad;
};

// One data block of a grid input table, found through the table's index
// block (TableIndex.data_addresses / data_checksums, schema.zig:80-260).
struct ResolveItem {
    uint64_t index_ptr;    // the table's index block in the grid
    uint32_t k;            // data block ordinal in the table
    uint32_t seg;          // global segment slot (Stream::seg_ptr entry) to fill
    uint32_t check;        // InputCheck slot to fill
    uint32_t value_count;  // values of the block (full except the table's last)
    uint32_t job;          // JobResultDev index
    uint32_t cks_off, addr_off; // index layout of the job's tree
    uint32_t pad;
};

// Slot (= index into the acquire-order address list / output arena) of data
// block `k`: every earlier table consumed dbcm data blocks plus one index block.
__host__ __device__ inline uint32_t data_block_slot(uint32_t k, uint32_t dbcm) { return k + k / dbcm; }
// Slot of the index block of table `t` whose last data block is `k_last`.
__host__ __device__ inline uint32_t index_block_slot(uint32_t t, uint32_t k_last) { return k_last + t + 1; }

__host__ __device__ inline uint64_t sector_ceil(uint64_t x) {
    return (x + kSectorSize - 1) / kSectorSize * kSectorSize;
}

// Global-address-space accessors. Pointers that reach a kernel through a
// struct are generic (flat); flat loads also count against lgkmcnt, so an LDS
// wait would wait for HBM too. These force global_load/global_store.
#define TBC_GLOBAL __attribute__((address_space(1)))
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <class T> __device__ __forceinline__ T gld(const void *p) { return *(const TBC_GLOBAL T *)p; }
template <class T> __device__ __forceinline__ void gst(void *p, const T &v) { *(TBC_GLOBAL T *)p = v; }

// Output block `slot` of job j (acquire order): a per-job arena, or the grid
// slot of its acquired address.
__device__ inline uint8_t *block_ptr(const JobDesc &j, uint32_t slot) {
    if (j.grid_base) return j.grid_base + (size_t)(gld<uint64_t>(j.addresses + slot) - 1) * j.block_size;
    return j.out_blocks + (size_t)slot * j.block_size;
}

// The header fields a compaction's table iterators assert of a grid input
// block once its checksum and address are the expected ones: cluster,
// command, block type and tree, and for a data block its value count, value
// size and size (TableData.Metadata, schema.zig:264-275), for an index block
// its data block count and layout (TableIndex.Metadata, schema.zig:87-98).
// Returns 0, or 7 (TBC_BLOCK_UNEXPECTED_HEADER).
__device__ inline uint32_t grid_header_check(const JobDesc &j, const InputCheck &c, uint32_t block_size) {
    const uint8_t *blk = (const uint8_t *)(uintptr_t)c.ptr;
    const uint32_t size = gld<uint32_t>(blk + 96);
    bool ok = gld<uint64_t>(blk + 80) == j.cluster_lo && gld<uint64_t>(blk + 88) == j.cluster_hi &&
              blk[110] == 20 && blk[240] == c.kind && gld<uint16_t>(blk + 140) == j.tree_id && size <= block_size;
    if (c.kind == 5)
        ok = ok && gld<uint32_t>(blk + 132) == c.value_count && gld<uint32_t>(blk + 136) == j.value_size &&
             size == 256 + c.value_count * j.value_size;
    else
        ok = ok && gld<uint32_t>(blk + 128) == c.value_count && gld<uint32_t>(blk + 132) == j.dbcm &&
             gld<uint32_t>(blk + 136) == j.key_size && size == j.index_size;
    return ok ? 0u : 7u;
}

// Cursor over a stream's segments (input data blocks): the segment holding
// an element index, moving forward only (wave-uniform advance).
struct SegCursor {
    const uint64_t *ptrs;
    const uint32_t *pre;
    uint32_t nseg, seg, lo, hi;
    uint64_t base;
    __device__ __forceinline__ void load() {
        lo = gld<uint32_t>(pre + seg);
        hi = gld<uint32_t>(pre + seg + 1);
        base = gld<uint64_t>(ptrs + seg);
    }
    __device__ __forceinline__ void init(const Stream &s, uint32_t seg0) {
        ptrs = s.seg_ptr;
        pre = s.seg_pre;
        nseg = s.nseg;
        seg = nseg ? (seg0 < nseg ? seg0 : nseg - 1) : 0;
        if (nseg) load();
        else lo = hi = 0, base = 0;
    }
    // Move forward to the segment holding element `idx` (wave-uniform).
    __device__ __forceinline__ void advance(uint32_t idx) {
        while (seg + 1 < nseg && idx >= hi) {
            seg++;
            load();
        }
    }
    // Address of element idx >= lo (per lane; usually inside the cursor's segment).
    __device__ __forceinline__ const uint8_t *elem(uint32_t idx, uint32_t vs) const {
        uint32_t s = seg, l = lo, h = hi;
        uint64_t b = base;
        while (idx >= h && s + 1 < nseg) {
            s++;
            l = h;
            h = gld<uint32_t>(pre + s + 1);
            b = gld<uint64_t>(ptrs + s);
        }
        return (const uint8_t *)(uintptr_t)b + (size_t)(idx - l) * vs;
    }
};

// Copy `count` staged values (source and destination pointers in LDS), 16
// bytes per lane: eight loads in flight per lane before their stores (a
// load-store loop keeps one, and is latency-bound).
__device__ __forceinline__ void copy_staged(const uint64_t *src, const uint64_t *dst, uint32_t count,
                                            uint32_t cpv_log) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t total = count << cpv_log;
    const uint32_t qmask = (1u << cpv_log) - 1;
    for (uint32_t c0 = 0; c0 < total; c0 += 64 * 8) {
        u32x4 v[8];
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
            const uint32_t c = c0 + lane + 64 * u;
            if (c < total) v[u] = gld<u32x4>((const uint8_t *)(uintptr_t)src[c >> cpv_log] + 16 * (c & qmask));
        }
#pragma unroll
        for (uint32_t u = 0; u < 8; u++) {
            const uint32_t c = c0 + lane + 64 * u;
            if (c < total) gst<u32x4>((uint8_t *)(uintptr_t)dst[c >> cpv_log] + 16 * (c & qmask), v[u]);
        }
    }
}

__device__ inline const JobDesc &job_of_result(const JobDesc *jobs, int njobs, uint32_t job_index) {
    int found = 0;
    for (int k = 0; k < njobs; k++)
        if (jobs[k].job_index == job_index) found = k;
    return jobs[found];
}

// Find the job owning global index `g` given a per-job base field (ascending).
template <class F>
__device__ inline int find_job(const JobDesc *jobs, int njobs, uint32_t g, F base_of) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (base_of(jobs[mid]) <= g) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

} // namespace tbc

// Kernel launchers (implemented in the .hip translation units).
struct hipStream_t_;
namespace tbc {
// The mask merge of every job of a batch: merge-path splits, survivor and
// side masks per tile, then the tile offsets and each job's output shape.
int launch_merge(const JobDesc *d_jobs, const JobDesc *h_jobs, int njobs, SplitDesc *d_splits,
                 uint64_t *d_status, uint64_t *d_masks, uint32_t *d_block_tile, const TileRef *d_order,
                 JobResultDev *d_results, void *stream, void (*mark)(void *, const char *), void *mark_ctx,
                 uint32_t phase = 0);
// Merge-path splits at the data-block boundaries of speculated jobs
// (d_bsplits[dblock_base + k] for block k) and their results (every value
// survives).
int launch_partition_blocks(const JobDesc *d_jobs, int njobs, uint32_t total_dblocks, SplitDesc *d_bsplits,
                            JobResultDev *d_results, void *stream);
// Pipelined speculated batches: merge-path splits every kUniqueTile merged
// positions of every speculated job plus its speculative results, then ONE
// merge of each tile writing every value straight to its output slot (every
// value survives) with the speculation checks (a broken job is marked for
// the recomputation phase).
// A pinned host buffer to device memory by a compute kernel on `stream`
// (grid.hip k_upload).
// zero_bytes at `zero` are cleared by the same launch (a batch's zeroed
// scratch: one kernel instead of an upload and a fill).
int launch_upload(void *dst, const void *host_src, uint64_t bytes, void *stream, void *zero = nullptr,
                  uint64_t zero_bytes = 0);
int launch_merge_unique(const JobDesc *d_jobs, const JobDesc *h_jobs, int njobs, SplitDesc *d_usplits,
                        JobResultDev *d_results, uint32_t *d_ticket, void *stream, void (*mark)(void *, const char *),
                        void *mark_ctx, void *part_stream = nullptr, void *part_done = nullptr);
int launch_blocks(const JobDesc *d_jobs, int njobs, uint32_t total_tiles, uint32_t total_dblocks, uint32_t total_tables,
                  uint32_t *d_ready,
                  JobResultDev *d_results, uint8_t *d_infos, const uint64_t *d_status, const uint64_t *d_masks,
                  const uint32_t *d_block_tile, const SplitDesc *d_splits, bool values_only, bool maybe_sparse,
                  void *stream,
                  void (*mark)(void *, const char *), void *mark_ctx, bool bodies_done = false,
                  const SplitDesc *d_bsplits = nullptr, uint32_t phase = 0, bool index_blocks = true);
int launch_validate_blocks(const uint64_t *d_ptrs, const uint64_t *d_expect, uint32_t count, uint32_t block_size,
                          uint8_t *d_out, void *stream);
// Grid inputs of a batch (engine.hip): resolve data blocks from the index
// blocks, header checks of every input block (cheap), the full
// read_block_validate of the unverified ones (side stream), and marking the
// outputs as trusted.
int launch_grid_resolve(const ResolveItem *d_items, uint32_t count, uint64_t *d_seg_ptr, InputCheck *d_checks,
                        const uint8_t *grid_base, uint64_t grid_blocks, uint32_t block_size, JobResultDev *d_results,
                        void *stream);
int launch_grid_expect(const ResolveItem *d_items, uint32_t count, InputCheck *d_checks, void *stream);
int launch_blocks_front(const JobDesc *d_jobs, int njobs, uint32_t total_tiles, uint32_t total_dblocks,
                        uint32_t *d_ready, const JobResultDev *d_results, const uint64_t *d_status,
                        const uint64_t *d_masks, const SplitDesc *d_splits, void *stream,
                        void (*mark)(void *, const char *), void *mark_ctx, bool bodies_done);
// Tail pairing (engine.hip grid_tail_pair): one batch's half of a paired
// tail launch.
struct TailHalf {
    const JobDesc *jobs;
    int njobs;
    uint32_t dblocks, tables;
    JobResultDev *res;
    uint8_t *infos;
    const uint32_t *ready;
};
struct ChainHalf { // k_data_blocks_pair's kernel argument
    const JobDesc *jobs;
    int njobs;
    uint32_t total;
    const JobResultDev *res;
    const uint32_t *ready;
    uint32_t c, wgs; // chain waves per workgroup, workgroups
};
int launch_blocks_tail_pair(const TailHalf &a, const TailHalf &b, void *stream, void (*mark)(void *, const char *),
                            void *ctx_a, void *ctx_b, bool compact = false);
int launch_blocks_tail(const JobDesc *d_jobs, int njobs, uint32_t total_dblocks, uint32_t total_tables,
                       JobResultDev *d_results, uint8_t *d_infos, const uint64_t *d_status, const uint64_t *d_masks,
                       const uint32_t *d_block_tile, const SplitDesc *d_splits, const uint32_t *d_ready,
                       void *stream, void (*mark)(void *, const char *), void *mark_ctx, bool compact = false);
int launch_index_blocks(const JobDesc *d_jobs, int njobs, uint32_t total_tables, JobResultDev *d_results,
                        uint8_t *d_infos, void *stream);
// tbc_compaction_seal (one seal job): chains + headers of its data blocks and
// their index entries, then its index blocks from the entries in place.
int launch_seal(const JobDesc *d_job, uint32_t blocks, uint32_t tables, JobResultDev *d_results, uint8_t *d_infos,
                void *stream);
// The bodies of the jobs the merge decided (k_assemble; phase 0 / 1 as
// phase_skips).
int launch_assemble(const JobDesc *d_jobs, int njobs, uint32_t total_tiles, uint32_t *d_ready,
                    const JobResultDev *d_results, const uint64_t *d_status, const uint64_t *d_masks,
                    const SplitDesc *d_bsplits, uint32_t phase, void *stream);
int launch_grid_checks(const InputCheck *d_checks, uint32_t count, const uint8_t *d_verified, const JobDesc *d_jobs,
                       int njobs, JobResultDev *d_results, uint32_t block_size, void *stream);
int launch_grid_validate(const InputCheck *d_checks, uint32_t count, uint8_t *d_verified, const JobDesc *d_jobs,
                         int njobs, JobResultDev *d_results, uint32_t block_size, void *stream);
int launch_grid_mark(const JobDesc *d_jobs, int njobs, uint8_t *d_verified, const JobResultDev *d_results,
                     void *stream);
// The chain-wave count above which a batch is in the throughput regime
// (aegis.hip).
uint32_t fused_max_chain_waves();
// ManifestLog.close_block of `count` staged manifest blocks (grid addresses in
// d_addresses): body checksums, then the header chain in order.
// previous_address (with no d_previous_checksum) must name a verified manifest
// block of the grid; otherwise the new blocks' header checksums are left
// zero (every later read fails validation), they are marked unverified and
// *d_error is set. Closed blocks are marked verified by the chain kernel itself.
int launch_manifest_close(const uint64_t *d_addresses, uint32_t count, uint8_t *grid_base, uint32_t block_size,
                          uint64_t previous_address, const uint64_t *d_previous_checksum, uint8_t *d_verified,
                          uint32_t *d_error, void *stream);
// The grid's `verified` byte of every listed block set to `value` (one launch).
int launch_grid_set_verified(const uint64_t *d_addresses, uint32_t count, uint8_t *d_verified, uint8_t value,
                             void *stream);
int launch_checksum_batch(const uint64_t *d_ptrs, const uint64_t *d_lens, uint32_t count, uint8_t *d_out,
                          void *stream);
// One copy of tbc_copy_device_batch: chunks [chunk0, chunk0 + ceil(bytes / copy_chunk_bytes())).
struct CopyItem {
    void *dst;
    const void *src;
    uint64_t bytes;
    uint32_t chunk0, pad;
};
int launch_copy_batch(const CopyItem *d_items, uint32_t count, uint32_t chunks, void *stream);
uint64_t copy_chunk_bytes();
struct SortItem {
    void *values;
    uint32_t n, value_size, timestamp_offset, key_kind;
    void *out; // null: sorted in place; else the sorted values go here and `values` is only read
};
// Enqueues the whole sort of a batch of memtables (no host wait); `host` is
// pinned staging of sort_host_bytes() that must outlive the enqueued copy.
int launch_sort_batch(const SortItem *items, uint32_t count, void *scratch, uint64_t scratch_bytes, uint64_t *status,
                      uint64_t status_words, uint32_t *epoch, void *host, void *stream);
uint64_t sort_scratch_bytes(const SortItem *items, uint32_t count);
uint64_t sort_status_words(const SortItem *items, uint32_t count);
uint64_t sort_host_bytes(const SortItem *items, uint32_t count);
// One level of the pairwise k-way merge tree (kway.hip): d_pairs holds
// npairs KPair descriptors (kway_pair_bytes() each), slots = sum(tiles_cap + 1),
// tiles = sum(tiles_cap) with tiles of kway_pair_tile() merged positions.
int launch_kway_level(uint32_t key_kind, bool descending, const void *d_pairs, uint32_t npairs, uint32_t slots,
                      uint32_t tiles, uint32_t vs, uint32_t ts, uint32_t *splits, uint64_t *masks, uint32_t *tile_cnt,
                      uint32_t *tile_off, void *stream);
uint32_t kway_pair_tile();
uint32_t kway_pair_bytes();
} // namespace tbc
