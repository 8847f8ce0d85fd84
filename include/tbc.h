/*
 * tbc.h — C ABI of the MI355X-native LSM compaction engine for TigerBeetle's
 * forest ("tbc" = TigerBeetle compaction).
 *
 * This is the drop-in boundary a Zig host adapter `@cImport`s. It replaces
 * the data-parallel internals of the reference's comptime-generic
 * `CompactionType(Table, Tree, Storage)` (src/lsm/compaction.zig:56-60) and
 * `TableMemoryType.sort` (src/lsm/table_memory.zig:140-154) while the
 * `Tree`/`Compaction` surface the grooves use stays unchanged
 * (see INTEGRATION.md for the adapter and the binding stub).
 *
 * Conventions (following the only existing C ABI of the reference,
 * src/clients/c/tb_client.h:170-240):
 *   - plain pointers and sizes, no C++ types, every call returns tbc_status;
 *   - all device memory is either allocated through tbc_device_alloc or is a
 *     HIP device pointer owned by the caller;
 *   - nothing blocks except the explicitly synchronous calls (documented);
 *     compaction batches are submitted and then polled from the host event
 *     loop (the reference is single-threaded and never blocks:
 *     src/storage.zig:108-131).
 */
#ifndef TBC_H
#define TBC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TBC_ABI_VERSION 7u

typedef enum tbc_status {
    TBC_OK = 0,
    TBC_PENDING = 1,              /* batch still running on the device */
    TBC_ERR_INVALID_ARGUMENT = 2, /* a reference comptime/assert precondition is violated */
    TBC_ERR_DEVICE = 3,           /* HIP runtime error (or no device) */
    TBC_ERR_OUT_OF_MEMORY = 4,    /* static arena exhausted (reference panics: compaction.zig:307-318) */
    TBC_ERR_CAPACITY = 5,         /* address list / output too small for the worst case */
    TBC_ERR_INVARIANT = 6,        /* an input broke a reference invariant (e.g. unsorted table) */
    TBC_ERR_BLOCK_INVALID = 7,    /* a grid input block failed read_block_from_cache's checks or
                                     read_block_validate (grid.zig:802-841, 1059-1084) */
} tbc_status;

/* Key of a tree's Value (src/lsm/groove.zig:22-76, src/lsm/composite_key.zig:7-70). */
typedef enum tbc_key_kind {
    TBC_KEY_TIMESTAMP = 0,      /* object tree: u64 key = timestamp & ~(1<<63) */
    TBC_KEY_ID_U128 = 1,        /* IdTreeValue{id: u128, timestamp: u64, padding: u64} */
    TBC_KEY_COMPOSITE_U64 = 2,  /* CompositeKey(u64){field: u64, timestamp: u64}, Key = u128 */
    TBC_KEY_COMPOSITE_U128 = 3, /* CompositeKey(u128){field: u128, timestamp: u64, pad: u64}, Key = u256 */
} tbc_key_kind;

/* TableUsage (src/lsm/table.zig:18-32). */
typedef enum tbc_usage {
    TBC_USAGE_GENERAL = 0,
    TBC_USAGE_SECONDARY_INDEX = 1,
} tbc_usage;

/* The comptime parameters of one `TableType` (src/lsm/table.zig:47-62). The
 * derived layout (block_value_count_max, data_block_count_max, index layout)
 * is computed exactly as table.zig:107-129 / schema.zig:119-157 do. */
typedef struct tbc_tree {
    uint16_t tree_id;  /* StateMachine.constants.tree_ids (src/state_machine.zig:78-111) */
    uint8_t key_kind;  /* tbc_key_kind */
    uint8_t usage;     /* tbc_usage */
    uint32_t value_size;            /* @sizeOf(Value): 16, 32, 128 or 256 */
    uint32_t timestamp_offset;      /* byte offset of the u64 timestamp (tombstone bit 63) */
    uint32_t table_value_count_max; /* Table.value_count_max */
} tbc_tree;

/* Derived layout, as reported by tbc_tree_layout_get(). */
typedef struct tbc_tree_layout {
    uint32_t key_size;              /* @sizeOf(Key) */
    uint32_t block_value_count_max; /* table.zig:116-119 */
    uint32_t data_block_count_max;  /* table.zig:122 */
    uint32_t index_size;            /* schema.zig:139-140 */
    uint32_t index_checksums_offset;
    uint32_t index_keys_min_offset;
    uint32_t index_keys_max_offset;
    uint32_t index_addresses_offset;
} tbc_tree_layout;

typedef struct tbc_config {
    int32_t device;        /* HIP device ordinal */
    uint32_t block_size;   /* constants.block_size (config.zig:139): 1 MiB prod, 4 KiB test_min */
    uint64_t arena_bytes;  /* static device scratch arena; 0 = default (256 MiB) */
    uint32_t flags;        /* TBC_CONFIG_* */
    uint32_t reserved;
} tbc_config;

#define TBC_CONFIG_PROFILE 1u /* record hipEvents around every kernel (tbc_batch_kernel_times) */
/* Block pass of TBC_COMPACTION_UNIQUE_KEYS batches. By default a batch
 * submitted while an earlier batch's tail is still running is pipelined (its
 * bodies merged on the engine stream, its AEGIS chains on a tail stream
 * beside other batches' chains: throughput), and a batch submitted alone
 * takes the fused pass (every chain at once, bodies built beside them:
 * latency). PIPELINE / LATENCY force one or the other. */
#define TBC_CONFIG_PIPELINE 2u
#define TBC_CONFIG_LATENCY 4u

typedef struct tbc_engine tbc_engine;
typedef struct tbc_batch tbc_batch;

/* One input data block's values (device pointer), or a whole immutable table. */
typedef struct tbc_segment {
    const void *values; /* device pointer, 16-byte aligned */
    uint32_t count;     /* number of values */
    uint32_t reserved;
} tbc_segment;

/* tbc_compaction.flags. VALUES_ONLY: the survivors only — data-block bodies
 * (values at +256 of each data-block slot) and the result counts; no headers,
 * checksums, index blocks or TableInfos. Phase 1 of a job split by key range
 * across GPUs (tigerbeetle_amd/split.py); every job of a batch must agree.
 * GRID: inputs and outputs live in a tbc_grid, see below: disk tables are
 * named by table reference (tables_a / tables_b; an immutable A still comes
 * as one segment), their data blocks are found through their index blocks
 * on the device, and every output block is written to the grid at its
 * acquired address (segments_b and output_blocks are ignored). */
#define TBC_COMPACTION_VALUES_ONLY 1u
#define TBC_COMPACTION_GRID 2u
/* UNIQUE_KEYS (per compaction, may differ within a batch): the caller expects
 * no key to occur twice in A u B and no tombstone to be dropped — true by
 * construction for trees whose keys are never updated or removed (the id
 * trees, the object and index trees of immutable objects such as Transfers).
 * Then every value survives, every output block's contents are known before
 * any merge, and the engine starts all AEGIS chains at once, producers
 * merging each block's values as its chain absorbs them (no merge pass in
 * front). The expectation is verified on the device; a compaction that
 * breaks it is recomputed through the ordinary merge path in the same batch
 * (identical results, slower; tbc_batch_speculation reports it). Honoured in
 * the latency regime of a plain batch (no GRID / VALUES_ONLY, few enough
 * output blocks that every chain runs at once); ignored elsewhere. */
#define TBC_COMPACTION_UNIQUE_KEYS 4u
/* COUNT_ONLY: the merge alone (survivor rules included); the result's
 * value_count is the number of survivors and nothing is written
 * (output_blocks may be NULL; if not, the count is also stored there as a
 * u64 on the device, in engine-stream order, for a caller that exchanges it
 * without a host wait). Phase A of a job split by key range
 * (tbc_compaction.output_offset, tbc_compaction_seal). */
#define TBC_COMPACTION_COUNT_ONLY 8u

/* ---- GPU-resident grid (src/vsr/grid.zig, src/lsm/set_associative_cache.zig) ----
 * The blocks of the data file's grid zone for addresses [1, block_count],
 * resident in HBM (block `address` at slot address - 1; one MI355X holds
 * ~270k 1 MiB blocks). A compaction's output blocks stay there and are the
 * next compaction's inputs with no PCIe round trip. Blocks written by the
 * engine are trusted like grid cache hits (read_block_from_cache compares
 * the header checksum with the expected one, grid.zig:802-841); blocks staged
 * from storage are fully validated (read_block_validate: header and body
 * AEGIS, grid.zig:1059-1084) by the first batch that reads them, on a second
 * stream concurrently with its compaction. */
typedef struct tbc_grid tbc_grid;

/* A disk table as Compaction.Context names it (TableInfoReference,
 * compaction.zig:84-99; manifest TableInfo, schema.zig:489-509): its index
 * block's address and checksum, and its value count (every data block of a
 * table is full except the last, compaction.zig:806-850). */
typedef struct tbc_table_ref {
    uint64_t address;     /* index block address */
    uint64_t checksum[2]; /* index block checksum, u128 little-endian words */
    uint64_t value_count;
} tbc_table_ref;

/* One `Compaction.start(Context)` (src/lsm/compaction.zig:84-99, 280-404). */
typedef struct tbc_compaction {
    tbc_tree tree;
    uint8_t a_immutable;     /* 1: table_info_a = .immutable (sorted TableMemory values, one segment) */
    uint8_t drop_tombstones; /* Manifest.compaction_must_drop_tombstones (manifest.zig:547-574) */
    uint8_t level_b;         /* Context.level_b (manifest label of the output tables) */
    uint8_t flags;           /* TBC_COMPACTION_* (0 for a reference compaction) */
    uint32_t reserved1;
    const tbc_segment *segments_a; /* host array; A's data blocks in key order (or 1 immutable segment) */
    uint32_t segment_count_a;
    uint32_t segment_count_b;
    const tbc_segment *segments_b; /* host array; level-B tables' data blocks, ascending range_b order */
    uint64_t cluster[2];           /* superblock.working.cluster (u128, little-endian words) */
    uint64_t snapshot_min;         /* snapshot_min_for_table_output(op_min) (compaction.zig:981-985) */
    const uint64_t *addresses;     /* host array: grid.acquire() sequence of the reservation */
    uint32_t address_count;        /* >= (|B tables| + 1) * block_count_max, the reservation size */
    uint32_t reserved2;
    void *output_blocks;           /* device: address_count * block_size bytes; block i <-> addresses[i] */
    /* TBC_COMPACTION_GRID only: */
    tbc_grid *grid;
    const tbc_table_ref *tables_a; /* host array: table_info_a.disk (0 or 1 table; none if immutable) */
    const tbc_table_ref *tables_b; /* host array: range_b.tables in ascending key order */
    uint32_t table_count_a;
    uint32_t table_count_b;
    /* VALUES_ONLY only (0 otherwise): this compaction is one key range of a
     * job split across GPUs, preceded in the job's merged output by
     * output_offset survivors of the other ranges. Survivor i is written at
     * the job's output position output_offset + i: data block
     * k = position / block_value_count_max, slot k + k / data_block_count_max
     * of output_blocks (the whole job's acquire order), so every rank builds
     * its part of the job's blocks in place (tbc_compaction_seal). */
    uint64_t output_offset;
} tbc_compaction;

/* ---- sealing a job split by key range -----------------------
 * The blocks of ONE job whose survivors were written in place across ranks
 * (VALUES_ONLY + output_offset; a straddling data block's values gathered by
 * its owner): data blocks [block_first, block_first + block_count) get their
 * headers and checksums (data_block_finish, table.zig:306-384) and their
 * index entries (checksum, key_min, key_max, address) written into their
 * table's index block slot; then the index blocks of tables
 * [table_first, table_first + table_count) are sealed from the entries found
 * in their slots (index_block_finish, table.zig:403-457: every entry of such
 * a table must be in place, written by this engine or copied in from the
 * rank that finished that block) with one TableInfo each (level_b).
 * value_count is the whole job's survivor count: it fixes every block and
 * table boundary. One batch on the engine stream; tbc_batch_result(0)
 * reports the data blocks and tables of this call and its TableInfos. */
typedef struct tbc_seal {
    tbc_tree tree;
    uint64_t cluster[2];
    uint64_t snapshot_min;
    uint8_t level_b;
    uint8_t reserved[3];
    uint32_t address_count;    /* the job's acquire order (all of it) */
    const uint64_t *addresses; /* host array */
    void *output_blocks;       /* device: the job's output blocks, address_count * block_size bytes */
    uint64_t value_count;      /* survivors of the whole job */
    uint32_t block_first, block_count;
    uint32_t table_first, table_count;
} tbc_seal;

/* Per-compaction result (after tbc_batch_poll returned TBC_OK). */
typedef struct tbc_compaction_result {
    uint64_t value_count;      /* values written across all output tables */
    uint32_t data_block_count; /* data blocks written */
    uint32_t table_count;      /* output tables (one index block each) */
    uint32_t block_count;      /* data + index blocks = addresses consumed, in acquire order */
    uint32_t status;           /* tbc_status of this compaction */
} tbc_compaction_result;

/* ---- engine ---------------------------------------------------------------- */
uint32_t tbc_abi_version(void);
tbc_status tbc_engine_init(const tbc_config *config, tbc_engine **out_engine);
void tbc_engine_deinit(tbc_engine *engine);
tbc_status tbc_tree_layout_get(const tbc_engine *engine, const tbc_tree *tree, tbc_tree_layout *out_layout);
/* Diagnostics: bytes of the static device and pinned host arenas held by
 * submitted batches and k-way merges not yet released, and how many of them.
 * Released handles give their region back (out of order too, once the
 * regions above it are released), so a steady-state caller sees these bounded. */
tbc_status tbc_engine_arena_usage(const tbc_engine *engine, uint64_t *out_device_bytes, uint64_t *out_host_bytes,
                                  uint32_t *out_regions);

/* ---- grid ------------------------------------------------------------------- */
tbc_status tbc_grid_init(tbc_engine *engine, uint64_t block_count, tbc_grid **out_grid);
void tbc_grid_deinit(tbc_grid *grid);
/* A replica restart (superblock open from a checkpoint): the grid's cache is
 * cold, so every block is untrusted until a batch that reads it validates it
 * in full (read_block_validate). Enqueued after every running batch tail. */
tbc_status tbc_grid_invalidate(tbc_grid *grid);
/* Device pointer of the block at `address` (1 <= address <= block_count). */
tbc_status tbc_grid_block_pointer(const tbc_grid *grid, uint64_t address, void **out_ptr);
/* grid.read_block from storage: stage `count` host block images (block_size
 * bytes each, the on-disk image [0, sector_ceil(size)) is what matters) into
 * the grid, enqueued on the engine stream (no host wait beyond the pinned
 * staging copy; images in a range registered with tbc_host_register are
 * copied by DMA, and the call waits for those copies, so every host buffer
 * may be reused as soon as it returns). The blocks are marked unverified
 * (before any image lands) until a batch validates them. */
tbc_status tbc_grid_put_blocks(tbc_grid *grid, const uint64_t *addresses, const void *const *host_blocks,
                               uint32_t count);
/* grid.write_block towards storage: copy `count` blocks' images
 * [0, block_size) to host buffers; returns once the buffers hold them. Waits
 * (on the device) for every batch tail enqueued so far. Buffers inside a
 * range registered with tbc_host_register are written by DMA directly; others
 * go through the pinned staging ring with every slot in flight. */
tbc_status tbc_grid_get_blocks(tbc_grid *grid, const uint64_t *addresses, void *const *host_blocks,
                               uint32_t count);

/* ---- ManifestLog.close_block (src/lsm/manifest_log.zig:876-952) ----------------
 * Close `count` manifest blocks of the log, oldest first, into the grid at
 * `addresses` (ManifestLog.acquire_block's grid.acquire, one each). The host
 * packs each block image as the reference's append/close_block do (header:
 * cluster, size = 256 + 128 * entry_count, command block, metadata
 * {previous checksum left 0, previous address, entry_count}, address,
 * block_type manifest; body: the 128-byte TableInfo entries; zero padding to
 * the sector); the engine stages the images into their grid slots and, on
 * the device, sets every block's checksum_body, its metadata's previous
 * checksum (block i links block i-1; block 0 links `previous_checksum`, or,
 * when that is NULL, the header checksum of the block at `previous_address`
 * in the grid — an earlier close — or 0 when previous_address is 0) and its
 * header checksum. Enqueued on the engine stream; no host wait beyond the
 * pinned staging copies. The blocks are trusted grid blocks afterwards. When
 * `previous_checksum` is NULL, the block at `previous_address` must be a
 * verified manifest block of this grid (closed by an earlier call); if it is
 * not, nothing is linked: the new blocks keep a zero header checksum (every
 * later read fails validation), are marked unverified, and the grid's next
 * tbc_manifest_close_status returns TBC_ERR_BLOCK_INVALID (the device found
 * it after this call returned).
 * TBC_ERR_INVALID_ARGUMENT if a packed header contradicts its address, the
 * chain or ManifestNode.metadata's asserts (schema.zig:534-554). */
tbc_status tbc_manifest_close_blocks(tbc_grid *grid, const uint64_t *addresses, const void *const *host_images,
                                     uint32_t count, uint64_t previous_address, const uint64_t *previous_checksum);
/* Outcome of the grid's manifest closes enqueued so far (the log's
 * close_block callback, manifest_log.zig:903-952): waits for them, then
 * TBC_ERR_BLOCK_INVALID once if any refused to link since the last call,
 * TBC_OK otherwise. Only this call reports (and clears) a refusal. */
tbc_status tbc_manifest_close_status(tbc_grid *grid);

/* ---- TableMemory on the device (src/lsm/table_memory.zig:79-124) ------------
 * Groove.insert/update -> Tree.put (groove.zig:911-1006, tree.zig:268-270)
 * append values to the mutable table; here the appends stream into device
 * memory through pinned staging (host memcpy + async H2D on the engine
 * stream), so the bar-end sort (tbc_sort_values_batch) and the immutable
 * table's compaction read it in place: no H2D step at the bar end. */
typedef struct tbc_memtable tbc_memtable;
tbc_status tbc_memtable_init(tbc_engine *engine, const tbc_tree *tree, uint32_t capacity, tbc_memtable **out);
void tbc_memtable_deinit(tbc_memtable *memtable);
/* TableMemory.put of `count` values (host memory, value_size bytes each):
 * TBC_ERR_CAPACITY past value_count_max (the reference asserts). */
tbc_status tbc_memtable_put(tbc_memtable *memtable, const void *values, uint32_t count);
/* Device pointer and value count (for sort jobs and immutable compactions). */
tbc_status tbc_memtable_values(const tbc_memtable *memtable, void **out_values, uint32_t *out_count);
/* make_mutable: empty the table (after its immutable compaction flushed it). */
tbc_status tbc_memtable_reset(tbc_memtable *memtable);
/* Bar end of a forest (Tree.swap_mutable_and_immutable + TableMemory.make_immutable,
 * tree.zig:979-999, table_memory.zig:110-154), for every pair at once: the
 * values put into mutables[i] become immutables[i]'s, in key order, and
 * mutables[i] is emptied. immutables[i] must be empty (flushed, then
 * tbc_memtable_reset) and of the same tree and capacity. A table whose puts
 * arrived in key order (in_order[i] != 0, the reference's sorted flag,
 * table_memory.zig:83-87; in_order may be NULL) trades buffers with its
 * immutable table; the others are sorted by ONE segmented out-of-place sort
 * (tbc_sort_job.values_out) from the mutable buffers into the immutable
 * ones. Enqueued on the engine stream; later puts into the mutable tables
 * are ordered after the sort's reads. */
tbc_status tbc_memtable_make_immutable(tbc_engine *engine, tbc_memtable *const *mutables,
                                       tbc_memtable *const *immutables, const uint8_t *in_order, uint32_t count);

/* ---- registered host memory ------------------------------------------------
 * hipHostRegister of a caller range (TigerBeetle's I/O buffers are allocated
 * once at startup): tbc_grid_put_blocks / tbc_grid_get_blocks move blocks
 * from or into a registered range by DMA, without the staging ring's host
 * copy. Ranges must not overlap; unregister waits for enqueued work. */
tbc_status tbc_host_register(tbc_engine *engine, void *ptr, uint64_t bytes);
tbc_status tbc_host_unregister(tbc_engine *engine, void *ptr);

/* ---- device memory (staging for the host adapter; synchronous copies) ------ */
tbc_status tbc_device_alloc(tbc_engine *engine, uint64_t bytes, void **out_ptr);
tbc_status tbc_device_free(tbc_engine *engine, void *ptr);
tbc_status tbc_copy_to_device(tbc_engine *engine, void *dst, const void *src, uint64_t bytes);
tbc_status tbc_copy_to_host(tbc_engine *engine, void *dst, const void *src, uint64_t bytes);
/* Device-to-device copy enqueued on the engine stream (no host wait): e.g.
 * landing a bar's mutable table next to the sort that consumes it. */
tbc_status tbc_copy_device_async(tbc_engine *engine, void *dst, const void *src, uint64_t bytes);
/* Many device-to-device copies in ONE launch on the engine stream (no host
 * wait): e.g. landing every memtable of a bar at once. Copies whose
 * addresses and size are multiples of 16 bytes go to one kernel; any other
 * is a copy of its own, in order. The copies must not overlap each other. */
typedef struct tbc_copy {
    void *dst;
    const void *src;
    uint64_t bytes;
} tbc_copy;
tbc_status tbc_copy_device_batch(tbc_engine *engine, const tbc_copy *copies, uint32_t count);
tbc_status tbc_memset_device(tbc_engine *engine, void *dst, int value, uint64_t bytes);
/* The engine stream (a hipStream_t): work a caller orders with the engine's
 * (a collective over the split's exchange buffers, torch.cuda.ExternalStream)
 * goes on it. */
tbc_status tbc_engine_stream(tbc_engine *engine, void **out_stream);
/* Waits for every enqueued call. (A refused manifest close is reported by
 * tbc_manifest_close_status, not here.) Any call that launches work returns
 * TBC_ERR_DEVICE if a HIP error of an earlier call is still unreported. */
tbc_status tbc_synchronize(tbc_engine *engine);

/* ---- vsr.checksum (src/vsr/checksum.zig:50-59) ------------------------------ */
/* Synchronous batched AEGIS-128L checksums. messages/lengths are host arrays
 * of device pointers; each message buffer must be readable up to its length
 * rounded up to 4 bytes. Writes count * 16 bytes (u128 LE) to checksums_out (host). */
tbc_status tbc_checksum_batch(tbc_engine *engine, const void *const *messages, const uint64_t *lengths,
                              uint32_t count, uint8_t *checksums_out);

/* ---- grid.read_block_validate (src/vsr/grid.zig:1059-1084) ---------------------- */
/* Result per block, in the reference's check order. */
typedef enum tbc_block_check {
    TBC_BLOCK_VALID = 0,
    TBC_BLOCK_INVALID_CHECKSUM = 1,      /* header checksum (bytes [16, 256)) */
    TBC_BLOCK_UNEXPECTED_COMMAND = 2,    /* command != block (20) */
    TBC_BLOCK_INVALID_CHECKSUM_BODY = 3, /* body checksum (bytes [256, size)) */
    TBC_BLOCK_UNEXPECTED_CHECKSUM = 4,   /* header checksum != the expected (manifest/index) checksum */
    TBC_BLOCK_UNEXPECTED_ADDRESS = 5,    /* header address != the expected address (reference asserts) */
    TBC_BLOCK_INVALID_SIZE = 6,          /* size outside [256, block_size] (reference asserts) */
    TBC_BLOCK_UNEXPECTED_HEADER = 7,     /* grid input: cluster, block type, tree, value count or size
                                            differ from the table it was reached from (reference asserts) */
} tbc_block_check;
/* Synchronous batched validation of device-resident blocks (16-byte aligned
 * device pointers, block_size readable). expect_checksums: 2 u64 (u128 LE)
 * per block; expect_addresses: 1 u64 per block; results_out: count bytes. */
tbc_status tbc_blocks_validate(tbc_engine *engine, const void *const *blocks, const uint64_t *expect_checksums,
                               const uint64_t *expect_addresses, uint32_t count, uint8_t *results_out);

/* ---- TableMemory.sort (src/lsm/table_memory.zig:140-154) ---------------------- */
/* Synchronous stable ascending sort of `count` values (device memory) by key.
 * A no-op when the keys are already non-decreasing (table_memory.zig:83-87). */
tbc_status tbc_sort_values(tbc_engine *engine, const tbc_tree *tree, void *values, uint32_t count);
/* Asynchronous variant: enqueued on the engine stream ahead of later batches. */
tbc_status tbc_sort_values_async(tbc_engine *engine, const tbc_tree *tree, void *values, uint32_t count);

/* Bar end of a whole forest: every tree's mutable table sorted by ONE
 * segmented launch sequence (tree.zig:979-999 calls TableMemory.sort once per
 * tree; the batch is the same work without a launch train per tree). Same
 * semantics per table as tbc_sort_values; tables that are already sorted are
 * left untouched. Enqueued on the engine stream with no host wait: the digit
 * plan (which key bits vary, which passes run) is computed and read on the
 * device (sort.hip k_sort_layout / k_sort_plan). */
typedef struct tbc_sort_job {
    tbc_tree tree;
    void *values;   /* device pointer, 16-byte aligned */
    uint32_t count;
    uint32_t reserved;
    /* NULL: sorted in place. Otherwise the sorted values are written here
     * (device, 16-byte aligned, count * value_size bytes, not overlapping
     * `values`) and `values` is only read: the put-order values are read
     * once and written once, with no copy of the table (a table already in
     * order is copied as is). */
    void *values_out;
} tbc_sort_job;
tbc_status tbc_sort_values_batch(tbc_engine *engine, const tbc_sort_job *jobs, uint32_t count);

/* ---- scan path: k-way merge ------------------------------------------------
 * Replaces KWayMergeIteratorType(...).init + pop-until-null
 * (src/lsm/k_way_merge.zig:8-205) with stream_precedence(a, b) = a > b (the
 * reference's own tests, :239-244: a higher stream index wins on equal keys;
 * order streams oldest -> newest). Each stream holds `count` values (device,
 * 16-byte aligned) sorted by key_from_value in the merge direction, possibly
 * with repeated keys; the merged values (one per key: the first of the
 * winning stream's run) are written to `out_values` (device, capacity = the
 * streams' total). tbc_kway_merge_submit enqueues the merge and returns at
 * once (the scan's iterator polls it like a grid read, src/lsm/scan_tree.zig);
 * the merged count is read with tbc_kway_count once tbc_kway_poll returns
 * TBC_OK. tbc_kway_merge is the blocking form (tests, tools). */
#define TBC_KWAY_STREAMS_MAX 64u
typedef struct tbc_kway tbc_kway;
tbc_status tbc_kway_merge_submit(tbc_engine *engine, const tbc_tree *tree, const tbc_segment *streams,
                                 uint32_t stream_count, uint32_t descending, void *out_values, tbc_kway **out_merge);
tbc_status tbc_kway_poll(tbc_kway *merge);
tbc_status tbc_kway_wait(tbc_kway *merge);
tbc_status tbc_kway_count(const tbc_kway *merge, uint64_t *out_count);
void tbc_kway_release(tbc_kway *merge);
tbc_status tbc_kway_merge(tbc_engine *engine, const tbc_tree *tree, const tbc_segment *streams, uint32_t stream_count,
                          uint32_t descending, void *out_values, uint64_t *out_count);

/* ---- compaction ------------------------------------------------------------- */
/* Enqueue `count` independent compactions (one half-bar's jobs) as one batch.
 * All input/output device memory must stay valid until the batch completes.
 * Batches may be submitted without waiting for earlier ones: a batch whose
 * output blocks overlap those of an earlier batch still being checksummed
 * waits for it on the device; other batches run beside it. A batch's output
 * blocks may be read or overwritten by other calls (tbc_copy_to_host,
 * tbc_copy_device_async, tbc_memset_device, ...) only after tbc_batch_poll or
 * tbc_batch_wait has returned its result: parts of a batch (its chains,
 * index blocks and results) run on tail streams those calls do not wait for. */
tbc_status tbc_compaction_submit(tbc_engine *engine, const tbc_compaction *compactions, uint32_t count,
                                 tbc_batch **out_batch);
/* Non-blocking: TBC_PENDING while running, then TBC_OK or the first error. */
tbc_status tbc_batch_poll(tbc_batch *batch);
/* Enqueue the sealing of one split job's blocks (see tbc_seal above). */
tbc_status tbc_compaction_seal(tbc_engine *engine, const tbc_seal *seal, tbc_batch **out_batch);
/* Blocking wait (tests / benchmarks only; the adapter polls). */
tbc_status tbc_batch_wait(tbc_batch *batch);
/* Results of compaction `index`; table_infos receives table_count entries of
 * 128-byte schema.ManifestNode.TableInfo (src/lsm/schema.zig:489-509) encoded
 * for Manifest.insert_table at level_b (manifest.zig:233-255). */
tbc_status tbc_batch_result(tbc_batch *batch, uint32_t index, tbc_compaction_result *out_result,
                            uint8_t *table_infos, uint32_t table_info_capacity);
/* Outcome of TBC_COMPACTION_UNIQUE_KEYS for compaction `index` once the batch
 * is complete: TBC_SPECULATION_NONE (not speculated), _HELD (blocks written
 * by the speculative pass) or _BROKEN (a key repeated or a tombstone was
 * dropped: recomputed through the merge path, same results). */
#define TBC_SPECULATION_NONE 0u
#define TBC_SPECULATION_HELD 1u
#define TBC_SPECULATION_BROKEN 2u
tbc_status tbc_batch_speculation(tbc_batch *batch, uint32_t index, uint32_t *out_outcome);
/* TBC_CONFIG_PROFILE on (1) or off (0) for the batches submitted after this
 * call; a batch keeps what it was submitted with. The marks cost the engine
 * stream time (config 1: ~1.3 ms per 40 ms step), so a timed loop runs
 * without them and profiled steps follow it. */
tbc_status tbc_engine_set_profile(tbc_engine *engine, uint32_t on);
/* Per-kernel device times of the batch in microseconds (TBC_CONFIG_PROFILE).
 * names/us are host arrays of `capacity` entries; returns the entry count in *out_count. */
tbc_status tbc_batch_kernel_times(tbc_batch *batch, const char **names, double *us, uint32_t capacity,
                                  uint32_t *out_count);
void tbc_batch_release(tbc_batch *batch);

#ifdef __cplusplus
}
#endif
#endif /* TBC_H */
