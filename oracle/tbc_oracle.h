/*
 * tbc_oracle.h — CPU restatement of TigerBeetle's LSM compaction hot path.
 *
 * TEST INFRASTRUCTURE ONLY. This library is the parity checker and the CPU
 * baseline ("port") for the GPU compaction engine in tigerbeetle_amd/. Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 * The product path (libtbc.so) never links, loads or calls it.
 *
 * Parity pinning: the AEGIS-128L checksum is pinned against the reference's own
 * known-answer tests (src/vsr/checksum.zig:94-112 test vectors and the
 * :146-195 "checksum stability" hash over 896 cases). Merge / block layout
 * bytes are pinned structurally (the reference has no golden block bytes; see
 * SURVEY.md §8c) — every function cites the reference lines it restates.
 *
 * Single-threaded and allocation-light, like the reference's event loop
 * (src/storage.zig:108-131).
 */
#ifndef TBC_ORACLE_H
#define TBC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- AEGIS-128L checksum (src/vsr/checksum.zig:38-85) ------------------ */

/* 1 if the AES-NI path is used by tbo_checksum (runtime CPU dispatch). */
int tbo_has_aesni(void);
/* Force the portable (T-table) AES path even when AES-NI exists. */
void tbo_force_portable(int on);
/* checksum(source) -> u128 written little-endian into out[16]. */
void tbo_checksum(const void *source, uint64_t len, uint8_t out[16]);
/* The AEGIS state after init with key=0, nonce=0 (8 AES blocks, 128 B).
 * The GPU kernels start from this seed (checksum.zig:40-46 seed_state). */
void tbo_aegis_seed_state(uint8_t out[128]);

/* ---- Tree layout (table.zig:107-129, schema.zig:119-157,293-314) -------- */

enum {
    TBO_KEY_TIMESTAMP = 0,      /* object trees: u64 key = timestamp & ~bit63 */
    TBO_KEY_ID_U128 = 1,        /* IdTreeValue{id u128, timestamp u64, pad u64} */
    TBO_KEY_COMPOSITE_U64 = 2,  /* CompositeKey(u64){field u64, timestamp u64} */
    TBO_KEY_COMPOSITE_U128 = 3, /* CompositeKey(u128){field u128, ts u64, pad u64} */
};
enum { TBO_USAGE_GENERAL = 0, TBO_USAGE_SECONDARY_INDEX = 1 };

typedef struct tbo_tree {
    uint16_t tree_id;
    uint8_t key_kind;
    uint8_t usage;
    uint32_t value_size;
    uint32_t timestamp_offset; /* byte offset of the u64 timestamp in Value */
    uint32_t key_size;         /* @sizeOf(Key): 8, 16 or 32 */
    uint32_t block_size;
    uint32_t block_value_count_max;
    uint32_t data_block_count_max;
    uint32_t value_count_max; /* per table */
    /* TableIndex layout (schema.zig:119-157) */
    uint32_t index_size;
    uint32_t index_checksums_offset;
    uint32_t index_keys_min_offset;
    uint32_t index_keys_max_offset;
    uint32_t index_addresses_offset;
} tbo_tree;

/* Returns 0 on success. */
int tbo_tree_init(tbo_tree *tree, uint16_t tree_id, uint8_t key_kind, uint8_t usage,
                  uint32_t value_size, uint32_t timestamp_offset,
                  uint32_t table_value_count_max, uint32_t block_size);

/* key_from_value as 4 little-endian u64 limbs (limb[0] least significant). */
void tbo_key(const tbo_tree *tree, const uint8_t *value, uint64_t limbs[4]);
int tbo_tombstone(const tbo_tree *tree, const uint8_t *value);

/* ---- TableMemory.sort (table_memory.zig:140-154) ------------------------ */
/* Stable ascending sort of n values by key (std.mem.sort is a stable block
 * sort in Zig 0.11). scratch must hold n*value_size bytes (may be NULL:
 * allocated internally). */
int tbo_sort_values(const tbo_tree *tree, uint8_t *values, uint32_t n);

/* ---- Compaction (compaction.zig:280-985, table.zig:242-457) ------------- */

typedef struct tbo_segment {
    const uint8_t *values; /* values of one input data block (or the whole immutable table) */
    uint32_t count;
} tbo_segment;

typedef struct tbo_job {
    const tbo_tree *tree;
    int a_immutable; /* 1: A = sorted immutable table memory (one segment); 0: A = disk table blocks */
    const tbo_segment *segments_a;
    uint32_t segment_count_a;
    const tbo_segment *segments_b; /* level-B tables' data blocks, ascending */
    uint32_t segment_count_b;
    int drop_tombstones;
    uint8_t level_b;
    uint64_t cluster_lo, cluster_hi;
    uint64_t snapshot_min; /* snapshot_min_for_table_output(op_min) */
    const uint64_t *addresses; /* grid.acquire() sequence within the reservation */
    uint32_t address_count;
    uint8_t *out_blocks; /* block_size bytes per block, in acquire order */
    uint32_t out_block_capacity;
    uint8_t *out_table_infos; /* 128 B ManifestNode.TableInfo per output table */
    uint32_t out_table_capacity;
    /* results */
    uint64_t out_value_count;
    uint32_t out_data_block_count;
    uint32_t out_table_count;
    uint32_t out_block_count;
} tbo_job;

enum {
    TBO_OK = 0,
    TBO_ERR_INVALID = 1,
    TBO_ERR_CAPACITY = 2,
    TBO_ERR_INVARIANT = 3, /* a reference assert would fire */
};

int tbo_compact(tbo_job *job);

/* vsr.sector_ceil (vsr.zig:905-908) with sector_size = 4096. */
uint64_t tbo_sector_ceil(uint64_t offset);

#ifdef __cplusplus
}
#endif
#endif
