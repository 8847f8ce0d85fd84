/*
 * tbc_oracle.c — CPU restatement of TigerBeetle's LSM compaction hot path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline). See tbc_oracle.h.
 *
 * Reference: /root/reference (TigerBeetle @ 2024-03, Zig 0.11.0). Each function
 * cites the lines it restates. AEGIS-128L follows Zig 0.11 std
 * `std.crypto.auth.aegis.Aegis128LMac_128` (third-party to the reference,
 * pinned by scripts/install_zig.sh:4; call site src/vsr/checksum.zig:38-85)
 * and is accepted only because it reproduces the reference KATs
 * (checksum.zig:94-112, :146-195) — see tests/test_oracle.py.
 */
#include "tbc_oracle.h"

#include <stdlib.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#include <cpuid.h>
#endif

/* ------------------------------------------------------------------------ */
/* Little-endian helpers                                                     */
/* ------------------------------------------------------------------------ */

static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline void wr64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static inline void wr16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }

/* ------------------------------------------------------------------------ */
/* AES round (portable T-tables and AES-NI)                                  */
/* ------------------------------------------------------------------------ */

static uint8_t sbox[256];
static uint32_t T0[256], T1[256], T2[256], T3[256];
static int tables_ready = 0;
static int use_aesni = -1;
static int force_portable = 0;

static inline uint8_t rotl8(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }
static inline uint8_t xtime(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1B : 0)); }

static void tables_init(void) {
    if (tables_ready) return;
    /* FIPS-197 S-box from the multiplicative inverse + affine map. */
    uint8_t p = 1, q = 1;
    do {
        p = (uint8_t)(p ^ (p << 1) ^ ((p & 0x80) ? 0x1B : 0));
        q ^= (uint8_t)(q << 1);
        q ^= (uint8_t)(q << 2);
        q ^= (uint8_t)(q << 4);
        if (q & 0x80) q ^= 0x09;
        uint8_t x = (uint8_t)(q ^ rotl8(q, 1) ^ rotl8(q, 2) ^ rotl8(q, 3) ^ rotl8(q, 4));
        sbox[p] = (uint8_t)(x ^ 0x63);
    } while (p != 1);
    sbox[0] = 0x63;
    for (int i = 0; i < 256; i++) {
        uint32_t s = sbox[i], s2 = xtime((uint8_t)s), s3 = s2 ^ s;
        /* Column as a little-endian dword: byte r = row r. */
        T0[i] = s2 | (s << 8) | (s << 16) | (s3 << 24);
        T1[i] = s3 | (s2 << 8) | (s << 16) | (s << 24);
        T2[i] = s | (s3 << 8) | (s2 << 16) | (s << 24);
        T3[i] = s | (s << 8) | (s3 << 16) | (s2 << 24);
    }
    tables_ready = 1;
}

/* AESENC(state, rk) = MixColumns(ShiftRows(SubBytes(state))) ^ rk, one AES
 * block as 4 little-endian column dwords. */
static inline void aesenc_portable(uint32_t out[4], const uint32_t in[4], const uint32_t rk[4]) {
    for (int c = 0; c < 4; c++) {
        out[c] = T0[in[c] & 0xff] ^ T1[(in[(c + 1) & 3] >> 8) & 0xff] ^
                 T2[(in[(c + 2) & 3] >> 16) & 0xff] ^ T3[in[(c + 3) & 3] >> 24] ^ rk[c];
    }
}

typedef struct { uint32_t s[8][4]; } aegis_state;

static const uint8_t AEGIS_C0[16] = {0x00, 0x01, 0x01, 0x02, 0x03, 0x05, 0x08, 0x0d,
                                     0x15, 0x22, 0x37, 0x59, 0x90, 0xe9, 0x79, 0x62};
static const uint8_t AEGIS_C1[16] = {0xdb, 0x3d, 0x18, 0x55, 0x6d, 0xc2, 0x2f, 0xf1,
                                     0x20, 0x11, 0x31, 0x42, 0x73, 0xb5, 0x28, 0xdd};

/* State128L.update(d1, d2): S[i] = AESENC(S[i-1], S[i]) for i=7..1,
 * S[0] = AESENC(S[7]_old, S[0]); S[0] ^= d1; S[4] ^= d2. */
static inline void aegis_update_portable(aegis_state *st, const uint32_t m0[4], const uint32_t m1[4]) {
    uint32_t tmp[4], n[4];
    memcpy(tmp, st->s[7], 16);
    for (int i = 7; i > 0; i--) {
        aesenc_portable(n, st->s[i - 1], st->s[i]);
        memcpy(st->s[i], n, 16);
    }
    aesenc_portable(n, tmp, st->s[0]);
    memcpy(st->s[0], n, 16);
    for (int c = 0; c < 4; c++) {
        st->s[0][c] ^= m0[c];
        st->s[4][c] ^= m1[c];
    }
}

static aegis_state seed_state;
static int seed_ready = 0;

/* Aegis128LMac_128.init(key = 0) (checksum.zig:43-46): nonce = 0, so the
 * initial blocks are [0, C1, C0, C1, 0, C0, C1, C0], then 10 updates(0, 0). */
static void seed_init(void) {
    if (seed_ready) return;
    tables_init();
    aegis_state st;
    memset(&st, 0, sizeof st);
    memcpy(st.s[1], AEGIS_C1, 16);
    memcpy(st.s[2], AEGIS_C0, 16);
    memcpy(st.s[3], AEGIS_C1, 16);
    memcpy(st.s[5], AEGIS_C0, 16);
    memcpy(st.s[6], AEGIS_C1, 16);
    memcpy(st.s[7], AEGIS_C0, 16);
    uint32_t zero[4] = {0, 0, 0, 0};
    for (int i = 0; i < 10; i++) aegis_update_portable(&st, zero, zero);
    seed_state = st;
    seed_ready = 1;
}

static void checksum_portable(const uint8_t *src, uint64_t len, uint8_t out[16]) {
    aegis_state st = seed_state;
    uint64_t full = len / 32;
    uint32_t m0[4], m1[4];
    for (uint64_t i = 0; i < full; i++) {
        memcpy(m0, src + 32 * i, 16);
        memcpy(m1, src + 32 * i + 16, 16);
        aegis_update_portable(&st, m0, m1);
    }
    uint64_t rem = len % 32;
    if (rem) { /* AegisMac.final: zero-padded partial block */
        uint8_t pad[32] = {0};
        memcpy(pad, src + 32 * full, rem);
        memcpy(m0, pad, 16);
        memcpy(m1, pad + 16, 16);
        aegis_update_portable(&st, m0, m1);
    }
    /* State128L.mac(adlen = len, mlen = 0): sizes = LE64(adlen*8) || LE64(0). */
    uint8_t sizes[16] = {0};
    wr64(sizes, len * 8);
    uint32_t tmp[4];
    memcpy(tmp, sizes, 16);
    for (int c = 0; c < 4; c++) tmp[c] ^= st.s[2][c];
    for (int i = 0; i < 7; i++) aegis_update_portable(&st, tmp, tmp);
    uint32_t tag[4] = {0, 0, 0, 0};
    for (int b = 0; b < 7; b++)
        for (int c = 0; c < 4; c++) tag[c] ^= st.s[b][c];
    memcpy(out, tag, 16);
}

#if defined(__x86_64__)
__attribute__((target("aes,sse4.1"))) static void checksum_aesni(const uint8_t *src, uint64_t len,
                                                                 uint8_t out[16]) {
    __m128i S[8];
    for (int i = 0; i < 8; i++) S[i] = _mm_loadu_si128((const __m128i *)seed_state.s[i]);
#define AEGIS_UPDATE(M0, M1)                                                                   \
    do {                                                                                       \
        __m128i t7 = S[7];                                                                     \
        S[7] = _mm_aesenc_si128(S[6], S[7]);                                                   \
        S[6] = _mm_aesenc_si128(S[5], S[6]);                                                   \
        S[5] = _mm_aesenc_si128(S[4], S[5]);                                                   \
        S[4] = _mm_aesenc_si128(S[3], S[4]);                                                   \
        S[3] = _mm_aesenc_si128(S[2], S[3]);                                                   \
        S[2] = _mm_aesenc_si128(S[1], S[2]);                                                   \
        S[1] = _mm_aesenc_si128(S[0], S[1]);                                                   \
        S[0] = _mm_xor_si128(_mm_aesenc_si128(t7, S[0]), (M0));                                \
        S[4] = _mm_xor_si128(S[4], (M1));                                                      \
    } while (0)
    uint64_t full = len / 32;
    for (uint64_t i = 0; i < full; i++) {
        __m128i m0 = _mm_loadu_si128((const __m128i *)(src + 32 * i));
        __m128i m1 = _mm_loadu_si128((const __m128i *)(src + 32 * i + 16));
        AEGIS_UPDATE(m0, m1);
    }
    uint64_t rem = len % 32;
    if (rem) {
        uint8_t pad[32] = {0};
        memcpy(pad, src + 32 * full, rem);
        __m128i m0 = _mm_loadu_si128((const __m128i *)pad);
        __m128i m1 = _mm_loadu_si128((const __m128i *)(pad + 16));
        AEGIS_UPDATE(m0, m1);
    }
    __m128i tmp = _mm_xor_si128(_mm_set_epi64x(0, (long long)(len * 8)), S[2]);
    for (int i = 0; i < 7; i++) AEGIS_UPDATE(tmp, tmp);
    __m128i tag = _mm_xor_si128(_mm_xor_si128(_mm_xor_si128(S[0], S[1]), _mm_xor_si128(S[2], S[3])),
                                _mm_xor_si128(_mm_xor_si128(S[4], S[5]), S[6]));
    _mm_storeu_si128((__m128i *)out, tag);
#undef AEGIS_UPDATE
}
#endif

int tbo_has_aesni(void) {
    if (use_aesni < 0) {
        use_aesni = 0;
#if defined(__x86_64__)
        unsigned a, b, c, d;
        if (__get_cpuid(1, &a, &b, &c, &d)) use_aesni = (c & bit_AES) ? 1 : 0;
#endif
    }
    return use_aesni && !force_portable;
}

void tbo_force_portable(int on) { force_portable = on; }

/* vsr.checksum (checksum.zig:50-59) via ChecksumStream (67-85). */
void tbo_checksum(const void *source, uint64_t len, uint8_t out[16]) {
    seed_init();
#if defined(__x86_64__)
    if (tbo_has_aesni()) {
        checksum_aesni((const uint8_t *)source, len, out);
        return;
    }
#endif
    checksum_portable((const uint8_t *)source, len, out);
}

void tbo_aegis_seed_state(uint8_t out[128]) {
    seed_init();
    memcpy(out, seed_state.s, 128);
}

/* ------------------------------------------------------------------------ */
/* Tree layout                                                               */
/* ------------------------------------------------------------------------ */

#define HEADER_SIZE 256u
#define SECTOR_SIZE 4096u

uint64_t tbo_sector_ceil(uint64_t offset) {
    return ((offset + SECTOR_SIZE - 1) / SECTOR_SIZE) * SECTOR_SIZE;
}

static int is_pow2(uint32_t x) { return x && !(x & (x - 1)); }

/* TableType.layout (table.zig:107-129), TableIndex.init (schema.zig:119-157),
 * TableData.init (schema.zig:293-314). */
int tbo_tree_init(tbo_tree *t, uint16_t tree_id, uint8_t key_kind, uint8_t usage,
                  uint32_t value_size, uint32_t timestamp_offset,
                  uint32_t table_value_count_max, uint32_t block_size) {
    memset(t, 0, sizeof *t);
    if (tree_id == 0 || key_kind > TBO_KEY_COMPOSITE_U128 || usage > TBO_USAGE_SECONDARY_INDEX) return TBO_ERR_INVALID;
    if (!is_pow2(value_size) || !is_pow2(block_size) || block_size % SECTOR_SIZE) return TBO_ERR_INVALID;
    if (timestamp_offset + 8 > value_size || table_value_count_max == 0) return TBO_ERR_INVALID;
    uint32_t key_size = key_kind == TBO_KEY_TIMESTAMP ? 8 : key_kind == TBO_KEY_COMPOSITE_U128 ? 32 : 16;
    uint32_t body = block_size - HEADER_SIZE;
    uint32_t vcm = body / value_size;
    if (vcm == 0) return TBO_ERR_INVALID;
    uint32_t dbcm = (table_value_count_max + vcm - 1) / vcm;
    uint32_t table_data_blocks_max = body / (32 + 8); /* constants.zig:567-574 */
    if (dbcm > table_data_blocks_max) return TBO_ERR_INVALID;
    t->tree_id = tree_id;
    t->key_kind = key_kind;
    t->usage = usage;
    t->value_size = value_size;
    t->timestamp_offset = timestamp_offset;
    t->key_size = key_size;
    t->block_size = block_size;
    t->block_value_count_max = vcm;
    t->data_block_count_max = dbcm;
    t->value_count_max = table_value_count_max;
    t->index_checksums_offset = HEADER_SIZE;
    t->index_keys_min_offset = HEADER_SIZE + dbcm * 32;
    t->index_keys_max_offset = t->index_keys_min_offset + dbcm * key_size;
    t->index_addresses_offset = t->index_keys_max_offset + dbcm * key_size;
    t->index_size = t->index_addresses_offset + dbcm * 8;
    if (t->index_size > block_size) return TBO_ERR_INVALID;
    return TBO_OK;
}

#define TOMBSTONE_BIT (1ull << 63)

/* key_from_value: groove.zig:27-29 (object), :59-61 (id), composite_key.zig:48-50. */
void tbo_key(const tbo_tree *t, const uint8_t *v, uint64_t k[4]) {
    k[0] = k[1] = k[2] = k[3] = 0;
    switch (t->key_kind) {
    case TBO_KEY_TIMESTAMP:
        k[0] = rd64(v + t->timestamp_offset) & ~TOMBSTONE_BIT;
        break;
    case TBO_KEY_ID_U128:
        k[0] = rd64(v);
        k[1] = rd64(v + 8);
        break;
    case TBO_KEY_COMPOSITE_U64:
        k[0] = rd64(v + 8) & ~TOMBSTONE_BIT;
        k[1] = rd64(v);
        break;
    case TBO_KEY_COMPOSITE_U128:
        k[0] = rd64(v + 16) & ~TOMBSTONE_BIT;
        k[1] = rd64(v);
        k[2] = rd64(v + 8);
        break;
    }
}

/* tombstone(): bit 63 of the value's timestamp (groove.zig:34-36, :66-68,
 * composite_key.zig:56-58). */
int tbo_tombstone(const tbo_tree *t, const uint8_t *v) {
    return (rd64(v + t->timestamp_offset) & TOMBSTONE_BIT) != 0;
}

/* tombstone_from_key (composite_key.zig:64-73): the value {field = key >> 64,
 * timestamp = key | tombstone_bit, padding = 0} of a composite tree; returns
 * TBO_ERR_INVALID if the key's timestamp already has the tombstone bit. */
int tbo_tombstone_from_key(const tbo_tree *t, const uint64_t k[4], uint8_t *v) {
    if (t->key_kind != TBO_KEY_COMPOSITE_U64 && t->key_kind != TBO_KEY_COMPOSITE_U128) return TBO_ERR_INVALID;
    if (k[0] & TOMBSTONE_BIT) return TBO_ERR_INVALID;
    memset(v, 0, t->value_size);
    const uint64_t ts = k[0] | TOMBSTONE_BIT;
    memcpy(v, &k[1], 8);
    if (t->key_kind == TBO_KEY_COMPOSITE_U128) memcpy(v + 8, &k[2], 8);
    memcpy(v + t->timestamp_offset, &ts, 8);
    return TBO_OK;
}

static inline int key_cmp(const uint64_t a[4], const uint64_t b[4]) {
    for (int i = 3; i >= 0; i--) {
        if (a[i] < b[i]) return -1;
        if (a[i] > b[i]) return 1;
    }
    return 0;
}

/* ------------------------------------------------------------------------ */
/* TableMemory.sort (table_memory.zig:140-154)                               */
/* ------------------------------------------------------------------------ */

typedef struct { uint64_t k[4]; uint32_t i; } sort_item;

static void merge_sort_items(sort_item *a, sort_item *tmp, uint32_t n) {
    /* Bottom-up stable merge sort. */
    for (uint32_t w = 1; w < n; w *= 2) {
        for (uint32_t lo = 0; lo < n; lo += 2 * w) {
            uint32_t mid = lo + w < n ? lo + w : n;
            uint32_t hi = lo + 2 * w < n ? lo + 2 * w : n;
            uint32_t i = lo, j = mid, o = lo;
            while (i < mid && j < hi) {
                /* Take from the right run only if strictly less: stable. */
                if (key_cmp(a[j].k, a[i].k) < 0) tmp[o++] = a[j++];
                else tmp[o++] = a[i++];
            }
            while (i < mid) tmp[o++] = a[i++];
            while (j < hi) tmp[o++] = a[j++];
        }
        memcpy(a, tmp, (size_t)n * sizeof(sort_item));
    }
}

int tbo_sort_values(const tbo_tree *t, uint8_t *values, uint32_t n) {
    if (n < 2) return TBO_OK;
    const uint32_t vs = t->value_size;
    /* TableMemory.put tracks `sorted`; sort() is a no-op if keys arrived in
     * non-decreasing order (table_memory.zig:83-87, 141). */
    int sorted = 1;
    uint64_t prev[4], cur[4];
    tbo_key(t, values, prev);
    for (uint32_t i = 1; i < n && sorted; i++) {
        tbo_key(t, values + (size_t)i * vs, cur);
        if (key_cmp(prev, cur) > 0) sorted = 0;
        memcpy(prev, cur, sizeof cur);
    }
    if (sorted) return TBO_OK;
    sort_item *items = (sort_item *)malloc((size_t)n * sizeof(sort_item));
    sort_item *tmp = (sort_item *)malloc((size_t)n * sizeof(sort_item));
    uint8_t *copy = (uint8_t *)malloc((size_t)n * vs);
    if (!items || !tmp || !copy) {
        free(items); free(tmp); free(copy);
        return TBO_ERR_CAPACITY;
    }
    for (uint32_t i = 0; i < n; i++) {
        tbo_key(t, values + (size_t)i * vs, items[i].k);
        items[i].i = i;
    }
    merge_sort_items(items, tmp, n);
    memcpy(copy, values, (size_t)n * vs);
    for (uint32_t i = 0; i < n; i++) memcpy(values + (size_t)i * vs, copy + (size_t)items[i].i * vs, vs);
    free(items); free(tmp); free(copy);
    return TBO_OK;
}

/* ------------------------------------------------------------------------ */
/* Compaction                                                                */
/* ------------------------------------------------------------------------ */

typedef struct builder {
    uint64_t key_min[4], key_max[4];
    uint8_t *index_block;
    uint8_t *data_block;
    uint32_t data_block_count;
    uint32_t value_count;
    uint32_t value_count_total;
} builder;

typedef struct run {
    const tbo_tree *t;
    tbo_job *job;
    builder b;
    const uint8_t *values_in[2];
    uint32_t values_in_len[2];
    uint8_t *data_blocks[2]; /* Compaction.data_blocks (compaction.zig:115) */
    const uint8_t *immutable; /* context.table_info_a.immutable remainder */
    uint32_t immutable_len;
    uint32_t seg_a, seg_b;
    uint32_t acquired;
    int exhausted;
    int error;
} run;

static void write_key(const tbo_tree *t, uint8_t *dst, const uint64_t k[4]) {
    for (uint32_t i = 0; i < t->key_size / 8; i++) wr64(dst + 8 * i, k[i]);
}

/* Header.Block defaults + fields (message_header.zig:1153-1178). */
static void header_block(uint8_t *h, const tbo_job *job, uint32_t size, uint64_t address,
                         uint64_t snapshot, uint8_t block_type) {
    memset(h, 0, HEADER_SIZE);
    wr64(h + 80, job->cluster_lo);
    wr64(h + 88, job->cluster_hi);
    wr32(h + 96, size);
    /* epoch @100 = 0, view @104 = 0, version @108 = vsr.Version = 0 (vsr.zig:63) */
    h[110] = 20; /* Command.block (vsr.zig:196) */
    wr64(h + 224, address);
    wr64(h + 232, snapshot);
    h[240] = block_type;
}

/* set_checksum_body then set_checksum (message_header.zig:101-125). */
static void header_checksums(uint8_t *block, uint32_t size) {
    tbo_checksum(block + HEADER_SIZE, size - HEADER_SIZE, block + 32);
    tbo_checksum(block + 16, HEADER_SIZE - 16, block);
}

static uint64_t acquire(run *r) {
    /* grid.acquire(reservation): the next free address of the reservation, in
     * order (free_set.zig:302-345). The caller passes that sequence in. */
    if (r->acquired >= r->job->address_count || r->acquired >= r->job->out_block_capacity) {
        r->error = TBO_ERR_CAPACITY;
        return 0;
    }
    return r->job->addresses[r->acquired];
}

/* grid.create_block: the block image is [0, sector_ceil(size)) with the tail
 * zeroed (grid.zig:641-702, storage_checker.zig:305-310). */
static void emit_block(run *r, const uint8_t *block, uint32_t size) {
    uint8_t *dst = r->job->out_blocks + (size_t)r->acquired * r->t->block_size;
    memcpy(dst, block, size);
    uint64_t ceil = tbo_sector_ceil(size);
    memset(dst + size, 0, ceil - size);
    r->acquired += 1;
}

/* Table.Builder.data_block_finish (table.zig:306-384). */
static void data_block_finish(run *r, uint64_t address) {
    const tbo_tree *t = r->t;
    builder *b = &r->b;
    uint8_t *block = b->data_block;
    uint32_t size = HEADER_SIZE + b->value_count * t->value_size;
    header_block(block, r->job, size, address, r->job->snapshot_min, 5 /* BlockType.data */);
    /* TableData.Metadata (schema.zig:264-275) */
    wr32(block + 128, t->block_value_count_max);
    wr32(block + 132, b->value_count);
    wr32(block + 136, t->value_size);
    wr16(block + 140, t->tree_id);
    header_checksums(block, size);

    const uint8_t *values = block + HEADER_SIZE;
    uint64_t key_min[4], key_max[4];
    tbo_key(t, values, key_min);
    tbo_key(t, values + (size_t)(b->value_count - 1) * t->value_size, key_max);
    if (b->value_count > 1 && key_cmp(key_min, key_max) >= 0) r->error = TBO_ERR_INVARIANT;

    uint32_t current = b->data_block_count;
    write_key(t, b->index_block + t->index_keys_min_offset + current * t->key_size, key_min);
    write_key(t, b->index_block + t->index_keys_max_offset + current * t->key_size, key_max);
    wr64(b->index_block + t->index_addresses_offset + current * 8, address);
    memcpy(b->index_block + t->index_checksums_offset + current * 32, block, 16); /* .value */
    memset(b->index_block + t->index_checksums_offset + current * 32 + 16, 0, 16); /* .padding */

    if (current == 0) memcpy(b->key_min, key_min, sizeof key_min);
    if (current > 0 && key_cmp(b->key_max, key_min) >= 0) r->error = TBO_ERR_INVARIANT;
    memcpy(b->key_max, key_max, sizeof key_max);

    b->data_block_count += 1;
    b->value_count_total += b->value_count;
    b->value_count = 0;
    emit_block(r, block, size);
}

/* Table.Builder.index_block_finish (table.zig:403-457) + TreeTableInfo.encode
 * (manifest.zig:121-149) for Manifest.insert_table (manifest.zig:233-255). */
static void index_block_finish(run *r, uint64_t address) {
    const tbo_tree *t = r->t;
    builder *b = &r->b;
    uint8_t *block = b->index_block;
    header_block(block, r->job, t->index_size, address, r->job->snapshot_min, 4 /* BlockType.index */);
    /* TableIndex.Metadata (schema.zig:87-98) */
    wr32(block + 128, b->data_block_count);
    wr32(block + 132, t->data_block_count_max);
    wr32(block + 136, t->key_size);
    wr16(block + 140, t->tree_id);
    /* TableIndex.padding (schema.zig:233-259): zero the unused slots. */
    uint32_t used = b->data_block_count, max = t->data_block_count_max;
    memset(block + t->index_checksums_offset + used * 32, 0, (max - used) * 32);
    memset(block + t->index_keys_min_offset + used * t->key_size, 0, (max - used) * t->key_size);
    memset(block + t->index_keys_max_offset + used * t->key_size, 0, (max - used) * t->key_size);
    memset(block + t->index_addresses_offset + used * 8, 0, (max - used) * 8);
    header_checksums(block, t->index_size);

    if (r->job->out_table_count >= r->job->out_table_capacity) {
        r->error = TBO_ERR_CAPACITY;
    } else {
        /* schema.ManifestNode.TableInfo (schema.zig:489-509) */
        uint8_t *info = r->job->out_table_infos + (size_t)r->job->out_table_count * 128;
        memset(info, 0, 128);
        write_key(t, info + 0, b->key_min);
        write_key(t, info + 32, b->key_max);
        memcpy(info + 64, block, 16); /* checksum; checksum_padding @80 = 0 */
        wr64(info + 96, address);
        wr64(info + 104, r->job->snapshot_min);
        wr64(info + 112, ~0ull); /* snapshot_max = maxInt(u64) (manifest.zig:43) */
        wr32(info + 120, b->value_count_total);
        wr16(info + 124, t->tree_id);
        info[126] = (uint8_t)((r->job->level_b & 0x3f) | (1u << 6)); /* Label{level, .insert} */
        r->job->out_table_count += 1;
    }
    emit_block(r, block, t->index_size);
    b->data_block_count = 0;
    b->value_count = 0;
    b->value_count_total = 0;
}

/* Compaction.fill_immutable_values (compaction.zig:483-559). */
static uint32_t fill_immutable_values(run *r, uint8_t *target, uint32_t target_len) {
    const tbo_tree *t = r->t;
    const uint32_t vs = t->value_size;
    const uint8_t *source = r->immutable;
    uint32_t source_len = r->immutable_len;
    uint32_t si = 0, ti = 0;
    uint64_t k0[4], k1[4];
    while (ti < target_len && si < source_len) {
        memcpy(target + (size_t)ti * vs, source + (size_t)si * vs, vs);
        int next_equal = 0;
        if (si + 1 < source_len) {
            tbo_key(t, source + (size_t)si * vs, k0);
            tbo_key(t, source + (size_t)(si + 1) * vs, k1);
            next_equal = key_cmp(k0, k1) == 0;
        }
        if (next_equal) {
            if (t->usage == TBO_USAGE_SECONDARY_INDEX) {
                /* cancel out put and remove (508-517) */
                if (tbo_tombstone(t, source + (size_t)si * vs) ==
                    tbo_tombstone(t, source + (size_t)(si + 1) * vs))
                    r->error = TBO_ERR_INVARIANT;
                si += 2;
            } else {
                si += 1; /* last of a run of duplicates wins (519-523) */
            }
        } else {
            si += 1;
            ti += 1;
        }
    }
    r->immutable += (size_t)si * vs;
    r->immutable_len -= si;
    return ti;
}

/* Table.data_block_values(builder.data_block) slots. */
static inline uint8_t *out_slot(run *r, uint32_t index) {
    return r->b.data_block + HEADER_SIZE + (size_t)index * r->t->value_size;
}

/* Compaction.copy (compaction.zig:688-710). */
static void do_copy(run *r, int level) {
    const uint32_t vs = r->t->value_size;
    uint32_t room = r->t->block_value_count_max - r->b.value_count;
    uint32_t len = r->values_in_len[level] < room ? r->values_in_len[level] : room;
    memcpy(out_slot(r, r->b.value_count), r->values_in[level], (size_t)len * vs);
    r->values_in[level] += (size_t)len * vs;
    r->values_in_len[level] -= len;
    r->b.value_count += len;
}

/* Compaction.copy_drop_tombstones (compaction.zig:712-741). */
static void do_copy_drop_tombstones(run *r) {
    const tbo_tree *t = r->t;
    const uint32_t vs = t->value_size;
    uint32_t ia = 0, out = r->b.value_count;
    const uint8_t *a = r->values_in[0];
    while (ia < r->values_in_len[0] && out < t->block_value_count_max) {
        const uint8_t *va = a + (size_t)ia * vs;
        ia += 1;
        if (tbo_tombstone(t, va)) {
            if (t->usage == TBO_USAGE_SECONDARY_INDEX) r->error = TBO_ERR_INVARIANT;
            continue;
        }
        memcpy(out_slot(r, out), va, vs);
        out += 1;
    }
    r->values_in[0] += (size_t)ia * vs;
    r->values_in_len[0] -= ia;
    r->b.value_count = out;
}

/* Compaction.merge (compaction.zig:743-804). */
static void do_merge(run *r) {
    const tbo_tree *t = r->t;
    const uint32_t vs = t->value_size;
    const uint8_t *a = r->values_in[0], *b = r->values_in[1];
    uint32_t na = r->values_in_len[0], nb = r->values_in_len[1];
    uint32_t ia = 0, ib = 0, out = r->b.value_count;
    uint64_t ka[4], kb[4];
    while (ia < na && ib < nb && out < t->block_value_count_max) {
        const uint8_t *va = a + (size_t)ia * vs, *vb = b + (size_t)ib * vs;
        tbo_key(t, va, ka);
        tbo_key(t, vb, kb);
        int o = key_cmp(ka, kb);
        if (o < 0) {
            ia += 1;
            if (r->job->drop_tombstones && tbo_tombstone(t, va)) {
                if (t->usage == TBO_USAGE_SECONDARY_INDEX) r->error = TBO_ERR_INVARIANT;
                continue;
            }
            memcpy(out_slot(r, out++), va, vs);
        } else if (o > 0) {
            ib += 1;
            memcpy(out_slot(r, out++), vb, vs);
        } else {
            ia += 1;
            ib += 1;
            if (t->usage == TBO_USAGE_SECONDARY_INDEX) {
                if (tbo_tombstone(t, va) == tbo_tombstone(t, vb)) r->error = TBO_ERR_INVARIANT;
                continue;
            } else if (r->job->drop_tombstones) {
                if (tbo_tombstone(t, va)) continue;
            }
            memcpy(out_slot(r, out++), va, vs);
        }
    }
    r->values_in[0] += (size_t)ia * vs;
    r->values_in_len[0] -= ia;
    r->values_in[1] += (size_t)ib * vs;
    r->values_in_len[1] -= ib;
    r->b.value_count = out;
}

/* Compaction.start → loop_start → iterator_check(.a/.b) → compact →
 * write_blocks, until exhausted (compaction.zig:280-921). */
int tbo_compact(tbo_job *job) {
    if (!job || !job->tree) return TBO_ERR_INVALID;
    const tbo_tree *t = job->tree;
    const uint32_t vs = t->value_size;
    if (job->a_immutable && job->segment_count_a > 1) return TBO_ERR_INVALID;
    /* Move-table (compaction.zig:296-298): disk A with no level-B tables writes
     * no blocks — only the manifest entry moves. The caller handles it. */
    job->out_value_count = 0;
    job->out_data_block_count = 0;
    job->out_table_count = 0;
    job->out_block_count = 0;

    run r;
    memset(&r, 0, sizeof r);
    r.t = t;
    r.job = job;
    r.b.index_block = (uint8_t *)calloc(1, t->block_size);
    r.b.data_block = (uint8_t *)calloc(1, t->block_size);
    r.data_blocks[0] = (uint8_t *)calloc(1, t->block_size);
    r.data_blocks[1] = (uint8_t *)calloc(1, t->block_size);
    if (!r.b.index_block || !r.b.data_block || !r.data_blocks[0] || !r.data_blocks[1]) {
        free(r.b.index_block); free(r.b.data_block); free(r.data_blocks[0]); free(r.data_blocks[1]);
        return TBO_ERR_CAPACITY;
    }
    if (job->a_immutable && job->segment_count_a == 1) {
        r.immutable = job->segments_a[0].values;
        r.immutable_len = job->segments_a[0].count;
    }

    for (;;) {
        /* iterator_check(.a) (compaction.zig:443-477) */
        if (r.values_in_len[0] == 0) {
            if (job->a_immutable) {
                if (r.immutable_len > 0) {
                    uint8_t *target = r.data_blocks[0] + HEADER_SIZE;
                    uint32_t filled = fill_immutable_values(&r, target, t->block_value_count_max);
                    if (filled == 0 && t->usage != TBO_USAGE_SECONDARY_INDEX) r.error = TBO_ERR_INVARIANT;
                    r.values_in[0] = target;
                    r.values_in_len[0] = filled;
                }
            } else if (r.seg_a < job->segment_count_a) {
                /* TableDataIterator.next + copy of the data block (compaction.zig:603-613) */
                const tbo_segment *s = &job->segments_a[r.seg_a++];
                memcpy(r.data_blocks[0] + HEADER_SIZE, s->values, (size_t)s->count * vs);
                r.values_in[0] = r.data_blocks[0] + HEADER_SIZE;
                r.values_in_len[0] = s->count;
            }
        }
        /* iterator_check(.b) */
        if (r.values_in_len[1] == 0 && r.seg_b < job->segment_count_b) {
            const tbo_segment *s = &job->segments_b[r.seg_b++];
            memcpy(r.data_blocks[1] + HEADER_SIZE, s->values, (size_t)s->count * vs);
            r.values_in[1] = r.data_blocks[1] + HEADER_SIZE;
            r.values_in_len[1] = s->count;
        }
        /* compact() (compaction.zig:647-686) */
        if (r.values_in_len[0] == 0 && r.values_in_len[1] == 0) {
            r.exhausted = 1;
        } else if (r.values_in_len[0] == 0) {
            do_copy(&r, 1);
        } else if (r.values_in_len[1] == 0) {
            if (job->drop_tombstones) do_copy_drop_tombstones(&r);
            else do_copy(&r, 0);
        } else {
            do_merge(&r);
        }
        /* write_blocks() (compaction.zig:806-850) */
        int data_full = r.b.value_count == t->block_value_count_max;
        int index_full = r.b.data_block_count == t->data_block_count_max;
        if (data_full || index_full || (r.exhausted && r.b.value_count > 0)) {
            uint64_t address = acquire(&r);
            if (r.error) break;
            data_block_finish(&r, address);
            job->out_data_block_count += 1;
        }
        index_full = r.b.data_block_count == t->data_block_count_max;
        if (index_full || (r.exhausted && r.b.data_block_count > 0)) {
            uint64_t address = acquire(&r);
            if (r.error) break;
            job->out_value_count += r.b.value_count_total;
            index_block_finish(&r, address);
        }
        if (r.error || r.exhausted) break;
    }
    job->out_block_count = r.acquired;
    free(r.b.index_block);
    free(r.b.data_block);
    free(r.data_blocks[0]);
    free(r.data_blocks[1]);
    return r.error;
}
