/*
 * benchmark_load.c — the `tigerbeetle benchmark` default load, regenerated
 * on the host (BASELINE.json configs[0]).
 *
 * Restates src/tigerbeetle/benchmark_load.zig:
 *   - accounts 1..account_count (IdPermutation .identity, :132-138, :222-237:
 *     ledger 2, code 1, flags 0, user data 0);
 *   - transfers with ids 1..transfer_count, in batches of
 *     transfer_count_per_batch = 8190 (:50-53), each drawing from ONE
 *     std.rand.DefaultPrng.init(42) stream (:132) in the order of the
 *     reference's struct literal (:287-315): debit index uintLessThan,
 *     credit index uintLessThan (+1 mod count when equal), user_data_128
 *     int(u128), user_data_64 int(u64), user_data_32 int(u32), code
 *     int(u16) +| 1, amount random_int_exponential(u64, 10_000) +| 1, then the
 *     arrival-time draw random_int_exponential(u64, 1000 ns) (:312-313);
 *     pending_id = timeout = 0, ledger 2, flags 0;
 *   - the state machine's effects of each committed batch
 *     (src/state_machine.zig:1035 timestamps `prepare_timestamp - len + i + 1`,
 *     :1328-1340 transfers.insert then accounts.update(dr), accounts.update(cr)
 *     with debits_posted / credits_posted += amount).
 *
 * Deviations (stated in DESIGN.md §10): DefaultPrng is Zig 0.11's Xoshiro256
 * (xoshiro256++ seeded by SplitMix64, pinned by the checksum stability KAT in
 * tests/zig_prng.py) and Random.int / uintLessThan are restated exactly, but
 * Random.floatExp (a Ziggurat in Zig std, not in the reference tree) is
 * replaced by inversion of one 53-bit draw, so the exponential variates
 * differ; batches are always full (the reference fills a batch with the
 * transfers whose arrival time has passed, which depends on wall-clock
 * latency); prepare timestamps advance by one batch interval of the offered
 * load (8190 x 1000 ns) per op instead of the replica's clock.
 *
 * Host-side workload generation only (bench / tests); not part of libtbc.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef struct tbl_prng {
    uint64_t s[4];
} tbl_prng;

static uint64_t splitmix64(uint64_t *x) {
    uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

/* std.rand.Xoshiro256.next (xoshiro256++). */
static uint64_t next(tbl_prng *p) {
    uint64_t *s = p->s;
    const uint64_t r = rotl(s[0] + s[3], 23) + s[0];
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
}

void tbl_prng_init(tbl_prng *p, uint64_t seed) {
    uint64_t x = seed;
    for (int i = 0; i < 4; i++) p->s[i] = splitmix64(&x);
}

/* Random.uintLessThan(u64, n): Lemire's method with the rejection tweak. */
static uint64_t uint_less_than(tbl_prng *p, uint64_t n) {
    uint64_t x = next(p);
    unsigned __int128 m = (unsigned __int128)x * n;
    uint64_t l = (uint64_t)m;
    if (l < n) {
        uint64_t t = (uint64_t)0 - n;
        if (t >= n) {
            t -= n;
            if (t >= n) t %= n;
        }
        while (l < t) {
            x = next(p);
            m = (unsigned __int128)x * n;
            l = (uint64_t)m;
        }
    }
    return (uint64_t)(m >> 64);
}

/* random_int_exponential(u64, avg) (src/testing/fuzz.zig:16-24) with the
 * exponential variate by inversion (see the header). lossyCast truncates. */
static uint64_t int_exponential(tbl_prng *p, uint64_t avg) {
    const double u = (double)(next(p) >> 11) * (1.0 / 9007199254740992.0);
    const double e = -log1p(-u) * (double)avg;
    if (!(e > 0)) return 0;
    if (e >= 18446744073709551615.0) return UINT64_MAX;
    return (uint64_t)e;
}

static void put_u64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static void put_u32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }
static void put_u16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }
static uint64_t get_u64(const uint8_t *p) {
    uint64_t v;
    memcpy(&v, p, 8);
    return v;
}

/* tigerbeetle.Account (src/tigerbeetle.zig:7-40) as created by the benchmark. */
void tbl_account(uint64_t index, uint64_t timestamp, uint8_t *out128) {
    memset(out128, 0, 128);
    put_u64(out128 + 0, index + 1); /* id = identity.encode(index + 1) */
    put_u32(out128 + 112, 2);       /* ledger */
    put_u16(out128 + 116, 1);       /* code */
    put_u64(out128 + 120, timestamp);
}

/* One create_transfers batch: `count` Transfers (128 B, src/tigerbeetle.zig:80-104)
 * with ids first_index+1.., committed at `prepare_timestamp`, and the 2*count
 * Account values the commit puts into accounts' object tree (dr then cr per
 * transfer). `accounts` holds the current Account of every account (updated). */
void tbl_transfers(tbl_prng *p, uint64_t first_index, uint32_t count, uint64_t account_count,
                   uint64_t prepare_timestamp, uint8_t *accounts, uint8_t *transfers_out, uint8_t *account_puts_out) {
    for (uint32_t i = 0; i < count; i++) {
        uint8_t *t = transfers_out + 128ull * i;
        const uint64_t dr = uint_less_than(p, account_count);
        uint64_t cr = uint_less_than(p, account_count);
        if (dr == cr) cr = (cr + 1) % account_count;
        const uint64_t ud128_lo = next(p), ud128_hi = next(p);
        const uint64_t ud64 = next(p);
        const uint32_t ud32 = (uint32_t)next(p);
        const uint16_t code16 = (uint16_t)next(p);
        const uint16_t code = code16 == 0xffff ? 0xffff : (uint16_t)(code16 + 1);
        uint64_t amount = int_exponential(p, 10000);
        amount = amount == UINT64_MAX ? amount : amount + 1;
        (void)int_exponential(p, 1000); /* transfer_next_arrival_ns += ... */
        memset(t, 0, 128);
        put_u64(t + 0, first_index + i + 1); /* id */
        put_u64(t + 16, dr + 1);             /* debit_account_id */
        put_u64(t + 32, cr + 1);             /* credit_account_id */
        put_u64(t + 48, amount);             /* amount (u128) */
        put_u64(t + 80, ud128_lo);           /* user_data_128 */
        put_u64(t + 88, ud128_hi);
        put_u64(t + 96, ud64);   /* user_data_64 */
        put_u32(t + 104, ud32);  /* user_data_32 */
        put_u32(t + 112, 2);     /* ledger */
        put_u16(t + 116, code);  /* code */
        const uint64_t ts = prepare_timestamp - count + i + 1;
        put_u64(t + 120, ts);
        /* accounts.update(dr), accounts.update(cr): debits/credits_posted += amount */
        uint8_t *a_dr = accounts + 128ull * dr, *a_cr = accounts + 128ull * cr;
        put_u64(a_dr + 32, get_u64(a_dr + 32) + amount); /* debits_posted (u128, < 2^64 here) */
        memcpy(account_puts_out + 256ull * i, a_dr, 128);
        put_u64(a_cr + 64, get_u64(a_cr + 64) + amount); /* credits_posted */
        memcpy(account_puts_out + 256ull * i + 128, a_cr, 128);
    }
}
