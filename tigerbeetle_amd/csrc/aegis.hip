// aegis.hip — AEGIS-128L block checksums and block finishing on gfx950.
//
// vsr.checksum (src/vsr/checksum.zig:38-85) is Zig 0.11 std
// Aegis128LMac_128 with key = 0 and nonce = 0: the message is absorbed as
// associated data, 32 bytes per State128L.update, zero-padded tail, then
// finalised with LE64(len*8) || 0. It is sequential per message, so the
// parallelism is (#messages x 32 lanes):
//
//   * one message per 32-lane group (two groups per wave64);
//   * lane (p, c) owns column c (a little-endian dword) of AEGIS block p;
//   * an AES round is four T-table lookups in LDS per lane, combined across
//     the quad with DPP quad_perm (MixColumns/ShiftRows), no VGPR tables;
//   * AEGIS' block rotation S'[i] = AESRound(S[i-1]) ^ S[i] is turned into a
//     label rotation: quad p keeps its register and becomes block label+1,
//     so the only cross-quad move is the round key S[label+1], fetched off
//     the dependency chain (DPP row_ror + permlane16_swap when a chain runs
//     alone per SIMD, one ds_bpermute when four chains share a SIMD);
//   * message words are prefetched a whole group (64 updates) ahead.
//
// Block finishing (Table.Builder.data_block_finish / index_block_finish,
// src/lsm/table.zig:306-457) is fused here: body assembly (producer waves
// copy the surviving values into the output block from the merge's masks
// while the chain waves of the same workgroup checksum what is already in
// place), body checksum, header fields, header checksum, index-block body,
// TableInfo.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "tbc_internal.h"
#include "keys.h"

namespace tbc {

// --------------------------------------------------------------------------
// Compile-time AES T-tables and the AEGIS seed state.
// --------------------------------------------------------------------------

struct AesTables {
    uint32_t t[4][256];
};

constexpr uint8_t xtime_c(uint8_t x) { return (uint8_t)((x << 1) ^ ((x & 0x80) ? 0x1B : 0)); }
constexpr uint8_t rotl8_c(uint8_t x, int s) { return (uint8_t)((x << s) | (x >> (8 - s))); }

struct Sbox {
    uint8_t s[256];
};

constexpr Sbox make_sbox() {
    Sbox sb{};
    uint8_t p = 1, q = 1;
    do {
        p = (uint8_t)(p ^ (uint8_t)(p << 1) ^ ((p & 0x80) ? 0x1B : 0));
        q ^= (uint8_t)(q << 1);
        q ^= (uint8_t)(q << 2);
        q ^= (uint8_t)(q << 4);
        if (q & 0x80) q ^= 0x09;
        uint8_t x = (uint8_t)(q ^ rotl8_c(q, 1) ^ rotl8_c(q, 2) ^ rotl8_c(q, 3) ^ rotl8_c(q, 4));
        sb.s[p] = (uint8_t)(x ^ 0x63);
    } while (p != 1);
    sb.s[0] = 0x63;
    return sb;
}

constexpr AesTables make_tables() {
    AesTables t{};
    Sbox sb = make_sbox();
    for (int i = 0; i < 256; i++) {
        uint32_t s = sb.s[i], s2 = xtime_c((uint8_t)s), s3 = s2 ^ s;
        t.t[0][i] = s2 | (s << 8) | (s << 16) | (s3 << 24);
        t.t[1][i] = s3 | (s2 << 8) | (s << 16) | (s << 24);
        t.t[2][i] = s | (s3 << 8) | (s2 << 16) | (s << 24);
        t.t[3][i] = s | (s << 8) | (s3 << 16) | (s2 << 24);
    }
    return t;
}

struct AegisSeed {
    uint32_t s[8][4];
};

constexpr void aesenc_c(const AesTables &T, uint32_t out[4], const uint32_t in[4], const uint32_t rk[4]) {
    for (int c = 0; c < 4; c++)
        out[c] = T.t[0][in[c] & 0xff] ^ T.t[1][(in[(c + 1) & 3] >> 8) & 0xff] ^
                 T.t[2][(in[(c + 2) & 3] >> 16) & 0xff] ^ T.t[3][in[(c + 3) & 3] >> 24] ^ rk[c];
}

// Aegis128LMac_128.init(key = 0): blocks [0, C1, C0, C1, 0, C0, C1, C0], then
// 10 x update(0, 0) (checksum.zig:43-46 seed_state).
constexpr AegisSeed make_seed() {
    AesTables T = make_tables();
    const uint8_t c0[16] = {0x00, 0x01, 0x01, 0x02, 0x03, 0x05, 0x08, 0x0d,
                            0x15, 0x22, 0x37, 0x59, 0x90, 0xe9, 0x79, 0x62};
    const uint8_t c1[16] = {0xdb, 0x3d, 0x18, 0x55, 0x6d, 0xc2, 0x2f, 0xf1,
                            0x20, 0x11, 0x31, 0x42, 0x73, 0xb5, 0x28, 0xdd};
    uint32_t C0[4] = {}, C1[4] = {};
    for (int c = 0; c < 4; c++) {
        C0[c] = c0[4 * c] | (c0[4 * c + 1] << 8) | (c0[4 * c + 2] << 16) | ((uint32_t)c0[4 * c + 3] << 24);
        C1[c] = c1[4 * c] | (c1[4 * c + 1] << 8) | (c1[4 * c + 2] << 16) | ((uint32_t)c1[4 * c + 3] << 24);
    }
    AegisSeed st{};
    for (int c = 0; c < 4; c++) {
        st.s[1][c] = C1[c];
        st.s[2][c] = C0[c];
        st.s[3][c] = C1[c];
        st.s[5][c] = C0[c];
        st.s[6][c] = C1[c];
        st.s[7][c] = C0[c];
    }
    for (int r = 0; r < 10; r++) {
        uint32_t tmp[4] = {st.s[7][0], st.s[7][1], st.s[7][2], st.s[7][3]};
        uint32_t n[4] = {};
        for (int i = 7; i > 0; i--) {
            aesenc_c(T, n, st.s[i - 1], st.s[i]);
            for (int c = 0; c < 4; c++) st.s[i][c] = n[c];
        }
        aesenc_c(T, n, tmp, st.s[0]);
        for (int c = 0; c < 4; c++) st.s[0][c] = n[c];
    }
    return st;
}

__constant__ AesTables c_aes = make_tables();
__constant__ AegisSeed c_seed = make_seed();

// --------------------------------------------------------------------------
// Lane helpers.
// --------------------------------------------------------------------------

// quad_perm DPP: lane c of each quad reads lane sel[c] of the same quad.
template <int S0, int S1, int S2, int S3>
__device__ __forceinline__ uint32_t quad_perm(uint32_t v) {
    constexpr int ctrl = S0 | (S1 << 2) | (S2 << 4) | (S3 << 6);
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, 0xf, 0xf, true);
}

__device__ __forceinline__ uint32_t bpermute(uint32_t byte_addr, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)byte_addr, (int)v);
}

// T-tables in LDS, replicated once per bank so that a 32-lane group's lookups
// never conflict (ds_read_b32 banks are (addr/4) mod 32 per 32-lane group):
// entry T_r[b] for lane bank k lives at
//     (r >> 1) * 64 KiB + b * 256 + (r & 1) * 128 + k * 4,
// so one v_perm_b32 builds the address {k*4, b, region, 0} from the state
// column and a per-lane base, and the (r & 1) half is the ds_read offset.
constexpr uint32_t kTableBytes = 131072;
constexpr uint32_t kTableDwords = kTableBytes / 4;

__device__ __forceinline__ void load_tables(uint32_t *sT) {
    for (uint32_t i = threadIdx.x; i < kTableDwords; i += blockDim.x) {
        const uint32_t r = ((i >> 14) << 1) | ((i >> 5) & 1);
        const uint32_t b = (i >> 6) & 255;
        sT[i] = c_aes.t[r][b];
    }
}

struct TableBase {
    uint32_t lo, hi; // {k*4, -, 0, 0} and {k*4, -, 1, 0}
    __device__ __forceinline__ TableBase() {
        const uint32_t k = threadIdx.x & 31;
        lo = k * 4;
        hi = k * 4 | 0x10000u;
    }
};

__device__ __forceinline__ uint32_t lds_u32(const uint32_t *sT, uint32_t byte_off) {
    return *(const uint32_t *)((const char *)sT + byte_off);
}

// One AES round (no round key) of column c: T0[b0(c)] ^ T1[b1(c+1)] ^
// T2[b2(c+2)] ^ T3[b3(c+3)]; each lane looks up its own column's four bytes
// and the quad exchanges the partial products. `acc` (the round key, already
// xored with the message word) is folded in first so the chain ends with the
// last lookup to return.
__device__ __forceinline__ uint32_t aes_col(const uint32_t *sT, const TableBase &tb, uint32_t x, uint32_t acc) {
    // v_perm_b32 selector bytes: 0-3 pick src1 (base), 4-7 pick src0 (x).
    const uint32_t a0 = __builtin_amdgcn_perm(x, tb.lo, 0x03020400u);
    const uint32_t a1 = __builtin_amdgcn_perm(x, tb.lo, 0x03020500u);
    const uint32_t a2 = __builtin_amdgcn_perm(x, tb.hi, 0x03020600u);
    const uint32_t a3 = __builtin_amdgcn_perm(x, tb.hi, 0x03020700u);
    const uint32_t t0 = lds_u32(sT, a0);
    const uint32_t t1 = lds_u32(sT, a1 + 128);
    const uint32_t t2 = lds_u32(sT, a2);
    const uint32_t t3 = lds_u32(sT, a3 + 128);
    uint32_t r = acc ^ t0;
    r ^= quad_perm<1, 2, 3, 0>(t1);
    r ^= quad_perm<2, 3, 0, 1>(t2);
    r ^= quad_perm<3, 0, 1, 2>(t3);
    return r;
}

// One AEGIS update step of lane (p, c): S'[label+1] = AESRound(S[label]) ^
// S[label+1] ^ m, with the round key S[label+1] = x of quad p+1.
struct StepBpermute {
    __device__ static __forceinline__ uint32_t step(const uint32_t *sT, const TableBase &tb, uint32_t key_src,
                                                    uint32_t x, uint32_t m) {
        const uint32_t key = bpermute(key_src, x);
        return aes_col(sT, tb, x, key ^ m);
    }
};

// Message sources. Whole 32-byte blocks are read in two stages so that a
// source with an indirection can run its first stage further ahead:
//   addr(off)  where the dword at byte `off` lives (the offset is clamped, so
//              it is always in bounds and the prefetch ring never waits on a
//              divergent branch);
//   word(a)    the dword itself;
//   exact(off) the dword at `off`, zero beyond `len` (AegisMac.final
//              zero-pads the tail), for the last partial 32-byte block;
//   sink(off, w) called once for every absorbed dword below `len` (a source
//              that also materialises the message stores it there).
// Offsets are multiples of 4; buffers are readable up to len rounded up to 4.
struct GlobalMsg {
    using Addr = const uint8_t *;
    const uint8_t *base;
    uint32_t len;
    uint32_t max_off;
    __device__ __forceinline__ GlobalMsg(const uint8_t *b, uint32_t l)
        : base(b), len(l), max_off(l >= 4 ? (l & ~3u) - 4 : 0) {}
    __device__ __forceinline__ Addr addr(uint32_t off) const { return base + (off < max_off ? off : max_off); }
    __device__ __forceinline__ uint32_t word(Addr a) const { return gld<uint32_t>(a); }
    __device__ __forceinline__ uint32_t exact(uint32_t off) const {
        if (off >= len) return 0;
        uint32_t v = gld<uint32_t>(base + off);
        uint32_t rem = len - off;
        if (rem < 4) v &= (1u << (8 * rem)) - 1u;
        return v;
    }
    __device__ __forceinline__ void sink(uint32_t, uint32_t) const {}
    __device__ __forceinline__ void ready(uint32_t) const {}
};

struct LdsMsg {
    using Addr = uint32_t;
    const uint32_t *base; // dword-aligned LDS pointer
    uint32_t len;
    uint32_t max_off;
    __device__ __forceinline__ LdsMsg(const uint32_t *b, uint32_t l)
        : base(b), len(l), max_off(l >= 4 ? (l & ~3u) - 4 : 0) {}
    __device__ __forceinline__ Addr addr(uint32_t off) const { return off < max_off ? off : max_off; }
    __device__ __forceinline__ uint32_t word(Addr a) const { return base[a >> 2]; }
    __device__ __forceinline__ uint32_t exact(uint32_t off) const {
        if (off >= len) return 0;
        uint32_t v = base[off >> 2];
        uint32_t rem = len - off;
        if (rem < 4) v &= (1u << (8 * rem)) - 1u;
        return v;
    }
    __device__ __forceinline__ void sink(uint32_t, uint32_t) const {}
    __device__ __forceinline__ void ready(uint32_t) const {}
};

// A data block body that the producer waves of the same workgroup are still
// assembling in the output block: before the chain loads the words of a
// group it waits until the producer's LDS progress word covers them. The
// producer publishes progress in whole 256-byte units (or the full length),
// after its stores have completed, so every cache line the chain pulls into
// L1 is already final.
struct BodyMsg {
    using Addr = const uint8_t *;
    const uint8_t *base;
    uint32_t len;
    uint32_t max_off;
    const uint32_t *prog; // LDS
    uint32_t *err;        // JobResultDev.invariant: set if the producer never delivers
    mutable uint32_t seen = 0; // progress already acquired: no LDS read, no fence below it
    uint32_t *cons = nullptr;  // LDS: this chain's position, for the producer's throttle
    __device__ __forceinline__ BodyMsg(const uint8_t *b, uint32_t l, const uint32_t *p, uint32_t *e, uint32_t *c)
        : base(b), len(l), max_off(l >= 4 ? l - 4 : 0), prog(p), err(e), cons(c) {}
    __device__ __forceinline__ Addr addr(uint32_t off) const { return base + (off < max_off ? off : max_off); }
    __device__ __forceinline__ uint32_t word(Addr a) const { return gld<uint32_t>(a); }
    __device__ __forceinline__ uint32_t exact(uint32_t off) const { return off < len ? gld<uint32_t>(base + off) : 0u; }
    __device__ __forceinline__ void sink(uint32_t, uint32_t) const {}
    __device__ __forceinline__ void ready(uint32_t upto) const {
        const uint32_t need = upto < len ? upto : len;
        if ((threadIdx.x & 31) == 0) __hip_atomic_store(cons, need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        // Whole wave: both 32-lane groups' blocks covered by what was acquired.
        if (!__any(need > seen)) return;
        uint32_t have = 0;
        for (uint32_t spins = 0;; spins++) {
            have = __hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            const bool late = have < need;
            if (!__any(late)) break;
            if (spins > (1u << 22)) { // bounded: report instead of hanging
                if (late) gst<uint32_t>(err, 0xdeadu);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        seen = have; // everything published up to `have` is now visible to this wave
    }
};

// One AEGIS update step with the round key fetched by VALU lane moves instead
// of LDS: row_ror:12 brings quad p+1 within a 16-lane row, and quads 3 and 7
// of a 32-lane group take it from the other row of the pair, which
// permlane16_swap supplies. The four table reads are issued first; the key
// and message word are folded in under their latency (tools/aegis_lab.hip:
// 59 vs 64 ns per update at one wave per SIMD).
__device__ __forceinline__ uint32_t key_valu(uint32_t x) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t r = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x12C, 0xf, 0xf, false); // row_ror:12
    const auto sw = __builtin_amdgcn_permlane16_swap(r, r, false, false);
    const uint32_t other = (lane & 16) ? sw[0] : sw[1];
    return ((lane & 15) >= 12) ? other : r;
}

struct StepValuKey {
    __device__ static __forceinline__ uint32_t step(const uint32_t *sT, const TableBase &tb, uint32_t, uint32_t x,
                                                    uint32_t m) {
        const uint32_t a0 = __builtin_amdgcn_perm(x, tb.lo, 0x03020400u);
        const uint32_t a1 = __builtin_amdgcn_perm(x, tb.lo, 0x03020500u);
        const uint32_t a2 = __builtin_amdgcn_perm(x, tb.hi, 0x03020600u);
        const uint32_t a3 = __builtin_amdgcn_perm(x, tb.hi, 0x03020700u);
        const uint32_t t0 = lds_u32(sT, a0);
        const uint32_t t1 = lds_u32(sT, a1 + 128);
        const uint32_t t2 = lds_u32(sT, a2);
        const uint32_t t3 = lds_u32(sT, a3 + 128);
        uint32_t r = (key_valu(x) ^ m) ^ t0;
        r ^= quad_perm<1, 2, 3, 0>(t1);
        r ^= quad_perm<2, 3, 0, 1>(t2);
        r ^= quad_perm<3, 0, 1, 2>(t3);
        return r;
    }
};

// Compact T-tables (the chain server, round 5): T0 and T2 only, each
// replicated once per bank as the full layout is, in 64 KiB — entry T0[b]
// for lane bank k at b * 256 + k * 4, T2[b] at b * 256 + 128 + k * 4 — and
// T1 = rotl(T0, 8), T3 = rotl(T2, 8) (AES: T_r[x] = rotl(T0[x], 8r)). Two
// v_alignbit_b32 per column step buy back 64 KiB of each chain CU's LDS, so
// a front's workgroups (16-52 KiB: merges, sorts) fit beside the server's.
constexpr uint32_t kCompactTableBytes = 65536;
constexpr uint32_t kCompactTableDwords = kCompactTableBytes / 4;

__device__ __forceinline__ void load_tables_compact(uint32_t *sT) {
    for (uint32_t i = threadIdx.x; i < kCompactTableDwords; i += blockDim.x) {
        const uint32_t b = i >> 6, half = (i >> 5) & 1;
        sT[i] = c_aes.t[half ? 2 : 0][b];
    }
}

__device__ __forceinline__ uint32_t rotl8(uint32_t v) { return __builtin_amdgcn_alignbit(v, v, 24); }

struct StepCompact {
    __device__ static __forceinline__ uint32_t step(const uint32_t *sT, const TableBase &tb, uint32_t key_src,
                                                    uint32_t x, uint32_t m) {
        const uint32_t key = bpermute(key_src, x);
        const uint32_t a0 = __builtin_amdgcn_perm(x, tb.lo, 0x03020400u);
        const uint32_t a1 = __builtin_amdgcn_perm(x, tb.lo, 0x03020500u);
        const uint32_t a2 = __builtin_amdgcn_perm(x, tb.lo, 0x03020600u);
        const uint32_t a3 = __builtin_amdgcn_perm(x, tb.lo, 0x03020700u);
        const uint32_t t0 = lds_u32(sT, a0);
        const uint32_t t1 = rotl8(lds_u32(sT, a1));
        const uint32_t t2 = lds_u32(sT, a2 + 128);
        const uint32_t t3 = rotl8(lds_u32(sT, a3 + 128));
        uint32_t r = (key ^ m) ^ t0;
        r ^= quad_perm<1, 2, 3, 0>(t1);
        r ^= quad_perm<2, 3, 0, 1>(t2);
        r ^= quad_perm<3, 0, 1, 2>(t3);
        return r;
    }
};

// Shared T-tables (index blocks, round 5): the four tables once, T_r[b] at
// dword r * 256 + b — 4 KiB instead of 128. Lanes whose bytes fall in one
// bank serialise, which costs nothing that matters for an index block's
// short message, and the index-block workgroup (4 KiB of tables + its 16 KiB
// image) starts on a CU beside a chain workgroup's 136 KiB instead of
// waiting for one to leave (config 2: k_index_blocks ~1.1 ms of which ~1 ms
// waiting).
constexpr uint32_t kSharedTableDwords = 1024;

struct StepShared {
    __device__ static __forceinline__ uint32_t step(const uint32_t *sT, const TableBase &, uint32_t key_src,
                                                    uint32_t x, uint32_t m) {
        const uint32_t key = bpermute(key_src, x);
        const uint32_t t0 = sT[x & 0xffu];
        const uint32_t t1 = sT[256 + ((x >> 8) & 0xffu)];
        const uint32_t t2 = sT[512 + ((x >> 16) & 0xffu)];
        const uint32_t t3 = sT[768 + (x >> 24)];
        uint32_t r = (key ^ m) ^ t0;
        r ^= quad_perm<1, 2, 3, 0>(t1);
        r ^= quad_perm<2, 3, 0, 1>(t2);
        r ^= quad_perm<3, 0, 1, 2>(t3);
        return r;
    }
};

// The T-table layout a step reads, its loader, and the step the same
// kernel's header checksums use (full tables: VALU round keys; compact and
// shared: their own step).
template <class Step> struct TableLayout {
    static constexpr uint32_t kDwords = kTableDwords;
    using HeaderStep = StepValuKey;
    __device__ static __forceinline__ void load(uint32_t *sT) { load_tables(sT); }
};
template <> struct TableLayout<StepCompact> {
    static constexpr uint32_t kDwords = kCompactTableDwords;
    using HeaderStep = StepCompact;
    __device__ static __forceinline__ void load(uint32_t *sT) { load_tables_compact(sT); }
};
template <> struct TableLayout<StepShared> {
    static constexpr uint32_t kDwords = kSharedTableDwords;
    using HeaderStep = StepShared;
    __device__ static __forceinline__ void load(uint32_t *sT) {
        for (uint32_t i = threadIdx.x; i < kSharedTableDwords; i += blockDim.x) sT[i] = c_aes.t[i >> 8][i & 255];
    }
};

// A step with `kMaskedMsg` takes the message word and its lane masks (the
// lanes whose block absorbs it this step) instead of the selected word
// (tools/aegis_lab.hip: hand-scheduled variants, measured no faster alone).
template <class S, class = void> struct StepMasked {
    static constexpr bool value = false;
};
template <class S> struct StepMasked<S, decltype((void)S::kMaskedMsg)> {
    static constexpr bool value = S::kMaskedMsg;
};

// AEGIS-128L MAC of one message per 32-lane group. The two groups of a wave
// may absorb messages of different lengths: both lengths are read into
// scalars, so the control flow stays wave-uniform. Returns column c of the
// 128-bit tag in every lane (c = lane & 3).
//
// Schedule, in 8-update windows (256 message bytes): whole windows of the
// shorter message run in the lean loop (`fast`, pure absorb); the windows
// where the shorter message ends (its partial tail and 7 finalisation
// updates) run per-step mode selection (`slow`); then the longer message
// continues in the lean loop (the finished group's lanes compute junk, its
// tag is already captured) and ends the same way. Every load stays inside
// its own group's message (addresses are clamped to it).
template <class Msg, class Step = StepValuKey, uint32_t kGroup = 8>
__device__ __forceinline__ uint32_t aegis_mac32(const uint32_t *sT, const Msg &msg) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t g = lane & 31, half = lane & 32;
    const uint32_t p = g >> 2, c = g & 3;
    const uint32_t key_src = (half + (((p + 1) & 7) << 2) + c) << 2; // quad p+1, same column

    const TableBase tb;
    uint32_t x = c_seed.s[p][c];
    const uint32_t len = msg.len; // this group's length
    const uint32_t n_abs = (len + 31) >> 5;
    const uint32_t len_0 = __builtin_amdgcn_readlane(len, 0), len_1 = __builtin_amdgcn_readlane(len, 32);
    const uint32_t abs_0 = (len_0 + 31) >> 5, abs_1 = (len_1 + 31) >> 5;
    const uint32_t len_s = len_0 < len_1 ? len_0 : len_1, len_l = len_0 < len_1 ? len_1 : len_0;

    // Which steps (u mod 4) inject a message word into this lane, and where
    // that word sits inside each 256-byte (8-update) window.
    const uint32_t k_lo = (3 - p) & 3;
    const uint32_t lab_lo = (p + k_lo + 1) & 7; // 0 -> M0, 4 -> M1
    const uint32_t off_lo = 32 * k_lo + 4 * (lab_lo + c);
    const uint32_t off_hi = 32 * (k_lo + 4) + 4 * ((lab_lo ^ 4) + c);
    bool need[4];
    uint64_t need_m[4];
    uint32_t need_v[4];
#pragma unroll
    for (int k = 0; k < 4; k++) {
        need[k] = ((p + k + 1) & 3) == 0;
        need_m[k] = __ballot(need[k]);
        need_v[k] = need[k] ? ~0u : 0u;
    }

#define AEGIS_STEP(K, WLO, WHI)                                                   \
    do {                                                                          \
        if constexpr (StepMasked<Step>::value) {                                  \
            x = Step::step_m(sT, tb, key_src, x, (K) < 4 ? (WLO) : (WHI), need_m[(K)&3], need_v[(K)&3]); \
        } else {                                                                  \
            uint32_t m_ = need[(K)&3] ? ((K) < 4 ? (WLO) : (WHI)) : 0u;           \
            x = Step::step(sT, tb, key_src, x, m_);                               \
        }                                                                         \
    } while (0)

    // Lean loop over windows [w0, w1) of whole 32-byte blocks of both
    // messages, in groups of kGroup windows (64 updates, 2 KiB per message). At
    // the top of each group the words of the next group are loaded (a full
    // group ahead of use, so the compiler's loop back-edge vmcnt(0) finds
    // them landed) and the addresses of the group after resolved.
    // kGroup: windows per group (8: 64 updates, ~3.8 us, hide two dependent
    // gathers; the chain server's direct loads take 4, half the registers).
    auto fast = [&](uint32_t w0, uint32_t w1) {
        if (w0 >= w1) return;
        const uint32_t groups = (w1 - w0 + kGroup - 1) / kGroup;
        typename Msg::Addr ad[2 * kGroup];
        auto resolve = [&](uint32_t base) {
#pragma unroll
            for (int d = 0; d < kGroup; d++) {
                ad[2 * d] = msg.addr(base + 256 * d + off_lo);
                ad[2 * d + 1] = msg.addr(base + 256 * d + off_hi);
            }
        };
        uint32_t cur[2 * kGroup];
        msg.ready(256 * (w0 + kGroup));
        resolve(256 * w0);
#pragma unroll
        for (int i = 0; i < 2 * kGroup; i++) cur[i] = msg.word(ad[i]);
        resolve(256 * (w0 + kGroup));
        for (uint32_t grp = 0; grp < groups; grp++) {
            const uint32_t wg = w0 + kGroup * grp;
            uint32_t nxt[2 * kGroup];
            msg.ready(256 * (wg + 2 * kGroup));
#pragma unroll
            for (int i = 0; i < 2 * kGroup; i++) nxt[i] = msg.word(ad[i]);
            resolve(256 * (wg + 2 * kGroup));
#pragma unroll
            for (int d = 0; d < kGroup; d++) {
                if (wg + d < w1) {
                    msg.sink(256 * (wg + d) + off_lo, cur[2 * d]);
                    msg.sink(256 * (wg + d) + off_hi, cur[2 * d + 1]);
                }
            }
#pragma unroll
            for (int d = 0; d < kGroup; d++) {
                if (wg + d < w1) {
                    const uint32_t cl = cur[2 * d], ch = cur[2 * d + 1];
                    AEGIS_STEP(0, cl, ch);
                    AEGIS_STEP(1, cl, ch);
                    AEGIS_STEP(2, cl, ch);
                    AEGIS_STEP(3, cl, ch);
                    AEGIS_STEP(4, cl, ch);
                    AEGIS_STEP(5, cl, ch);
                    AEGIS_STEP(6, cl, ch);
                    AEGIS_STEP(7, cl, ch);
                }
            }
#pragma unroll
            for (int i = 0; i < 2 * kGroup; i++) cur[i] = nxt[i];
        }
    };
#undef AEGIS_STEP

    // Windows [w0, w1) with per-step modes: absorb (exact words, zero past
    // len), finalise (tmp = (LE64(len*8) || 0) ^ S2, injected 7 times), or
    // frozen once the group's 7 finalisation updates are done; the tag
    // (S0 ^ ... ^ S6) is captured right after the last one.
    uint32_t tmp = 0, tag = 0;
    auto slow = [&](uint32_t w0, uint32_t w1) {
        for (uint32_t w = w0; w < w1; w++) {
            const uint32_t o_lo = 256 * w + off_lo, o_hi = 256 * w + off_hi;
            msg.ready(256 * (w + 1));
            const uint32_t wl = msg.exact(o_lo), wh = msg.exact(o_hi);
            if (o_lo < len) msg.sink(o_lo, wl);
            if (o_hi < len) msg.sink(o_hi, wh);
#pragma unroll
            for (uint32_t k = 0; k < 8; k++) {
                const uint32_t u = 8 * w + k;
                if (u == abs_0 || u == abs_1) { // a group starts finalising (scalar test)
                    const uint32_t q2 = (2 - n_abs) & 7;
                    const uint64_t bits = (uint64_t)len * 8;
                    uint32_t t = bpermute((half + (q2 << 2) + c) << 2, x);
                    t ^= c == 0 ? (uint32_t)bits : c == 1 ? (uint32_t)(bits >> 32) : 0u;
                    if (u == n_abs) tmp = t;
                }
                const uint32_t word = u < n_abs ? (k < 4 ? wl : wh) : tmp;
                const uint32_t xn = Step::step(sT, tb, key_src, x, need[k & 3] ? word : 0u);
                x = u < n_abs + 7 ? xn : x;
                if (u + 1 == abs_0 + 7 || u + 1 == abs_1 + 7) { // a group has finished (scalar test)
                    const uint32_t q7 = (7 - (n_abs + 7)) & 7;
                    const uint32_t s7 = bpermute((half + (q7 << 2) + c) << 2, x);
                    uint32_t t = x;
                    t ^= (uint32_t)__shfl_xor((int)t, 4, 64);
                    t ^= (uint32_t)__shfl_xor((int)t, 8, 64);
                    t ^= (uint32_t)__shfl_xor((int)t, 16, 64);
                    if (u + 1 == n_abs + 7) tag = t ^ s7;
                }
            }
        }
    };

    const uint32_t win_s = len_s >> 8, win_l = len_l >> 8;    // whole windows
    const uint32_t end_s = (((len_s + 31) >> 5) + 14) >> 3;    // windows until finalised
    const uint32_t end_l = (((len_l + 31) >> 5) + 14) >> 3;
    fast(0, win_s);
    if (end_s <= win_l) {
        slow(win_s, end_s);
        fast(end_s, win_l);
        slow(win_l, end_l);
    } else {
        slow(win_s, end_l);
    }
    return tag;
}

// --------------------------------------------------------------------------
// Kernels.
// --------------------------------------------------------------------------

// tbc_checksum_batch: two messages per wave, one per 32-lane group (an odd
// last message is computed by both groups, written once). Every pointer must
// be readable (the host substitutes a valid one for empty messages).
__global__ __launch_bounds__(1024) void k_checksum_batch(const uint64_t *ptrs, const uint64_t *lens, uint32_t count,
                                                       uint8_t *out) {
    __shared__ uint32_t sT[kTableDwords];
    load_tables(sT);
    __syncthreads();
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (2 * wave >= count) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t mine = 2 * wave + (lane >> 5);
    const uint32_t i = mine < count ? mine : mine - 1;
    GlobalMsg m((const uint8_t *)ptrs[i], (uint32_t)lens[i]);
    uint32_t tag = aegis_mac32(sT, m);
    if ((lane & 31) < 4 && mine < count) gst<uint32_t>(out + 16 * (size_t)i + 4 * (lane & 3), tag);
}

// ManifestLog.close_block (src/lsm/manifest_log.zig:876-952) of manifest
// blocks already staged in the grid (header fields packed by the host, entries
// in the body, zero padding): the body checksums, one message per 32-lane
// group, in parallel ...
__global__ __launch_bounds__(1024) void k_manifest_bodies(const uint64_t *addresses, uint32_t count,
                                                          uint8_t *grid_base, uint32_t block_size) {
    __shared__ uint32_t sT[kTableDwords];
    load_tables(sT);
    __syncthreads();
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (2 * wave >= count) return;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t mine = 2 * wave + (lane >> 5);
    const uint32_t i = mine < count ? mine : mine - 1;
    uint8_t *blk = grid_base + (size_t)(addresses[i] - 1) * block_size;
    GlobalMsg m(blk + kHeaderSize, gld<uint32_t>(blk + 96) - kHeaderSize);
    const uint32_t tag = aegis_mac32(sT, m);
    if ((lane & 31) < 4 && mine < count) gst<uint32_t>(blk + 32 + 4 * (lane & 3), tag); // set_checksum_body
}

// ... then the header chain, in log order on one wave: each header's metadata
// links the previous block's header checksum (the first block's comes from
// the host, or from the header of `previous_address` in the grid, written by
// an earlier close on this stream), then set_checksum over [16, 256).
//
// The grid's previous block is only linked if it is a verified manifest block
// (BlockType.manifest = 3, schema.zig:63): otherwise nothing is chained, the
// closed blocks keep a zero header checksum (so any later read fails
// read_block_validate), their verified bytes are cleared (an address reused
// after a checkpoint may still be marked from its earlier block) and the
// refusal is reported in the engine's error word (tbc_synchronize returns
// TBC_ERR_BLOCK_INVALID). Linked blocks are marked verified here, one store
// per block.
__global__ __launch_bounds__(64) void k_manifest_chain(const uint64_t *addresses, uint32_t count, uint8_t *grid_base,
                                                       uint32_t block_size, uint64_t previous_address,
                                                       const uint64_t *previous_checksum, uint8_t *verified,
                                                       uint32_t *error) {
    __shared__ uint32_t sT[kTableDwords];
    __shared__ uint32_t hdr[64];
    const uint32_t lane = threadIdx.x;
    if (!previous_checksum && previous_address) {
        const uint8_t *pb = grid_base + (size_t)(previous_address - 1) * block_size;
        if (!verified[previous_address - 1] || pb[240] != 3) { // not a trusted manifest block: refuse to link
            for (uint32_t i = lane; i < count; i += 64) verified[addresses[i] - 1] = 0;
            for (uint32_t i = 0; i < count; i++)
                if (lane < 4) gst<uint32_t>(grid_base + (size_t)(addresses[i] - 1) * block_size + 4 * lane, 0u);
            if (lane == 0) gst<uint32_t>(error, 1u);
            return;
        }
    }
    load_tables(sT);
    __syncthreads();
    uint32_t prev = 0; // lane c < 4: column c of the previous block's checksum
    if (lane < 4) {
        if (previous_checksum)
            prev = (uint32_t)(previous_checksum[lane >> 1] >> (32 * (lane & 1)));
        else if (previous_address)
            prev = gld<uint32_t>(grid_base + (size_t)(previous_address - 1) * block_size + 4 * lane);
    }
    for (uint32_t i = 0; i < count; i++) {
        uint8_t *blk = grid_base + (size_t)(addresses[i] - 1) * block_size;
        hdr[lane] = gld<uint32_t>(blk + 4 * lane);
        __builtin_amdgcn_wave_barrier();
        if (lane < 4) {
            hdr[32 + lane] = prev; // Metadata.previous_manifest_block_checksum
            gst<uint32_t>(blk + 128 + 4 * lane, prev);
        }
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        LdsMsg m(hdr + 4, kHeaderSize - 16);
        const uint32_t tag = aegis_mac32(sT, m);
        // Lanes c < 4 of the lower group hold column c of the tag.
        if (lane < 4) gst<uint32_t>(blk + 4 * lane, tag);
        prev = lane < 4 ? tag : 0u;
        if (lane == 0) verified[addresses[i] - 1] = 1; // engine-written: trusted like compaction outputs
        __builtin_amdgcn_wave_barrier();
    }
}

// grid.read_block_validate (src/vsr/grid.zig:1059-1084) for a batch of
// blocks: one wave per block, the lower 32-lane group checksums the header
// (bytes [16, 256)), the upper group the body ([256, size)); then the checks
// in the reference's order. Result codes: tbc_block_check (tbc.h).
// One wave: the checks of read_block_validate in its order; the result is
// valid in lane 0.
__device__ __forceinline__ uint32_t validate_block_wave(const uint32_t *sT, const uint8_t *blk, uint32_t block_size,
                                                        uint64_t expect_lo, uint64_t expect_hi, uint64_t address) {
    const uint32_t lane = threadIdx.x & 63, g = lane & 31;
    const uint32_t size = gld<uint32_t>(blk + 96);
    const bool size_ok = size >= kHeaderSize && size <= block_size;
    const bool upper = lane >= 32;
    GlobalMsg m(upper ? blk + kHeaderSize : blk + 16, upper ? (size_ok ? size - kHeaderSize : 0u) : 240u);
    const uint32_t tag = aegis_mac32(sT, m);
    // Lane g < 4 of each group compares its column with the stored checksum.
    const uint32_t stored = g < 4 ? gld<uint32_t>(blk + (upper ? 32 : 0) + 4 * g) : tag;
    const uint64_t bad = __ballot(tag != stored);
    const bool header_ok = (bad & 0xfull) == 0, body_ok = ((bad >> 32) & 0xfull) == 0;
    if (!header_ok) return 1;                                           // invalid_checksum
    if (blk[110] != 20) return 2;                                       // unexpected_command (Command.block)
    if (!size_ok) return 6;                                             // size out of bounds (reference asserts)
    if (!body_ok) return 3;                                             // invalid_checksum_body
    if (gld<uint64_t>(blk) != expect_lo || gld<uint64_t>(blk + 8) != expect_hi) return 4; // unexpected_checksum
    if (gld<uint64_t>(blk + 224) != address) return 5;                  // address (reference asserts)
    return 0;
}

__global__ __launch_bounds__(1024) void k_validate_blocks(const uint64_t *ptrs, const uint64_t *expect, uint32_t count,
                                                          uint32_t block_size, uint8_t *out) {
    __shared__ uint32_t sT[kTableDwords];
    load_tables(sT);
    __syncthreads();
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (wave >= count) return;
    const uint32_t r = validate_block_wave(sT, (const uint8_t *)ptrs[wave], block_size, expect[3 * wave],
                                           expect[3 * wave + 1], expect[3 * wave + 2]);
    if ((threadIdx.x & 63) == 0) out[wave] = (uint8_t)r;
}

__device__ __forceinline__ void report_block_error(uint32_t *slot, uint32_t code) {
    uint32_t expected = 0;
    __hip_atomic_compare_exchange_strong(slot, &expected, code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
}

// Grid inputs of a batch that were staged from storage (unverified):
// read_block_validate, one wave per block, failures reported on the owning
// job (first code wins), validated blocks marked trusted. Workgroups whose
// blocks are all verified leave before loading the tables.
__global__ __launch_bounds__(1024) void k_grid_validate(const InputCheck *checks, uint32_t count, uint8_t *verified,
                                                        const JobDesc *jobs, int njobs, JobResultDev *res,
                                                        uint32_t block_size) {
    __shared__ uint32_t sT[kTableDwords];
    __shared__ uint32_t s_any;
    const uint32_t wave = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (threadIdx.x == 0) s_any = 0;
    __syncthreads();
    InputCheck c{};
    bool todo = false;
    if (wave < count) {
        c = checks[wave];
        todo = c.address && !verified[c.address - 1];
    }
    if (todo && (threadIdx.x & 63) == 0) atomicOr(&s_any, 1u);
    __syncthreads();
    if (!s_any) return;
    load_tables(sT);
    __syncthreads();
    if (!todo) return;
    uint32_t r = validate_block_wave(sT, (const uint8_t *)(uintptr_t)c.ptr, block_size, c.checksum[0],
                                     c.checksum[1], c.address);
    if (r == 0) r = grid_header_check(job_of_result(jobs, njobs, c.job), c, block_size);
    if ((threadIdx.x & 63) == 0) {
        if (r) report_block_error(&res[c.job].block_error, r);
        else verified[c.address - 1] = 1;
    }
}

// Key (as 4 little-endian limbs) of a value; see composite_key.zig:48-50,
// groove.zig:27-29, 59-61.
__device__ __forceinline__ void value_key(const JobDesc &j, const uint8_t *v, uint64_t k[4]) {
    k[1] = k[2] = k[3] = 0;
    switch (j.key_kind) {
    case kKeyTimestamp: k[0] = ld64(v + j.timestamp_offset) & ~kTombstoneBit; break;
    case kKeyIdU128: k[0] = ld64(v); k[1] = ld64(v + 8); break;
    case kKeyCompositeU64: k[0] = ld64(v + 8) & ~kTombstoneBit; k[1] = ld64(v); break;
    default: k[0] = ld64(v + 16) & ~kTombstoneBit; k[1] = ld64(v); k[2] = ld64(v + 8); break;
    }
}

// Header.Block dword `i` (message_header.zig:1153-1178) for a data or index block.
struct HeaderFields {
    uint64_t cluster_lo, cluster_hi, address, snapshot;
    uint32_t size;
    uint32_t meta0, meta1, meta2, meta3; // first 14 metadata bytes as dwords (u32,u32,u32,u16)
    uint32_t block_type;
};

__device__ __forceinline__ uint32_t header_dword(const HeaderFields &h, uint32_t i, uint32_t tag_c) {
    switch (i) {
    case 8: case 9: case 10: case 11: return tag_c; // checksum_body (caller passes column i-8)
    case 20: return (uint32_t)h.cluster_lo;
    case 21: return (uint32_t)(h.cluster_lo >> 32);
    case 22: return (uint32_t)h.cluster_hi;
    case 23: return (uint32_t)(h.cluster_hi >> 32);
    case 24: return h.size;
    case 27: return 20u << 16; // version 0, command .block = 20 (vsr.zig:196), replica 0
    case 32: return h.meta0;
    case 33: return h.meta1;
    case 34: return h.meta2;
    case 35: return h.meta3;
    case 56: return (uint32_t)h.address;
    case 57: return (uint32_t)(h.address >> 32);
    case 58: return (uint32_t)h.snapshot;
    case 59: return (uint32_t)(h.snapshot >> 32);
    case 60: return h.block_type;
    default: return 0;
    }
}

// Fill a 256-byte header in LDS (hdr: 64 dwords), checksum [16, 256), and
// return the header checksum column in every lane.
template <class Step = StepValuKey>
__device__ __forceinline__ uint32_t finish_header(const uint32_t *sT, uint32_t *hdr, const HeaderFields &h,
                                                  uint32_t body_tag) {
    const uint32_t lane = threadIdx.x & 63, g = lane & 31;
    // Lane g writes dwords g and g + 32; dwords 8..11 hold the body tag column g & 3.
    hdr[g] = header_dword(h, g, body_tag);
    hdr[g + 32] = header_dword(h, g + 32, body_tag);
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    LdsMsg m(hdr + 4, kHeaderSize - 16);
    uint32_t tag = aegis_mac32<LdsMsg, Step>(sT, m);
    return tag;
}

// Producer: assemble the body of data block k of job j (output values
// [k*vcm, k*vcm + cnt)) from the merge's masks, 64 merged positions per step.
// Lane l owns merged position 64w + l of tile t: its side (from-A bit), its
// input index (cursor + side bits below it), and, if it survives, its output
// position (cursor + survivor bits below it); survivors of this block copy
// their value into place with 16-byte loads and stores. Progress (body bytes
// final and visible) goes to *prog in 256-byte units, after the stores have
// completed, for the chain waves of the workgroup (BodyMsg::ready).

// A job whose survivors are under a quarter of its merged positions (heavy
// dedup, e.g. an object tree updated many times per key) leaves its survivors
// scattered: one producer wave gathering them sequentially cannot keep ahead
// of the chain. Such jobs' bodies are assembled beforehand by k_assemble,
// parallel over the whole chip, and their producers only publish.
__device__ __forceinline__ bool sparse_job(const JobDesc &j, const JobResultDev *res) {
    return res[j.job_index].value_count * 4 < (uint64_t)(j.a.n + j.b.n);
}


// Producer throttle: a speculated producer stays at most `lead` body bytes ahead of
// what its block's chain has asked for (BodyMsg::ready stores the chain's
// position in LDS). Unthrottled, a producer runs up to a whole block ahead of
// its chain at the start of the kernel, every producer of the chip at once;
// throttled, the input reads spread over the chain's time (config 2: 2.46 ->
// 2.36 ms). The chains' re-reads of the bodies still miss L2 at any lead
// from 4 to 64 KiB (256 blocks per XCD churn ~3 MiB of L2
// per chain step). The lead is at least one unpublished
// step, so a chain waiting for data never waits on its throttled producer;
// bounded anyway. The merge-path producer (produce_body) is not throttled:
// there it cost 2-4 % on configs 4 and 5. TBC_LEAD_BYTES overrides the lead
// for ablation builds.
#ifndef TBC_LEAD_BYTES
#define TBC_LEAD_BYTES 12288
#endif
constexpr uint32_t kLeadBytes = TBC_LEAD_BYTES;
__device__ __forceinline__ void throttle(const uint32_t *cons, uint32_t produced, uint32_t lead) {
    if (!cons) return;
    for (uint32_t spins = 0; spins < (1u << 21); spins++) {
        const uint32_t c = __hip_atomic_load(cons, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (produced <= c + lead) return;
        __builtin_amdgcn_s_sleep(2);
    }
}

__device__ __forceinline__ void produce_body(const JobDesc &j, uint32_t k, uint32_t cnt, const uint64_t *status,
                                             const uint64_t *masks, const uint32_t *block_tile,
                                             const SplitDesc *splits, uint8_t *body, uint32_t *prog,
                                             uint32_t *err, uint64_t *stage) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t lt = (1ull << lane) - 1;
    const uint32_t vs = j.value_size;
    const uint32_t n = j.a.n + j.b.n;
    const uint64_t out_begin = (uint64_t)k * j.vcm, out_end = out_begin + cnt;
    const uint32_t len = cnt * vs;
    uint32_t t = __builtin_amdgcn_readfirstlane(gld<uint32_t>(block_tile + j.dblock_base + k));
    const SplitDesc sp = splits[j.split_base + t];
    uint64_t out_cur = gld<uint64_t>(status + j.tile_base + t) >> 32;
    uint32_t a_cur = sp.i, b_cur = t * kMergeTile - sp.i;
    SegCursor ca, cb;
    ca.init(j.a, sp.seg_a);
    cb.init(j.b, sp.seg_b);
    // A tile's 64 mask words (32 survivor, 32 from-A) arrive in ONE load, one
    // word per lane, and the next tile's are in flight meanwhile: walking a
    // word is register work, so sparse survivors (heavy dedup, e.g. 2 updates
    // per transfer over 10k accounts) cost no memory latency per word.
    constexpr uint32_t W = kMergeTile / 64;
    auto tile_words = [&](uint32_t tt) -> uint64_t {
        const uint32_t tc = tt < j.tile_count ? tt : j.tile_count - 1;
        return gld<uint64_t>(masks + (size_t)(j.tile_base + tc) * (2 * W) + lane);
    };
    auto word_of = [](uint64_t v, uint32_t src) -> uint64_t {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, (int)src);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), (int)src);
        return (uint64_t)hi << 32 | lo;
    };
    uint64_t cur = tile_words(t), nxt = tile_words(t + 1);
    // Survivors are staged as (source, destination) pairs in this wave's LDS
    // slots and copied 64 at a time: dense words (64 survivors) flush every
    // word as before, sparse ones (heavy dedup: ~1 survivor per word) share
    // one memory round trip per 64 survivors instead of one per word.
    uint64_t *st_src = stage, *st_dst = stage + 64;
    const uint32_t cpv_log = __builtin_ctz(vs >> 4);
    uint32_t pend = 0, since = 0;
    auto flush = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        copy_staged(st_src, st_dst, pend, cpv_log);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        pend = 0;
        since++;
    };
    uint32_t w = 0;
    while (out_cur < out_end) {
        const uint64_t sm = word_of(cur, w), am = word_of(cur, W + w);
        const uint32_t pos0 = t * kMergeTile + 64 * w;
        const uint64_t valid = n - pos0 >= 64 ? ~0ull : ((1ull << (n - pos0)) - 1);
        const uint32_t ns = __builtin_popcountll(sm);
        if (ns && out_cur + ns > out_begin) {
            ca.advance(a_cur);
            cb.advance(b_cur);
            const uint64_t o = out_cur + __builtin_popcountll(sm & lt);
            const bool mine = ((sm >> lane) & 1) && o >= out_begin && o < out_end;
            const uint64_t mm = __ballot(mine);
            const uint32_t m_cnt = __builtin_popcountll(mm);
            if (pend + m_cnt > 64) flush();
            if (mine) {
                const bool from_a = (am >> lane) & 1;
                const uint8_t *src = from_a ? ca.elem(a_cur + __builtin_popcountll(am & lt), vs)
                                            : cb.elem(b_cur + __builtin_popcountll(valid & ~am & lt), vs);
                const uint32_t slot = pend + __builtin_popcountll(mm & lt);
                st_src[slot] = (uint64_t)(uintptr_t)src;
                st_dst[slot] = (uint64_t)(uintptr_t)(body + (size_t)(o - out_begin) * vs);
            }
            pend += m_cnt;
        }
        a_cur += __builtin_popcountll(am);
        b_cur += __builtin_popcountll(valid & ~am);
        out_cur += ns;
        if (++w == W) {
            w = 0;
            if (++t >= j.tile_count && out_cur < out_end) { // masks disagree with the scan: report, release
                if (lane == 0) gst<uint32_t>(err, 0xbad0u);
                out_cur = out_end;
            }
            cur = nxt;
            nxt = tile_words(t + 1);
        }
        if (pend == 64) flush();
        // Publish after every 4 flushes (and at the end): stores complete,
        // then progress (whole 256-byte units of the flushed prefix).
        const bool end = out_cur >= out_end;
        if (end && pend) flush();
        if (since >= 4 || end) {
            since = 0;
            const uint64_t done = (out_cur < out_end ? out_cur : out_end) - pend;
            const uint32_t bytes = done > out_begin ? (uint32_t)(done - out_begin) * vs : 0u;
            const uint32_t pub = bytes >= len ? len : (bytes & ~255u);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(prog, pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
}

// A 4-byte store; write-through (sc1: the line leaves this XCD's L2 at once)
// when WT, so another CU that acquires after a later signal of this wave
// sees it without a release fence (MI355X_MICROARCH.md, inter-workgroup
// visibility). The chain server's outputs are stored this way.
template <bool WT> __device__ __forceinline__ void st32(void *p, uint32_t v) {
    if constexpr (WT) __hip_atomic_store((uint32_t *)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else gst<uint32_t>(p, v);
}

// Data block k of job j, body checksummed (`body_tag`: column lane & 3 of
// the tag, per 32-lane group): header fields, header checksum, the header
// and the zeroed sector tail stored by the `writer` group.
template <bool WT = false, class Step = StepValuKey>
__device__ __forceinline__ void finish_data_block(const uint32_t *sT, uint32_t *hdr, const JobDesc &j, uint32_t k,
                                                  uint32_t cnt, uint32_t body_tag, bool writer) {
    const uint32_t slot = data_block_slot(k, j.dbcm);
    uint8_t *blk = block_ptr(j, slot);
    const uint32_t size = kHeaderSize + cnt * j.value_size;
    HeaderFields h;
    h.cluster_lo = j.cluster_lo;
    h.cluster_hi = j.cluster_hi;
    h.address = gld<uint64_t>(j.addresses + slot);
    h.snapshot = j.snapshot_min;
    h.size = size;
    h.meta0 = j.vcm;        // TableData.Metadata.value_count_max
    h.meta1 = cnt;          // .value_count
    h.meta2 = j.value_size; // .value_size
    h.meta3 = j.tree_id;    // .tree_id (u16), reserved = 0
    h.block_type = 5;       // BlockType.data (schema.zig:65)
    const uint32_t hdr_tag = finish_header<Step>(sT, hdr, h, body_tag);
    const uint32_t g = threadIdx.x & 31;
    if (g < 4) hdr[g] = hdr_tag;
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (writer) {
        st32<WT>(blk + 4 * g, hdr[g]);
        st32<WT>(blk + 4 * (g + 32), hdr[g + 32]);
        // Zero [size, sector_ceil(size)) (grid.zig:686).
        const uint32_t end = (uint32_t)sector_ceil(size);
        for (uint32_t o = size + 4 * g; o < end; o += 128) st32<WT>(blk + o, 0u);
    }
    __builtin_amdgcn_wave_barrier();
}

// Producer of a speculated job (TBC_COMPACTION_UNIQUE_KEYS): no merge pass ran.
// If no key occurs twice in A u B and no tombstone is dropped, every value
// survives (compaction.zig:483-559 dedup and :757-798 merge rules all keep
// it), so block k is merged positions [k * vcm, k * vcm + cnt) and the
// producer merges them itself, 64 outputs per step: lane l holds A[ia + l]
// and B[ib + l]; A[ia + l] lands at l + |{B-window keys < it}| and B[ib + l]
// at l + |{A-window keys <= it}| (A first on equal keys); the outputs below
// 64 are exactly the next 64 merged values. Both ranks are binary searches
// over the other window's keys by ds_bpermute (no LDS). The speculation
// holds iff no output key equals its merged predecessor's and, when dropping
// tombstones, no A output is a tombstone: an equal key of B for an A value is
// its lower bound in the B window (a B value equal to an A value follows it),
// equal keys inside a stream are adjacent lanes, and the values before the
// block on each side carry the check across blocks and steps. A broken
// speculation marks the job (JobResultDev.spec): the batch's second phase
// recomputes its blocks through the merge path, bit-exact; the chains of
// this pass absorb what was written and are overwritten.
//
// VW > 0 (values of 16 or 32 bytes, VW x 16 B): each lane loads its whole A
// and B value into registers with the window and stores it straight to its
// output slot, one memory round trip per step; the key is taken from the
// registers. VW = 0 (larger values, whose chains leave the producer more
// time): keys only, the outputs copied through the wave's LDS staging.
// Progress is published every other step, once the stores have completed.
template <int KIND>
__device__ __forceinline__ Key<KeyLimbs<KIND>::value> key_of_words(const uint64_t *w, uint32_t ts_word) {
    Key<KeyLimbs<KIND>::value> k;
    if constexpr (KIND == kKeyTimestamp) {
        uint64_t t = w[0];
#pragma unroll
        for (int q = 1; q < 4; q++)
            if (ts_word == (uint32_t)q) t = w[q];
        k.l[0] = t & ~kTombstoneBit;
    } else if constexpr (KIND == kKeyIdU128) {
        k.l[0] = w[0];
        k.l[1] = w[1];
    } else if constexpr (KIND == kKeyCompositeU64) {
        k.l[0] = w[1] & ~kTombstoneBit;
        k.l[1] = w[0];
    } else {
        k.l[0] = w[2] & ~kTombstoneBit;
        k.l[1] = w[0];
        k.l[2] = w[1];
    }
    return k;
}

template <int KIND, int VW>
__device__ __forceinline__ void produce_unique(const JobDesc &j, uint32_t k, uint32_t cnt, const SplitDesc &sp,
                                               uint8_t *body, uint32_t *prog, uint32_t *err, uint32_t *spec,
                                               uint64_t *stage, const uint32_t *cons) {
    constexpr int KL = KeyLimbs<KIND>::value;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t vs = j.value_size, ts = j.timestamp_offset, na = j.a.n, nb = j.b.n;
    const uint32_t len = cnt * vs;
    uint32_t ia = sp.i, ib = k * j.vcm - sp.i;
    SegCursor ca, cb;
    ca.init(j.a, sp.seg_a); // segment of A[max(ia - 1, 0)]
    cb.init(j.b, sp.seg_b); // segment of B[min(ib, nb - 1)]
    Key<KL> inf;
#pragma unroll
    for (int l = 0; l < KL; l++) inf.l[l] = ~0ull;
    // Keys of the values just before the block on each side.
    bool has_a = ia > 0, has_b = ib > 0;
    Key<KL> last_a = inf, last_b = inf;
    if (has_a) last_a = load_key<KIND>(ca.elem(ia - 1, vs), ts);
    if (has_b) {
        const uint32_t s = sp.pad; // segment of B[ib - 1]
        last_b = load_key<KIND>((const uint8_t *)(uintptr_t)gld<uint64_t>(j.b.seg_ptr + s) +
                                    (size_t)(ib - 1 - gld<uint32_t>(j.b.seg_pre + s)) * vs, ts);
    }
    uint64_t *st_src = stage, *st_dst = stage + 64;
    const uint32_t cpv_log = __builtin_ctz(vs >> 4);
    bool bad = false;
    // Window at (ia, ib): pointers and values or keys; invalid lanes +inf.
    const uint8_t *pa, *pb;
    u32x4 xa[VW > 0 ? VW : 1], xb[VW > 0 ? VW : 1];
    Key<KL> ka, kb;
    uint32_t nav, nbv;
    auto load_window = [&]() {
        ca.advance(ia);
        cb.advance(ib);
        nav = na - ia < 64 ? na - ia : 64;
        nbv = nb - ib < 64 ? nb - ib : 64;
        pa = lane < nav ? ca.elem(ia + lane, vs) : nullptr;
        pb = lane < nbv ? cb.elem(ib + lane, vs) : nullptr;
        if constexpr (VW > 0) {
#pragma unroll
            for (int q = 0; q < VW; q++) {
                xa[q] = pa ? gld<u32x4>(pa + 16 * q) : u32x4{0, 0, 0, 0};
                xb[q] = pb ? gld<u32x4>(pb + 16 * q) : u32x4{0, 0, 0, 0};
            }
        } else {
            ka = pa ? load_key<KIND>(pa, ts) : inf;
            kb = pb ? load_key<KIND>(pb, ts) : inf;
        }
    };
    auto words_key = [&](const u32x4 *x, bool valid) {
        uint64_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int q = 0; q < VW; q++) {
            w[2 * q] = (uint64_t)x[q].y << 32 | x[q].x;
            w[2 * q + 1] = (uint64_t)x[q].w << 32 | x[q].z;
        }
        return valid ? key_of_words<KIND>(w, ts >> 3) : inf;
    };
    load_window();
    uint32_t out = 0, since = 0, published = 0;
    while (out < cnt) {
        const uint32_t E = cnt - out < 64 ? cnt - out : 64;
        if constexpr (VW > 0) {
            ka = words_key(xa, pa != nullptr);
            kb = words_key(xb, pb != nullptr);
            // The window has landed, and the previous steps' stores were
            // issued before it (nothing after it): the wait is free; publish.
            if (out != published) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                if (lane == 0) __hip_atomic_store(prog, (out * vs) & ~255u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                published = out;
            }
        }
        // Ranks: lower bound of ka among the B window, upper bound of kb among the A window.
        uint32_t lo_a = 0, hi_a = nbv, lo_b = 0, hi_b = nav;
#pragma unroll
        for (int it = 0; it < 7; it++) {
            const uint32_t ma = (lo_a + hi_a) >> 1, mb = (lo_b + hi_b) >> 1;
            const Key<KL> at_b = key_of_lane(kb, ma < 63 ? ma : 63);
            const Key<KL> at_a = key_of_lane(ka, mb < 63 ? mb : 63);
            if (lo_a < hi_a) {
                if (key_lt(at_b, ka)) lo_a = ma + 1;
                else hi_a = ma;
            }
            if (lo_b < hi_b) {
                if (key_le(at_a, kb)) lo_b = mb + 1;
                else hi_b = mb;
            }
        }
        const uint32_t pos_a = lane + lo_a, pos_b = lane + lo_b;
        const bool ea = lane < nav && pos_a < E, eb = lane < nbv && pos_b < E;
        const uint32_t n_a = __builtin_popcountll(__ballot(ea)), n_b = __builtin_popcountll(__ballot(eb));
        // Equal neighbours (speculation broken) and dropped tombstones.
        const Key<KL> lb = key_of_lane(kb, lo_a < 63 ? lo_a : 63);
        const Key<KL> prev_a = key_of_lane(ka, lane ? lane - 1 : 0);
        const Key<KL> prev_b = key_of_lane(kb, lane ? lane - 1 : 0);
        bool eq = ea && lo_a < nbv && key_eq(lb, ka);
        eq |= ea && (lane ? key_eq(prev_a, ka) : (has_a && key_eq(last_a, ka)));
        eq |= eb && (lane ? key_eq(prev_b, kb) : (has_b && key_eq(last_b, kb)));
        if (j.drop_tombstones && ea) eq |= (ld64(pa + ts) >> 63) != 0;
        bad |= __ballot(eq) != 0;
        if (n_a + n_b != E) { // the windows always hold the next E values: a broken invariant
            if (lane == 0) gst<uint32_t>(err, 0xbad1u);
            bad = true;
            break;
        }
        if (n_a) last_a = key_of_lane(ka, n_a - 1), has_a = true;
        if (n_b) last_b = key_of_lane(kb, n_b - 1), has_b = true;
        if constexpr (VW > 0) {
            // Every output straight from its lane's registers.
            if (ea)
#pragma unroll
                for (int q = 0; q < VW; q++) gst<u32x4>(body + (size_t)(out + pos_a) * vs + 16 * q, xa[q]);
            if (eb)
#pragma unroll
                for (int q = 0; q < VW; q++) gst<u32x4>(body + (size_t)(out + pos_b) * vs + 16 * q, xb[q]);
            ia += n_a;
            ib += n_b;
            out += E;
            if (out < cnt) load_window();
        } else {
            // Stage this step's copies, then load the next window before copying.
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            if (ea) {
                st_src[pos_a] = (uint64_t)(uintptr_t)pa;
                st_dst[pos_a] = (uint64_t)(uintptr_t)(body + (size_t)(out + pos_a) * vs);
            }
            if (eb) {
                st_src[pos_b] = (uint64_t)(uintptr_t)pb;
                st_dst[pos_b] = (uint64_t)(uintptr_t)(body + (size_t)(out + pos_b) * vs);
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            ia += n_a;
            ib += n_b;
            out += E;
            throttle(cons, out * vs, 3 * 64 * vs > kLeadBytes ? 3 * 64 * vs : kLeadBytes);
            if (out < cnt) load_window();
            copy_staged(st_src, st_dst, E, cpv_log);
        }
        // VW = 0: publish every other step (and at the end): stores complete,
        // then progress in whole 256-byte units. VW > 0: at the end (else at
        // the next window's arrival).
        if (VW > 0 ? out >= cnt : (++since >= 2 || out >= cnt)) {
            since = 0;
            const uint32_t bytes = out * vs;
            const uint32_t pub = bytes >= len ? len : (bytes & ~255u);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(prog, pub, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }
    if (bad) {
        if (lane == 0) {
            __hip_atomic_store(spec, kSpecBroken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(j.spec_any, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        // The chains still run to the end of the block: release them.
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        if (lane == 0) __hip_atomic_store(prog, len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// Wide steps for small values (VW x 16 B, VW = 1 or 2): 128 outputs per
// memory round trip. Lane l holds A[ia + l + 64q] and B[ib + l + 64q] in slot
// q < 2 (whole values in registers). Only the A values are ranked among the
// B window (lower bound, binary search over window positions: lane m & 63,
// slot m >> 6, by ds_bpermute); a B value's position is its index plus the
// number of A values ranked at or before it, from a 128-bin histogram of
// the A ranks in the wave's LDS slot and a wave prefix sum. The speculation
// checks, stores and publication are produce_unique's.
template <int KL> __device__ __forceinline__ Key<KL> key_of_slot(const Key<KL> (&k)[2], uint32_t pos) {
    const Key<KL> k0 = key_of_lane(k[0], pos & 63), k1 = key_of_lane(k[1], pos & 63);
    return (pos >> 6) & 1 ? k1 : k0;
}

template <int KL> __device__ __forceinline__ Key<KL> key_readlane(const Key<KL> &k, uint32_t src) {
    Key<KL> r;
#pragma unroll
    for (int l = 0; l < KL; l++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)k.l[l], (int)src);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(k.l[l] >> 32), (int)src);
        r.l[l] = (uint64_t)hi << 32 | lo;
    }
    return r;
}

// Inclusive wave prefix sum by DPP (row shifts, then row broadcasts 15/31).
__device__ __forceinline__ uint32_t wave_scan_incl(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, true); // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, true); // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, true); // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, true); // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false); // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false); // row_bcast:31
    return x;
}

// Key of lane - 1 (wave_shr:1 DPP; lane 0 gets `first`).
template <int KL> __device__ __forceinline__ Key<KL> key_prev_lane(const Key<KL> &k, const Key<KL> &first) {
    Key<KL> r;
    const bool l0 = (threadIdx.x & 63) == 0;
#pragma unroll
    for (int l = 0; l < KL; l++) {
        const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)k.l[l], 0x138, 0xf, 0xf, false);
        const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(k.l[l] >> 32), 0x138, 0xf, 0xf,
                                                                  false);
        r.l[l] = l0 ? first.l[l] : ((uint64_t)hi << 32 | lo);
    }
    return r;
}

template <int KL> __device__ __forceinline__ Key<KL> key_lds(const uint64_t *keys, uint32_t pos) {
    Key<KL> r;
#pragma unroll
    for (int l = 0; l < KL; l++) r.l[l] = keys[l * 128 + pos];
    return r;
}

template <int KIND, int VW>
__device__ __forceinline__ void produce_unique_wide(const JobDesc &j, uint32_t k, uint32_t cnt, const SplitDesc &sp,
                                                    uint8_t *body, uint32_t *prog, uint32_t *err, uint32_t *spec,
                                                    uint64_t *stage, const uint32_t *cons) {
    constexpr int KL = KeyLimbs<KIND>::value;
    constexpr uint32_t W = 128;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t vs = j.value_size, ts = j.timestamp_offset, na = j.a.n, nb = j.b.n;
    const uint32_t len = cnt * vs;
    uint32_t ia = sp.i, ib = k * j.vcm - sp.i;
    SegCursor ca, cb;
    ca.init(j.a, sp.seg_a); // segment of A[max(ia - 1, 0)]
    cb.init(j.b, sp.seg_b); // segment of B[min(ib, nb - 1)]
    Key<KL> inf;
#pragma unroll
    for (int l = 0; l < KL; l++) inf.l[l] = ~0ull;
    bool has_a = ia > 0, has_b = ib > 0;
    Key<KL> last_a = inf, last_b = inf;
    if (has_a) last_a = load_key<KIND>(ca.elem(ia - 1, vs), ts);
    if (has_b) {
        const uint32_t s = sp.pad; // segment of B[ib - 1]
        last_b = load_key<KIND>((const uint8_t *)(uintptr_t)gld<uint64_t>(j.b.seg_ptr + s) +
                                    (size_t)(ib - 1 - gld<uint32_t>(j.b.seg_pre + s)) * vs, ts);
    }
    uint64_t *bkeys = stage;                     // KL x 128 keys of the B window
    uint32_t *hist = (uint32_t *)(stage + 3 * 128); // 128 bins
    bool bad = false;
    u32x4 xa[2][VW], xb[2][VW];
    bool va[2], vb[2];
    uint32_t nav, nbv;
    auto load_window = [&]() {
        ca.advance(ia);
        cb.advance(ib);
        nav = na - ia < W ? na - ia : W;
        nbv = nb - ib < W ? nb - ib : W;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const uint32_t idx = lane + 64 * q;
            va[q] = idx < nav;
            vb[q] = idx < nbv;
            const uint8_t *pa = va[q] ? ca.elem(ia + idx, vs) : nullptr;
            const uint8_t *pb = vb[q] ? cb.elem(ib + idx, vs) : nullptr;
#pragma unroll
            for (int v = 0; v < VW; v++) {
                xa[q][v] = pa ? gld<u32x4>(pa + 16 * v) : u32x4{0, 0, 0, 0};
                xb[q][v] = pb ? gld<u32x4>(pb + 16 * v) : u32x4{0, 0, 0, 0};
            }
        }
    };
    auto words = [&](const u32x4 *x, uint64_t (&w)[4]) {
        w[0] = w[1] = w[2] = w[3] = 0;
#pragma unroll
        for (int v = 0; v < VW; v++) {
            w[2 * v] = (uint64_t)x[v].y << 32 | x[v].x;
            w[2 * v + 1] = (uint64_t)x[v].w << 32 | x[v].z;
        }
    };
    load_window();
    uint32_t out = 0, published = 0;
    while (out < cnt) {
        const uint32_t E = cnt - out < W ? cnt - out : W;
        Key<KL> ka[2], kb[2];
        bool ta[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            uint64_t w[4];
            words(xa[q], w);
            ka[q] = va[q] ? key_of_words<KIND>(w, ts >> 3) : inf;
            ta[q] = (((ts >> 3) == 0 ? w[0] : (ts >> 3) == 1 ? w[1] : (ts >> 3) == 2 ? w[2] : w[3]) >> 63) != 0;
            words(xb[q], w);
            kb[q] = vb[q] ? key_of_words<KIND>(w, ts >> 3) : inf;
        }
        // The window has landed, and the previous steps' stores were issued
        // before it (nothing after it): the wait is free; publish.
        if (out != published) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(prog, (out * vs) & ~255u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            published = out;
        }
        // The B window's keys into this wave's LDS (limb-major, 128 per limb).
#pragma unroll
        for (int q = 0; q < 2; q++)
#pragma unroll
            for (int l = 0; l < KL; l++) bkeys[l * 128 + lane + 64 * q] = kb[q].l[l];
        hist[lane] = 0;
        hist[lane + 64] = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // A ranks among the B window (lower bound): the bucket of 16 among
        // eight splitters B[16s + 15] (uniform LDS reads, all independent;
        // positions past the window hold +inf), then a binary search of the
        // bucket in LDS.
        uint32_t lo[2] = {0, 0}, hi[2];
#pragma unroll
        for (int sp = 0; sp < 8; sp++) {
            const Key<KL> at = key_lds<KL>(bkeys, 16 * sp + 15);
#pragma unroll
            for (int q = 0; q < 2; q++) lo[q] += key_lt(at, ka[q]) ? 16u : 0u;
        }
#pragma unroll
        for (int q = 0; q < 2; q++) hi[q] = lo[q] + 15 < nbv ? lo[q] + 15 : nbv;
#pragma unroll
        for (int it = 0; it < 4; it++) {
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const uint32_t m = (lo[q] + hi[q]) >> 1;
                const Key<KL> at = key_lds<KL>(bkeys, m < W - 1 ? m : W - 1);
                if (lo[q] < hi[q]) {
                    if (key_lt(at, ka[q])) lo[q] = m + 1;
                    else hi[q] = m;
                }
            }
        }
        // Histogram of the A ranks, prefix: A values at or before each B position.
#pragma unroll
        for (int q = 0; q < 2; q++)
            if (va[q] && lo[q] < W) __hip_atomic_fetch_add(&hist[lo[q]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        uint32_t c0 = wave_scan_incl(hist[lane]), c1 = wave_scan_incl(hist[lane + 64]);
        c1 += __builtin_amdgcn_readlane((int)c0, 63);
        uint32_t pos_a[2], pos_b[2];
        bool ea[2], eb[2];
        pos_a[0] = lane + lo[0];
        pos_a[1] = lane + 64 + lo[1];
        pos_b[0] = lane + c0;
        pos_b[1] = lane + 64 + c1;
        uint32_t n_a = 0, n_b = 0;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            ea[q] = va[q] && pos_a[q] < E;
            eb[q] = vb[q] && pos_b[q] < E;
            n_a += __builtin_popcountll(__ballot(ea[q]));
            n_b += __builtin_popcountll(__ballot(eb[q]));
        }
        // Equal neighbours (speculation broken) and dropped tombstones.
        bool eq = false;
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const Key<KL> lb = key_lds<KL>(bkeys, lo[q] < W - 1 ? lo[q] : W - 1);
            eq |= ea[q] && lo[q] < nbv && key_eq(lb, ka[q]);
            const Key<KL> first_a = q == 0 ? last_a : key_readlane(ka[0], 63);
            const Key<KL> first_b = q == 0 ? last_b : key_readlane(kb[0], 63);
            const bool ha = q == 0 ? has_a : true, hb = q == 0 ? has_b : true;
            const Key<KL> pa_ = key_prev_lane(ka[q], first_a), pb_ = key_prev_lane(kb[q], first_b);
            eq |= ea[q] && (lane || ha) && key_eq(pa_, ka[q]);
            eq |= eb[q] && (lane || hb) && key_eq(pb_, kb[q]);
            if (j.drop_tombstones) eq |= ea[q] && ta[q];
        }
        bad |= __ballot(eq) != 0;
        if (n_a + n_b != E) { // the windows always hold the next E values: a broken invariant
            if (lane == 0) gst<uint32_t>(err, 0xbad2u);
            bad = true;
            break;
        }
        if (n_a) {
            const uint32_t t = n_a - 1;
            last_a = key_readlane(t < 64 ? ka[0] : ka[1], t & 63);
            has_a = true;
        }
        if (n_b) {
            const uint32_t t = n_b - 1;
            last_b = key_readlane(t < 64 ? kb[0] : kb[1], t & 63);
            has_b = true;
        }
#pragma unroll
        for (int q = 0; q < 2; q++) {
            if (ea[q])
#pragma unroll
                for (int v = 0; v < VW; v++) gst<u32x4>(body + (size_t)(out + pos_a[q]) * vs + 16 * v, xa[q][v]);
            if (eb[q])
#pragma unroll
                for (int v = 0; v < VW; v++) gst<u32x4>(body + (size_t)(out + pos_b[q]) * vs + 16 * v, xb[q][v]);
        }
        ia += n_a;
        ib += n_b;
        out += E;
        throttle(cons, out * vs, kLeadBytes);
        if (out < cnt) load_window();
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if (bad && lane == 0) {
        __hip_atomic_store(spec, kSpecBroken, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_add(j.spec_any, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) __hip_atomic_store(prog, len, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

template <int KIND>
__device__ __forceinline__ void produce_unique_vs(const JobDesc &j, uint32_t k, uint32_t cnt, const SplitDesc &sp,
                                                  uint8_t *body, uint32_t *prog, uint32_t *err, uint32_t *spec,
                                                  uint64_t *stage, const uint32_t *cons) {
    if (j.value_size == 32) produce_unique_wide<KIND, 2>(j, k, cnt, sp, body, prog, err, spec, stage, cons);
    else if (j.value_size == 16) produce_unique_wide<KIND, 1>(j, k, cnt, sp, body, prog, err, spec, stage, cons);
    else produce_unique<KIND, 0>(j, k, cnt, sp, body, prog, err, spec, stage, cons);
}

// Data blocks: data_block_finish (table.zig:306-384) for every output data
// block. Blocks are numbered batch-wide by their upper bound (job base + k).
// A workgroup holds C chain waves and 2C producer waves: chain wave c takes
// blocks 2w and 2w+1 (w = blockIdx * C + c), one per 32-lane group, whatever
// their lengths (aegis_mac32 takes two lengths), and producer 2c + h
// assembles block 2w + h in the output block while the chain absorbs it.
// Config 2's 2,016 blocks need 1,008 chain waves: one per SIMD. A group
// whose block does not exist (dedup left fewer blocks than the bound) mirrors
// its partner's block without writing, so all its loads stay valid.
//
// Throughput regime (many more blocks than SIMDs, e.g. config 5's 13,824
// blocks): `Fused = false`. The bodies are first assembled by k_assemble (one
// wave per block, every CU, no LDS tables: HBM-bound), then this kernel runs
// chain waves only, up to 16 per workgroup (4 per SIMD), so the AES rounds of
// four waves hide each other's LDS latency instead of one chain per SIMD
// waiting on it.
// Fused: C chain + 2C producer waves, C <= 4 (768 threads), so the kernel may
// use 168 VGPRs (3 waves per SIMD) and the producers do not spill.
constexpr uint32_t kMaxChainWaves = 4;
constexpr uint32_t kStageWords = 448; // producer LDS (u64): 3 x 128 B-window key limbs + 128 rank bins
constexpr uint32_t kMaxChainOnlyWaves = 16;
// Above this many chain waves (2 per SIMD) the two-pass path wins.
constexpr uint32_t kFusedMaxChainWaves = 2048;

template <bool Fused, class ChainStep = StepBpermute, uint32_t kHdrMax = (Fused ? kMaxChainWaves : kMaxChainOnlyWaves)>
__device__ __forceinline__ void data_blocks(const JobDesc *jobs, int njobs, uint32_t total, const JobResultDev *res,
                                            const uint64_t *status, const uint64_t *masks,
                                            const uint32_t *block_tile, const SplitDesc *splits,
                                            uint32_t chain_waves, const uint32_t *ready, const SplitDesc *bsplits,
                                            uint32_t phase, uint32_t bid) {
    constexpr uint32_t kHdrWaves = kHdrMax; // header scratch: one row per chain wave of the workgroup
    using Layout = TableLayout<ChainStep>;
    __shared__ uint32_t sT[Layout::kDwords];
    __shared__ uint32_t sHdr[kHdrWaves][2][64];
    __shared__ uint32_t sProg[2 * kMaxChainWaves];
    __shared__ uint32_t sCons[2 * kMaxChainWaves]; // the chains' positions (body bytes needed so far)
    // Producer LDS: copy staging (merge-path producers), or the speculated
    // producers' B window keys + rank histogram; everything the tables,
    // headers and progress words leave of the CU's 160 KiB.
    __shared__ uint64_t sStage[Fused ? 2 * kMaxChainWaves : 1][kStageWords];
    const uint32_t C = chain_waves;
    auto locate = [&](uint32_t m, int &ji_, uint32_t &k_) {
        ji_ = find_job(jobs, njobs, m, [](const JobDesc &d) { return d.dblock_base; });
        k_ = m - jobs[ji_].dblock_base + jobs[ji_].block_lo;
        return m < total && k_ < res[jobs[ji_].job_index].data_block_count &&
               (phase != 1 || !phase_skips(jobs[ji_], res, phase));
    };
    if (phase == 1) { // recomputation of broken speculations: leave at once if none of ours
        int ji_;
        uint32_t k_;
        const bool mine = threadIdx.x < 2 * C && locate(2 * bid * C + threadIdx.x, ji_, k_);
        if (!__syncthreads_or(mine)) return;
    }
    Layout::load(sT);
    if (threadIdx.x < 2 * kMaxChainWaves) sProg[threadIdx.x] = sCons[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t wave_in_block = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63;
    auto block_count = [&](const JobDesc &j, uint32_t k_) {
        const uint64_t n_out = res[j.job_index].value_count;
        const uint64_t first = (uint64_t)k_ * j.vcm;
        return (uint32_t)((n_out - first) < j.vcm ? (n_out - first) : j.vcm);
    };
    int ji;
    uint32_t k;
    if (Fused && wave_in_block >= C) { // producer
        const uint32_t p = wave_in_block - C;
        const uint32_t mine = 2 * (bid * C + (p >> 1)) + (p & 1);
        if (!locate(mine, ji, k)) return;
        const JobDesc &j = jobs[ji];
        if (j.unique && phase != 1) { // speculated: merges the block's values itself
            uint8_t *blk = block_ptr(j, data_block_slot(k, j.dbcm));
            const SplitDesc sp = bsplits[j.dblock_base + k];
            uint32_t *err = const_cast<uint32_t *>(&res[j.job_index].invariant);
            uint32_t *spec = const_cast<uint32_t *>(&res[j.job_index].spec);
            uint64_t *stage = sStage[Fused ? p : 0];
            const uint32_t cnt = block_count(j, k);
            switch (j.key_kind) {
            case kKeyTimestamp:
                produce_unique_vs<kKeyTimestamp>(j, k, cnt, sp, blk + kHeaderSize, &sProg[p], err, spec, stage,
                                                   &sCons[p]);
                break;
            case kKeyIdU128:
                produce_unique_vs<kKeyIdU128>(j, k, cnt, sp, blk + kHeaderSize, &sProg[p], err, spec, stage,
                                                   &sCons[p]);
                break;
            case kKeyCompositeU64:
                produce_unique_vs<kKeyCompositeU64>(j, k, cnt, sp, blk + kHeaderSize, &sProg[p], err, spec, stage,
                                                   &sCons[p]);
                break;
            default:
                produce_unique_vs<kKeyCompositeU128>(j, k, cnt, sp, blk + kHeaderSize, &sProg[p], err, spec, stage,
                                                   &sCons[p]);
                break;
            }
            return;
        }
        if (sparse_job(j, res)) { // body written by k_assemble (stream order)
            if (lane == 0)
                __hip_atomic_store(&sProg[p], block_count(j, k) * j.value_size, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
            return;
        }
        uint8_t *blk = block_ptr(j, data_block_slot(k, j.dbcm));
        produce_body(j, k, block_count(j, k), status, masks, block_tile, splits, blk + kHeaderSize, &sProg[p],
                     const_cast<uint32_t *>(&res[j.job_index].invariant), sStage[Fused ? p : 0]);
        return;
    }
    // The chain is the critical path and mostly waits on LDS: let its
    // instructions win the SIMD's issue arbitration over the producers'.
    if constexpr (Fused) __builtin_amdgcn_s_setprio(2);
    if (!Fused && wave_in_block >= C) return; // a paired launch's narrower half (k_data_blocks_pair)
    const uint32_t wave = bid * C + wave_in_block;
    const bool upper = lane >= 32;
    const uint32_t mine = 2 * wave + (upper ? 1u : 0u);
    const bool live = locate(mine, ji, k);
    const bool live_lo = __builtin_amdgcn_readlane((int)live, 0) != 0;
    const bool live_hi = __builtin_amdgcn_readlane((int)live, 32) != 0;
    if (!live_lo && !live_hi) return;
    if (!live) locate(mine ^ 1u, ji, k); // mirror the partner's block, write nothing
    const bool writer = live;
    const uint32_t src_half = (upper ? 1u : 0u) ^ (live ? 0u : 1u);
    const JobDesc &j = jobs[ji];
    const uint32_t cnt = block_count(j, k);
    const uint32_t size = kHeaderSize + cnt * j.value_size;
    const uint32_t slot = data_block_slot(k, j.dbcm);
    uint8_t *blk = block_ptr(j, slot);

    uint32_t body_tag;
    if constexpr (Fused) {
        BodyMsg body(blk + kHeaderSize, cnt * j.value_size, &sProg[2 * wave_in_block + src_half],
                     const_cast<uint32_t *>(&res[j.job_index].invariant), &sCons[2 * wave_in_block + src_half]);
        body_tag = aegis_mac32(sT, body);
    } else {
        (void)src_half;
        // Four chains per SIMD are VALU-issue-bound, not latency-bound: take
        // the round key with one ds_bpermute (LDS pipe) instead of the six
        // VALU lane moves that win when a chain waits alone on LDS latency.
        // k_assemble ran before this kernel (stream order): every survivor of
        // the block must have landed.
        // (A speculated job whose speculation held was merged by
        // k_merge_unique, before this kernel in stream order: no counts.)
        // (Seal jobs: the caller placed the bodies, tbc_compaction_seal.)
        const bool produced = (j.unique && res[j.job_index].spec != kSpecBroken) || j.seal;
        if (!produced &&
            __hip_atomic_load(ready + j.dblock_base + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != cnt)
            gst<uint32_t>(const_cast<uint32_t *>(&res[j.job_index].invariant), 0xdeafu);
        GlobalMsg body(blk + kHeaderSize, cnt * j.value_size);
        body_tag = aegis_mac32<GlobalMsg, ChainStep>(sT, body);
    }

    (void)size;
    finish_data_block<false, typename Layout::HeaderStep>(sT, sHdr[wave_in_block][upper ? 1 : 0], j, k, cnt, body_tag,
                                                          writer);
}

// kHdrMax: the most chain waves a launch's workgroups hold (their header
// rows in LDS: 512 B each); tails of at most 8 chain waves per workgroup
// take 4 KiB instead of 8, room for one more front workgroup on their CUs.
template <bool Fused, class ChainStep = StepBpermute, uint32_t kHdrMax = (Fused ? kMaxChainWaves : kMaxChainOnlyWaves)>
__global__ __launch_bounds__(Fused ? 3 * 64 * kMaxChainWaves : 1024) void k_data_blocks(
    const JobDesc *jobs, int njobs, uint32_t total, const JobResultDev *res, const uint64_t *status,
    const uint64_t *masks, const uint32_t *block_tile, const SplitDesc *splits, uint32_t chain_waves,
    const uint32_t *ready, const SplitDesc *bsplits, uint32_t phase) {
    data_blocks<Fused, ChainStep, kHdrMax>(jobs, njobs, total, res, status, masks, block_tile, splits, chain_waves,
                                           ready, bsplits, phase, blockIdx.x);
}

// Two grid batches' chains in one launch (tail pairing, engine.hip
// grid_tail_pair): workgroups [0, a.wgs) take batch a's blocks, the rest
// batch b's, each half with its own chain waves per workgroup.
template <class ChainStep>
__global__ __launch_bounds__(1024) void k_data_blocks_pair(ChainHalf a, ChainHalf b) {
    const bool second = blockIdx.x >= a.wgs;
    const ChainHalf &x = second ? b : a;
    data_blocks<false, ChainStep, 8>(x.jobs, x.njobs, x.total, x.res, nullptr, nullptr, nullptr, nullptr, x.c,
                                     x.ready, nullptr, 0u, second ? blockIdx.x - a.wgs : blockIdx.x);
}

// The recomputation of broken speculations (phase 1) in its own symbol, so
// profiles keep it apart from the block pass.
__global__ __launch_bounds__(3 * 64 * kMaxChainWaves) void k_data_blocks_redo(
    const JobDesc *jobs, int njobs, uint32_t total, const JobResultDev *res, const uint64_t *status,
    const uint64_t *masks, const uint32_t *block_tile, const SplitDesc *splits, uint32_t chain_waves,
    const uint32_t *ready) {
    data_blocks<true>(jobs, njobs, total, res, status, masks, block_tile, splits, chain_waves, ready, nullptr, 1u,
                      blockIdx.x);
}

// Throughput regime, pass 1: assemble every data block body from the merge's
// masks, parallel over merge positions (not sequential per block like the
// fused path's producers): one workgroup per merge tile; the tile's output
// offset (k_tile_scan) and A/B cursors (merge-path split) plus per-mask-word
// prefix counts give every survivor its source value and output slot.
// HBM-bound: every survivor is read once and written once.
//
// Per half tile (1,024 merged positions) every survivor's source pointer is
// staged in LDS first (each wave stages 4 mask words), then the workgroup
// copies them in output order, 16 bytes per lane and 8 loads in flight per
// lane, each destination found from the output position (a per-half table
// of the data blocks' addresses). Round 4 copied one mask word's survivors
// per wave at a time — for 16-32 byte values 1-2 KiB per wave per memory
// round trip, here 8 KiB: config 1's assembly 12.3 -> 9.1 ms per step,
// config 3's 804 -> 635 us, config 4's 262 -> 212 us; config 5's 128-byte
// values unchanged (gpurun_out/r05k). A job with vcm < 15 or values over 256 bytes (none of
// TigerBeetle's trees at 4 KiB blocks or more) finds each destination by a
// division instead of the table.
constexpr uint32_t kHalfTile = kMergeTile / 2;
constexpr uint32_t kHalfBlocks = kHalfTile / 15 + 3;

template <bool SparseOnly>
__global__ __launch_bounds__(256) void k_assemble(const JobDesc *jobs, int njobs, uint32_t total_tiles,
                                                       const uint64_t *status, const uint64_t *masks,
                                                       const SplitDesc *splits, uint32_t *ready,
                                                       const JobResultDev *res, uint32_t phase) {
    constexpr uint32_t W = kMergeTile / 64;       // mask words per kind per tile
    __shared__ uint32_t s_pre[3][W + 1];          // survivors, A taken, B taken before word w
    __shared__ uint64_t s_src[kHalfTile];         // source of each survivor of the half
    __shared__ uint64_t s_blk[kHalfBlocks];       // data block k_first + i of the half's survivors
    const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const uint64_t lt = (1ull << lane) - 1;
    if (phase == 1 && *(volatile const uint32_t *)jobs[0].spec_any == 0) return; // no speculation broke
    for (uint32_t g = blockIdx.x; g < total_tiles; g += gridDim.x) {
        const int ji = find_job(jobs, njobs, g, [](const JobDesc &d) { return d.tile_base; });
        const JobDesc &j = jobs[ji];
        if (phase_skips(j, res, phase)) continue;          // uniform per workgroup
        if (SparseOnly && !sparse_job(j, res)) continue; // uniform per workgroup
        const uint32_t t = g - j.tile_base;
        const uint32_t n = j.a.n + j.b.n, vs = j.value_size, vcm = j.vcm;
        const uint64_t *m = masks + (size_t)g * (2 * W);
        const SplitDesc sp = splits[j.split_base + t];
        const uint32_t out0 = (uint32_t)(gld<uint64_t>(status + g) >> 32);
        const uint32_t a0 = sp.i, b0 = t * kMergeTile - sp.i;
        auto valid_of = [&](uint32_t w) -> uint64_t {
            const uint32_t pos0 = t * kMergeTile + 64 * w;
            return pos0 >= n ? 0ull : (n - pos0 >= 64 ? ~0ull : ((1ull << (n - pos0)) - 1));
        };
        __syncthreads(); // the previous tile's readers of s_pre / s_src are done
        if (tid < W) {
            const uint64_t sm = gld<uint64_t>(m + tid), am = gld<uint64_t>(m + W + tid);
            s_pre[0][tid + 1] = __builtin_popcountll(sm);
            s_pre[1][tid + 1] = __builtin_popcountll(am);
            s_pre[2][tid + 1] = __builtin_popcountll(valid_of(tid) & ~am);
        }
        __syncthreads();
        if (tid < 3) {
            uint32_t acc = 0;
            s_pre[tid][0] = 0;
            for (uint32_t w = 1; w <= W; w++) {
                acc += s_pre[tid][w];
                s_pre[tid][w] = acc;
            }
        }
        __syncthreads();
        SegCursor ca, cb;
        ca.init(j.a, sp.seg_a);
        cb.init(j.b, sp.seg_b);
        const uint32_t cpv_log = __builtin_ctz(vs >> 4), qmask = (1u << cpv_log) - 1;
        for (uint32_t h = 0; h < 2; h++) {
            const uint32_t w0 = h * (W / 2);
            if (t * kMergeTile + 64 * w0 >= n) break; // uniform
            const uint32_t s0 = s_pre[0][w0], S = s_pre[0][w0 + W / 2] - s0;
            if (S == 0) continue; // uniform
            const uint32_t obase = (uint32_t)j.out_offset + out0 + s0; // the half's first output position
            const bool fast = vcm >= 15 && vs <= 256; // uniform
            const uint32_t kfirst = obase / vcm;
            const uint32_t nblk = (obase + S - 1) / vcm - kfirst + 1;
            if (fast && tid < nblk)
                s_blk[tid] = (uint64_t)(uintptr_t)(block_ptr(j, data_block_slot(kfirst + tid, j.dbcm)) + kHeaderSize);
            // Stage: wave wv takes words w0 + wv + 4i, all of its mask words
            // loaded at once (one round trip, not one per word).
            constexpr uint32_t kWaveWords = W / 2 / 4;
            uint64_t smv[kWaveWords], amv[kWaveWords];
#pragma unroll
            for (uint32_t i = 0; i < kWaveWords; i++) {
                const uint32_t w = w0 + wv + 4 * i;
                smv[i] = gld<uint64_t>(m + w);
                amv[i] = gld<uint64_t>(m + W + w);
            }
#pragma unroll
            for (uint32_t i = 0; i < kWaveWords; i++) {
                const uint32_t w = w0 + wv + 4 * i;
                if (t * kMergeTile + 64 * w >= n) break;
                const uint64_t sm = smv[i], am = amv[i];
                if (sm == 0) continue;
                const uint64_t valid = valid_of(w);
                const uint32_t ab = a0 + s_pre[1][w], bb = b0 + s_pre[2][w];
                ca.advance(ab);
                cb.advance(bb);
                if ((sm >> lane) & 1) {
                    const uint32_t r = __builtin_popcountll(sm & lt);
                    const uint8_t *src = ((am >> lane) & 1) ? ca.elem(ab + __builtin_popcountll(am & lt), vs)
                                                            : cb.elem(bb + __builtin_popcountll(valid & ~am & lt), vs);
                    s_src[s_pre[0][w] - s0 + r] = (uint64_t)(uintptr_t)src;
                }
            }
            __syncthreads();
            // Copy in output order: chunk c = survivor c >> cpv_log, 16-byte
            // piece c & qmask; a lane's chunks are 256 apart.
            const uint32_t total = S << cpv_log;
            const uint32_t ds = 256u >> cpv_log; // survivors between a lane's chunks (vs <= 256)
            for (uint32_t c = tid; !fast && c < total; c += 256) { // one chunk at a time (rare layouts)
                const uint32_t o = obase + (c >> cpv_log);
                const uint32_t k = o / vcm;
                const u32x4 v = gld<u32x4>((const uint8_t *)(uintptr_t)s_src[c >> cpv_log] + 16 * (c & qmask));
                gst<u32x4>(block_ptr(j, data_block_slot(k, j.dbcm)) + kHeaderSize + (size_t)(o - k * vcm) * vs +
                               16 * (c & qmask), v);
            }
            for (uint32_t c0 = 0; fast && c0 < total; c0 += 256 * 8) {
                const uint32_t sl = (c0 + tid) >> cpv_log;
                uint32_t k = (obase + sl) / vcm - kfirst;
                uint32_t rem = obase + sl - (kfirst + k) * vcm;
                u32x4 v[8];
#pragma unroll
                for (uint32_t u = 0; u < 8; u++) { // unconditional (clamped): all eight source reads, then all loads
                    const uint32_t c = c0 + tid + 256 * u < total ? c0 + tid + 256 * u : total - 1;
                    v[u] = gld<u32x4>((const uint8_t *)(uintptr_t)s_src[c >> cpv_log] + 16 * (c & qmask));
                }
#pragma unroll
                for (uint32_t u = 0; u < 8; u++) {
                    const uint32_t c = c0 + tid + 256 * u;
                    if (c < total) {
                        uint8_t *dst = (uint8_t *)(uintptr_t)s_blk[k] + (size_t)rem * vs + 16 * (c & qmask);
                        gst<u32x4>(dst, v[u]);
                    }
                    rem += ds;
                    while (rem >= vcm) {
                        rem -= vcm;
                        k++;
                    }
                }
            }
            __syncthreads(); // s_src and s_blk are rewritten by the next half
        }
        // Count the survivors landed in every data block (as k_assemble).
        if (tid == 0 && j.out_offset == 0) {
            const uint32_t cnt = s_pre[0][W];
            uint32_t o = out0;
            while (o < out0 + cnt) {
                const uint32_t k = o / vcm;
                const uint32_t e = (k + 1) * vcm < out0 + cnt ? (k + 1) * vcm : out0 + cnt;
                __hip_atomic_fetch_add(ready + j.dblock_base + k, e - o, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                o = e;
            }
        }
    }
}

// LDS ordering among the lanes of one wave (the only wave left running).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// Index blocks: index_block_finish (table.zig:403-457) + the TableInfo
// manifest entry (manifest.zig:121-149, schema.zig:489-509). One table per
// wave (both groups compute it; the lower group writes).
constexpr uint32_t kIndexLdsBytes = 16384;

template <class Step = StepShared, uint32_t kThreads = 64>
__global__ __launch_bounds__(kThreads) void k_index_blocks(const JobDesc *jobs, int njobs, JobResultDev *res,
                                                         uint8_t *infos) {
    using Layout = TableLayout<Step>;
    __shared__ uint32_t sT[Layout::kDwords];
    __shared__ uint32_t sIdx[kIndexLdsBytes / 4];
    __shared__ uint64_t sKeys[2][4];
    // The workgroup's waves load the tables (replicated 128 KiB tables took
    // sixteen: one wave alone spent ~50 us on them); wave 0 then builds the
    // table's index block.
    Layout::load(sT);
    __syncthreads();
    if (threadIdx.x >= 64) return;
    const uint32_t wave = blockIdx.x;
    const int ji = find_job(jobs, njobs, wave, [](const JobDesc &d) { return d.table_base; });
    const JobDesc &j = jobs[ji];
    const uint32_t t = wave - j.table_base + j.table_lo; // the job's table index
    const uint32_t lane = threadIdx.x & 63, g = lane & 31;
    const uint32_t db = res[j.job_index].data_block_count;
    const uint32_t tables = res[j.job_index].table_count;
    if (t - j.table_lo >= j.table_max || t >= tables) return;
    const uint64_t n_out = res[j.job_index].value_count;
    const uint32_t k0 = t * j.dbcm;
    const uint32_t nblk = (db - k0) < j.dbcm ? (db - k0) : j.dbcm;
    const uint32_t k_last = k0 + nblk - 1;
    const uint32_t ks = j.key_size;
    uint8_t *idx = (uint8_t *)sIdx;
    for (uint32_t i = lane; i < j.index_size / 4; i += 64) sIdx[i] = 0;
    wave_sync();
    const uint8_t *image = block_ptr(j, index_block_slot(t, k_last)); // seal jobs: the entries in place
    for (uint32_t s = lane; s < nblk; s += 64) {
        const uint32_t k = k0 + s;
        const uint64_t first = (uint64_t)k * j.vcm;
        const uint32_t cnt = (uint32_t)((n_out - first) < j.vcm ? (n_out - first) : j.vcm);
        const uint32_t slot = data_block_slot(k, j.dbcm);
        const uint8_t *blk = block_ptr(j, slot);
        uint64_t kmin[4] = {0, 0, 0, 0}, kmax[4] = {0, 0, 0, 0};
        uint64_t *cks = (uint64_t *)(idx + j.idx_checksums_off + 32 * s);
        if (j.seal) {
            for (uint32_t l = 0; l < ks / 8; l++) {
                kmin[l] = ld64(image + j.idx_keys_min_off + ks * s + 8 * l);
                kmax[l] = ld64(image + j.idx_keys_max_off + ks * s + 8 * l);
            }
            cks[0] = ld64(image + j.idx_checksums_off + 32 * s);
            cks[1] = ld64(image + j.idx_checksums_off + 32 * s + 8);
        } else {
            value_key(j, blk + kHeaderSize, kmin);
            value_key(j, blk + kHeaderSize + (size_t)(cnt - 1) * j.value_size, kmax);
            cks[0] = ld64(blk);
            cks[1] = ld64(blk + 8);
        }
        for (uint32_t l = 0; l < ks / 8; l++) {
            ((uint64_t *)(idx + j.idx_keys_min_off + ks * s))[l] = kmin[l];
            ((uint64_t *)(idx + j.idx_keys_max_off + ks * s))[l] = kmax[l];
        }
        ((uint64_t *)(idx + j.idx_addresses_off))[s] = gld<uint64_t>(j.addresses + slot);
        if (s == 0)
            for (int l = 0; l < 4; l++) sKeys[0][l] = kmin[l];
        if (s == nblk - 1)
            for (int l = 0; l < 4; l++) sKeys[1][l] = kmax[l];
    }
    wave_sync();
    LdsMsg body(sIdx + kHeaderSize / 4, j.index_size - kHeaderSize);
    const uint32_t body_tag = aegis_mac32<LdsMsg, Step>(sT, body);
    const uint32_t index_slot = index_block_slot(t, k_last);
    HeaderFields h;
    h.cluster_lo = j.cluster_lo;
    h.cluster_hi = j.cluster_hi;
    h.address = gld<uint64_t>(j.addresses + index_slot);
    h.snapshot = j.snapshot_min;
    h.size = j.index_size;
    h.meta0 = nblk;       // TableIndex.Metadata.data_block_count
    h.meta1 = j.dbcm;     // .data_block_count_max
    h.meta2 = ks;         // .key_size
    h.meta3 = j.tree_id;  // .tree_id
    h.block_type = 4;     // BlockType.index (schema.zig:64)
    wave_sync();
    const uint32_t hdr_tag = finish_header<Step>(sT, sIdx, h, body_tag);
    wave_sync();
    if (lane < 4) sIdx[lane] = hdr_tag;
    wave_sync();
    uint8_t *blk = block_ptr(j, index_slot);
    for (uint32_t i = lane; i < j.index_size / 4; i += 64) gst<uint32_t>(blk + 4 * i, sIdx[i]);
    const uint32_t end = (uint32_t)sector_ceil(j.index_size);
    for (uint32_t o = j.index_size + 4 * lane; o < end; o += 256) gst<uint32_t>(blk + o, 0u);

    // ManifestNode.TableInfo (schema.zig:489-509).
    if (lane < 32) {
        const uint64_t vcount = (n_out - (uint64_t)k0 * j.vcm) < (uint64_t)nblk * j.vcm
                                    ? (n_out - (uint64_t)k0 * j.vcm)
                                    : (uint64_t)nblk * j.vcm;
        uint32_t *info = (uint32_t *)(infos + (size_t)(j.info_base + t - j.table_lo) * kTableInfoSize);
        uint32_t v = 0;
        const uint32_t i = g; // dwords 0..31
        if (i < 8) {
            const uint32_t l = i >> 1;
            v = (4 * i < ks) ? (uint32_t)(sKeys[0][l] >> (32 * (i & 1))) : 0u;
        } else if (i < 16) {
            const uint32_t ii = i - 8, l = ii >> 1;
            v = (4 * ii < ks) ? (uint32_t)(sKeys[1][l] >> (32 * (ii & 1))) : 0u;
        } else if (i < 20) {
            v = sIdx[i - 16]; // index block checksum
        } else if (i == 24) v = (uint32_t)h.address;
        else if (i == 25) v = (uint32_t)(h.address >> 32);
        else if (i == 26) v = (uint32_t)j.snapshot_min;
        else if (i == 27) v = (uint32_t)(j.snapshot_min >> 32);
        else if (i == 28 || i == 29) v = 0xffffffffu; // snapshot_max = maxInt(u64)
        else if (i == 30) v = (uint32_t)vcount;
        else if (i == 31) v = (uint32_t)j.tree_id | ((uint32_t)((j.level_b & 0x3f) | (1u << 6)) << 16);
        gst<uint32_t>(info + i, v);
    }
}

// Pipelined batches (tbc_compaction_submit, grid mode): the data block
// addresses of every output table's index block (TableIndex.data_addresses,
// schema.zig:80-260), written with the bodies so that a later batch can
// resolve these tables before this batch's chains have sealed them. The seal
// (k_index_blocks) rewrites the same values with the rest of the block.
__global__ __launch_bounds__(256) void k_index_layout(const JobDesc *jobs, int njobs, uint32_t total,
                                                      const JobResultDev *res) {
    const uint32_t m = blockIdx.x * 256 + threadIdx.x;
    if (m >= total) return;
    const int ji = find_job(jobs, njobs, m, [](const JobDesc &d) { return d.dblock_base; });
    const JobDesc &j = jobs[ji];
    const uint32_t k = m - j.dblock_base;
    const uint32_t db = res[j.job_index].data_block_count;
    if (k >= db) return;
    const uint32_t t = k / j.dbcm;
    const uint32_t k_last = ((t + 1) * j.dbcm < db ? (t + 1) * j.dbcm : db) - 1;
    uint8_t *idx = block_ptr(j, index_block_slot(t, k_last));
    gst<uint64_t>(idx + j.idx_addresses_off + 8 * (k - t * j.dbcm), gld<uint64_t>(j.addresses + data_block_slot(k, j.dbcm)));
}

// One workgroup per CU (the tables take 128 KiB of LDS): spread the waves
// over all 256 CUs, at most 16 waves per workgroup.
static uint32_t waves_per_block(uint32_t waves) {
    uint32_t w = (waves + 255) / 256;
    return w < 1 ? 1 : (w > 16 ? 16 : w);
}

int launch_validate_blocks(const uint64_t *d_ptrs, const uint64_t *d_expect, uint32_t count, uint32_t block_size,
                          uint8_t *d_out, void *stream) {
    if (count == 0) return 0;
    const uint32_t wpb = waves_per_block(count);
    hipLaunchKernelGGL(k_validate_blocks, dim3((count + wpb - 1) / wpb), dim3(64 * wpb), 0, (hipStream_t)stream,
                       d_ptrs, d_expect, count, block_size, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_grid_validate(const InputCheck *d_checks, uint32_t count, uint8_t *d_verified, const JobDesc *d_jobs,
                         int njobs, JobResultDev *d_results, uint32_t block_size, void *stream) {
    if (count == 0) return 0;
    const uint32_t wpb = waves_per_block(count);
    hipLaunchKernelGGL(k_grid_validate, dim3((count + wpb - 1) / wpb), dim3(64 * wpb), 0, (hipStream_t)stream,
                       d_checks, count, d_verified, d_jobs, njobs, d_results, block_size);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_manifest_close(const uint64_t *d_addresses, uint32_t count, uint8_t *grid_base, uint32_t block_size,
                          uint64_t previous_address, const uint64_t *d_previous_checksum, uint8_t *d_verified,
                          uint32_t *d_error, void *stream) {
    if (count == 0) return 0;
    const uint32_t wpb = waves_per_block((count + 1) / 2);
    hipLaunchKernelGGL(k_manifest_bodies, dim3(((count + 1) / 2 + wpb - 1) / wpb), dim3(64 * wpb), 0,
                       (hipStream_t)stream, d_addresses, count, grid_base, block_size);
    if (hipGetLastError() != hipSuccess) return -1;
    hipLaunchKernelGGL(k_manifest_chain, dim3(1), dim3(64), 0, (hipStream_t)stream, d_addresses, count, grid_base,
                       block_size, previous_address, d_previous_checksum, d_verified, d_error);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

int launch_checksum_batch(const uint64_t *d_ptrs, const uint64_t *d_lens, uint32_t count, uint8_t *d_out,
                          void *stream) {
    if (count == 0) return 0;
    const uint32_t wpb = waves_per_block(count);
    hipLaunchKernelGGL(k_checksum_batch, dim3((count + wpb - 1) / wpb), dim3(64 * wpb), 0, (hipStream_t)stream,
                       d_ptrs, d_lens, count, d_out);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

uint32_t fused_max_chain_waves() { return kFusedMaxChainWaves; }

template <bool SparseOnly>
static void run_assemble(uint32_t grid, hipStream_t s, const JobDesc *d_jobs, int njobs, uint32_t total_tiles,
                         const uint64_t *d_status, const uint64_t *d_masks, const SplitDesc *d_splits,
                         uint32_t *d_ready, const JobResultDev *d_results, uint32_t phase) {
    hipLaunchKernelGGL(k_assemble<SparseOnly>, dim3(grid), dim3(256), 0, s, d_jobs, njobs, total_tiles, d_status,
                       d_masks, d_splits, d_ready, d_results, phase);
}

int launch_blocks(const JobDesc *d_jobs, int njobs, uint32_t total_tiles, uint32_t total_dblocks, uint32_t total_tables,
                  uint32_t *d_ready,
                  JobResultDev *d_results, uint8_t *d_infos, const uint64_t *d_status, const uint64_t *d_masks,
                  const uint32_t *d_block_tile, const SplitDesc *d_splits, bool values_only, bool maybe_sparse,
                  void *stream,
                  void (*mark)(void *, const char *), void *mark_ctx, bool bodies_done,
                  const SplitDesc *d_bsplits, uint32_t phase, bool index_blocks) {
    hipStream_t s = (hipStream_t)stream;
    const uint32_t waves = (total_dblocks + 1) / 2; // chain waves
    if (values_only) {
        // Survivors only (TBC_COMPACTION_VALUES_ONLY): the bodies, no chains
        // and no index blocks.
        if (total_dblocks && !bodies_done) {
            const uint32_t agrid = total_tiles < 8192 ? total_tiles : 8192;
            run_assemble<false>(agrid, s, d_jobs, njobs, total_tiles, d_status, d_masks, d_splits, d_ready,
                               (const JobResultDev *)d_results, phase);
            if (hipGetLastError() != hipSuccess) return -1;
        }
        if (mark) mark(mark_ctx, "assemble");
        return 0;
    }
    if (total_dblocks && waves <= fused_max_chain_waves()) {
        // Latency regime: every chain is in flight at once; producers fill
        // the bodies while the chains absorb them.
        if (maybe_sparse) { // heavy-dedup jobs: bodies first, parallel (sparse_job decides on device)
            const uint32_t agrid = total_tiles < 8192 ? total_tiles : 8192;
            run_assemble<true>(agrid, s, d_jobs, njobs, total_tiles, d_status, d_masks, d_splits, d_ready,
                               (const JobResultDev *)d_results, phase);
            if (hipGetLastError() != hipSuccess) return -1;
            if (mark) mark(mark_ctx, phase ? "recompute_assemble" : "assemble");
        }
        uint32_t c = waves_per_block(waves);
        c = c > kMaxChainWaves ? kMaxChainWaves : c;
        if (phase == 1)
            hipLaunchKernelGGL(k_data_blocks_redo, dim3((waves + c - 1) / c), dim3(3 * 64 * c), 0, s, d_jobs, njobs,
                               total_dblocks, (const JobResultDev *)d_results, d_status, d_masks, d_block_tile,
                               d_splits, c, (const uint32_t *)d_ready);
        else
            hipLaunchKernelGGL(k_data_blocks<true>, dim3((waves + c - 1) / c), dim3(3 * 64 * c), 0, s, d_jobs, njobs,
                               total_dblocks, (const JobResultDev *)d_results, d_status, d_masks, d_block_tile,
                               d_splits, c, (const uint32_t *)d_ready, d_bsplits, 0u);
        if (hipGetLastError() != hipSuccess) return -1;
    } else if (total_dblocks) {
        // Throughput regime: assemble every body, then the chains, 4 per SIMD.
        // (Running k_assemble concurrently on a second stream, chains waiting
        // on the per-block counts, measured 2.2x SLOWER for config 5: the
        // chain workgroups leave the assemble waves too little of each CU.)
        // The counts stay as a check: a chain whose block is short of values
        // reports an invariant error instead of checksumming a partial body.
        if (!bodies_done) {
            const uint32_t agrid = total_tiles < 8192 ? total_tiles : 8192;
            run_assemble<false>(agrid, s, d_jobs, njobs, total_tiles, d_status, d_masks, d_splits, d_ready,
                               (const JobResultDev *)d_results, phase);
            if (hipGetLastError() != hipSuccess) return -1;
            if (mark) mark(mark_ctx, "assemble");
        }
        const uint32_t rounds = (waves + 256 * kMaxChainOnlyWaves - 1) / (256 * kMaxChainOnlyWaves);
        const uint32_t c = (waves + 256 * rounds - 1) / (256 * rounds);
        hipLaunchKernelGGL(k_data_blocks<false>, dim3((waves + c - 1) / c), dim3(64 * c), 0, s, d_jobs, njobs,
                           total_dblocks, (const JobResultDev *)d_results, d_status, d_masks, d_block_tile, d_splits,
                           c, (const uint32_t *)d_ready, d_bsplits, phase);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mark) mark(mark_ctx, phase ? "recompute_blocks" : "data_blocks");
    if (!index_blocks) return 0;
    if (total_tables) {
        hipLaunchKernelGGL((k_index_blocks<StepShared, 64>), dim3(total_tables), dim3(64), 0, s, d_jobs, njobs, d_results, d_infos);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mark) mark(mark_ctx, "index_blocks");
    return 0;
}

int launch_index_blocks(const JobDesc *d_jobs, int njobs, uint32_t total_tables, JobResultDev *d_results,
                        uint8_t *d_infos, void *stream) {
    if (!total_tables) return 0;
    hipLaunchKernelGGL((k_index_blocks<StepShared, 64>), dim3(total_tables), dim3(64), 0, (hipStream_t)stream, d_jobs, njobs,
                       d_results, d_infos);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Bodies of the jobs the merge decided (phase 0: every job not speculated;
// phase 1: the speculated jobs whose speculation broke), parallel over merge
// tiles; each block's landed count goes to d_ready.
int launch_assemble(const JobDesc *d_jobs, int njobs, uint32_t total_tiles, uint32_t *d_ready,
                    const JobResultDev *d_results, const uint64_t *d_status, const uint64_t *d_masks,
                    const SplitDesc *d_splits, uint32_t phase, void *stream) {
    if (!total_tiles) return 0;
    const uint32_t agrid = total_tiles < 8192 ? total_tiles : 8192;
    run_assemble<false>(agrid, (hipStream_t)stream, d_jobs, njobs, total_tiles, d_status, d_masks, d_splits, d_ready,
                               d_results, phase);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// Seal jobs (tbc_compaction_seal): one thread per finished data block writes
// its index entry — checksum (16 bytes, then 16 zero), key_min, key_max,
// address (TableIndex, schema.zig:80-260) — into its table's index block
// slot, where the table's owner (this rank, or another one the entries are
// sent to) seals the index block.
__global__ __launch_bounds__(256) void k_index_entries(const JobDesc *job, uint32_t blocks, const JobResultDev *res) {
    const uint32_t m = blockIdx.x * 256 + threadIdx.x;
    const JobDesc &j = *job;
    if (m >= blocks) return;
    const uint32_t k = j.block_lo + m;
    const uint32_t db = res->data_block_count;
    if (k >= db) return;
    const uint32_t t = k / j.dbcm, s = k - t * j.dbcm;
    const uint32_t k_last = ((t + 1) * j.dbcm < db ? (t + 1) * j.dbcm : db) - 1;
    const uint64_t first = (uint64_t)k * j.vcm;
    const uint32_t cnt = (uint32_t)((res->value_count - first) < j.vcm ? (res->value_count - first) : j.vcm);
    const uint32_t slot = data_block_slot(k, j.dbcm);
    const uint8_t *blk = block_ptr(j, slot);
    uint8_t *image = block_ptr(j, index_block_slot(t, k_last));
    uint64_t kmin[4], kmax[4];
    value_key(j, blk + kHeaderSize, kmin);
    value_key(j, blk + kHeaderSize + (size_t)(cnt - 1) * j.value_size, kmax);
    uint64_t *cks = (uint64_t *)(image + j.idx_checksums_off + 32 * s);
    cks[0] = ld64(blk);
    cks[1] = ld64(blk + 8);
    cks[2] = cks[3] = 0;
    for (uint32_t l = 0; l < j.key_size / 8; l++) {
        ((uint64_t *)(image + j.idx_keys_min_off + j.key_size * s))[l] = kmin[l];
        ((uint64_t *)(image + j.idx_keys_max_off + j.key_size * s))[l] = kmax[l];
    }
    ((uint64_t *)(image + j.idx_addresses_off))[s] = gld<uint64_t>(j.addresses + slot);
}

int launch_seal(const JobDesc *d_job, uint32_t blocks, uint32_t tables, JobResultDev *d_results, uint8_t *d_infos,
                void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (blocks) {
        const uint32_t waves = (blocks + 1) / 2;
        const uint32_t rounds = (waves + 256 * kMaxChainOnlyWaves - 1) / (256 * kMaxChainOnlyWaves);
        const uint32_t c = (waves + 256 * rounds - 1) / (256 * rounds);
        hipLaunchKernelGGL((k_data_blocks<false, StepValuKey>), dim3((waves + c - 1) / c), dim3(64 * c), 0, s, d_job,
                           1, blocks, (const JobResultDev *)d_results, (const uint64_t *)nullptr,
                           (const uint64_t *)nullptr, (const uint32_t *)nullptr, (const SplitDesc *)nullptr, c,
                           (const uint32_t *)nullptr, (const SplitDesc *)nullptr, 0u);
        if (hipGetLastError() != hipSuccess) return -1;
        hipLaunchKernelGGL(k_index_entries, dim3((blocks + 255) / 256), dim3(256), 0, s, d_job, blocks,
                           (const JobResultDev *)d_results);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (tables) {
        hipLaunchKernelGGL((k_index_blocks<StepShared, 64>), dim3(tables), dim3(64), 0, s, d_job, 1, d_results, d_infos);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    return 0;
}

// Pipelined batch, front (engine stream, in order with every later batch's
// front): every body assembled, and the output index blocks' data addresses.
int launch_blocks_front(const JobDesc *d_jobs, int njobs, uint32_t total_tiles, uint32_t total_dblocks,
                        uint32_t *d_ready, const JobResultDev *d_results, const uint64_t *d_status,
                        const uint64_t *d_masks, const SplitDesc *d_splits, void *stream,
                        void (*mark)(void *, const char *), void *mark_ctx, bool bodies_done) {
    hipStream_t s = (hipStream_t)stream;
    if (total_dblocks) {
        if (!bodies_done) {
            const uint32_t agrid = total_tiles < 8192 ? total_tiles : 8192;
            run_assemble<false>(agrid, s, d_jobs, njobs, total_tiles, d_status, d_masks, d_splits, d_ready, d_results,
                                0u);
            if (hipGetLastError() != hipSuccess) return -1;
        }
        hipLaunchKernelGGL(k_index_layout, dim3((total_dblocks + 255) / 256), dim3(256), 0, s, d_jobs, njobs,
                           total_dblocks, d_results);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mark) mark(mark_ctx, "assemble");
    return 0;
}

// Pipelined batch, tail (one of the engine's tail streams, after the front):
// the chains and headers of every data block, then the index blocks. Tails
// of consecutive batches run concurrently, so their chains share the chip.
int launch_blocks_tail(const JobDesc *d_jobs, int njobs, uint32_t total_dblocks, uint32_t total_tables,
                       JobResultDev *d_results, uint8_t *d_infos, const uint64_t *d_status, const uint64_t *d_masks,
                       const uint32_t *d_block_tile, const SplitDesc *d_splits, const uint32_t *d_ready,
                       void *stream, void (*mark)(void *, const char *), void *mark_ctx, bool compact) {
    hipStream_t s = (hipStream_t)stream;
    const uint32_t waves = (total_dblocks + 1) / 2;
    if (total_dblocks && compact) {
        // Grid batches: compact tables (72 KiB of LDS instead of 136), so the
        // next batches' mask merges of multi-limb keys (33-49 KiB of keys in
        // LDS: id and composite trees) and bar-end sorts fit beside them.
        // Config 1 44.5 -> 41.9 ms (mask merges 13.7 -> 10.7 ms per step; the
        // chains 115 -> 142 ms of summed time, off the critical path),
        // gpurun_out/r05w. Non-grid batches keep the full tables (§4.1).
        uint32_t c = waves > 512 ? 8u : 4u;
        if (c > waves) c = waves;
        hipLaunchKernelGGL((k_data_blocks<false, StepCompact, 8>), dim3((waves + c - 1) / c), dim3(64 * c), 0, s, d_jobs,
                           njobs, total_dblocks, (const JobResultDev *)d_results, d_status, d_masks, d_block_tile,
                           d_splits, c, d_ready, (const SplitDesc *)nullptr, 0u);
        if (hipGetLastError() != hipSuccess) return -1;
    } else if (total_dblocks) {
        if (waves <= 1024) { // latency regime: one chain per SIMD, round keys by VALU lane moves
            // A chain workgroup holds a whole CU's LDS (the tables), so
            // concurrent tails share the chip by CUs: pack four chain waves
            // per CU (one per SIMD), eight (two per SIMD, the chains' best
            // throughput) once a batch alone would take over half the CUs,
            // so that two consecutive batches' tails fill the chip (config 2:
            // 8 vs 12 waves, 1.98–2.02 vs 2.01–2.05 ms per step over three
            // calls, gpurun_out/r04).
            uint32_t c = waves > 512 ? 8u : 4u;
            if (c > waves) c = waves;
            // Two or more chains per SIMD share its VALU issue: the round key by
            // one ds_bpermute (LDS pipe) instead of six VALU lane moves, as the
            // throughput regime does.
            const bool bperm = c >= 8;
            if (bperm)
                hipLaunchKernelGGL((k_data_blocks<false, StepBpermute, 8>), dim3((waves + c - 1) / c), dim3(64 * c), 0, s,
                                   d_jobs, njobs, total_dblocks, (const JobResultDev *)d_results, d_status, d_masks,
                                   d_block_tile, d_splits, c, d_ready, (const SplitDesc *)nullptr, 0u);
            else
                hipLaunchKernelGGL((k_data_blocks<false, StepValuKey, 8>), dim3((waves + c - 1) / c), dim3(64 * c), 0, s,
                                   d_jobs, njobs, total_dblocks, (const JobResultDev *)d_results, d_status, d_masks,
                                   d_block_tile, d_splits, c, d_ready, (const SplitDesc *)nullptr, 0u);
        } else {
            const uint32_t rounds = (waves + 256 * kMaxChainOnlyWaves - 1) / (256 * kMaxChainOnlyWaves);
            const uint32_t c = (waves + 256 * rounds - 1) / (256 * rounds);
            hipLaunchKernelGGL((k_data_blocks<false, StepBpermute>), dim3((waves + c - 1) / c), dim3(64 * c), 0,
                               s, d_jobs, njobs, total_dblocks, (const JobResultDev *)d_results, d_status, d_masks,
                               d_block_tile, d_splits, c, d_ready, (const SplitDesc *)nullptr, 0u);
        }
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mark) mark(mark_ctx, "data_blocks");
    if (total_tables) {
        // Index blocks read shared T-tables (StepShared: 20 KiB of LDS with
        // the index image, not 144), so their one-wave workgroups start
        // beside chain workgroups instead of waiting for a CU to empty. The
        // chains keep the full tables: compact ones cost them 2,462 -> 3,142
        // us per step in config 2 (gpurun_out/r05h).
        hipLaunchKernelGGL((k_index_blocks<StepShared, 64>), dim3(total_tables), dim3(64), 0, s, d_jobs, njobs,
                           d_results, d_infos);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mark) mark(mark_ctx, "index_blocks");
    return 0;
}

// Tail pairing: two grid batches' chains in one launch, then each batch's
// index blocks. Each half packs its chains as launch_blocks_tail would (4
// chain waves per workgroup, 8 above 512 waves); the round key comes by
// VALU lane moves unless a half runs two chains per SIMD.
int launch_blocks_tail_pair(const TailHalf &a, const TailHalf &b, void *stream, void (*mark)(void *, const char *),
                            void *ctx_a, void *ctx_b, bool compact) {
    hipStream_t s = (hipStream_t)stream;
    auto half = [](const TailHalf &t) {
        ChainHalf h{t.jobs, t.njobs, t.dblocks, t.res, t.ready, 0u, 0u};
        const uint32_t waves = (t.dblocks + 1) / 2;
        if (!waves) return h;
        h.c = waves > 512 ? 8u : 4u;
        if (h.c > waves) h.c = waves;
        h.wgs = (waves + h.c - 1) / h.c;
        return h;
    };
    const ChainHalf ha = half(a), hb = half(b);
    const uint32_t c = ha.c > hb.c ? ha.c : hb.c;
    if (ha.wgs + hb.wgs) {
        if (compact)
            hipLaunchKernelGGL((k_data_blocks_pair<StepCompact>), dim3(ha.wgs + hb.wgs), dim3(64 * c), 0, s, ha, hb);
        else if (c >= 8)
            hipLaunchKernelGGL((k_data_blocks_pair<StepBpermute>), dim3(ha.wgs + hb.wgs), dim3(64 * c), 0, s, ha, hb);
        else
            hipLaunchKernelGGL((k_data_blocks_pair<StepValuKey>), dim3(ha.wgs + hb.wgs), dim3(64 * c), 0, s, ha, hb);
        if (hipGetLastError() != hipSuccess) return -1;
    }
    if (mark) {
        mark(ctx_a, "data_blocks");
        mark(ctx_b, "data_blocks");
    }
    for (int i = 0; i < 2; i++) {
        const TailHalf &t = i ? b : a;
        if (t.tables) {
            hipLaunchKernelGGL((k_index_blocks<StepShared, 64>), dim3(t.tables), dim3(64), 0, s, t.jobs, t.njobs, t.res,
                               t.infos);
            if (hipGetLastError() != hipSuccess) return -1;
        }
        if (mark) mark(i ? ctx_b : ctx_a, "index_blocks");
    }
    return 0;
}

} // namespace tbc
