// engine.cpp — the C ABI (include/tbc.h) over the HIP kernels.
//
// The engine mirrors TigerBeetle's static-allocation discipline
// (docs/TIGER_STYLE.md): one device arena and one pinned host arena are
// allocated at init, every batch carves its descriptors, scratch and result
// buffers out of them, and nothing is allocated on the hot path. A batch is
// all of a half-bar's compactions (Forest.compact -> Groove.compact ->
// Tree.compact, src/lsm/forest.zig:319-342) submitted at once; the host event
// loop polls it (hipEventQuery) instead of blocking, like the reference's
// callback loop (src/storage.zig:108-131).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <cstring>
#include <ctime>
#include <new>
#include <vector>

#include "../../include/tbc.h"
#include "tbc_internal.h"

using namespace tbc;

namespace {

constexpr uint64_t kDefaultArena = 256ull << 20;
constexpr uint64_t kPinnedArena = 64ull << 20;
constexpr uint32_t kIndexLdsMax = 16384; // k_index_blocks LDS image
constexpr int kMaxMarks = 16;

uint64_t align_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

// A stack of regions: a batch or k-way merge opens one at submit and closes
// it at release. Closing the topmost region pops it and every closed region
// below it, so regions released out of order are reclaimed as soon as the
// ones above them are; the top never grows past the live regions' extent.
// (Synchronous calls take scratch above the top with alloc() and restore it.)
// Device scratch and pinned staging of the batches in flight. Regions are
// closed in any order (a pipelined caller releases its oldest batch first
// while newer ones run); an allocation takes the first gap at or after the
// end of the last one, else the first gap from the start (next fit), so a
// steady stream of batches cycles through the arena. (Round 4's stack freed
// a region only once every region above it had closed: a caller that always
// kept a batch in flight never reclaimed anything and ran out after a few
// hundred batches.)
struct Arena {
    struct Region {
        uint64_t start, end, id;
    };
    uint8_t *base = nullptr;
    uint64_t size = 0, cursor = 0, next_id = 1, used = 0;
    std::vector<Region> regions; // open, by start
    // A region of `bytes`; *id identifies it for close().
    uint8_t *open(uint64_t bytes, uint64_t *id) {
        bytes = align_up(bytes ? bytes : 1, 256);
        for (int pass = 0; pass < 2; pass++) {
            uint64_t prev = 0;
            for (size_t i = 0; i <= regions.size(); i++) {
                const uint64_t gap_end = i < regions.size() ? regions[i].start : size;
                uint64_t s = prev;
                if (pass == 0) s = std::max(s, cursor); // next fit: at or after the last allocation
                if (s + bytes <= gap_end) {
                    regions.insert(regions.begin() + (long)i, Region{s, s + bytes, next_id});
                    *id = next_id++;
                    cursor = s + bytes;
                    used += bytes;
                    return base + s;
                }
                if (i < regions.size()) prev = regions[i].end;
            }
        }
        return nullptr;
    }
    void close(uint64_t id) {
        for (size_t i = 0; i < regions.size(); i++)
            if (regions[i].id == id) {
                used -= regions[i].end - regions[i].start;
                regions.erase(regions.begin() + (long)i);
                break;
            }
    }
    size_t live() const { return regions.size(); }
};

struct Layout {
    uint32_t key_size, vcm, dbcm, index_size;
    uint32_t cks_off, kmin_off, kmax_off, addr_off;
};

bool compute_layout(const tbc_tree *t, uint32_t block_size, Layout *L) {
    if (!t || t->tree_id == 0 || t->key_kind > TBC_KEY_COMPOSITE_U128 || t->usage > TBC_USAGE_SECONDARY_INDEX)
        return false;
    const uint32_t vs = t->value_size;
    if (vs < 16 || (vs & (vs - 1)) || t->timestamp_offset + 8 > vs || (t->timestamp_offset & 7)) return false;
    if (t->table_value_count_max == 0) return false;
    const uint32_t key_size = t->key_kind == TBC_KEY_TIMESTAMP ? 8 : t->key_kind == TBC_KEY_COMPOSITE_U128 ? 32 : 16;
    // Value layouts fixed by the key kind (groove.zig:48-56, composite_key.zig:17-46).
    if (t->key_kind == TBC_KEY_ID_U128 && (vs != 32 || t->timestamp_offset != 16)) return false;
    if (t->key_kind == TBC_KEY_COMPOSITE_U64 && (vs != 16 || t->timestamp_offset != 8)) return false;
    if (t->key_kind == TBC_KEY_COMPOSITE_U128 && (vs != 32 || t->timestamp_offset != 16)) return false;
    const uint32_t body = block_size - kHeaderSize;
    const uint32_t vcm = body / vs; // table.zig:116-119
    if (vcm == 0) return false;
    const uint32_t dbcm = (t->table_value_count_max + vcm - 1) / vcm; // table.zig:122
    if (dbcm > body / (32 + 8)) return false;                          // constants.zig:567-574
    L->key_size = key_size;
    L->vcm = vcm;
    L->dbcm = dbcm;
    L->cks_off = kHeaderSize;
    L->kmin_off = kHeaderSize + dbcm * 32;
    L->kmax_off = L->kmin_off + dbcm * key_size;
    L->addr_off = L->kmax_off + dbcm * key_size;
    L->index_size = L->addr_off + dbcm * 8; // schema.zig:139-140
    return L->index_size <= block_size;
}

} // namespace

// Pinned staging ring for host -> device streams (TableMemory.put, blocks read
// from storage): the host copies into a slot, the engine stream copies the
// slot to the device; a slot is reused once its copy's event has passed, so
// a producer only waits when it runs kSlots slots ahead of the device.
template <int N, uint64_t B> struct Ring {
    static constexpr int kSlots = N;
    static constexpr uint64_t kSlotBytes = B;
    uint8_t *base = nullptr;
    hipEvent_t ev[kSlots] = {};
    bool used[kSlots] = {};
    int next = 0;
    // The next slot, once the stream has passed its previous user.
    uint8_t *take(int *slot) {
        const int k = next;
        next = (next + 1) % kSlots;
        if (used[k] && hipEventSynchronize(ev[k]) != hipSuccess) return nullptr;
        *slot = k;
        return base + (uint64_t)k * kSlotBytes;
    }
};
// Bulk host<->device staging (blocks, puts).
using Staging = Ring<8, 8ull << 20>;
// Small descriptors (copy lists, sort plans, manifest addresses): many small
// slots, so the host may run many bar-end sorts ahead of the engine stream
// before it waits for a slot (with the bulk ring's 8 slots it waited on the
// sort four ops back: config 1's host spent 28 ms of a step there).
using DescRing = Ring<128, 64ull << 10>;

struct tbc_engine {
    int device = 0;
    uint32_t block_size = 0;
    uint32_t flags = 0;
    hipStream_t stream = nullptr;
    // Tail streams of pipelined (grid) batches: a batch's chains, index
    // blocks, input checks and results run on one of them, after its front
    // (merge + bodies) on `stream`; the next batch's front does not wait
    // for them, so consecutive batches' AEGIS chains share the chip. Main +
    // tails = one stream per hardware queue of the process
    // (GPU_MAX_HW_QUEUES, HIP's default 4): a stream sharing a queue would
    // inherit another's order.
    static constexpr int kMaxTails = 8;
    int ntails = 3;
    hipStream_t tail[kMaxTails] = {};
    hipEvent_t tail_ev[kMaxTails] = {}; // the last batch finished on each tail
    DescRing desc;
    // Caller-provided output ranges [lo, hi) of non-grid batches whose tails
    // may still read them, with an event recorded after each such tail: a
    // later batch writing into one of them waits for that event
    // (tbc_compaction_submit).
    struct TailOutputs {
        hipEvent_t done;
        std::vector<std::pair<uint64_t, uint64_t>> ranges;
    };
    std::vector<TailOutputs> tail_out;
    int next_tail = 0;
    // Engine-stream writes to memory a caller may hand a later batch as
    // input (memtable puts, bar-end sorts, device copies, the outputs of
    // batches not listed in tail_out): a batch whose descriptors and
    // partition go ahead on a tail stream (submit_impl's early prep) reads
    // its inputs there, off the engine stream, so that tail waits for the
    // last such write. `ext_dirty`: a write was enqueued since ext_ev was
    // last recorded; `ext_live`: ext_ev may not have passed yet.
    hipEvent_t ext_ev = nullptr;
    bool ext_dirty = false, ext_live = false;
    // Tail pairing: a grid batch whose tail waits for the next grid batch,
    // so that both batches' chains run as one launch on one tail stream
    // (grid_tail_pair); launched alone by any other call (flush_tail).
    // (Round 5's chain server — persistent chain waves taking any batch's
    // blocks from a device ring — measured slower on every config and was
    // removed in round 6: DESIGN 4.8.)
    tbc_batch *deferred = nullptr;
    bool pair_tails = true;
    Arena dev, host;
    Staging staging;
    // Host ranges the caller registered (tbc_host_register: hipHostRegister):
    // blocks to or from them are copied by DMA directly, without the staging
    // ring's host memcpy (TigerBeetle's I/O buffers are allocated once at
    // startup, so a replica registers them once).
    std::vector<std::pair<uint64_t, uint64_t>> registered;
    std::vector<hipEvent_t> event_pool;
    // Merge mask buffer (2 bits per merged position of a batch: 512 bytes
    // per tile). Batches run in stream order, so one buffer serves them all;
    // it only grows (after a stream drain), which a steady-state caller sees once.
    uint64_t *masks = nullptr;
    uint64_t mask_words = 0;
    // The last seal (tbc_compaction_seal, on a tail stream): engine-stream
    // copies wait for it (they may read the index entries it wrote).
    hipEvent_t seal_ev = nullptr;
    bool seal_pending = false;
    // Memtable sort scratch (keys, indices, histograms, look-back words, the
    // tables' copies): grown on demand like the masks.
    uint8_t *sort_scratch = nullptr;
    uint64_t sort_scratch_size = 0;
    // Its look-back words: zeroed when allocated, then tagged with a fresh
    // epoch per pass launch (sort.hip), so no pass clears them.
    uint64_t *sort_status = nullptr;
    uint64_t sort_status_words = 0;
    uint32_t sort_epoch = 1;
    // k-way merge scratch (level outputs, splits, masks, counts, descriptors):
    // merges run in stream order, so one growable buffer serves them all.
    uint8_t *copy_desc = nullptr; // tbc_copy_device_batch descriptors (device, grown once)
    uint64_t copy_desc_size = 0;
    uint8_t *kway_scratch = nullptr;
    uint64_t kway_scratch_size = 0;
    // (Bar-end sorts run on the engine stream. Round 3's sort stream of its
    // own measured slower — a fifth stream shares a hardware queue with a
    // tail and inherits its order — and was removed in round 6: DESIGN 3.)
};

struct tbc_grid {
    tbc_engine *engine = nullptr;
    uint8_t *base = nullptr;
    uint64_t block_count = 0;
    uint8_t *verified = nullptr; // device, per slot: written by the engine or validated (trusted like a cache hit)
    // Manifest closes the device refused (ManifestLog.close_block onto an
    // untrusted previous block): a device word set by the close's chain,
    // read and cleared by tbc_manifest_close_status.
    uint32_t *d_error = nullptr;
};

struct tbc_memtable {
    tbc_engine *engine = nullptr;
    tbc_tree tree{};
    uint8_t *values = nullptr;
    uint32_t capacity = 0, count = 0;
};

// hipEventQuery / hipStreamQuery answer "not ready" through the runtime's
// last-error slot, where a later `hipGetLastError() != hipSuccess` check
// after a kernel launch would take it for a launch failure: consume it.
static hipError_t event_query(hipEvent_t ev) {
    const hipError_t q = hipEventQuery(ev);
    if (q == hipErrorNotReady) (void)hipGetLastError();
    return q;
}
static hipError_t stream_query(hipStream_t s) {
    const hipError_t q = hipStreamQuery(s);
    if (q == hipErrorNotReady) (void)hipGetLastError();
    return q;
}

// A failing call reports its HIP error through its status: consume it from
// the runtime's last-error slot so that the next call does not report it too.
static tbc_status failed(tbc_status st) {
    (void)hipGetLastError();
    return st;
}

// A HIP error no call has reported (a call whose result the engine ignores:
// an event recorded for a profile mark, a synchronize at release): the next
// call that launches work returns TBC_ERR_DEVICE for it rather than drop it
// (the reference panics on a failure rather than continuing,
// compaction.zig:307-318). The engine's own queries consume their "not
// ready" (event_query, stream_query), and failing calls consume what they
// report (failed()).
static bool no_stale_error() {
    const hipError_t err = hipGetLastError();
    if (err == hipSuccess) return true;
    fprintf(stderr, "tbc: an unreported HIP error of an earlier call is pending: %s (%d)\n", hipGetErrorString(err),
            (int)err);
    return false;
}

static hipEvent_t take_event(tbc_engine *e) {
    if (e->event_pool.empty()) {
        hipEvent_t ev;
        if (hipEventCreate(&ev) != hipSuccess) return nullptr;
        return ev;
    }
    hipEvent_t ev = e->event_pool.back();
    e->event_pool.pop_back();
    return ev;
}

static bool is_registered(const tbc_engine *e, const void *p, uint64_t bytes) {
    const uint64_t lo = (uint64_t)(uintptr_t)p, hi = lo + bytes;
    for (const auto &r : e->registered)
        if (r.first <= lo && hi <= r.second) return true;
    return false;
}

// Host -> device through the pinned ring, enqueued on the engine stream
// (registered memory: one direct DMA, which still reads the caller's buffer
// after the call returns: *direct tells the caller to wait for it).
static bool stage_h2d(tbc_engine *e, void *dst, const void *src, uint64_t bytes, bool *direct = nullptr) {
    if (is_registered(e, src, bytes)) {
        if (direct) *direct = true;
        return hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->stream) == hipSuccess;
    }
    Staging &st = e->staging;
    const uint8_t *s = (const uint8_t *)src;
    uint8_t *d = (uint8_t *)dst;
    while (bytes) {
        const int slot = st.next;
        st.next = (st.next + 1) % Staging::kSlots;
        if (st.used[slot] && hipEventSynchronize(st.ev[slot]) != hipSuccess) return false;
        const uint64_t n = bytes < Staging::kSlotBytes ? bytes : Staging::kSlotBytes;
        uint8_t *p = st.base + (uint64_t)slot * Staging::kSlotBytes;
        memcpy(p, s, n);
        if (hipMemcpyAsync(d, p, n, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
            hipEventRecord(st.ev[slot], e->stream) != hipSuccess)
            return false;
        st.used[slot] = true;
        s += n;
        d += n;
        bytes -= n;
    }
    return true;
}

// Device -> host of many ranges. Registered destinations: direct DMA, one
// wait at the end. Others through the pinned ring with every slot in flight:
// a slot's chunk is copied out (host memcpy) only when the ring comes back to
// it, so the DMA of the next chunks overlaps the memcpy of earlier ones
// (round 3 waited for each chunk before issuing the next: 7.2 GB/s).
struct D2H {
    void *dst;
    const void *src;
    uint64_t bytes;
};
static bool stage_d2h_many(tbc_engine *e, const D2H *items, uint32_t count) {
    Staging &st = e->staging;
    struct Pending {
        uint8_t *dst = nullptr;
        uint64_t n = 0;
    } pend[Staging::kSlots];
    bool ok = true;
    // A slot's earlier user (an H2D stage) must be done before it is refilled.
    for (int k = 0; k < Staging::kSlots; k++)
        if (st.used[k] && hipEventSynchronize(st.ev[k]) != hipSuccess) return false;
    auto drain = [&](int slot) {
        if (!pend[slot].n) return;
        ok = ok && hipEventSynchronize(st.ev[slot]) == hipSuccess;
        if (ok) memcpy(pend[slot].dst, st.base + (uint64_t)slot * Staging::kSlotBytes, pend[slot].n);
        pend[slot].n = 0;
    };
    bool direct = false;
    for (uint32_t i = 0; ok && i < count; i++) {
        const uint8_t *s = (const uint8_t *)items[i].src;
        uint8_t *d = (uint8_t *)items[i].dst;
        uint64_t bytes = items[i].bytes;
        if (is_registered(e, d, bytes)) {
            ok = hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToHost, e->stream) == hipSuccess;
            direct = true;
            continue;
        }
        while (ok && bytes) {
            const int slot = st.next;
            st.next = (st.next + 1) % Staging::kSlots;
            drain(slot);
            const uint64_t n = bytes < Staging::kSlotBytes ? bytes : Staging::kSlotBytes;
            uint8_t *p = st.base + (uint64_t)slot * Staging::kSlotBytes;
            ok = ok && hipMemcpyAsync(p, s, n, hipMemcpyDeviceToHost, e->stream) == hipSuccess &&
                 hipEventRecord(st.ev[slot], e->stream) == hipSuccess;
            st.used[slot] = true;
            pend[slot].dst = d;
            pend[slot].n = n;
            s += n;
            d += n;
            bytes -= n;
        }
    }
    for (int k = 0; k < Staging::kSlots; k++) drain((st.next + k) % Staging::kSlots);
    if (direct) ok = ok && hipStreamSynchronize(e->stream) == hipSuccess;
    return ok;
}

// A list of 64-bit values (block addresses) copied to the device through a
// pinned staging slot, into a device arena region the caller closes once the
// work using it is enqueued (later arena users are later on the same stream).
static const uint64_t *stage_u64s(tbc_engine *e, const uint64_t *values, uint32_t count, uint64_t *region) {
    Staging &st = e->staging;
    const uint64_t bytes = 8ull * count;
    if (bytes > Staging::kSlotBytes) return nullptr;
    const int slot = st.next;
    st.next = (st.next + 1) % Staging::kSlots;
    if (st.used[slot] && hipEventSynchronize(st.ev[slot]) != hipSuccess) return nullptr;
    uint8_t *host = st.base + (uint64_t)slot * Staging::kSlotBytes;
    memcpy(host, values, bytes);
    uint8_t *d = e->dev.open(bytes, region);
    if (!d) return nullptr;
    const bool ok = hipMemcpyAsync(d, host, bytes, hipMemcpyHostToDevice, e->stream) == hipSuccess &&
                    hipEventRecord(st.ev[slot], e->stream) == hipSuccess;
    st.used[slot] = true;
    if (!ok) {
        e->dev.close(*region);
        return nullptr;
    }
    return (const uint64_t *)d;
}

constexpr uint64_t kInitialMaskWords = (1ull << 28) / kMergeTile * (2 * kMergeTile / 64);
static bool ensure_masks(tbc_engine *e, uint64_t words) {
    if (words <= e->mask_words) return true;
    if (hipStreamSynchronize(e->stream) != hipSuccess) return false;
    if (e->masks) hipFree(e->masks);
    e->masks = nullptr;
    e->mask_words = 0;
    const uint64_t want = align_up(words, 1ull << 16);
    if (hipMalloc((void **)&e->masks, want * 8) != hipSuccess) {
        e->masks = nullptr;
        return false;
    }
    e->mask_words = want;
    return true;
}

struct tbc_batch {
    tbc_engine *engine = nullptr;
    uint32_t count = 0;
    uint64_t dev_region = 0, host_region = 0; // arena regions (Arena::open) closed on release
    JobResultDev *h_results = nullptr;
    uint8_t *h_infos = nullptr;
    std::vector<uint32_t> info_base; // per original job index
    std::vector<uint32_t> status;    // host-side validation status per job
    hipEvent_t done = nullptr;
    hipEvent_t fork = nullptr;                          // end of the front (pipelined batches)
    hipEvent_t prep = nullptr;                          // descriptors + partition done ahead on a tail
    hipStream_t mark_stream = nullptr;                  // where mark_cb records
    // A batch split into job groups (tbc_compaction_submit): the groups'
    // batches, and per job its group and index there.
    std::vector<tbc_batch *> children;
    std::vector<std::pair<uint32_t, uint32_t>> job_map;
    hipEvent_t marks[kMaxMarks] = {};
    const char *mark_names[kMaxMarks] = {};
    int nmarks = 0;
    bool complete = false;
    tbc_status result = TBC_PENDING;
    // tbc_compaction_seal: what the call finished (the device results hold
    // the whole job's shape, which its kernels need).
    bool seal = false;
    tbc_compaction_result seal_result{};
    bool count_only = false; // TBC_COMPACTION_COUNT_ONLY: value_count only
    // A grid batch's tail (chains, index blocks, input checks, results), as
    // enqueued when the batch is submitted or, deferred for pairing, later.
    struct GridTail {
        TailHalf half{};
        const uint64_t *status = nullptr;
        const uint32_t *block_tile = nullptr;
        const SplitDesc *splits = nullptr;
        const ResolveItem *resolve = nullptr;
        uint32_t n_resolve = 0, n_checks = 0;
        InputCheck *checks = nullptr;
        tbc_grid *grid = nullptr;
        uint64_t copy_bytes = 0;
    } gt;
};

struct tbc_kway {
    tbc_engine *engine = nullptr;
    hipEvent_t done = nullptr;
    uint32_t *h_count = nullptr; // pinned: the merged value count
    uint64_t host_region = 0; // pinned arena region (device scratch is the engine's)
    bool arena = false;
    bool complete = false;
    tbc_status result = TBC_OK;
    uint64_t count = 0;
};

// TBC_DEBUG_SYNC=1 (tools only): wait up to 5 s for every stage of a batch
// and name the one that does not finish.
static void debug_stage(hipStream_t s, const char *name) {
    static const bool on = getenv("TBC_DEBUG_SYNC") != nullptr;
    if (!on) return;
    for (int i = 0; i < 5000; i++) {
        const hipError_t q = stream_query(s);
        if (q == hipSuccess) {
            fprintf(stderr, "tbc debug: stage %s done\n", name);
            return;
        }
        if (q != hipErrorNotReady) {
            fprintf(stderr, "tbc debug: stage %s error %d\n", name, (int)q);
            return;
        }
        struct timespec ts = {0, 1000000};
        nanosleep(&ts, nullptr);
    }
    fprintf(stderr, "tbc debug: stage %s NOT DONE after 5 s\n", name);
}

static void mark_cb(void *ctx, const char *name) {
    tbc_batch *b = (tbc_batch *)ctx;
    hipStream_t s = b->mark_stream ? b->mark_stream : b->engine->stream;
    debug_stage(s, name);
    if (!b->marks[0] || b->nmarks >= kMaxMarks) return; // profiled iff submitted with TBC_CONFIG_PROFILE
    hipEventRecord(b->marks[b->nmarks], s);
    b->mark_names[b->nmarks++] = name;
}

// Every stream of the engine drained (internal: no deferred-error report).
static bool sync_streams(tbc_engine *e);
static void flush_tail(tbc_engine *e, bool drain = false);
static tbc_status sort_batch(tbc_engine *e, const tbc_sort_job *jobs, uint32_t count);

// Later work on the engine stream that touches grid blocks (staging blocks in
// or out, synchronous checks) waits for every batch tail enqueued so far.
static bool join_tails(tbc_engine *e) {
    flush_tail(e);
    for (int t = 0; t < e->ntails; t++)
        if (hipStreamWaitEvent(e->stream, e->tail_ev[t], 0) != hipSuccess) return false;
    return true;
}

// Engine-stream copies may read what the last seal (on a tail) wrote.
static bool wait_seal(tbc_engine *e) {
    if (!e->seal_pending) return true;
    e->seal_pending = false; // the engine stream is ordered after it from here on
    return hipStreamWaitEvent(e->stream, e->seal_ev, 0) == hipSuccess;
}

// An engine-stream write a later batch may take as input (tbc_engine::ext_ev).
static void note_write(tbc_engine *e) { e->ext_dirty = true; }

// Stream P (a batch's early prep on a tail) ordered after every such write
// enqueued so far; no wait once the last one has passed.
static bool order_after_writes(tbc_engine *e, hipStream_t P) {
    if (e->ext_dirty) {
        if (hipEventRecord(e->ext_ev, e->stream) != hipSuccess) return false;
        e->ext_dirty = false;
        e->ext_live = true;
    }
    if (e->ext_live && event_query(e->ext_ev) == hipSuccess) e->ext_live = false;
    return !e->ext_live || hipStreamWaitEvent(P, e->ext_ev, 0) == hipSuccess;
}

extern "C" {

uint32_t tbc_abi_version(void) { return TBC_ABI_VERSION; }

tbc_status tbc_engine_set_profile(tbc_engine *e, uint32_t on) {
    if (!e) return TBC_ERR_INVALID_ARGUMENT;
    e->flags = on ? (e->flags | TBC_CONFIG_PROFILE) : (e->flags & ~(uint32_t)TBC_CONFIG_PROFILE);
    return TBC_OK;
}

tbc_status tbc_engine_init(const tbc_config *config, tbc_engine **out_engine) {
    if (!config || !out_engine) return TBC_ERR_INVALID_ARGUMENT;
    *out_engine = nullptr;
    const uint32_t bs = config->block_size;
    if (bs < kSectorSize || (bs & (bs - 1)) || bs % kSectorSize) return TBC_ERR_INVALID_ARGUMENT;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= config->device || config->device < 0)
        return failed(TBC_ERR_DEVICE);
    if (hipSetDevice(config->device) != hipSuccess) return failed(TBC_ERR_DEVICE);
    tbc_engine *e = new (std::nothrow) tbc_engine();
    if (!e) return failed(TBC_ERR_OUT_OF_MEMORY);
    e->device = config->device;
    e->block_size = bs;
    e->flags = config->flags;
    e->dev.size = config->arena_bytes ? config->arena_bytes : kDefaultArena;
    e->host.size = kPinnedArena;
    // (The engine stream at the highest priority measured no different for
    // config 1, 52.3 vs 52.0 ms: DESIGN 4.3.)
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        delete e;
        return failed(TBC_ERR_DEVICE);
    }
    if (hipMalloc((void **)&e->dev.base, e->dev.size) != hipSuccess) {
        hipStreamDestroy(e->stream);
        delete e;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    if (hipHostMalloc((void **)&e->host.base, e->host.size, hipHostMallocDefault) != hipSuccess) {
        hipFree(e->dev.base);
        hipStreamDestroy(e->stream);
        delete e;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    bool ok = true;
    // Streams, one per hardware queue of the process (GPU_MAX_HW_QUEUES,
    // HIP's default 4): the engine stream and the tails. Tails (chains,
    // index blocks, input checks, results) run at the engine stream's
    // priority: round 3 measured the highest tail priority (its workgroups
    // dispatched ahead of the next front) slower on one box, config 1 130 vs
    // 108 ms and config 5 15.0 vs 14.4 ms (the fronts are the critical path).
    {
        const char *q = getenv("GPU_MAX_HW_QUEUES");
        const int queues = q && atoi(q) > 0 ? atoi(q) : 4;
        const char *pt = getenv("TBC_PAIR_TAILS"); // 0 = every grid tail alone (test_gpu_pairing.py compares)
        e->pair_tails = !(pt && pt[0] == '0');
        const int want = queues - 1;
        e->ntails = want < 1 ? 1 : (want > tbc_engine::kMaxTails ? tbc_engine::kMaxTails : want);
    }
    for (int t = 0; ok && t < e->ntails; t++)
        ok = hipStreamCreateWithFlags(&e->tail[t], hipStreamNonBlocking) == hipSuccess &&
             hipEventCreateWithFlags(&e->tail_ev[t], hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&e->seal_ev, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipEventCreateWithFlags(&e->ext_ev, hipEventDisableTiming) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&e->staging.base, Staging::kSlots * Staging::kSlotBytes, hipHostMallocDefault) ==
                  hipSuccess;
    for (int s = 0; ok && s < Staging::kSlots; s++)
        ok = hipEventCreateWithFlags(&e->staging.ev[s], hipEventDisableTiming) == hipSuccess;
    ok = ok && hipHostMalloc((void **)&e->desc.base, DescRing::kSlots * DescRing::kSlotBytes, hipHostMallocDefault) ==
                   hipSuccess;
    for (int s = 0; ok && s < DescRing::kSlots; s++)
        ok = hipEventCreateWithFlags(&e->desc.ev[s], hipEventDisableTiming) == hipSuccess;
    // The merge's mask buffer, sized up front for batches of up to 2^28
    // values (64 MiB of HBM), so submitting never waits on the device to grow
    // it; a larger batch still grows it (after a stream synchronize).
    ok = ok && ensure_masks(e, kInitialMaskWords);
    if (!ok) {
        tbc_engine_deinit(e);
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    *out_engine = e;
    return TBC_OK;
}

void tbc_engine_deinit(tbc_engine *e) {
    flush_tail(e);
    if (!e) return;
    hipSetDevice(e->device);
    hipStreamSynchronize(e->stream);
    for (int t = 0; t < e->ntails; t++)
        if (e->tail[t]) hipStreamSynchronize(e->tail[t]);
    for (auto &t : e->tail_out) e->event_pool.push_back(t.done);
    for (hipEvent_t ev : e->event_pool) hipEventDestroy(ev);
    for (const auto &r : e->registered) hipHostUnregister((void *)(uintptr_t)r.first);
    for (int s = 0; s < Staging::kSlots; s++)
        if (e->staging.ev[s]) hipEventDestroy(e->staging.ev[s]);
    if (e->staging.base) hipHostFree(e->staging.base);
    for (int s = 0; s < DescRing::kSlots; s++)
        if (e->desc.ev[s]) hipEventDestroy(e->desc.ev[s]);
    if (e->desc.base) hipHostFree(e->desc.base);
    hipHostFree(e->host.base);
    hipFree(e->dev.base);
    if (e->masks) hipFree(e->masks);
    if (e->sort_scratch) hipFree(e->sort_scratch);
    if (e->sort_status) hipFree(e->sort_status);
    if (e->kway_scratch) hipFree(e->kway_scratch);
    if (e->copy_desc) hipFree(e->copy_desc);
    for (int t = 0; t < e->ntails; t++) {
        if (e->tail_ev[t]) hipEventDestroy(e->tail_ev[t]);
        if (e->tail[t]) hipStreamDestroy(e->tail[t]);
    }
    if (e->seal_ev) hipEventDestroy(e->seal_ev);
    if (e->ext_ev) hipEventDestroy(e->ext_ev);
    hipStreamDestroy(e->stream);
    // Errors of the drained work were the batches' to report: none is left
    // pending for the next engine's first call.
    (void)hipGetLastError();
    delete e;
}

tbc_status tbc_engine_arena_usage(const tbc_engine *e, uint64_t *dev_bytes, uint64_t *host_bytes, uint32_t *regions) {
    if (!e || !dev_bytes || !host_bytes || !regions) return TBC_ERR_INVALID_ARGUMENT;
    *dev_bytes = e->dev.used;
    *host_bytes = e->host.used;
    *regions = (uint32_t)(e->dev.live() + e->host.live());
    return TBC_OK;
}

tbc_status tbc_grid_init(tbc_engine *e, uint64_t block_count, tbc_grid **out) {
    if (!e || !out || block_count == 0) return TBC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    hipSetDevice(e->device);
    tbc_grid *g = new (std::nothrow) tbc_grid();
    if (!g) return failed(TBC_ERR_OUT_OF_MEMORY);
    g->engine = e;
    g->block_count = block_count;
    if (hipMalloc((void **)&g->base, block_count * e->block_size) != hipSuccess) {
        delete g;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    if (hipMalloc((void **)&g->verified, block_count) != hipSuccess ||
        hipMemsetAsync(g->verified, 0, block_count, e->stream) != hipSuccess ||
        hipMalloc((void **)&g->d_error, 256) != hipSuccess || hipMemsetAsync(g->d_error, 0, 256, e->stream) != hipSuccess) {
        if (g->d_error) hipFree(g->d_error);
        if (g->verified) hipFree(g->verified);
        hipFree(g->base);
        delete g;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    *out = g;
    return TBC_OK;
}

void tbc_grid_deinit(tbc_grid *g) {
    if (!g) return;
    hipSetDevice(g->engine->device);
    sync_streams(g->engine);
    hipFree(g->d_error);
    hipFree(g->verified);
    hipFree(g->base);
    delete g;
}

tbc_status tbc_grid_invalidate(tbc_grid *g) {
    flush_tail(g ? g->engine : nullptr);
    if (!g) return TBC_ERR_INVALID_ARGUMENT;
    tbc_engine *e = g->engine;
    hipSetDevice(e->device);
    if (!join_tails(e)) return failed(TBC_ERR_DEVICE); // no running batch marks a block after this
    return hipMemsetAsync(g->verified, 0, g->block_count, e->stream) == hipSuccess ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_grid_block_pointer(const tbc_grid *g, uint64_t address, void **out) {
    if (!g || !out || address == 0 || address > g->block_count) return TBC_ERR_INVALID_ARGUMENT;
    *out = g->base + (address - 1) * g->engine->block_size;
    return TBC_OK;
}

tbc_status tbc_grid_put_blocks(tbc_grid *g, const uint64_t *addresses, const void *const *blocks, uint32_t count) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    flush_tail(g ? g->engine : nullptr);
    if (!g || (count && (!addresses || !blocks))) return TBC_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < count; i++)
        if (addresses[i] == 0 || addresses[i] > g->block_count || !blocks[i]) return TBC_ERR_INVALID_ARGUMENT;
    tbc_engine *e = g->engine;
    hipSetDevice(e->device);
    if (!join_tails(e)) return failed(TBC_ERR_DEVICE); // no running batch reads a block being replaced
    if (!count) return TBC_OK;
    // Validate before trusting: every staged block's verified byte is cleared
    // BEFORE any image lands (stream order), so a call that fails halfway
    // never leaves an untrusted image marked verified. One launch per address
    // list that fits a staging slot.
    constexpr uint32_t kChunk = (uint32_t)(Staging::kSlotBytes / 8);
    for (uint32_t c0 = 0; c0 < count; c0 += kChunk) {
        const uint32_t n = count - c0 < kChunk ? count - c0 : kChunk;
        uint64_t region = 0;
        const uint64_t *d_addr = stage_u64s(e, addresses + c0, n, &region);
        if (!d_addr) return failed(TBC_ERR_DEVICE);
        const bool ok = launch_grid_set_verified(d_addr, n, g->verified, 0, e->stream) == 0;
        e->dev.close(region);
        if (!ok) return failed(TBC_ERR_DEVICE);
    }
    bool direct = false;
    note_write(e);
    for (uint32_t i = 0; i < count; i++)
        if (!stage_h2d(e, g->base + (addresses[i] - 1) * e->block_size, blocks[i], e->block_size, &direct))
            return failed(TBC_ERR_DEVICE);
    // A registered source is read by DMA after the enqueue: the caller may
    // reuse its buffer once this returns, so wait for those copies (pageable
    // sources were already copied into the pinned ring).
    if (direct) {
        hipEvent_t ev = take_event(e);
        const bool ok = ev && hipEventRecord(ev, e->stream) == hipSuccess && hipEventSynchronize(ev) == hipSuccess;
        if (ev) e->event_pool.push_back(ev);
        if (!ok) return failed(TBC_ERR_DEVICE);
    }
    return TBC_OK;
}

tbc_status tbc_grid_get_blocks(tbc_grid *g, const uint64_t *addresses, void *const *blocks, uint32_t count) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    flush_tail(g ? g->engine : nullptr);
    if (!g || (count && (!addresses || !blocks))) return TBC_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < count; i++)
        if (addresses[i] == 0 || addresses[i] > g->block_count || !blocks[i]) return TBC_ERR_INVALID_ARGUMENT;
    tbc_engine *e = g->engine;
    hipSetDevice(e->device);
    if (!join_tails(e)) return failed(TBC_ERR_DEVICE); // blocks still being sealed by a batch tail
    std::vector<D2H> items(count);
    for (uint32_t i = 0; i < count; i++)
        items[i] = D2H{blocks[i], g->base + (addresses[i] - 1) * e->block_size, e->block_size};
    return stage_d2h_many(e, items.data(), count) ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_manifest_close_blocks(tbc_grid *g, const uint64_t *addresses, const void *const *host_images,
                                     uint32_t count, uint64_t previous_address, const uint64_t *previous_checksum) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    flush_tail(g ? g->engine : nullptr);
    if (!g || (count && (!addresses || !host_images))) return TBC_ERR_INVALID_ARGUMENT;
    tbc_engine *e = g->engine;
    const uint32_t bs = e->block_size;
    const uint32_t entry_max = (bs - kHeaderSize) / kTableInfoSize;
    if (previous_address > g->block_count) return TBC_ERR_INVALID_ARGUMENT;
    // The host packs the header fields (ManifestLog.acquire_block + the
    // metadata of close_block); check them as verify_block and
    // ManifestNode.metadata (schema.zig:534-554) will.
    for (uint32_t i = 0; i < count; i++) {
        const uint8_t *h = (const uint8_t *)host_images[i];
        if (!h || addresses[i] == 0 || addresses[i] > g->block_count) return TBC_ERR_INVALID_ARGUMENT;
        uint32_t size, entries;
        uint64_t address, prev_address;
        memcpy(&size, h + 96, 4);
        memcpy(&entries, h + 168, 4);
        memcpy(&address, h + 224, 8);
        memcpy(&prev_address, h + 160, 8);
        const uint64_t want_prev = i == 0 ? previous_address : addresses[i - 1];
        if (size < kHeaderSize + kTableInfoSize || size > bs || (size - kHeaderSize) % kTableInfoSize ||
            entries != (size - kHeaderSize) / kTableInfoSize || entries > entry_max || address != addresses[i] ||
            prev_address != want_prev || h[110] != 20 || h[240] != 3)
            return TBC_ERR_INVALID_ARGUMENT;
    }
    if (!count) return TBC_OK;
    hipSetDevice(e->device);
    // No wait for the tails still running (round 4 joined them, stalling the
    // engine stream for up to a chain time per close): a manifest block's
    // address comes from the log's own reservation, so no running tail
    // writes it or reads it (a released address is reused only after the
    // next checkpoint, and the replica checkpoints with no grid IO in
    // flight); the chain reads only the previous manifest block, closed
    // earlier on this stream; the verified bytes it sets are its own blocks'.
    // Addresses and the previous checksum go through a pinned staging slot
    // (reusable once the stream has passed this close), the images through
    // the staging ring into their grid slots.
    Staging &st = e->staging;
    const uint64_t meta = 8ull * count + 16;
    if (meta > Staging::kSlotBytes) return TBC_ERR_CAPACITY;
    bool direct = false;
    note_write(e);
    for (uint32_t i = 0; i < count; i++) {
        uint32_t size;
        memcpy(&size, (const uint8_t *)host_images[i] + 96, 4);
        if (!stage_h2d(e, g->base + (addresses[i] - 1) * bs, host_images[i], sector_ceil(size), &direct))
            return failed(TBC_ERR_DEVICE);
    }
    if (direct) { // registered images are read by DMA after the enqueue: done before returning
        hipEvent_t ev = take_event(e);
        const bool ok = ev && hipEventRecord(ev, e->stream) == hipSuccess && hipEventSynchronize(ev) == hipSuccess;
        if (ev) e->event_pool.push_back(ev);
        if (!ok) return failed(TBC_ERR_DEVICE);
    }
    const int slot = st.next;
    st.next = (st.next + 1) % Staging::kSlots;
    if (st.used[slot] && hipEventSynchronize(st.ev[slot]) != hipSuccess) return failed(TBC_ERR_DEVICE);
    uint8_t *host = st.base + (uint64_t)slot * Staging::kSlotBytes;
    memcpy(host, addresses, 8ull * count);
    if (previous_checksum) memcpy(host + 8ull * count, previous_checksum, 16);
    // The device copy of the descriptors lives in the slot's mirror in the
    // device arena region of this call (freed once enqueued work is ordered
    // before any later arena use: the region is closed after the launch and
    // the next user of the arena is later on the same stream).
    uint64_t region = 0;
    uint8_t *d = e->dev.open(meta, &region);
    if (!d) return failed(TBC_ERR_OUT_OF_MEMORY);
    // The chain kernel marks the closed blocks verified (trusted like
    // compaction outputs), or refuses to link an untrusted previous block.
    bool ok = hipMemcpyAsync(d, host, meta, hipMemcpyHostToDevice, e->stream) == hipSuccess &&
              launch_manifest_close((const uint64_t *)d, count, g->base, bs, previous_address,
                                    previous_checksum ? (const uint64_t *)(d + 8ull * count) : nullptr, g->verified,
                                    g->d_error, e->stream) == 0 &&
              hipEventRecord(st.ev[slot], e->stream) == hipSuccess;
    st.used[slot] = true;
    e->dev.close(region);
    return ok ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_memtable_init(tbc_engine *e, const tbc_tree *tree, uint32_t capacity, tbc_memtable **out) {
    if (!e || !tree || !out) return TBC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    Layout L;
    if (!compute_layout(tree, e->block_size, &L) || capacity == 0 || capacity > tree->table_value_count_max)
        return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    tbc_memtable *m = new (std::nothrow) tbc_memtable();
    if (!m) return failed(TBC_ERR_OUT_OF_MEMORY);
    m->engine = e;
    m->tree = *tree;
    m->capacity = capacity;
    // +16: buffers are readable past the last value (sort/merge key loads of a 16-byte value).
    if (hipMalloc((void **)&m->values, (uint64_t)capacity * tree->value_size + 16) != hipSuccess) {
        delete m;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    *out = m;
    return TBC_OK;
}

void tbc_memtable_deinit(tbc_memtable *m) {
    if (!m) return;
    hipSetDevice(m->engine->device);
    hipStreamSynchronize(m->engine->stream);
    hipFree(m->values);
    delete m;
}

tbc_status tbc_memtable_put(tbc_memtable *m, const void *values, uint32_t count) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    if (!m || (count && !values)) return TBC_ERR_INVALID_ARGUMENT;
    if ((uint64_t)m->count + count > m->capacity) return TBC_ERR_CAPACITY; // table_memory.zig:80
    if (!count) return TBC_OK;
    hipSetDevice(m->engine->device);
    const uint64_t vs = m->tree.value_size;
    if (!stage_h2d(m->engine, m->values + m->count * vs, values, count * vs))
        return failed(TBC_ERR_DEVICE);
    note_write(m->engine);
    m->count += count;
    return TBC_OK;
}

tbc_status tbc_memtable_values(const tbc_memtable *m, void **out_values, uint32_t *out_count) {
    if (!m || !out_values || !out_count) return TBC_ERR_INVALID_ARGUMENT;
    *out_values = m->values;
    *out_count = m->count;
    return TBC_OK;
}

tbc_status tbc_memtable_reset(tbc_memtable *m) {
    if (!m) return TBC_ERR_INVALID_ARGUMENT;
    m->count = 0;
    return TBC_OK;
}

tbc_status tbc_memtable_make_immutable(tbc_engine *e, tbc_memtable *const *mutables, tbc_memtable *const *immutables,
                                       const uint8_t *in_order, uint32_t count) {
    if (!e || (count && (!mutables || !immutables))) return TBC_ERR_INVALID_ARGUMENT;
    std::vector<tbc_sort_job> jobs;
    for (uint32_t i = 0; i < count; i++) {
        const tbc_memtable *m = mutables[i], *im = immutables[i];
        if (!m || !im || m == im || m->engine != e || im->engine != e || im->count ||
            m->capacity != im->capacity || memcmp(&m->tree, &im->tree, sizeof m->tree))
            return TBC_ERR_INVALID_ARGUMENT;
    }
    auto sorted = [&](uint32_t i) { return mutables[i]->count && !(in_order && in_order[i]); };
    for (uint32_t i = 0; i < count; i++) {
        if (!sorted(i)) continue;
        tbc_sort_job j{};
        j.tree = mutables[i]->tree;
        j.values = mutables[i]->values;
        j.count = mutables[i]->count;
        j.values_out = immutables[i]->values;
        jobs.push_back(j);
    }
    if (!jobs.empty()) {
        const tbc_status st = sort_batch(e, jobs.data(), (uint32_t)jobs.size());
        if (st != TBC_OK) return st;
    }
    for (uint32_t i = 0; i < count; i++) {
        tbc_memtable *m = mutables[i], *im = immutables[i];
        if (!sorted(i)) std::swap(m->values, im->values); // in key order (or empty): the buffer changes hands
        im->count = m->count;
        m->count = 0;
    }
    return TBC_OK;
}

tbc_status tbc_tree_layout_get(const tbc_engine *e, const tbc_tree *tree, tbc_tree_layout *out) {
    if (!e || !tree || !out) return TBC_ERR_INVALID_ARGUMENT;
    Layout L;
    if (!compute_layout(tree, e->block_size, &L)) return TBC_ERR_INVALID_ARGUMENT;
    out->key_size = L.key_size;
    out->block_value_count_max = L.vcm;
    out->data_block_count_max = L.dbcm;
    out->index_size = L.index_size;
    out->index_checksums_offset = L.cks_off;
    out->index_keys_min_offset = L.kmin_off;
    out->index_keys_max_offset = L.kmax_off;
    out->index_addresses_offset = L.addr_off;
    return TBC_OK;
}

tbc_status tbc_host_register(tbc_engine *e, void *ptr, uint64_t bytes) {
    flush_tail(e);
    if (!e || !ptr || !bytes) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    const uint64_t lo = (uint64_t)(uintptr_t)ptr;
    for (const auto &r : e->registered)
        if (lo < r.second && r.first < lo + bytes) return TBC_ERR_INVALID_ARGUMENT; // overlaps a registered range
    if (hipHostRegister(ptr, bytes, hipHostRegisterDefault) != hipSuccess) return failed(TBC_ERR_DEVICE);
    e->registered.push_back({lo, lo + bytes});
    return TBC_OK;
}

tbc_status tbc_host_unregister(tbc_engine *e, void *ptr) {
    flush_tail(e);
    if (!e || !ptr) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    const uint64_t lo = (uint64_t)(uintptr_t)ptr;
    for (size_t i = 0; i < e->registered.size(); i++)
        if (e->registered[i].first == lo) {
            // Copies from or into it may still be enqueued.
            if (!sync_streams(e)) return failed(TBC_ERR_DEVICE);
            e->registered.erase(e->registered.begin() + (long)i);
            return hipHostUnregister(ptr) == hipSuccess ? TBC_OK : failed(TBC_ERR_DEVICE);
        }
    return TBC_ERR_INVALID_ARGUMENT;
}

tbc_status tbc_device_alloc(tbc_engine *e, uint64_t bytes, void **out_ptr) {
    if (!e || !out_ptr) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    return hipMalloc(out_ptr, bytes ? bytes : 1) == hipSuccess ? TBC_OK : failed(TBC_ERR_OUT_OF_MEMORY);
}

tbc_status tbc_device_free(tbc_engine *e, void *ptr) {
    if (!e) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    return hipFree(ptr) == hipSuccess ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_copy_to_device(tbc_engine *e, void *dst, const void *src, uint64_t bytes) {
    flush_tail(e);
    if (!e) return TBC_ERR_INVALID_ARGUMENT;
    if (!bytes) return TBC_OK;
    hipSetDevice(e->device);
    if (!wait_seal(e) || hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, e->stream) != hipSuccess)
        return failed(TBC_ERR_DEVICE);
    return hipStreamSynchronize(e->stream) == hipSuccess ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_copy_to_host(tbc_engine *e, void *dst, const void *src, uint64_t bytes) {
    flush_tail(e);
    if (!e) return TBC_ERR_INVALID_ARGUMENT;
    if (!bytes) return TBC_OK;
    hipSetDevice(e->device);
    if (!wait_seal(e) || hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, e->stream) != hipSuccess)
        return failed(TBC_ERR_DEVICE);
    return hipStreamSynchronize(e->stream) == hipSuccess ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_copy_device_async(tbc_engine *e, void *dst, const void *src, uint64_t bytes) {
    if (!e || (bytes && (!dst || !src))) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    if (!wait_seal(e)) return failed(TBC_ERR_DEVICE);
    note_write(e);
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, e->stream) == hipSuccess ? TBC_OK
                                                                                          : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_copy_device_batch(tbc_engine *e, const tbc_copy *copies, uint32_t count) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    if (!e || (count && !copies)) return TBC_ERR_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < count; i++)
        if (copies[i].bytes && (!copies[i].dst || !copies[i].src)) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    if (!wait_seal(e)) return failed(TBC_ERR_DEVICE);
    std::vector<CopyItem> items;
    uint64_t chunks = 0;
    const uint64_t cb = copy_chunk_bytes();
    for (uint32_t i = 0; i < count; i++) {
        const tbc_copy &c = copies[i];
        if (!c.bytes) continue;
        if (((uintptr_t)c.dst | (uintptr_t)c.src | c.bytes) & 15) { // unaligned: a copy of its own, in order
            if (hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToDevice, e->stream) != hipSuccess)
                return failed(TBC_ERR_DEVICE);
            continue;
        }
        items.push_back(CopyItem{c.dst, c.src, c.bytes, (uint32_t)chunks, 0});
        chunks += (c.bytes + cb - 1) / cb;
        if (chunks > 0x7fffffffu) return TBC_ERR_INVALID_ARGUMENT;
    }
    note_write(e); // (unaligned copies above were enqueued already)
    if (items.empty()) return TBC_OK;
    const uint64_t need = sizeof(CopyItem) * items.size();
    if (need > Staging::kSlotBytes) return TBC_ERR_CAPACITY;
    if (need > e->copy_desc_size) { // grows once (a stream drain)
        if (hipStreamSynchronize(e->stream) != hipSuccess) return failed(TBC_ERR_DEVICE);
        if (e->copy_desc) hipFree(e->copy_desc);
        e->copy_desc = nullptr;
        e->copy_desc_size = 0;
        const uint64_t want = align_up(need, 1ull << 16);
        if (hipMalloc((void **)&e->copy_desc, want) != hipSuccess) return failed(TBC_ERR_OUT_OF_MEMORY);
        e->copy_desc_size = want;
    }
    // The descriptors go through a pinned slot (a small one when they fit),
    // reusable once the stream has passed this copy.
    const bool small = need <= DescRing::kSlotBytes;
    int slot = 0;
    uint8_t *host = small ? e->desc.take(&slot) : e->staging.take(&slot);
    if (!host) return failed(TBC_ERR_DEVICE);
    memcpy(host, items.data(), need);
    bool ok = launch_upload(e->copy_desc, host, need, e->stream) == 0 &&
              launch_copy_batch((const CopyItem *)e->copy_desc, (uint32_t)items.size(), (uint32_t)chunks,
                                e->stream) == 0;
    hipEvent_t &ev = small ? e->desc.ev[slot] : e->staging.ev[slot];
    ok = hipEventRecord(ev, e->stream) == hipSuccess && ok;
    (small ? e->desc.used[slot] : e->staging.used[slot]) = true;
    return ok ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_memset_device(tbc_engine *e, void *dst, int value, uint64_t bytes) {
    if (!e) return TBC_ERR_INVALID_ARGUMENT;
    if (!bytes) return TBC_OK;
    hipSetDevice(e->device);
    if (!wait_seal(e) || hipMemsetAsync(dst, value, bytes, e->stream) != hipSuccess)
        return failed(TBC_ERR_DEVICE);
    return hipStreamSynchronize(e->stream) == hipSuccess ? TBC_OK : failed(TBC_ERR_DEVICE);
}

static bool sync_streams(tbc_engine *e) {
    hipSetDevice(e->device);
    flush_tail(e, true);
    bool ok = hipStreamSynchronize(e->stream) == hipSuccess;
    for (int t = 0; t < e->ntails; t++) ok = ok && hipStreamSynchronize(e->tail[t]) == hipSuccess;
    return ok;
}

tbc_status tbc_engine_stream(tbc_engine *e, void **out_stream) {
    if (!e || !out_stream) return TBC_ERR_INVALID_ARGUMENT;
    *out_stream = (void *)e->stream;
    return TBC_OK;
}

tbc_status tbc_synchronize(tbc_engine *e) {
    if (!e) return TBC_ERR_INVALID_ARGUMENT;
    return sync_streams(e) ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_manifest_close_status(tbc_grid *g) {
    if (!g) return TBC_ERR_INVALID_ARGUMENT;
    tbc_engine *e = g->engine;
    hipSetDevice(e->device);
    // The closes are engine-stream work: once the stream has passed them,
    // the word holds whether any of them refused to link (set by the chain
    // kernel), reported here once.
    uint32_t err = 0;
    if (hipMemcpyAsync(&err, g->d_error, 4, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        return failed(TBC_ERR_DEVICE);
    if (!err) return TBC_OK;
    if (hipMemsetAsync(g->d_error, 0, 4, e->stream) != hipSuccess || hipStreamSynchronize(e->stream) != hipSuccess)
        return failed(TBC_ERR_DEVICE);
    return TBC_ERR_BLOCK_INVALID;
}

tbc_status tbc_checksum_batch(tbc_engine *e, const void *const *messages, const uint64_t *lengths, uint32_t count,
                              uint8_t *checksums_out) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    flush_tail(e);
    if (!e || (count && (!messages || !lengths || !checksums_out))) return TBC_ERR_INVALID_ARGUMENT;
    if (!count) return TBC_OK;
    for (uint32_t i = 0; i < count; i++)
        if (lengths[i] > 0xffffffffull || (lengths[i] && !messages[i])) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    if (!join_tails(e)) return failed(TBC_ERR_DEVICE); // the messages may be blocks a batch tail still writes
    uint64_t rd = 0, rh = 0; // regions for this synchronous call, closed before it returns
    uint8_t *d = e->dev.open(16ull * count + 16ull * count, &rd);
    uint8_t *h = d ? e->host.open(16ull * count + 16ull * count, &rh) : nullptr;
    if (!d || !h) {
        if (d) e->dev.close(rd);
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    uint64_t *hp = (uint64_t *)h;
    uint64_t *hl = hp + count;
    for (uint32_t i = 0; i < count; i++) {
        hp[i] = lengths[i] ? (uint64_t)(uintptr_t)messages[i] : (uint64_t)(uintptr_t)d; // empty: any readable pointer
        hl[i] = lengths[i];
    }
    tbc_status st = TBC_OK;
    if (hipMemcpyAsync(d, h, 16ull * count, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        launch_checksum_batch((const uint64_t *)d, (const uint64_t *)d + count, count, d + 16ull * count,
                              e->stream) != 0 ||
        hipMemcpyAsync(h + 16ull * count, d + 16ull * count, 16ull * count, hipMemcpyDeviceToHost, e->stream) !=
            hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        st = failed(TBC_ERR_DEVICE);
    if (st == TBC_OK) memcpy(checksums_out, h + 16ull * count, 16ull * count);
    e->dev.close(rd);
    e->host.close(rh);
    return st;
}

tbc_status tbc_blocks_validate(tbc_engine *e, const void *const *blocks, const uint64_t *expect_checksums,
                               const uint64_t *expect_addresses, uint32_t count, uint8_t *results_out) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    flush_tail(e);
    if (!e || (count && (!blocks || !expect_checksums || !expect_addresses || !results_out)))
        return TBC_ERR_INVALID_ARGUMENT;
    if (!count) return TBC_OK;
    for (uint32_t i = 0; i < count; i++)
        if (!blocks[i] || ((uintptr_t)blocks[i] & 15)) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    if (!join_tails(e)) return failed(TBC_ERR_DEVICE); // the messages may be blocks a batch tail still writes
    const uint64_t in_bytes = 32ull * count, out_off = align_up(in_bytes, 256);
    uint64_t rd = 0, rh = 0; // regions for this synchronous call, closed before it returns
    uint8_t *d = e->dev.open(out_off + count, &rd);
    uint8_t *h = d ? e->host.open(out_off + count, &rh) : nullptr;
    if (!d || !h) {
        if (d) e->dev.close(rd);
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    uint64_t *hp = (uint64_t *)h, *hx = hp + count;
    for (uint32_t i = 0; i < count; i++) {
        hp[i] = (uint64_t)(uintptr_t)blocks[i];
        hx[3 * i] = expect_checksums[2 * i];
        hx[3 * i + 1] = expect_checksums[2 * i + 1];
        hx[3 * i + 2] = expect_addresses[i];
    }
    tbc_status st = TBC_OK;
    if (hipMemcpyAsync(d, h, in_bytes, hipMemcpyHostToDevice, e->stream) != hipSuccess ||
        launch_validate_blocks((const uint64_t *)d, (const uint64_t *)d + count, count, e->block_size, d + out_off,
                               e->stream) != 0 ||
        hipMemcpyAsync(h + out_off, d + out_off, count, hipMemcpyDeviceToHost, e->stream) != hipSuccess ||
        hipStreamSynchronize(e->stream) != hipSuccess)
        st = failed(TBC_ERR_DEVICE);
    if (st == TBC_OK) memcpy(results_out, h + out_off, count);
    e->dev.close(rd);
    e->host.close(rh);
    return st;
}

static tbc_status sort_batch(tbc_engine *e, const tbc_sort_job *jobs, uint32_t count) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    if (!e || (count && !jobs)) return TBC_ERR_INVALID_ARGUMENT;
    std::vector<SortItem> items(count);
    for (uint32_t k = 0; k < count; k++) {
        const tbc_sort_job &j = jobs[k];
        Layout L;
        if (!compute_layout(&j.tree, e->block_size, &L) || (j.count && !j.values) || ((uintptr_t)j.values & 15) ||
            ((uintptr_t)j.values_out & 15))
            return TBC_ERR_INVALID_ARGUMENT;
        const uint64_t nb = (uint64_t)j.count * j.tree.value_size;
        if (j.values_out && j.count && (uint8_t *)j.values_out < (uint8_t *)j.values + nb &&
            (uint8_t *)j.values < (uint8_t *)j.values_out + nb)
            return TBC_ERR_INVALID_ARGUMENT; // overlapping out of place
        items[k] = SortItem{j.values, j.count, j.tree.value_size, j.tree.timestamp_offset, j.tree.key_kind,
                            j.values_out};
    }
    hipSetDevice(e->device);
    // The bar-end sort runs on the engine stream (a sort stream of its own
    // shared a hardware queue with a tail and measured slower: round 3,
    // config 1 130 vs 75 ms, config 3 4.28 vs 3.78 ms).
    hipStream_t ss = e->stream;
    const uint64_t need = sort_scratch_bytes(items.data(), count);
    const uint64_t host_need = sort_host_bytes(items.data(), count);
    if (host_need > Staging::kSlotBytes) return TBC_ERR_CAPACITY;
    if (need > e->sort_scratch_size) { // grows once per larger bar (a stream drain)
        if (hipStreamSynchronize(e->stream) != hipSuccess) return failed(TBC_ERR_DEVICE);
        if (e->sort_scratch) hipFree(e->sort_scratch);
        e->sort_scratch = nullptr;
        e->sort_scratch_size = 0;
        const uint64_t want = align_up(need + need / 8, 1ull << 24);
        if (hipMalloc((void **)&e->sort_scratch, want) != hipSuccess) {
            e->sort_scratch = nullptr;
            return failed(TBC_ERR_OUT_OF_MEMORY);
        }
        e->sort_scratch_size = want;
    }
    const uint64_t words = sort_status_words(items.data(), count);
    if (words > e->sort_status_words) {
        if (hipStreamSynchronize(e->stream) != hipSuccess) return failed(TBC_ERR_DEVICE);
        if (e->sort_status) hipFree(e->sort_status);
        e->sort_status = nullptr;
        e->sort_status_words = 0;
        const uint64_t want = align_up(words + words / 8, 1ull << 20);
        if (hipMalloc((void **)&e->sort_status, 8 * want) != hipSuccess) {
            e->sort_status = nullptr;
            return failed(TBC_ERR_OUT_OF_MEMORY);
        }
        if (hipMemsetAsync(e->sort_status, 0, 8 * want, e->stream) != hipSuccess ||
            hipStreamSynchronize(e->stream) != hipSuccess)
            return failed(TBC_ERR_DEVICE);
        e->sort_status_words = want;
    }
    // The descriptors go through a pinned slot (a small one when they fit),
    // reusable once the stream has passed this sort.
    const bool small = host_need <= DescRing::kSlotBytes;
    int slot = 0;
    uint8_t *host = small ? e->desc.take(&slot) : e->staging.take(&slot);
    if (!host) return failed(TBC_ERR_DEVICE);
    hipEvent_t &slot_ev = small ? e->desc.ev[slot] : e->staging.ev[slot];
    note_write(e);
    int rc = launch_sort_batch(items.data(), count, e->sort_scratch, e->sort_scratch_size, e->sort_status,
                               e->sort_status_words, &e->sort_epoch, host, ss);
    if (hipEventRecord(slot_ev, ss) != hipSuccess) rc = -1;
    if (rc) {
        const hipError_t err = hipGetLastError();
        fprintf(stderr, "tbc: bar-end sort of %u tables not enqueued (step %d): %s (%d)\n", count, rc,
                hipGetErrorString(err), (int)err);
    }
    (small ? e->desc.used[slot] : e->staging.used[slot]) = true;
    return rc == 0 ? TBC_OK : failed(TBC_ERR_DEVICE);
}

tbc_status tbc_sort_values_batch(tbc_engine *e, const tbc_sort_job *jobs, uint32_t count) {
    return sort_batch(e, jobs, count);
}

tbc_status tbc_sort_values_async(tbc_engine *e, const tbc_tree *tree, void *values, uint32_t count) {
    if (!e || !tree) return TBC_ERR_INVALID_ARGUMENT;
    tbc_sort_job j{};
    j.tree = *tree;
    j.values = values;
    j.count = count;
    return sort_batch(e, &j, 1);
}

tbc_status tbc_sort_values(tbc_engine *e, const tbc_tree *tree, void *values, uint32_t count) {
    flush_tail(e);
    tbc_status st = tbc_sort_values_async(e, tree, values, count);
    if (st != TBC_OK) return st;
    return sync_streams(e) ? TBC_OK : failed(TBC_ERR_DEVICE);
}

// Host image of kway.hip's KPair (kway_pair_bytes() checks the size).
struct KPairHost {
    uint64_t a, b, na, nb, out, n_out;
    uint32_t tile_base, split_base, tiles_cap, pad;
};

tbc_status tbc_kway_merge_submit(tbc_engine *e, const tbc_tree *tree, const tbc_segment *streams,
                                 uint32_t stream_count, uint32_t descending, void *out_values, tbc_kway **out) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    flush_tail(e);
    Layout L;
    if (!e || !tree || !out || (stream_count && !streams) || stream_count > TBC_KWAY_STREAMS_MAX ||
        !compute_layout(tree, e->block_size, &L) || ((uintptr_t)out_values & 15) ||
        kway_pair_bytes() != sizeof(KPairHost))
        return TBC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    uint64_t n = 0;
    for (uint32_t s = 0; s < stream_count; s++) {
        if (streams[s].count && (!streams[s].values || ((uintptr_t)streams[s].values & 15)))
            return TBC_ERR_INVALID_ARGUMENT;
        n += streams[s].count;
    }
    if (n >= 0x7fffffffull) return TBC_ERR_INVALID_ARGUMENT;
    if (n && !out_values) return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    tbc_kway *k = new (std::nothrow) tbc_kway();
    if (!k) return failed(TBC_ERR_OUT_OF_MEMORY);
    k->engine = e;
    if (!n) { // nothing to merge: complete at once
        k->complete = true;
        *out = k;
        return TBC_OK;
    }
    const uint32_t vs = tree->value_size, T = kway_pair_tile();
    // The tree of levels: level 0 pairs streams (2q, 2q + 1), the higher one
    // first on equal keys (an odd last stream pairs with nothing, which still
    // collapses its runs); every next level pairs the previous outputs.
    // Counts: [0, k) the input counts, then one output count per pair.
    struct Node { uint64_t ptr; uint32_t count_slot; uint64_t cap; };
    std::vector<Node> cur;
    std::vector<uint32_t> counts(stream_count);
    for (uint32_t s = 0; s < stream_count; s++) {
        cur.push_back(Node{(uint64_t)(uintptr_t)streams[s].values, s, streams[s].count});
        counts[s] = streams[s].count;
    }
    std::vector<std::vector<KPairHost>> levels;
    uint32_t next_count = stream_count;
    const uint32_t empty_slot = 2 * TBC_KWAY_STREAMS_MAX + 1; // always zero
    uint64_t max_slots = 0, max_tiles = 0;
    int level = 0;
    // temp output offsets (bytes) inside ping-pong buffer level % 2; final level writes out_values
    while (true) {
        const bool last = cur.size() <= 2;
        std::vector<KPairHost> pairs;
        std::vector<Node> nxt;
        uint64_t off = 0;
        uint32_t tiles = 0, slots = 0;
        for (size_t q = 0; q < cur.size(); q += 2) {
            const Node lo = cur[q];
            const bool has_hi = q + 1 < cur.size();
            KPairHost P{};
            const Node A = has_hi ? cur[q + 1] : lo; // the higher stream (or the only one)
            P.a = A.ptr;
            P.na = A.count_slot;                      // patched to device pointers below
            P.b = has_hi ? lo.ptr : A.ptr;
            P.nb = has_hi ? lo.count_slot : empty_slot;
            const uint64_t cap = A.cap + (has_hi ? lo.cap : 0);
            P.out = last ? (uint64_t)(uintptr_t)out_values : off; // temp: offset, patched below
            P.n_out = next_count;
            P.tile_base = tiles;
            P.split_base = slots;
            P.tiles_cap = (uint32_t)((cap + T - 1) / T);
            tiles += P.tiles_cap;
            slots += P.tiles_cap + 1;
            nxt.push_back(Node{last ? (uint64_t)(uintptr_t)out_values : off, next_count, cap});
            off += cap * vs;
            next_count++;
            pairs.push_back(P);
        }
        max_slots = std::max<uint64_t>(max_slots, slots);
        max_tiles = std::max<uint64_t>(max_tiles, tiles);
        levels.push_back(pairs);
        level++;
        if (last) break;
        cur = nxt;
        // mark the offsets of this level's outputs as temp (resolved when the buffers exist)
        for (auto &nd : cur) nd.ptr |= (1ull << 63) | ((uint64_t)((level - 1) & 1) << 62);
    }
    // Device memory: temp ping-pong buffers (stream-ordered), scratch, counts, descriptors.
    const uint64_t temp_bytes = align_up(n * vs, 256);
    const uint64_t n_levels = levels.size();
    uint8_t *temp[2] = {nullptr, nullptr};
    const uint64_t scratch_bytes = align_up(4 * max_slots, 256) + align_up(8 * 2 * (T / 64) * max_tiles, 256) +
                                   2 * align_up(4 * max_tiles, 256);
    const uint64_t count_bytes = align_up(4 * (2 * TBC_KWAY_STREAMS_MAX + 2), 256);
    uint64_t npairs_total = 0;
    for (auto &lv : levels) npairs_total += lv.size();
    const uint64_t desc_bytes = align_up(sizeof(KPairHost) * npairs_total, 256);
    const uint64_t need = 2 * temp_bytes + scratch_bytes + count_bytes + desc_bytes;
    if (need > e->kway_scratch_size) { // grows once per larger merge (a stream drain)
        if (hipStreamSynchronize(e->stream) != hipSuccess) {
            delete k;
            return failed(TBC_ERR_DEVICE);
        }
        if (e->kway_scratch) hipFree(e->kway_scratch);
        e->kway_scratch = nullptr;
        e->kway_scratch_size = 0;
        const uint64_t want = align_up(need + need / 8, 1ull << 24);
        if (hipMalloc((void **)&e->kway_scratch, want) != hipSuccess) {
            e->kway_scratch = nullptr;
            delete k;
            return failed(TBC_ERR_OUT_OF_MEMORY);
        }
        e->kway_scratch_size = want;
    }
    temp[0] = e->kway_scratch;
    temp[1] = e->kway_scratch + temp_bytes;
    uint8_t *scratch = e->kway_scratch + 2 * temp_bytes;
    uint8_t *h = e->host.open(count_bytes + desc_bytes + 256, &k->host_region);
    if (!h) {
        delete k;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    k->arena = true;
    uint32_t *splits = (uint32_t *)scratch;
    uint64_t *masks = (uint64_t *)(scratch + align_up(4 * max_slots, 256));
    uint32_t *tile_cnt = (uint32_t *)((uint8_t *)masks + align_up(8 * 2 * (T / 64) * max_tiles, 256));
    uint32_t *tile_off = (uint32_t *)((uint8_t *)tile_cnt + align_up(4 * max_tiles, 256));
    uint32_t *d_counts = (uint32_t *)(scratch + scratch_bytes);
    uint8_t *d_desc = scratch + scratch_bytes + count_bytes;
    uint32_t *h_counts = (uint32_t *)h;
    KPairHost *h_desc = (KPairHost *)(h + count_bytes);
    memset(h_counts, 0, count_bytes);
    for (uint32_t s = 0; s < stream_count; s++) h_counts[s] = counts[s];
    auto resolve = [&](uint64_t ptr) -> uint64_t {
        if (!(ptr >> 63)) return ptr;
        const int buf = (int)((ptr >> 62) & 1);
        return (uint64_t)(uintptr_t)temp[buf] + (ptr & ((1ull << 62) - 1));
    };
    uint64_t di = 0;
    for (uint64_t lv = 0; lv < n_levels; lv++) {
        for (auto &P : levels[lv]) {
            KPairHost Q = P;
            Q.a = resolve(P.a);
            Q.b = resolve(P.b);
            Q.na = (uint64_t)(uintptr_t)(d_counts + P.na);
            Q.nb = (uint64_t)(uintptr_t)(d_counts + P.nb);
            Q.n_out = (uint64_t)(uintptr_t)(d_counts + P.n_out);
            if (lv + 1 < n_levels) Q.out = (uint64_t)(uintptr_t)temp[lv & 1] + P.out;
            h_desc[di++] = Q;
        }
    }
    k->h_count = h_counts + (2 * TBC_KWAY_STREAMS_MAX); // the final count lands here
    const uint32_t final_slot = levels.back()[0].n_out;
    k->done = take_event(e);
    note_write(e);
    bool ok = k->done && hipMemcpyAsync(d_counts, h_counts, count_bytes + desc_bytes, hipMemcpyHostToDevice, e->stream) ==
                        hipSuccess;
    di = 0;
    for (uint64_t lv = 0; ok && lv < n_levels; lv++) {
        uint32_t slots = 0, tiles = 0;
        for (auto &P : levels[lv]) {
            slots += P.tiles_cap + 1;
            tiles += P.tiles_cap;
        }
        ok = launch_kway_level(tree->key_kind, descending != 0, d_desc + sizeof(KPairHost) * di,
                               (uint32_t)levels[lv].size(), slots, tiles, vs, tree->timestamp_offset, splits, masks,
                               tile_cnt, tile_off, e->stream) == 0;
        if (!ok) fprintf(stderr, "tbc: k-way level %u (%u pairs, %u tiles) failed to launch: %s\n", (unsigned)lv,
                         (unsigned)levels[lv].size(), tiles, hipGetErrorString(hipGetLastError()));
        debug_stage(e->stream, "kway level");
        di += levels[lv].size();
    }
    ok = ok && hipMemcpyAsync(k->h_count, d_counts + final_slot, 4, hipMemcpyDeviceToHost, e->stream) == hipSuccess &&
         hipEventRecord(k->done, e->stream) == hipSuccess;
    if (!ok) {
        fprintf(stderr, "tbc: k-way merge enqueue failed: %s\n", hipGetErrorString(hipGetLastError()));
        hipStreamSynchronize(e->stream);
        tbc_kway_release(k);
        return failed(TBC_ERR_DEVICE);
    }
    *out = k;
    return TBC_OK;
}

tbc_status tbc_kway_poll(tbc_kway *k) {
    if (!k) return TBC_ERR_INVALID_ARGUMENT;
    if (k->complete) return k->result;
    hipSetDevice(k->engine->device);
    const hipError_t q = event_query(k->done);
    if (q == hipErrorNotReady) return TBC_PENDING;
    if (q != hipSuccess) fprintf(stderr, "tbc: k-way merge failed on the device: %s (%d)\n", hipGetErrorString(q), (int)q);
    k->complete = true;
    k->result = q == hipSuccess ? TBC_OK : failed(TBC_ERR_DEVICE);
    if (k->result == TBC_OK) k->count = *k->h_count;
    return k->result;
}

tbc_status tbc_kway_wait(tbc_kway *k) {
    if (!k) return TBC_ERR_INVALID_ARGUMENT;
    if (k->complete) return k->result;
    hipSetDevice(k->engine->device);
    if (const hipError_t q = hipEventSynchronize(k->done); q != hipSuccess) {
        fprintf(stderr, "tbc: k-way merge failed on the device: %s (%d)\n", hipGetErrorString(q), (int)q);
        k->complete = true;
        k->result = failed(TBC_ERR_DEVICE);
        return k->result;
    }
    return tbc_kway_poll(k);
}

tbc_status tbc_kway_count(const tbc_kway *k, uint64_t *out_count) {
    if (!k || !out_count) return TBC_ERR_INVALID_ARGUMENT;
    if (!k->complete) return TBC_PENDING;
    if (k->result != TBC_OK) return k->result;
    *out_count = k->count;
    return TBC_OK;
}

void tbc_kway_release(tbc_kway *k) {
    if (!k) return;
    tbc_engine *e = k->engine;
    hipSetDevice(e->device);
    if (!k->complete && k->done) hipEventSynchronize(k->done);
    if (k->done) e->event_pool.push_back(k->done);
    if (k->arena) e->host.close(k->host_region);
    delete k;
}

tbc_status tbc_kway_merge(tbc_engine *e, const tbc_tree *tree, const tbc_segment *streams, uint32_t stream_count,
                          uint32_t descending, void *out_values, uint64_t *out_count) {
    if (!out_count) return TBC_ERR_INVALID_ARGUMENT;
    *out_count = 0;
    tbc_kway *k = nullptr;
    tbc_status st = tbc_kway_merge_submit(e, tree, streams, stream_count, descending, out_values, &k);
    if (st != TBC_OK) return st;
    st = tbc_kway_wait(k);
    if (st == TBC_OK) st = tbc_kway_count(k, out_count);
    tbc_kway_release(k);
    return st;
}

// A batch's chains (data-block headers and checksums) and index blocks on
// tail stream T, after its front.
static bool tail_chains(tbc_batch *b, hipStream_t T, const JobDesc *d_jobs, int njobs, uint32_t dblocks,
                        uint32_t tables, JobResultDev *d_res, uint8_t *d_infos, const uint64_t *d_status,
                        const uint32_t *d_block_tile, const SplitDesc *d_splits, const uint32_t *d_ready, bool compact) {
    return launch_blocks_tail(d_jobs, njobs, dblocks, tables, d_res, d_infos, d_status, b->engine->masks, d_block_tile,
                              d_splits, d_ready, T, mark_cb, b, compact) == 0;
}

// Grid batch, tail after its chains and index blocks: the input checks
// (after every earlier tail: they read blocks earlier batches sealed), the
// outputs marked trusted, the results, the done events.
static bool grid_tail_rest(tbc_engine *e, tbc_batch *b, int ti) {
    const auto &g = b->gt;
    hipStream_t T = e->tail[ti];
    bool ok = true;
    for (int o = 0; ok && o < e->ntails; o++)
        if (o != ti) ok = hipStreamWaitEvent(T, e->tail_ev[o], 0) == hipSuccess;
    if (ok && g.n_checks)
        ok = launch_grid_expect(g.resolve, g.n_resolve, g.checks, T) == 0 &&
             launch_grid_validate(g.checks, g.n_checks, g.grid->verified, g.half.jobs, g.half.njobs, g.half.res,
                                  e->block_size, T) == 0 &&
             launch_grid_checks(g.checks, g.n_checks, g.grid->verified, g.half.jobs, g.half.njobs, g.half.res,
                                e->block_size, T) == 0;
    // Outputs written by the engine are trusted like the reference's grid
    // cache entries (grid.zig:802-841), once the job's inputs checked out.
    if (ok) ok = launch_grid_mark(g.half.jobs, g.half.njobs, g.grid->verified, g.half.res, T) == 0;
    mark_cb(b, "grid_check");
    ok = ok && hipMemcpyAsync(b->h_results, g.half.res, g.copy_bytes, hipMemcpyDeviceToHost, T) == hipSuccess;
    return ok && hipEventRecord(b->done, T) == hipSuccess && hipEventRecord(e->tail_ev[ti], T) == hipSuccess;
}

static int take_tail(tbc_engine *e) {
    const int ti = e->next_tail;
    e->next_tail = (ti + 1) % e->ntails;
    return ti;
}

// A grid batch's whole tail on the next tail stream, after its front. A
// drain (the caller waits next: no front follows to share the CUs with)
// runs the chains on the full tables, one chain per SIMD (latency regime).
static bool grid_tail_alone(tbc_engine *e, tbc_batch *b, bool drain) {
    const auto &g = b->gt;
    const int ti = take_tail(e);
    hipStream_t T = e->tail[ti];
    bool ok = hipStreamWaitEvent(T, b->fork, 0) == hipSuccess;
    b->mark_stream = T;
    mark_cb(b, "tail_wait");
    if (ok && g.half.njobs)
        ok = tail_chains(b, T, g.half.jobs, g.half.njobs, g.half.dblocks, g.half.tables, g.half.res, g.half.infos,
                         g.status, g.block_tile, g.splits, g.half.ready, !drain);
    return ok && grid_tail_rest(e, b, ti);
}

// Tail pairing (round 5). A grid batch's chains take one AEGIS chain time
// (~2 ms per 1 MiB block) however few blocks it has, and only the tail
// streams (one per hardware queue beside the engine stream: three) run them
// concurrently; config 1's batches have a few hundred blocks each, so three
// tails held ~40 % of the CUs while the batches queued for a tail
// (tail_wait 28 ms per step). A grid batch's tail therefore waits for the
// next grid batch's front and both batches' chains run as ONE launch
// (k_data_blocks_pair) on one tail: twice the chains in flight per tail.
// Any other call launches a waiting tail alone first (flush_tail), so a
// caller that waits for a batch before submitting the next never pairs.
static bool grid_tail_pair(tbc_engine *e, tbc_batch *p, tbc_batch *b) {
    const int ti = take_tail(e);
    hipStream_t T = e->tail[ti];
    bool ok = hipStreamWaitEvent(T, b->fork, 0) == hipSuccess; // after both fronts (engine stream order)
    p->mark_stream = b->mark_stream = T;
    mark_cb(p, "tail_wait");
    mark_cb(b, "tail_wait_paired");
    ok = ok && launch_blocks_tail_pair(p->gt.half, b->gt.half, T, mark_cb, p, b, true) == 0;
    return ok && grid_tail_rest(e, p, ti) && grid_tail_rest(e, b, ti);
}

static void flush_tail(tbc_engine *e, bool drain) {
    tbc_batch *p = e ? e->deferred : nullptr;
    if (!p) return;
    e->deferred = nullptr;
    if (!grid_tail_alone(e, p, drain)) {
        p->complete = true;
        p->result = failed(TBC_ERR_DEVICE);
    }
}

static tbc_status submit_impl(tbc_engine *e, const tbc_compaction *jobs_in, uint32_t count, bool pipeline,
                              tbc_batch **out) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    if (!e || !out || (count && !jobs_in)) return TBC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    hipSetDevice(e->device);
    tbc_batch *b = new (std::nothrow) tbc_batch();
    if (!b) return failed(TBC_ERR_OUT_OF_MEMORY);
    b->engine = e;
    b->count = count;
    b->info_base.resize(count);
    b->status.assign(count, TBC_OK);

    // Validate and describe each compaction (host side of Compaction.start).
    std::vector<JobDesc> hj(count);
    std::vector<uint32_t> order(count);
    uint64_t seg_words = 0, addr_words = 0;
    const uint8_t flags0 = count ? jobs_in[0].flags : 0;
    // Dedup (immutable A), tombstone drops or secondary-index put/remove
    // cancellation (an A tombstone and its B put both vanish, merge.hip) can
    // leave a job's survivors sparse; only then may the block phase
    // pre-assemble (aegis.hip sparse_job decides per job on the device).
    bool maybe_sparse = false;
    for (uint32_t i = 0; i < count; i++)
        maybe_sparse |= jobs_in[i].a_immutable || jobs_in[i].drop_tombstones ||
                        jobs_in[i].tree.usage == TBC_USAGE_SECONDARY_INDEX;
    // Input segments per job (device pointer of the first value, count): given
    // directly, or (grid) one per data block of each input table, the
    // pointers filled on the device from the tables' index blocks.
    std::vector<std::vector<std::pair<uint64_t, uint32_t>>> seg_in(2 * (size_t)count);
    std::vector<InputCheck> checks;      // index blocks now, data blocks' slots filled by k_grid_resolve
    std::vector<ResolveItem> resolve;    // seg field: (job, side, segment) until the bases are known
    std::vector<uint32_t> resolve_side;
    const bool grid_mode = (flags0 & TBC_COMPACTION_GRID) != 0;
    tbc_grid *grid0 = grid_mode && count ? jobs_in[0].grid : nullptr;
    for (uint32_t i = 0; i < count; i++) {
        const tbc_compaction &c = jobs_in[i];
        JobDesc &d = hj[i];
        memset(&d, 0, sizeof d);
        Layout L;
        const bool grid = (c.flags & TBC_COMPACTION_GRID) != 0;
        const bool count_only = (c.flags & TBC_COMPACTION_COUNT_ONLY) != 0;
        if (!compute_layout(&c.tree, e->block_size, &L) || L.index_size > kIndexLdsMax ||
            (c.a_immutable && c.segment_count_a > 1) || (!grid && !c.output_blocks && !count_only) ||
            (c.segment_count_a && !c.segments_a) || (!grid && c.segment_count_b && !c.segments_b) ||
            (c.address_count && !c.addresses) ||
            (c.flags & ~(TBC_COMPACTION_VALUES_ONLY | TBC_COMPACTION_GRID | TBC_COMPACTION_UNIQUE_KEYS |
                         TBC_COMPACTION_COUNT_ONLY)) ||
            ((c.flags ^ flags0) & ~TBC_COMPACTION_UNIQUE_KEYS) || (grid && count_only) ||
            (c.output_offset && !(c.flags & TBC_COMPACTION_VALUES_ONLY)) ||
            (grid && ((c.flags & TBC_COMPACTION_VALUES_ONLY) || c.grid != grid0 || !c.grid || c.grid->engine != e ||
                      (c.table_count_a && (c.a_immutable || !c.tables_a)) || (c.table_count_b && !c.tables_b) ||
                      (!c.a_immutable && c.segment_count_a)))) {
            delete b;
            return TBC_ERR_INVALID_ARGUMENT;
        }
        if (grid)
            for (uint32_t a = 0; a < c.address_count; a++)
                if (c.addresses[a] == 0 || c.addresses[a] > c.grid->block_count) { delete b; return TBC_ERR_INVALID_ARGUMENT; }
        uint64_t na = 0, nb = 0;
        for (int side = 0; side < 2; side++) {
            auto &out_segs = seg_in[2 * (size_t)i + side];
            uint64_t &n_side = side == 0 ? na : nb;
            const uint32_t ntab = grid ? (side == 0 ? c.table_count_a : c.table_count_b) : 0;
            for (uint32_t t = 0; t < ntab; t++) {
                const tbc_table_ref &r = (side == 0 ? c.tables_a : c.tables_b)[t];
                const uint64_t nblk = (r.value_count + L.vcm - 1) / L.vcm;
                if (r.address == 0 || r.address > c.grid->block_count || r.value_count == 0 || nblk > L.dbcm) {
                    delete b;
                    return TBC_ERR_INVALID_ARGUMENT;
                }
                const uint64_t index_ptr = (uint64_t)(uintptr_t)c.grid->base + (r.address - 1) * e->block_size;
                checks.push_back(InputCheck{index_ptr, r.address, {r.checksum[0], r.checksum[1]}, (uint32_t)nblk, i,
                                            4u, 0u});
                for (uint64_t k = 0; k < nblk; k++) {
                    const uint32_t cnt = (uint32_t)std::min<uint64_t>(L.vcm, r.value_count - k * L.vcm);
                    resolve.push_back(ResolveItem{index_ptr, (uint32_t)k, (uint32_t)out_segs.size(), 0u, cnt, i,
                                                  L.cks_off, L.addr_off, 0u});
                    resolve_side.push_back((uint32_t)side);
                    out_segs.push_back({0, cnt}); // pointer from the index block, on the device
                    n_side += cnt;
                }
            }
            const uint32_t ns = grid ? (side == 0 && c.a_immutable ? c.segment_count_a : 0)
                                     : (side == 0 ? c.segment_count_a : c.segment_count_b);
            for (uint32_t s = 0; s < ns; s++) {
                const tbc_segment &g = (side == 0 ? c.segments_a : c.segments_b)[s];
                const uint64_t ptr = (uint64_t)(uintptr_t)g.values;
                if (!g.count || !ptr || (ptr & 15)) { delete b; return TBC_ERR_INVALID_ARGUMENT; }
                out_segs.push_back({ptr, g.count});
                n_side += g.count;
            }
        }
        if (na + nb > 0xffff0000ull) { delete b; return TBC_ERR_INVALID_ARGUMENT; }
        const uint64_t n = na + nb;
        const uint64_t db_max = (n + L.vcm - 1) / L.vcm;
        const uint64_t tables_max = (db_max + L.dbcm - 1) / L.dbcm;
        // (An offset range writes only its data blocks' slots: checked below.)
        if (!count_only && !c.output_offset && db_max + tables_max > c.address_count) {
            delete b;
            return TBC_ERR_CAPACITY;
        }
        if (c.output_offset && n) { // the job's slot of the last global data block this range writes
            const uint64_t k_last = (c.output_offset + n - 1) / L.vcm;
            if (k_last + k_last / L.dbcm + 1 > c.address_count) { delete b; return TBC_ERR_CAPACITY; }
        }
        d.key_kind = c.tree.key_kind;
        d.usage = c.tree.usage;
        d.value_size = c.tree.value_size;
        d.timestamp_offset = c.tree.timestamp_offset;
        d.key_size = L.key_size;
        d.vcm = L.vcm;
        d.dbcm = L.dbcm;
        d.index_size = L.index_size;
        d.idx_checksums_off = L.cks_off;
        d.idx_keys_min_off = L.kmin_off;
        d.idx_keys_max_off = L.kmax_off;
        d.idx_addresses_off = L.addr_off;
        d.block_size = e->block_size;
        d.tree_id = c.tree.tree_id;
        d.a_immutable = c.a_immutable ? 1 : 0;
        d.drop_tombstones = c.drop_tombstones ? 1 : 0;
        d.level_b = c.level_b;
        d.cluster_lo = c.cluster[0];
        d.cluster_hi = c.cluster[1];
        d.snapshot_min = c.snapshot_min;
        d.a.nseg = (uint32_t)seg_in[2 * (size_t)i].size();
        d.a.n = (uint32_t)na;
        d.b.nseg = (uint32_t)seg_in[2 * (size_t)i + 1].size();
        d.b.n = (uint32_t)nb;
        for (int side = 0; side < 2; side++) {
            const auto &segs = seg_in[2 * (size_t)i + side];
            bool uniform = !segs.empty();
            for (size_t q = 0; q + 1 < segs.size() && uniform; q++) uniform = segs[q].second == segs[0].second;
            (side == 0 ? d.a : d.b).uniform = uniform && !segs.empty() && segs.back().second <= segs[0].second
                                                  ? segs[0].second : 0;
        }
        d.address_count = c.address_count;
        d.out_offset = c.output_offset;
        d.out_blocks = grid ? nullptr : (uint8_t *)c.output_blocks;
        d.grid_base = grid ? c.grid->base : nullptr;
        d.merge_tile = kMergeTile;
        d.dblock_max = (uint32_t)db_max;
        d.table_max = (uint32_t)tables_max;
        d.job_index = i;
        seg_words += 2ull * (seg_in[2 * (size_t)i].size() + seg_in[2 * (size_t)i + 1].size()) + 2;
        addr_words += c.address_count;
        order[i] = i;
    }
    // (Round 3's staged merge — values held in registers across a look-back,
    // R + W — measured slower than the mask merge + k_assemble and was
    // removed in round 5)
    for (uint32_t i = 0; i < count; i++) {
        JobDesc &d = hj[i];
        const uint64_t n = (uint64_t)d.a.n + d.b.n;
        d.tile_count = (uint32_t)((n + d.merge_tile - 1) / d.merge_tile);
    }
    // Group jobs by key kind (one kernel instantiation per kind) and assign
    // batch-wide bases in that order.
    std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return hj[x].key_kind < hj[y].key_kind; });
    uint64_t all_tiles = 0;
    for (uint32_t i = 0; i < count; i++) all_tiles += hj[i].tile_count;
    if (!ensure_masks(e, all_tiles * (2 * kMergeTile / 64))) {
        delete b;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    std::vector<JobDesc> sj(count);
    uint32_t tiles = 0, splits = 0, dblocks = 0, tables = 0, infos = 0;
    for (uint32_t k = 0; k < count; k++) {
        sj[k] = hj[order[k]];
        JobDesc &d = sj[k];
        d.tile_base = tiles;
        d.split_base = splits;
        d.dblock_base = dblocks;
        d.table_base = tables;
        d.info_base = infos;
        b->info_base[d.job_index] = infos;
        tiles += d.tile_count;
        splits += d.tile_count + 1;
        dblocks += d.dblock_max;
        tables += d.table_max;
        infos += d.table_max;
    }

    // TBC_COMPACTION_UNIQUE_KEYS is honoured in the latency regime of a plain
    // batch: every chain runs at once, so starting them before any merge is
    // what it buys (aegis.hip produce_unique).
    const bool spec_regime = !grid_mode && !pipeline &&
                             !(flags0 & (TBC_COMPACTION_VALUES_ONLY | TBC_COMPACTION_COUNT_ONLY)) &&
                             (uint64_t)(dblocks + 1) / 2 <= fused_max_chain_waves();
    // (The speculated batch's index blocks and results go to a tail stream:
    // round 3, one box: config 2 2.276/2.251 -> 2.235/2.222 ms.)
    // Pipelined speculated batch (round 4): the speculated bodies are merged
    // on the engine stream (k_merge_unique) and the chains run on a tail
    // stream, packed on a share of the CUs, so chains of batches in flight
    // together share the chip (throughput), instead of one fused block pass
    // on the engine stream holding every SIMD (latency: 2,016 chains at once
    // take one chain's time, ~1.9 ms per 1 MiB block, whatever else waits).
    // Chosen when an earlier batch's tail is still running (the caller
    // pipelines), or always / never with TBC_CONFIG_PIPELINE / _LATENCY.
    const bool spec_pipe = spec_regime && !(e->flags & TBC_CONFIG_LATENCY) &&
                           ((e->flags & TBC_CONFIG_PIPELINE) || !e->tail_out.empty());
    // (Grid batches do not speculate: round 4 merged their UNIQUE_KEYS jobs
    // tile by tile too — bodies written once, R + W instead of the mask merge
    // + assembly's R + 2 W — and config 1 measured slower, 54.2 vs 52.1 ms
    // per step: its half-bars are small, and the speculation's extra launches
    // and recompute phase cost more than the assembly they save. That A/B
    // path was removed in round 6.)
    bool any_unique = false;
    for (uint32_t k = 0; k < count; k++) {
        JobDesc &d = sj[k];
        d.unique = spec_regime && (jobs_in[d.job_index].flags & TBC_COMPACTION_UNIQUE_KEYS) && d.dblock_max > 0;
        any_unique |= d.unique != 0;
    }
    // Pipelined: the speculated jobs' tiles of kUniqueTile positions and
    // their merge-path splits (merge.hip k_merge_unique; round 4 measured it
    // faster than one producer wave per block).
    const bool unique_tiles = any_unique && spec_pipe;
    uint32_t utiles = 0, usplits = 0;
    for (uint32_t k = 0; k < count; k++) {
        JobDesc &d = sj[k];
        d.utile_base = utiles;
        d.usplit_base = usplits;
        d.utile_count = 0;
        if (unique_tiles && d.unique) {
            const uint64_t n = (uint64_t)d.a.n + d.b.n;
            d.utile_count = (uint32_t)((n + kUniqueTile - 1) / kUniqueTile);
            utiles += d.utile_count;
            usplits += d.utile_count + 1;
        }
    }

    // Device layout of the batch.
    const uint64_t sz_jobs = align_up(sizeof(JobDesc) * (uint64_t)count, 256);
    const uint64_t sz_segs = align_up(8 * seg_words + 4 * seg_words, 256);
    const uint64_t sz_addr = align_up(8 * addr_words, 256);
    const uint64_t sz_order = align_up(sizeof(TileRef) * (uint64_t)tiles, 256);
    const uint64_t n_checks = checks.size() + resolve.size(); // index blocks, then data blocks
    const uint64_t sz_checks = align_up(sizeof(InputCheck) * n_checks, 256);
    const uint64_t sz_resolve = align_up(sizeof(ResolveItem) * (uint64_t)resolve.size(), 256);
    const uint64_t sz_in = sz_jobs + sz_segs + sz_addr + sz_order + sz_checks + sz_resolve;
    // tile splits, then (speculated jobs) one split per data block, then the
    // unique-tile splits (pipelined speculated batches)
    const uint64_t sz_splits =
        align_up(sizeof(SplitDesc) * ((uint64_t)splits + (any_unique ? dblocks : 0)) + sizeof(UniqueSplit) * usplits,
                 256) +
        align_up(sizeof(SplitSeg) * (uint64_t)splits, 256);
    // tile status + block_tile + per-block assembled-value counts (throughput regime)
    // tile status, block tiles, per-block landed counts, the assembling
    // merge's look-back words (one per tile) and its ticket counters
    const uint64_t sz_tiles = align_up(8ull * tiles + 8ull * dblocks + 8 + 8ull * tiles + 16 + 32 + 8 + 4ull * tables, 256);
    const uint64_t sz_res = align_up(sizeof(JobResultDev) * (uint64_t)count, 256);
    const uint64_t sz_infos = align_up(kTableInfoSize * (uint64_t)infos, 256);
    uint8_t *dbase = e->dev.open(sz_in + sz_splits + sz_tiles + sz_res + sz_infos, &b->dev_region);
    uint8_t *hbase = dbase ? e->host.open(sz_in + sz_res + sz_infos, &b->host_region) : nullptr;
    if (!dbase || !hbase) {
        if (dbase) e->dev.close(b->dev_region);
        delete b;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    uint8_t *d_in = dbase;
    SplitDesc *d_splits = (SplitDesc *)(dbase + sz_in);
    SplitDesc *d_bsplits = any_unique ? d_splits + splits : nullptr;
    SplitDesc *d_usplits = usplits ? d_splits + splits + dblocks : nullptr;
    SplitSeg *d_ssegs = (SplitSeg *)(dbase + sz_in + sz_splits - align_up(sizeof(SplitSeg) * (uint64_t)splits, 256));
    uint64_t *d_status = (uint64_t *)(dbase + sz_in + sz_splits);
    uint32_t *d_block_tile = (uint32_t *)(d_status + tiles);
    uint32_t *d_ready = d_block_tile + dblocks;
    uint64_t *d_lookback = (uint64_t *)(uintptr_t)align_up((uint64_t)(uintptr_t)(d_ready + dblocks + 2), 8);
    uint32_t *d_ticket = (uint32_t *)(d_lookback + tiles);
    const bool merge_bodies = false;
    JobResultDev *d_res = (JobResultDev *)(dbase + sz_in + sz_splits + sz_tiles);
    uint8_t *d_infos = dbase + sz_in + sz_splits + sz_tiles + sz_res;
    b->h_results = (JobResultDev *)(hbase + sz_in);
    b->h_infos = hbase + sz_in + sz_res;

    // Fill the staging image: segment pointers/prefixes and addresses, with
    // device addresses patched into the job descriptors.
    uint8_t *h_in = hbase;
    uint64_t *hseg = (uint64_t *)(h_in + sz_jobs);
    const uint64_t seg_ptr_words = seg_words;
    uint32_t *hpre = (uint32_t *)(hseg + seg_ptr_words);
    uint64_t *haddr = (uint64_t *)(h_in + sz_jobs + sz_segs);
    const uint64_t dev_seg = (uint64_t)(uintptr_t)(d_in + sz_jobs);
    const uint64_t dev_pre = dev_seg + 8 * seg_ptr_words;
    const uint64_t dev_addr = (uint64_t)(uintptr_t)(d_in + sz_jobs + sz_segs);
    uint64_t sp = 0, ap = 0;
    std::vector<uint64_t> seg_base(2 * (size_t)count);
    for (uint32_t k = 0; k < count; k++) {
        JobDesc &d = sj[k];
        const tbc_compaction &c = jobs_in[d.job_index];
        for (int side = 0; side < 2; side++) {
            const auto &segs = seg_in[2 * (size_t)d.job_index + side];
            seg_base[2 * (size_t)d.job_index + side] = sp;
            const uint32_t ns = (uint32_t)segs.size();
            Stream &st = side == 0 ? d.a : d.b;
            st.seg_ptr = (const uint64_t *)(uintptr_t)(dev_seg + 8 * sp);
            st.seg_pre = (const uint32_t *)(uintptr_t)(dev_pre + 4 * sp);
            uint32_t pre = 0;
            for (uint32_t s = 0; s < ns; s++) {
                hseg[sp + s] = segs[s].first;
                hpre[sp + s] = pre;
                pre += segs[s].second;
            }
            hpre[sp + ns] = pre;
            sp += ns + 1;
        }
        d.addresses = (const uint64_t *)(uintptr_t)(dev_addr + 8 * ap);
        memcpy(haddr + ap, c.addresses, 8ull * c.address_count);
        ap += c.address_count;
    }
    for (uint32_t k = 0; k < count; k++) {
        sj[k].spec_any = d_ticket + 4;
        sj[k].split_segs = d_ssegs + sj[k].split_base;
    }
    memcpy(h_in, sj.data(), sizeof(JobDesc) * count);
    InputCheck *hchecks = (InputCheck *)(h_in + sz_jobs + sz_segs + sz_addr + sz_order);
    InputCheck *d_checks = (InputCheck *)(d_in + sz_jobs + sz_segs + sz_addr + sz_order);
    ResolveItem *hres = (ResolveItem *)(h_in + sz_jobs + sz_segs + sz_addr + sz_order + sz_checks);
    const ResolveItem *d_resolve = (const ResolveItem *)(d_in + sz_jobs + sz_segs + sz_addr + sz_order + sz_checks);
    if (!checks.empty()) memcpy(hchecks, checks.data(), sizeof(InputCheck) * checks.size());
    for (size_t r = 0; r < resolve.size(); r++) {
        ResolveItem it = resolve[r];
        it.seg = (uint32_t)(seg_base[2 * (size_t)it.job + resolve_side[r]] + it.seg);
        it.check = (uint32_t)(checks.size() + r);
        hres[r] = it;
    }
    // Tile order: per key kind (contiguous jobs), round-robin over the jobs.
    TileRef *horder = (TileRef *)(h_in + sz_jobs + sz_segs + sz_addr);
    const TileRef *d_order = (const TileRef *)(d_in + sz_jobs + sz_segs + sz_addr);
    {
        uint32_t o = 0, first = 0;
        while (first < count) {
            uint32_t last = first;
            while (last + 1 < count && sj[last + 1].key_kind == sj[first].key_kind) last++;
            uint32_t max_tiles = 0;
            for (uint32_t k = first; k <= last; k++) max_tiles = std::max(max_tiles, sj[k].tile_count);
            for (uint32_t r = 0; r < max_tiles; r++)
                for (uint32_t k = first; k <= last; k++)
                    if (r < sj[k].tile_count) horder[o++] = TileRef{k, r};
            first = last + 1;
        }
    }

    for (int m = 0; m < kMaxMarks; m++) {
        if (e->flags & TBC_CONFIG_PROFILE) {
            if (e->event_pool.empty()) {
                hipEvent_t ev;
                hipEventCreate(&ev);
                e->event_pool.push_back(ev);
            }
            b->marks[m] = e->event_pool.back();
            e->event_pool.pop_back();
        }
    }
    if (e->event_pool.empty()) {
        hipEvent_t ev;
        hipEventCreate(&ev);
        e->event_pool.push_back(ev);
    }
    b->done = e->event_pool.back();
    e->event_pool.pop_back();

    hipStream_t s = e->stream;
    bool ok = true;
    // A pipelined batch of speculated jobs whose inputs no batch in flight
    // is writing: its descriptors go up and its
    // partition runs on the tail its chains will take (idle by then: three
    // batches back), so the engine stream goes from the previous batch's
    // merge straight to this one's (config 2: ~60 us of upload, partition
    // and launch gaps per step off the engine stream).
    hipStream_t P = s;
    if (spec_pipe && !grid_mode && !(e->flags & TBC_CONFIG_LATENCY)) {
        bool early = count > 0;
        for (uint32_t k = 0; k < count && early; k++) early = sj[k].unique != 0;
        for (uint32_t i = 0; i < count && early; i++)
            for (int side = 0; side < 2 && early; side++)
                for (const auto &g : seg_in[2 * (size_t)i + side]) {
                    const uint64_t lo = g.first, hi = g.first + (uint64_t)g.second * hj[i].value_size;
                    for (const auto &t : e->tail_out)
                        for (const auto &r : t.ranges) early = early && !(lo < r.second && r.first < hi);
                    if (!early) break;
                }
        if (early) {
            b->prep = take_event(e);
            if (b->prep) {
                P = e->tail[e->next_tail];
                // Inputs the engine stream wrote (puts, sorts, copies, earlier
                // batches' outputs not in tail_out) are read here off that
                // stream: P waits for the last such write.
                ok = order_after_writes(e, P);
            }
        }
    }
    // This batch's engine-stream outputs, unless its tail lists them in
    // tail_out (the pipelined and latency-regime speculated batches do).
    const bool outputs_tracked = !grid_mode && !(flags0 & TBC_COMPACTION_COUNT_ONLY) &&
                                 (pipeline || (any_unique && spec_regime));
    if (!outputs_tracked) note_write(e);
    // The descriptors up; tile status, block tiles and results zeroed
    // (contiguous) by the same launch.
    ok = ok && launch_upload(d_in, h_in, sz_in, P, d_status, sz_tiles + sz_res) == 0;
    mark_cb(b, "start");
    if (grid_mode) {
        // Pipelined: the front (input data blocks found through their index
        // blocks, merge, bodies, index block addresses) on the engine stream;
        // the tail (chains, index blocks, input checks, results) on a tail
        // stream. The input checks read blocks earlier batches wrote, so they
        // wait for every earlier tail; nothing else of the tail does.
        if (ok && !resolve.empty())
            ok = launch_grid_resolve(d_resolve, (uint32_t)resolve.size(), (uint64_t *)(uintptr_t)dev_seg, d_checks,
                                     grid0->base, grid0->block_count, e->block_size, d_res, s) == 0;
        // The mask merge, then the bodies (k_assemble) and the index
        // blocks' data addresses.
        if (ok && count)
            ok = launch_merge((const JobDesc *)d_in, sj.data(), (int)count, d_splits, d_status, e->masks,
                              d_block_tile, d_order, d_res, s, mark_cb, b) == 0;
        if (ok && count)
            ok = launch_blocks_front((const JobDesc *)d_in, (int)count, tiles, dblocks, d_ready, d_res, d_status,
                                     e->masks, d_splits, s, mark_cb, b, merge_bodies) == 0;
        b->fork = take_event(e);
        ok = ok && b->fork && hipEventRecord(b->fork, s) == hipSuccess;
        auto &g = b->gt;
        g.half = TailHalf{(const JobDesc *)d_in, (int)count, dblocks, tables, d_res, d_infos, d_ready};
        g.status = d_status;
        g.block_tile = d_block_tile;
        g.splits = d_splits;
        g.resolve = d_resolve;
        g.n_resolve = (uint32_t)resolve.size();
        g.n_checks = (uint32_t)n_checks;
        g.checks = d_checks;
        g.grid = grid0;
        g.copy_bytes = sz_res + sz_infos;
        const bool pairable = e->pair_tails && count && dblocks;
        if (ok && pairable && e->deferred) {
            tbc_batch *p = e->deferred;
            e->deferred = nullptr;
            if (!grid_tail_pair(e, p, b)) {
                p->complete = true;
                p->result = failed(TBC_ERR_DEVICE);
                ok = false;
            }
        } else if (ok && pairable) {
            e->deferred = b;
        } else if (ok) {
            flush_tail(e);
            ok = grid_tail_alone(e, b, false);
        }
    } else if (pipeline) {
        // A group of a split batch: front (merge + bodies) on the engine
        // stream, chains and index blocks on a tail stream, so the group's
        // chains run beside the next group's merge and body assembly.
        if (ok && count)
            ok = launch_merge((const JobDesc *)d_in, sj.data(), (int)count, d_splits, d_status, e->masks,
                              d_block_tile, d_order, d_res, s, mark_cb, b) == 0;
        if (ok && count)
            ok = launch_blocks_front((const JobDesc *)d_in, (int)count, tiles, dblocks, d_ready, d_res, d_status,
                                     e->masks, d_splits, s, mark_cb, b, merge_bodies) == 0;
        const int ti = e->next_tail;
        e->next_tail = (e->next_tail + 1) % e->ntails;
        hipStream_t T = e->tail[ti];
        b->fork = take_event(e);
        ok = ok && b->fork && hipEventRecord(b->fork, s) == hipSuccess && hipStreamWaitEvent(T, b->fork, 0) == hipSuccess;
        b->mark_stream = T;
        mark_cb(b, "tail_wait");
        if (ok && count)
            ok = tail_chains(b, T, (const JobDesc *)d_in, (int)count, dblocks, tables, d_res, d_infos, d_status,
                             d_block_tile, d_splits, d_ready, false);
        ok = ok && hipMemcpyAsync(b->h_results, d_res, sz_res + sz_infos, hipMemcpyDeviceToHost, T) == hipSuccess;
        ok = ok && hipEventRecord(b->done, T) == hipSuccess && hipEventRecord(e->tail_ev[ti], T) == hipSuccess;
        if (ok) {
            tbc_engine::TailOutputs to;
            to.done = take_event(e);
            ok = to.done && hipEventRecord(to.done, T) == hipSuccess;
            for (uint32_t i = 0; ok && i < count; i++) {
                const uint64_t lo = (uint64_t)(uintptr_t)jobs_in[i].output_blocks;
                to.ranges.push_back({lo, lo + (uint64_t)jobs_in[i].address_count * e->block_size});
            }
            if (ok) e->tail_out.push_back(std::move(to));
            else if (to.done) e->event_pool.push_back(to.done);
        }
    } else if (flags0 & TBC_COMPACTION_COUNT_ONLY) {
        // The merge alone: survivor counts (k_tile_scan's results), nothing written.
        b->count_only = true;
        if (ok && count)
            ok = launch_merge((const JobDesc *)d_in, sj.data(), (int)count, d_splits, d_status, e->masks,
                              d_block_tile, d_order, d_res, s, mark_cb, b) == 0;
        // A job with output_blocks also gets its count there (u64, device,
        // stream order), for a caller that exchanges it on the device.
        for (uint32_t i = 0; ok && i < count; i++)
            if (jobs_in[i].output_blocks)
                ok = hipMemcpyAsync(jobs_in[i].output_blocks, &d_res[i].value_count, 8, hipMemcpyDeviceToDevice, s) ==
                     hipSuccess;
        ok = ok && hipMemcpyAsync(b->h_results, d_res, sz_res, hipMemcpyDeviceToHost, s) == hipSuccess;
        ok = ok && hipEventRecord(b->done, s) == hipSuccess;
    } else if (any_unique && spec_pipe) {
        // Front (engine stream): block splits and results of the speculated
        // jobs, the merge of the others and their bodies, the speculated
        // bodies, then the recomputation of broken speculations (merge and
        // bodies; each kernel leaves at once when none broke). Tail: the
        // chains of every data block, the index blocks, the results.
        const JobDesc *dj = (const JobDesc *)d_in;
        bool any_plain = false; // jobs not speculated: mask merge and assembly
        for (uint32_t k = 0; k < count; k++) any_plain |= !sj[k].unique;
        ok = ok && launch_merge_unique(dj, sj.data(), (int)count, d_usplits, d_res, d_ticket + 5, s, mark_cb, b,
                                       P != s ? (void *)P : nullptr, (void *)b->prep) == 0;
        ok = ok && launch_merge(dj, sj.data(), (int)count, d_splits, d_status, e->masks, d_block_tile, d_order,
                                d_res, s, mark_cb, b, 0) == 0;
        if (any_plain) {
            ok = ok && launch_assemble(dj, (int)count, tiles, d_ready, d_res, d_status, e->masks, d_splits, 0, s) == 0;
            mark_cb(b, "assemble");
        }
        ok = ok && launch_merge(dj, sj.data(), (int)count, d_splits, d_status, e->masks, d_block_tile, d_order,
                                d_res, s, mark_cb, b, 1) == 0;
        ok = ok && launch_assemble(dj, (int)count, tiles, d_ready, d_res, d_status, e->masks, d_splits, 1, s) == 0;
        mark_cb(b, "recompute_assemble");
        const int ti = e->next_tail;
        e->next_tail = (e->next_tail + 1) % e->ntails;
        hipStream_t T = e->tail[ti];
        b->fork = take_event(e);
        ok = ok && b->fork && hipEventRecord(b->fork, s) == hipSuccess && hipStreamWaitEvent(T, b->fork, 0) == hipSuccess;
        b->mark_stream = T;
        mark_cb(b, "tail_wait");
        ok = ok && tail_chains(b, T, dj, (int)count, dblocks, tables, d_res, d_infos, d_status, d_block_tile,
                               d_splits, d_ready, false);
        ok = ok && hipMemcpyAsync(b->h_results, d_res, sz_res + sz_infos, hipMemcpyDeviceToHost, T) == hipSuccess;
        ok = ok && hipEventRecord(b->done, T) == hipSuccess && hipEventRecord(e->tail_ev[ti], T) == hipSuccess;
        if (ok) {
            tbc_engine::TailOutputs to;
            to.done = take_event(e);
            ok = to.done && hipEventRecord(to.done, T) == hipSuccess;
            for (uint32_t i = 0; ok && i < count; i++) {
                const uint64_t lo = (uint64_t)(uintptr_t)jobs_in[i].output_blocks;
                to.ranges.push_back({lo, lo + (uint64_t)jobs_in[i].address_count * e->block_size});
            }
            if (ok) e->tail_out.push_back(std::move(to));
            else if (to.done) e->event_pool.push_back(to.done);
        }
    } else if (any_unique) {
        // Speculated jobs: their block splits and results first, then the
        // merge of the others, then ONE block pass for all (speculated
        // producers merge their blocks themselves), then the recomputation of
        // broken speculations (every kernel leaves at once when none broke),
        // then the index blocks.
        const JobDesc *dj = (const JobDesc *)d_in;
        ok = ok && launch_partition_blocks(dj, (int)count, dblocks, d_bsplits, d_res, s) == 0;
        mark_cb(b, "partition_blocks");
        ok = ok && launch_merge(dj, sj.data(), (int)count, d_splits, d_status, e->masks, d_block_tile, d_order,
                                d_res, s, mark_cb, b, 0) == 0;
        ok = ok && launch_blocks(dj, (int)count, tiles, dblocks, tables, d_ready, d_res, d_infos, d_status, e->masks,
                                 d_block_tile, d_splits, false, maybe_sparse, s, mark_cb, b, false, d_bsplits, 0,
                                 false) == 0;
        ok = ok && launch_merge(dj, sj.data(), (int)count, d_splits, d_status, e->masks, d_block_tile, d_order,
                                d_res, s, mark_cb, b, 1) == 0;
        ok = ok && launch_blocks(dj, (int)count, tiles, dblocks, tables, d_ready, d_res, d_infos, d_status, e->masks,
                                 d_block_tile, d_splits, false, true, s, mark_cb, b, false, d_bsplits, 1, false) == 0;
        // The index blocks and the results go to a tail stream, so the next
        // batch's front starts as soon as this batch's data blocks (and any
        // recomputation, which uses the engine's mask buffer) are done. A
        // later batch into the same output blocks waits for this tail.
        const int ti = e->next_tail;
        e->next_tail = (e->next_tail + 1) % e->ntails;
        hipStream_t T = e->tail[ti];
        b->fork = take_event(e);
        ok = ok && b->fork && hipEventRecord(b->fork, s) == hipSuccess && hipStreamWaitEvent(T, b->fork, 0) == hipSuccess;
        b->mark_stream = T;
        ok = ok && launch_index_blocks(dj, (int)count, tables, d_res, d_infos, T) == 0;
        mark_cb(b, "index_blocks");
        ok = ok && hipMemcpyAsync(b->h_results, d_res, sz_res + sz_infos, hipMemcpyDeviceToHost, T) == hipSuccess;
        ok = ok && hipEventRecord(b->done, T) == hipSuccess && hipEventRecord(e->tail_ev[ti], T) == hipSuccess;
        if (ok) {
            tbc_engine::TailOutputs to;
            to.done = take_event(e);
            ok = to.done && hipEventRecord(to.done, T) == hipSuccess;
            for (uint32_t i = 0; ok && i < count; i++) {
                const uint64_t lo = (uint64_t)(uintptr_t)jobs_in[i].output_blocks;
                to.ranges.push_back({lo, lo + (uint64_t)jobs_in[i].address_count * e->block_size});
            }
            if (ok) e->tail_out.push_back(std::move(to));
            else if (to.done) e->event_pool.push_back(to.done);
        }
    } else {
        if (ok && count)
            ok = launch_merge((const JobDesc *)d_in, sj.data(), (int)count, d_splits, d_status, e->masks,
                              d_block_tile, d_order, d_res, s, mark_cb, b) == 0;
        if (ok && count)
            ok = launch_blocks((const JobDesc *)d_in, (int)count, tiles, dblocks, tables, d_ready, d_res, d_infos,
                               d_status, e->masks, d_block_tile, d_splits, (flags0 & TBC_COMPACTION_VALUES_ONLY) != 0,
                               maybe_sparse, s, mark_cb, b, merge_bodies) == 0;
        ok = ok && hipMemcpyAsync(b->h_results, d_res, sz_res + sz_infos, hipMemcpyDeviceToHost, s) == hipSuccess;
        ok = ok && hipEventRecord(b->done, s) == hipSuccess;
    }
    if (!ok) {
        sync_streams(e);
        tbc_batch_release(b);
        return failed(TBC_ERR_DEVICE);
    }
    *out = b;
    return TBC_OK;
}

// Above fused_max_chain_waves() chain waves a batch is in the throughput
// regime: it is split into job groups that pipeline (each group's chains
// beside the next group's merge and bodies).
constexpr uint32_t kMaxGroups = 4; // config 5: 1 -> 16.1, 2 -> 14.6, 3 -> 14.4, 4 -> 14.3, 6 -> 17.2 ms

// The checks submit_impl makes of one non-grid compaction, for a batch that
// is split into groups: every job is checked before any group is enqueued,
// so a rejected batch touches nothing on the device.
static tbc_status check_plain_job(const tbc_engine *e, const tbc_compaction &c, uint8_t flags0) {
    Layout L;
    if (!compute_layout(&c.tree, e->block_size, &L) || L.index_size > kIndexLdsMax ||
        (c.a_immutable && c.segment_count_a > 1) || !c.output_blocks || (c.segment_count_a && !c.segments_a) ||
        (c.segment_count_b && !c.segments_b) || (c.address_count && !c.addresses) ||
        (c.flags & ~(TBC_COMPACTION_VALUES_ONLY | TBC_COMPACTION_GRID | TBC_COMPACTION_UNIQUE_KEYS)) ||
        ((c.flags ^ flags0) & ~TBC_COMPACTION_UNIQUE_KEYS) || (c.flags & TBC_COMPACTION_GRID) || c.output_offset)
        return TBC_ERR_INVALID_ARGUMENT;
    uint64_t n = 0;
    for (int side = 0; side < 2; side++) {
        const uint32_t ns = side == 0 ? c.segment_count_a : c.segment_count_b;
        for (uint32_t k = 0; k < ns; k++) {
            const tbc_segment &g = (side == 0 ? c.segments_a : c.segments_b)[k];
            if (!g.count || !g.values || ((uintptr_t)g.values & 15)) return TBC_ERR_INVALID_ARGUMENT;
            n += g.count;
        }
    }
    if (n > 0xffff0000ull) return TBC_ERR_INVALID_ARGUMENT;
    const uint64_t db_max = (n + L.vcm - 1) / L.vcm;
    if (db_max + (db_max + L.dbcm - 1) / L.dbcm > c.address_count) return TBC_ERR_CAPACITY;
    return TBC_OK;
}

tbc_status tbc_compaction_submit(tbc_engine *e, const tbc_compaction *jobs_in, uint32_t count, tbc_batch **out) {
    if (!e || !out || (count && !jobs_in)) return TBC_ERR_INVALID_ARGUMENT;
    // A grid batch may pair with a deferred grid tail; anything else
    // launches it first.
    if (!count || !(jobs_in[0].flags & TBC_COMPACTION_GRID)) flush_tail(e);
    // A batch with caller-provided output blocks may write blocks an earlier
    // batch's tail (its chains) still reads, when the caller reuses them
    // while that batch is in flight: its fronts then start after that tail.
    // Batches into other blocks overlap earlier tails, as grid batches (whose
    // outputs are freshly acquired addresses) always do.
    if (count && !(jobs_in[0].flags & TBC_COMPACTION_GRID)) {
        hipSetDevice(e->device);
        auto &pend = e->tail_out;
        for (size_t k = 0; k < pend.size();) {
            if (event_query(pend[k].done) == hipSuccess) { // that tail is done with its outputs
                e->event_pool.push_back(pend[k].done);
                pend.erase(pend.begin() + (long)k);
                continue;
            }
            bool alias = false;
            for (uint32_t i = 0; i < count && !alias; i++) {
                const uint64_t lo = (uint64_t)(uintptr_t)jobs_in[i].output_blocks;
                const uint64_t hi = lo + (uint64_t)jobs_in[i].address_count * e->block_size;
                for (const auto &r : pend[k].ranges)
                    if (lo < r.second && r.first < hi) {
                        alias = true;
                        break;
                    }
            }
            if (alias && hipStreamWaitEvent(e->stream, pend[k].done, 0) != hipSuccess) return failed(TBC_ERR_DEVICE);
            k++;
        }
    }
    uint32_t groups = 1;
    std::vector<uint64_t> n(count, 0);
    if (count >= 2 &&
        !(jobs_in[0].flags & (TBC_COMPACTION_GRID | TBC_COMPACTION_VALUES_ONLY | TBC_COMPACTION_COUNT_ONLY))) {
        uint64_t waves = 0;
        for (uint32_t i = 0; i < count; i++) {
            const tbc_compaction &c = jobs_in[i];
            Layout L;
            if (!compute_layout(&c.tree, e->block_size, &L) || (c.segment_count_a && !c.segments_a) ||
                (c.segment_count_b && !c.segments_b))
                return submit_impl(e, jobs_in, count, false, out); // reports the error
            for (uint32_t k = 0; k < c.segment_count_a; k++) n[i] += c.segments_a[k].count;
            for (uint32_t k = 0; k < c.segment_count_b; k++) n[i] += c.segments_b[k].count;
            waves += (n[i] + L.vcm - 1) / L.vcm / 2;
        }
        const uint32_t max_groups = kMaxGroups;
        const uint64_t min_waves = fused_max_chain_waves();
        if (waves > min_waves && max_groups > 1) groups = std::min<uint32_t>(max_groups, count);
    }
    if (groups == 1) return submit_impl(e, jobs_in, count, false, out);
    for (uint32_t i = 0; i < count; i++)
        if (const tbc_status st = check_plain_job(e, jobs_in[i], jobs_in[0].flags); st != TBC_OK) return st;
    // Contiguous groups of about equal input (job order kept inside a group).
    uint64_t total = 0;
    for (uint32_t i = 0; i < count; i++) total += n[i];
    tbc_batch *parent = new (std::nothrow) tbc_batch();
    if (!parent) return failed(TBC_ERR_OUT_OF_MEMORY);
    parent->engine = e;
    parent->count = count;
    parent->job_map.resize(count);
    uint32_t first = 0;
    uint64_t acc = 0;
    for (uint32_t g = 0; g < groups && first < count; g++) {
        uint32_t last = first + 1;
        acc += n[first];
        const uint64_t goal = total * (g + 1) / groups;
        while (last < count && (count - last) > (groups - g - 1) && acc + n[last] / 2 <= goal) acc += n[last++];
        if (g == groups - 1) {
            while (last < count) acc += n[last++];
        }
        tbc_batch *child = nullptr;
        const tbc_status st = submit_impl(e, jobs_in + first, last - first, true, &child);
        if (st != TBC_OK) {
            for (auto it = parent->children.rbegin(); it != parent->children.rend(); ++it) tbc_batch_release(*it);
            delete parent;
            return st;
        }
        for (uint32_t i = first; i < last; i++)
            parent->job_map[i] = {(uint32_t)parent->children.size(), i - first};
        parent->children.push_back(child);
        first = last;
    }
    *out = parent;
    return TBC_OK;
}

tbc_status tbc_compaction_seal(tbc_engine *e, const tbc_seal *sl, tbc_batch **out) {
    if (!no_stale_error()) return TBC_ERR_DEVICE; // an earlier call's unreported failure
    flush_tail(e);
    if (!e || !sl || !out) return TBC_ERR_INVALID_ARGUMENT;
    *out = nullptr;
    Layout L;
    if (!compute_layout(&sl->tree, e->block_size, &L) || L.index_size > kIndexLdsMax || !sl->output_blocks ||
        !sl->addresses || !sl->value_count)
        return TBC_ERR_INVALID_ARGUMENT;
    const uint64_t db = (sl->value_count + L.vcm - 1) / L.vcm, tables = (db + L.dbcm - 1) / L.dbcm;
    if (db + tables > sl->address_count) return TBC_ERR_CAPACITY;
    if ((uint64_t)sl->block_first + sl->block_count > db || (uint64_t)sl->table_first + sl->table_count > tables)
        return TBC_ERR_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    tbc_batch *b = new (std::nothrow) tbc_batch();
    if (!b) return failed(TBC_ERR_OUT_OF_MEMORY);
    b->engine = e;
    b->count = 1;
    b->info_base.assign(1, 0);
    b->status.assign(1, TBC_OK);
    b->seal = true;
    // What this call finishes: its data blocks and tables, their values.
    {
        tbc_compaction_result &r = b->seal_result;
        const uint64_t T = (uint64_t)L.vcm * L.dbcm;
        const uint64_t v0 = (uint64_t)sl->table_first * T;
        const uint64_t v1 = std::min<uint64_t>((uint64_t)(sl->table_first + sl->table_count) * T, sl->value_count);
        r.value_count = sl->table_count ? v1 - v0 : 0;
        r.data_block_count = sl->block_count;
        r.table_count = sl->table_count;
        r.block_count = sl->block_count + sl->table_count;
    }
    JobDesc d;
    memset(&d, 0, sizeof d);
    d.key_kind = sl->tree.key_kind;
    d.usage = sl->tree.usage;
    d.value_size = sl->tree.value_size;
    d.timestamp_offset = sl->tree.timestamp_offset;
    d.key_size = L.key_size;
    d.vcm = L.vcm;
    d.dbcm = L.dbcm;
    d.index_size = L.index_size;
    d.idx_checksums_off = L.cks_off;
    d.idx_keys_min_off = L.kmin_off;
    d.idx_keys_max_off = L.kmax_off;
    d.idx_addresses_off = L.addr_off;
    d.block_size = e->block_size;
    d.tree_id = sl->tree.tree_id;
    d.level_b = sl->level_b;
    d.cluster_lo = sl->cluster[0];
    d.cluster_hi = sl->cluster[1];
    d.snapshot_min = sl->snapshot_min;
    d.address_count = sl->address_count;
    d.out_blocks = (uint8_t *)sl->output_blocks;
    d.merge_tile = kMergeTile;
    d.dblock_max = sl->block_count;
    d.table_max = sl->table_count;
    d.block_lo = sl->block_first;
    d.table_lo = sl->table_first;
    d.seal = 1;
    JobResultDev r0;
    memset(&r0, 0, sizeof r0);
    r0.value_count = sl->value_count;
    r0.data_block_count = (uint32_t)db;
    r0.table_count = (uint32_t)tables;
    r0.block_count = (uint32_t)(db + tables);
    const uint64_t sz_job = align_up(sizeof(JobDesc), 256), sz_addr = align_up(8ull * sl->address_count, 256);
    const uint64_t sz_res = align_up(sizeof(JobResultDev), 256);
    const uint64_t sz_infos = align_up(kTableInfoSize * (uint64_t)std::max<uint32_t>(1, sl->table_count), 256);
    uint8_t *dbase = e->dev.open(sz_job + sz_addr + sz_res + sz_infos, &b->dev_region);
    uint8_t *hbase = dbase ? e->host.open(sz_job + sz_addr + sz_res + sz_infos, &b->host_region) : nullptr;
    if (!dbase || !hbase) {
        if (dbase) e->dev.close(b->dev_region);
        delete b;
        return failed(TBC_ERR_OUT_OF_MEMORY);
    }
    d.addresses = (const uint64_t *)(dbase + sz_job);
    memcpy(hbase, &d, sizeof d);
    memcpy(hbase + sz_job, sl->addresses, 8ull * sl->address_count);
    memcpy(hbase + sz_job + sz_addr, &r0, sizeof r0);
    JobResultDev *d_res = (JobResultDev *)(dbase + sz_job + sz_addr);
    b->h_results = (JobResultDev *)(hbase + sz_job + sz_addr);
    b->h_infos = hbase + sz_job + sz_addr + sz_res;
    b->done = take_event(e);
    b->fork = take_event(e);
    // On a tail stream (round 5): after the engine stream's work so far (the
    // bodies it seals) and after every tail (blocks an earlier seal or batch
    // tail still writes), so the engine stream runs on — a split's seal
    // chains beside the next fronts. Engine-stream copies that read what a
    // seal wrote wait for it (seal_ev, tbc_copy_device_batch).
    const int ti = take_tail(e);
    hipStream_t T = e->tail[ti];
    bool ok = b->done != nullptr && b->fork != nullptr && hipEventRecord(b->fork, e->stream) == hipSuccess &&
              hipStreamWaitEvent(T, b->fork, 0) == hipSuccess;
    for (int o = 0; ok && o < e->ntails; o++)
        if (o != ti) ok = hipStreamWaitEvent(T, e->tail_ev[o], 0) == hipSuccess;
    ok = ok && hipMemcpyAsync(dbase, hbase, sz_job + sz_addr + sz_res, hipMemcpyHostToDevice, T) == hipSuccess &&
         launch_seal((const JobDesc *)dbase, sl->block_count, sl->table_count, d_res, dbase + sz_job + sz_addr + sz_res,
                     T) == 0 &&
         hipMemcpyAsync(b->h_results, d_res, sz_res + sz_infos, hipMemcpyDeviceToHost, T) == hipSuccess &&
         hipEventRecord(b->done, T) == hipSuccess && hipEventRecord(e->tail_ev[ti], T) == hipSuccess &&
         hipEventRecord(e->seal_ev, T) == hipSuccess;
    e->seal_pending = ok;
    if (ok) { // a later batch into these blocks starts after this seal (submit's tail_out check)
        tbc_engine::TailOutputs to;
        to.done = take_event(e);
        ok = to.done && hipEventRecord(to.done, T) == hipSuccess;
        // Only the slots this seal writes (a split rank's output_blocks is
        // its allocation minus the slots before it: ADVICE r5): its data
        // blocks, and the index blocks of their tables and of the sealed ones.
        const uint64_t base = (uint64_t)(uintptr_t)sl->output_blocks, bs = e->block_size;
        auto k_last = [&](uint64_t t) { return std::min<uint64_t>((t + 1) * L.dbcm, db) - 1; };
        uint64_t s_lo = UINT64_MAX, s_hi = 0;
        auto span = [&](uint64_t slot) { s_lo = std::min(s_lo, slot); s_hi = std::max(s_hi, slot + 1); };
        if (sl->block_count) {
            const uint64_t k0 = sl->block_first, k1 = k0 + sl->block_count - 1;
            span(data_block_slot((uint32_t)k0, L.dbcm));
            span(index_block_slot((uint32_t)(k1 / L.dbcm), (uint32_t)k_last(k1 / L.dbcm)));
        }
        if (sl->table_count) {
            span(index_block_slot(sl->table_first, (uint32_t)k_last(sl->table_first)));
            const uint64_t t1 = (uint64_t)sl->table_first + sl->table_count - 1;
            span(index_block_slot((uint32_t)t1, (uint32_t)k_last(t1)));
        }
        if (s_hi > s_lo) to.ranges.push_back({base + s_lo * bs, base + s_hi * bs});
        if (ok) e->tail_out.push_back(std::move(to));
        else if (to.done) e->event_pool.push_back(to.done);
    }
    if (!ok) {
        sync_streams(e);
        tbc_batch_release(b);
        return failed(TBC_ERR_DEVICE);
    }
    *out = b;
    return TBC_OK;
}

static tbc_status batch_finish(tbc_batch *b) {
    b->complete = true;
    b->result = TBC_OK;
    for (uint32_t i = 0; i < b->count; i++) {
        JobResultDev &r = b->h_results[i];
        if (r.invariant) r.status = TBC_ERR_INVARIANT;
        if (r.block_error) r.status = TBC_ERR_BLOCK_INVALID;
        if (r.status != TBC_OK && b->result == TBC_OK) b->result = (tbc_status)r.status;
    }
    return b->result;
}

static tbc_status parent_finish(tbc_batch *b, bool wait) {
    tbc_status res = TBC_OK;
    for (tbc_batch *c : b->children) {
        const tbc_status st = wait ? tbc_batch_wait(c) : tbc_batch_poll(c);
        if (st == TBC_PENDING) return TBC_PENDING;
        if (st != TBC_OK && res == TBC_OK) res = st;
    }
    b->complete = true;
    b->result = res;
    return res;
}

tbc_status tbc_batch_poll(tbc_batch *b) {
    flush_tail(b ? b->engine : nullptr);
    if (!b) return TBC_ERR_INVALID_ARGUMENT;
    if (b->complete) return b->result;
    if (!b->children.empty()) return parent_finish(b, false);
    hipSetDevice(b->engine->device);
    hipError_t q = event_query(b->done);
    if (q == hipErrorNotReady) return TBC_PENDING;
    if (q != hipSuccess) {
        fprintf(stderr, "tbc: batch failed on the device: %s (%d)\n", hipGetErrorString(q), (int)q);
        b->complete = true;
        b->result = failed(TBC_ERR_DEVICE);
        return b->result;
    }
    return batch_finish(b);
}

tbc_status tbc_batch_wait(tbc_batch *b) {
    flush_tail(b ? b->engine : nullptr, true);
    if (!b) return TBC_ERR_INVALID_ARGUMENT;
    if (b->complete) return b->result;
    if (!b->children.empty()) return parent_finish(b, true);
    hipSetDevice(b->engine->device);
    // Poll like the adapter's event loop would (tbc_batch_poll), instead of a
    // blocking hipEventSynchronize whose OS wake-up adds milliseconds of
    // jitter: spin for the first 200 us, then yield the core between polls
    // (20 us sleeps), so a long batch does not hold a host core.
    hipError_t q;
    const auto t0 = std::chrono::steady_clock::now();
    while ((q = event_query(b->done)) == hipErrorNotReady) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) {
            const timespec ts{0, 20000};
            nanosleep(&ts, nullptr);
        }
    }
    if (q != hipSuccess) {
        fprintf(stderr, "tbc: batch failed on the device: %s (%d)\n", hipGetErrorString(q), (int)q);
        b->complete = true;
        b->result = failed(TBC_ERR_DEVICE);
        return b->result;
    }
    return batch_finish(b);
}

tbc_status tbc_batch_result(tbc_batch *b, uint32_t index, tbc_compaction_result *out, uint8_t *table_infos,
                            uint32_t table_info_capacity) {
    if (!b || !out || index >= b->count) return TBC_ERR_INVALID_ARGUMENT;
    if (!b->complete) return TBC_PENDING;
    if (!b->children.empty()) {
        const auto m = b->job_map[index];
        return tbc_batch_result(b->children[m.first], m.second, out, table_infos, table_info_capacity);
    }
    if (b->result == TBC_ERR_DEVICE) return failed(TBC_ERR_DEVICE);
    const JobResultDev &r = b->h_results[index];
    out->value_count = r.value_count;
    out->data_block_count = r.data_block_count;
    out->table_count = r.table_count;
    out->block_count = r.block_count;
    out->status = r.status;
    if (b->seal) {
        *out = b->seal_result;
        out->status = r.status;
    }
    if (b->count_only) out->data_block_count = out->table_count = out->block_count = 0; // nothing written
    if (table_infos) {
        if (table_info_capacity < out->table_count) return TBC_ERR_CAPACITY;
        memcpy(table_infos, b->h_infos + (size_t)b->info_base[index] * kTableInfoSize,
               (size_t)out->table_count * kTableInfoSize);
    }
    return TBC_OK;
}

tbc_status tbc_batch_speculation(tbc_batch *b, uint32_t index, uint32_t *out) {
    if (!b || !out || index >= b->count) return TBC_ERR_INVALID_ARGUMENT;
    if (!b->complete) return TBC_PENDING;
    if (!b->children.empty()) {
        const auto m = b->job_map[index];
        return tbc_batch_speculation(b->children[m.first], m.second, out);
    }
    if (b->result == TBC_ERR_DEVICE) return failed(TBC_ERR_DEVICE);
    *out = b->h_results[index].spec;
    return TBC_OK;
}

tbc_status tbc_batch_kernel_times(tbc_batch *b, const char **names, double *us, uint32_t capacity,
                                  uint32_t *out_count) {
    if (!b || !out_count) return TBC_ERR_INVALID_ARGUMENT;
    if (!b->complete) return TBC_PENDING;
    if (!b->children.empty()) { // summed over the groups, by name
        std::vector<const char *> nm;
        std::vector<double> t;
        for (tbc_batch *c : b->children) {
            const char *cn[kMaxMarks];
            double cu[kMaxMarks];
            uint32_t k = 0;
            const tbc_status st = tbc_batch_kernel_times(c, cn, cu, kMaxMarks, &k);
            if (st != TBC_OK) return st;
            for (uint32_t i = 0; i < k; i++) {
                size_t j = 0;
                while (j < nm.size() && strcmp(nm[j], cn[i]) != 0) j++;
                if (j == nm.size()) {
                    nm.push_back(cn[i]);
                    t.push_back(0.0);
                }
                t[j] += cu[i];
            }
        }
        uint32_t n = 0;
        for (; n < nm.size() && n < capacity; n++) {
            if (names) names[n] = nm[n];
            if (us) us[n] = t[n];
        }
        *out_count = n;
        return TBC_OK;
    }
    uint32_t n = 0;
    for (int m = 1; m < b->nmarks && n < capacity; m++) {
        float ms = 0;
        if (hipEventElapsedTime(&ms, b->marks[m - 1], b->marks[m]) != hipSuccess) return failed(TBC_ERR_DEVICE);
        if (names) names[n] = b->mark_names[m];
        if (us) us[n] = ms * 1000.0;
        n++;
    }
    *out_count = n;
    return TBC_OK;
}

void tbc_batch_release(tbc_batch *b) {
    flush_tail(b ? b->engine : nullptr);
    if (!b) return;
    if (!b->children.empty()) { // reverse order: the groups' arena regions are a stack
        for (auto it = b->children.rbegin(); it != b->children.rend(); ++it) tbc_batch_release(*it);
        delete b;
        return;
    }
    tbc_engine *e = b->engine;
    hipSetDevice(e->device);
    if (!b->complete && b->done) hipEventSynchronize(b->done);
    for (int m = 0; m < kMaxMarks; m++)
        if (b->marks[m]) e->event_pool.push_back(b->marks[m]);
    if (b->done) e->event_pool.push_back(b->done);
    if (b->fork) e->event_pool.push_back(b->fork);
    if (b->prep) e->event_pool.push_back(b->prep);
    if (b->h_results) {
        e->dev.close(b->dev_region);
        e->host.close(b->host_region);
    }
    delete b;
}

} // extern "C"
