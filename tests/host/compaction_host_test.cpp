// Harness for the C++ host mirror (tigerbeetle_amd/host/compaction.hpp):
// three compactions of one half-bar (disk A + B tables, immutable A sorted on
// the device, and a move-table), scheduled as one GPU batch, compared byte for
// byte with the CPU oracle (oracle/tbc_oracle.c).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../oracle/tbc_oracle.h"
#include "../../tigerbeetle_amd/host/compaction.hpp"

using namespace tbc_host;

static uint64_t sm_state = 0x1234;
static uint64_t rnd() {
    uint64_t z = (sm_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

#define REQUIRE(x)                                                                      \
    do {                                                                                \
        if (!(x)) {                                                                     \
            std::fprintf(stderr, "FAILED %s:%d: %s\n", __FILE__, __LINE__, #x);         \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

struct Buf {
    Engine &e;
    void *p = nullptr;
    size_t n;
    Buf(Engine &e_, size_t n_) : e(e_), n(n_) { check(tbc_device_alloc(e.handle(), n, &p), "alloc"); }
    ~Buf() { tbc_device_free(e.handle(), p); }
    void put(const void *src, size_t bytes, size_t off = 0) {
        check(tbc_copy_to_device(e.handle(), (char *)p + off, src, bytes), "h2d");
    }
    void get(void *dst, size_t bytes, size_t off = 0) {
        check(tbc_copy_to_host(e.handle(), dst, (char *)p + off, bytes), "d2h");
    }
};

// IdTreeValue{id, timestamp, padding} (groove.zig:48-56), ids strictly increasing.
static std::vector<uint8_t> id_values(size_t n, uint64_t start, uint64_t step) {
    std::vector<uint8_t> v(n * 32, 0);
    uint64_t id = start;
    for (size_t i = 0; i < n; i++) {
        id += 1 + rnd() % step;
        uint64_t w[4] = {id, 0, 1 + (rnd() >> 2), 0};
        std::memcpy(&v[32 * i], w, 32);
    }
    return v;
}

int main() {
    const uint32_t bs = 4096;
    Engine eng(0, bs);
    const uint32_t vcm = (bs - 256) / 32; // 120

    // Tree 1: transfers.id with 1000-value tables on 4 KiB blocks.
    tbc_tree id_tree{8, TBC_KEY_ID_U128, TBC_USAGE_GENERAL, 32, 16, 1000};
    tbo_tree oid;
    REQUIRE(tbo_tree_init(&oid, 8, TBO_KEY_ID_U128, TBO_USAGE_GENERAL, 32, 16, 1000, bs) == 0);

    // --- compaction 1: disk A (700 values) + 2 B tables (600, 500) -------------
    auto a = id_values(700, 0, 9);
    auto b = id_values(1100, 3, 9);
    std::vector<std::vector<uint8_t>> blocks; // host blocks for the oracle
    Buf grid(eng, 64 * bs);
    std::vector<tbc_segment> seg_a, seg_b;
    std::vector<tbo_segment> oseg_a, oseg_b;
    uint32_t k = 0;
    auto stage = [&](const std::vector<uint8_t> &vals, size_t first, size_t count, std::vector<tbc_segment> &segs,
                     std::vector<tbo_segment> &osegs) {
        for (size_t i = first; i < first + count; i += vcm, k++) {
            const size_t c = std::min<size_t>(vcm, first + count - i);
            grid.put(&vals[32 * i], 32 * c, (size_t)k * bs + 256);
            segs.push_back(tbc_segment{(char *)grid.p + (size_t)k * bs + 256, (uint32_t)c, 0});
            osegs.push_back(tbo_segment{&vals[32 * i], (uint32_t)c});
        }
    };
    stage(a, 0, 700, seg_a, oseg_a);
    stage(b, 0, 600, seg_b, oseg_b);
    stage(b, 600, 500, seg_b, oseg_b);

    const uint32_t reserve1 = 3 * (9 + 1); // (|B| + 1) * block_count_max (compaction.zig:316-318)
    std::vector<uint64_t> addrs1(reserve1);
    for (uint32_t i = 0; i < reserve1; i++) addrs1[i] = 100 + 2 * i;
    Buf out1(eng, (size_t)reserve1 * bs);

    // --- compaction 2: immutable A of a secondary index, unsorted memtable ---
    tbc_tree ci_tree{17, TBC_KEY_COMPOSITE_U64, TBC_USAGE_SECONDARY_INDEX, 16, 8, 2000};
    tbo_tree oci;
    REQUIRE(tbo_tree_init(&oci, 17, TBO_KEY_COMPOSITE_U64, TBO_USAGE_SECONDARY_INDEX, 16, 8, 2000, bs) == 0);
    const size_t nm = 1500;
    std::vector<uint8_t> mem(nm * 16);
    for (size_t i = 0; i < nm; i++) {
        uint64_t w[2] = {rnd() % 40 /* ledger */, 1 + i /* timestamp */};
        std::memcpy(&mem[16 * i], w, 16);
    }
    Buf memtable(eng, mem.size());
    memtable.put(mem.data(), mem.size());
    const uint32_t reserve2 = 1 * (1 + 1) * 1 + 16;
    std::vector<uint64_t> addrs2(reserve2);
    for (uint32_t i = 0; i < reserve2; i++) addrs2[i] = 5000 + i;
    Buf out2(eng, (size_t)reserve2 * bs);

    Scheduler sched(eng);
    Compaction c1(id_tree), c2(ci_tree), c3(id_tree);
    int callbacks = 0;

    Context ctx1;
    ctx1.op_min = 32;
    ctx1.a_segments = seg_a;
    ctx1.level_b = 1;
    ctx1.range_b_segments = seg_b;
    ctx1.range_b_empty = false;
    ctx1.drop_tombstones = false;
    ctx1.cluster[0] = 0xC1;
    ctx1.reservation = addrs1;
    ctx1.output_blocks = out1.p;
    ctx1.callback = [&](Compaction &) { callbacks++; };
    c1.start(sched, ctx1);

    // Bar end: TableMemory.sort on the device, then the immutable compaction.
    table_memory_sort(eng, ci_tree, memtable.p, (uint32_t)nm);
    Context ctx2;
    ctx2.op_min = 48;
    ctx2.a_immutable = true;
    ctx2.a_segments = {tbc_segment{memtable.p, (uint32_t)nm, 0}};
    ctx2.level_b = 0;
    ctx2.range_b_empty = true;
    ctx2.drop_tombstones = true;
    ctx2.cluster[0] = 0xC1;
    ctx2.reservation = addrs2;
    ctx2.output_blocks = out2.p;
    ctx2.callback = [&](Compaction &) { callbacks++; };
    c2.start(sched, ctx2);

    // Move-table: disk A, no overlapping B (compaction.zig:296-298, 352-370).
    Context ctx3;
    ctx3.op_min = 32;
    ctx3.a_segments = seg_a;
    ctx3.level_b = 2;
    ctx3.range_b_empty = true;
    std::memset(ctx3.a_table_info, 0xAB, 128);
    ctx3.callback = [&](Compaction &) { callbacks++; };
    c3.start(sched, ctx3);
    REQUIRE(c3.move_table());

    sched.run_to_completion();
    REQUIRE(callbacks == 3);
    REQUIRE(c1.state() == Compaction::State::tables_writing_done);

    // Oracle for compaction 1.
    {
        std::vector<uint8_t> oblocks((size_t)reserve1 * bs), oinfos(128 * reserve1);
        tbo_job j{};
        j.tree = &oid;
        j.segments_a = oseg_a.data();
        j.segment_count_a = (uint32_t)oseg_a.size();
        j.segments_b = oseg_b.data();
        j.segment_count_b = (uint32_t)oseg_b.size();
        j.level_b = 1;
        j.cluster_lo = 0xC1;
        j.snapshot_min = snapshot_min_for_table_output(32);
        j.addresses = addrs1.data();
        j.address_count = reserve1;
        j.out_blocks = oblocks.data();
        j.out_block_capacity = reserve1;
        j.out_table_infos = oinfos.data();
        j.out_table_capacity = reserve1;
        REQUIRE(tbo_compact(&j) == 0);
        const tbc_compaction_result &r = c1.result();
        REQUIRE(r.block_count == j.out_block_count);
        REQUIRE(r.table_count == j.out_table_count);
        std::vector<uint8_t> got((size_t)r.block_count * bs);
        out1.get(got.data(), got.size());
        for (uint32_t i = 0; i < r.block_count; i++) {
            uint32_t size;
            std::memcpy(&size, &oblocks[(size_t)i * bs + 96], 4);
            const size_t img = (size + 4095) / 4096 * 4096;
            REQUIRE(std::memcmp(&got[(size_t)i * bs], &oblocks[(size_t)i * bs], img) == 0);
        }
        auto entries = c1.apply_to_manifest();
        REQUIRE(entries.size() == j.out_table_count);
        for (size_t t = 0; t < entries.size(); t++)
            REQUIRE(std::memcmp(entries[t].table_info, &oinfos[128 * t], 128) == 0);
        c1.transition_to_idle();
        REQUIRE(c1.state() == Compaction::State::idle);
    }
    // Oracle for compaction 2 (sort + immutable dedup with secondary-index cancellation).
    {
        std::vector<uint8_t> sorted = mem;
        REQUIRE(tbo_sort_values(&oci, sorted.data(), (uint32_t)nm) == 0);
        tbo_segment s{sorted.data(), (uint32_t)nm};
        std::vector<uint8_t> oblocks((size_t)reserve2 * bs), oinfos(128 * reserve2);
        tbo_job j{};
        j.tree = &oci;
        j.a_immutable = 1;
        j.segments_a = &s;
        j.segment_count_a = 1;
        j.drop_tombstones = 1;
        j.level_b = 0;
        j.cluster_lo = 0xC1;
        j.snapshot_min = snapshot_min_for_table_output(48);
        j.addresses = addrs2.data();
        j.address_count = reserve2;
        j.out_blocks = oblocks.data();
        j.out_block_capacity = reserve2;
        j.out_table_infos = oinfos.data();
        j.out_table_capacity = reserve2;
        const int rc = tbo_compact(&j);
        REQUIRE(rc == 0 || rc == TBO_ERR_INVARIANT); // random memtable may pair equal keys
        const tbc_compaction_result &r = c2.result();
        REQUIRE(r.block_count == j.out_block_count);
        std::vector<uint8_t> got((size_t)r.block_count * bs);
        out2.get(got.data(), got.size());
        for (uint32_t i = 0; i < r.block_count; i++) {
            uint32_t size;
            std::memcpy(&size, &oblocks[(size_t)i * bs + 96], 4);
            REQUIRE(std::memcmp(&got[(size_t)i * bs], &oblocks[(size_t)i * bs], (size + 4095) / 4096 * 4096) == 0);
        }
    }
    // Move-table: one move entry, no blocks.
    {
        auto entries = c3.apply_to_manifest();
        REQUIRE(entries.size() == 1 && entries[0].operation == ManifestEntry::Operation::move_to_level_b);
        REQUIRE(entries[0].table_info[0] == 0xAB);
    }
    std::printf("compaction_host_test OK\n");
    return 0;
}
