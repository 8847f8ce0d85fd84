// compaction.hpp — C++ host mirror of TigerBeetle's CompactionType over the
// tbc C ABI (include/tbc.h). Header-only, C++17.
//
// The reference's host side is Zig (src/lsm/compaction.zig:56-985); Zig is
// not available in this image, so this restates the same surface and state
// machine in C++ for hosts that link libtbc.so directly:
//
//   Compaction::init / deinit / reset           compaction.zig:171-263
//   Compaction::start(Context)                  compaction.zig:280-404
//     (move-table short-circuit, reservation, drop_tombstones)
//   Scheduler::tick()  — the grid.on_next_tick loop: submits every started
//     compaction of the half-bar as ONE batch, then polls it; completed
//     compactions reach state tables_writing_done and their callback fires
//     (done_on_next_tick, compaction.zig:921-937)
//   Compaction::apply_to_manifest               compaction.zig:939-973
//     (returns the manifest entries: inserts of the output TableInfos, or the
//     move of table A)
//   Compaction::transition_to_idle              compaction.zig:265-275
//   TableMemory::sort                           table_memory.zig:140-154
//
// Like the reference (which asserts and panics on these paths), contract
// violations throw std::logic_error and engine failures std::runtime_error.
#pragma once

#include <cstdint>
#include <cstring>
#include <functional>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/tbc.h"

namespace tbc_host {

constexpr uint64_t lsm_batch_multiple = 32; // config.zig:142

// compaction.zig:981-985
inline uint64_t snapshot_min_for_table_output(uint64_t op_min) {
    if (op_min == 0 || op_min % (lsm_batch_multiple / 2) != 0) throw std::logic_error("op_min not a half-bar start");
    return op_min + lsm_batch_multiple / 2;
}
// compaction.zig:977-979
inline uint64_t snapshot_max_for_table_input(uint64_t op_min) { return snapshot_min_for_table_output(op_min) - 1; }

inline void check(tbc_status s, const char *what) {
    if (s != TBC_OK) throw std::runtime_error(std::string(what) + " failed: status " + std::to_string((int)s));
}

class Engine {
  public:
    explicit Engine(int device, uint32_t block_size = 1u << 20, uint32_t flags = 0) {
        tbc_config c{};
        c.device = device;
        c.block_size = block_size;
        c.flags = flags;
        check(tbc_engine_init(&c, &e_), "tbc_engine_init");
        block_size_ = block_size;
    }
    ~Engine() { tbc_engine_deinit(e_); }
    Engine(const Engine &) = delete;
    Engine &operator=(const Engine &) = delete;
    tbc_engine *handle() const { return e_; }
    uint32_t block_size() const { return block_size_; }

  private:
    tbc_engine *e_ = nullptr;
    uint32_t block_size_ = 0;
};

// A manifest entry queued by a compaction (compaction.zig:120-133).
struct ManifestEntry {
    enum class Operation { insert_to_level_b, move_to_level_b } operation;
    uint8_t table_info[128]; // schema.ManifestNode.TableInfo (schema.zig:489-509)
};

class Compaction;
using Callback = std::function<void(Compaction &)>;

// compaction.zig:84-99
struct Context {
    uint64_t op_min = 0;
    // table_info_a: either the immutable table (sorted values in device
    // memory) or a disk table (its data blocks, device pointers to values).
    bool a_immutable = false;
    std::vector<tbc_segment> a_segments;
    uint8_t a_table_info[128] = {}; // disk A's TableInfo (for the move-table case)
    uint8_t level_b = 0;
    // range_b: the data blocks of the overlapping level-B tables, ascending.
    std::vector<tbc_segment> range_b_segments;
    bool range_b_empty = true;
    // Manifest.compaction_must_drop_tombstones(level_b, range_b) (manifest.zig:547-574)
    bool drop_tombstones = false;
    uint64_t cluster[2] = {0, 0};
    // grid.reserve(...) then the acquire order of that reservation (free_set.zig:240-345)
    std::vector<uint64_t> reservation;
    void *output_blocks = nullptr; // device, reservation.size() * block_size
    Callback callback;
};

class Scheduler;

class Compaction {
  public:
    enum class State { idle, compacting, tables_writing_done, applied_to_manifest };

    explicit Compaction(const tbc_tree &tree) : tree_(tree) {}

    // compaction.zig:228-263
    void reset() {
        state_ = State::idle;
        move_table_ = false;
        entries_.clear();
        result_ = {};
    }

    State state() const { return state_; }
    bool move_table() const { return move_table_; }
    const Context &context() const { return ctx_; }
    const tbc_compaction_result &result() const { return result_; }
    const std::vector<ManifestEntry> &manifest_entries() const { return entries_; }

    // compaction.zig:280-404
    void start(Scheduler &scheduler, Context ctx);

    // compaction.zig:939-973: the manifest updates, in order. Input tables
    // become invisible at snapshot_max_for_table_input(op_min) (the caller's
    // Manifest.update_table); output tables are inserted.
    std::vector<ManifestEntry> apply_to_manifest() {
        if (state_ != State::tables_writing_done) throw std::logic_error("apply_to_manifest: not done");
        state_ = State::applied_to_manifest;
        return entries_;
    }

    // compaction.zig:265-275
    void transition_to_idle() {
        if (state_ != State::applied_to_manifest) throw std::logic_error("transition_to_idle: not applied");
        state_ = State::idle;
    }

  private:
    friend class Scheduler;
    tbc_tree tree_;
    State state_ = State::idle;
    bool move_table_ = false;
    Context ctx_;
    std::vector<ManifestEntry> entries_;
    tbc_compaction_result result_{};
    std::vector<uint8_t> infos_;
};

// The event-loop side: gathers the compactions started in this half-bar
// (Forest.compact -> Groove.compact -> Tree.compact fan-out), submits them as
// one GPU batch and polls it (never blocks unless asked to).
class Scheduler {
  public:
    explicit Scheduler(Engine &engine) : engine_(engine) {}
    ~Scheduler() {
        if (batch_) tbc_batch_release(batch_);
    }

    void enqueue(Compaction &c) { pending_.push_back(&c); }

    // One grid.on_next_tick: returns true when nothing is outstanding.
    bool tick() {
        if (!batch_ && !pending_.empty()) submit();
        if (!batch_) return finish_moves();
        const tbc_status s = tbc_batch_poll(batch_);
        if (s == TBC_PENDING) return false;
        check(s, "tbc_batch_poll");
        complete();
        return true;
    }

    void run_to_completion() {
        while (!tick()) {
            if (batch_) check(tbc_batch_wait(batch_), "tbc_batch_wait");
        }
    }

  private:
    bool finish_moves() {
        std::vector<Compaction *> moves;
        moves.swap(moves_);
        for (Compaction *c : moves) {
            c->state_ = Compaction::State::tables_writing_done;
            if (c->ctx_.callback) c->ctx_.callback(*c);
        }
        return moves_.empty() && pending_.empty();
    }

    void submit() {
        std::vector<tbc_compaction> jobs;
        for (Compaction *c : pending_) {
            if (c->move_table_) {
                moves_.push_back(c);
                continue;
            }
            tbc_compaction j{};
            j.tree = c->tree_;
            j.a_immutable = c->ctx_.a_immutable;
            j.drop_tombstones = c->ctx_.drop_tombstones;
            j.level_b = c->ctx_.level_b;
            j.segments_a = c->ctx_.a_segments.data();
            j.segment_count_a = (uint32_t)c->ctx_.a_segments.size();
            j.segments_b = c->ctx_.range_b_segments.data();
            j.segment_count_b = (uint32_t)c->ctx_.range_b_segments.size();
            j.cluster[0] = c->ctx_.cluster[0];
            j.cluster[1] = c->ctx_.cluster[1];
            j.snapshot_min = snapshot_min_for_table_output(c->ctx_.op_min);
            j.addresses = c->ctx_.reservation.data();
            j.address_count = (uint32_t)c->ctx_.reservation.size();
            j.output_blocks = c->ctx_.output_blocks;
            jobs.push_back(j);
            submitted_.push_back(c);
        }
        pending_.clear();
        if (!jobs.empty()) check(tbc_compaction_submit(engine_.handle(), jobs.data(), (uint32_t)jobs.size(), &batch_),
                                 "tbc_compaction_submit");
    }

    void complete() {
        for (size_t i = 0; i < submitted_.size(); i++) {
            Compaction *c = submitted_[i];
            tbc_compaction_result r{};
            check(tbc_batch_result(batch_, (uint32_t)i, &r, nullptr, 0), "tbc_batch_result");
            c->infos_.assign((size_t)r.table_count * 128, 0);
            check(tbc_batch_result(batch_, (uint32_t)i, &r, c->infos_.data(), r.table_count), "tbc_batch_result");
            c->result_ = r;
            for (uint32_t t = 0; t < r.table_count; t++) {
                ManifestEntry m{};
                m.operation = ManifestEntry::Operation::insert_to_level_b;
                std::memcpy(m.table_info, c->infos_.data() + 128 * t, 128);
                c->entries_.push_back(m);
            }
        }
        tbc_batch_release(batch_);
        batch_ = nullptr;
        std::vector<Compaction *> done;
        done.swap(submitted_);
        for (Compaction *c : done) {
            c->state_ = Compaction::State::tables_writing_done;
            if (c->ctx_.callback) c->ctx_.callback(*c);
        }
        finish_moves();
    }

    Engine &engine_;
    tbc_batch *batch_ = nullptr;
    std::vector<Compaction *> pending_, submitted_, moves_;
};

inline void Compaction::start(Scheduler &scheduler, Context ctx) {
    if (state_ != State::idle) throw std::logic_error("Compaction.start: not idle");
    ctx_ = std::move(ctx);
    entries_.clear();
    // compaction.zig:296-298: a disk table with no overlapping level-B tables moves.
    move_table_ = !ctx_.a_immutable && ctx_.range_b_empty;
    if (!move_table_ && !ctx_.drop_tombstones && ctx_.level_b + 1 >= 7)
        throw std::logic_error("the last level must drop tombstones"); // compaction.zig:326
    state_ = State::compacting;
    if (move_table_) {
        ManifestEntry m{};
        m.operation = ManifestEntry::Operation::move_to_level_b;
        std::memcpy(m.table_info, ctx_.a_table_info, 128);
        entries_.push_back(m);
    }
    scheduler.enqueue(*this);
}

// TableMemory.sort (table_memory.zig:140-154) on device-resident values.
inline void table_memory_sort(Engine &engine, const tbc_tree &tree, void *values, uint32_t count) {
    check(tbc_sort_values(engine.handle(), &tree, values, count), "tbc_sort_values");
}

} // namespace tbc_host
