// rlo_trace.hpp -- the drop-in's RLO_TRACE_DIR record log (diagnostics), shared by the application thread and the
// pump thread of a rank process (rootless_ops.cpp), header-only so tests/test_host_trace.py can drive the same code
// on the CPU under AddressSanitizer.
//
// Every command posted, every event taken off the pickup ring and handled, and every advance of the kernel's command
// head, with the host clock (CLOCK_MONOTONIC: one clock for every rank process of the node), written to
// dir/trace_rank<R>_e<id>.txt at cleanup; tools/dropin_legs.py splits a bcast's and a host-judged proposal's time
// into legs from them.
#pragma once
#include <cstdint>
#include <cstdio>
#include <mutex>
#include <vector>

namespace rlo {

struct TraceRec {
    int64_t t;
    char what;  // 'P' command posted, 'S' event seen (pump), 'H' event handled (app thread), 'C' commands consumed
    uint32_t kind;
    int32_t origin, id, from;
    uint32_t aux;
};

class TraceLog {
  public:
    static constexpr size_t kMaxRecs = size_t(1) << 22;

    void add(const TraceRec& r) {
        std::lock_guard<std::mutex> lk(mu_);
        if (recs_.size() < kMaxRecs) recs_.push_back(r);
    }

    // Takes the records out under the lock and writes the copy.  Iterating the live vector while the other thread
    // appended was the round-5 8-rank drop-in SIGSEGV: cleanup wrote the trace while the pump thread
    // -- which steps in for an engine whose application thread has not progressed for 200 us, as it had not while
    // fprintf-ing ~10^5 lines -- still appended 'C' records as the kernel consumed the rank's last commands; a
    // push_back that reallocated left the writer iterating freed memory.  Records added after the take are kept for
    // a later write.  Returns the number of records written, -1 if the file cannot be opened.
    long write(const char* path, const char* header) {
        std::vector<TraceRec> out;
        {
            std::lock_guard<std::mutex> lk(mu_);
            out.swap(recs_);
        }
        FILE* f = std::fopen(path, "w");
        if (!f) return -1;
        if (header) std::fputs(header, f);
        for (const TraceRec& r : out)
            std::fprintf(f, "%lld %c %u %d %d %d %u\n", (long long)r.t, r.what, r.kind, r.origin, r.id, r.from, r.aux);
        std::fclose(f);
        return (long)out.size();
    }

    size_t size() {
        std::lock_guard<std::mutex> lk(mu_);
        return recs_.size();
    }

  private:
    std::mutex mu_;
    std::vector<TraceRec> recs_;
};

}  // namespace rlo
