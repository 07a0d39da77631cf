"""The drop-in's RLO_TRACE_DIR log on the CPU under AddressSanitizer.

Round 5's 8-rank drop-in `iar` run under RLO_TRACE_DIR died with SIGSEGV in a rank process.  Cause:
RLO_progress_engine_cleanup wrote the trace by iterating the engine's record vector while the pump thread -- which
steps in for an engine whose application thread has not made progress for 200 us, as it had not while writing the
file -- still appended 'C' records (the kernel consuming the rank's last commands, rootless_ops.cpp pump()).  A
push_back that reallocated left the writer iterating freed memory.

The driver below runs the code the library runs (csrc/rlo_trace.hpp, TraceLog) with one thread appending as the pump
does while another writes, under ASan; the control runs the round-5 writer's pattern (iterate the live vector, the
appender under its own lock) and must be caught as a heap-use-after-free -- the test shows the mechanism, then that
the fix removes it.  No GPU.
"""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "rootless-coll-mpi-ops_amd", "csrc")

DRIVER = r"""
#include <atomic>
#include <cstdio>
#include <cstring>
#include <thread>
#include "rlo_trace.hpp"

// the round-5 writer's pattern: the appender locks, the writer iterates the live vector without the lock
struct Unsafe {
    std::mutex mu;
    std::vector<rlo::TraceRec> tr;
    void add(const rlo::TraceRec& r) { std::lock_guard<std::mutex> lk(mu); tr.push_back(r); }
    long write(const char* path) {
        FILE* f = std::fopen(path, "w");
        long n = 0;
        for (const rlo::TraceRec& r : tr) {
            std::fprintf(f, "%lld %c %u %d %d %d %u\n", (long long)r.t, r.what, r.kind, r.origin, r.id, r.from, r.aux);
            n++;
        }
        std::fclose(f);
        return n;
    }
};

template <class L>
long run(L& log, const char* path, long pre, long (*wr)(L&, const char*)) {
    for (long i = 0; i < pre; i++) log.add(rlo::TraceRec{i, 'S', 1u, 0, (int)i, 0, 0u});
    std::atomic<bool> stop{false};
    long extra = 0;
    std::thread pump([&] {  // the pump thread: 'C' records while the kernel consumes commands
        while (!stop.load(std::memory_order_relaxed)) { log.add(rlo::TraceRec{extra, 'C', 0u, -1, (int)extra, -1, 0u}); extra++; }
    });
    const long n = wr(log, path);
    stop = true;
    pump.join();
    return n + extra * 0;
}

long wr_fixed(rlo::TraceLog& l, const char* p) { return l.write(p, "# test\n"); }
long wr_unsafe(Unsafe& l, const char* p) { return l.write(p); }

int main(int argc, char** argv) {
    const long pre = 1L << 18;  // the vector's capacity is 2^18 when the writer starts: the next push_back reallocates
    if (argc > 2 && std::strcmp(argv[1], "unsafe") == 0) {
        Unsafe u;
        std::printf("wrote %ld\n", run(u, argv[2], pre, wr_unsafe));
        return 0;
    }
    rlo::TraceLog t;
    const long n = run(t, argv[2], pre, wr_fixed);
    // the records added while writing stay in the log for a later write, none lost
    const size_t left = t.size();
    const long m = t.write(argv[2], nullptr);
    std::printf("wrote %ld then %ld (left %zu)\n", n, m, left);
    return (n >= pre && m == (long)left) ? 0 : 3;
}
"""


def _build(tmp_path):
    if not shutil.which("g++"):
        pytest.skip("g++ not available")
    src = tmp_path / "trace_drv.cpp"
    src.write_text(DRIVER)
    exe = tmp_path / "trace_drv"
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address", "-fno-omit-frame-pointer", "-pthread",
                    "-I", CSRC, str(src), "-o", str(exe)], check=True)
    return exe


def _run(exe, mode, out):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0")
    env.pop("LD_PRELOAD", None)
    return subprocess.run([str(exe), mode, str(out)], capture_output=True, text=True, timeout=120, env=env)


def test_trace_write_while_pump_appends_is_clean_under_asan(tmp_path):
    exe = _build(tmp_path)
    for i in range(3):
        r = _run(exe, "fixed", tmp_path / ("fixed%d.txt" % i))
        assert r.returncode == 0 and "AddressSanitizer" not in r.stderr, r.stdout + r.stderr[-3000:]


def test_round5_trace_writer_pattern_is_a_use_after_free(tmp_path):
    """the control: the pattern the library had is caught by ASan (heap-use-after-free in the writer)"""
    exe = _build(tmp_path)
    caught = False
    for i in range(5):
        r = _run(exe, "unsafe", tmp_path / ("unsafe%d.txt" % i))
        if "heap-use-after-free" in r.stderr:
            caught = True
            break
    assert caught, "the round-5 writer pattern was expected to read freed memory"
