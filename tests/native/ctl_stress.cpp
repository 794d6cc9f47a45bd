// Stress of the shared-memory step-boundary agreement (csrc/native/ctl.{h,cpp}), built by
// tests/test_sanitizers.py with -fsanitize=thread: 8 "ranks" (threads) step through
// boundaries with random skew, rank 0 proposes periodic checkpoints on its own clock, and a
// preemption request reaches each rank at a different boundary (a signal's delivery skew);
// every rank that sees it proposes, as checkpoint/agreement.py does.
//
// Checked, over many trials: every rank saves the preemption at the same ordinal; every
// periodic target at or below it is saved by every rank and at no other ordinal; no rank is
// ever past a target it is told about (the protocol's invariant); and ThreadSanitizer sees no
// data race in the protocol's accesses.
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <random>
#include <set>
#include <thread>
#include <vector>

#include "../../csrc/native/ctl.h"

namespace {

struct RankLog {
  uint64_t preempt_at = 0;
  std::vector<uint64_t> periodic;
  int violations = 0;
};

void spin(std::mt19937& rng, unsigned max_iters) {
  volatile unsigned sink = 0;
  const unsigned n = rng() % (max_iters + 1);
  for (unsigned i = 0; i < n; ++i) sink = sink + i;
  if (rng() % 16 == 0) sched_yield();
}

bool trial(int world, unsigned seed) {
  std::vector<uint64_t> block_storage(tpi::ctl::bytes(world) / 8 + 8);
  void* block = block_storage.data();
  tpi::ctl::init(block, world);
  std::atomic<bool> requested{false};
  std::vector<RankLog> logs(world);
  std::vector<std::thread> threads;
  for (int r = 0; r < world; ++r) {
    threads.emplace_back([&, r] {
      std::mt19937 rng(seed * 131 + (unsigned)r);
      RankLog& log = logs[r];
      const int skew = (int)(rng() % 4);  // boundaries before this rank "sees the signal"
      int seen_for = -1;
      for (uint64_t ordinal = 1; ordinal < 100000; ++ordinal) {
        spin(rng, 2000);
        bool preempt = false;
        if (requested.load(std::memory_order_relaxed)) {
          if (seen_for < 0) seen_for = 0;
          preempt = seen_for++ >= skew;
        }
        const bool due = r == 0 && ordinal % (3 + rng() % 5) == 0;
        uint64_t pre = 0, per = 0;
        tpi::ctl::arrive(block, r, ordinal, &pre, &per);
        if (preempt && !pre) pre = tpi::ctl::propose_preempt(block, world, r);
        if (due && r == 0) {
          const uint64_t proposed = tpi::ctl::propose_periodic(block, world, r);
          if (proposed) per = proposed;
        }
        if (pre && ordinal > pre) ++log.violations;  // past a target: a missed save
        if (per && ordinal == per) log.periodic.push_back(ordinal);
        if (pre && ordinal >= pre) {
          log.preempt_at = ordinal;
          return;
        }
        if (r == world - 1 && ordinal == 40 + seed % 60)
          requested.store(true, std::memory_order_relaxed);
      }
    });
  }
  for (auto& t : threads) t.join();
  bool ok = true;
  const uint64_t p = logs[0].preempt_at;
  std::set<uint64_t> expect(logs[0].periodic.begin(), logs[0].periodic.end());
  for (int r = 0; r < world; ++r) {
    if (logs[r].preempt_at != p || p == 0) {
      fprintf(stderr, "trial %u: rank %d saved the preemption at %llu, rank 0 at %llu\n", seed,
              r, (unsigned long long)logs[r].preempt_at, (unsigned long long)p);
      ok = false;
    }
    if (logs[r].violations) {
      fprintf(stderr, "trial %u: rank %d passed a target %d time(s)\n", seed, r,
              logs[r].violations);
      ok = false;
    }
    std::set<uint64_t> mine(logs[r].periodic.begin(), logs[r].periodic.end());
    if (mine != expect) {
      fprintf(stderr, "trial %u: rank %d periodic saves differ from rank 0's\n", seed, r);
      ok = false;
    }
  }
  return ok;
}

}  // namespace

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 200;
  const int world = argc > 2 ? atoi(argv[2]) : 8;
  int bad = 0;
  for (int t = 0; t < trials; ++t) bad += !trial(world, (unsigned)t + 1);
  if (bad) {
    fprintf(stderr, "%d of %d trials failed\n", bad, trials);
    return 1;
  }
  printf("ctl stress ok: %d trials x %d ranks\n", trials, world);
  return 0;
}
