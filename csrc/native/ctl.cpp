// Shared-memory step-boundary agreement (see ctl.h for the protocol and its argument).
#include "ctl.h"

#include <sched.h>

#include <algorithm>
#include <cstring>

namespace tpi {
namespace ctl {
namespace {

inline uint64_t* word(void* base, uint64_t line) {
  return reinterpret_cast<uint64_t*>(static_cast<char*>(base) + line * kLine);
}
inline const uint64_t* word(const void* base, uint64_t line) {
  return reinterpret_cast<const uint64_t*>(static_cast<const char*>(base) + line * kLine);
}

inline uint64_t load(const uint64_t* p) { return __atomic_load_n(p, __ATOMIC_SEQ_CST); }
inline void store(uint64_t* p, uint64_t v) { __atomic_store_n(p, v, __ATOMIC_SEQ_CST); }

// A target is BUSY only for the few loads of a proposal; spin past it.
uint64_t settled(const uint64_t* p) {
  uint64_t v;
  for (int spins = 0; (v = load(p)) == kBusy; ++spins)
    if (spins > 64) sched_yield();
  return v;
}

// min / max ordinal over the ranks other than `self` (-1: all)
void extremes(const void* base, int world, int self, uint64_t* lo, uint64_t* hi) {
  uint64_t mn = ~0ull, mx = 0;
  for (int r = 0; r < world; ++r) {
    if (r == self) continue;
    const uint64_t c = load(word(base, 3 + (uint64_t)r));
    mn = std::min(mn, c);
    mx = std::max(mx, c);
  }
  *lo = mn;
  *hi = mx;
}

}  // namespace

uint64_t bytes(int world) { return kLine * (3 + (uint64_t)std::max(world, 1)); }

void init(void* base, int world) {
  std::memset(base, 0, bytes(world));
  word(base, 0)[1] = (uint64_t)world;
  store(word(base, 0), kMagic);
}

bool valid(const void* base, int world) {
  return load(word(base, 0)) == kMagic && word(base, 0)[1] == (uint64_t)world;
}

void arrive(void* base, int rank, uint64_t ordinal, uint64_t* preempt, uint64_t* periodic) {
  store(word(base, 3 + (uint64_t)rank), ordinal);
  *preempt = settled(word(base, 1));
  *periodic = settled(word(base, 2));
}

// The proposer itself has published its ordinal but not yet passed that boundary, so it
// can be the target; any other rank may already have passed its published ordinal.
static uint64_t choose(const void* base, int world, int self) {
  uint64_t lo, hi;
  extremes(base, world, self, &lo, &hi);
  const uint64_t own = load(word(base, 3 + (uint64_t)self));
  return std::max(own, world > 1 ? hi + 1 : own);
}

uint64_t propose_preempt(void* base, int world, int self) {
  uint64_t* target = word(base, 1);
  uint64_t expected = 0;
  if (!__atomic_compare_exchange_n(target, &expected, kBusy, false, __ATOMIC_SEQ_CST,
                                   __ATOMIC_SEQ_CST))
    return settled(target);  // another rank chose it (or is choosing it)
  const uint64_t t = choose(base, world, self);
  store(target, t);
  return t;
}

uint64_t propose_periodic(void* base, int world, int self) {
  uint64_t* target = word(base, 2);
  uint64_t current = settled(target);
  if (!__atomic_compare_exchange_n(target, &current, kBusy, false, __ATOMIC_SEQ_CST,
                                   __ATOMIC_SEQ_CST))
    return 0;  // raced with another proposer: leave it to that one
  uint64_t lo, hi;
  extremes(base, world, -1, &lo, &hi);
  if (current != 0 && lo <= current) {  // someone has not passed the last one yet
    store(target, current);
    return 0;
  }
  const uint64_t t = choose(base, world, self);
  store(target, t);
  return t;
}

uint64_t ordinal_of(const void* base, int rank) { return load(word(base, 3 + (uint64_t)rank)); }

}  // namespace ctl
}  // namespace tpi
