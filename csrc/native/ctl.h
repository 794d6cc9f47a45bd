// Step-boundary agreement between the ranks of one task on one node (shared memory).
//
// The reference has no notion of a consistent save point: its spot recovery restores whatever
// the 10 s workdir sync last uploaded, and the user script resumes from its own files
// (machine-script.sh.tpl:89,118-124; README.md:88-101).  Here a preempted gang checkpoints
// tensors, and every rank must save the *same* step.  A collective per step (all-reduce of a
// "stop" flag) would put a host<->device sync or a TCP round trip on every step; the ranks of
// a task share a node, so they agree through one cache line per rank instead:
//
//   block   [0]  magic | world            (64 B line)
//           [1]  preempt target ordinal   (0: none, BUSY: being chosen)
//           [2]  periodic target ordinal  (single proposer: rank 0)
//           [3+r] boundary ordinal last reached by rank r
//
// A rank at boundary c stores c into its line and then loads the targets (both seq_cst).  A
// proposer (itself at boundary c, not yet passed) swaps a target to BUSY, then reads every
// other rank's line and publishes max(c, their max + 1).  In the single total order of seq_cst
// operations, a rank whose load saw "no target" stored its ordinal before the proposer read
// it, so the published target is never behind any rank: every rank reaches the target ordinal
// (now or in the future) and saves there, and nobody saves at any other boundary.  Cost per
// step: one store and two loads.
#pragma once

#include <cstdint>

namespace tpi {
namespace ctl {

constexpr uint64_t kMagic = 0x314C5443495054ull;  // "TPICTL1"
constexpr uint64_t kBusy = ~0ull;
constexpr uint64_t kLine = 64;

uint64_t bytes(int world);
void init(void* base, int world);
// Returns false if the block is not an initialised control block for `world` ranks.
bool valid(const void* base, int world);
// Publish that `rank` reached boundary `ordinal`; returns the current targets.
void arrive(void* base, int rank, uint64_t ordinal, uint64_t* preempt, uint64_t* periodic);
// Choose the preempt target (once per block; `self` = the proposing rank, which has arrived
// at its current boundary but not passed it): max(own ordinal, other ranks' max + 1), or the
// target another rank chose.
uint64_t propose_preempt(void* base, int world, int self);
// Choose a periodic target if every rank has passed the previous one; 0 if not.
uint64_t propose_periodic(void* base, int world, int self);
uint64_t ordinal_of(const void* base, int rank);

}  // namespace ctl
}  // namespace tpi
