// tpi-supervisor: the class of the on-node runtime (one process per task).  The member
// functions live in supervisor.cpp (event loop, journal, state, reaping, settling),
// supervisor_ranks.cpp (spawning ranks, standbys and preloaded successors, their output and
// notify pipes) and supervisor_control.cpp (signals, control socket, deadline, limits, the
// workdir stager, exit tracing, requeue); see supervisor.cpp for what the runtime does.
#pragma once
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <poll.h>
#include <sched.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/prctl.h>
#include <sys/signalfd.h>
#include <sys/socket.h>
#include <sys/un.h>
#include <dirent.h>
#include <ftw.h>
#include <sys/stat.h>
#include <sys/time.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <string>
#include <vector>

#include "json.h"

using tpi::json::quote;
using tpi::json::Value;

#include "common.h"
#include "container_sync.h"
#include "memory_guard.h"

namespace tpi_sup {

class Supervisor {
 public:
  explicit Supervisor(Spec spec);
  int run();

 private:
  Spec s_;
  std::vector<Rank> ranks_;
  std::vector<Rank> detached_;  // released incarnations still exiting
  std::vector<Rank> standby_;   // per rank index: warm successor waiting for "go" (pid > 0)
  bool machine_logs_ = false;   // TPI_MACHINE_LOGS set in the task environment (tpl:109)
  int sfd_ = -1;
  int ctl_fd_ = -1;
  double started_ = 0, respawn_at_ = 0;
  bool stop_ = false, timed_out_ = false, dirty_ = true;
  bool resources_released_ = false;  // leases gone; released processes may still be exiting
  bool requeued_ = false;            // the queue waiter was started (it owns state.json)
  bool settled_ = false;  // final sync + final state written; only reaping released processes
  int total_restarts_ = 0;
  pid_t stager_pid_ = -1;
  bool staged_ = false;
  bool requeue_ = false;  // reclaimed (spot): ranks go down, the task goes back to the queue
  double next_disk_check_ = 0;
  MemoryGuard memory_{s_, [this](const std::string& c, const std::vector<std::string>& d) {
    event(c, d);
  }};

  // ---- machine-type limits: the workdir's disk use (memory: memory_guard.h) ----------------
  static thread_local uint64_t du_total_;
  static int du_visit(const char*, const struct stat* st, int type, struct FTW*);
  uint64_t workdir_bytes();
  void check_limits(double t);
  bool disk_exceeded_ = false;

  // ---- off-node container mirror ------------------------------------------------------------
  ContainerSync sync_{s_, [this](const std::string& c, const std::vector<std::string>& d) {
    event(c, d);
  }};

  // ---- workdir stager ----------------------------------------------------------------------
  int stager_fd_ = -1;            // the stager's stdout ("staged ..." line), while staging
  double stager_deadline_ = 0;
  std::string stager_out_;

  void stage();
  void read_stager();
  void stage_failed(const std::string& why);
  bool start_stager();
  void stop_stager();
  void stager_exited(int st);
  void event(const std::string& code, const std::vector<std::string>& desc);
  static const char* state_name(Rank::State st);
  int running() const;
  void write_state(const char* phase = nullptr);
  std::string state_json(const char* phase = nullptr);
  void write_status(Rank& r, const std::string& result, const std::string& code,
                    const std::string& status);
  std::vector<std::string> rank_env(const Rank& r);
  void spawn(Rank& r, bool standby = false, bool preload = false);
  void spawn_standby(Rank& r, bool preload = false);

  // Preloaded successors (spec "preload_argv", TPI_PRELOAD=1): every running Python rank keeps
  // a process that has imported PyTorch and this package and waits on its activation pipe
  // (runtime/preload.py); the respawn activates it like a warm standby, so a cold successor
  // skips the interpreter start and the imports (~1.8 s of its 1.9 s).  Started kPreloadDelay
  // after the rank (not competing with its own start-up), at most two per incarnation.  A hot
  // standby (which the script itself parks, GPU initialised) takes precedence.
  static constexpr double kPreloadDelay = 2.0;
  void keep_preloaded();

  // Hot standby (spec "standby_hot"): every running, standby-capable rank keeps a successor
  // that has already imported its framework and initialised the GPU, so on preemption it is
  // activated the moment the old rank releases -- with a streamed spill, while the spill is
  // still running.  At most two per incarnation (a standby that keeps dying is not retried).
  //
  // A successor that is restoring does not get its own standby yet: starting one (interpreter,
  // framework import, GPU context, engine, spill mapping) competes with the restore for CPU
  // and GPU.  It comes after the successor reports "restored", or kStandbyHold seconds.
  static constexpr double kStandbyHold = 10.0;
  void keep_hot_standbys();
  void discard_standby(int index, const char* why);
  bool activate_standby(Rank& r);
  void join_cgroup(int index, pid_t pid);
  static std::vector<pid_t> device_holders(pid_t pgid, const std::string& device);

  // Evidence for warming a parked preloaded successor's GPU (spec "preload_gpu_auto"): the
  // successor runs the script in-process, so a context it creates before the script starts is
  // one the script would otherwise create itself -- unless the script forks GPU-using workers
  // before it touches the GPU (they cannot use a context inherited over fork()).  The running
  // incarnation tells which kind the script is: one process of the rank holding the GPU device
  // in two samples -> "warm" (the successor initialises the GPU now: ~0.13 s off a cold
  // recovery, profiles/round5/r5ai); two or more -> the successor stays plain; none yet -> ask
  // again later.
  double next_evidence_ = 0;
  void check_preload_evidence(double t);
  void emit_line(Rank& r, const std::string& line);
  void pump(Rank& r);
  bool notified(Rank& r);
  void release_predecessors(int index, const char* why);
  void handoff_released();
  void close_log(Rank& r);
  void terminate(Rank& r, TermReason why);

  // Exit trace: a released or discarded process should be gone within ~1-2 s (its kernel
  // teardown: unpinning the host region, freeing HBM and the GPU context).  Where one spends
  // longer shows in /proc: its scheduler state (D = uninterruptible, inside the driver or the
  // mm teardown; Z = exited, not yet reaped) and the kernel function it sleeps in (wchan),
  // journalled whenever they change, with its resident set, every kTraceInterval seconds.
  static constexpr double kTraceInterval = 0.1;
  static constexpr int kTraceMax = 64;  // events per process

  static std::string thread_waits(pid_t pid);
  void trace_exits(double t);
  void check_grace(double t);
  void check_deadline(double t);
  void check_respawn(double t);
  void next_master_port();
  void pick_master_port(int from);
  void handle_signals();
  void request_stop(const std::string& source);
  bool request_preempt(const std::string& source, int rank = -1);
  bool request_requeue(const std::string& source);
  void open_control();
  void close_control();
  void handle_control();
  void reap();
  void on_exit(Rank& r, int st);
  bool ranks_settled();
  bool all_finished() { return ranks_settled() && detached_.empty(); }

  void release_resources();
  void settle();
  void drain_rank_logs();
  int finish();
  bool spawn_requeue();
};

}  // namespace tpi_sup
