// tpi-supervisor: the on-node runtime of a task (one process per task).
//
// It replaces the reference's per-VM machinery -- the cloud scaling group that keeps
// `parallelism` machines alive and the systemd unit + bash sync loops of
// task/common/machine/machine-script.sh.tpl -- with one event loop on this node:
//
//  * spawns `parallelism` rank processes (own process group, cwd = task workdir, env from
//    the spec plus RANK/WORLD_SIZE/LOCAL_RANK/MASTER_* and HIP_VISIBLE_DEVICES for the GPUs
//    placed for that rank); PR_SET_PDEATHSIG ties them to the supervisor;
//  * streams every stdout/stderr line straight into reports/task-<machine uuid> as
//    "YYYY-MM-DDTHH:MM:SSZ line" the moment it arrives (the reference polls journald every
//    5 s, tpl:108-116; this is the first-log-latency floor);
//  * writes reports/status-<uuid> = {"result","code","status"} when a rank exits on its own
//    (systemd ExecStop semantics, tpl:51) and nothing when it was preempted or stopped;
//  * enforces the absolute deadline (RuntimeMaxSec, tpl:36-41): SIGTERM, grace, SIGKILL,
//    status result "timeout";
//  * preemption: SIGUSR1 to the supervisor, or a rank dying of SIGTERM / exiting 143 (the
//    code the checkpoint handler uses after spilling to host DRAM), respawns the rank(s)
//    with a new machine identity -- gang-wide when ranks are coupled by RCCL -- like the
//    scaling group replacing a reclaimed spot VM (tpl:89, resource_auto_scaling_group.go);
//  * early hand-off: a rank that has spilled its checkpoint writes "released" to TPI_NOTIFY_FD;
//    its successor is spawned at once while the old process is still tearing down its
//    address space (unpinning a 100 GB host region takes ~1.4 s), and the old one is reaped
//    in the background;
//  * warm standby (spec "standby", opt-in): when a rank that announced "standby" is preempted, its
//    successor is spawned
//    at once with TPI_STANDBY=1 and imports/maps what it can while the old rank is still
//    spilling; it blocks in preemption.standby() until "go" arrives on TPI_STANDBY_FD, written
//    when the old rank has released (or exited as preempted);
//  * SIGTERM/SIGINT/SIGHUP = stop (`leo stop`, scale to 0): ranks terminated, no status;
//  * control socket supervisor/control.sock (AF_UNIX, mode 0600; SURVEY.md §2.10 "local
//    supervisor API"): one request line, one JSON reply line -- `ping`, `state` (live rank
//    table, fresher than state.json), `preempt` (= SIGUSR1), `preempt <rank>` (one rank;
//    the gang follows when `gang` is set), `stop` (= SIGTERM);
//  * exits when no rank is left to run ("no waste" auto-cleanup, tpl:10-15), removing its
//    GPU lease files.
//
// State for readers: supervisor/state.json (atomically replaced) and an append-only
// supervisor/events.jsonl journal.
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

namespace {

class Supervisor {
 public:
  explicit Supervisor(Spec spec) : s_(std::move(spec)) {
    ranks_.resize(s_.parallelism);
    standby_.resize(s_.parallelism);
    for (auto& kv : s_.env)
      if (kv.first == "TPI_MACHINE_LOGS" && !kv.second.empty()) machine_logs_ = true;
    for (int i = 0; i < s_.parallelism; ++i) {
      ranks_[i].index = i;
      ranks_[i].gpus = s_.rank_gpus[i];
      ranks_[i].restarts = s_.restart_base;
    }
    total_restarts_ = s_.restart_base;
  }

  int run() {
    sigset_t mask;
    sigemptyset(&mask);
    for (int sig : {SIGCHLD, SIGTERM, SIGINT, SIGHUP, SIGUSR1, SIGUSR2}) sigaddset(&mask, sig);
    sigprocmask(SIG_BLOCK, &mask, nullptr);
    sfd_ = signalfd(-1, &mask, SFD_CLOEXEC | SFD_NONBLOCK);
    signal(SIGPIPE, SIG_IGN);
    open_control();
    unlink(s_.requeue_path.c_str());  // a reclaimed incarnation's marker
    started_ = now();
    memory_.start();
    event("supervisor-start", {"pid " + std::to_string(getpid()),
                               "parallelism " + std::to_string(s_.parallelism)});
    if (s_.deadline > 0 && now() >= s_.deadline) {
      // Past the deadline before running (tpl:38-41): nothing may run any more.
      for (auto& r : ranks_) {
        r.uuid = uuid4();
        write_status(r, "timeout", "", "killed");
        r.state = Rank::DONE;
      }
      event("deadline", {"deadline passed before start"});
      return finish();
    }
    if (!s_.stager_argv.empty()) {
      // The reference restores the workdir before the task service starts (tpl:89).  Here the
      // stager loads it while the ranks start (their imports overlap the H2D), and attach()
      // blocks until the manifest lands; "before_ranks" keeps the strict order.
      if (s_.stage_before_ranks) {
        write_state("staging");
        signal_ready();
        stage();
      } else {
        start_stager();
      }
    }
    for (auto& r : ranks_)
      if (r.state == Rank::PENDING) spawn(r);
    write_state();
    signal_ready();
    double last_state = now();
    while (true) {
      double t = now();
      check_deadline(t);
      check_grace(t);
      check_respawn(t);
      check_limits(t);
      sync_.check(t);
      trace_exits(t);
      // Every rank is down (exited, or released after its save): the GPUs, cores and memory
      // go back to the node now, not when the last released process has been reaped -- its
      // kernel teardown (unpinning a 100 GB host region, freeing HBM) can take seconds, and a
      // queued task or an on-demand reclaim would wait for it (tpl:10-15: the group scales to
      // 0 right after the task's exit).
      if (!resources_released_ && ranks_settled()) release_resources();
      // ... and the task is over for its users at the same moment: final sync, final state,
      // control socket closed.  Released processes still tearing down (a 100 GB pinned region
      // can take 10-18 s to unmap after a hot hand-off) are traced and reaped by this process
      // behind that, on no user-visible path (tpl:10-15,51: status, then scale to 0).
      if (!settled_ && resources_released_) settle();
      if (all_finished()) break;
      double timeout = 2.0;
      if (s_.deadline > 0 && !timed_out_) timeout = std::min(timeout, s_.deadline - t);
      for (auto* list : {&ranks_, &detached_})
        for (auto& r : *list)
          if (r.pid > 0 && r.term_at > 0 && !r.killed)
            timeout = std::min(timeout, r.term_at + s_.grace - t);
      if (s_.exit_trace)
        for (auto& d : detached_)
          if (d.pid > 0 && (d.exit_requested_at > 0 || d.killed))
            timeout = std::min(timeout, kTraceInterval);
      if (respawn_at_ > 0) timeout = std::min(timeout, respawn_at_ - t);
      if (s_.rank_memory_kb) timeout = std::min(timeout, memory_.next_check() - t);
      if (!s_.preload_argv.empty())  // the next preloaded successor due
        for (auto& r : ranks_)
          if (r.state == Rank::RUNNING && r.pid > 0 && r.term_at == 0 &&
              standby_[r.index].pid <= 0 && r.hot_spawns < 2)
            timeout = std::min(timeout, std::max(r.hold_until, r.started + kPreloadDelay) - t);
      if (s_.preload_gpu_auto)
        for (auto& r : ranks_)
          if (standby_[r.index].pid > 0 && standby_[r.index].preloaded &&
              standby_[r.index].preload_gpu == 0)
            timeout = std::min(timeout, next_evidence_ - t);
      if (s_.disk_limit_bytes) timeout = std::min(timeout, next_disk_check_ - t);
      timeout = sync_.timeout(t, timeout);
      if (stager_fd_ >= 0) timeout = std::min(timeout, stager_deadline_ - t);
      timeout = std::max(timeout, 0.0);
      std::vector<struct pollfd> pfds;
      pfds.push_back({sfd_, POLLIN, 0});
      std::vector<std::pair<Rank*, bool>> owners;  // (rank, notify pipe?)
      for (auto* list : {&ranks_, &detached_, &standby_})
        for (auto& r : *list) {
          if (r.fd >= 0) {
            pfds.push_back({r.fd, POLLIN, 0});
            owners.push_back({&r, false});
          }
          if (r.nfd >= 0) {
            pfds.push_back({r.nfd, POLLIN, 0});
            owners.push_back({&r, true});
          }
        }
      size_t nrank_fds = pfds.size();
      if (ctl_fd_ >= 0) pfds.push_back({ctl_fd_, POLLIN, 0});
      const size_t stager_slot = pfds.size();
      if (stager_fd_ >= 0) pfds.push_back({stager_fd_, POLLIN, 0});
      int rc = poll(pfds.data(), pfds.size(), (int)(timeout * 1000) + 1);
      if (rc < 0 && errno != EINTR) break;
      bool released = false;
      for (size_t i = 1; i < nrank_fds; ++i) {
        if (!(pfds[i].revents & (POLLIN | POLLHUP | POLLERR))) continue;
        if (owners[i - 1].second) released |= notified(*owners[i - 1].first);
        else pump(*owners[i - 1].first);
      }
      if (released) handoff_released();
      if (s_.standby_hot) keep_hot_standbys();
      if (!s_.preload_argv.empty()) {
        keep_preloaded();
        check_preload_evidence(now());
      }
      if (pfds[0].revents & POLLIN) handle_signals();
      if (ctl_fd_ >= 0 && nrank_fds < pfds.size() && (pfds[nrank_fds].revents & POLLIN))
        handle_control();
      if (stager_fd_ >= 0 && stager_slot < pfds.size() &&
          (pfds[stager_slot].revents & (POLLIN | POLLHUP | POLLERR)))
        read_stager();
      if (stager_fd_ >= 0 && now() >= stager_deadline_) stage_failed("timed out");
      if (dirty_ || now() - last_state > 5) {
        write_state();
        last_state = now();
        dirty_ = false;
      }
    }
    return finish();
  }

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
  static int du_visit(const char*, const struct stat* st, int type, struct FTW*) {
    if (type == FTW_F) du_total_ += (uint64_t)st->st_blocks * 512;
    return 0;
  }
  uint64_t workdir_bytes() {
    du_total_ = 0;
    nftw(s_.workdir.c_str(), du_visit, 32, FTW_PHYS | FTW_MOUNT);
    return du_total_;
  }

  void check_limits(double t) {
    for (auto& k : memory_.check(t, ranks_)) {
      // like a container OOM kill: no grace, the rank fails (no respawn)
      Rank& r = ranks_[k.index];
      r.reason = TermReason::OOM;
      if (r.term_at == 0) r.term_at = t;
      kill(-r.pid, SIGKILL);
      kill(r.pid, SIGKILL);
      r.killed = true;
      event("rank-oom-killed", k.desc);
    }
    if (s_.disk_limit_bytes && t >= next_disk_check_ && !stop_) {
      next_disk_check_ = t + s_.disk_interval;
      const uint64_t used = workdir_bytes();
      if (used > s_.disk_limit_bytes) {
        // ephemeral-storage eviction: every rank is terminated and fails
        event("disk-limit", {"workdir " + std::to_string(used / 1000000) + " MB",
                             "limit " + std::to_string(s_.disk_limit_bytes / 1000000) + " MB"});
        for (int i = 0; i < s_.parallelism; ++i) discard_standby(i, "disk limit");
        for (auto& r : ranks_)
          if (r.state == Rank::RUNNING) terminate(r, TermReason::DISK);
        respawn_at_ = 0;
        for (auto& r : ranks_)
          if (r.state == Rank::PREEMPTED || r.state == Rank::PENDING) {
            write_status(r, "disk-limit", "", "killed");
            r.state = Rank::DONE;
          }
        disk_exceeded_ = true;
      }
    }
  }
  bool disk_exceeded_ = false;

  // ---- off-node container mirror ------------------------------------------------------------
  ContainerSync sync_{s_, [this](const std::string& c, const std::vector<std::string>& d) {
    event(c, d);
  }};

  // ---- workdir stager ----------------------------------------------------------------------
  int stager_fd_ = -1;            // the stager's stdout ("staged ..." line), while staging
  double stager_deadline_ = 0;
  std::string stager_out_;

  // Blocking variant ("before_ranks"): start the stager and wait for "staged".
  void stage() {
    if (!start_stager()) return;
    while (!stop_ && stager_fd_ >= 0) {
      const double left = stager_deadline_ - now();
      if (left <= 0) {
        stage_failed("timed out");
        break;
      }
      struct pollfd pf[3] = {{stager_fd_, POLLIN, 0}, {sfd_, POLLIN, 0}, {ctl_fd_, POLLIN, 0}};
      int rc = poll(pf, ctl_fd_ >= 0 ? 3 : 2, (int)(std::min(left, 1.0) * 1000) + 1);
      if (rc < 0 && errno != EINTR) break;
      if (pf[0].revents & (POLLIN | POLLHUP | POLLERR)) read_stager();
      if (pf[1].revents & POLLIN) handle_signals();
      if (ctl_fd_ >= 0 && (pf[2].revents & POLLIN)) handle_control();
    }
    if (!staged_ && stager_fd_ >= 0) stage_failed("stopped");
  }

  // The stager's stdout: "staged <stats>" once every copy is in HBM and verified.
  void read_stager() {
    char buf[4096];
    ssize_t n = read(stager_fd_, buf, sizeof(buf));
    if (n < 0 && (errno == EAGAIN || errno == EINTR)) return;
    if (n <= 0) {  // EOF: the stager died before staging finished
      stage_failed("stager exited");
      return;
    }
    stager_out_.append(buf, (size_t)n);
    size_t nl = stager_out_.find('\n');
    if (nl != std::string::npos && stager_out_.compare(0, 7, "staged ") == 0) {
      staged_ = true;
      event("workdir-staged", {"manifest " + s_.stager_manifest, stager_out_.substr(7, nl - 7)});
      close(stager_fd_);
      stager_fd_ = -1;
    }
  }

  // Ranks blocked in attach() see "<manifest>.failed" and raise instead of timing out.
  void stage_failed(const std::string& why) {
    if (stager_fd_ >= 0) close(stager_fd_);
    stager_fd_ = -1;
    event("stage-failed", {stop_ ? "stopped" : why, "see " + s_.stager_log});
    atomic_write(s_.stager_manifest + ".failed", why + " (see " + s_.stager_log + ")\n");
    stop_stager();
  }

  bool start_stager() {
    unlink(s_.stager_manifest.c_str());  // a previous incarnation's
    unlink((s_.stager_manifest + ".failed").c_str());
    int p[2];
    if (pipe2(p, O_CLOEXEC)) {
      stage_failed(std::string("pipe: ") + strerror(errno));
      return false;
    }
    int logfd = open(s_.stager_log.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    std::vector<std::string> env;
    bool has_path = false;
    for (auto& kv : s_.env) {
      if (kv.first == "PATH") has_path = true;
      env.push_back(kv.first + "=" + kv.second);
    }
    if (!has_path) env.push_back("PATH=/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin");
    if (!s_.stager_gpus.empty()) env.push_back("HIP_VISIBLE_DEVICES=" + s_.stager_gpus);
    std::vector<char*> envp, argv;
    for (auto& e : env) envp.push_back(const_cast<char*>(e.c_str()));
    envp.push_back(nullptr);
    for (auto& a : s_.stager_argv) argv.push_back(const_cast<char*>(a.c_str()));
    argv.push_back(nullptr);
    pid_t parent = getpid();
    pid_t pid = fork();
    if (pid == 0) {
      setpgid(0, 0);
      prctl(PR_SET_PDEATHSIG, SIGTERM);
      if (getppid() != parent) _exit(127);
      sigset_t none;
      sigemptyset(&none);
      sigprocmask(SIG_SETMASK, &none, nullptr);
      int devnull = open("/dev/null", O_RDONLY);
      if (devnull >= 0) dup2(devnull, 0);
      dup2(p[1], 1);
      if (logfd >= 0) dup2(logfd, 2);
      if (chdir(s_.task_dir.c_str())) _exit(126);
      execve(argv[0], argv.data(), envp.data());
      dprintf(2, "tpi-supervisor: exec %s: %s\n", argv[0], strerror(errno));
      _exit(127);
    }
    close(p[1]);
    if (logfd >= 0) close(logfd);
    if (pid < 0) {
      close(p[0]);
      stage_failed(std::string("fork: ") + strerror(errno));
      return false;
    }
    stager_pid_ = pid;
    stager_fd_ = p[0];
    fcntl(stager_fd_, F_SETFL, fcntl(stager_fd_, F_GETFL) | O_NONBLOCK);
    stager_deadline_ = now() + s_.stager_timeout;
    stager_out_.clear();
    event("stager-start", {"pid " + std::to_string(pid)});
    return true;
  }

  // SIGTERM (the stager writes dirty shards back first), then SIGKILL after the grace period.
  void stop_stager() {
    if (stager_pid_ <= 0) return;
    kill(stager_pid_, SIGTERM);
    const double until = now() + std::max(s_.grace, 5.0);
    int st = 0;
    pid_t got = 0;
    while ((got = waitpid(stager_pid_, &st, WNOHANG)) == 0 && now() < until) usleep(10000);
    if (got == 0) {
      kill(-stager_pid_, SIGKILL);
      kill(stager_pid_, SIGKILL);
      got = waitpid(stager_pid_, &st, 0);
    }
    if (got == stager_pid_) stager_exited(st);
    stager_pid_ = -1;
  }

  void stager_exited(int st) {
    event("stager-exit", {WIFSIGNALED(st) ? std::string("signal ") + signame(WTERMSIG(st))
                                          : "code " + std::to_string(WEXITSTATUS(st))});
    stager_pid_ = -1;
  }

  void event(const std::string& code, const std::vector<std::string>& desc) {
    std::string line = "{\"time\": " + std::to_string(now()) + ", \"code\": " + quote(code) +
                       ", \"description\": [";
    for (size_t i = 0; i < desc.size(); ++i) line += (i ? ", " : "") + quote(desc[i]);
    line += "]}\n";
    int fd = open(s_.events_path.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    if (fd >= 0) {
      write_all(fd, line);
      close(fd);
    }
    if (machine_logs_) {  // TPI_MACHINE_LOGS: the node-side journal of every live machine
      std::string text = utc_stamp(now()) + " tpi-supervisor: " + code;
      for (auto& d : desc) text += " " + d;
      text += "\n";
      for (auto* list : {&ranks_, &standby_})
        for (auto& r : *list)
          if (r.pid > 0 && !r.uuid.empty()) {
            const std::string path = s_.reports_dir + "/machine-" + r.uuid;
            int mfd = open(path.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
            if (mfd >= 0) {
              write_all(mfd, text);
              close(mfd);
            }
          }
    }
    dirty_ = true;
  }

  static const char* state_name(Rank::State st) {
    switch (st) {
      case Rank::PENDING: return "pending";
      case Rank::RUNNING: return "running";
      case Rank::DONE: return "done";
      default: return "preempted";
    }
  }

  int running() const {
    int n = 0;
    for (auto& r : ranks_) n += r.state == Rank::RUNNING;
    return n;
  }

  void write_state(const char* phase = nullptr) {
    if (requeued_ || settled_) return;  // the queue waiter owns state.json / it is final
    atomic_write(s_.state_path, state_json(phase));
  }

  std::string state_json(const char* phase = nullptr) {
    std::string p = phase ? phase
                    : stop_ ? "stopping"
                    : timed_out_ ? "timing-out"
                    : respawn_at_ > 0 ? "respawning"
                    : resources_released_ ? "draining"
                                          : "running";
    std::string out = "{\"pid\": " + std::to_string(getpid()) +
                      ", \"task_id\": " + quote(s_.task_id) + ", \"phase\": " + quote(p) +
                      ", \"started_at\": " + std::to_string(started_) +
                      ", \"heartbeat\": " + std::to_string(now()) +
                      ", \"running\": " + std::to_string(running()) +
                      ", \"restarts\": " + std::to_string(total_restarts_) +
                      ", \"stager_pid\": " + std::to_string(stager_pid_) +
                      ", \"memory_guard\": " + quote(memory_.guard()) + ", \"ranks\": [";
    for (size_t i = 0; i < ranks_.size(); ++i) {
      auto& r = ranks_[i];
      out += std::string(i ? ", " : "") + "{\"rank\": " + std::to_string(r.index) +
             ", \"pid\": " + std::to_string(r.pid) + ", \"uuid\": " + quote(r.uuid) +
             ", \"gpus\": " + quote(r.gpus) + ", \"state\": " + quote(state_name(r.state)) +
             ", \"restarts\": " + std::to_string(r.restarts) +
             ", \"exit_code\": " + std::to_string(r.exit_code) +
             ", \"exit_signal\": " + std::to_string(r.exit_signal) + "}";
    }
    out += "]}\n";
    return out;
  }

  void write_status(Rank& r, const std::string& result, const std::string& code,
                    const std::string& status) {
    std::string body = "{\"result\": " + quote(result) + ", \"code\": " + quote(code) +
                       ", \"status\": " + quote(status) + "}";
    std::string path = s_.reports_dir + "/status-" + r.uuid;
    std::string tmp = s_.reports_dir + "/.status-" + r.uuid + ".tmp";
    int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd >= 0) {
      write_all(fd, body);
      close(fd);
      rename(tmp.c_str(), path.c_str());
    }
  }

  std::vector<std::string> rank_env(const Rank& r) {
    std::vector<std::string> env;
    bool has_path = false;
    for (auto& kv : s_.env) {
      if (kv.first == "PATH") has_path = true;
      env.push_back(kv.first + "=" + kv.second);
    }
    if (!has_path) env.push_back("PATH=/usr/local/sbin:/usr/local/bin:/usr/sbin:/usr/bin:/sbin:/bin");
    auto add = [&](const std::string& k, const std::string& v) { env.push_back(k + "=" + v); };
    add("TPI_MACHINE_IDENTITY", r.uuid);
    add("TPI_LOG_DIRECTORY", s_.reports_dir);
    add("TPI_DATA_DIRECTORY", s_.workdir);
    add("TPI_TASK_IDENTIFIER", s_.task_id);
    add("TPI_TASK_DIRECTORY", s_.task_dir);
    add("TPI_RESTART_COUNT", std::to_string(r.restarts));
    add("TPI_EVENTS_FILE", s_.events_path);  // ranks journal checkpoint phases here
    add("TPI_NOTIFY_FD", "3");                 // "released": spill done, respawn may start
    add("TPI_REQUEUE_FILE", s_.requeue_path);  // exists: reclaimed, no successor here
    add("TPI_REGIONS_FILE", s_.regions_path);  // checkpoint regions: not the working set
    // SIGTERM -> SIGKILL window: a preempted rank saves at its next step boundary and falls
    // back to an immediate save after half of it (checkpoint/preemption.py)
    add("TPI_GRACE_SECONDS", std::to_string(s_.grace));
    // runtime/stage.py attach(): maps the rank's copy, waiting for the manifest if the stager
    // is still loading
    if (staged_ || stager_fd_ >= 0) add("TPI_HBM_WORKDIR", s_.stager_manifest);
    if (s_.deadline > 0) {
      add("TPI_DEADLINE", std::to_string((long long)s_.deadline));
      add("TPI_REMAINING_RUN_TIME", std::to_string((long long)(s_.deadline - now())));
    }
    add("RANK", std::to_string(r.index));
    add("LOCAL_RANK", std::to_string(r.index));
    add("WORLD_SIZE", std::to_string(s_.parallelism));
    add("LOCAL_WORLD_SIZE", std::to_string(s_.parallelism));
    add("GROUP_RANK", "0");
    add("MASTER_ADDR", s_.master_addr);
    add("MASTER_PORT", std::to_string(s_.master_port));
    add("JOB_COMPLETION_INDEX", std::to_string(r.index));  // k8s Indexed Job parity
    if (!r.gpus.empty()) {
      add("HIP_VISIBLE_DEVICES", r.gpus);
      add("TPI_GPUS", r.gpus);
      add("TPI_RANK_GPUS", s_.rank_local_gpus[r.index]);
    }
    return env;
  }

  void spawn(Rank& r, bool standby = false, bool preload = false) {
    r.uuid = uuid4();
    r.partial.clear();
    r.reason = TermReason::NONE;
    r.term_at = 0;
    r.killed = false;
    r.exit_code = -1;
    r.exit_signal = 0;
    std::string logpath = s_.reports_dir + "/task-" + r.uuid;
    r.logfd = open(logpath.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    int p[2], pn[2] = {-1, -1}, go[2] = {-1, -1};
    if (pipe2(pn, O_CLOEXEC)) pn[0] = pn[1] = -1;
    if (standby && pipe2(go, O_CLOEXEC)) go[0] = go[1] = -1;
    if (pipe2(p, O_CLOEXEC) || (standby && go[0] < 0)) {
      for (int fd : {pn[0], pn[1], go[0], go[1]})
        if (fd >= 0) close(fd);
      event("rank-spawn-failed", {"rank " + std::to_string(r.index), strerror(errno)});
      r.state = Rank::DONE;
      write_status(r, "resources", "", "exited");
      return;
    }
    std::vector<std::string> env = rank_env(r);
    if (standby) {
      env.push_back("TPI_STANDBY=1");
      env.push_back("TPI_STANDBY_FD=4");
    }
    std::vector<char*> envp;
    for (auto& e : env) envp.push_back(const_cast<char*>(e.c_str()));
    envp.push_back(nullptr);
    bool shebang = false;
    {
      int sf = open(s_.script.c_str(), O_RDONLY | O_CLOEXEC);
      char hb[2] = {0, 0};
      if (sf >= 0) {
        shebang = read(sf, hb, 2) == 2 && hb[0] == '#' && hb[1] == '!';
        close(sf);
      }
    }
    std::string exec_cmd = "exec \"$0\"";
    // a preloaded successor parks outside the rank's memory cgroup (its imported interpreter
    // would eat into the running rank's limit); it joins the cgroup when it is activated
    const std::string cg_procs = preload ? std::string() : memory_.cgroup_procs(r.index);
    pid_t parent = getpid();
    pid_t pid = fork();
    if (pid == 0) {
      setpgid(0, 0);
      if (!cg_procs.empty()) {  // before exec: everything the rank allocates is capped
        char num[32];
        const int n = snprintf(num, sizeof(num), "%d\n", (int)getpid());
        const int cfd = open(cg_procs.c_str(), O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
        if (cfd >= 0) {
          if (write(cfd, num, (size_t)n) != n) {
          }
          close(cfd);
        }
      }
      prctl(PR_SET_PDEATHSIG, SIGTERM);
      if (getppid() != parent) _exit(127);
      sigset_t none;
      sigemptyset(&none);
      sigprocmask(SIG_SETMASK, &none, nullptr);
      for (int sig : {SIGCHLD, SIGTERM, SIGINT, SIGHUP, SIGUSR1, SIGUSR2, SIGPIPE})
        signal(sig, SIG_DFL);
      int devnull = open("/dev/null", O_RDONLY);
      if (devnull >= 0) dup2(devnull, 0);
      dup2(p[1], 1);
      dup2(p[1], 2);
      // notify pipe -> fd 3, standby activation pipe -> fd 4 (via temporaries >= 10 so
      // neither dup2 can clobber the other's source)
      const int nt = pn[1] >= 0 ? fcntl(pn[1], F_DUPFD_CLOEXEC, 10) : -1;
      const int gt = go[0] >= 0 ? fcntl(go[0], F_DUPFD_CLOEXEC, 10) : -1;
      if (nt >= 0) dup2(nt, 3);
      if (gt >= 0) dup2(gt, 4);
      // the rank's host work (pinned spills, page-cache reads, CRC combine) stays on the
      // socket of its GPUs; best effort: a cpuset that excludes those cores keeps its own mask
      if (!s_.rank_cpus[r.index].empty()) {
        cpu_set_t set;
        CPU_ZERO(&set);
        for (int c : s_.rank_cpus[r.index])
          if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &set);
        (void)sched_setaffinity(0, sizeof(set), &set);
      }
      if (chdir(s_.workdir.c_str())) {
        dprintf(2, "tpi-supervisor: chdir %s: %s\n", s_.workdir.c_str(), strerror(errno));
        _exit(126);
      }
      if (preload) {  // runtime/preload.py: imports now, runs the script once activated
        std::vector<char*> pargv;
        for (auto& a : s_.preload_argv) pargv.push_back(const_cast<char*>(a.c_str()));
        pargv.push_back(const_cast<char*>(s_.script.c_str()));
        pargv.push_back(nullptr);
        execve(pargv[0], pargv.data(), envp.data());
      } else if (s_.login_shell) {
        const char* argv[] = {s_.shell.c_str(), "-lc", exec_cmd.c_str(), s_.script.c_str(), nullptr};
        execve(s_.shell.c_str(), const_cast<char**>(argv), envp.data());
      } else if (shebang) {
        const char* argv[] = {s_.script.c_str(), nullptr};
        execve(s_.script.c_str(), const_cast<char**>(argv), envp.data());
      } else {
        const char* argv[] = {"/bin/sh", s_.script.c_str(), nullptr};
        execve("/bin/sh", const_cast<char**>(argv), envp.data());
      }
      dprintf(2, "tpi-supervisor: exec %s: %s\n", s_.script.c_str(), strerror(errno));
      _exit(127);
    }
    close(p[1]);
    if (pn[1] >= 0) close(pn[1]);
    if (go[0] >= 0) close(go[0]);
    if (pid < 0) {
      close(p[0]);
      if (pn[0] >= 0) close(pn[0]);
      if (go[1] >= 0) close(go[1]);
      event("rank-spawn-failed", {"rank " + std::to_string(r.index), strerror(errno)});
      r.state = Rank::DONE;
      write_status(r, "resources", "", "exited");
      return;
    }
    setpgid(pid, pid);
    fcntl(p[0], F_SETFL, fcntl(p[0], F_GETFL) | O_NONBLOCK);
    r.pid = pid;
    r.fd = p[0];
    if (pn[0] >= 0) fcntl(pn[0], F_SETFL, fcntl(pn[0], F_GETFL) | O_NONBLOCK);
    r.nfd = pn[0];
    r.gofd = go[1];
    r.standby_capable = false;
    r.state = Rank::RUNNING;
    r.started = now();
    r.first_output = false;
    r.released = false;
    r.hold_until = (!standby && r.restarts > 0) ? r.started + kStandbyHold : 0;
    if (!standby) r.hot_spawns = 0;  // a new incarnation: its own standby budget
    std::vector<std::string> desc = {"rank " + std::to_string(r.index), "pid " + std::to_string(pid),
                                     "machine " + r.uuid, "gpus " + (r.gpus.empty() ? "-" : r.gpus),
                                     "restart " + std::to_string(r.restarts)};
    if (preload) desc.push_back("preloaded");
    r.preloaded = preload;
    r.preload_gpu = 0;
    r.gpu_evidence = 0;
    event(standby ? "standby-start" : "rank-start", desc);
  }

  // Warm successor of rank r, spawned while r is being preempted.
  void spawn_standby(Rank& r, bool preload = false) {
    Rank& sb = standby_[r.index];
    if (sb.pid > 0 || stop_ || timed_out_) return;
    if (!preload && (!s_.standby || !r.standby_capable)) return;
    if (s_.max_restarts >= 0 && r.restarts >= s_.max_restarts) return;
    sb = Rank();
    sb.index = r.index;
    sb.gpus = r.gpus;
    sb.restarts = r.restarts + 1;
    spawn(sb, true, preload);
    if (sb.state != Rank::RUNNING) sb = Rank();
  }

  // Preloaded successors (spec "preload_argv", TPI_PRELOAD=1): every running Python rank keeps
  // a process that has imported PyTorch and this package and waits on its activation pipe
  // (runtime/preload.py); the respawn activates it like a warm standby, so a cold successor
  // skips the interpreter start and the imports (~1.8 s of its 1.9 s).  Started kPreloadDelay
  // after the rank (not competing with its own start-up), at most two per incarnation.  A hot
  // standby (which the script itself parks, GPU initialised) takes precedence.
  static constexpr double kPreloadDelay = 2.0;
  void keep_preloaded() {
    const double t = now();
    for (auto& r : ranks_) {
      if (r.state != Rank::RUNNING || r.pid <= 0 || r.term_at > 0 ||
          standby_[r.index].pid > 0 || r.hot_spawns >= 2 || t < r.hold_until ||
          t < r.started + kPreloadDelay || (s_.standby_hot && r.standby_capable))
        continue;
      ++r.hot_spawns;
      spawn_standby(r, true);
    }
  }

  // Hot standby (spec "standby_hot"): every running, standby-capable rank keeps a successor
  // that has already imported its framework and initialised the GPU, so on preemption it is
  // activated the moment the old rank releases -- with a streamed spill, while the spill is
  // still running.  At most two per incarnation (a standby that keeps dying is not retried).
  //
  // A successor that is restoring does not get its own standby yet: starting one (interpreter,
  // framework import, GPU context, engine, spill mapping) competes with the restore for CPU
  // and GPU.  It comes after the successor reports "restored", or kStandbyHold seconds.
  static constexpr double kStandbyHold = 10.0;
  void keep_hot_standbys() {
    const double t = now();
    for (auto& r : ranks_) {
      if (r.state != Rank::RUNNING || r.pid <= 0 || !r.standby_capable || r.term_at > 0 ||
          standby_[r.index].pid > 0 || r.hot_spawns >= 2 || t < r.hold_until)
        continue;
      ++r.hot_spawns;
      spawn_standby(r);
    }
  }

  // Kill an unused standby; its process is reaped (and its log drained) from detached_.
  void discard_standby(int index, const char* why) {
    Rank& sb = standby_[index];
    if (sb.pid <= 0) return;
    if (sb.gofd >= 0) close(sb.gofd);  // EOF without "go": the standby exits on its own
    sb.gofd = -1;
    kill(-sb.pid, SIGKILL);
    kill(sb.pid, SIGKILL);
    sb.killed = true;
    sb.term_at = now();
    sb.exit_requested_at = sb.term_at;
    sb.state = Rank::DONE;
    sb.unused_standby = true;
    // A standby that never ran the script leaves no machine log: nothing printed yet, or a
    // preloaded successor (it never runs the script before activation; what it printed while
    // parked is start-up noise, e.g. libdrm's when it warmed its GPU context).
    struct stat st;
    if (sb.logfd >= 0 && (sb.preloaded || (fstat(sb.logfd, &st) == 0 && st.st_size == 0)))
      unlink((s_.reports_dir + "/task-" + sb.uuid).c_str());
    event("standby-discarded", {"rank " + std::to_string(index), "machine " + sb.uuid, why});
    detached_.push_back(sb);
    sb = Rank();
  }

  // Rank r (PREEMPTED) resumes in its standby: the standby becomes the rank's incarnation.
  bool activate_standby(Rank& r) {
    Rank& sb = standby_[r.index];
    if (sb.pid <= 0) return false;
    // the rendezvous port of this incarnation (the standby was spawned with the previous one)
    const std::string go = "go port=" + std::to_string(s_.master_port) + "\n";
    const bool sent = sb.gofd >= 0 && write(sb.gofd, go.data(), go.size()) == (ssize_t)go.size();
    if (sb.gofd >= 0) close(sb.gofd);
    sb.gofd = -1;
    if (!sent) {
      discard_standby(r.index, "activation failed");
      return false;
    }
    std::vector<std::string> how = {"warm standby"};
    if (sb.preloaded) {
      how.push_back("preloaded");
      if (sb.preload_gpu > 0) how.push_back("GPU warmed");
      join_cgroup(r.index, sb.pid);
    }
    const int restarts = r.restarts;
    r.uuid = sb.uuid;
    r.pid = sb.pid;
    r.fd = sb.fd;
    r.logfd = sb.logfd;
    r.nfd = sb.nfd;
    r.partial = sb.partial;
    r.started = sb.started;
    r.first_output = sb.first_output;
    r.standby_capable = sb.standby_capable;
    r.hot_spawns = 0;
    r.restarts = restarts;
    r.reason = TermReason::NONE;
    r.term_at = 0;
    r.killed = false;
    r.released = false;
    r.exit_code = -1;
    r.exit_signal = 0;
    r.state = Rank::RUNNING;
    r.hold_until = now() + kStandbyHold;
    sb = Rank();
    std::vector<std::string> desc = {"rank " + std::to_string(r.index),
                                     "pid " + std::to_string(r.pid), "machine " + r.uuid,
                                     "gpus " + (r.gpus.empty() ? "-" : r.gpus),
                                     "restart " + std::to_string(r.restarts)};
    desc.insert(desc.end(), how.begin(), how.end());
    event("rank-start", desc);
    return true;
  }

  // Move a (preloaded) process into rank `index`'s memory cgroup, where the rank's own
  // processes are placed at their spawn; memory it charged while parked stays where it was.
  void join_cgroup(int index, pid_t pid) {
    const std::string procs = memory_.cgroup_procs(index);
    if (procs.empty() || pid <= 0) return;
    const int cfd = open(procs.c_str(), O_WRONLY | O_APPEND | O_CLOEXEC);
    if (cfd < 0) return;
    const std::string num = std::to_string((int)pid) + "\n";
    if (write(cfd, num.data(), num.size()) != (ssize_t)num.size()) {
    }
    close(cfd);
  }

  // Processes of process group `pgid` (a rank: the supervisor makes each rank a group leader)
  // that hold `device` open.
  static std::vector<pid_t> device_holders(pid_t pgid, const std::string& device) {
    std::vector<pid_t> out;
    DIR* proc = opendir("/proc");
    if (!proc) return out;
    char path[96], buf[512], link[256];
    while (struct dirent* de = readdir(proc)) {
      if (de->d_name[0] < '0' || de->d_name[0] > '9') continue;
      snprintf(path, sizeof(path), "/proc/%s/stat", de->d_name);
      if (!read_small(path, buf, sizeof(buf))) continue;
      const char* rp = strrchr(buf, ')');
      int ppid = 0, pgrp = 0;
      char state = 0;
      if (!rp || sscanf(rp + 1, " %c %d %d", &state, &ppid, &pgrp) != 3 || pgrp != pgid) continue;
      snprintf(path, sizeof(path), "/proc/%s/fd", de->d_name);
      DIR* fds = opendir(path);
      if (!fds) continue;
      bool holds = false;
      while (struct dirent* fe = readdir(fds)) {
        if (fe->d_name[0] == '.') continue;
        char fpath[160];
        snprintf(fpath, sizeof(fpath), "/proc/%s/fd/%s", de->d_name, fe->d_name);
        const ssize_t n = readlink(fpath, link, sizeof(link) - 1);
        if (n <= 0) continue;
        link[n] = 0;
        if (device == link) {
          holds = true;
          break;
        }
      }
      closedir(fds);
      if (holds) out.push_back((pid_t)atoi(de->d_name));
    }
    closedir(proc);
    return out;
  }

  // Evidence for warming a parked preloaded successor's GPU (spec "preload_gpu_auto"): the
  // successor runs the script in-process, so a context it creates before the script starts is
  // one the script would otherwise create itself -- unless the script forks GPU-using workers
  // before it touches the GPU (they cannot use a context inherited over fork()).  The running
  // incarnation tells which kind the script is: one process of the rank holding the GPU device
  // in two samples -> "warm" (the successor initialises the GPU now: ~0.13 s off a cold
  // recovery, profiles/round5/r5ai); two or more -> the successor stays plain; none yet -> ask
  // again later.
  double next_evidence_ = 0;
  void check_preload_evidence(double t) {
    if (!s_.preload_gpu_auto || t < next_evidence_) return;
    next_evidence_ = t + s_.preload_evidence_interval;
    for (auto& r : ranks_) {
      Rank& sb = standby_[r.index];
      if (r.state != Rank::RUNNING || r.pid <= 0 || r.term_at > 0 || sb.pid <= 0 ||
          !sb.preloaded || sb.preload_gpu != 0 || sb.gofd < 0)
        continue;
      const std::vector<pid_t> holders = device_holders(r.pid, s_.preload_gpu_device);
      if (holders.empty()) continue;
      if (holders.size() > 1) {
        sb.preload_gpu = -1;
        event("preload-plain", {"rank " + std::to_string(r.index),
                                std::to_string(holders.size()) + " processes of the rank hold " +
                                    s_.preload_gpu_device,
                                "the preloaded successor leaves the GPU to the script"});
        continue;
      }
      if (++sb.gpu_evidence < 2) continue;
      static const char kWarm[] = "warm\n";
      if (write(sb.gofd, kWarm, sizeof(kWarm) - 1) != (ssize_t)(sizeof(kWarm) - 1)) continue;
      sb.preload_gpu = 1;
      event("preload-gpu-warm", {"rank " + std::to_string(r.index),
                                 "pid " + std::to_string(holders[0]) + " alone holds " +
                                     s_.preload_gpu_device,
                                 "the preloaded successor initialises its GPU context now"});
    }
  }

  void emit_line(Rank& r, const std::string& line) {
    if (r.logfd < 0) return;
    const double t = now();
    write_all(r.logfd, utc_stamp(t) + " " + line + "\n");
    if (!r.first_output) {  // phase journal: start -> first log line of this incarnation
      r.first_output = true;
      char ms[32];
      snprintf(ms, sizeof(ms), "%.1f ms", (t - r.started) * 1e3);
      event("rank-first-output", {"rank " + std::to_string(r.index), ms});
    }
  }

  void pump(Rank& r) {
    char buf[65536];
    for (;;) {
      ssize_t n = read(r.fd, buf, sizeof(buf));
      if (n > 0) {
        r.partial.append(buf, (size_t)n);
        size_t start = 0, nl;
        while ((nl = r.partial.find('\n', start)) != std::string::npos) {
          emit_line(r, r.partial.substr(start, nl - start));
          start = nl + 1;
        }
        r.partial.erase(0, start);
        if (r.partial.size() > (1 << 20)) {
          emit_line(r, r.partial);
          r.partial.clear();
        }
        continue;
      }
      if (n == 0) {  // EOF: every writer (rank and its children) closed the pipe
        if (!r.partial.empty()) emit_line(r, r.partial);
        r.partial.clear();
        close(r.fd);
        r.fd = -1;
        if (r.pid < 0) close_log(r);
        return;
      }
      if (errno == EINTR) continue;
      return;  // EAGAIN
    }
  }

  // Notify pipe readable: returns true when the rank announced "released" and may be handed
  // off (its spill is complete -- or streaming -- and the supervisor is terminating it as a
  // preemption or a reclaim).  One message per line:
  //   released      the save no longer needs this process's place: respawn / requeue now
  //   standby       the script calls preemption.standby() (warm successors possible)
  //   restored      this incarnation restored its state: its predecessor may go
  //   restored hbm  ... from the predecessor's HBM: the predecessor goes only after "closed"
  //   closed        the IPC mappings of the predecessor's HBM are gone
  bool notified(Rank& r) {
    char buf[256];
    bool got = false;
    for (;;) {
      ssize_t n = read(r.nfd, buf, sizeof(buf));
      if (n > 0) {
        r.note.append(buf, (size_t)n);
        size_t start = 0, nl;
        while ((nl = r.note.find('\n', start)) != std::string::npos) {
          const std::string msg = r.note.substr(start, nl - start);
          start = nl + 1;
          if (msg == "released") {
            got = true;
          } else if (msg == "standby") {
            r.standby_capable = true;
          } else if (msg.compare(0, 8, "restored") == 0) {
            r.hold_until = 0;  // its hot standby may start now
            if (msg == "restored hbm") {
              r.awaiting_close = true;  // the predecessor's memory is still mapped here
            } else {
              release_predecessors(r.index, "successor restored");
            }
          } else if (msg == "closed") {
            r.awaiting_close = false;
            release_predecessors(r.index, "successor closed the HBM hand-off");
          }
        }
        r.note.erase(0, start);
        if (r.note.size() > 4096) r.note.clear();
        continue;
      }
      if (n == 0) {
        close(r.nfd);
        r.nfd = -1;
      } else if (errno == EINTR) {
        continue;
      }
      break;
    }
    if (!got || r.pid <= 0 || r.state != Rank::RUNNING || stop_ || timed_out_) return false;
    if (!(r.reason == TermReason::PREEMPT || r.reason == TermReason::REQUEUE ||
          (r.reason == TermReason::NONE && s_.respawn_on_sigterm)))
      return false;
    r.released = true;
    return true;
  }

  // The successor of rank `index` no longer needs its predecessor (restored from the host
  // region, closed its HBM imports, or died): a predecessor that lingers after its spill
  // (keeping its host region pinned so its teardown cannot slow the restore's DMA, and its
  // exported HBM mapped) may exit now.
  void release_predecessors(int index, const char* why) {
    for (auto& d : detached_)
      if (d.index == index && d.pid > 0 && d.exit_requested_at <= 0 && !d.killed) {
        kill(d.pid, SIGUSR2);
        d.exit_requested_at = now();
        event("predecessor-exit-requested", {"rank " + std::to_string(index),
                                             "machine " + d.uuid, why});
      }
  }

  // Released ranks become PREEMPTED now; their old process keeps draining its log and is
  // reaped (or killed after the grace period) from detached_.
  void handoff_released() {
    for (auto& r : ranks_) {
      if (!r.released || r.pid <= 0) continue;
      r.released = false;
      Rank old = r;
      if (old.nfd >= 0) close(old.nfd);
      old.nfd = -1;
      old.state = Rank::DONE;
      if (old.term_at == 0) old.term_at = now();
      detached_.push_back(old);
      std::vector<std::string> desc = {"rank " + std::to_string(r.index), "machine " + r.uuid,
                                       "pid " + std::to_string(r.pid)};
      r.pid = -1;
      r.fd = -1;
      r.logfd = -1;
      r.nfd = -1;
      r.partial.clear();
      r.note.clear();
      r.awaiting_close = false;
      if (r.reason == TermReason::REQUEUE) {
        // reclaimed: its checkpoint is in host memory and its HBM is free; nobody restores
        // from this GPU, so it may exit now and its resources go to the reclaiming task
        // without waiting for its teardown (release_resources once the gang is down)
        Rank& d = detached_.back();
        kill(d.pid, SIGUSR2);
        d.exit_requested_at = now();
        r.exit_code = -1;
        r.state = Rank::DONE;
        desc.push_back("requeue");
        event("rank-released", desc);
        desc.pop_back();
        event("rank-requeued", desc);
        continue;
      }
      r.exit_code = 143;
      r.state = Rank::PREEMPTED;
      event("rank-released", desc);
      if (s_.gang)
        for (auto& o : ranks_)
          if (o.state == Rank::RUNNING) terminate(o, TermReason::PREEMPT);
      respawn_at_ = now() + s_.respawn_delay;
    }
  }

  void close_log(Rank& r) {
    if (r.logfd >= 0) {
      struct stat st;
      // a standby that never ran the script (a preloaded one, or killed before it printed)
      // leaves no empty machine log behind for `leo read`
      const bool empty = r.unused_standby && fstat(r.logfd, &st) == 0 && st.st_size == 0;
      close(r.logfd);
      r.logfd = -1;
      if (empty) unlink((s_.reports_dir + "/task-" + r.uuid).c_str());
    }
  }

  void terminate(Rank& r, TermReason why) {
    if (r.pid <= 0 || r.state != Rank::RUNNING) return;
    if (r.reason == TermReason::NONE || why == TermReason::STOP || why == TermReason::DISK ||
        (why == TermReason::REQUEUE && r.reason == TermReason::PREEMPT))
      r.reason = why;
    if (r.term_at == 0) {
      r.term_at = now();
      kill(-r.pid, SIGTERM);
      kill(r.pid, SIGTERM);
    }
  }

  // Exit trace: a released or discarded process should be gone within ~1-2 s (its kernel
  // teardown: unpinning the host region, freeing HBM and the GPU context).  Where one spends
  // longer shows in /proc: its scheduler state (D = uninterruptible, inside the driver or the
  // mm teardown; Z = exited, not yet reaped) and the kernel function it sleeps in (wchan),
  // journalled whenever they change, with its resident set, every kTraceInterval seconds.
  static constexpr double kTraceInterval = 0.1;
  static constexpr int kTraceMax = 64;  // events per process

  static std::string thread_waits(pid_t pid) {
    std::string out;
    char path[96], buf[512];
    snprintf(path, sizeof(path), "/proc/%d/task", (int)pid);
    DIR* d = opendir(path);
    if (!d) return "-";
    while (struct dirent* e = readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      std::string one = e->d_name;
      snprintf(path, sizeof(path), "/proc/%d/task/%s/stat", (int)pid, e->d_name);
      if (read_small(path, buf, sizeof(buf))) {
        const char* rp = strrchr(buf, ')');
        one += std::string(":") + (rp && rp[1] == ' ' ? rp[2] : '?');
      }
      snprintf(path, sizeof(path), "/proc/%d/task/%s/wchan", (int)pid, e->d_name);
      if (read_small(path, buf, sizeof(buf)) && buf[0]) one += std::string(":") + buf;
      snprintf(path, sizeof(path), "/proc/%d/task/%s/stack", (int)pid, e->d_name);
      if (read_small(path, buf, sizeof(buf))) {  // "[<0>] func+0x../0x..\n..."
        std::string top(buf);
        top = top.substr(0, top.find('\n'));
        const size_t sp = top.find(' ');
        one += ":" + (sp == std::string::npos ? top : top.substr(sp + 1));
      }
      out += (out.empty() ? "" : " ") + one;
    }
    closedir(d);
    return out.empty() ? "-" : out;
  }

  void trace_exits(double t) {
    if (!s_.exit_trace) return;
    for (auto& d : detached_) {
      if (d.pid <= 0 || (d.exit_requested_at <= 0 && !d.killed)) continue;
      if (d.exit_requested_at <= 0) d.exit_requested_at = d.term_at > 0 ? d.term_at : t;
      if (d.trace_events >= kTraceMax || t - d.trace_last_at < kTraceInterval * 0.9) continue;
      char path[64], buf[512];
      snprintf(path, sizeof(path), "/proc/%d/stat", (int)d.pid);
      if (!read_small(path, buf, sizeof(buf))) continue;
      const char* rp = strrchr(buf, ')');
      char state = rp && rp[1] == ' ' ? rp[2] : '?';
      snprintf(path, sizeof(path), "/proc/%d/wchan", (int)d.pid);
      char wchan[128] = "-";
      if (read_small(path, wchan, sizeof(wchan)) && !wchan[0]) snprintf(wchan, sizeof(wchan), "-");
      long rss_mb = -1, threads = -1;
      snprintf(path, sizeof(path), "/proc/%d/status", (int)d.pid);
      std::ifstream in(path);
      std::string key;
      while (in >> key) {
        long value = 0;
        if (key == "VmRSS:" && in >> value) rss_mb = value / 1024;
        else if (key == "Threads:" && in >> value) threads = value;
        in.ignore(1 << 16, '\n');
      }
      const std::string sample = std::string(1, state) + " " + wchan;
      // a change of state / wait point, or once a second while nothing changes (RSS drains)
      if (sample == d.trace_last && t - d.trace_last_at < 1.0) continue;
      d.trace_last = sample;
      d.trace_last_at = t;
      ++d.trace_events;
      char el[48];
      snprintf(el, sizeof(el), "+%.3f s", t - d.exit_requested_at);
      std::vector<std::string> desc = {"rank " + std::to_string(d.index), "machine " + d.uuid,
                                       "pid " + std::to_string(d.pid), el,
                                       std::string("state ") + state,
                                       std::string("wchan ") + wchan,
                                       "rss " + std::to_string(rss_mb) + " MB",
                                       "threads " + std::to_string(threads)};
      // The last threads of an exiting process (the leader already a zombie): where each one
      // waits in the kernel, and the top of its kernel stack where /proc lets us read it
      // (root only) -- the teardown's slow path, named.
      if (threads > 0 && threads <= 4) desc.push_back("tasks " + thread_waits(d.pid));
      event("exit-trace", desc);
    }
  }

  void check_grace(double t) {
    for (auto* list : {&ranks_, &detached_})
      for (auto& r : *list)
        if (r.pid > 0 && r.term_at > 0 && !r.killed && t >= r.term_at + s_.grace) {
          kill(-r.pid, SIGKILL);
          kill(r.pid, SIGKILL);
          r.killed = true;
          event("rank-killed", {"rank " + std::to_string(r.index), "grace period expired"});
        }
  }

  void check_deadline(double t) {
    if (s_.deadline <= 0 || timed_out_ || t < s_.deadline) return;
    timed_out_ = true;
    respawn_at_ = 0;
    event("deadline", {"timeout reached"});
    for (int i = 0; i < s_.parallelism; ++i) discard_standby(i, "deadline");
    for (auto& r : ranks_) {
      if (r.state == Rank::RUNNING) {
        terminate(r, TermReason::TIMEOUT);
      } else if (r.state == Rank::PREEMPTED || r.state == Rank::PENDING) {
        write_status(r, "timeout", "", "killed");
        r.state = Rank::DONE;
      }
    }
  }

  void check_respawn(double t) {
    if (respawn_at_ <= 0 || t < respawn_at_ || stop_ || timed_out_ || requeue_ ||
        disk_exceeded_)
      return;
    if (s_.gang && running() > 0) return;  // wait for the whole gang to go down
    respawn_at_ = 0;
    if (s_.gang && s_.parallelism > 1) next_master_port();
    for (auto& r : ranks_)
      if (r.state == Rank::PREEMPTED) {
        if (s_.max_restarts >= 0 && r.restarts >= s_.max_restarts) {
          write_status(r, "start-limit-hit", "", "exited");
          r.state = Rank::DONE;
          discard_standby(r.index, "restart limit");
          event("rank-restart-limit", {"rank " + std::to_string(r.index)});
          continue;
        }
        r.restarts++;
        total_restarts_++;
        event("respawn", {"rank " + std::to_string(r.index),
                          "restart " + std::to_string(r.restarts)});
        if (!activate_standby(r)) spawn(r);
      }
  }

  // A fresh rendezvous port for every gang incarnation: a predecessor that lingers after its
  // spill (early hand-off) may still hold the old one -- rank 0's TCPStore listens on it.
  void next_master_port() {
    for (int i = 1; i <= 256; ++i) {
      int port = s_.master_port + i;
      if (port > 65000) port = 20000 + port % 1000;
      int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
      struct sockaddr_in a;
      memset(&a, 0, sizeof(a));
      a.sin_family = AF_INET;
      a.sin_port = htons((uint16_t)port);
      a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
      const bool free_port = fd >= 0 && bind(fd, (struct sockaddr*)&a, sizeof(a)) == 0;
      if (fd >= 0) close(fd);
      if (free_port) {
        s_.master_port = port;
        event("rendezvous", {"master port " + std::to_string(port)});
        return;
      }
    }
  }

  void handle_signals() {
    struct signalfd_siginfo si;
    while (read(sfd_, &si, sizeof(si)) == sizeof(si)) {
      switch (si.ssi_signo) {
        case SIGCHLD: reap(); break;
        case SIGTERM:
        case SIGINT:
        case SIGHUP:
          request_stop(std::string("signal ") + signame(si.ssi_signo));
          break;
        case SIGUSR1:
          request_preempt("signal USR1");
          break;
        default: break;
      }
    }
    reap();
  }

  void request_stop(const std::string& source) {
    if (stop_) return;
    stop_ = true;
    respawn_at_ = 0;
    event("stop-requested", {source});
    for (int i = 0; i < s_.parallelism; ++i) discard_standby(i, "stop");
    for (auto& r : ranks_) {
      if (r.state == Rank::RUNNING) terminate(r, TermReason::STOP);
      else if (r.state != Rank::DONE) r.state = Rank::DONE;
    }
    dirty_ = true;
  }

  // rank < 0: every rank.  A single preempted rank takes its gang down with it when it exits
  // (reap), like a reclaimed spot VM of a coupled group.
  bool request_preempt(const std::string& source, int rank = -1) {
    if (stop_ || timed_out_) return false;
    if (rank >= (int)ranks_.size() || (rank >= 0 && ranks_[rank].state != Rank::RUNNING))
      return false;
    event("preempt-requested", {rank < 0 ? "all ranks" : "rank " + std::to_string(rank), source});
    for (auto& r : ranks_)
      if (rank < 0 || r.index == rank) terminate(r, TermReason::PREEMPT);
    for (auto& r : ranks_)
      if ((rank < 0 || r.index == rank) && r.state == Rank::RUNNING) spawn_standby(r);
    dirty_ = true;
    return true;
  }

  // Spot reclaim (an on-demand task needs this task's GPUs): every rank is preempted --
  // checkpointed as usual -- but not respawned here; once the gang is down the reservation is
  // released and the task goes back to the node queue (requeue_argv), to resume wherever it
  // is placed next (resource_auto_scaling_group.go:51-106: a reclaimed spot instance is
  // replaced when capacity returns).
  bool request_requeue(const std::string& source) {
    if (stop_ || timed_out_ || s_.requeue_argv.empty()) return false;
    if (requeue_) return true;
    requeue_ = true;
    respawn_at_ = 0;
    // before any SIGTERM: a rank that sees the marker saves without hand-off and leaves
    atomic_write(s_.requeue_path, source + "\n");
    event("requeue-requested", {source});
    for (int i = 0; i < s_.parallelism; ++i) discard_standby(i, "requeue");
    for (auto& r : ranks_) {
      if (r.state == Rank::RUNNING) {
        terminate(r, TermReason::REQUEUE);
      } else if (r.state == Rank::PREEMPTED || r.state == Rank::PENDING) {
        r.state = Rank::DONE;  // between preemption and respawn: resumes after the queue
        r.reason = TermReason::REQUEUE;
      }
    }
    dirty_ = true;
    return true;
  }

  // ---- control socket --------------------------------------------------------------------
  // sun_path holds 108 bytes and task directories can be longer, so bind/connect go through
  // /proc/self/fd/<dirfd>/<name> (the client in backends/node.py does the same).
  void open_control() {
    size_t slash = s_.control_path.rfind('/');
    std::string dir = slash == std::string::npos ? "." : s_.control_path.substr(0, slash);
    std::string name = slash == std::string::npos ? s_.control_path
                                                  : s_.control_path.substr(slash + 1);
    int dfd = open(dir.c_str(), O_PATH | O_DIRECTORY | O_CLOEXEC);
    if (dfd < 0) return;
    unlinkat(dfd, name.c_str(), 0);
    struct sockaddr_un addr;
    memset(&addr, 0, sizeof(addr));
    addr.sun_family = AF_UNIX;
    int n = snprintf(addr.sun_path, sizeof(addr.sun_path), "/proc/self/fd/%d/%s", dfd,
                     name.c_str());
    int fd = socket(AF_UNIX, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
    mode_t old = umask(077);  // the socket file is created 0600: owner-only control
    bool ok = fd >= 0 && n > 0 && n < (int)sizeof(addr.sun_path) &&
              bind(fd, (struct sockaddr*)&addr, sizeof(addr)) == 0 && listen(fd, 16) == 0;
    umask(old);
    close(dfd);
    if (!ok) {
      if (fd >= 0) close(fd);
      event("control-unavailable", {strerror(errno)});
      return;
    }
    ctl_fd_ = fd;
  }

  void close_control() {
    if (ctl_fd_ < 0) return;
    close(ctl_fd_);
    ctl_fd_ = -1;
    unlink(s_.control_path.c_str());
  }

  void handle_control() {
    for (;;) {
      int c = accept4(ctl_fd_, nullptr, nullptr, SOCK_CLOEXEC);
      if (c < 0) return;  // EAGAIN: drained
      // One request line; a client that sends nothing within 200 ms is dropped so the event
      // loop never stalls on it.
      std::string req;
      char buf[256];
      double until = now() + 0.2;
      while (req.find('\n') == std::string::npos && req.size() < 4096) {
        struct pollfd p = {c, POLLIN, 0};
        int left = (int)((until - now()) * 1000);
        if (left <= 0 || poll(&p, 1, left) <= 0) break;
        ssize_t got = read(c, buf, sizeof(buf));
        if (got <= 0) break;
        req.append(buf, (size_t)got);
      }
      size_t end = req.find_first_of("\r\n");
      if (end != std::string::npos) req.resize(end);
      std::string reply;
      if (req == "ping") {
        reply = "{\"ok\": true, \"pid\": " + std::to_string(getpid()) +
                ", \"task_id\": " + quote(s_.task_id) + "}\n";
      } else if (req == "state") {
        reply = state_json();
      } else if (req == "preempt" || req.compare(0, 8, "preempt ") == 0) {
        int rank = -1;
        bool parsed = true;
        if (req.size() > 8) {
          char* endp = nullptr;
          long v = strtol(req.c_str() + 8, &endp, 10);
          parsed = endp && *endp == '\0' && v >= 0 && v < (long)ranks_.size();
          rank = (int)v;
        }
        bool ok = parsed && request_preempt("control socket", rank);
        reply = ok ? "{\"ok\": true}\n"
                   : "{\"ok\": false, \"error\": \"no running rank to preempt\"}\n";
      } else if (req == "stop") {
        request_stop("control socket");
        reply = "{\"ok\": true}\n";
      } else if (req == "requeue" || req.compare(0, 8, "requeue ") == 0) {
        const bool ok = request_requeue(req.size() > 8 ? req.substr(8) : "control socket");
        reply = ok ? "{\"ok\": true}\n"
                   : "{\"ok\": false, \"error\": \"task cannot be requeued\"}\n";
      } else {
        reply = "{\"ok\": false, \"error\": " + quote("unknown command: " + req) + "}\n";
      }
      write_all(c, reply);
      close(c);
    }
  }

  void reap() {
    for (;;) {
      int st = 0;
      pid_t pid = waitpid(-1, &st, WNOHANG);
      if (pid <= 0) return;
      if (pid == stager_pid_) {  // the stager died while ranks still use the images
        stager_exited(st);
        continue;
      }
      if (pid == sync_.pid()) {
        sync_.exited(st);
        continue;
      }
      for (size_t i = 0; i < detached_.size(); ++i)
        if (detached_[i].pid == pid) {
          Rank& d = detached_[i];
          if (d.fd >= 0) pump(d);
          if (d.fd >= 0) close(d.fd);
          close_log(d);
          const std::string code = WIFSIGNALED(st) ? std::string("signal ") + signame(WTERMSIG(st))
                                                   : "code " + std::to_string(WEXITSTATUS(st));
          std::vector<std::string> desc = {"rank " + std::to_string(d.index),
                                           "machine " + d.uuid, code};
          if (d.exit_requested_at > 0) {
            char took[64];
            snprintf(took, sizeof(took), "%.3f s after the exit request",
                     now() - d.exit_requested_at);
            desc.push_back(took);
          }
          event("rank-released-exit", desc);
          detached_.erase(detached_.begin() + i);
          break;
        }
      for (auto& sb : standby_)
        if (sb.pid == pid) {  // a standby died before it was activated
          if (sb.fd >= 0) pump(sb);
          for (int fd : {sb.fd, sb.nfd, sb.gofd})
            if (fd >= 0) close(fd);
          close_log(sb);
          event("standby-exit", {"rank " + std::to_string(sb.index), "machine " + sb.uuid,
                                 WIFSIGNALED(st) ? std::string("signal ") + signame(WTERMSIG(st))
                                                 : "code " + std::to_string(WEXITSTATUS(st))});
          sb = Rank();
        }
      for (auto& r : ranks_)
        if (r.pid == pid) on_exit(r, st);
    }
  }

  void on_exit(Rank& r, int st) {
    if (r.nfd >= 0) notified(r);  // "closed" / "restored" written just before the exit
    if (r.awaiting_close) {  // died with the predecessor's HBM mapped: the kernel unmapped it
      r.awaiting_close = false;
      release_predecessors(r.index, "successor exited");
    }
    if (r.fd >= 0) pump(r);  // drain what is already buffered
    if (r.nfd >= 0) {
      close(r.nfd);
      r.nfd = -1;
    }
    r.pid = -1;
    if (r.fd < 0) close_log(r);
    bool signaled = WIFSIGNALED(st);
    int sig = signaled ? WTERMSIG(st) : 0;
    int code = WIFEXITED(st) ? WEXITSTATUS(st) : -1;
    if (signaled && sig == SIGKILL && !r.killed && r.reason == TermReason::NONE) {
      if (memory_.oom_by_cgroup(r.index)) {  // the kernel stopped it at the cgroup cap
        r.reason = TermReason::OOM;
        event("rank-oom-killed", {"rank " + std::to_string(r.index), "memory cgroup cap",
                                  "limit " + std::to_string(s_.rank_memory_kb / 1024) + " MB"});
      }
    }
    r.exit_code = code;
    r.exit_signal = sig;
    std::string code_s = signaled ? signame(sig) : std::to_string(code);
    std::string status_s = signaled ? (WCOREDUMP(st) ? "dumped" : "killed") : "exited";
    std::vector<std::string> desc = {"rank " + std::to_string(r.index), "machine " + r.uuid,
                                     (signaled ? "signal " : "code ") + code_s};
    if (r.reason == TermReason::STOP || stop_) {
      discard_standby(r.index, "stop");
      r.state = Rank::DONE;  // scaled to zero: no status (the machine was "shut down")
      event("rank-stopped", desc);
      return;
    }
    if (r.reason == TermReason::TIMEOUT) {
      discard_standby(r.index, "timeout");
      r.state = Rank::DONE;
      write_status(r, "timeout", code_s, status_s);
      event("rank-timeout", desc);
      return;
    }
    if (r.reason == TermReason::OOM || r.reason == TermReason::DISK) {
      const bool oom = r.reason == TermReason::OOM;
      discard_standby(r.index, oom ? "memory limit" : "disk limit");
      r.state = Rank::DONE;
      write_status(r, oom ? "oom" : "disk-limit", code_s, status_s);
      event(oom ? "rank-oom" : "rank-disk-limit", desc);
      if (oom && s_.fail_fast)
        for (auto& o : ranks_)
          if (o.state == Rank::RUNNING) terminate(o, TermReason::FAILFAST);
      return;
    }
    if (r.reason == TermReason::REQUEUE && !(WIFEXITED(st) && code == 0)) {
      r.state = Rank::DONE;  // no status: the task is not over, it waits for capacity again
      event("rank-requeued", desc);
      return;
    }
    bool preempted = r.reason == TermReason::PREEMPT ||
                     (s_.respawn_on_sigterm && r.reason == TermReason::NONE &&
                      ((signaled && sig == SIGTERM) || code == 143));
    if (preempted && !timed_out_) {
      r.state = Rank::PREEMPTED;
      event("rank-preempted", desc);
      if (s_.gang)
        for (auto& o : ranks_)
          if (o.state == Rank::RUNNING) terminate(o, TermReason::PREEMPT);
      respawn_at_ = now() + s_.respawn_delay;
      return;
    }
    r.state = Rank::DONE;
    discard_standby(r.index, "rank finished");
    std::string result = signaled ? "signal" : (code == 0 ? "success" : "exit-code");
    if (r.reason == TermReason::FAILFAST) result = "signal";
    write_status(r, result, code_s, status_s);
    event("rank-exit", desc);
    if (!signaled && code != 0 && s_.fail_fast)
      for (auto& o : ranks_)
        if (o.state == Rank::RUNNING) terminate(o, TermReason::FAILFAST);
  }

  // No rank will run again and none is running: only released / discarded processes may
  // still be exiting.
  bool ranks_settled() {
    for (auto& r : ranks_)
      if (r.state != Rank::DONE || r.pid > 0) return false;
    for (auto& sb : standby_)
      if (sb.pid > 0) return false;
    return true;
  }

  bool all_finished() { return ranks_settled() && detached_.empty(); }

  // Give the task's node resources back: the stager (its HBM workdir images), the GPU lease
  // files and the reservation; a reclaimed task goes back to the queue.  Released processes
  // that are still tearing down are left to exit (traced, reaped, SIGKILLed after the grace
  // period) -- they hold no state anybody needs: their checkpoint is in host memory.
  void release_resources() {
    if (resources_released_) return;
    resources_released_ = true;
    // predecessors still lingering for a successor that will never come (or is done)
    for (auto& d : detached_)
      if (d.pid > 0 && d.exit_requested_at <= 0 && !d.killed) {
        kill(d.pid, SIGUSR2);
        d.exit_requested_at = now();
      }
    stop_stager();
    int unlinked = 0, exiting = 0;
    // A GPU lease becomes its drain marker (gpu-N.lease -> gpu-N.drain, same JSON, with the
    // driver's VRAM count at the reservation): the next task placed on that GPU waits until
    // the driver has taken this task's HBM back (placement.settle_gpus) -- released processes
    // may still be exiting, and the driver wipes freed VRAM for seconds after that.
    for (auto& l : s_.leases) {
      static const std::string kLease = ".lease";
      bool gpu = l.size() > kLease.size() &&
                 l.compare(l.size() - kLease.size(), kLease.size(), kLease) == 0;
      std::string drain = gpu ? l.substr(0, l.size() - kLease.size()) + ".drain" : "";
      unlinked += (gpu ? rename(l.c_str(), drain.c_str()) : unlink(l.c_str())) == 0;
    }
    for (auto& d : detached_) exiting += d.pid > 0;
    event("resources-released", {std::to_string(unlinked) + " lease file(s)",
                                 std::to_string(exiting) + " released process(es) still exiting"});
    dirty_ = true;
  }

  // Every rank is down and the resources are back: finish the task for its users now --
  // drain the ranks' logs, run the final (awaited) off-node sync, then either put the task
  // back into the queue or write the final state -- instead of after the last released
  // process has been reaped.  The final sync runs before the requeue, so the next
  // incarnation never mirrors a container this one is still writing.
  void settle() {
    if (settled_) return;
    drain_rank_logs();
    sync_.final();  // the logs and statuses of every rank are written by now
    bool pending = false;  // a reclaimed rank that has not finished on its own
    if (requeue_ && !stop_ && !timed_out_)
      for (auto& r : ranks_)
        if (r.reason == TermReason::REQUEUE && !(r.exit_signal == 0 && r.exit_code == 0))
          pending = true;
    close_control();  // the next incarnation (requeued or restarted) binds the same path
    if (pending) requeued_ = spawn_requeue();
    int exiting = 0;
    for (auto& d : detached_) exiting += d.pid > 0;
    event("supervisor-settled", {requeued_ ? "requeued" : stop_ ? "stopped" : "all ranks finished",
                                 std::to_string(exiting) + " released process(es) still exiting"});
    if (!requeued_) write_state("stopped");
    settled_ = true;
  }

  // Ranks are gone; give lingering writers (daemonized children) a moment, then close.
  void drain_rank_logs() {
    double until = now() + 0.5;
    while (now() < until) {
      bool open_fd = false;
      std::vector<struct pollfd> pfds;
      std::vector<Rank*> owners;
      for (auto& r : ranks_)
        if (r.fd >= 0) {
          open_fd = true;
          pfds.push_back({r.fd, POLLIN, 0});
          owners.push_back(&r);
        }
      if (!open_fd) break;
      poll(pfds.data(), pfds.size(), 50);
      for (size_t i = 0; i < pfds.size(); ++i)
        if (pfds[i].revents) pump(*owners[i]);
    }
    for (auto& r : ranks_) {
      if (r.fd >= 0) {
        if (!r.partial.empty()) emit_line(r, r.partial);
        close(r.fd);
        r.fd = -1;
      }
      close_log(r);
    }
  }

  int finish() {
    release_resources();
    settle();
    memory_.cleanup();
    event("supervisor-exit", {requeued_ ? "requeued" : stop_ ? "stopped" : "all ranks finished"});
    signal_ready();
    return 0;
  }

  // Detached (own session) child that puts the task back into the node queue; it owns
  // state.json from here on (phase "queued").
  bool spawn_requeue() {
    write_state("requeued");
    pid_t pid = fork();
    if (pid < 0) {
      event("requeue-failed", {strerror(errno)});
      return false;
    }
    if (pid == 0) {
      setsid();
      if (fork() != 0) _exit(0);  // the grandchild is reparented: no zombie, no pdeathsig
      sigset_t none;
      sigemptyset(&none);
      sigprocmask(SIG_SETMASK, &none, nullptr);
      for (int sig : {SIGCHLD, SIGTERM, SIGINT, SIGHUP, SIGUSR1, SIGUSR2, SIGPIPE})
        signal(sig, SIG_DFL);
      int devnull = open("/dev/null", O_RDWR);
      if (devnull >= 0) {
        dup2(devnull, 0);
        dup2(devnull, 1);
      }
      std::vector<char*> argv;
      for (auto& a : s_.requeue_argv) argv.push_back(const_cast<char*>(a.c_str()));
      argv.push_back(nullptr);
      execv(argv[0], argv.data());
      _exit(127);
    }
    int st = 0;
    waitpid(pid, &st, 0);
    event("requeued", {"waiting for capacity"});
    return true;
  }
};

thread_local uint64_t Supervisor::du_total_ = 0;

}  // namespace

#ifndef TPI_VERSION_STRING
#define TPI_VERSION_STRING "0.0.0-dev"
#endif

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "--version") {
    printf("tpi-supervisor %s\n", TPI_VERSION_STRING);
    return 0;
  }
  bool daemonize = argc >= 3 && std::string(argv[1]) == "--daemon";
  const char* spec_path = daemonize ? argv[2] : (argc >= 2 ? argv[1] : nullptr);
  if (!spec_path) {
    fprintf(stderr, "usage: %s [--daemon] <spec.json>\n", argv[0]);
    return 2;
  }
  try {
    Spec spec = load_spec(spec_path);
    if (daemonize) {
      int p[2];
      if (pipe2(p, O_CLOEXEC)) throw std::runtime_error("pipe2 failed");
      pid_t pid = fork();
      if (pid < 0) throw std::runtime_error("fork failed");
      if (pid > 0) {  // launcher: report the daemon's pid once it is ready
        close(p[1]);
        char c;
        ssize_t n;
        do {
          n = read(p[0], &c, 1);
        } while (n < 0 && errno == EINTR);
        printf("%d\n", (int)pid);
        fflush(stdout);
        _exit(n == 1 ? 0 : 1);
      }
      close(p[0]);
      g_ready_fd = p[1];
      setsid();
      dup2(2, 1);  // stdout -> the supervisor log the launcher gave us as stderr
    }
    Supervisor sup(std::move(spec));
    return sup.run();
  } catch (const std::exception& e) {
    fprintf(stderr, "tpi-supervisor: %s\n", e.what());
    return 1;
  }
}
