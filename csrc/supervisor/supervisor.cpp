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
#include "supervisor.h"

namespace tpi_sup {

Supervisor::Supervisor(Spec spec) : s_(std::move(spec)) {
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

int Supervisor::run() {
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
  if (s_.master_port_probe) pick_master_port(0);
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

void Supervisor::event(const std::string& code, const std::vector<std::string>& desc) {
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

const char* Supervisor::state_name(Rank::State st) {
  switch (st) {
    case Rank::PENDING: return "pending";
    case Rank::RUNNING: return "running";
    case Rank::DONE: return "done";
    default: return "preempted";
  }
}

int Supervisor::running() const {
  int n = 0;
  for (auto& r : ranks_) n += r.state == Rank::RUNNING;
  return n;
}

void Supervisor::write_state(const char* phase) {
  if (requeued_ || settled_) return;  // the queue waiter owns state.json / it is final
  atomic_write(s_.state_path, state_json(phase));
}

std::string Supervisor::state_json(const char* phase) {
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

void Supervisor::write_status(Rank& r, const std::string& result, const std::string& code, const std::string& status) {
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

void Supervisor::reap() {
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

void Supervisor::on_exit(Rank& r, int st) {
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
bool Supervisor::ranks_settled() {
  for (auto& r : ranks_)
    if (r.state != Rank::DONE || r.pid > 0) return false;
  for (auto& sb : standby_)
    if (sb.pid > 0) return false;
  return true;
}

// Give the task's node resources back: the stager (its HBM workdir images), the GPU lease
// files and the reservation; a reclaimed task goes back to the queue.  Released processes
// that are still tearing down are left to exit (traced, reaped, SIGKILLed after the grace
// period) -- they hold no state anybody needs: their checkpoint is in host memory.
void Supervisor::release_resources() {
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
void Supervisor::settle() {
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
void Supervisor::drain_rank_logs() {
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

int Supervisor::finish() {
  release_resources();
  settle();
  memory_.cleanup();
  event("supervisor-exit", {requeued_ ? "requeued" : stop_ ? "stopped" : "all ranks finished"});
  signal_ready();
  return 0;
}

thread_local uint64_t Supervisor::du_total_ = 0;

}  // namespace tpi_sup

using namespace tpi_sup;

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
