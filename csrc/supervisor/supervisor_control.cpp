// tpi-supervisor (supervisor.h), control: signals and the control socket, the deadline,
// the grace period and respawns, host-memory and disk limits, the workdir stager, the exit
// trace of released processes, and the requeue of a reclaimed task.
#include "supervisor.h"

namespace tpi_sup {

int Supervisor::du_visit(const char*, const struct stat* st, int type, struct FTW*) {
  if (type == FTW_F) du_total_ += (uint64_t)st->st_blocks * 512;
  return 0;
}

uint64_t Supervisor::workdir_bytes() {
  du_total_ = 0;
  nftw(s_.workdir.c_str(), du_visit, 32, FTW_PHYS | FTW_MOUNT);
  return du_total_;
}

void Supervisor::check_limits(double t) {
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

// Blocking variant ("before_ranks"): start the stager and wait for "staged".
void Supervisor::stage() {
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
void Supervisor::read_stager() {
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
void Supervisor::stage_failed(const std::string& why) {
  if (stager_fd_ >= 0) close(stager_fd_);
  stager_fd_ = -1;
  event("stage-failed", {stop_ ? "stopped" : why, "see " + s_.stager_log});
  atomic_write(s_.stager_manifest + ".failed", why + " (see " + s_.stager_log + ")\n");
  stop_stager();
}

bool Supervisor::start_stager() {
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
void Supervisor::stop_stager() {
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

void Supervisor::stager_exited(int st) {
  event("stager-exit", {WIFSIGNALED(st) ? std::string("signal ") + signame(WTERMSIG(st))
                                        : "code " + std::to_string(WEXITSTATUS(st))});
  stager_pid_ = -1;
}

void Supervisor::terminate(Rank& r, TermReason why) {
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

std::string Supervisor::thread_waits(pid_t pid) {
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

void Supervisor::trace_exits(double t) {
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

void Supervisor::check_grace(double t) {
  for (auto* list : {&ranks_, &detached_})
    for (auto& r : *list)
      if (r.pid > 0 && r.term_at > 0 && !r.killed && t >= r.term_at + s_.grace) {
        kill(-r.pid, SIGKILL);
        kill(r.pid, SIGKILL);
        r.killed = true;
        event("rank-killed", {"rank " + std::to_string(r.index), "grace period expired"});
      }
}

void Supervisor::check_deadline(double t) {
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

void Supervisor::check_respawn(double t) {
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
void Supervisor::next_master_port() { pick_master_port(1); }

// The first port at master_port + from, ... that binds on the loopback (spec
// "master_port_probe": the task's first incarnation, so `tpi apply` does not probe ports
// itself -- its Python side then needs no socket module).
void Supervisor::pick_master_port(int from) {
  for (int i = from; i <= from + 255; ++i) {
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
      if (port == s_.master_port && from == 0) return;  // the base itself: nothing to say
      s_.master_port = port;
      event("rendezvous", {"master port " + std::to_string(port)});
      return;
    }
  }
}

void Supervisor::handle_signals() {
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

void Supervisor::request_stop(const std::string& source) {
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
bool Supervisor::request_preempt(const std::string& source, int rank) {
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
bool Supervisor::request_requeue(const std::string& source) {
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
void Supervisor::open_control() {
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

void Supervisor::close_control() {
  if (ctl_fd_ < 0) return;
  close(ctl_fd_);
  ctl_fd_ = -1;
  unlink(s_.control_path.c_str());
}

void Supervisor::handle_control() {
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

// Detached (own session) child that puts the task back into the node queue; it owns
// state.json from here on (phase "queued").
bool Supervisor::spawn_requeue() {
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

}  // namespace tpi_sup
