// tpi-supervisor (supervisor.h), ranks: spawning ranks, warm and hot standbys and preloaded
// successors (with the evidence that lets a preloaded successor warm its GPU), their output
// pipes (machine logs) and notify pipes (released / restored / closed / standby).
#include "supervisor.h"

namespace tpi_sup {

std::vector<std::string> Supervisor::rank_env(const Rank& r) {
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

void Supervisor::spawn(Rank& r, bool standby, bool preload) {
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
void Supervisor::spawn_standby(Rank& r, bool preload) {
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

void Supervisor::keep_preloaded() {
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

void Supervisor::keep_hot_standbys() {
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
void Supervisor::discard_standby(int index, const char* why) {
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
bool Supervisor::activate_standby(Rank& r) {
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
void Supervisor::join_cgroup(int index, pid_t pid) {
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
std::vector<pid_t> Supervisor::device_holders(pid_t pgid, const std::string& device) {
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

void Supervisor::check_preload_evidence(double t) {
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

void Supervisor::emit_line(Rank& r, const std::string& line) {
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

void Supervisor::pump(Rank& r) {
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
bool Supervisor::notified(Rank& r) {
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
void Supervisor::release_predecessors(int index, const char* why) {
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
void Supervisor::handoff_released() {
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

void Supervisor::close_log(Rank& r) {
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

}  // namespace tpi_sup
