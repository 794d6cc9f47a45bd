// Shared pieces of the supervisor: small I/O helpers, the rank record and the task spec.
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

namespace tpi_sup {

inline double now() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

inline std::string read_file(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw std::runtime_error("cannot read " + path);
  std::stringstream ss;
  ss << in.rdbuf();
  return ss.str();
}

inline void write_all(int fd, const std::string& s) {
  const char* p = s.data();
  size_t left = s.size();
  while (left) {
    ssize_t n = write(fd, p, left);
    if (n < 0) {
      if (errno == EINTR) continue;
      return;
    }
    p += n;
    left -= (size_t)n;
  }
}

inline bool atomic_write(const std::string& path, const std::string& data) {
  std::string tmp = path + ".tmp";
  int fd = open(tmp.c_str(), O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) return false;
  write_all(fd, data);
  close(fd);
  return rename(tmp.c_str(), path.c_str()) == 0;
}

inline std::string uuid4() {
  unsigned char b[16];
  int fd = open("/dev/urandom", O_RDONLY | O_CLOEXEC);
  if (fd < 0 || read(fd, b, 16) != 16) {
    for (int i = 0; i < 16; ++i) b[i] = (unsigned char)(rand() & 0xff);
  }
  if (fd >= 0) close(fd);
  b[6] = (b[6] & 0x0f) | 0x40;
  b[8] = (b[8] & 0x3f) | 0x80;
  char out[37];
  snprintf(out, sizeof(out),
           "%02x%02x%02x%02x-%02x%02x-%02x%02x-%02x%02x-%02x%02x%02x%02x%02x%02x", b[0], b[1],
           b[2], b[3], b[4], b[5], b[6], b[7], b[8], b[9], b[10], b[11], b[12], b[13], b[14],
           b[15]);
  return out;
}

inline std::string utc_stamp(double t) {
  time_t s = (time_t)t;
  struct tm tm;
  gmtime_r(&s, &tm);
  char buf[32];
  strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%SZ", &tm);
  return buf;
}

inline const char* signame(int sig) {
  switch (sig) {
    case SIGTERM: return "TERM";
    case SIGKILL: return "KILL";
    case SIGINT: return "INT";
    case SIGHUP: return "HUP";
    case SIGSEGV: return "SEGV";
    case SIGABRT: return "ABRT";
    case SIGBUS: return "BUS";
    case SIGFPE: return "FPE";
    case SIGILL: return "ILL";
    case SIGPIPE: return "PIPE";
    case SIGQUIT: return "QUIT";
    case SIGUSR1: return "USR1";
    case SIGUSR2: return "USR2";
    default: return "UNKNOWN";
  }
}

enum class TermReason { NONE, STOP, PREEMPT, TIMEOUT, FAILFAST, REQUEUE, OOM, DISK };

// --daemon: the launching parent blocks on this pipe until the ranks are spawned and the
// first state.json is on disk, so "create returned" implies "supervisor visible".
inline int g_ready_fd = -1;

inline void signal_ready() {
  if (g_ready_fd >= 0) {
    write_all(g_ready_fd, "1");
    close(g_ready_fd);
    g_ready_fd = -1;
  }
}

struct Rank {
  int index = 0;
  std::string gpus;
  pid_t pid = -1;
  int fd = -1;
  int logfd = -1;
  int nfd = -1;  // read end of the rank's notify pipe (TPI_NOTIFY_FD in the rank)
  std::string uuid;
  std::string partial;
  std::string note;  // partial line read from the notify pipe
  enum State { PENDING, RUNNING, DONE, PREEMPTED } state = PENDING;
  int restarts = 0;
  TermReason reason = TermReason::NONE;
  double term_at = 0;
  bool killed = false;
  int exit_code = -1, exit_signal = 0;
  double started = 0;
  bool first_output = false;  // phase journal: first line of this incarnation seen
  bool released = false;      // wrote "released" on its notify pipe
  bool standby_capable = false;  // announced "standby" (calls preemption.standby())
  int hot_spawns = 0;            // hot standbys started for this incarnation
  bool unused_standby = false;   // a standby discarded before activation (empty log: removed)
  int gofd = -1;                 // standby only: write end of its activation pipe
  double hold_until = 0;  // a resuming incarnation: no new hot standby until it restored
  // preloaded successor (runtime/preload.py) only: parked outside the rank's memory cgroup
  // (it joins at activation), and whether its GPU context was warmed on evidence
  // (+1 warmed, -1 kept plain, 0 undecided) after `gpu_evidence` agreeing samples
  bool preloaded = false;
  int preload_gpu = 0;
  int gpu_evidence = 0;
  // restored from its predecessor's HBM ("restored hbm"): the predecessor must stay alive
  // until this incarnation has unmapped the IPC imports ("closed") or died
  bool awaiting_close = false;
  // detached (released / discarded): when it was told to go, and the exit trace so far
  double exit_requested_at = 0;
  std::string trace_last;
  double trace_last_at = 0;
  int trace_events = 0;
};

struct Spec {
  std::string task_id, task_dir, workdir, script, shell = "/bin/bash";
  std::vector<std::pair<std::string, std::string>> env;
  double deadline = 0;
  int parallelism = 1;
  std::vector<std::string> rank_gpus;        // HIP_VISIBLE_DEVICES (the task's GPU set)
  std::vector<std::string> rank_local_gpus;  // the rank's own GPUs, task-visible numbering
  std::vector<std::vector<int>> rank_cpus;   // NUMA-local cores of the rank's GPUs (affinity)
  std::string master_addr = "127.0.0.1";
  int master_port = 29500;
  bool master_port_probe = false;  // master_port is a base: take the first free port from it
  bool gang = true, fail_fast = true, respawn_on_sigterm = true, login_shell = false;
  bool standby = false;
  bool standby_hot = false;  // keep the standby running before any preemption
  int max_restarts = -1;
  double grace = 30, respawn_delay = 0;
  std::string reports_dir, state_path, events_path, control_path;
  // written before a spot reclaim's SIGTERM: the ranks save without hand-off, free their HBM
  // and leave at once (TPI_REQUEUE_FILE; nobody restores from this GPU)
  std::string requeue_path;
  bool exit_trace = true;  // journal state/wchan of released processes until they are reaped
  std::vector<std::string> leases;
  // workdir stager (spec "stager", runtime/stage.py): started before the ranks, holds the
  // HBM copies of the workdir for the task's lifetime
  std::vector<std::string> stager_argv;
  std::string stager_manifest, stager_log, stager_gpus;
  double stager_timeout = 600;
  // false (default): ranks start while the stager loads (attach() waits for the manifest),
  // so staging is off the first-log path; true: ranks start once the workdir is in HBM
  bool stage_before_ranks = false;
  // machine-type limits (resource_job.go:112-118 turns cpu/memory/disk into pod limits):
  // host memory per rank (its process group; 0 = none) and the task's workdir size
  uint64_t rank_memory_kb = 0;
  uint64_t disk_limit_bytes = 0;
  // hard cap: each rank's processes in a memory cgroup (v2 memory.max / v1
  // memory.limit_in_bytes) of rank_memory + headroom -- "auto" (the hierarchy this process is
  // in, when writable), "off", or a cgroup directory; the poll below keeps enforcing the limit
  // itself (without checkpoint regions), the cgroup stops a runaway allocation between polls
  std::string cgroup = "auto";
  int cgroup_version = 0;
  uint64_t cgroup_headroom_kb = 0;  // checkpoint regions (shm pages charge the first toucher)
  std::string regions_path;         // checkpoint regions announced by the ranks (host.py)
  double memory_interval = 1.0, disk_interval = 10.0;
  double memory_fast_interval = 0.02;  // statm poll of the ranks' process trees (s)
  // spot reclaim: after `requeue` the task goes back to the node queue through this command
  std::vector<std::string> requeue_argv;
  // off-node storage.container mirror (storage/remote.py): run every sync_interval s while
  // ranks run (tpl:118-124) and once, awaited, when they are done (ExecStop's final copy)
  std::vector<std::string> sync_argv;
  // preloaded successors (TPI_PRELOAD): the launcher; the script path is appended
  std::vector<std::string> preload_argv;
  // TPI_PRELOAD=1/auto: warm the parked successor's GPU context ("warm" on its activation
  // pipe) once the running rank shows it is safe -- exactly one of the rank's processes holds
  // the GPU device (preload_gpu_device, /dev/kfd), over two samples
  bool preload_gpu_auto = false;
  std::string preload_gpu_device = "/dev/kfd";
  double preload_evidence_interval = 1.0;
  double sync_interval = 10, sync_timeout = 600;
  int restart_base = 0;  // restarts of earlier supervisors of this task (requeued incarnations)
};

inline Spec load_spec(const std::string& path) {
  Value v = tpi::json::parse(read_file(path));
  Spec s;
  s.task_id = v["task_id"].str();
  s.task_dir = v["task_dir"].str();
  s.workdir = v["workdir"].str();
  s.script = v["script"].str();
  s.shell = v["shell"].str("/bin/bash");
  for (auto& kv : v["env"].o) s.env.emplace_back(kv.first, kv.second.str());
  s.deadline = v["deadline"].num(0);
  s.parallelism = std::max(1, (int)v["parallelism"].num(1));
  for (auto& r : v["ranks"].a) {
    s.rank_gpus.push_back(r["gpus"].str());
    s.rank_local_gpus.push_back(r["rank_gpus"].str());
    std::vector<int> cpus;
    for (auto& c : r["cpus"].a) cpus.push_back((int)c.num(-1));
    s.rank_cpus.push_back(cpus);
  }
  s.rank_gpus.resize(s.parallelism);
  s.rank_local_gpus.resize(s.parallelism);
  s.rank_cpus.resize(s.parallelism);
  s.master_addr = v["master_addr"].str("127.0.0.1");
  s.master_port = (int)v["master_port"].num(29500);
  s.master_port_probe = v["master_port_probe"].boolean(false);
  s.gang = v["gang"].boolean(true);
  s.fail_fast = v["fail_fast"].boolean(s.parallelism > 1);
  s.respawn_on_sigterm = v["respawn_on_sigterm"].boolean(true);
  s.login_shell = v["login_shell"].boolean(false);
  s.max_restarts = (int)v["max_restarts"].num(-1);
  s.grace = v["grace_seconds"].num(30);
  s.respawn_delay = v["respawn_delay"].num(0);
  s.standby = v["standby"].boolean(false);
  s.standby_hot = s.standby && v["standby_hot"].boolean(false);
  s.reports_dir = v["reports_dir"].str(s.task_dir + "/reports");
  s.state_path = v["state_path"].str(s.task_dir + "/supervisor/state.json");
  s.events_path = v["events_path"].str(s.task_dir + "/supervisor/events.jsonl");
  s.control_path = v["control_path"].str(s.task_dir + "/supervisor/control.sock");
  {
    const size_t slash = s.state_path.rfind('/');
    const std::string dir = slash == std::string::npos ? "." : s.state_path.substr(0, slash);
    s.requeue_path = v["requeue_path"].str(dir + "/requeue");
  }
  s.exit_trace = v["exit_trace"].boolean(true);
  for (auto& l : v["leases"].a) s.leases.push_back(l.str());
  const Value& st = v["stager"];
  for (auto& a : st["argv"].a) s.stager_argv.push_back(a.str());
  s.stager_manifest = st["manifest"].str();
  s.stager_log = st["log"].str(s.task_dir + "/supervisor/stager.log");
  s.stager_gpus = st["gpus"].str();
  s.stager_timeout = st["timeout"].num(600);
  s.stage_before_ranks = st["before_ranks"].boolean(false);
  const Value& lim = v["limits"];
  s.rank_memory_kb = (uint64_t)lim["rank_memory_mb"].num(0) * 1024;
  s.disk_limit_bytes = (uint64_t)(lim["disk_gb"].num(0) * 1e9);
  s.memory_interval = lim["memory_interval"].num(1.0);
  s.memory_fast_interval = lim["memory_fast_interval"].num(0.02);
  s.cgroup = lim["cgroup"].str("auto");
  s.cgroup_version = (int)lim["cgroup_version"].num(0);
  s.cgroup_headroom_kb = (uint64_t)lim["cgroup_headroom_mb"].num(0) * 1024;
  {
    const size_t slash = s.state_path.rfind('/');
    const std::string dir = slash == std::string::npos ? "." : s.state_path.substr(0, slash);
    s.regions_path = v["regions_path"].str(dir + "/regions");
  }
  s.disk_interval = lim["disk_interval"].num(10.0);
  for (auto& a : v["requeue_argv"].a) s.requeue_argv.push_back(a.str());
  for (auto& a : v["sync"]["argv"].a) s.sync_argv.push_back(a.str());
  for (auto& a : v["preload_argv"].a) s.preload_argv.push_back(a.str());
  s.preload_gpu_auto = v["preload_gpu_auto"].boolean(false);
  s.preload_gpu_device = v["preload_gpu_device"].str("/dev/kfd");
  s.preload_evidence_interval = v["preload_evidence_interval"].num(1.0);
  s.sync_interval = v["sync"]["interval"].num(10);
  s.sync_timeout = v["sync"]["timeout"].num(600);
  s.restart_base = (int)v["restart_base"].num(0);
  if (s.workdir.empty() || s.script.empty()) throw std::runtime_error("spec needs workdir+script");
  return s;
}

// Small /proc file into buf (NUL-terminated); false when unreadable or empty.
inline bool read_small(const char* path, char* buf, size_t cap) {
  int fd = open(path, O_RDONLY | O_CLOEXEC);
  if (fd < 0) return false;
  ssize_t n = read(fd, buf, cap - 1);
  close(fd);
  if (n <= 0) return false;
  buf[n] = 0;
  return true;
}

}  // namespace tpi_sup
