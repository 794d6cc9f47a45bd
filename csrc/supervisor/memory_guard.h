// Host-memory limit of a task's ranks (the machine type's memory, enforced per rank).
//
// Reference: k8s turns the machine type into pod limits the kernel enforces
// (task/k8s/resources/resource_job.go:107-118).  Here each rank gets a memory cgroup where the
// hierarchy is writable (the hard cap), and a /proc poll of its process tree in any case: every
// memory_interval a full scan, every memory_fast_interval (20 ms) where no cgroup could be made
// (an unprivileged box) a statm sum -- with checkpoint regions, which mirror device state,
// never counted.  The supervisor kills what check() returns and reads cgroup OOM kills back
// on a rank's exit (oom_by_cgroup).
#pragma once

#include <dirent.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <fstream>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "common.h"

namespace tpi_sup {

class MemoryGuard {
 public:
  using EventFn = std::function<void(const std::string&, const std::vector<std::string>&)>;
  struct Kill {
    int index;                      // rank over its limit: kill it now (no grace, no respawn)
    std::vector<std::string> desc;  // for the rank-oom-killed event
  };

  MemoryGuard(const Spec& s, EventFn event) : s_(s), event_(std::move(event)) {}

  // Which guard runs ("cgroup v2", "poll 20 ms", "" without a limit), for state.json.
  const std::string& guard() const { return memory_guard_; }
  // cgroup.procs file a new rank joins before exec ("" without a cgroup).
  std::string cgroup_procs(int index) const {
    return index < (int)cg_dirs_.size() && !cg_dirs_[index].empty()
               ? cg_dirs_[index] + "/cgroup.procs" : std::string();
  }
  // A SIGKILLed rank: did the kernel stop it at its cgroup cap (a new OOM kill counted)?
  bool oom_by_cgroup(int index) {
    const uint64_t kills = cgroup_oom_kills(index);
    if (index < 0 || index >= (int)cg_oom_.size() || kills <= cg_oom_[index]) return false;
    cg_oom_[index] = kills;
    return true;
  }
  double next_check() const { return next_memory_check_; }
  // At the supervisor's start: a cgroup per rank where the hierarchy allows, else the poll.
  void start() { setup(); }
  // At its end: the (by then empty) cgroups go.
  void cleanup() { remove_cgroups(); }

  std::vector<Kill> check(double t, const std::vector<Rank>& ranks) {
    std::vector<Kill> kills;
    if (s_.rank_memory_kb && t >= next_memory_check_) {
      const bool fast = cg_version_ == 0 && s_.memory_fast_interval > 0;
      next_memory_check_ = t + (fast ? std::min(s_.memory_fast_interval, s_.memory_interval)
                                     : s_.memory_interval);
      if ((int)mem_.size() != s_.parallelism) mem_.assign(s_.parallelism, MemTrack());
      const bool full = t >= next_memory_scan_;
      std::map<long, GroupMemory> groups;
      if (full) {
        next_memory_scan_ = t + s_.memory_interval;
        std::set<long> pgids;
        for (auto& r : ranks)
          if (r.state == Rank::RUNNING && r.pid > 0 && !r.killed) pgids.insert(r.pid);
        if (!pgids.empty()) groups = groups_memory(pgids);
      }
      std::vector<Region> regions;
      bool regions_loaded = false;
      for (auto& r : ranks) {
        if (r.state != Rank::RUNNING || r.pid <= 0 || r.killed) continue;
        MemTrack& m = mem_[r.index];
        if (m.pid != r.pid) m = MemTrack(), m.pid = r.pid;
        if (full) {
          auto g = groups.find(r.pid);
          m.members = g == groups.end() ? std::vector<long>() : g->second.pids;
        }
        std::vector<long> pids;
        tree_pids(r.pid, pids);
        for (long p : m.members)
          if (std::find(pids.begin(), pids.end(), p) == pids.end()) pids.push_back(p);
        const uint64_t rss = resident_kb(pids);
        // quick bound: the counted size at the last split plus any growth since (new
        // resident pages are at most new private pages); before any split, the resident set
        // minus the regions' share measured last time
        const uint64_t bound = m.valid ? m.counted_at + (rss > m.rss_at ? rss - m.rss_at : 0)
                                       : (rss > region_kb_[r.index] ? rss - region_kb_[r.index] : 0);
        if (bound <= s_.rank_memory_kb) continue;
        if (!regions_loaded) regions = load_regions(), regions_loaded = true;
        const auto split = pss_split_kb(pids, regions);
        region_kb_[r.index] = split.second;
        const uint64_t kb = split.first - std::min(split.first, split.second);
        m.rss_at = rss;
        m.counted_at = kb;
        m.valid = true;
        if (kb <= s_.rank_memory_kb) continue;
        std::vector<std::string> desc = {"rank " + std::to_string(r.index),
                                         "memory " + std::to_string(kb / 1024) + " MB",
                                         "limit " + std::to_string(s_.rank_memory_kb / 1024) +
                                             " MB"};
        if (split.second)
          desc.push_back("checkpoint regions " + std::to_string(split.second / 1024) +
                         " MB not counted");
        kills.push_back({r.index, desc});
      }
    }
    return kills;

  }

 private:
  const Spec& s_;
  EventFn event_;
  double next_memory_check_ = 0, next_memory_scan_ = 0;
  std::string memory_guard_;

  // ---- machine-type limits -------------------------------------------------------------------
  // Host memory of the ranks' process groups, from one pass over /proc.  The resident set
  // (/proc/<pid>/statm) is O(1) per process but counts pages shared inside a group (forked
  // data-loader workers, a spill region mapped twice) once per member, so it is an upper bound.
  // Only a group whose bound is over its limit pays for the proportional set size
  // (smaps_rollup walks the page tables: tens of ms for a 100 GB pinned spill), which splits
  // shared pages between their users and decides the OOM kill.

  struct GroupMemory {
    uint64_t rss_kb = 0;
    std::vector<long> pids;
  };

  static std::map<long, GroupMemory> groups_memory(const std::set<long>& pgids) {
    static const uint64_t page_kb = (uint64_t)sysconf(_SC_PAGESIZE) / 1024;
    std::map<long, GroupMemory> out;
    DIR* d = opendir("/proc");
    if (!d) return out;
    while (struct dirent* e = readdir(d)) {
      char* end = nullptr;
      long pid = strtol(e->d_name, &end, 10);
      if (!end || *end || pid <= 0) continue;
      char path[64], buf[512];
      snprintf(path, sizeof(path), "/proc/%ld/stat", pid);
      if (!read_small(path, buf, sizeof(buf))) continue;
      const char* rp = strrchr(buf, ')');
      long pgrp = 0, ppid = 0;
      char state = 0;
      if (!rp || sscanf(rp + 1, " %c %ld %ld", &state, &ppid, &pgrp) != 3 || !pgids.count(pgrp))
        continue;
      snprintf(path, sizeof(path), "/proc/%ld/statm", pid);
      if (!read_small(path, buf, sizeof(buf))) continue;
      unsigned long long size = 0, resident = 0;
      if (sscanf(buf, "%llu %llu", &size, &resident) != 2) continue;
      GroupMemory& g = out[pgrp];
      g.rss_kb += resident * page_kb;
      g.pids.push_back(pid);
    }
    closedir(d);
    return out;
  }

  static uint64_t pss_kb(const std::vector<long>& pids) {
    uint64_t total = 0;
    for (long pid : pids) {
      std::ifstream in("/proc/" + std::to_string(pid) + "/smaps_rollup");
      std::string key;
      uint64_t value;
      while (in >> key) {
        if (key == "Pss:" && in >> value) {
          total += value;
          break;
        }
        in.ignore(1 << 20, '\n');
      }
    }
    return total;
  }

  // Checkpoint spill regions announced by the ranks (checkpoint/host.py: one line
  // "<pid> <start> <end> <path|->" per mapping).  They mirror device state -- a rank's
  // checkpoint of 100+ GB of HBM -- and are not its working set, so the limit leaves them out
  // (a file-backed region matches by path in every process that maps it, an anonymous one by
  // the announcing pid and address range).
  struct Region {
    long pid = 0;
    uint64_t start = 0, end = 0;
    std::string path;
  };

  std::vector<Region> load_regions() const {
    std::vector<Region> out;
    std::ifstream in(s_.regions_path);
    std::string line;
    while (std::getline(in, line)) {
      Region r;
      char path[4096] = "";
      unsigned long long a = 0, b = 0;
      if (sscanf(line.c_str(), "%ld %llx %llx %4095[^\n]", &r.pid, &a, &b, path) < 3) continue;
      r.start = a;
      r.end = b;
      if (strcmp(path, "-") != 0) r.path = path;
      out.push_back(r);
    }
    return out;
  }

  // Proportional set size of a group, and the part of it in checkpoint regions (kB).
  static std::pair<uint64_t, uint64_t> pss_split_kb(const std::vector<long>& pids,
                                                    const std::vector<Region>& regions) {
    if (regions.empty()) return {pss_kb(pids), 0};
    uint64_t total = 0, excluded = 0;
    for (long pid : pids) {
      std::ifstream in("/proc/" + std::to_string(pid) + "/smaps");
      std::string line;
      bool skip = false;
      while (std::getline(in, line)) {
        if (line.empty()) continue;
        const char c = line[0];
        if ((c >= '0' && c <= '9') || (c >= 'a' && c <= 'f')) {  // "start-end perms ... path"
          unsigned long long a = 0, b = 0;
          int consumed = 0;
          skip = false;
          if (sscanf(line.c_str(), "%llx-%llx %*s %*s %*s %*s%n", &a, &b, &consumed) < 2) continue;
          std::string path = consumed > 0 && (size_t)consumed < line.size()
                                 ? line.substr((size_t)consumed) : std::string();
          path.erase(0, path.find_first_not_of(' '));
          const std::string deleted = " (deleted)";
          if (path.size() > deleted.size() &&
              path.compare(path.size() - deleted.size(), deleted.size(), deleted) == 0)
            path.resize(path.size() - deleted.size());
          for (const Region& r : regions)
            if ((!r.path.empty() && r.path == path) ||
                (r.path.empty() && r.pid == pid && a < r.end && r.start < b)) {
              skip = true;
              break;
            }
        } else if (line.compare(0, 4, "Pss:") == 0) {
          const uint64_t v = strtoull(line.c_str() + 4, nullptr, 10);
          total += v;
          if (skip) excluded += v;
        }
      }
    }
    return {total, excluded};
  }

  std::map<int, uint64_t> region_kb_;  // rank index -> its regions' share at the last check

  // ---- memory cgroups (the hard cap) ----------------------------------------------------------
  // k8s turns the machine type into a pod memory limit (resource_job.go:112-118): the kernel
  // stops a container at it, however fast it allocates.  The /proc poll above sees a rank only
  // every memory_interval; a rank that allocates faster than that could take the node down
  // first.  So each rank also gets a memory cgroup -- v2 memory.max or v1
  // memory.limit_in_bytes -- when the hierarchy is writable (root, or a delegated subtree),
  // capped at limit + headroom: shm pages of a checkpoint region are charged to the cgroup of
  // the process that first touched them, so a GPU rank gets room for its GPUs' HBM.
  std::vector<std::string> cg_dirs_;  // per rank index; empty: no cgroup
  std::vector<uint64_t> cg_oom_;      // kernel OOM kills seen per rank
  int cg_version_ = 0;
  std::string cg_root_;

  static bool write_text(const std::string& path, const std::string& text, bool append = false) {
    int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_CLOEXEC | (append ? O_APPEND : O_TRUNC),
                  0644);
    if (fd < 0) return false;
    const ssize_t n = write(fd, text.data(), text.size());
    const int saved = errno;
    close(fd);
    errno = saved;
    return n == (ssize_t)text.size();
  }

  // Our own cgroup path ("" controller: the v2 entry "0::/path").
  static std::string own_cgroup(const std::string& controller) {
    std::ifstream in("/proc/self/cgroup");
    std::string line;
    while (std::getline(in, line)) {
      const size_t a = line.find(':'), b = line.find(':', a + 1);
      if (a == std::string::npos || b == std::string::npos) continue;
      const std::string ctl = line.substr(a + 1, b - a - 1), path = line.substr(b + 1);
      if (controller.empty() ? (line.compare(0, a, "0") == 0 && ctl.empty())
                             : ("," + ctl + ",").find("," + controller + ",") != std::string::npos)
        return path == "/" ? "" : path;
    }
    return "";
  }

  // cgroups of supervisors that died without cleaning up (tpi-<task>-<pid>-r<i>)
  static void sweep_stale_cgroups(const std::string& root) {
    DIR* d = opendir(root.c_str());
    if (!d) return;
    while (struct dirent* e = readdir(d)) {
      const std::string name = e->d_name;
      if (name.compare(0, 4, "tpi-") != 0) continue;
      const size_t r = name.rfind("-r"), dash = r == std::string::npos ? r : name.rfind('-', r - 1);
      if (dash == std::string::npos) continue;
      const long pid = strtol(name.c_str() + dash + 1, nullptr, 10);
      if (pid > 0 && kill((pid_t)pid, 0) != 0 && errno == ESRCH)
        rmdir((root + "/" + name).c_str());
    }
    closedir(d);
  }

  void setup() {
    cg_dirs_.assign(s_.parallelism, "");
    cg_oom_.assign(s_.parallelism, 0);
    if (!s_.rank_memory_kb) return;
    if (s_.cgroup.empty() || s_.cgroup == "off") {
      memory_guard_ = "poll " + std::to_string((int)(s_.memory_fast_interval * 1000)) + " ms";
      event_("memory-guard", {memory_guard_, "cgroup off",
                             "limit " + std::to_string(s_.rank_memory_kb / 1024) + " MB"});
      return;
    }
    std::string root, why;
    int ver = s_.cgroup_version;
    struct stat st;
    if (s_.cgroup == "auto") {
      if (stat("/sys/fs/cgroup/cgroup.controllers", &st) == 0) {
        ver = 2;
        root = "/sys/fs/cgroup" + own_cgroup("");
        // children need the memory controller in our subtree (granted only where the
        // hierarchy is delegated to us)
        write_text(root + "/cgroup.subtree_control", "+memory");
      } else if (stat("/sys/fs/cgroup/memory/memory.limit_in_bytes", &st) == 0) {
        ver = 1;
        const std::string own = "/sys/fs/cgroup/memory" + own_cgroup("memory");
        root = stat(own.c_str(), &st) == 0 ? own : "/sys/fs/cgroup/memory";
      } else {
        why = "no cgroup memory controller";
      }
    } else {
      root = s_.cgroup;
      if (!ver) ver = stat((root + "/cgroup.controllers").c_str(), &st) == 0 ? 2 : 1;
    }
    const uint64_t bytes = (s_.rank_memory_kb + s_.cgroup_headroom_kb) * 1024;
    if (why.empty()) {
      sweep_stale_cgroups(root);
      for (int i = 0; i < s_.parallelism; ++i) {
        const std::string dir = root + "/tpi-" + s_.task_id + "-" + std::to_string(getpid()) +
                                "-r" + std::to_string(i);
        if (mkdir(dir.c_str(), 0755) && errno != EEXIST) {
          why = "mkdir " + dir + ": " + strerror(errno);
          break;
        }
        cg_dirs_[i] = dir;
        const std::string limit = dir + (ver == 2 ? "/memory.max" : "/memory.limit_in_bytes");
        if (!write_text(limit, std::to_string(bytes))) {
          why = "write " + limit + ": " + strerror(errno);
          break;
        }
        if (ver == 2) write_text(dir + "/memory.swap.max", "0");
      }
    }
    if (!why.empty()) {
      for (auto& d : cg_dirs_)
        if (!d.empty()) {
          rmdir(d.c_str());
          d.clear();
        }
      memory_guard_ = "poll " + std::to_string((int)(s_.memory_fast_interval * 1000)) + " ms";
      event_("memory-cgroup-unavailable", {why, "the /proc poll enforces the limit"});
      event_("memory-guard", {memory_guard_, "statm of each rank's process tree",
                             "limit " + std::to_string(s_.rank_memory_kb / 1024) + " MB"});
      return;
    }
    cg_version_ = ver;
    cg_root_ = root;
    memory_guard_ = "cgroup v" + std::to_string(ver);
    event_("memory-cgroup", {"v" + std::to_string(ver), root,
                            "cap " + std::to_string(bytes >> 20) + " MB per rank",
                            "limit " + std::to_string(s_.rank_memory_kb / 1024) + " MB (poll)"});
  }

  uint64_t cgroup_oom_kills(int index) {
    if (index < 0 || index >= (int)cg_dirs_.size() || cg_dirs_[index].empty()) return 0;
    std::ifstream in(cg_dirs_[index] + (cg_version_ == 2 ? "/memory.events" : "/memory.oom_control"));
    std::string key;
    uint64_t value = 0;
    while (in >> key) {
      if (key == "oom_kill" && in >> value) return value;
      in.ignore(1 << 16, '\n');
    }
    return 0;
  }

  void remove_cgroups() {
    for (auto& d : cg_dirs_)
      if (!d.empty()) rmdir(d.c_str());
  }


  // ---- the fast guard (no cgroup) -----------------------------------------------------------
  // Where the kernel cap is refused (an unprivileged box), the limit is only as good as the
  // poll.  Every memory_fast_interval (20 ms) each rank's process tree -- the rank and its
  // descendants, from /proc/<pid>/task/<tid>/children, plus the process-group members of the
  // last full /proc scan (orphans reparented away from the tree) -- is summed from statm
  // (microseconds per process).  The expensive proportional split runs only when that bound,
  // advanced from the last split by the growth of the resident set since, passes the limit.
  struct MemTrack {
    long pid = 0;
    uint64_t rss_at = 0, counted_at = 0;  // resident set and counted PSS at the last split
    bool valid = false;
    std::vector<long> members;  // process-group members seen by the last full scan
  };

  static void tree_pids(long root, std::vector<long>& out, int depth = 0) {
    out.push_back(root);
    if (depth > 16) return;
    char path[64];
    snprintf(path, sizeof(path), "/proc/%ld/task", root);
    DIR* d = opendir(path);
    if (!d) return;
    std::vector<long> kids;
    while (struct dirent* e = readdir(d)) {
      if (e->d_name[0] < '0' || e->d_name[0] > '9') continue;
      char cpath[96], buf[4096];
      snprintf(cpath, sizeof(cpath), "/proc/%ld/task/%s/children", root, e->d_name);
      if (!read_small(cpath, buf, sizeof(buf))) continue;
      char* p = buf;
      while (*p) {
        char* end = nullptr;
        long c = strtol(p, &end, 10);
        if (end == p) break;
        if (c > 0) kids.push_back(c);
        p = end;
      }
    }
    closedir(d);
    for (long c : kids) tree_pids(c, out, depth + 1);
  }

  static uint64_t resident_kb(const std::vector<long>& pids) {
    static const uint64_t page_kb = (uint64_t)sysconf(_SC_PAGESIZE) / 1024;
    uint64_t kb = 0;
    char path[64], buf[256];
    for (long pid : pids) {
      snprintf(path, sizeof(path), "/proc/%ld/statm", pid);
      if (!read_small(path, buf, sizeof(buf))) continue;
      unsigned long long size = 0, resident = 0;
      if (sscanf(buf, "%llu %llu", &size, &resident) == 2) kb += resident * page_kb;
    }
    return kb;
  }


  std::vector<MemTrack> mem_;
};

}  // namespace tpi_sup
