// The off-node container mirror of a task (storage/remote.py + storage/objectstore.py run as
// `sync_argv`): every `sync_interval` s while the ranks run, one at a time, and once more --
// awaited, bounded by `sync_timeout` -- when they are done, so the task is over only once its
// data and reports are in the container.
//
// Reference: the machine script's 10 s data loop and its final copy
// (task/common/machine/machine-script.sh.tpl:118-124).
#pragma once

#include <fcntl.h>
#include <signal.h>
#include <stdio.h>
#include <sys/prctl.h>
#include <sys/types.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "common.h"

namespace tpi_sup {

class ContainerSync {
 public:
  using EventFn = std::function<void(const std::string&, const std::vector<std::string>&)>;

  ContainerSync(const Spec& s, EventFn event) : s_(s), event_(std::move(event)) {}

  bool enabled() const { return !s_.sync_argv.empty(); }
  pid_t pid() const { return pid_; }

  // The periodic mirror: started when due and none is running (the first one interval after
  // the start).
  void check(double t) {
    if (!enabled() || s_.sync_interval <= 0 || pid_ > 0 || t < next_) return;
    if (next_ == 0) {
      next_ = t + s_.sync_interval;
      return;
    }
    next_ = t + s_.sync_interval;
    pid_ = spawn();
  }

  // How long the supervisor's poll may sleep before the next mirror is due.
  double timeout(double t, double current) const {
    if (!enabled() || s_.sync_interval <= 0 || pid_ > 0) return current;
    return std::min(current, next_ - t);
  }

  // The periodic mirror was reaped.
  void exited(int st) {
    pid_ = -1;
    const bool ok = WIFEXITED(st) && WEXITSTATUS(st) == 0;
    if (!ok && ++failures_ <= 5)  // journal the first failures, not every retry
      event_("remote-sync-failed",
             {WIFSIGNALED(st) ? std::string("signal ") + signame(WTERMSIG(st))
                              : "code " + std::to_string(WEXITSTATUS(st)),
              "see " + s_.events_path + ".sync.log"});
  }

  // The final mirror, awaited (after a running periodic one).
  void final() {
    if (!enabled()) return;
    const double t0 = now();
    int st = 0;
    if (pid_ > 0 && waitpid(pid_, &st, 0) == pid_) exited(st);
    pid_t pid = spawn();
    if (pid <= 0) {
      event_("remote-sync-failed", {"fork failed"});
      return;
    }
    pid_t got = 0;
    while ((got = waitpid(pid, &st, WNOHANG)) == 0 && now() - t0 < s_.sync_timeout) usleep(5000);
    if (got == 0) {
      kill(-pid, SIGKILL);
      kill(pid, SIGKILL);
      waitpid(pid, &st, 0);
    }
    char took[48];
    snprintf(took, sizeof(took), "%.3f s", now() - t0);
    const bool ok = got == pid && WIFEXITED(st) && WEXITSTATUS(st) == 0;
    event_(ok ? "remote-synced" : "remote-sync-failed",
           {ok ? "final" : (got == 0 ? "final: timed out" : "final"), took});
  }

 private:
  // The mirror command in a process group of its own, stdout discarded, stderr to
  // <events>.sync.log; it dies with the supervisor.
  pid_t spawn() {
    std::vector<char*> argv;
    for (auto& a : s_.sync_argv) argv.push_back(const_cast<char*>(a.c_str()));
    argv.push_back(nullptr);
    int logfd = open((s_.events_path + ".sync.log").c_str(),
                     O_WRONLY | O_CREAT | O_APPEND | O_CLOEXEC, 0644);
    pid_t parent = getpid();
    pid_t pid = fork();
    if (pid == 0) {
      setpgid(0, 0);
      prctl(PR_SET_PDEATHSIG, SIGTERM);
      if (getppid() != parent) _exit(127);
      sigset_t none;
      sigemptyset(&none);
      sigprocmask(SIG_SETMASK, &none, nullptr);
      int devnull = open("/dev/null", O_RDWR);
      if (devnull >= 0) {
        dup2(devnull, 0);
        dup2(devnull, 1);
      }
      if (logfd >= 0) dup2(logfd, 2);
      execv(argv[0], argv.data());
      _exit(127);
    }
    if (logfd >= 0) close(logfd);
    return pid;
  }

  const Spec& s_;
  EventFn event_;
  pid_t pid_ = -1;
  double next_ = 0;
  int failures_ = 0;
};

}  // namespace tpi_sup
