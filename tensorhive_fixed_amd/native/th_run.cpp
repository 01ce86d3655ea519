// th-run: the task supervisor that replaces GNU `screen` for tensorhive_fixed_amd.
//
// Reference behaviour being replaced (tensorhive/core/task_nursery.py:47-152): tasks were run as
//   screen -Dm -S tensorhive_task_<id> bash -c "<cmd> |& tee --ignore-interrupts <log>" & echo $!
// and controlled with `screen -X stuff ^C` / `screen -X quit` / `kill -9` / `screen -ls`.
//
//   th-run spawn --name NAME --log FILE [--state-dir DIR] [--env K=V]... [--cwd DIR]
//                [--max-restarts N] [--restart-delay S] [--notify SOCK] -- CMD ARGS...
//       Detaches (double fork + setsid), starts CMD in its OWN process group with stdout+stderr
//       on a pipe, and prints the pid of CMD (== its pgid) on stdout, then returns.  A small
//       monitor process (own session, ignores SIGINT/SIGTERM/SIGHUP like `tee --ignore-interrupts`)
//       copies the pipe into FILE line by line, reaps CMD and records its exit status.  With
//       --max-restarts N a run that exits non-zero is started again (new pid/pgid, same log,
//       TH_RUN_RESTART=k in its env) up to N times, unless the stop was requested through th-run
//       (SURVEY §5 failure row: restart policy; the reference only detects failures).  With
//       --notify SOCK (or $TH_RUN_NOTIFY) the monitor sends one datagram to that unix socket when
//       the task has exited and its state says so: the daemon's scheduler wakes on the event
//       instead of discovering the exit by polling (core/events.py).
//   th-run interrupt|terminate|kill (--name NAME | --pid PID) [--state-dir DIR]
//       SIGINT / SIGTERM / SIGKILL to the task's whole process group (torchrun + all ranks).
//   th-run ls [--all] [--state-dir DIR]     one JSON object per session (live ones by default)
//   th-run status --name NAME               JSON of one session
//   th-run wait --name NAME [--timeout S]   block until the task exits; exit code = task's
//
// State: one `NAME.state` key=value file per session in the state dir (default
// $TH_RUN_STATE_DIR or ~/.local/state/tensorhive/th-run), written atomically (rename).  These
// files are the durable PID truth the daemon re-adopts after a restart.  They also carry the
// session id, uid and user the task runs as: the daemon accepts a GPU process's
// TENSORHIVE_TASK_ID only when the process is in that session (or descends from the monitor)
// and runs as that uid (core/attribution.py).
#include <dirent.h>
#include <errno.h>
#include <fcntl.h>
#include <pwd.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/types.h>
#include <sys/un.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <map>
#include <string>
#include <vector>

namespace {

std::string state_dir_default() {
  const char* e = getenv("TH_RUN_STATE_DIR");
  if (e && *e) return e;
  const char* home = getenv("HOME");
  return std::string(home ? home : "/tmp") + "/.local/state/tensorhive/th-run";
}

int mkdirs(const std::string& path) {
  std::string cur;
  for (size_t i = 0; i < path.size(); ++i) {
    cur += path[i];
    if ((path[i] == '/' && i > 0) || i + 1 == path.size()) {
      if (mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return -1;
    }
  }
  return 0;
}

std::string dirname_of(const std::string& p) {
  size_t k = p.rfind('/');
  return k == std::string::npos ? "." : (k == 0 ? "/" : p.substr(0, k));
}

std::string stop_marker(const std::string& dir, const std::string& name) { return dir + "/" + name + ".stop"; }

std::string expand_home(const std::string& p) {
  if (!p.empty() && p[0] == '~') {
    const char* home = getenv("HOME");
    return std::string(home ? home : "") + p.substr(1);
  }
  return p;
}

typedef std::map<std::string, std::string> KV;

bool write_state(const std::string& dir, const std::string& name, const KV& kv) {
  std::string path = dir + "/" + name + ".state";
  std::string tmp = path + ".tmp." + std::to_string(getpid());
  FILE* f = fopen(tmp.c_str(), "w");
  if (!f) return false;
  for (const auto& it : kv) fprintf(f, "%s=%s\n", it.first.c_str(), it.second.c_str());
  fflush(f);
  fsync(fileno(f));
  fclose(f);
  return rename(tmp.c_str(), path.c_str()) == 0;
}

bool read_state(const std::string& path, KV& kv) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return false;
  char line[8192];
  while (fgets(line, sizeof line, f)) {
    char* eq = strchr(line, '=');
    if (!eq) continue;
    *eq = 0;
    std::string v(eq + 1);
    while (!v.empty() && (v.back() == '\n' || v.back() == '\r')) v.pop_back();
    kv[line] = v;
  }
  fclose(f);
  return true;
}

std::string json_escape(const std::string& s) {
  std::string o;
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\n': o += "\\n"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20) {
          char b[8];
          snprintf(b, sizeof b, "\\u%04x", c);
          o += b;
        } else {
          o += (char)c;
        }
    }
  }
  return o;
}

bool pid_alive(long pid) {
  if (pid <= 0) return false;
  if (kill((pid_t)pid, 0) == 0) return true;
  return errno == EPERM;
}

// Live = the task runs, or it is between a failed run and its restart (monitor alive).
bool session_alive(KV& kv) {
  if (kv["status"] == "running") return pid_alive(atol(kv["pid"].c_str()));
  if (kv["status"] == "restarting") return pid_alive(atol(kv["monitor_pid"].c_str()));
  return false;
}

std::string to_json(const KV& kv, bool alive) {
  std::string o = "{";
  bool first = true;
  for (const auto& it : kv) {
    if (!first) o += ",";
    first = false;
    const bool num = it.first == "pid" || it.first == "pgid" || it.first == "monitor_pid" ||
                     it.first == "exit_code" || it.first == "started" || it.first == "ended" ||
                     it.first == "first_pid" || it.first == "restarts" || it.first == "max_restarts" ||
                     it.first == "last_exit_code" || it.first == "sid" || it.first == "uid" ||
                     it.first == "ended_ms";
    o += "\"" + json_escape(it.first) + "\":";
    if (num && !it.second.empty())
      o += it.second;
    else
      o += "\"" + json_escape(it.second) + "\"";
  }
  o += std::string(first ? "" : ",") + "\"alive\":" + (alive ? "true" : "false") + "}";
  return o;
}

long long now_ms() {
  struct timespec t;
  clock_gettime(CLOCK_REALTIME, &t);
  return (long long)t.tv_sec * 1000 + t.tv_nsec / 1000000;
}

// Task-exit event: one datagram to the daemon's (or the node agent's) unix socket, sent after the
// state file says `exited`, so whoever wakes on it reads the final state (core/events.py).  A hint
// only: a missing or full socket loses nothing but latency (the daemon still polls).
void notify_event(const std::string& path, const KV& st) {
  if (path.empty() || path.size() >= sizeof(((struct sockaddr_un*)nullptr)->sun_path)) return;
  int fd = socket(AF_UNIX, SOCK_DGRAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return;
  struct sockaddr_un a;
  memset(&a, 0, sizeof a);
  a.sun_family = AF_UNIX;
  memcpy(a.sun_path, path.c_str(), path.size());
  std::string msg = "{\"event\":\"task_exit\"";
  for (const char* k : {"name", "pid", "exit_code", "restarts", "ended_ms", "user"}) {
    auto it = st.find(k);
    if (it == st.end()) continue;
    const bool num = strcmp(k, "name") != 0 && strcmp(k, "user") != 0;
    msg += std::string(",\"") + k + "\":" + (num ? it->second : "\"" + json_escape(it->second) + "\"");
  }
  msg += "}";
  (void)sendto(fd, msg.data(), msg.size(), MSG_DONTWAIT, (struct sockaddr*)&a, sizeof a);
  close(fd);
}

void write_all(int fd, const char* p, ssize_t n) {
  while (n > 0) {
    ssize_t w = write(fd, p, (size_t)n);
    if (w < 0) {
      if (errno == EINTR) continue;
      return;
    }
    p += w;
    n -= w;
  }
}

int usage() {
  fprintf(stderr,
          "usage: th-run spawn --name NAME --log FILE [--state-dir D] [--env K=V].. [--cwd D]\n"
          "                    [--max-restarts N] [--restart-delay S] [--notify SOCK] -- CMD..\n"
          "       th-run interrupt|terminate|kill (--name NAME | --pid PID) [--state-dir D]\n"
          "       th-run ls [--all] [--state-dir D] | status --name NAME | wait --name NAME [--timeout S]\n");
  return 2;
}

struct Args {
  std::string cmd, name, log, state_dir, cwd, notify;
  long pid = -1;
  double timeout = -1, restart_delay = 1.0;
  int max_restarts = 0;
  bool all = false;
  std::vector<std::string> env;
  std::vector<std::string> argv;
};

bool parse(int argc, char** argv, Args& a) {
  if (argc < 2) return false;
  a.cmd = argv[1];
  a.state_dir = state_dir_default();
  if (const char* n = getenv("TH_RUN_NOTIFY")) a.notify = n;
  for (int i = 2; i < argc; ++i) {
    std::string s = argv[i];
    auto need = [&](std::string& dst) {
      if (i + 1 >= argc) return false;
      dst = argv[++i];
      return true;
    };
    if (s == "--") {
      for (int j = i + 1; j < argc; ++j) a.argv.push_back(argv[j]);
      break;
    } else if (s == "--name") {
      if (!need(a.name)) return false;
    } else if (s == "--log") {
      if (!need(a.log)) return false;
    } else if (s == "--state-dir") {
      if (!need(a.state_dir)) return false;
    } else if (s == "--cwd") {
      if (!need(a.cwd)) return false;
    } else if (s == "--notify") {
      if (!need(a.notify)) return false;
    } else if (s == "--env") {
      std::string e;
      if (!need(e)) return false;
      a.env.push_back(e);
    } else if (s == "--pid") {
      std::string p;
      if (!need(p)) return false;
      a.pid = atol(p.c_str());
    } else if (s == "--timeout") {
      std::string t;
      if (!need(t)) return false;
      a.timeout = atof(t.c_str());
    } else if (s == "--max-restarts") {
      std::string t;
      if (!need(t)) return false;
      a.max_restarts = atoi(t.c_str());
    } else if (s == "--restart-delay") {
      std::string t;
      if (!need(t)) return false;
      a.restart_delay = atof(t.c_str());
    } else if (s == "--all") {
      a.all = true;
    } else {
      return false;
    }
  }
  a.state_dir = expand_home(a.state_dir);
  a.log = expand_home(a.log);
  return true;
}

// ------------------------------------------------------------------------------- spawn
int do_spawn(Args& a) {
  if (a.name.empty() || a.log.empty() || a.argv.empty()) return usage();
  if (mkdirs(a.state_dir) != 0 || mkdirs(dirname_of(a.log)) != 0) {
    perror("th-run: mkdir");
    return 1;
  }
  int hs[2];  // handshake: grandchild command pid back to the caller
  if (pipe(hs) != 0) return 1;
  pid_t p1 = fork();
  if (p1 < 0) return 1;
  if (p1 > 0) {  // caller: read the command pid, print it, done
    close(hs[1]);
    long cpid = -1;
    ssize_t n = read(hs[0], &cpid, sizeof cpid);
    close(hs[0]);
    waitpid(p1, nullptr, 0);
    if (n != (ssize_t)sizeof cpid || cpid <= 0) {
      fprintf(stderr, "th-run: spawn failed\n");
      return 1;
    }
    printf("%ld\n", cpid);
    fflush(stdout);
    return 0;
  }
  // first child -> new session, then fork the monitor so it is not a session leader's child
  close(hs[0]);
  setsid();
  pid_t p2 = fork();
  if (p2 < 0) _exit(1);
  if (p2 > 0) _exit(0);
  // monitor process.  INT/TERM/HUP are BLOCKED across every fork below: the task child resets
  // them to SIG_DFL before unblocking (a signal sent the moment its pid is known is then delivered
  // with the default action instead of being lost to an inherited SIG_IGN); the monitor ignores them.
  sigset_t guard, prev;
  sigemptyset(&guard);
  sigaddset(&guard, SIGINT);
  sigaddset(&guard, SIGTERM);
  sigaddset(&guard, SIGHUP);
  signal(SIGPIPE, SIG_IGN);
  int logfd = open(a.log.c_str(), O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (logfd < 0) _exit(1);
  const std::string stopf = stop_marker(a.state_dir, a.name);
  unlink(stopf.c_str());  // a fresh session: no stop request yet
  KV st;
  st["name"] = a.name;
  st["monitor_pid"] = std::to_string((long)getpid());
  st["started"] = std::to_string((long)time(nullptr));
  st["log"] = a.log;
  std::string cmdline;
  for (auto& s : a.argv) cmdline += (cmdline.empty() ? "" : " ") + s;
  st["cmd"] = cmdline;
  st["max_restarts"] = std::to_string(a.max_restarts);
  if (!a.notify.empty()) st["notify"] = a.notify;
  // Attestation of the task's processes (core/attribution.py): every process the task starts is
  // in THIS session (the first child's setsid above) unless it calls setsid itself, and then its
  // parent chain still reaches this monitor.  Neither can be joined by a process started outside
  // the session, whatever it puts in its environment; the uid says who the task runs as.
  st["sid"] = std::to_string((long)getsid(0));
  st["uid"] = std::to_string((long)getuid());
  {
    struct passwd pw, *res = nullptr;
    char pbuf[4096];
    if (getpwuid_r(getuid(), &pw, pbuf, sizeof pbuf, &res) == 0 && res) st["user"] = res->pw_name;
  }
  int restarts = 0, code = -1;
  for (;;) {
    sigprocmask(SIG_BLOCK, &guard, &prev);
    int out[2];
    if (pipe(out) != 0) _exit(1);
    pid_t c = fork();
    if (c < 0) _exit(1);
    if (c == 0) {  // the task: own process group, default signal dispositions
      setpgid(0, 0);
      signal(SIGINT, SIG_DFL);
      signal(SIGTERM, SIG_DFL);
      signal(SIGHUP, SIG_DFL);
      signal(SIGPIPE, SIG_DFL);
      sigprocmask(SIG_SETMASK, &prev, nullptr);
      dup2(out[1], 1);
      dup2(out[1], 2);
      close(out[0]);
      close(out[1]);
      close(logfd);
      if (restarts == 0) close(hs[1]);
      int devnull = open("/dev/null", O_RDONLY);
      if (devnull >= 0) {
        dup2(devnull, 0);
        close(devnull);
      }
      for (const auto& e : a.env) putenv(strdup(e.c_str()));
      putenv(strdup(("TH_RUN_RESTART=" + std::to_string(restarts)).c_str()));
      if (!a.cwd.empty() && chdir(expand_home(a.cwd).c_str()) != 0) perror("th-run: chdir");
      std::vector<char*> av;
      for (auto& s : a.argv) av.push_back(const_cast<char*>(s.c_str()));
      av.push_back(nullptr);
      execvp(av[0], av.data());
      fprintf(stderr, "th-run: exec %s: %s\n", av[0], strerror(errno));
      _exit(127);
    }
    setpgid(c, c);  // race-free: both sides set it
    signal(SIGINT, SIG_IGN);
    signal(SIGTERM, SIG_IGN);
    signal(SIGHUP, SIG_IGN);
    sigprocmask(SIG_SETMASK, &prev, nullptr);
    close(out[1]);
    st["pid"] = std::to_string((long)c);
    st["pgid"] = std::to_string((long)c);
    if (restarts == 0) st["first_pid"] = std::to_string((long)c);
    // every incarnation's pid, so a caller holding ANY of them still finds the session
    st["pids"] += (st["pids"].empty() ? "" : ",") + std::to_string((long)c);
    st["restarts"] = std::to_string(restarts);
    st["status"] = "running";
    write_state(a.state_dir, a.name, st);
    // A stop requested while this run was being started (after the restart loop's last check)
    // found no live process group; honour it now so a stopped task never runs to completion.
    if (restarts > 0 && access(stopf.c_str(), F_OK) == 0) kill(-c, SIGTERM);
    if (restarts == 0) {
      long cpid = (long)c;
      write_all(hs[1], (const char*)&cpid, sizeof cpid);
      close(hs[1]);
      int devnull = open("/dev/null", O_RDWR);
      if (devnull >= 0) {
        dup2(devnull, 0);
        dup2(devnull, 1);
        dup2(devnull, 2);
        close(devnull);
      }
    }
    char buf[65536];
    for (;;) {
      ssize_t n = read(out[0], buf, sizeof buf);
      if (n < 0 && errno == EINTR) continue;
      if (n <= 0) break;
      write_all(logfd, buf, n);
    }
    close(out[0]);
    int wst = 0;
    while (waitpid(c, &wst, 0) < 0 && errno == EINTR) {
    }
    code = WIFEXITED(wst) ? WEXITSTATUS(wst) : (WIFSIGNALED(wst) ? 128 + WTERMSIG(wst) : -1);
    // Restart policy: a failed run is restarted up to --max-restarts times, unless the exit was
    // requested (interrupt/terminate/kill through th-run leave a stop marker first).
    if (code == 0 || restarts >= a.max_restarts || access(stopf.c_str(), F_OK) == 0) break;
    ++restarts;
    char note[256];
    const int k = snprintf(note, sizeof note, "[th-run] exit code %d; restart %d/%d in %.1f s\n", code, restarts,
                           a.max_restarts, a.restart_delay);
    write_all(logfd, note, k);
    st["status"] = "restarting";
    st["last_exit_code"] = std::to_string(code);
    write_state(a.state_dir, a.name, st);
    bool stop = false;
    for (double w = 0; w < a.restart_delay && !stop; w += 0.05) {
      usleep(50000);
      stop = access(stopf.c_str(), F_OK) == 0;
    }
    if (stop) break;
  }
  st["status"] = "exited";
  st["exit_code"] = std::to_string(code);
  st["restarts"] = std::to_string(restarts);
  st["ended"] = std::to_string((long)time(nullptr));
  st["ended_ms"] = std::to_string(now_ms());
  write_state(a.state_dir, a.name, st);
  notify_event(a.notify, st);
  unlink(stopf.c_str());
  close(logfd);
  _exit(0);
}

bool lookup(const Args& a, KV& kv) {
  if (a.name.empty()) return false;
  return read_state(a.state_dir + "/" + a.name + ".state", kv);
}

bool pid_in_history(KV& kv, long pid) {
  if (atol(kv["pgid"].c_str()) == pid || atol(kv["first_pid"].c_str()) == pid) return true;
  const std::string& h = kv["pids"];
  size_t i = 0;
  while (i < h.size()) {
    size_t j = h.find(',', i);
    if (j == std::string::npos) j = h.size();
    if (atol(h.substr(i, j - i).c_str()) == pid) return true;
    i = j + 1;
  }
  return false;
}

// Name of the live session that has ever run as `pid` ("" if none).
std::string session_of_pid(const std::string& dir, long pid) {
  DIR* d = opendir(dir.c_str());
  if (!d) return "";
  std::string found;
  struct dirent* e;
  while ((e = readdir(d)) != nullptr && found.empty()) {
    std::string n = e->d_name;
    if (n.size() < 7 || n.substr(n.size() - 6) != ".state") continue;
    KV kv;
    if (read_state(dir + "/" + n, kv) && kv["status"] != "exited" && pid_in_history(kv, pid)) found = kv["name"];
  }
  closedir(d);
  return found;
}

int do_signal(const Args& a, int sig) {
  long pg = a.pid;
  std::string name = a.name;
  bool restarting = false;
  if (pg <= 0) {
    KV kv;
    if (!lookup(a, kv)) {
      fprintf(stderr, "th-run: no session %s\n", a.name.c_str());
      return 3;
    }
    if (kv["status"] == "exited") return 4;
    pg = atol(kv["pgid"].c_str());
    restarting = kv["status"] == "restarting";
  } else {
    name = session_of_pid(a.state_dir, pg);
    if (!name.empty()) {  // signal the current incarnation of a restarted task
      KV kv;
      if (read_state(a.state_dir + "/" + name + ".state", kv)) {
        pg = atol(kv["pgid"].c_str());
        restarting = kv["status"] == "restarting";
      }
    }
  }
  if (!name.empty()) {  // a requested stop is never undone by the restart policy
    FILE* f = fopen(stop_marker(a.state_dir, name).c_str(), "w");
    if (f) fclose(f);
  }
  if (pg <= 0) return 3;
  if (kill(-(pid_t)pg, sig) != 0 && kill((pid_t)pg, sig) != 0) {
    // Between a failed run and its restart there is no process to signal: the stop marker
    // written above already keeps the next run from starting, so the request succeeded.
    if (errno == ESRCH && restarting) return 0;
    perror("th-run: kill");
    return 1;
  }
  return 0;
}

int do_ls(const Args& a) {
  DIR* d = opendir(a.state_dir.c_str());
  if (!d) return 0;
  struct dirent* e;
  while ((e = readdir(d)) != nullptr) {
    std::string n = e->d_name;
    if (n.size() < 7 || n.substr(n.size() - 6) != ".state") continue;
    KV kv;
    if (!read_state(a.state_dir + "/" + n, kv)) continue;
    const bool alive = session_alive(kv);
    if (!alive && !a.all) continue;
    printf("%s\n", to_json(kv, alive).c_str());
  }
  closedir(d);
  return 0;
}

int do_status(const Args& a) {
  KV kv;
  if (!lookup(a, kv)) return 3;
  printf("%s\n", to_json(kv, session_alive(kv)).c_str());
  return 0;
}

int do_wait(const Args& a) {
  struct timespec t0;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (;;) {
    KV kv;
    if (!lookup(a, kv)) return 3;
    if (kv["status"] == "exited") return atoi(kv["exit_code"].c_str());
    if (!pid_alive(atol(kv["pid"].c_str())) && !pid_alive(atol(kv["monitor_pid"].c_str()))) return 137;
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    const double el = (t.tv_sec - t0.tv_sec) + 1e-9 * (t.tv_nsec - t0.tv_nsec);
    if (a.timeout >= 0 && el > a.timeout) return 124;
    usleep(20000);
  }
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  if (!parse(argc, argv, a)) return usage();
  if (a.cmd == "spawn") return do_spawn(a);
  if (a.cmd == "interrupt") return do_signal(a, SIGINT);
  if (a.cmd == "terminate") return do_signal(a, SIGTERM);
  if (a.cmd == "kill") return do_signal(a, SIGKILL);
  if (a.cmd == "ls") return do_ls(a);
  if (a.cmd == "status") return do_status(a);
  if (a.cmd == "wait") return do_wait(a);
  return usage();
}
