// Host-side self test of the native runtime (tony_native.cpp), built with AddressSanitizer +
// UndefinedBehaviorSanitizer by `make asan` (the reference ran findbugs; this is
// the native-code counterpart).  Exercises every entry point that runs without a GPU: gang spawn
// with stdout/stderr redirection and a new session, process-group kill, port reservation with and
// without SO_REUSEPORT, and the amd-smi probe (which must fail cleanly when no GPU / amd-smi is there).
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

extern "C" {
int tony_spawn(char* const argv[], char* const envp[], const char* cwd, const char* out_path, const char* err_path,
               int new_session, int* pid_out);
int tony_kill_tree(int pgid, int sig);
int tony_reserve_port(int port, int reuse_port, int* fd_out);
int tony_release_port(int fd);
int tony_smi_init(void);
void tony_smi_shutdown(void);
}

static int failures = 0;
#define CHECK(cond)                                                       \
  do {                                                                    \
    if (!(cond)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                         \
    }                                                                     \
  } while (0)

static std::string slurp(const std::string& path) {
  std::ifstream f(path);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

int main() {
  char tmpl[] = "/tmp/tony_native_selftestXXXXXX";
  const char* dir = mkdtemp(tmpl);
  CHECK(dir != nullptr);
  const std::string out = std::string(dir) + "/out", err = std::string(dir) + "/err";
  // spawn: a shell that writes to both streams and reports its session id == pid
  {
    char a0[] = "/bin/sh", a1[] = "-c", a2[] = "echo hello; echo oops 1>&2; echo $TONY_X; ps -o sid= -p $$";
    char* argv[] = {a0, a1, a2, nullptr};
    char e0[] = "TONY_X=env-ok", e1[] = "PATH=/usr/bin:/bin";
    char* envp[] = {e0, e1, nullptr};
    int pid = -1;
    CHECK(tony_spawn(argv, envp, dir, out.c_str(), err.c_str(), 1, &pid) == 0);
    CHECK(pid > 0);
    int st = 0;
    CHECK(waitpid(pid, &st, 0) == pid);
    CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);
    const std::string o = slurp(out);
    CHECK(o.find("hello") != std::string::npos && o.find("env-ok") != std::string::npos);
    CHECK(o.find(std::to_string(pid)) != std::string::npos);  // its own session
    CHECK(slurp(err).find("oops") != std::string::npos);
  }
  // spawn of a missing program fails with an errno, never crashes
  {
    char a0[] = "/nonexistent/tony-binary";
    char* argv[] = {a0, nullptr};
    char* envp[] = {nullptr};
    int pid = -1;
    CHECK(tony_spawn(argv, envp, nullptr, nullptr, nullptr, 1, &pid) < 0 || (pid > 0 && waitpid(pid, nullptr, 0)));
  }
  // kill_tree: a sleeping process group dies with SIGKILL
  {
    char a0[] = "/bin/sh", a1[] = "-c", a2[] = "sleep 30 & sleep 30";
    char* argv[] = {a0, a1, a2, nullptr};
    char e1[] = "PATH=/usr/bin:/bin";
    char* envp[] = {e1, nullptr};
    int pid = -1;
    CHECK(tony_spawn(argv, envp, nullptr, nullptr, nullptr, 1, &pid) == 0);
    usleep(100000);
    CHECK(tony_kill_tree(pid, SIGKILL) == 0);
    int st = 0;
    CHECK(waitpid(pid, &st, 0) == pid && WIFSIGNALED(st));
    CHECK(tony_kill_tree(1, SIGKILL) < 0);  // refuses init / whole-session kills
  }
  // ports: an ephemeral port, then two SO_REUSEPORT holders of the same port
  {
    int fd = -1;
    const int port = tony_reserve_port(0, 0, &fd);
    CHECK(port > 0 && fd >= 0);
    CHECK(tony_release_port(fd) == 0);
    int f1 = -1, f2 = -1;
    const int p1 = tony_reserve_port(0, 1, &f1);
    CHECK(p1 > 0);
    CHECK(tony_reserve_port(p1, 1, &f2) == p1);
    CHECK(tony_release_port(f1) == 0 && tony_release_port(f2) == 0);
    CHECK(tony_release_port(-1) < 0);
  }
  // amd-smi: whatever the machine, init/shutdown must be clean (idempotent shutdown)
  {
    const int n = tony_smi_init();
    std::printf("amd-smi devices: %d\n", n);
    tony_smi_shutdown();
    tony_smi_shutdown();
  }
  std::printf(failures ? "native selftest: %d FAILURE(S)\n" : "native selftest: ok\n", failures);
  return failures ? 1 : 0;
}
