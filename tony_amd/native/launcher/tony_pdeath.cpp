// tony_pdeath: exec a command that dies with the process that started it.
//
//   tony_pdeath <parent-pid> <argv...>
//
// The task agent (agent/executor.py) runs gRPC threads; forking it to run Python code between fork
// and exec (subprocess's preexec_fn) runs gRPC's at-fork handlers in the child, which can abort it.
// Instead the agent starts this helper with a plain fork/exec (vfork path, no Python in the child):
// it arms PR_SET_PDEATHSIG, re-checks that the agent is still alive (it may have died before the
// signal was armed) and execs the user command in place.
#include <sys/prctl.h>
#include <unistd.h>

#include <csignal>
#include <cstdio>
#include <cstdlib>

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <parent-pid> <command> [args...]\n", argv[0]);
    return 2;
  }
  const long parent = std::strtol(argv[1], nullptr, 10);
  if (prctl(PR_SET_PDEATHSIG, SIGKILL) != 0) {
    std::perror("prctl(PR_SET_PDEATHSIG)");
    return 2;
  }
  if (parent > 0 && getppid() != static_cast<pid_t>(parent)) return 137;  // the agent is already gone
  execvp(argv[2], argv + 2);
  std::perror("execvp");
  return 127;
}
