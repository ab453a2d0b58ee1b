// tony_amd native host runtime: the pieces of TonY's NodeManager / TaskExecutor /
// GpuDiscoverer that sit on the OS and driver boundary, as one small C ABI
// library loaded by ctypes (tony_amd/native/__init__.py).
//
//  * tony_spawn        posix_spawn a task agent in its own session (so the whole
//                      task tree is one process group), stdout/stderr redirected
//                      to per-task log files, working dir set -- the "container
//                      launch" of T/ApplicationMaster.java:1154-1222 on one node.
//  * tony_kill_tree    signal a process group (TonY stops containers with a 15 s
//                      grace, T/ApplicationMaster.java:760-777).
//  * tony_reserve_port bind a TCP port (optionally SO_REUSEPORT) and keep the fd:
//                      the task's advertised host:port (T/ReusablePort.java,
//                      TR/reserve_reusable_port.py).
//  * tony_smi_*        GPU inventory and sampling through amd-smi (libamd_smi.so,
//                      dlopen'd): the MI355X replacement of the nvidia-smi XML
//                      parser (T/util/gpu/GpuDiscoverer.java:43-209) -- BDF, UUID,
//                      NUMA node, VRAM, busy %, power, temperature, xGMI links.
#include <amd_smi/amdsmi.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <signal.h>
#include <spawn.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/types.h>
#include <unistd.h>

#include <mutex>
#include <vector>

#define API extern "C" __attribute__((visibility("default")))

// ---------------------------------------------------------------- processes --
API int tony_spawn(char* const argv[], char* const envp[], const char* cwd, const char* out_path,
                   const char* err_path, int new_session, int* pid_out) {
  posix_spawn_file_actions_t fa;
  posix_spawnattr_t attr;
  if (posix_spawn_file_actions_init(&fa) != 0) return -errno;
  posix_spawnattr_init(&attr);
  short flags = POSIX_SPAWN_SETSIGMASK | POSIX_SPAWN_SETSIGDEF;
#ifdef POSIX_SPAWN_SETSID
  if (new_session) flags |= POSIX_SPAWN_SETSID;
#else
  if (new_session) flags |= POSIX_SPAWN_SETPGROUP;  // pgid = pid
#endif
  posix_spawnattr_setflags(&attr, flags);
  sigset_t empty, all;
  sigemptyset(&empty);
  sigfillset(&all);
  posix_spawnattr_setsigmask(&attr, &empty);
  posix_spawnattr_setsigdefault(&attr, &all);
  int rc = 0;
  if (out_path && *out_path)
    rc |= posix_spawn_file_actions_addopen(&fa, 1, out_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
  if (err_path && *err_path)
    rc |= posix_spawn_file_actions_addopen(&fa, 2, err_path, O_WRONLY | O_CREAT | O_APPEND, 0644);
  rc |= posix_spawn_file_actions_addopen(&fa, 0, "/dev/null", O_RDONLY, 0);
  if (cwd && *cwd) rc |= posix_spawn_file_actions_addchdir_np(&fa, cwd);
  pid_t pid = -1;
  if (rc == 0) rc = posix_spawnp(&pid, argv[0], &fa, &attr, argv, envp);
  posix_spawn_file_actions_destroy(&fa);
  posix_spawnattr_destroy(&attr);
  if (rc != 0) return -rc;
  *pid_out = pid;
  return 0;
}

API int tony_kill_tree(int pgid, int sig) {
  if (pgid <= 1) return -EINVAL;
  if (kill(-pgid, sig) != 0) return -errno;
  return 0;
}

// -------------------------------------------------------------------- ports --
// Returns the bound port (>0) and the listening fd, or -errno.
API int tony_reserve_port(int port, int reuse_port, int* fd_out) {
  int fd = socket(AF_INET, SOCK_STREAM | SOCK_CLOEXEC, 0);
  if (fd < 0) return -errno;
  int one = 1;
  setsockopt(fd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  if (reuse_port && setsockopt(fd, SOL_SOCKET, SO_REUSEPORT, &one, sizeof(one)) != 0) {
    int e = errno;
    close(fd);
    return -e;
  }
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_ANY);
  a.sin_port = htons(static_cast<uint16_t>(port));
  if (bind(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || listen(fd, 16) != 0) {
    int e = errno;
    close(fd);
    return -e;
  }
  socklen_t len = sizeof(a);
  getsockname(fd, reinterpret_cast<sockaddr*>(&a), &len);
  *fd_out = fd;
  return ntohs(a.sin_port);
}

API int tony_release_port(int fd) { return close(fd) == 0 ? 0 : -errno; }

// ------------------------------------------------------------------- amd-smi --
namespace {

struct Smi {
  void* h = nullptr;
  decltype(&amdsmi_init) init = nullptr;
  decltype(&amdsmi_shut_down) shut_down = nullptr;
  decltype(&amdsmi_get_socket_handles) sockets = nullptr;
  decltype(&amdsmi_get_processor_handles) processors = nullptr;
  decltype(&amdsmi_get_processor_type) ptype = nullptr;
  decltype(&amdsmi_get_gpu_device_bdf) bdf = nullptr;
  decltype(&amdsmi_get_gpu_device_uuid) uuid = nullptr;
  decltype(&amdsmi_topo_get_numa_node_number) numa = nullptr;
  decltype(&amdsmi_get_gpu_vram_usage) vram = nullptr;
  decltype(&amdsmi_get_gpu_activity) activity = nullptr;
  decltype(&amdsmi_get_power_info) power = nullptr;
  decltype(&amdsmi_get_temp_metric) temp = nullptr;
  decltype(&amdsmi_topo_get_link_type) link_type = nullptr;
  decltype(&amdsmi_get_gpu_total_ecc_count) ecc = nullptr;
  decltype(&amdsmi_get_gpu_metrics_info) metrics = nullptr;
  std::vector<amdsmi_processor_handle> gpus;
  bool ready = false;
};

Smi g_smi;
std::mutex g_smi_mu;

template <typename T>
void sym(void* h, const char* name, T& out) {
  out = reinterpret_cast<T>(dlsym(h, name));
}

}  // namespace

API int tony_smi_init(void) {
  std::lock_guard<std::mutex> lk(g_smi_mu);
  if (g_smi.ready) return static_cast<int>(g_smi.gpus.size());
  const char* names[] = {"libamd_smi.so", "libamd_smi.so.26", "/opt/rocm/lib/libamd_smi.so"};
  for (const char* n : names) {
    g_smi.h = dlopen(n, RTLD_NOW | RTLD_LOCAL);
    if (g_smi.h) break;
  }
  if (!g_smi.h) return -1;
  sym(g_smi.h, "amdsmi_init", g_smi.init);
  sym(g_smi.h, "amdsmi_shut_down", g_smi.shut_down);
  sym(g_smi.h, "amdsmi_get_socket_handles", g_smi.sockets);
  sym(g_smi.h, "amdsmi_get_processor_handles", g_smi.processors);
  sym(g_smi.h, "amdsmi_get_processor_type", g_smi.ptype);
  sym(g_smi.h, "amdsmi_get_gpu_device_bdf", g_smi.bdf);
  sym(g_smi.h, "amdsmi_get_gpu_device_uuid", g_smi.uuid);
  sym(g_smi.h, "amdsmi_topo_get_numa_node_number", g_smi.numa);
  sym(g_smi.h, "amdsmi_get_gpu_vram_usage", g_smi.vram);
  sym(g_smi.h, "amdsmi_get_gpu_activity", g_smi.activity);
  sym(g_smi.h, "amdsmi_get_power_info", g_smi.power);
  sym(g_smi.h, "amdsmi_get_temp_metric", g_smi.temp);
  sym(g_smi.h, "amdsmi_topo_get_link_type", g_smi.link_type);
  sym(g_smi.h, "amdsmi_get_gpu_total_ecc_count", g_smi.ecc);
  sym(g_smi.h, "amdsmi_get_gpu_metrics_info", g_smi.metrics);
  if (!g_smi.init || !g_smi.sockets || !g_smi.processors) return -2;
  if (g_smi.init(AMDSMI_INIT_AMD_GPUS) != AMDSMI_STATUS_SUCCESS) return -3;
  uint32_t ns = 0;
  if (g_smi.sockets(&ns, nullptr) != AMDSMI_STATUS_SUCCESS) return -4;
  std::vector<amdsmi_socket_handle> socks(ns);
  g_smi.sockets(&ns, socks.data());
  for (uint32_t s = 0; s < ns; ++s) {
    uint32_t np = 0;
    if (g_smi.processors(socks[s], &np, nullptr) != AMDSMI_STATUS_SUCCESS) continue;
    std::vector<amdsmi_processor_handle> ps(np);
    g_smi.processors(socks[s], &np, ps.data());
    for (auto p : ps) {
      processor_type_t t = AMDSMI_PROCESSOR_TYPE_AMD_GPU;
      if (g_smi.ptype && g_smi.ptype(p, &t) == AMDSMI_STATUS_SUCCESS && t != AMDSMI_PROCESSOR_TYPE_AMD_GPU) continue;
      g_smi.gpus.push_back(p);
    }
  }
  g_smi.ready = true;
  return static_cast<int>(g_smi.gpus.size());
}

API void tony_smi_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_smi_mu);
  if (g_smi.ready && g_smi.shut_down) g_smi.shut_down();
  g_smi.ready = false;
  g_smi.gpus.clear();
}

struct tony_gpu_info {
  char bdf[32];
  char uuid[64];
  int32_t numa_node;
  uint32_t vram_total_mb;
};

struct tony_gpu_sample {
  uint32_t gfx_busy_pct;
  uint32_t mem_busy_pct;
  uint32_t vram_used_mb;
  uint32_t vram_total_mb;
  double power_w;
  double temp_c;
  // RAS: accumulated ECC error counts (uncorrectable growth = a GPU fault)
  uint64_t ecc_correctable;
  uint64_t ecc_uncorrectable;
  // xGMI traffic: accumulated KB over all links (read / written by this GPU) and the link bitrate
  uint64_t xgmi_read_kb;
  uint64_t xgmi_write_kb;
  uint32_t xgmi_link_speed_gbps;
  uint32_t xgmi_link_width;
};

API int tony_smi_info(int idx, tony_gpu_info* out) {
  std::lock_guard<std::mutex> lk(g_smi_mu);
  if (!g_smi.ready || idx < 0 || idx >= static_cast<int>(g_smi.gpus.size())) return -1;
  auto p = g_smi.gpus[idx];
  memset(out, 0, sizeof(*out));
  out->numa_node = -1;
  amdsmi_bdf_t b{};
  if (g_smi.bdf && g_smi.bdf(p, &b) == AMDSMI_STATUS_SUCCESS)
    snprintf(out->bdf, sizeof(out->bdf), "%04x:%02x:%02x.%x", static_cast<unsigned>(b.domain_number),
             static_cast<unsigned>(b.bus_number), static_cast<unsigned>(b.device_number),
             static_cast<unsigned>(b.function_number));
  unsigned int ulen = sizeof(out->uuid);
  if (g_smi.uuid) g_smi.uuid(p, &ulen, out->uuid);
  uint32_t numa = 0;
  if (g_smi.numa && g_smi.numa(p, &numa) == AMDSMI_STATUS_SUCCESS) out->numa_node = static_cast<int32_t>(numa);
  amdsmi_vram_usage_t v{};
  if (g_smi.vram && g_smi.vram(p, &v) == AMDSMI_STATUS_SUCCESS) out->vram_total_mb = v.vram_total;
  return 0;
}

API int tony_smi_sample(int idx, tony_gpu_sample* out) {
  std::lock_guard<std::mutex> lk(g_smi_mu);
  if (!g_smi.ready || idx < 0 || idx >= static_cast<int>(g_smi.gpus.size())) return -1;
  auto p = g_smi.gpus[idx];
  memset(out, 0, sizeof(*out));
  int ok = 0;
  amdsmi_engine_usage_t u{};
  if (g_smi.activity && g_smi.activity(p, &u) == AMDSMI_STATUS_SUCCESS) {
    out->gfx_busy_pct = u.gfx_activity;
    out->mem_busy_pct = u.umc_activity;
    ++ok;
  }
  amdsmi_vram_usage_t v{};
  if (g_smi.vram && g_smi.vram(p, &v) == AMDSMI_STATUS_SUCCESS) {
    out->vram_used_mb = v.vram_used;
    out->vram_total_mb = v.vram_total;
    ++ok;
  }
  amdsmi_power_info_t pw{};
  if (g_smi.power && g_smi.power(p, &pw) == AMDSMI_STATUS_SUCCESS) {
    out->power_w = pw.current_socket_power ? pw.current_socket_power : pw.average_socket_power;
    ++ok;
  }
  int64_t t = 0;
  if (g_smi.temp && g_smi.temp(p, AMDSMI_TEMPERATURE_TYPE_HOTSPOT, AMDSMI_TEMP_CURRENT, &t) == AMDSMI_STATUS_SUCCESS) {
    out->temp_c = static_cast<double>(t);
    ++ok;
  }
  amdsmi_error_count_t ec{};
  if (g_smi.ecc && g_smi.ecc(p, &ec) == AMDSMI_STATUS_SUCCESS) {
    out->ecc_correctable = ec.correctable_count;
    out->ecc_uncorrectable = ec.uncorrectable_count;
  }
  if (g_smi.metrics) {
    // the metrics table is large: keep it off the (monitor thread's) stack
    static thread_local amdsmi_gpu_metrics_t m;
    memset(&m, 0, sizeof(m));
    if (g_smi.metrics(p, &m) == AMDSMI_STATUS_SUCCESS) {
      for (int l = 0; l < AMDSMI_MAX_NUM_XGMI_LINKS; ++l) {
        // unsupported entries read as all-ones
        if (m.xgmi_read_data_acc[l] != UINT64_MAX) out->xgmi_read_kb += m.xgmi_read_data_acc[l];
        if (m.xgmi_write_data_acc[l] != UINT64_MAX) out->xgmi_write_kb += m.xgmi_write_data_acc[l];
      }
      if (m.xgmi_link_speed != UINT16_MAX) out->xgmi_link_speed_gbps = m.xgmi_link_speed;
      if (m.xgmi_link_width != UINT16_MAX) out->xgmi_link_width = m.xgmi_link_width;
    }
  }
  return ok > 0 ? 0 : -2;
}

// link type between two GPUs: 0 unknown, 1 PCIe, 2 xGMI; hops in *hops.
API int tony_smi_link(int a, int b, int* hops) {
  std::lock_guard<std::mutex> lk(g_smi_mu);
  if (!g_smi.ready || !g_smi.link_type) return -1;
  const int n = static_cast<int>(g_smi.gpus.size());
  if (a < 0 || b < 0 || a >= n || b >= n) return -1;
  uint64_t h = 0;
  amdsmi_link_type_t t = AMDSMI_LINK_TYPE_UNKNOWN;
  if (g_smi.link_type(g_smi.gpus[a], g_smi.gpus[b], &h, &t) != AMDSMI_STATUS_SUCCESS) return -2;
  *hops = static_cast<int>(h);
  if (t == AMDSMI_LINK_TYPE_XGMI) return 2;
  if (t == AMDSMI_LINK_TYPE_PCIE) return 1;
  return 0;
}
