// perc_runtime.cc -- perc_hip_runtimes (include/perc.h): which HIP runtime
// copies the process has mapped.  Host-only C++ (g++): the loader's object
// list (dl_iterate_phdr) and dladdr of the runtime entry libperc calls.
#include <dlfcn.h>
#include <limits.h>
#include <link.h>
#include <stdlib.h>
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

extern "C" int hipGetDeviceCount(int* count);  // (libamdhip64's C entry point)

namespace {
std::string canon(const char* f) {
  char rp[PATH_MAX];
  return std::string(f && realpath(f, rp) ? rp : (f ? f : ""));
}
int visit(dl_phdr_info* info, size_t, void* data) {
  auto* v = static_cast<std::vector<std::string>*>(data);
  if (info->dlpi_name && std::strstr(info->dlpi_name, "libamdhip64")) {
    const std::string p = canon(info->dlpi_name);
    if (std::find(v->begin(), v->end(), p) == v->end()) v->push_back(p);
  }
  return 0;
}
}  // namespace

extern "C" int perc_hip_runtimes(char* buf, int cap) {
  // the copy libperc's calls resolve to first, then every other one mapped
  std::vector<std::string> paths;
  Dl_info di{};
  if (dladdr(reinterpret_cast<void*>(&hipGetDeviceCount), &di) && di.dli_fname)
    paths.push_back(canon(di.dli_fname));
  dl_iterate_phdr(visit, &paths);
  if (buf && cap > 0) {
    std::string all;
    for (const auto& p : paths) all += (all.empty() ? "" : ";") + p;
    std::snprintf(buf, (size_t)cap, "%s", all.c_str());
  }
  return (int)paths.size();
}
