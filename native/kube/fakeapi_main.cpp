// yoda-fake-apiserver-native: the epoll fake kube-apiserver (fakeapi.hpp) as a process.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include <sys/syscall.h>
#include <unistd.h>

#include <tuple>
#include <utility>
#include <vector>

#include "build_id.h"
#include "fakeapi.hpp"

namespace yoda_sampler {   // native/core/sampler.cpp
void start(const std::vector<int>& tids, int period_us, bool stacks);
bool dump(const std::string& path);
}  // namespace yoda_sampler

int main(int argc, char** argv) {
  yk::FakeApiOptions o;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char* name) -> std::string {
      if (i + 1 >= argc) {
        fprintf(stderr, "%s needs a value\n", name);
        exit(2);
      }
      return argv[++i];
    };
    if (a == "--host") o.host = val("--host");
    else if (a == "--port") o.port = std::atoi(val("--port").c_str());
    else if (a == "--port-file") o.port_file = val("--port-file");
    else if (a == "--token") o.token = val("--token");
    else if (a == "--history") o.history = size_t(std::atoll(val("--history").c_str()));
    else if (a == "--bookmark-interval") o.bookmark_interval_s = std::atof(val("--bookmark-interval").c_str());
    else if (a == "--build-id") {
      printf("%s\n", YODA_BUILD_ID);
      return 0;
    } else if (a == "-h" || a == "--help") {
      printf("usage: yoda-fake-apiserver-native [--host H] [--port P] [--port-file F] [--token T] "
             "[--history N] [--bookmark-interval S]\n");
      return 0;
    } else {
      fprintf(stderr, "unknown argument %s\n", a.c_str());
      return 2;
    }
  }
  // YODA_APISERVER_PROF=<file>: sample this (single-threaded) server's CPU for its whole life
  // and write the samples at exit (utils/native_prof.py::load_dump)
  const char* prof = getenv("YODA_APISERVER_PROF");
  if (prof && *prof) {
    const char* us = getenv("YODA_NATIVE_PROF");
    yoda_sampler::start({(int)syscall(SYS_gettid)}, us && atoi(us) > 1 ? atoi(us) : 200,
                        getenv("YODA_NATIVE_PROF_STACKS") != nullptr);
  }
  const int rc = yk::run_fake_apiserver(o);
  if (prof && *prof) yoda_sampler::dump(prof);
  return rc;
}
