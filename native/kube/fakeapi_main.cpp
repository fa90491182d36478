// yoda-fake-apiserver-native: the epoll fake kube-apiserver (fakeapi.hpp) as a process.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "build_id.h"
#include "fakeapi.hpp"

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
  return yk::run_fake_apiserver(o);
}
