// Native fake kube-apiserver: the REST subset the scheduler, sniffer, webhook and leader
// election use, served by one epoll thread. It exists so HTTP-transport benchmarks measure
// the *scheduler*: the Python fake apiserver (yoda_scheduler_amd/fakeapi/http.py) costs
// ~100 µs of its own CPU per request, which caps an HTTP burst long before the scheduler.
//
// Semantics mirror yoda_scheduler_amd/fakeapi/server.py (the reference model, with the
// fuller test suite): global resourceVersion, create/get/update(+status)/merge-patch/
// delete, paged lists with continue tokens, field selectors on lists and watches (objects
// entering/leaving the selector arrive as ADDED/DELETED), watch resumption from a
// resourceVersion with a bounded history (410 Gone beyond it), BOOKMARKs, pods/binding
// (404 / 409 on uid mismatch or an already-bound pod; Binding annotations copied onto the
// pod), bearer-token auth, and the /debug/bench/* burst driver with per-pod
// create→bind latency on the server's clock. Watch frames are encoded once per event and
// shared by every watcher.
#pragma once

#include <cstdint>
#include <string>

namespace yk {

struct FakeApiOptions {
  std::string host = "127.0.0.1";
  int port = 0;
  std::string port_file;
  std::string token;               // non-empty: require "Authorization: Bearer <token>"
  size_t history = 200000;         // retained watch events per resource
  double bookmark_interval_s = 0;  // > 0: periodic BOOKMARKs to watchers that asked for them
};

// Runs until SIGTERM/SIGINT. Returns the process exit code.
int run_fake_apiserver(const FakeApiOptions& opt);

}  // namespace yk
