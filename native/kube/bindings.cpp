// pybind11 bindings of the native Kubernetes transport (module yoda_scheduler_amd._native._yoda_kube).
#include <algorithm>
#include <pybind11/pybind11.h>

#include "build_id.h"
#include <pybind11/stl.h>

#include "json.hpp"
#include "flatjson.hpp"
#include "project.hpp"
#include "transport.hpp"

namespace py = pybind11;
using namespace yk;

namespace {

py::object kv_dict(const std::vector<KV>& kvs) {
  py::dict d;
  for (const auto& kv : kvs) d[py::str(kv.first)] = py::str(kv.second);
  return std::move(d);
}

py::list term_list(const TermP& t) {
  py::list out;
  for (const auto& r : t) {
    py::list vals;
    for (const auto& v : r.values) vals.append(py::str(v));
    out.append(py::make_tuple(py::str(r.key), py::str(r.op), vals));
  }
  return out;
}

// positional arguments of PodInfo's fast constructor (yoda_scheduler_amd/kube/native.py)
// LabelSelector.native() tuple of a projected selector (sorted, de-duplicated expression values)
py::object sel_tuple(bool has, const std::vector<KV>& labels, const std::vector<SelReqP>& exprs) {
  if (!has) return py::none();
  py::list lab, ex;
  for (const auto& kv : labels) lab.append(py::make_tuple(py::str(kv.first), py::str(kv.second)));
  for (const auto& e : exprs) {
    std::vector<std::string> vals = e.values;
    std::sort(vals.begin(), vals.end());
    vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
    py::tuple vt(vals.size());
    for (size_t i = 0; i < vals.size(); ++i) vt[i] = py::str(vals[i]);
    ex.append(py::make_tuple(py::str(e.key), py::str(e.op), vt));
  }
  return py::make_tuple(py::none(), false, py::tuple(lab), py::tuple(ex));
}

// (required affinity, required anti, preferred affinity, preferred anti) of
// (topologyKey, namespaces | None, selector | None, weight), or None without pod (anti-)affinity
py::object pod_aff_tuple(const PodProj& p) {
  if (!p.cold().has_pod_aff) return py::none();
  auto lst = [](const std::vector<PodProj::PodTermP>& v) {
    py::list out;
    for (const auto& t : v) {
      py::object ns = py::none();
      if (!t.ns.empty()) {
        py::tuple nt(t.ns.size());
        for (size_t i = 0; i < t.ns.size(); ++i) nt[i] = py::str(t.ns[i]);
        ns = std::move(nt);
      }
      out.append(py::make_tuple(py::str(t.key), ns, sel_tuple(t.has_sel, t.labels, t.exprs), t.weight));
    }
    return out;
  };
  return py::make_tuple(lst(p.cold().aff_req), lst(p.cold().anti_req), lst(p.cold().aff_pref), lst(p.cold().anti_pref));
}

py::tuple info_args(const PodProj& p) {
  py::object ann = p.cold().has_annotations ? kv_dict(p.cold().annotations) : py::none();
  py::object nsel = p.cold().has_node_selector ? kv_dict(p.cold().node_selector) : py::none();
  py::object req = py::none(), pref = py::none();
  if (p.cold().has_affinity) {
    py::list r;
    for (const auto& t : p.cold().req_terms) r.append(term_list(t));
    py::list pf;
    for (const auto& wt : p.cold().pref_terms) pf.append(py::make_tuple(wt.first, term_list(wt.second)));
    req = std::move(r);
    pref = std::move(pf);
  }
  py::object tols = py::none();
  if (!p.cold().tolerations.empty()) {
    py::list t;
    for (const auto& x : p.cold().tolerations)
      t.append(py::make_tuple(x.has_key ? py::object(py::str(x.key)) : py::object(py::none()), py::str(x.value),
                              py::str(x.op), py::str(x.effect)));
    tols = std::move(t);
  }
  py::object ports = py::none();
  if (!p.cold().ports.empty()) {
    py::list t;
    for (const auto& x : p.cold().ports) t.append(py::make_tuple(x.host_port, py::str(x.protocol), py::str(x.host_ip)));
    ports = std::move(t);
  }
  py::object ext = py::none();
  if (!p.cold().ext.empty()) {
    py::dict d;
    for (const auto& e : p.cold().ext) d[py::str(e.first)] = e.second;
    ext = std::move(d);
  }
  py::list images;
  for (const auto& im : p.images) images.append(py::str(im));
  const PodProj::Owners* o = p.owners.get();
  py::object owner = o && o->has_owner ? py::object(py::make_tuple(py::str(o->owner_api), py::str(o->owner_kind),
                                                                  py::str(o->owner_name), py::str(o->owner_uid)))
                                       : py::object(py::none());
  py::object avoid = o && o->has_avoid ? py::object(py::make_tuple(py::str(o->avoid_kind), py::str(o->avoid_uid)))
                                       : py::object(py::none());
  py::object spread = py::none();
  if (!p.cold().spread.empty()) {
    // (topologyKey, maxSkew, whenUnsatisfiable, LabelSelector.native() tuple | None)
    static const char* kWhen[3] = {"DoNotSchedule", "ScheduleAnyway", "?"};
    py::list l;
    for (const auto& c : p.cold().spread) {
      py::object sel = sel_tuple(c.has_sel, c.labels, c.exprs);
      l.append(py::make_tuple(py::str(c.key), c.max_skew, py::str(kWhen[c.when]), sel));
    }
    spread = std::move(l);
  }
  return py::make_tuple(py::str(p.uid), py::str(p.ns), py::str(p.name), kv_dict(p.labels), ann, py::str(p.sched),
                        py::str(p.node), p.cpu, p.mem, p.nzc, p.nzm, p.priority, nsel, req, pref, tols, ports,
                        p.flags, py::str(p.creation), ext, images, p.containers, owner, avoid, spread, p.deleting,
                        pod_aff_tuple(p));
}

std::shared_ptr<PodEv> project_bytes(const std::string& raw) {
  auto pe = std::make_shared<PodEv>();
  try {
    Value v = parse(raw);
    project_pod(v, pe->p);
  } catch (const ParseError& e) {
    throw py::value_error(std::string("invalid JSON at ") + std::to_string(e.pos) + ": " + e.what);
  }
  pe->raw = raw;
  return pe;
}

}  // namespace

PYBIND11_MODULE(_yoda_kube, m) {
  m.def("build_id", [] { return std::string(YODA_BUILD_ID); }, "hash of the sources this module was built from");
  m.doc() = "Native Kubernetes API transport: pipelined HTTP/1.1 (+TLS), watch decoding, pod projection";

  py::class_<PodEv, std::shared_ptr<PodEv>>(m, "PodEvent")
      .def_property_readonly("ok", [](const PodEv& e) { return e.full().ok; })
      .def_property_readonly("uid", [](const PodEv& e) { return e.p.uid; })
      .def_property_readonly("namespace", [](const PodEv& e) { return e.p.ns; })
      .def_property_readonly("name", [](const PodEv& e) { return e.p.name; })
      .def_property_readonly("key", [](const PodEv& e) { return e.p.ns + "/" + e.p.name; })
      .def_property_readonly("rv", [](const PodEv& e) { return e.p.rv; })
      .def_property_readonly("node", [](const PodEv& e) { return e.p.node; })
      .def_property_readonly("scheduler", [](const PodEv& e) { return e.p.sched; })
      .def_property_readonly("phase", [](const PodEv& e) { return e.p.phase; })
      .def_property_readonly("deleting", [](const PodEv& e) { return e.p.deleting; })
      .def_property_readonly("hash", [](const PodEv& e) { return e.hash(); })
      .def_property_readonly("flags", [](const PodEv& e) { return e.full().flags; })
      .def_property_readonly("claims", [](const PodEv& e) { return e.full().cold().claims; })
      .def_property_readonly("labels_hash", [](const PodEv& e) { return e.p.labels_hash; })
      // status.conditions' PodScheduled entry: (status, reason, message, lastTransitionTime) or None
      .def_property_readonly("sched_cond", [](const PodEv& e) -> py::object {
        const PodProj& p = e.full();
        if (!p.sched_cond) return py::none();
        const auto& c = *p.sched_cond;
        return py::make_tuple(c.status, c.reason, c.msg, c.ltt);
      })
      // (key, uid, node, scheduler, phase, hash): the per-event fields in one call
      .def("ident", [](const PodEv& e) {
        const PodProj& p = e.full();
        return py::make_tuple(py::str(p.ns + "/" + p.name), py::str(p.uid), py::str(p.node),
                              py::str(p.sched), py::str(p.phase), e.hash());
      })
      .def("raw", [](const PodEv& e) {
        const std::string_view r = e.raw_view();
        return py::bytes(r.data(), r.size());
      })
      .def("info_args", [](const PodEv& e) -> py::object {
        const PodProj& p = e.full();
        if (!p.ok) return py::none();
        return info_args(p);
      });

  m.def("project", &project_bytes, py::arg("raw"), "Project a pod's JSON (tests / tooling).");
  // every watch event allocates, fills and frees one PodEv on two threads: its size is a cost of
  // every pod event (round 5 grew it 984 → 1184 bytes, −8 % on the headline; tests pin it)
  m.attr("SIZEOF_POD_EV") = (int)sizeof(PodEv);
  m.attr("SIZEOF_POD_PROJ") = (int)sizeof(PodProj);
  m.def("project_flat_nohash", [](const std::string& raw) {
    auto pe = std::make_shared<PodEv>();
    FlatDoc d;
    if (!d.parse(raw)) throw py::value_error("invalid JSON");
    project_pod_nohash(d.root(), pe->p);
    pe->hash_of = &spec_meta_hash_of;
    pe->raw = raw;
    return pe;
  }, py::arg("raw"), "As the watch stream decodes an ADDED pod with a lane attached (hash on first use).");
  m.def("project_flat", [](const std::string& raw) {
    auto pe = std::make_shared<PodEv>();
    if (!project_pod_text(raw, pe->p)) throw py::value_error("invalid JSON");
    pe->raw = raw;
    return pe;
  }, py::arg("raw"), "Project a pod's JSON through the flat decoder the watch stream uses.");
  // the watch stream's light path vs its parser path, for parity tests: (type, object text,
  // identity tuple), or None when the scanner defers to the parser
  auto ident_tuple = [](const PodProj& p) {
    return py::make_tuple(p.ns, p.name, p.uid, p.rv, p.creation, p.deleting, p.sched, p.node, p.phase);
  };
  m.def("scan_identity", [ident_tuple](const std::string& line, bool only_md) -> py::object {
    PodEv e;
    char t = 0;
    std::string_view obj;
    if (!scan_watch_identity(line, &t, &obj, e.p, only_md)) return py::none();
    const bool partial = e.p.ident_partial;
    if (partial) {                         // completed as the transport's PodEv::full() does
      e.raw.assign(obj.data(), obj.size());
      e.light = true;
      e.complete = &complete_pod_ev;
      e.full();
    }
    return py::make_tuple(std::string(1, t), std::string(obj), ident_tuple(e.p), partial);
  }, py::arg("line"), py::arg("only_md") = false,
     "(type, object text, identity tuple, scanned to metadata only) or None when the parser must decide");
  m.def("scan_labels_hash", [](const std::string& line) -> py::object {
    PodProj p;
    char t = 0;
    std::string_view obj;
    if (!scan_watch_identity(line, &t, &obj, p, false)) return py::none();
    return py::int_(p.labels_hash);
  }, py::arg("line"), "the labels hash the watch identity scanner computes for a watch line");
  m.def("flat_identity", [ident_tuple](const std::string& line) -> py::object {
    FlatDoc d;
    if (!d.parse(line) || !d.root().is(FlatDoc::Obj)) return py::none();
    const FlatDoc::View obj = d.root().get("object");
    if (!obj) return py::none();
    PodProj p;
    project_identity(obj, p);
    const std::string_view t = d.root().sv("type");
    return py::make_tuple(std::string(1, t == "ADDED" ? 'A' : t == "MODIFIED" ? 'M' : t == "DELETED" ? 'D' : '?'),
                          std::string(obj.raw()), ident_tuple(p));
  }, py::arg("line"));
  // PodList body → (resourceVersion, continue, [PodEvent]) — relists of large clusters
  // never build Python dicts either
  m.def("project_list", [](const std::string& body) {
    std::vector<std::shared_ptr<PodEv>> evs;
    std::string rv, cont;
    {
      py::gil_scoped_release rel;
      Value v;
      try {
        v = parse(body);
      } catch (const ParseError& e) {
        py::gil_scoped_acquire acq;
        throw py::value_error(std::string("invalid JSON list: ") + e.what);
      }
      if (const Value* m = v.get("metadata")) {
        rv = std::string(m->sv("resourceVersion"));
        cont = std::string(m->sv("continue"));
      }
      if (const Value* items = v.get("items"); items && items->t == Value::Arr) {
        evs.reserve(items->arr.size());
        for (const auto& it : items->arr) {
          auto pe = std::make_shared<PodEv>();
          project_pod(it, pe->p);
          pe->raw = dump(it);
          evs.push_back(std::move(pe));
        }
      }
    }
    py::list out;
    for (auto& e : evs) out.append(py::cast(e));
    return py::make_tuple(rv, cont, out);
  });
  m.def("quantity", [](const std::string& text, int scale) -> py::object {
    int64_t out;
    Value v = Value::str(text);
    if (!quantity_scaled(v, scale, &out)) return py::none();
    return py::int_(out);
  });
  m.def("canonical", [](const std::string& raw) {
    try {
      return py::bytes(dump(parse(raw)));
    } catch (const ParseError& e) {
      throw py::value_error(std::string("invalid JSON: ") + e.what);
    }
  }, "Parse + compact re-serialise (tests of the JSON codec).");
  m.def("merge_patch", [](const std::string& target, const std::string& patch) {
    Value t = parse(target);
    merge_patch(t, parse(patch));
    return py::bytes(dump(t));
  });

  py::class_<Transport>(m, "Transport")
      .def(py::init([](const std::string& host, int port, bool tls, const std::string& prefix, const std::string& ca,
                       const std::string& cert, const std::string& key, bool insecure, const std::string& token,
                       int conns, int max_inflight, double qps, int burst) {
             ClientConfig c;
             c.host = host;
             c.port = port;
             c.tls = tls;
             c.prefix = prefix;
             c.ca_file = ca;
             c.cert_file = cert;
             c.key_file = key;
             c.insecure = insecure;
             c.token = token;
             c.conns = conns;
             c.max_inflight = max_inflight;
             c.qps = qps;
             c.burst = burst;
             return std::make_unique<Transport>(std::move(c));
           }),
           py::arg("host"), py::arg("port"), py::arg("tls") = false, py::arg("prefix") = "", py::arg("ca") = "",
           py::arg("cert") = "", py::arg("key") = "", py::arg("insecure") = false, py::arg("token") = "",
           py::arg("conns") = 8, py::arg("max_inflight") = 64, py::arg("qps") = 0.0, py::arg("burst") = 0)
      .def("fileno", &Transport::fd)
      .def("request", [](Transport& t, const std::string& method, const std::string& path, py::bytes body,
                         const std::string& ctype, bool limited, double timeout) {
             return t.request(method, path, std::string(body), ctype, limited, timeout);
           }, py::arg("method"), py::arg("path"), py::arg("body") = py::bytes(), py::arg("content_type") = "",
           py::arg("limited") = true, py::arg("timeout") = 0.0)
      .def("bind", &Transport::bind, py::arg("namespace"), py::arg("name"), py::arg("uid"), py::arg("node"),
           py::arg("annotations"), py::arg("timeout") = 0.0)
      // [(namespace, name, uid, node, annotations), ...] -> id of the first (ids consecutive)
      .def("bind_many", [](Transport& t, const py::list& items, double timeout) {
             std::vector<Transport::BindSpec> binds(items.size());
             for (size_t k = 0; k < binds.size(); ++k) {
               py::tuple it = items[k].cast<py::tuple>();
               if (it.size() != 5) throw py::value_error("bind_many: (namespace, name, uid, node, annotations)");
               Transport::BindSpec& b = binds[k];
               b.ns = it[0].cast<std::string>();
               b.name = it[1].cast<std::string>();
               b.uid = it[2].cast<std::string>();
               b.node = it[3].cast<std::string>();
               b.annotations = it[4].cast<std::vector<KV>>();
             }
             return t.bind_many(binds, timeout);
           }, py::arg("binds"), py::arg("timeout") = 0.0)
      .def("watch", &Transport::watch, py::arg("path"), py::arg("pods") = false, py::arg("idle_timeout") = 0.0)
      .def("cancel", &Transport::cancel)
      .def("set_token", &Transport::set_token)
      .def("set_rate", &Transport::set_rate, py::arg("qps"), py::arg("burst"))
      // native pod lane seam (lane_port.hpp): raw pointers, handed to _yoda_core's Lane
      .def("port_ptr", [](Transport& t) { return (uintptr_t) static_cast<PodPort*>(&t); })
      .def("set_pod_sink", [](Transport& t, uintptr_t sink) {
             py::gil_scoped_release rel;
             t.set_pod_sink(reinterpret_cast<PodSink*>(sink));
           }, py::arg("sink"), "attach (pointer from Lane.sink_ptr()) or detach (0) the pod event sink")
      .def("close", [](Transport& t) {
        py::gil_scoped_release rel;
        t.close();
      })
      .def("stats", [](Transport& t) {
        TransportStats s = t.stats();
        py::dict d;
        d["requests"] = s.requests;
        d["responses"] = s.responses;
        d["errors"] = s.errors;
        d["timeouts"] = s.timeouts;
        d["connects"] = s.connects;
        d["watch_events"] = s.watch_events;
        d["watch_bytes"] = s.watch_bytes;
        d["parse_errors"] = s.parse_errors;
        d["watch_cpu_s"] = s.watch_cpu_s;
        d["slab_deletions"] = s.slab_deletions;
        d["recycled"] = s.recycled;
        d["sink_sent"] = s.sink_sent;
        d["sink_answered"] = s.sink_answered;
        d["sink_queue_s"] = s.sink_queue_s;
        d["sink_queue_max_s"] = s.sink_queue_max_s;
        d["sink_rtt_s"] = s.sink_rtt_s;
        d["sink_rtt_max_s"] = s.sink_rtt_max_s;
        d["bytes_out"] = s.bytes_out;
        d["bytes_in"] = s.bytes_in;
        d["throttled"] = s.throttled;
        return d;
      })
      // [(0, id, status, body) | (1, id, [(type, rv, PodEvent | bytes | None, ident | None), ...]) |
      //  (2, id, status, body)]; ident = PodEvent.ident(), built here in the same pass
      .def("drain", [](Transport& t) {
        std::vector<Completion> cs = t.drain();
        // leaked on purpose: must outlive interpreter finalisation
        static py::object* types = new py::object[5]{py::str("ADDED"), py::str("MODIFIED"), py::str("DELETED"),
                                                      py::str("BOOKMARK"), py::str("ERROR")};
        py::list out;
        for (auto& c : cs) {
          if (c.kind == Completion::kEvents) {
            py::list evs;
            for (auto& e : c.events) {
              int ti = e.type == 'A' ? 0 : e.type == 'M' ? 1 : e.type == 'D' ? 2 : e.type == 'B' ? 3 : 4;
              py::object payload, ident = py::none();
              if (e.pod) {
                payload = py::cast(e.pod);
                const PodProj& p = e.pod->full();
                ident = py::make_tuple(py::str(p.ns + "/" + p.name), py::str(p.uid), py::str(p.node), py::str(p.sched),
                                       py::str(p.phase), e.pod->hash());
              } else if (e.type == 'B') {
                payload = py::none();
              } else {
                payload = py::bytes(e.raw);
              }
              evs.append(py::make_tuple(types[ti], py::str(e.rv), payload, ident));
            }
            out.append(py::make_tuple(1, c.id, evs));
          } else if (c.kind == Completion::kWatchEnd) {
            out.append(py::make_tuple(int(c.kind), c.id, c.status, py::bytes(c.body), py::str(c.rv)));
          } else {
            out.append(py::make_tuple(int(c.kind), c.id, c.status, py::bytes(c.body)));
          }
        }
        return out;
      });
}
