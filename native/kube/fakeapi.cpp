// Native fake kube-apiserver (see fakeapi.hpp).
#include "fakeapi.hpp"
#include "flatjson.hpp"

#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <sys/epoll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <deque>
#include <map>
#include <memory>
#include <random>
#include <string>
#include <unordered_map>
#include <vector>

#include "http.hpp"
#include "json.hpp"

namespace yk {

namespace {

std::atomic<bool> g_stop{false};
void on_signal(int) { g_stop = true; }

double mono() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// second resolution, formatted once per second (the server is single-threaded)
const std::string& rfc3339_now() {
  static time_t last = -1;
  static std::string text;
  const time_t t = time(nullptr);
  if (t != last) {
    struct tm tm;
    gmtime_r(&t, &tm);
    char buf[32];
    strftime(buf, sizeof(buf), "%Y-%m-%dT%H:%M:%SZ", &tm);
    text = buf;
    last = t;
  }
  return text;
}

struct ResDef {
  const char* key;
  const char* group;
  const char* version;
  const char* name;
  const char* kind;
  bool namespaced;
  std::string api_version() const { return group[0] ? std::string(group) + "/" + version : std::string(version); }
};

// mirrors yoda_scheduler_amd/kube/resources.py
const ResDef kRes[] = {
    {"pods", "", "v1", "pods", "Pod", true},
    {"nodes", "", "v1", "nodes", "Node", false},
    {"events", "", "v1", "events", "Event", true},
    {"events.k8s.io", "events.k8s.io", "v1", "events", "Event", true},
    {"leases", "coordination.k8s.io", "v1", "leases", "Lease", true},
    {"scvs", "core.run-linux.com", "v1", "scvs", "Scv", false},
    {"configmaps", "", "v1", "configmaps", "ConfigMap", true},
    {"endpoints", "", "v1", "endpoints", "Endpoints", true},
    {"persistentvolumeclaims", "", "v1", "persistentvolumeclaims", "PersistentVolumeClaim", true},
    {"persistentvolumes", "", "v1", "persistentvolumes", "PersistentVolume", false},
    {"storageclasses", "storage.k8s.io", "v1", "storageclasses", "StorageClass", false},
    {"csinodes", "storage.k8s.io", "v1", "csinodes", "CSINode", false},
    {"poddisruptionbudgets", "policy", "v1", "poddisruptionbudgets", "PodDisruptionBudget", true},
    {"services", "", "v1", "services", "Service", true},
    {"replicationcontrollers", "", "v1", "replicationcontrollers", "ReplicationController", true},
    {"replicasets", "apps", "v1", "replicasets", "ReplicaSet", true},
    {"statefulsets", "apps", "v1", "statefulsets", "StatefulSet", true},
};

// A stored object version: its JSON text is the source of truth (every list and watch frame
// sends it as is); the DOM and the flat view of it are built on first use and kept (the server
// is single-threaded, versions are immutable). Hot pod writes (bind, delete) edit the text
// through the flat view's spans instead of copying and re-serialising a DOM.
struct Stored {
  std::string text;
  int64_t rv = 0;
  std::string ns;              // metadata.namespace
  size_t rv_off = std::string::npos, rv_len = 0;   // span of the resourceVersion value, if known
  mutable std::unique_ptr<Value> dom;
  mutable std::unique_ptr<FlatDoc> flat;
  // field-selector values read from this version (dotted path → value); a version made by
  // editing another inherits the entries its edits cannot have changed
  mutable std::vector<std::pair<std::string, std::string>> fields;
  const Value& v() const {
    if (!dom) dom = std::make_unique<Value>(parse(text));
    return *dom;
  }
  FlatDoc::View fv() const {
    if (!flat) {
      flat = std::make_unique<FlatDoc>();
      if (!flat->parse(text)) return FlatDoc::View();
    }
    return flat->root();
  }
};
using SP = std::shared_ptr<const Stored>;

// The span of `"resourceVersion":"<rv>"`'s value in a text we produced, when it occurs once
// (a JSON string cannot contain the unescaped pattern, so only a nested key could repeat it).
void locate_rv(Stored& s) {
  if (!s.rv) return;
  const std::string pat = "\"resourceVersion\":\"" + std::to_string(s.rv) + "\"";
  const size_t at = s.text.find(pat);
  if (at == std::string::npos || s.text.find(pat, at + 1) != std::string::npos) return;
  s.rv_off = at + 18;   // the opening quote of the value
  s.rv_len = pat.size() - 18;
}

SP make_stored(Value v) {
  auto s = std::make_shared<Stored>();
  s->text = dump(v);
  if (const Value* m = v.get("metadata")) {
    if (const Value* r = m->get("resourceVersion")) s->rv = r->as_int();
    s->ns = std::string(m->sv("namespace"));
  }
  s->dom = std::make_unique<Value>(std::move(v));
  locate_rv(*s);
  return s;
}

// a version made by editing `from` at `edited` (dotted paths): keeps the field-selector values
// no edit can have touched (neither path a prefix of the other). `rv_at`: where the caller put
// the resourceVersion value (its opening quote), when it knows — else it is searched for.
std::shared_ptr<Stored> make_stored_text(std::string text, int64_t rv, std::string ns, const Stored* from = nullptr,
                                         std::initializer_list<std::string_view> edited = {},
                                         size_t rv_at = std::string::npos) {
  auto s = std::make_shared<Stored>();
  s->text = std::move(text);
  s->rv = rv;
  s->ns = std::move(ns);
  if (rv_at != std::string::npos && rv > 0) {
    s->rv_off = rv_at;
    s->rv_len = std::to_string(rv).size() + 2;
  } else {
    locate_rv(*s);
  }
  if (from)
    for (const auto& f : from->fields) {
      bool hit = false;
      for (std::string_view e : edited) {
        const size_t n = std::min(e.size(), f.first.size());
        if (std::string_view(f.first).substr(0, n) == e.substr(0, n) &&
            (f.first.size() == n ? (e.size() == n || e[n] == '.') : f.first[n] == '.'))
          hit = true;
      }
      if (!hit) s->fields.push_back(f);
    }
  return s;
}

// Text edits of one JSON document: replace [beg, end) or insert at beg (beg == end). Edits
// must not overlap; applied in position order.
struct TextEdits {
  struct E {
    size_t beg, end;
    std::string text;
    bool mark = false;
  };
  std::vector<E> es;
  size_t marked = std::string::npos;   // after apply(): where the marked edit's text landed
  void replace(std::string_view doc, FlatDoc::View v, std::string t, bool mark = false) {
    const size_t b = size_t(v.raw().data() - doc.data());
    es.push_back({b, b + v.raw().size(), std::move(t), mark});
  }
  // a member at the front of object `o` (its text starts with '{')
  void insert_member(std::string_view doc, FlatDoc::View o, const std::string& member) {
    const size_t b = size_t(o.raw().data() - doc.data()) + 1;
    es.push_back({b, b, o.size() ? member + "," : member});
  }
  std::string apply(std::string_view doc) {
    std::sort(es.begin(), es.end(), [](const E& a, const E& b) { return a.beg < b.beg; });
    std::string out;
    size_t extra = 0;
    for (const E& e : es) extra += e.text.size();
    out.reserve(doc.size() + extra);
    size_t at = 0;
    for (const E& e : es) {
      out.append(doc.substr(at, e.beg - at));
      if (e.mark) marked = out.size();
      out.append(e.text);
      at = e.end;
    }
    out.append(doc.substr(at));
    return out;
  }
};

std::string quoted(std::string_view x) { return dump(Value::str(std::string(x))); }

struct HistEv {
  int64_t rv;
  char type;
  SP obj, old;
};

// field selectors (kube/fields.py): requirements AND'ed, '=', '==' and '!=' on dotted paths
struct FieldSel {
  struct Req {
    std::vector<std::string> path;
    std::string key;           // the dotted path
    bool eq;
    std::string val;
  };
  std::vector<Req> reqs;
  bool empty() const { return reqs.empty(); }

  static bool parse(const std::string& text, FieldSel& out) {
    size_t i = 0;
    while (i <= text.size()) {
      size_t c = text.find(',', i);
      std::string part(trim(std::string_view(text).substr(i, c == std::string::npos ? std::string::npos : c - i)));
      i = c == std::string::npos ? text.size() + 1 : c + 1;
      if (part.empty()) continue;
      Req r;
      size_t p;
      std::string k;
      if ((p = part.find("!=")) != std::string::npos) {
        k = part.substr(0, p);
        r.eq = false;
        r.val = part.substr(p + 2);
      } else if ((p = part.find("==")) != std::string::npos) {
        k = part.substr(0, p);
        r.eq = true;
        r.val = part.substr(p + 2);
      } else if ((p = part.find('=')) != std::string::npos) {
        k = part.substr(0, p);
        r.eq = true;
        r.val = part.substr(p + 1);
      } else {
        return false;
      }
      k = std::string(trim(k));
      r.key = k;
      r.val = std::string(trim(r.val));
      size_t s = 0;
      while (true) {
        size_t d = k.find('.', s);
        r.path.push_back(k.substr(s, d == std::string::npos ? std::string::npos : d - s));
        if (d == std::string::npos) break;
        s = d + 1;
      }
      out.reqs.push_back(std::move(r));
    }
    return true;
  }

  static std::string field(const Value& obj, const std::vector<std::string>& path) {
    const Value* v = &obj;
    for (const auto& k : path) {
      if (v->t != Value::Obj) return "";
      v = v->get(k);
      if (!v || v->t == Value::Null) return "";
    }
    if (v->t == Value::Str || v->t == Value::Num) return v->s;
    if (v->t == Value::Bool) return v->b ? "True" : "False";
    return dump(*v);
  }

  static std::string field(FlatDoc::View v, const std::vector<std::string>& path) {
    for (const auto& k : path) {
      if (!v.is(FlatDoc::Obj)) return "";
      v = v.get(k);
      if (!v || v.t() == FlatDoc::Null) return "";
    }
    if (v.t() == FlatDoc::Str || v.t() == FlatDoc::Num) return std::string(v.str());
    if (v.t() == FlatDoc::Bool) return v.b() ? "True" : "False";
    return dump(yk::parse(std::string(v.raw())));   // objects / arrays: the DOM's text
  }

  // through the version's field cache; a miss reads the DOM if it exists, else the flat view
  static const std::string& field(const Stored& s, const Req& r) {
    for (const auto& f : s.fields)
      if (f.first == r.key) return f.second;
    s.fields.emplace_back(r.key, s.dom ? field(*s.dom, r.path) : field(s.fv(), r.path));
    return s.fields.back().second;
  }

  bool matches(const Stored& s) const {
    for (const Req& r : reqs) {
      const std::string& v = field(s, r);
      if (r.eq ? v != r.val : v == r.val) return false;
    }
    return true;
  }

  bool matches(FlatDoc::View obj) const {
    for (size_t i = 0; i < reqs.size(); ++i) {
      std::string v = field(obj, reqs[i].path);
      if (reqs[i].eq) {
        if (v != reqs[i].val) return false;
      } else if (v == reqs[i].val) {
        return false;
      }
    }
    return true;
  }

  bool matches(const Value& obj) const {
    // group by path like the Python matcher: several '=' on one path never all hold
    for (size_t i = 0; i < reqs.size(); ++i) {
      std::string v = field(obj, reqs[i].path);
      if (reqs[i].eq) {
        if (v != reqs[i].val) return false;
      } else if (v == reqs[i].val) {
        return false;
      }
    }
    return true;
  }
};

char filter_event(const FieldSel& sel, char type, const Stored& obj, const Stored* old) {
  if (type == 'A' || type == 'D') return sel.matches(obj) ? type : 0;
  if (type != 'M') return type;
  bool now = sel.matches(obj);
  bool before = old && sel.matches(*old);
  if (now && before) return 'M';
  if (now) return 'A';
  if (before) return 'D';
  return 0;
}

const char* type_name(char t) {
  switch (t) {
    case 'A': return "ADDED";
    case 'M': return "MODIFIED";
    case 'D': return "DELETED";
    case 'B': return "BOOKMARK";
    default: return "ERROR";
  }
}

void chunk(std::string& out, std::string_view data) {
  char hdr[24];
  int n = snprintf(hdr, sizeof(hdr), "%zx\r\n", data.size());
  out.append(hdr, size_t(n));
  out.append(data);
  out.append("\r\n");
}

// one watch event as an HTTP chunk, appended straight to `out` (a connection's write buffer)
void append_frame(std::string& out, char type, const std::string& obj_text) {
  static constexpr std::string_view pre = "{\"type\":\"", mid = "\",\"object\":", post = "}\n";
  const std::string_view tn = type_name(type);
  const size_t n = pre.size() + tn.size() + mid.size() + obj_text.size() + post.size();
  char hdr[24];
  const int hn = snprintf(hdr, sizeof(hdr), "%zx\r\n", n);
  out.reserve(out.size() + size_t(hn) + n + 2);
  out.append(hdr, size_t(hn)).append(pre).append(tn).append(mid).append(obj_text).append(post).append("\r\n");
}

std::string frame(char type, const std::string& obj_text) {
  std::string out;
  append_frame(out, type, obj_text);
  return out;
}

const char* reason_phrase(int code) {
  switch (code) {
    case 200: return "OK";
    case 201: return "Created";
    case 400: return "Bad Request";
    case 401: return "Unauthorized";
    case 404: return "Not Found";
    case 405: return "Method Not Allowed";
    case 409: return "Conflict";
    case 410: return "Gone";
    case 422: return "Unprocessable Entity";
    case 500: return "Internal Server Error";
    default: return "Status";
  }
}

struct ApiErr {
  int code;
  std::string reason, message;
};

std::string status_text(const ApiErr& e) {
  Value s = Value::object();
  s.at("kind") = Value::str("Status");
  s.at("apiVersion") = Value::str("v1");
  s.at("status") = Value::str("Failure");
  s.at("message") = Value::str(e.message);
  s.at("reason") = Value::str(e.reason);
  s.at("code") = Value::num(int64_t(e.code));
  return dump(s);
}

struct Conn;

struct Watcher {
  Conn* conn = nullptr;
  struct ResState* rs = nullptr;
  FieldSel sel;
  std::string ns;          // namespaced watch: only this namespace
  double deadline = 0;
  bool bookmarks = false;
  bool dead = false;
};

struct ResState {
  const ResDef* def = nullptr;
  std::map<std::string, SP> objs;
  std::deque<HistEv> hist;
  int64_t oldest_rv = 0;
  std::vector<Watcher*> watchers;
};

struct Conn {
  int fd = -1;
  RequestParser rp;
  Request req;
  std::string wbuf;
  size_t woff = 0;
  std::unique_ptr<Watcher> watcher;
  bool close_after_write = false;
  bool want_out = false;
  bool epoll_out = false;   // EPOLLOUT registered (output left over from a short send)
  bool dead = false;
};

class Server {
 public:
  explicit Server(const FakeApiOptions& o) : opt_(o) {
    for (const auto& d : kRes) {
      auto rs = std::make_unique<ResState>();
      rs->def = &d;
      by_key_[d.key] = rs.get();
      by_path_[std::string(d.group) + "/" + d.name] = rs.get();
      res_.push_back(std::move(rs));
    }
    std::random_device rd;
    std::mt19937_64 g(rd());
    char buf[24];
    snprintf(buf, sizeof(buf), "%016llx", static_cast<unsigned long long>(g()));
    uid_prefix_ = std::string("nf") + buf;
  }

  int run();

 private:
  // ------------------------------------------------------------------ store
  std::string key_of(const ResDef& d, const Value& obj) const {
    const Value* m = obj.get("metadata");
    std::string name = m ? std::string(m->sv("name")) : "";
    if (!d.namespaced) return name;
    std::string ns = m ? std::string(m->sv("namespace")) : "";
    if (ns.empty()) ns = "default";
    return ns + "/" + name;
  }

  void emit(ResState& rs, char type, const SP& obj, const SP& old) {
    const int64_t rv = obj->rv ? obj->rv : last_rv_;
    rs.hist.push_back(HistEv{rv, type, obj, old});
    while (rs.hist.size() > opt_.history) {
      rs.oldest_rv = rs.hist.front().rv;
      rs.hist.pop_front();
    }
    if (rs.watchers.empty()) return;
    const std::string& ns = obj->ns;
    for (Watcher* w : rs.watchers) {
      if (w->dead) continue;
      if (!w->ns.empty() && ns != w->ns) continue;
      char t = w->sel.empty() ? type : filter_event(w->sel, type, *obj, old.get());
      if (!t) continue;
      append_frame(w->conn->wbuf, t, obj->text);      // no intermediate frame string
      mark_out(w->conn);
    }
  }

  std::string next_rv() { return std::to_string(++last_rv_); }

  SP create(ResState& rs, Value obj, const std::string& path_ns, ApiErr* err) {
    const ResDef& d = *rs.def;
    if (obj.t != Value::Obj) {
      *err = {400, "BadRequest", "object expected"};
      return nullptr;
    }
    Value& meta = obj.at("metadata");
    if (meta.t != Value::Obj) meta = Value::object();
    if (d.namespaced) {
      std::string_view ns = meta.sv("namespace");
      if (ns.empty()) meta.at("namespace") = Value::str(path_ns.empty() ? "default" : path_ns);
    }
    if (meta.sv("name").empty()) {
      std::string_view gen = meta.sv("generateName");
      if (gen.empty()) {
        *err = {422, "Invalid", "metadata.name required"};
        return nullptr;
      }
      char buf[8];
      snprintf(buf, sizeof(buf), "%05x", unsigned(++gen_counter_ & 0xfffff));
      meta.at("name") = Value::str(std::string(gen) + buf);
    }
    if (!obj.get("apiVersion")) obj.at("apiVersion") = Value::str(d.api_version());
    if (!obj.get("kind")) obj.at("kind") = Value::str(d.kind);
    Value& m2 = obj.at("metadata");
    if (m2.sv("uid").empty()) {
      char buf[24];
      snprintf(buf, sizeof(buf), "-%012llx", static_cast<unsigned long long>(++uid_counter_));
      m2.at("uid") = Value::str(uid_prefix_ + buf);
    }
    m2.at("resourceVersion") = Value::str(next_rv());
    if (!m2.get("creationTimestamp")) m2.at("creationTimestamp") = Value::str(rfc3339_now());
    std::string key = key_of(d, obj);
    if (rs.objs.count(key)) {
      --last_rv_;
      *err = {409, "AlreadyExists", std::string(d.key) + " " + key + " already exists"};
      return nullptr;
    }
    SP s = make_stored(std::move(obj));
    rs.objs[key] = s;
    if (&rs == by_key_["pods"]) create_log_[key] = mono();
    emit(rs, 'A', s, nullptr);
    return s;
  }

  SP update(ResState& rs, const Value& body, const std::string& path_ns, const std::string& name, bool status_only,
            ApiErr* err) {
    const ResDef& d = *rs.def;
    const Value* bm = body.get("metadata");
    std::string nm = bm ? std::string(bm->sv("name")) : "";
    if (nm.empty()) nm = name;
    std::string ns = bm ? std::string(bm->sv("namespace")) : "";
    if (ns.empty()) ns = path_ns.empty() ? "default" : path_ns;
    std::string key = d.namespaced ? ns + "/" + nm : nm;
    auto it = rs.objs.find(key);
    if (it == rs.objs.end()) {
      *err = {404, "NotFound", std::string(d.key) + " " + key + " not found"};
      return nullptr;
    }
    SP cur = it->second;
    std::string_view rv = bm ? bm->sv("resourceVersion") : std::string_view();
    const Value* cm = cur->v().get("metadata");
    if (!rv.empty() && cm && rv != cm->sv("resourceVersion")) {
      *err = {409, "Conflict", std::string(d.key) + " " + key + ": the object has been modified"};
      return nullptr;
    }
    Value nv;
    if (status_only) {
      nv = cur->v();
      const Value* st = body.get("status");
      nv.at("status") = st ? *st : Value();
    } else {
      nv = body;
      if (!body.get("status")) {
        if (const Value* cst = cur->v().get("status")) nv.at("status") = *cst;
      }
    }
    Value meta = cm ? *cm : Value::object();
    if (bm && bm->t == Value::Obj) {
      for (const auto& kv : bm->obj) {
        if (kv.first == "uid" || kv.first == "creationTimestamp" || kv.first == "resourceVersion") continue;
        meta.at(kv.first) = kv.second;
      }
    }
    meta.at("resourceVersion") = Value::str(next_rv());
    nv.at("metadata") = std::move(meta);
    SP s = make_stored(std::move(nv));
    it->second = s;
    emit(rs, 'M', s, cur);
    return s;
  }

  SP patch(ResState& rs, const Value& p, const std::string& path_ns, const std::string& name, ApiErr* err,
           bool strategic = false) {
    const ResDef& d = *rs.def;
    std::string key = d.namespaced ? (path_ns.empty() ? "default" : path_ns) + "/" + name : name;
    auto it = rs.objs.find(key);
    if (it == rs.objs.end()) {
      *err = {404, "NotFound", std::string(d.key) + " " + key + " not found"};
      return nullptr;
    }
    SP cur = it->second;
    Value nv = cur->v();
    if (strategic) strategic_merge_patch(nv, p);
    else merge_patch(nv, p);
    Value& meta = nv.at("metadata");
    if (meta.t != Value::Obj) meta = Value::object();
    meta.at("resourceVersion") = Value::str(next_rv());
    if (const Value* cm = cur->v().get("metadata")) {
      for (const char* k : {"uid", "name", "namespace", "creationTimestamp"})
        if (const Value* x = cm->get(k)) meta.at(k) = *x;
    }
    SP s = make_stored(std::move(nv));
    it->second = s;
    emit(rs, 'M', s, cur);
    return s;
  }

  SP remove(ResState& rs, const std::string& key, ApiErr* err) {
    auto it = rs.objs.find(key);
    if (it == rs.objs.end()) {
      *err = {404, "NotFound", std::string(rs.def->key) + " " + key + " not found"};
      return nullptr;
    }
    SP cur = it->second;
    rs.objs.erase(it);
    // the deleted object as stored, with the deletion's resourceVersion
    const std::string rvs = next_rv();
    SP s;
    if (cur->rv_off != std::string::npos) {
      std::string t;
      t.reserve(cur->text.size() + 4);
      t.append(cur->text, 0, cur->rv_off).append(quoted(rvs)).append(cur->text, cur->rv_off + cur->rv_len,
                                                                       std::string::npos);
      s = make_stored_text(std::move(t), last_rv_, cur->ns, cur.get(), {"metadata.resourceVersion"}, cur->rv_off);
    } else if (FlatDoc::View rvv = cur->fv() ? cur->fv().get("metadata").get("resourceVersion") : FlatDoc::View()) {
      TextEdits ed;
      ed.replace(cur->text, rvv, quoted(rvs), true);
      std::string t = ed.apply(cur->text);
      s = make_stored_text(std::move(t), last_rv_, cur->ns, cur.get(), {"metadata.resourceVersion"}, ed.marked);
    } else {
      Value gone = cur->v();
      gone.at("metadata").at("resourceVersion") = Value::str(rvs);
      s = make_stored(std::move(gone));
    }
    emit(rs, 'D', s, nullptr);
    return s;
  }

  // `body`: the Binding, read through a flat view (no DOM: only uid, target.name and the
  // annotations are used, the annotation values copied as their JSON text)
  bool bind(const std::string& ns, const std::string& name, FlatDoc::View body, ApiErr* err) {
    ResState& rs = *by_key_["pods"];
    std::string key = ns + "/" + name;
    auto it = rs.objs.find(key);
    if (it == rs.objs.end()) {
      *err = {404, "NotFound", "pods " + key + " not found"};
      return false;
    }
    SP cur = it->second;
    const std::string& doc = cur->text;
    FlatDoc::View root = cur->fv();
    if (!root.is(FlatDoc::Obj)) {
      *err = {500, "InternalError", "pods " + key + ": stored object unreadable"};
      return false;
    }
    FlatDoc::View meta = root.get("metadata"), spec = root.get("spec"), status = root.get("status");
    const FlatDoc::View bm = body.is(FlatDoc::Obj) ? body.get("metadata") : FlatDoc::View();
    std::string_view uid = bm.is(FlatDoc::Obj) ? bm.sv("uid") : std::string_view();
    if (!uid.empty() && meta && meta.sv("uid") != uid) {
      *err = {409, "Conflict", "pod " + key + " uid mismatch"};
      return false;
    }
    if (spec && !spec.sv("nodeName").empty()) {
      *err = {409, "Conflict", "pod " + key + " is already assigned to node " + std::string(spec.sv("nodeName"))};
      return false;
    }
    const FlatDoc::View tgt = body.is(FlatDoc::Obj) ? body.get("target") : FlatDoc::View();
    const std::string node = tgt.is(FlatDoc::Obj) ? std::string(tgt.sv("name")) : "";
    const std::string rvs = next_rv();
    TextEdits ed;
    // spec.nodeName
    const std::string nn = "\"nodeName\":" + quoted(node);
    if (spec.is(FlatDoc::Obj)) {
      if (FlatDoc::View x = spec.get("nodeName")) ed.replace(doc, x, quoted(node));
      else ed.insert_member(doc, spec, nn);
    } else if (spec) {
      ed.replace(doc, spec, "{" + nn + "}");
    } else {
      ed.insert_member(doc, root, "\"spec\":{" + nn + "}");
    }
    // status.conditions: PodScheduled replaced by a fresh True condition
    std::string conds = "[";
    FlatDoc::View oc = status.is(FlatDoc::Obj) ? status.get("conditions") : FlatDoc::View();
    if (oc.is(FlatDoc::Arr))
      for (FlatDoc::View c = oc.first(); c; c = c.next())
        if (c.sv("type") != "PodScheduled") conds.append(c.raw()).push_back(',');
    conds.append("{\"type\":\"PodScheduled\",\"status\":\"True\",\"lastTransitionTime\":\"")
        .append(rfc3339_now()).append("\"}]");
    if (status.is(FlatDoc::Obj)) {
      if (oc) ed.replace(doc, oc, conds);
      else ed.insert_member(doc, status, "\"conditions\":" + conds);
    } else if (status) {
      ed.replace(doc, status, "{\"conditions\":" + conds + "}");
    } else {
      ed.insert_member(doc, root, "\"status\":{\"conditions\":" + conds + "}");
    }
    // metadata: the Binding's annotations merged, a new resourceVersion
    if (meta.is(FlatDoc::Obj)) {
      if (FlatDoc::View x = meta.get("resourceVersion")) ed.replace(doc, x, quoted(rvs), true);
      else ed.insert_member(doc, meta, "\"resourceVersion\":" + quoted(rvs));
      const FlatDoc::View ann = bm.is(FlatDoc::Obj) ? bm.get("annotations") : FlatDoc::View();
      if (ann.is(FlatDoc::Obj) && ann.size()) {
        FlatDoc::View ma = meta.get("annotations");
        if (ma.is(FlatDoc::Obj)) {
          std::string add;
          for (FlatDoc::View kv = ann.first(); kv; kv = kv.next()) {
            if (FlatDoc::View x = ma.get(kv.key())) {
              ed.replace(doc, x, std::string(kv.raw()));
            } else {
              if (!add.empty()) add.push_back(',');
              add.append(quoted(kv.key())).push_back(':');
              add.append(kv.raw());
            }
          }
          if (!add.empty()) ed.insert_member(doc, ma, add);
        } else {
          std::string obj = "{";
          for (FlatDoc::View kv = ann.first(); kv; kv = kv.next()) {
            if (obj.size() > 1) obj.push_back(',');
            obj.append(quoted(kv.key())).push_back(':');
            obj.append(kv.raw());
          }
          obj.push_back('}');
          if (ma) ed.replace(doc, ma, obj);
          else ed.insert_member(doc, meta, "\"annotations\":" + obj);
        }
      }
    } else {
      *err = {500, "InternalError", "pods " + key + ": no metadata"};
      --last_rv_;
      return false;
    }
    std::string text = ed.apply(doc);
    SP s = make_stored_text(std::move(text), last_rv_, cur->ns, cur.get(),
                            {"spec.nodeName", "status.conditions", "metadata.resourceVersion", "metadata.annotations",
                             // an inserted spec / status holds only the edited member; one that
                             // was not an object was replaced whole
                             spec && !spec.is(FlatDoc::Obj) ? "spec" : "spec.nodeName",
                             status && !status.is(FlatDoc::Obj) ? "status" : "status.conditions"},
                            ed.marked);
    it->second = s;
    bind_log_[key] = mono();
    emit(rs, 'M', s, cur);
    return true;
  }

  // ------------------------------------------------------------------ HTTP
  void respond(Conn* c, int code, std::string_view body, bool keep_alive = true) {
    std::string& w = c->wbuf;
    char hdr[160];
    int n = snprintf(hdr, sizeof(hdr), "HTTP/1.1 %d %s\r\nContent-Type: application/json\r\nContent-Length: %zu\r\n%s\r\n",
                     code, reason_phrase(code), body.size(), keep_alive ? "" : "Connection: close\r\n");
    w.append(hdr, size_t(n));
    w.append(body);
    if (!keep_alive) c->close_after_write = true;
    mark_out(c);
  }

  void respond_err(Conn* c, const ApiErr& e) { respond(c, e.code, status_text(e)); }

  void mark_out(Conn* c) {
    if (!c->want_out) {
      c->want_out = true;
      dirty_.push_back(c);
    }
  }

  void handle(Conn* c, Request& req);
  void handle_bench(Conn* c, Request& req);
  void step_jobs();
  struct BenchJob {
    bool del = false;
    std::string tag, ts;
    size_t n = 0, next = 0;
    std::vector<std::string> keys;
  };
  std::deque<BenchJob> jobs_;
  // pods the bench bursts created: what a reset deletes (pods created through the API — a
  // populated cluster's bound pods, `bench.py --prefill` — stay)
  std::vector<std::string> bench_keys_;
  void handle_list(Conn* c, ResState& rs, const std::string& ns, const Request& req);
  void start_watch(Conn* c, ResState& rs, const std::string& ns, const Request& req);
  void finish_watch(Conn* c);
  void flush(Conn* c);
  void flush_dirty();   // every connection with pending output
  void close_conn(Conn* c);
  void send_bookmarks(ResState& rs);

  FakeApiOptions opt_;
  std::vector<std::unique_ptr<ResState>> res_;
  std::unordered_map<std::string, ResState*> by_key_, by_path_;
  int64_t last_rv_ = 0;
  uint64_t uid_counter_ = 0, gen_counter_ = 0;
  std::string uid_prefix_;
  int ep_ = -1, lfd_ = -1;
  std::vector<Conn*> dirty_;
  std::unordered_map<int, std::unique_ptr<Conn>> conns_;
  // bench
  std::vector<Value> templates_;
  struct TmplText {
    std::string ns, meta_rest, top_rest;   // ",members..." of metadata (less the per-pod ones) / of the root
  };
  std::vector<TmplText> tmpl_text_;
  std::unordered_map<std::string, double> create_log_, bind_log_;
  // where the event loop's time goes (seconds, cumulative; /debug/bench/status reports it):
  // requests by kind, the bench jobs' slices, socket reads + request parsing, response writes
  enum Prof { kBind, kEvent, kCreate, kDelete, kGetList, kWatch, kUpdate, kBench, kJobCreate, kJobDelete, kRead,
              kFlush, kNProf };
  double prof_[kNProf] = {};
  uint64_t prof_n_[kNProf] = {};
  static int prof_kind(const Request& r) {
    const std::string& p = r.path;
    if (p.rfind("/debug/", 0) == 0) return kBench;
    if (r.method == "POST") {
      if (p.size() >= 8 && p.compare(p.size() - 8, 8, "/binding") == 0) return kBind;
      if (p.size() >= 7 && p.compare(p.size() - 7, 7, "/events") == 0) return kEvent;
      return kCreate;
    }
    if (r.method == "DELETE") return kDelete;
    if (r.method == "GET") {
      const std::string& q = r.query;
      return q.find("watch=1") != std::string::npos || q.find("watch=true") != std::string::npos ? kWatch : kGetList;
    }
    return kUpdate;
  }
};

void Server::flush_dirty() {
  if (dirty_.empty()) return;
  std::vector<Conn*> d;
  d.swap(dirty_);
  const double tf = mono();
  for (Conn* c : d) flush(c);
  prof_[kFlush] += mono() - tf;
}

void Server::flush(Conn* c) {
  c->want_out = false;
  if (c->dead) return;
  while (c->woff < c->wbuf.size()) {
    ssize_t n = ::send(c->fd, c->wbuf.data() + c->woff, c->wbuf.size() - c->woff, MSG_NOSIGNAL);
    if (n < 0) {
      if (errno == EAGAIN || errno == EWOULDBLOCK) break;
      close_conn(c);
      return;
    }
    c->woff += size_t(n);
  }
  epoll_event ev{};
  ev.data.ptr = c;
  bool out = false;
  if (c->woff >= c->wbuf.size()) {
    c->wbuf.clear();
    c->woff = 0;
    if (c->close_after_write) {
      close_conn(c);
      return;
    }
    ev.events = EPOLLIN | EPOLLRDHUP;
  } else {
    if (c->woff > (4u << 20)) {
      c->wbuf.erase(0, c->woff);
      c->woff = 0;
    }
    ev.events = EPOLLIN | EPOLLOUT | EPOLLRDHUP;
    out = true;
  }
  // the registration changes only when a send falls short or the backlog drains
  if (out != c->epoll_out) {
    c->epoll_out = out;
    epoll_ctl(ep_, EPOLL_CTL_MOD, c->fd, &ev);
  }
}

void Server::close_conn(Conn* c) {
  if (c->dead) return;
  c->dead = true;
  if (c->watcher) {
    c->watcher->dead = true;
    auto& ws = c->watcher->rs->watchers;
    ws.erase(std::remove(ws.begin(), ws.end(), c->watcher.get()), ws.end());
  }
  epoll_ctl(ep_, EPOLL_CTL_DEL, c->fd, nullptr);
  ::close(c->fd);
}

void Server::finish_watch(Conn* c) {
  if (!c->watcher) return;
  auto& ws = c->watcher->rs->watchers;
  ws.erase(std::remove(ws.begin(), ws.end(), c->watcher.get()), ws.end());
  c->watcher.reset();
  c->wbuf.append("0\r\n\r\n");
  mark_out(c);
}

void Server::send_bookmarks(ResState& rs) {
  std::string obj = "{\"kind\":\"" + std::string(rs.def->kind) + "\",\"apiVersion\":\"" + rs.def->api_version() +
                    "\",\"metadata\":{\"resourceVersion\":\"" + std::to_string(last_rv_) + "\"}}";
  std::string f = frame('B', obj);
  for (Watcher* w : rs.watchers) {
    if (w->dead || !w->bookmarks) continue;
    w->conn->wbuf.append(f);
    mark_out(w->conn);
  }
}

void Server::handle_list(Conn* c, ResState& rs, const std::string& ns, const Request& req) {
  const ResDef& d = *rs.def;
  FieldSel sel;
  std::string fs = query_param(req.query, "fieldSelector");
  if (!fs.empty() && !FieldSel::parse(fs, sel)) {
    respond_err(c, {400, "BadRequest", "invalid field selector"});
    return;
  }
  long limit = std::atol(query_param(req.query, "limit", "0").c_str());
  std::string cont = query_param(req.query, "continue");
  int64_t rv = last_rv_;
  std::string start;
  bool paged = limit > 0 || !cont.empty();
  if (!cont.empty()) {
    size_t dot = cont.find('.');
    if (dot == std::string::npos) {
      respond_err(c, {400, "BadRequest", "invalid continue token"});
      return;
    }
    rv = std::atoll(cont.substr(0, dot).c_str());
    std::string hex = cont.substr(dot + 1);
    for (size_t i = 0; i + 1 < hex.size(); i += 2) start.push_back(char(unhex(hex[i]) * 16 + unhex(hex[i + 1])));
    if (rv < rs.oldest_rv) {
      respond_err(c, {410, "Expired", "the provided continue parameter is too old"});
      return;
    }
  }
  std::string out;
  out.reserve(4096);
  out.append("{\"kind\":\"").append(d.kind).append("List\",\"apiVersion\":\"").append(d.api_version());
  out.append("\",\"items\":[");
  long n = 0;
  std::string last_key;
  bool more = false;
  auto it = paged && !start.empty() ? rs.objs.upper_bound(start) : rs.objs.begin();
  for (; it != rs.objs.end(); ++it) {
    const Stored& s = *it->second;
    if (d.namespaced && !ns.empty() && s.ns != ns) continue;
    if (!sel.empty() && !sel.matches(s)) continue;
    if (paged && limit > 0 && n >= limit) {
      more = true;
      break;
    }
    if (n) out.push_back(',');
    out.append(s.text);
    last_key = it->first;
    ++n;
  }
  out.append("],\"metadata\":{\"resourceVersion\":\"").append(std::to_string(rv)).append("\"");
  if (more) {
    static const char hx[] = "0123456789abcdef";
    std::string tok = std::to_string(rv) + ".";
    for (unsigned char ch : last_key) {
      tok.push_back(hx[ch >> 4]);
      tok.push_back(hx[ch & 15]);
    }
    out.append(",\"continue\":\"").append(tok).append("\"");
  }
  out.append("}}");
  respond(c, 200, out);
}

void Server::start_watch(Conn* c, ResState& rs, const std::string& ns, const Request& req) {
  auto w = std::make_unique<Watcher>();
  std::string fs = query_param(req.query, "fieldSelector");
  if (!fs.empty() && !FieldSel::parse(fs, w->sel)) {
    respond_err(c, {400, "BadRequest", "invalid field selector"});
    return;
  }
  c->wbuf.append("HTTP/1.1 200 OK\r\nContent-Type: application/json\r\nTransfer-Encoding: chunked\r\n\r\n");
  mark_out(c);
  int64_t rv = std::atoll(query_param(req.query, "resourceVersion", "0").c_str());
  if (rv && rv < rs.oldest_rv) {
    chunk(c->wbuf, "{\"type\":\"ERROR\",\"object\":" + status_text({410, "Expired", "too old resource version"}) + "}\n");
    c->wbuf.append("0\r\n\r\n");
    return;
  }
  w->conn = c;
  w->rs = &rs;
  if (rs.def->namespaced) w->ns = ns;
  double to = std::atof(query_param(req.query, "timeoutSeconds", "300").c_str());
  w->deadline = mono() + (to > 0 ? to : 300);
  std::string bm = query_param(req.query, "allowWatchBookmarks");
  w->bookmarks = bm == "true" || bm == "1";
  if (rv) {
    for (const HistEv& h : rs.hist) {
      if (h.rv <= rv) continue;
      if (!w->ns.empty() && h.obj->ns != w->ns) continue;
      char t = w->sel.empty() ? h.type : filter_event(w->sel, h.type, *h.obj, h.old.get());
      if (!t) continue;
      append_frame(c->wbuf, t, h.obj->text);
    }
  }
  rs.watchers.push_back(w.get());
  c->watcher = std::move(w);
}

void Server::handle_bench(Conn* c, Request& req) {
  const std::string& p = req.path;
  ResState& pods = *by_key_["pods"];
  if (p == "/debug/bench/load") {
    Value b;
    try {
      b = parse(req.body);
    } catch (const ParseError&) {
      respond_err(c, {400, "BadRequest", "invalid JSON"});
      return;
    }
    templates_.clear();
    tmpl_text_.clear();
    if (const Value* ps = b.get("pods"); ps && ps->t == Value::Arr) templates_ = ps->arr;
    // each template as text around the per-pod metadata (name, uid, resourceVersion,
    // creationTimestamp): a burst pod is then spliced, not copied and re-serialised — what
    // create() would store, with those four members first in metadata
    for (const Value& t : templates_) {
      TmplText tt;
      Value o = t;
      if (o.t != Value::Obj) break;
      if (!o.get("apiVersion")) o.at("apiVersion") = Value::str(kRes[0].api_version());
      if (!o.get("kind")) o.at("kind") = Value::str(kRes[0].kind);
      Value& meta = o.at("metadata");
      if (meta.t != Value::Obj) meta = Value::object();
      if (meta.sv("namespace").empty()) meta.at("namespace") = Value::str("default");
      tt.ns = std::string(meta.sv("namespace"));
      Value rest = Value::object();
      for (auto& kv : meta.obj)
        if (kv.first != "name" && kv.first != "uid" && kv.first != "resourceVersion" &&
            kv.first != "creationTimestamp" && kv.first != "generateName")
          rest.obj.push_back(kv);
      const std::string mr = dump(rest);             // {...}
      tt.meta_rest = mr.size() > 2 ? "," + mr.substr(1, mr.size() - 2) : "";
      Value top = Value::object();
      for (auto& kv : o.obj)
        if (kv.first != "metadata") top.obj.push_back(kv);
      const std::string tr = dump(top);
      tt.top_rest = tr.size() > 2 ? "," + tr.substr(1, tr.size() - 2) : "";
      tmpl_text_.push_back(std::move(tt));
    }
    if (tmpl_text_.size() != templates_.size()) tmpl_text_.clear();   // a template create() must handle
    respond(c, 200, "{\"n\":" + std::to_string(templates_.size()) + "}");
    return;
  }
  if (p == "/debug/bench/burst") {
    Value b;
    try {
      b = parse(req.body.empty() ? std::string("{}") : req.body);
    } catch (const ParseError&) {
      respond_err(c, {400, "BadRequest", "invalid JSON"});
      return;
    }
    std::string tag = std::string(b.sv("tag"));
    if (tag.empty()) tag = "b";
    // created in slices between the event loop's turns, like a real apiserver serving the
    // burst's POSTs concurrently with everything else (the scheduler's Bindings included)
    BenchJob job;
    job.tag = tag;
    job.n = templates_.size();
    jobs_.push_back(std::move(job));
    respond(c, 200, "{\"n\":" + std::to_string(templates_.size()) + "}");
    return;
  }
  if (p == "/debug/bench/status") {
    std::string out = "{\"created\":" + std::to_string(create_log_.size()) + ",\"bound\":" + std::to_string(bind_log_.size());
    if (!query_param(req.query, "full").empty()) {
      out.append(",\"latencies\":[");
      double t0 = 1e300, tend = 0;
      for (const auto& kv : create_log_) t0 = std::min(t0, kv.second);
      bool first = true;
      char buf[40];
      for (const auto& kv : bind_log_) {
        tend = std::max(tend, kv.second);
        auto ci = create_log_.find(kv.first);
        if (ci == create_log_.end()) continue;
        if (!first) out.push_back(',');
        first = false;
        int n = snprintf(buf, sizeof(buf), "%.9f", kv.second - ci->second);
        out.append(buf, size_t(n));
      }
      int n = snprintf(buf, sizeof(buf), "%.9f", bind_log_.empty() ? 0.0 : tend - t0);
      out.append("],\"elapsed\":").append(buf, size_t(n));
      if (query_param(req.query, "full") == "2") {
        // [[created, bound], ...] seconds from the first create (bound -1: not yet), by creation
        std::vector<std::pair<double, double>> pts;
        for (const auto& kv : create_log_) {
          auto bi = bind_log_.find(kv.first);
          pts.emplace_back(kv.second - t0, bi == bind_log_.end() ? -1.0 : bi->second - t0);
        }
        std::sort(pts.begin(), pts.end());
        out.append(",\"timeline\":[");
        for (size_t k = 0; k < pts.size(); ++k) {
          n = snprintf(buf, sizeof(buf), "%s[%.6f,%.6f]", k ? "," : "", pts[k].first, pts[k].second);
          out.append(buf, size_t(n));
        }
        out.append("]");
      }
    }
    static const char* kProfName[kNProf] = {"bind", "event", "create", "delete", "get_list", "watch", "update",
                                             "bench", "job_create", "job_delete", "read", "flush"};
    out.append(",\"prof_s\":{");
    for (int q = 0; q < kNProf; ++q) {
      char buf[96];
      int n = snprintf(buf, sizeof(buf), "%s\"%s\":[%.6f,%llu]", q ? "," : "", kProfName[q], prof_[q],
                       static_cast<unsigned long long>(prof_n_[q]));
      out.append(buf, size_t(n));
    }
    out.append("}}");
    respond(c, 200, out);
    return;
  }
  if (p == "/debug/bench/reset") {
    BenchJob job;
    job.del = true;
    for (auto& k : bench_keys_)
      if (pods.objs.count(k)) job.keys.push_back(std::move(k));
    bench_keys_.clear();
    const size_t n = job.keys.size();
    jobs_.push_back(std::move(job));
    respond(c, 200, "{\"deleted\":" + std::to_string(n) + "}");
    return;
  }
  respond_err(c, {404, "NotFound", "no route for " + p});
}

// One slice (≤ 64 objects) of the oldest bench job: burst creation or reset deletion.
void Server::step_jobs() {
  if (jobs_.empty()) return;
  BenchJob& job = jobs_.front();
  ResState& pods = *by_key_["pods"];
  ApiErr err;
  if (job.del) {
    const size_t end = std::min(job.keys.size(), job.next + 64);
    for (; job.next < end; ++job.next) remove(pods, job.keys[job.next], &err);
    if (job.next >= job.keys.size()) {
      create_log_.clear();
      bind_log_.clear();
      jobs_.pop_front();
    }
    return;
  }
  if (job.next == 0) {
    create_log_.clear();
    bind_log_.clear();
    job.ts = rfc3339_now();
  }
  const size_t end = std::min(job.n, std::min(templates_.size(), job.next + 64));
  for (size_t i = job.next; i < end; ++i) {
    const std::string name = job.tag + "-" + std::to_string(i);
    if (!tmpl_text_.empty()) {
      const TmplText& tt = tmpl_text_[i];
      std::string key = tt.ns + "/" + name;
      if (pods.objs.count(key)) continue;
      char ub[24];
      snprintf(ub, sizeof(ub), "-%012llx", static_cast<unsigned long long>(++uid_counter_));
      const std::string rvs = next_rv();
      std::string text;
      text.reserve(tt.meta_rest.size() + tt.top_rest.size() + 160);
      text.append("{\"metadata\":{\"name\":").append(quoted(name));
      text.append(",\"uid\":").append(quoted(uid_prefix_ + ub));
      text.append(",\"resourceVersion\":");
      const size_t rv_at = text.size();
      text.append("\"").append(rvs).append("\"");
      text.append(",\"creationTimestamp\":\"").append(job.ts).append("\"");
      text.append(tt.meta_rest).append("}").append(tt.top_rest).append("}");
      SP s = make_stored_text(std::move(text), last_rv_, tt.ns, nullptr, {}, rv_at);
      pods.objs[key] = s;
      create_log_[key] = mono();
      bench_keys_.push_back(key);
      emit(pods, 'A', s, nullptr);
    } else {
      Value o = templates_[i];
      o.at("metadata").at("name") = Value::str(name);
      const std::string ns = o.at("metadata").get("namespace") ? o.at("metadata").at("namespace").s : "default";
      create(pods, std::move(o), "", &err);
      bench_keys_.push_back(ns + "/" + name);
    }
  }
  job.next = end;
  if (job.next >= std::min(job.n, templates_.size())) jobs_.pop_front();
}

void Server::handle(Conn* c, Request& req) {
  const std::string& path = req.path;
  if (path == "/healthz" || path == "/readyz" || path == "/livez") {
    respond(c, 200, "ok");
    return;
  }
  if (path == "/version") {
    respond(c, 200, "{\"major\":\"1\",\"minor\":\"20\",\"gitVersion\":\"v1.20.0-yoda-fake-native\"}");
    return;
  }
  if (path.rfind("/debug/bench/", 0) == 0) {
    handle_bench(c, req);
    return;
  }
  if (path == "/debug/bookmark") {
    auto it = by_key_.find(query_param(req.query, "resource", "pods"));
    if (it != by_key_.end()) send_bookmarks(*it->second);
    respond(c, 200, "{}");
    return;
  }
  if (!opt_.token.empty() && req.headers.get("authorization") != "Bearer " + opt_.token) {
    respond_err(c, {401, "Unauthorized", "Unauthorized"});
    return;
  }
  // /api/v1[/namespaces/NS]/RES[/NAME[/SUB]]  |  /apis/G/V[/namespaces/NS]/RES[/NAME[/SUB]]
  std::vector<std::string> parts;
  size_t s = 1;
  while (s <= path.size()) {
    size_t e = path.find('/', s);
    parts.push_back(url_decode(std::string_view(path).substr(s, e == std::string::npos ? std::string::npos : e - s)));
    if (e == std::string::npos) break;
    s = e + 1;
  }
  size_t i;
  std::string group;
  if (parts.size() >= 2 && parts[0] == "api" && parts[1] == "v1") {
    i = 2;
  } else if (parts.size() >= 3 && parts[0] == "apis") {
    group = parts[1];
    i = 3;
  } else {
    respond_err(c, {404, "NotFound", "no route for " + path});
    return;
  }
  std::string ns, name, sub;
  if (parts.size() > i + 2 && parts[i] == "namespaces") {
    ns = parts[i + 1];
    i += 2;
  }
  if (i >= parts.size() || parts.size() > i + 3) {
    respond_err(c, {404, "NotFound", "no route for " + path});
    return;
  }
  auto rit = by_path_.find(group + "/" + parts[i]);
  if (rit == by_path_.end()) {
    respond_err(c, {404, "NotFound", "no route for " + path});
    return;
  }
  ResState& rs = *rit->second;
  if (parts.size() > i + 1) name = parts[i + 1];
  if (parts.size() > i + 2) sub = parts[i + 2];
  const std::string& m = req.method;
  ApiErr err;
  if (m == "POST" && sub == "binding" && rs.def == &kRes[0]) {
    FlatDoc fd;
    if (!req.body.empty() && !fd.parse(req.body)) {
      respond_err(c, {400, "BadRequest", "invalid JSON body"});
      return;
    }
    if (bind(ns.empty() ? "default" : ns, name, req.body.empty() ? FlatDoc::View() : fd.root(), &err))
      respond(c, 201, "{\"kind\":\"Status\",\"apiVersion\":\"v1\",\"status\":\"Success\",\"code\":201}");
    else
      respond_err(c, err);
    return;
  }
  if (m == "GET") {
    if (name.empty()) {
      std::string w = query_param(req.query, "watch");
      if (w == "1" || w == "true") start_watch(c, rs, ns, req);
      else handle_list(c, rs, ns, req);
      return;
    }
    std::string key = rs.def->namespaced ? (ns.empty() ? "default" : ns) + "/" + name : name;
    auto it = rs.objs.find(key);
    if (it == rs.objs.end()) respond_err(c, {404, "NotFound", std::string(rs.def->key) + " " + key + " not found"});
    else respond(c, 200, it->second->text);
    return;
  }
  Value body;
  if (!req.body.empty()) {
    try {
      body = parse(req.body);
    } catch (const ParseError&) {
      respond_err(c, {400, "BadRequest", "invalid JSON body"});
      return;
    }
  }
  if (m == "POST") {
    SP s2 = create(rs, std::move(body), ns, &err);
    if (s2) respond(c, 201, s2->text);
    else respond_err(c, err);
    return;
  }
  if (m == "PUT") {
    SP s2 = update(rs, body, ns, name, sub == "status", &err);
    if (s2) respond(c, 200, s2->text);
    else respond_err(c, err);
    return;
  }
  if (m == "PATCH") {
    // application/merge-patch+json (RFC 7386) or application/strategic-merge-patch+json
    const bool strategic = req.headers.get("content-type").find("strategic-merge-patch") != std::string::npos;
    SP s2 = patch(rs, body, ns, name, &err, strategic);
    if (s2) respond(c, 200, s2->text);
    else respond_err(c, err);
    return;
  }
  if (m == "DELETE") {
    std::string key = rs.def->namespaced ? (ns.empty() ? "default" : ns) + "/" + name : name;
    SP s2 = remove(rs, key, &err);
    if (s2) respond(c, 200, s2->text);
    else respond_err(c, err);
    return;
  }
  respond_err(c, {405, "MethodNotAllowed", m});
}

int Server::run() {
  signal(SIGPIPE, SIG_IGN);
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);
  lfd_ = ::socket(AF_INET, SOCK_STREAM | SOCK_NONBLOCK | SOCK_CLOEXEC, 0);
  int one = 1;
  setsockopt(lfd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(uint16_t(opt_.port));
  if (inet_pton(AF_INET, opt_.host.c_str(), &a.sin_addr) != 1) {
    fprintf(stderr, "bad host %s\n", opt_.host.c_str());
    return 2;
  }
  if (::bind(lfd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 || ::listen(lfd_, 1024) != 0) {
    perror("bind/listen");
    return 2;
  }
  socklen_t al = sizeof(a);
  getsockname(lfd_, reinterpret_cast<sockaddr*>(&a), &al);
  int port = ntohs(a.sin_port);
  if (!opt_.port_file.empty()) {
    std::string tmp = opt_.port_file + ".tmp";
    FILE* f = fopen(tmp.c_str(), "w");
    if (f) {
      fprintf(f, "%d", port);
      fclose(f);
      rename(tmp.c_str(), opt_.port_file.c_str());
    }
  }
  printf("native fake apiserver listening on http://%s:%d\n", opt_.host.c_str(), port);
  fflush(stdout);
  ep_ = epoll_create1(EPOLL_CLOEXEC);
  epoll_event lev{};
  lev.events = EPOLLIN;
  lev.data.ptr = nullptr;
  epoll_ctl(ep_, EPOLL_CTL_ADD, lfd_, &lev);
  epoll_event evs[256];
  std::vector<char> buf(1 << 16);
  double next_tick = mono() + 0.5, next_bm = opt_.bookmark_interval_s > 0 ? mono() + opt_.bookmark_interval_s : 1e300;
  while (!g_stop) {
    int n = epoll_wait(ep_, evs, 256, jobs_.empty() ? 100 : 0);
    if (n < 0 && errno != EINTR) break;
    for (int k = 0; k < n; ++k) {
      if (evs[k].data.ptr == nullptr) {
        while (true) {
          int fd = ::accept4(lfd_, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
          if (fd < 0) break;
          setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          auto c = std::make_unique<Conn>();
          c->fd = fd;
          epoll_event ev{};
          ev.events = EPOLLIN | EPOLLRDHUP;
          ev.data.ptr = c.get();
          epoll_ctl(ep_, EPOLL_CTL_ADD, fd, &ev);
          conns_[fd] = std::move(c);
        }
        continue;
      }
      Conn* c = static_cast<Conn*>(evs[k].data.ptr);
      if (c->dead) continue;
      if (evs[k].events & EPOLLOUT) {
        const double tf = mono();
        flush(c);
        prof_[kFlush] += mono() - tf;
      }
      if (c->dead) continue;
      if (evs[k].events & (EPOLLIN | EPOLLRDHUP | EPOLLHUP | EPOLLERR)) {
        // everything in this block that is not a request's handler counts as reading
        const double tr = mono();
        double handled = 0;
        for (int q = 0; q < kNProf; ++q) handled -= prof_[q];
        while (!c->dead) {
          ssize_t r = ::recv(c->fd, buf.data(), buf.size(), 0);
          if (r < 0) {
            if (errno != EAGAIN && errno != EWOULDBLOCK) close_conn(c);
            break;
          }
          if (r == 0) {
            close_conn(c);
            break;
          }
          size_t off = 0;
          while (off < size_t(r) && !c->dead) {
            bool done = false;
            long used = c->rp.feed(buf.data() + off, size_t(r) - off, &done, c->req);
            if (used < 0) {
              respond(c, 400, status_text({400, "BadRequest", "malformed request"}), false);
              break;
            }
            off += size_t(used);
            if (done) {
              if (c->watcher) {
                // a request after a watch on the same connection: end the stream first
                finish_watch(c);
              }
              const int pk = prof_kind(c->req);
              const double th = mono();
              handle(c, c->req);
              prof_[pk] += mono() - th;
              prof_n_[pk]++;
              if (!c->req.keep_alive) c->close_after_write = true;
            }
          }
          if (size_t(r) < buf.size()) break;
        }
        for (int q = 0; q < kNProf; ++q) handled += prof_[q];
        prof_[kRead] += mono() - tr - handled;
      }
    }
    if (!jobs_.empty()) {
      // answers and watch events of this turn leave before the slice (≈ 64 objects of
      // work): a Binding's answer does not wait behind the burst's next creations
      flush_dirty();
      const int pk = jobs_.front().del ? kJobDelete : kJobCreate;
      const double tj = mono();
      step_jobs();
      prof_[pk] += mono() - tj;
      prof_n_[pk]++;
    }
    double now = mono();
    if (now >= next_tick) {
      next_tick = now + 0.5;
      for (auto& rs : res_) {
        std::vector<Watcher*> expired;
        for (Watcher* w : rs->watchers)
          if (!w->dead && now > w->deadline) expired.push_back(w);
        for (Watcher* w : expired) finish_watch(w->conn);
      }
    }
    if (now >= next_bm) {
      next_bm = now + opt_.bookmark_interval_s;
      for (auto& rs : res_) send_bookmarks(*rs);
    }
    flush_dirty();
    for (auto it = conns_.begin(); it != conns_.end();) {
      if (it->second->dead) it = conns_.erase(it);
      else ++it;
    }
  }
  for (auto& kv : conns_)
    if (!kv.second->dead) ::close(kv.second->fd);
  ::close(lfd_);
  ::close(ep_);
  return 0;
}

}  // namespace

int run_fake_apiserver(const FakeApiOptions& opt) {
  Server s(opt);
  return s.run();
}

}  // namespace yk
