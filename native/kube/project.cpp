// Pod projection (see project.hpp). Semantics follow models/pod.py exactly; every
// divergence is a fallback (`ok=false`), never a different answer.
#include "project.hpp"

#include <cstring>

#include <cstring>

namespace yk {

namespace {

constexpr int64_t kDefaultMilliCpu = 100;                 // upstream schedutil non-zero defaults
constexpr int64_t kDefaultMemory = 200LL * 1024 * 1024;

// Python Decimal-compatible parse of "[+-]digits[.digits][e[+-]digits]" into N × 10^e.
bool parse_decimal(std::string_view s, __int128* n, int* e) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) neg = s[i++] == '-';
  __int128 v = 0;
  int digits = 0, frac = 0;
  bool any = false;
  for (; i < s.size() && s[i] >= '0' && s[i] <= '9'; ++i) {
    v = v * 10 + (s[i] - '0');
    any = true;
    if (v != 0 && ++digits > 30) return false;
  }
  if (i < s.size() && s[i] == '.') {
    ++i;
    for (; i < s.size() && s[i] >= '0' && s[i] <= '9'; ++i) {
      v = v * 10 + (s[i] - '0');
      ++frac;
      any = true;
      if (v != 0 && ++digits > 30) return false;
    }
  }
  if (!any) return false;
  int ex = 0;
  if (i < s.size() && (s[i] == 'e' || s[i] == 'E')) {
    ++i;
    bool eneg = false;
    if (i < s.size() && (s[i] == '+' || s[i] == '-')) eneg = s[i++] == '-';
    bool ed = false;
    for (; i < s.size() && s[i] >= '0' && s[i] <= '9'; ++i) {
      ex = ex * 10 + (s[i] - '0');
      ed = true;
      if (ex > 400) return false;
    }
    if (!ed) return false;
    if (eneg) ex = -ex;
  }
  if (i != s.size()) return false;
  *n = neg ? -v : v;
  *e = ex - frac;
  return true;
}

bool ceil_scaled(__int128 n, int e, int bin_shift, int64_t* out) {
  // value = n × 10^e × 2^bin_shift; ceil toward +inf
  if (bin_shift) {
    if (n > ((__int128)1 << 100) || n < -((__int128)1 << 100)) return false;
    n <<= bin_shift;
  }
  if (e >= 0) {
    for (int k = 0; k < e; ++k) {
      n *= 10;
      if (n > (__int128)INT64_MAX || n < (__int128)INT64_MIN) return false;
    }
  } else {
    __int128 d = 1;
    for (int k = 0; k < -e; ++k) {
      d *= 10;
      if (d > ((__int128)1 << 120)) return false;
    }
    n = n >= 0 ? (n + d - 1) / d : n / d;
  }
  if (n > (__int128)INT64_MAX || n < (__int128)INT64_MIN) return false;
  *out = int64_t(n);
  return true;
}

bool is_basic(std::string_view k) { return k == "cpu" || k == "memory"; }

// models/pod.py::normalize_image: an image without a tag or digest means ":latest"
std::string normalize_image(std::string_view name) {
  const size_t c = name.rfind(':'), sl = name.rfind('/');
  const long ci = c == std::string_view::npos ? -1 : (long)c, si = sl == std::string_view::npos ? -1 : (long)sl;
  std::string out(name);
  if (ci <= si && name.find('@') == std::string_view::npos) out += ":latest";
  return out;
}

// Uniform read-only view of a decoded JSON value, over the DOM (json.hpp) or the flat
// document (flatjson.hpp): one projection body serves both, so they cannot drift apart.
struct DomN {
  const Value* v = nullptr;
  explicit operator bool() const { return v != nullptr; }
  bool obj() const { return v && v->t == Value::Obj; }
  bool arr() const { return v && v->t == Value::Arr; }
  bool str_t() const { return v && v->t == Value::Str; }
  bool num_t() const { return v && v->t == Value::Num; }
  bool null_t() const { return v && v->t == Value::Null; }
  DomN get(std::string_view k) const { return DomN{v ? v->get(k) : nullptr}; }
  std::string_view sv(std::string_view k) const { return v ? v->sv(k) : std::string_view(); }
  std::string_view str() const { return v->s; }
  bool truthy() const { return v && v->truthy(); }
  int64_t as_int(bool* ok) const { return v->as_int(ok); }
  template <class F> bool each(F f) const {     // members (key, value) / elements ("", value)
    if (v->t == Value::Obj) {
      for (const auto& m : v->obj)
        if (!f(std::string_view(m.first), DomN{&m.second})) return false;
    } else if (v->t == Value::Arr) {
      for (const auto& x : v->arr)
        if (!f(std::string_view(), DomN{&x})) return false;
    }
    return true;
  }
  uint64_t hash(uint64_t h) const { return yk::hash(v ? *v : Value(), h); }
};

struct FlatN {
  FlatDoc::View v;
  explicit operator bool() const { return bool(v); }
  bool obj() const { return v.is(FlatDoc::Obj); }
  bool arr() const { return v.is(FlatDoc::Arr); }
  bool str_t() const { return v.is(FlatDoc::Str); }
  bool num_t() const { return v.is(FlatDoc::Num); }
  bool null_t() const { return v.is(FlatDoc::Null); }
  FlatN get(std::string_view k) const { return FlatN{v.get(k)}; }
  std::string_view sv(std::string_view k) const { return v ? v.sv(k) : std::string_view(); }
  std::string_view str() const { return v.str(); }
  bool truthy() const { return v.truthy(); }
  int64_t as_int(bool* ok) const { return v.as_int(ok); }
  template <class F> bool each(F f) const {
    const bool o = v.is(FlatDoc::Obj);
    for (FlatDoc::View c = v.first(); c; c = c.next())
      if (!f(o ? c.key() : std::string_view(), FlatN{c})) return false;
    return true;
  }
  uint64_t hash(uint64_t h) const { return v ? v.hash(h) : hash_mix(h, Value::Null); }
};

template <class N>
bool term_of(N t, TermP& out) {
  out.clear();
  if (!t || !t.obj()) return !t || t.null_t();
  auto add = [&](N e, bool field) -> bool {
    if (!e.obj()) return false;
    SelReqP r;
    N k = e.get("key");
    if (k && !k.str_t()) return false;                    // null key: Python keeps None
    std::string key = k ? std::string(k.str()) : "";
    if (field) key = "@" + key;                           // a field requirement (engine: '@' keys)
    r.key = key;
    N op = e.get("operator");
    if (op && !op.str_t()) return false;
    r.op = op ? std::string(op.str()) : "In";
    N vs = e.get("values");
    if (vs && vs.arr()) {
      bool ok = vs.each([&](std::string_view, N x) {
        if (!x.str_t()) return false;                     // str(non-string) differs: Python decides
        r.values.emplace_back(x.str());
        return true;
      });
      if (!ok) return false;
    } else if (vs && !vs.null_t()) {
      return false;
    }
    out.push_back(std::move(r));
    return true;
  };
  if (N me = t.get("matchExpressions"); me && me.arr()) {
    if (!me.each([&](std::string_view, N e) { return add(e, false); })) return false;
  }
  if (N mf = t.get("matchFields"); mf && mf.arr()) {
    if (!mf.each([&](std::string_view, N e) { return add(e, true); })) return false;
  }
  return true;
}

template <class N>
bool kvs(N m, std::vector<KV>& out) {
  if (!m || m.null_t()) return true;
  if (!m.obj()) return false;
  return m.each([&](std::string_view k, N v) {
    if (!v.str_t()) return false;
    out.emplace_back(std::string(k), std::string(v.str()));
    return true;
  });
}

// metav1.LabelSelector (models/selectors.py::LabelSelector): matchLabels + matchExpressions with
// In / NotIn / Exists / DoesNotExist; false on a shape the Python path must decide
template <class N>
bool label_selector_of(N ls, std::vector<KV>& labels, std::vector<SelReqP>& exprs) {
  if (!ls.obj()) return false;
  N ml = ls.get("matchLabels");
  if (ml && ml.truthy() && !kvs(ml, labels)) return false;
  if (N me = ls.get("matchExpressions"); me && me.truthy()) {
    if (!me.arr()) return false;
    return me.each([&](std::string_view, N e) {
      if (!e.obj()) return false;
      SelReqP r;
      N ek = e.get("key");
      if (ek && !ek.str_t()) return false;
      r.key = ek ? std::string(ek.str()) : "";
      N op = e.get("operator");
      if (op && !op.str_t()) return false;
      r.op = op ? std::string(op.str()) : "In";
      if (r.op != "In" && r.op != "NotIn" && r.op != "Exists" && r.op != "DoesNotExist") return false;
      N vs = e.get("values");
      if (vs && vs.truthy()) {
        if (!vs.arr()) return false;
        if (!vs.each([&](std::string_view, N v) {
              if (!v.str_t()) return false;
              r.values.emplace_back(v.str());
              return true;
            }))
          return false;
      }
      exprs.push_back(std::move(r));
      return true;
    });
  }
  return true;
}

// one PodAffinityTerm: topologyKey, namespaces, labelSelector
template <class N>
bool pod_term_of(N t, PodProj::PodTermP& x) {
  if (!t || t.null_t()) return true;            // `or {}`: an empty term
  if (!t.obj()) return false;
  N k = t.get("topologyKey");
  if (k && !k.str_t() && !k.null_t()) return false;
  x.key = k && k.str_t() ? std::string(k.str()) : "";
  if (N ns = t.get("namespaces"); ns && ns.truthy()) {
    if (!ns.arr()) return false;
    if (!ns.each([&](std::string_view, N v) {
          if (!v.str_t()) return false;
          x.ns.emplace_back(v.str());
          return true;
        }))
      return false;
  }
  N ls = t.get("labelSelector");
  if (ls && !ls.null_t()) {
    x.has_sel = true;
    if (!label_selector_of(ls, x.labels, x.exprs)) return false;
  }
  return true;
}

template <class N>
uint64_t meta_hash(N meta) {
  uint64_t h = 0x51ed270b27cd1f47ull;
  if (!meta || !meta.obj()) return meta.hash(h);
  meta.each([&](std::string_view k, N v) {
    if (k == "resourceVersion" || k == "generation" || k == "managedFields") return true;
    h = v.hash(hash_text(k, hash_mix(h, Value::Str)));    // == hash(Value::str(k), h)
    return true;
  });
  return h;
}

bool quantity_text(std::string_view s, int scale, int64_t* out);

template <class N>
bool quantity_of(N q, int scale, int64_t* out) {
  if (!q.str_t() && !q.num_t()) return false;
  return quantity_text(q.str(), scale, out);
}

}  // namespace

bool quantity_scaled(const Value& q, int scale, int64_t* out) { return quantity_of(DomN{&q}, scale, out); }

namespace {

bool quantity_text(std::string_view s, int scale, int64_t* out) {
  // Python: str(q).strip()
  while (!s.empty() && (s.front() == ' ' || s.front() == '\t' || s.front() == '\n')) s.remove_prefix(1);
  while (!s.empty() && (s.back() == ' ' || s.back() == '\t' || s.back() == '\n')) s.remove_suffix(1);
  if (s.empty()) {
    *out = 0;
    return true;
  }
  static const struct { const char* suf; int shift; } kBin[] = {
      {"Ki", 10}, {"Mi", 20}, {"Gi", 30}, {"Ti", 40}, {"Pi", 50}, {"Ei", 60}};
  __int128 n;
  int e;
  for (const auto& b : kBin) {
    if (s.size() >= 2 && s.substr(s.size() - 2) == b.suf) {
      if (!parse_decimal(s.substr(0, s.size() - 2), &n, &e)) return false;
      return ceil_scaled(n, e + scale, b.shift, out);
    }
  }
  int dec = 0;
  bool has_dec = true;
  switch (s.back()) {
    case 'n': dec = -9; break;
    case 'u': dec = -6; break;
    case 'm': dec = -3; break;
    case 'k': dec = 3; break;
    case 'M': dec = 6; break;
    case 'G': dec = 9; break;
    case 'T': dec = 12; break;
    case 'P': dec = 15; break;
    case 'E': dec = 18; break;
    default: has_dec = false;
  }
  if (has_dec) {
    if (!parse_decimal(s.substr(0, s.size() - 1), &n, &e)) return false;
    return ceil_scaled(n, e + dec + scale, 0, out);
  }
  if (!parse_decimal(s, &n, &e)) return false;
  return ceil_scaled(n, e + scale, 0, out);
}

template <class N>
uint64_t spec_hash(N sp, uint64_t h) {
  // a missing / non-object spec hashes as the empty object the DOM projection substitutes
  return sp.obj() ? sp.hash(h) : hash_mix(hash_mix(h, Value::Obj), 0);
}

constexpr uint64_t kLabelsSeed = 0x6c6162656c73ull;   // "labels"

template <class N>
uint64_t labels_hash_of(N labels) {
  const uint64_t h = labels.hash(kLabelsSeed);
  return h ? h : 1;
}

thread_local bool t_skip_hash = false;   // project_pod_nohash

template <class N>
void project_generic(N pod, PodProj& p) {
  p = PodProj();
  // the rarely-present fields go into one record, attached when the projection ends (every
  // early return included) if any is set
  struct ColdCommit {
    PodProj& p;
    PodProj::Cold c;
    ~ColdCommit() {
      if (!c.empty()) p.cold_ = std::make_shared<const PodProj::Cold>(std::move(c));
    }
  } commit{p, {}};
  PodProj::Cold& cx = commit.c;
  N meta = pod.get("metadata");
  N spec = pod.get("spec");
  const N m = meta.obj() ? meta : N{};
  const N sp = spec.obj() ? spec : N{};
  N nsv = m.get("namespace");
  p.ns = nsv && nsv.str_t() ? std::string(nsv.str()) : "default";
  p.name = std::string(m.sv("name"));
  p.uid = std::string(m.sv("uid"));
  if (p.uid.empty()) p.uid = p.ns + "/" + p.name;
  p.rv = std::string(m.sv("resourceVersion"));
  p.creation = std::string(m.sv("creationTimestamp"));
  if (N d = m.get("deletionTimestamp")) p.deleting = d.truthy();
  std::string_view sched = sp.sv("schedulerName");
  p.sched = sched.empty() ? "default-scheduler" : std::string(sched);
  p.node = std::string(sp.sv("nodeName"));
  if (N st = pod.get("status")) p.phase = std::string(st.sv("phase"));
  if (t_skip_hash) p.hash_pending = true;
  else p.spec_meta_hash = spec_hash(sp, meta_hash(meta));
  p.labels_hash = labels_hash_of(m.get("labels"));
  if (N st = pod.get("status"); st && st.obj()) {
    if (N cs = st.get("conditions"); cs && cs.arr()) {
      cs.each([&](std::string_view, N c) {
        if (!c.obj() || c.sv("type") != "PodScheduled") return true;
        static const auto kTrue = std::make_shared<const PodProj::SchedCond>(PodProj::SchedCond{"True", "", "", ""});
        const std::string_view status = c.sv("status");
        if (status == "True") {
          p.sched_cond = kTrue;
        } else {
          p.sched_cond = std::make_shared<const PodProj::SchedCond>(PodProj::SchedCond{
              std::string(status), std::string(c.sv("reason")), std::string(c.sv("message")),
              std::string(c.sv("lastTransitionTime"))});
        }
        return false;                       // the first one, as a by-type merge keeps one
      });
    }
  }

  // ---- everything below: fall back to Python on any shape the projection does not mirror
  if (!kvs(m.get("labels"), p.labels)) return;
  if (N a = m.get("annotations"); a && a.truthy()) {
    cx.has_annotations = true;
    if (!kvs(a, cx.annotations)) return;
  } else if (a && !a.null_t() && !a.obj()) {
    return;
  }
  if (N pr = sp.get("priority"); pr && pr.truthy()) {
    bool ok;
    p.priority = pr.as_int(&ok);
    if (!ok || !pr.num_t()) return;
  }
  // requests: Σ containers, max with each init container, + overhead (models/pod.py::_requests)
  int64_t cpu = 0, mem = 0, nzc = 0, nzm = 0;
  auto reqs_of = [](N c) -> N {
    N r = c.get("resources");
    if (!r || !r.truthy()) return N{};
    N q = r.get("requests");
    return (q && q.truthy()) ? q : N{};
  };
  // requests beyond cpu/memory (models/pod.py::ext_requests): Σ containers, max with each
  // init container, + overhead, as integer units
  std::vector<std::pair<std::string, int64_t>> ext;
  auto ext_add = [&](N r, bool take_max) {
    if (!r || !r.obj()) return true;
    return r.each([&](std::string_view k, N q) {
      if (is_basic(k)) return true;
      int64_t v;
      if (!quantity_of(q, 0, &v)) return false;
      for (auto& e : ext)
        if (e.first == k) {
          e.second = take_max ? std::max(e.second, v) : e.second + v;
          return true;
        }
      ext.emplace_back(std::string(k), take_max ? std::max<int64_t>(0, v) : v);
      return true;
    });
  };
  int flags = 0;
  if (N cs = sp.get("containers"); cs && cs.arr()) {
    bool ok = cs.each([&](std::string_view, N c) {
      if (!c.obj()) return false;
      ++p.containers;
      if (N im = c.get("image"); im && im.truthy()) {
        if (!im.str_t()) return false;
        p.images.push_back(normalize_image(im.str()));
      }
      N r = reqs_of(c);
      if (r && !r.obj()) return false;
      if (!ext_add(r, false)) return false;
      int64_t v;
      if (N q = r ? r.get("cpu") : N{}) {
        if (!quantity_of(q, 3, &v)) return false;
        cpu += v;
        nzc += v;
      } else {
        nzc += kDefaultMilliCpu;
      }
      if (N q = r ? r.get("memory") : N{}) {
        if (!quantity_of(q, 0, &v)) return false;
        mem += v;
        nzm += v;
      } else {
        nzm += kDefaultMemory;
      }
      if (N ports = c.get("ports"); ports && ports.arr()) {
        bool pok = ports.each([&](std::string_view, N pt) {
          if (!pt.obj()) return false;
          N hp = pt.get("hostPort");
          if (!hp || !hp.truthy()) return true;
          bool iok;
          PortP port;
          port.host_port = hp.as_int(&iok);
          if (!iok || !hp.num_t()) return false;
          N proto = pt.get("protocol");
          if (proto && !proto.str_t()) return false;
          port.protocol = proto ? std::string(proto.str()) : "TCP";
          N ip = pt.get("hostIP");
          if (ip && !ip.str_t()) return false;
          port.host_ip = ip ? std::string(ip.str()) : "";
          cx.ports.push_back(std::move(port));
          return true;
        });
        if (!pok) return false;
      }
      return true;
    });
    if (!ok) return;
  } else if (N cs2 = sp.get("containers"); cs2 && cs2.truthy()) {
    return;
  }
  if (N ics = sp.get("initContainers"); ics && ics.arr()) {
    bool ok = ics.each([&](std::string_view, N c) {
      if (!c.obj()) return false;
      N r = reqs_of(c);
      if (r && !r.obj()) return false;
      if (!ext_add(r, true)) return false;
      int64_t v = 0;
      N q = r ? r.get("cpu") : N{};
      if (q && !quantity_of(q, 3, &v)) return false;
      if (!q) v = 0;
      cpu = std::max(cpu, v);
      nzc = std::max(nzc, q ? v : kDefaultMilliCpu);
      q = r ? r.get("memory") : N{};
      v = 0;
      if (q && !quantity_of(q, 0, &v)) return false;
      mem = std::max(mem, v);
      nzm = std::max(nzm, q ? v : kDefaultMemory);
      return true;
    });
    if (!ok) return;
  }
  if (N ov = sp.get("overhead"); ov && ov.truthy()) {
    if (!ov.obj() || !ext_add(ov, false)) return;
    int64_t v;
    if (N q = ov.get("cpu")) {
      if (!quantity_of(q, 3, &v)) return;
      cpu += v;
      nzc += v;
    }
    if (N q = ov.get("memory")) {
      if (!quantity_of(q, 0, &v)) return;
      mem += v;
      nzm += v;
    }
  }
  p.cpu = cpu;
  p.mem = mem;
  p.nzc = nzc;
  p.nzm = nzm;
  for (auto& e : ext)
    if (e.second) cx.ext.push_back(std::move(e));
  if (!cx.ext.empty()) flags |= PF_EXTENDED;
  if (!cx.ports.empty()) flags |= PF_HOST_PORTS;

  if (N ns = sp.get("nodeSelector"); ns && ns.truthy()) {
    cx.has_node_selector = true;
    if (!kvs(ns, cx.node_selector)) return;
  }
  if (N aff = sp.get("affinity"); aff && aff.truthy()) {
    if (!aff.obj()) return;
    cx.has_affinity = true;
    N na = aff.get("nodeAffinity");
    if (na && na.truthy()) {
      if (!na.obj()) return;
      N rq = na.get("requiredDuringSchedulingIgnoredDuringExecution");
      if (rq && rq.truthy()) {
        if (!rq.obj()) return;
        if (N terms = rq.get("nodeSelectorTerms"); terms && terms.truthy()) {
          if (!terms.arr()) return;
          bool ok = terms.each([&](std::string_view, N t) {
            TermP tp;
            if (!term_of(t, tp)) return false;
            cx.req_terms.push_back(std::move(tp));
            return true;
          });
          if (!ok) return;
        }
      }
      if (N pf = na.get("preferredDuringSchedulingIgnoredDuringExecution"); pf && pf.truthy()) {
        if (!pf.arr()) return;
        bool ok = pf.each([&](std::string_view, N x) {
          if (!x.obj()) return false;
          int64_t w = 0;
          if (N wv = x.get("weight")) {
            bool iok;
            w = wv.as_int(&iok);
            if (!iok || !wv.num_t()) return false;
          }
          TermP tp;
          N pref = x.get("preference");
          if (pref && !pref.obj() && !pref.null_t()) return false;
          if (!term_of(pref && pref.truthy() ? pref : N{}, tp)) return false;
          cx.pref_terms.emplace_back(w, std::move(tp));
          return true;
        });
        if (!ok) return;
      }
    }
    N pa = aff.get("podAffinity");
    N paa = aff.get("podAntiAffinity");
    if ((pa && pa.truthy()) || (paa && paa.truthy())) flags |= PF_POD_AFFINITY;
    if (paa && paa.obj()) {
      if (N r = paa.get("requiredDuringSchedulingIgnoredDuringExecution"); r && r.truthy()) flags |= PF_REQ_ANTI;
    }
    // the terms themselves (native InterPodAffinity)
    auto terms_of = [&](N kind, std::vector<PodProj::PodTermP>& req, std::vector<PodProj::PodTermP>& pref) -> bool {
      if (!kind || !kind.truthy()) return true;
      if (!kind.obj()) return false;
      if (N r = kind.get("requiredDuringSchedulingIgnoredDuringExecution"); r && r.truthy()) {
        if (!r.arr()) return false;
        if (!r.each([&](std::string_view, N t) {
              PodProj::PodTermP x;
              if (!pod_term_of(t, x)) return false;
              req.push_back(std::move(x));
              return true;
            }))
          return false;
      }
      if (N r = kind.get("preferredDuringSchedulingIgnoredDuringExecution"); r && r.truthy()) {
        if (!r.arr()) return false;
        if (!r.each([&](std::string_view, N w) {
              if (!w.obj()) return false;
              PodProj::PodTermP x;
              if (N wv = w.get("weight")) {
                bool iok;
                if (!wv.num_t()) return false;
                x.weight = wv.as_int(&iok);
                if (!iok) return false;
              }
              N t = w.get("podAffinityTerm");
              if (!pod_term_of(t && t.truthy() ? t : N{}, x)) return false;
              pref.push_back(std::move(x));
              return true;
            }))
          return false;
      }
      return true;
    };
    if ((pa && pa.truthy()) || (paa && paa.truthy())) {
      cx.has_pod_aff = true;
      if (!terms_of(pa, cx.aff_req, cx.aff_pref) || !terms_of(paa, cx.anti_req, cx.anti_pref)) return;
    }
  }
  if (N tols = sp.get("tolerations"); tols && tols.truthy()) {
    if (!tols.arr()) return;
    bool ok = tols.each([&](std::string_view, N t) {
      if (!t.obj()) return false;
      TolP tp;
      N k = t.get("key");
      if (k && !k.str_t() && !k.null_t()) return false;
      tp.has_key = k && k.str_t() && !k.str().empty();
      if (tp.has_key) tp.key = std::string(k.str());
      N v = t.get("value");
      if (v && !v.str_t() && !v.null_t()) return false;
      tp.value = (v && v.str_t()) ? std::string(v.str()) : "";
      N op = t.get("operator");
      if (op && !op.str_t() && !op.null_t()) return false;
      tp.op = (op && op.str_t() && !op.str().empty()) ? std::string(op.str()) : "Equal";
      N ef = t.get("effect");
      if (ef && !ef.str_t() && !ef.null_t()) return false;
      tp.effect = (ef && ef.str_t()) ? std::string(ef.str()) : "";
      cx.tolerations.push_back(std::move(tp));
      return true;
    });
    if (!ok) return;
  }
  if (N tsc = sp.get("topologySpreadConstraints"); tsc && tsc.truthy()) {
    flags |= PF_SPREAD;
    if (!tsc.arr()) return;
    // plugins/spread_affinity.py::_parse_constraints + models/selectors.py::LabelSelector
    bool ok = tsc.each([&](std::string_view, N c) {
      if (!c.obj()) return false;
      PodProj::SpreadP x;
      N k = c.get("topologyKey");
      if (k && !k.str_t()) return false;
      x.key = k ? std::string(k.str()) : "";
      if (N ms = c.get("maxSkew")) {
        bool iok;
        if (!ms.num_t()) return false;
        x.max_skew = ms.as_int(&iok);
        if (!iok) return false;
      }
      N wu = c.get("whenUnsatisfiable");
      if (wu && !wu.str_t()) return false;
      const std::string_view w = wu ? wu.str() : std::string_view("DoNotSchedule");
      x.when = w == "DoNotSchedule" ? 0 : w == "ScheduleAnyway" ? 1 : 2;
      if (x.when == 0) flags |= PF_SPREAD_HARD;
      N ls = c.get("labelSelector");
      if (ls && !ls.null_t()) {
        x.has_sel = true;
        if (!label_selector_of(ls, x.labels, x.exprs)) return false;
      }
      cx.spread.push_back(std::move(x));
      return true;
    });
    if (!ok) return;
  }
  if (N vols = sp.get("volumes"); vols && vols.arr()) {
    static const char* kDisks[] = {"gcePersistentDisk", "awsElasticBlockStore", "azureDisk", "cinder", "iscsi", "rbd"};
    bool ok = vols.each([&](std::string_view, N v) {
      if (!v.obj()) return false;
      if (N pvc = v.get("persistentVolumeClaim")) {
        flags |= PF_CLAIMS;
        N cn = pvc.obj() ? pvc.get("claimName") : N{};
        cx.claims.emplace_back(!cn ? std::string() : cn.str_t() ? std::string(cn.str()) : std::string("\x01"));
        cx.claim_pvc.push_back(1);
      } else if (v.get("ephemeral")) {
        flags |= PF_CLAIMS;
        N vn = v.get("name");
        cx.claims.emplace_back(vn && !vn.str_t() ? std::string("\x01") : p.name + "-" + std::string(vn ? vn.str() : ""));
        cx.claim_pvc.push_back(0);
      } else {
        for (const char* d : kDisks)
          if (v.get(d)) {
            flags |= PF_DISKS;
            break;
          }
      }
      return true;
    });
    if (!ok) return;
  }
  for (const auto& kv : p.labels)
    if (kv.first == "pod-group.scheduling.sigs.k8s.io") flags |= PF_POD_GROUP;
  if (N owners = m.get("ownerReferences"); owners && owners.arr()) {
    PodProj::Owners o;
    bool ok = owners.each([&](std::string_view, N r) {
      if (!r.obj()) return false;
      N c = r.get("controller");
      std::string_view kind = r.sv("kind");
      const bool ctl = c && c.truthy();
      if (ctl && (kind == "ReplicationController" || kind == "ReplicaSet" || kind == "StatefulSet"))
        flags |= PF_CONTROLLER;
      if (ctl && !o.has_owner) {            // DefaultSelector reads the first controller only
        o.has_owner = true;
        o.owner_api = std::string(r.sv("apiVersion"));
        o.owner_kind = std::string(kind);
        o.owner_name = std::string(r.sv("name"));
        o.owner_uid = std::string(r.sv("uid"));
      }
      if (ctl && !o.has_avoid && (kind == "ReplicationController" || kind == "ReplicaSet")) {
        o.has_avoid = true;                 // NodePreferAvoidPods: the first RC / RS controller
        o.avoid_kind = std::string(kind);
        o.avoid_uid = std::string(r.sv("uid"));
      }
      return true;
    });
    if (o.has_owner || o.has_avoid) p.owners = std::make_shared<const PodProj::Owners>(std::move(o));
    if (!ok) return;
  }
  p.flags = flags;
  p.ok = true;
}

}  // namespace

void project_pod(const Value& pod, PodProj& p) { project_generic(DomN{&pod}, p); }

void project_pod(const FlatDoc::View& pod, PodProj& p) { project_generic(FlatN{pod}, p); }

void project_pod_nohash(const FlatDoc::View& pod, PodProj& p) {
  t_skip_hash = true;
  project_generic(FlatN{pod}, p);
  t_skip_hash = false;
}

uint64_t spec_meta_hash_of(std::string_view text) {
  FlatDoc d;
  if (!d.parse(text)) return 0;
  const FlatN pod{d.root()};
  const FlatN meta = pod.get("metadata");
  const FlatN spec = pod.get("spec");
  return spec_hash(spec.obj() ? spec : FlatN{}, meta_hash(meta));
}

void project_identity(const FlatDoc::View& pod, PodProj& p) {
  p = PodProj();
  const FlatDoc::View meta = pod.get("metadata"), spec = pod.get("spec");
  const FlatDoc::View m = meta.is(FlatDoc::Obj) ? meta : FlatDoc::View();
  const FlatDoc::View sp = spec.is(FlatDoc::Obj) ? spec : FlatDoc::View();
  const FlatDoc::View nsv = m ? m.get("namespace") : FlatDoc::View();
  p.ns = nsv && nsv.is(FlatDoc::Str) ? std::string(nsv.str()) : "default";
  p.name = std::string(m ? m.sv("name") : std::string_view());
  p.uid = std::string(m ? m.sv("uid") : std::string_view());
  if (p.uid.empty()) p.uid = p.ns + "/" + p.name;
  p.rv = std::string(m ? m.sv("resourceVersion") : std::string_view());
  p.creation = std::string(m ? m.sv("creationTimestamp") : std::string_view());
  if (m)
    if (const FlatDoc::View d = m.get("deletionTimestamp")) p.deleting = d.truthy();
  const std::string_view sched = sp ? sp.sv("schedulerName") : std::string_view();
  p.sched = sched.empty() ? "default-scheduler" : std::string(sched);
  p.node = std::string(sp ? sp.sv("nodeName") : std::string_view());
  if (const FlatDoc::View st = pod.get("status")) p.phase = std::string(st.sv("phase"));
  p.labels_hash = labels_hash_of(FlatN{m ? m.get("labels") : FlatDoc::View()});
}

namespace {

// A skipping scanner over JSON text: walks members without building a document. Strings with
// escapes in a key or a value the caller reads make it give up (the caller then parses).
struct Skim {
  const char* p;
  const char* e;

  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  // any byte of an 8-byte word that is '"' or '\\' (SWAR: most strings here are short, so a
  // word at a time beats a memchr call per string)
  static bool quote_or_bs(uint64_t w) {
    constexpr uint64_t ones = 0x0101010101010101ull, highs = 0x8080808080808080ull;
    const uint64_t q = w ^ (ones * '"'), b = w ^ (ones * '\\');
    return (((q - ones) & ~q) | ((b - ones) & ~b)) & highs;
  }
  // p at '"': the raw content, whether it holds a backslash; p past the closing quote
  bool str(std::string_view* out, bool* esc) {
    if (p >= e || *p != '"') return false;
    const char* s = ++p;
    bool bs = false;
    for (;;) {
      while (e - p >= 8) {
        uint64_t w;
        std::memcpy(&w, p, 8);
        if (quote_or_bs(w)) break;
        p += 8;
      }
      while (p < e && *p != '"' && *p != '\\') ++p;
      if (p >= e) return false;
      if (*p == '\\') {                 // an escape: skip the escaped character
        bs = true;
        p += 2;
        if (p > e) return false;
        continue;
      }
      *out = std::string_view(s, size_t(p - s));
      *esc = bs;
      ++p;
      return true;
    }
  }
  bool skip() {
    ws();
    if (p >= e) return false;
    const char c = *p;
    std::string_view sv;
    bool esc;
    if (c == '"') return str(&sv, &esc);
    if (c == '{' || c == '[') {
      int depth = 0;
      while (p < e) {
        const char ch = *p;
        if (ch == '"') {
          if (!str(&sv, &esc)) return false;
          continue;
        }
        if (ch == '{' || ch == '[') {
          ++depth;
        } else if (ch == '}' || ch == ']') {
          if (--depth == 0) {
            ++p;
            return true;
          }
        }
        ++p;
      }
      return false;
    }
    const char* s = p;
    while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n' && *p != '\r' && *p != '\t') ++p;
    return p > s;
  }
  // members of the object at p: on(key) consumes the value and returns true, or returns false
  // to have it skipped. False on malformed input or an escaped key.
  template <class F>
  bool object(F&& on) {
    ws();
    if (p >= e || *p != '{') return false;
    ++p;
    ws();
    if (p < e && *p == '}') {
      ++p;
      return true;
    }
    for (;;) {
      ws();
      std::string_view k;
      bool esc;
      if (!str(&k, &esc) || esc) return false;
      ws();
      if (p >= e || *p != ':') return false;
      ++p;
      ws();
      if (!on(k) && !skip()) return false;
      ws();
      if (p < e && *p == ',') {
        ++p;
        continue;
      }
      if (p < e && *p == '}') {
        ++p;
        return true;
      }
      return false;
    }
  }
  // a member value read as FlatDoc's sv(): the string, or "" for any other type
  bool sv(std::string_view* out, bool* ok) {
    ws();
    if (p < e && *p == '"') {
      bool esc;
      if (!str(out, &esc)) return false;
      if (esc) *ok = false;
      return true;
    }
    *out = std::string_view();
    return skip();
  }
  // FlatDoc::View::truthy() of the value
  bool truthy(bool* out) {
    ws();
    if (p >= e) return false;
    const char* s = p;
    const char c = *p;
    if (!skip()) return false;
    const std::string_view t(s, size_t(p - s));
    if (c == '"') *out = t.size() > 2;
    else if (c == '{' || c == '[') *out = t.find_first_not_of(" \n\r\t", 1) != t.size() - 1;
    else if (c == 't') *out = true;
    else if (c == 'f' || c == 'n') *out = false;
    else *out = t.find_first_of("123456789") != std::string_view::npos;
    return true;
  }
};

}  // namespace

// labels_hash_of over a raw metadata.labels span (empty: no labels member); 0 when it does not parse
uint64_t labels_span_hash(std::string_view raw) {
  if (raw.empty()) return labels_hash_of(FlatN{FlatDoc::View()});
  {
    // the usual shape — an object of plain strings — hashed straight from the text, in the
    // order and with the mixing FlatDoc::View::hash uses (Obj, then per member key, Str, value,
    // then the member count): no document is built for an echo's labels
    Skim k{raw.data(), raw.data() + raw.size()};
    uint64_t h = hash_mix(kLabelsSeed, FlatDoc::Obj);
    uint64_t cnt = 0;
    bool plain = true;
    const bool parsed = k.object([&](std::string_view key) -> bool {
      std::string_view v;
      bool esc = false;
      k.ws();
      if (k.p >= k.e || *k.p != '"' || !k.str(&v, &esc) || esc) {
        plain = false;
        k.p = k.e;                    // stop: the parser below decides
        return true;
      }
      h = hash_text(v, hash_mix(hash_text(key, h), FlatDoc::Str));
      ++cnt;
      return true;
    });
    if (parsed && plain) {
      k.ws();
      if (k.p == k.e) {
        h = hash_mix(h, cnt);
        return h ? h : 1;
      }
    }
  }
  FlatDoc d;
  if (!d.parse(raw)) return 0;
  return labels_hash_of(FlatN{d.root()});
}

bool scan_watch_identity(std::string_view line, char* type, std::string_view* obj, PodProj& p, bool only_md) {
  // p: default-constructed by the caller (resetting a PodProj here cost a quarter of the scan)
  bool labels_seen = false;
  std::string_view labels_raw;
  Skim k{line.data(), line.data() + line.size()};
  bool ok = true, have_type = false, have_obj = false;
  std::string_view tname;
  bool seen_meta = false, seen_spec = false, seen_status = false;
  bool ns_set = false;
  int seen = 0;
  std::string_view ns, name, uid, rv, creation, sched, node, phase;
  bool deleting = false;
  auto meta = [&](std::string_view key) -> bool {
    if (key == "labels" && !labels_seen) {
      labels_seen = true;
      k.ws();
      const char* s0 = k.p;
      if (!k.skip()) return ok = false;
      labels_raw = std::string_view(s0, size_t(k.p - s0));
      return true;
    }
    if (key == "namespace") {
      if (ns_set) return false;
      ns_set = true;
      k.ws();
      if (k.p < k.e && *k.p == '"') {
        bool esc;
        if (!k.str(&ns, &esc)) return ok = false;
        if (esc) ok = false;
        return true;
      }
      ns = "default";
      return k.skip() || (ok = false);
    }
    // the first occurrence of a key counts, as FlatDoc::View::get finds it
    const int bit = key == "name" ? 1 : key == "uid" ? 2 : key == "resourceVersion" ? 4 : key == "creationTimestamp" ? 8
                    : key == "deletionTimestamp" ? 16 : 0;
    if (!bit || (seen & bit)) return false;
    seen |= bit;
    if (bit == 16) return k.truthy(&deleting) || (ok = false);
    std::string_view* f = bit == 1 ? &name : bit == 2 ? &uid : bit == 4 ? &rv : &creation;
    return k.sv(f, &ok) || (ok = false);
  };
  auto spec = [&](std::string_view key) -> bool {
    const int bit = key == "schedulerName" ? 32 : key == "nodeName" ? 64 : 0;
    if (!bit || (seen & bit)) return false;
    seen |= bit;
    return k.sv(bit == 32 ? &sched : &node, &ok) || (ok = false);
  };
  auto status = [&](std::string_view key) -> bool {
    if (key != "phase" || (seen & 128)) return false;
    seen |= 128;
    return k.sv(&phase, &ok) || (ok = false);
  };
  // DELETED (transport mode): the object's closing brace, found from the line's end — a watch
  // line is {"type":..,"object":{..}} — so the scan can stop after metadata (the lane drops a
  // deleted pod by key; sched / node / phase are filled on first use, PodProj::ident_partial)
  const char* obj_close = nullptr;
  auto pod = [&](std::string_view key) -> bool {
    k.ws();
    const bool is_obj = k.p < k.e && *k.p == '{';
    if (key == "metadata" && !seen_meta) {
      seen_meta = true;
      if (is_obj) {
        if (!k.object(meta)) return ok = false;
        if (obj_close) {
          k.p = obj_close;           // the object() loop then sees its closing brace
          p.ident_partial = true;
        }
        return true;
      }
    } else if (key == "spec" && !seen_spec) {
      seen_spec = true;
      if (is_obj) return k.object(spec) || (ok = false);
    } else if (key == "status" && !seen_status) {
      seen_status = true;
      if (is_obj) return k.object(status) || (ok = false);
    }
    return false;
  };
  auto top = [&](std::string_view key) -> bool {
    if (key == "type" && !have_type) {
      have_type = true;
      bool esc;
      k.ws();
      if (k.p >= k.e || *k.p != '"' || !k.str(&tname, &esc) || esc) return ok = false, true;
      // the caller only wants echoes and deletions: any other type ends the scan here (the
      // type leads the apiserver's watch line, so an ADDED pod is not scanned twice)
      if (only_md && tname != "MODIFIED" && tname != "DELETED") {
        ok = false;
        k.p = k.e;
      }
      return true;
    }
    if (key == "object" && !have_obj) {
      have_obj = true;
      k.ws();
      const char* s = k.p;
      if (only_md && have_type && tname == "DELETED" && k.p < k.e && *k.p == '{') {
        const char* q = k.e;
        while (q > k.p && (q[-1] == ' ' || q[-1] == '\n' || q[-1] == '\r' || q[-1] == '\t')) --q;
        if (q > k.p && q[-1] == '}') {       // the line's closing brace
          --q;
          while (q > k.p && (q[-1] == ' ' || q[-1] == '\n' || q[-1] == '\r' || q[-1] == '\t')) --q;
          if (q > k.p + 1 && q[-1] == '}') obj_close = q - 1;
        }
      }
      if (!k.object(pod)) return ok = false, true;
      *obj = std::string_view(s, size_t(k.p - s));
      return true;
    }
    return false;
  };
  if (!k.object(top) || !ok || !have_type || !have_obj) return false;
  k.ws();
  if (k.p != k.e) return false;
  *type = tname == "ADDED" ? 'A' : tname == "MODIFIED" ? 'M' : tname == "DELETED" ? 'D' : tname == "BOOKMARK" ? 'B'
          : tname == "ERROR" ? 'E' : '?';
  p.ns = ns_set ? std::string(ns) : "default";
  p.name = std::string(name);
  p.uid = std::string(uid);
  if (p.uid.empty()) p.uid = p.ns + "/" + p.name;
  p.rv = std::string(rv);
  p.creation = std::string(creation);
  p.deleting = deleting;
  p.sched = sched.empty() ? "default-scheduler" : std::string(sched);
  p.node = std::string(node);
  p.phase = std::string(phase);
  p.labels_hash = seen_meta ? labels_span_hash(labels_seen ? labels_raw : std::string_view()) : 0;
  return true;
}

void merge_non_identity(PodProj& d, PodProj&& s) {
  d.labels = std::move(s.labels);
  d.cpu = s.cpu;
  d.mem = s.mem;
  d.nzc = s.nzc;
  d.nzm = s.nzm;
  d.priority = s.priority;
  d.images = std::move(s.images);
  d.containers = s.containers;
  d.owners = std::move(s.owners);
  d.cold_ = std::move(s.cold_);
  d.flags = s.flags;
  d.spec_meta_hash = s.spec_meta_hash;
  d.ok = s.ok;
  d.sched_cond = std::move(s.sched_cond);
}

bool project_pod_text(std::string_view text, PodProj& p) {
  FlatDoc d;
  if (!d.parse(text)) return false;
  project_pod(d.root(), p);
  return true;
}

}  // namespace yk
