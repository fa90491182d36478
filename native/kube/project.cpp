// Pod projection (see project.hpp). Semantics follow models/pod.py exactly; every
// divergence is a fallback (`ok=false`), never a different answer.
#include "project.hpp"

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

bool starts_with(std::string_view s, std::string_view p) { return s.substr(0, p.size()) == p; }

bool is_basic(std::string_view k) { return k == "cpu" || k == "memory"; }

bool term_of(const Value* t, TermP& out) {
  out.clear();
  if (!t || t->t != Value::Obj) return t == nullptr || t->t == Value::Null;
  auto add = [&](const Value& e, bool field) -> bool {
    if (e.t != Value::Obj) return false;
    SelReqP r;
    const Value* k = e.get("key");
    if (k && k->t != Value::Str) return false;             // null key: Python keeps None
    std::string key = k ? k->s : "";
    if (field) {
      if (key != "metadata.name") return true;            // other fields: ignored (as in Python)
      key = "kubernetes.io/hostname";
    }
    r.key = key;
    const Value* op = e.get("operator");
    if (op && op->t != Value::Str) return false;
    r.op = op ? op->s : "In";
    const Value* vs = e.get("values");
    if (vs && vs->t == Value::Arr) {
      for (const auto& v : vs->arr) {
        if (v.t != Value::Str) return false;              // str(non-string) differs: Python decides
        r.values.push_back(v.s);
      }
    } else if (vs && vs->t != Value::Null) {
      return false;
    }
    out.push_back(std::move(r));
    return true;
  };
  if (const Value* me = t->get("matchExpressions"); me && me->t == Value::Arr) {
    for (const auto& e : me->arr)
      if (!add(e, false)) return false;
  }
  if (const Value* mf = t->get("matchFields"); mf && mf->t == Value::Arr) {
    for (const auto& e : mf->arr)
      if (!add(e, true)) return false;
  }
  return true;
}

bool kvs(const Value* m, std::vector<KV>& out) {
  if (!m || m->t == Value::Null) return true;
  if (m->t != Value::Obj) return false;
  out.reserve(m->obj.size());
  for (const auto& kv : m->obj) {
    if (kv.second.t != Value::Str) return false;
    out.emplace_back(kv.first, kv.second.s);
  }
  return true;
}

uint64_t meta_hash(const Value* meta) {
  uint64_t h = 0x51ed270b27cd1f47ull;
  if (!meta || meta->t != Value::Obj) return hash(meta ? *meta : Value(), h);
  for (const auto& m : meta->obj) {
    if (m.first == "resourceVersion" || m.first == "generation" || m.first == "managedFields") continue;
    h = hash(m.second, hash(Value::str(m.first), h));
  }
  return h;
}

}  // namespace

bool quantity_scaled(const Value& q, int scale, int64_t* out) {
  std::string_view s;
  if (q.t == Value::Str || q.t == Value::Num) s = q.s;
  else return false;
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

void project_pod(const Value& pod, PodProj& p) {
  p = PodProj();
  static const Value kEmpty = Value::object();
  const Value* meta = pod.get("metadata");
  const Value* spec = pod.get("spec");
  const Value& m = (meta && meta->t == Value::Obj) ? *meta : kEmpty;
  const Value& sp = (spec && spec->t == Value::Obj) ? *spec : kEmpty;
  p.ns = m.get("namespace") && m.get("namespace")->t == Value::Str ? m.get("namespace")->s : "default";
  p.name = std::string(m.sv("name"));
  p.uid = std::string(m.sv("uid"));
  if (p.uid.empty()) p.uid = p.ns + "/" + p.name;
  p.rv = std::string(m.sv("resourceVersion"));
  p.creation = std::string(m.sv("creationTimestamp"));
  if (const Value* d = m.get("deletionTimestamp")) p.deleting = d->truthy();
  std::string_view sched = sp.sv("schedulerName");
  p.sched = sched.empty() ? "default-scheduler" : std::string(sched);
  p.node = std::string(sp.sv("nodeName"));
  if (const Value* st = pod.get("status")) p.phase = std::string(st->sv("phase"));
  p.spec_meta_hash = hash(sp, meta_hash(meta));

  // ---- everything below: fall back to Python on any shape the projection does not mirror
  if (!kvs(m.get("labels"), p.labels)) return;
  if (const Value* a = m.get("annotations"); a && a->truthy()) {
    p.has_annotations = true;
    if (!kvs(a, p.annotations)) return;
  } else if (a && a->t != Value::Null && a->t != Value::Obj) {
    return;
  }
  if (const Value* pr = sp.get("priority"); pr && pr->truthy()) {
    bool ok;
    p.priority = pr->as_int(&ok);
    if (!ok || pr->t != Value::Num) return;
  }
  // requests: Σ containers, max with each init container, + overhead (models/pod.py::_requests)
  int64_t cpu = 0, mem = 0, nzc = 0, nzm = 0;
  auto reqs_of = [](const Value& c) -> const Value* {
    const Value* r = c.get("resources");
    if (!r || !r->truthy()) return nullptr;
    const Value* q = r->get("requests");
    return (q && q->truthy()) ? q : nullptr;
  };
  auto ext_in = [](const Value* r) {
    if (!r || r->t != Value::Obj) return false;
    for (const auto& kv : r->obj)
      if (!is_basic(kv.first)) return true;
    return false;
  };
  int flags = 0;
  if (const Value* cs = sp.get("containers"); cs && cs->t == Value::Arr) {
    for (const auto& c : cs->arr) {
      if (c.t != Value::Obj) return;
      const Value* r = reqs_of(c);
      if (r && r->t != Value::Obj) return;
      if (ext_in(r)) return;                          // extended resources: Python path
      int64_t v;
      if (const Value* q = r ? r->get("cpu") : nullptr) {
        if (!quantity_scaled(*q, 3, &v)) return;
        cpu += v;
        nzc += v;
      } else {
        nzc += kDefaultMilliCpu;
      }
      if (const Value* q = r ? r->get("memory") : nullptr) {
        if (!quantity_scaled(*q, 0, &v)) return;
        mem += v;
        nzm += v;
      } else {
        nzm += kDefaultMemory;
      }
      if (const Value* ports = c.get("ports"); ports && ports->t == Value::Arr) {
        for (const auto& pt : ports->arr) {
          if (pt.t != Value::Obj) return;
          const Value* hp = pt.get("hostPort");
          if (!hp || !hp->truthy()) continue;
          bool ok;
          PortP port;
          port.host_port = hp->as_int(&ok);
          if (!ok || hp->t != Value::Num) return;
          const Value* proto = pt.get("protocol");
          if (proto && proto->t != Value::Str) return;
          port.protocol = proto ? proto->s : "TCP";
          const Value* ip = pt.get("hostIP");
          if (ip && ip->t != Value::Str) return;
          port.host_ip = ip ? ip->s : "";
          p.ports.push_back(std::move(port));
        }
      }
    }
  } else if (const Value* cs2 = sp.get("containers"); cs2 && cs2->truthy()) {
    return;
  }
  if (const Value* ics = sp.get("initContainers"); ics && ics->t == Value::Arr) {
    for (const auto& c : ics->arr) {
      if (c.t != Value::Obj) return;
      const Value* r = reqs_of(c);
      if (r && r->t != Value::Obj) return;
      if (ext_in(r)) return;
      int64_t v = 0;
      const Value* q = r ? r->get("cpu") : nullptr;
      if (q && !quantity_scaled(*q, 3, &v)) return;
      if (!q) v = 0;
      cpu = std::max(cpu, v);
      nzc = std::max(nzc, q ? v : kDefaultMilliCpu);
      q = r ? r->get("memory") : nullptr;
      v = 0;
      if (q && !quantity_scaled(*q, 0, &v)) return;
      mem = std::max(mem, v);
      nzm = std::max(nzm, q ? v : kDefaultMemory);
    }
  }
  if (const Value* ov = sp.get("overhead"); ov && ov->truthy()) {
    if (ov->t != Value::Obj || ext_in(ov)) return;
    int64_t v;
    if (const Value* q = ov->get("cpu")) {
      if (!quantity_scaled(*q, 3, &v)) return;
      cpu += v;
      nzc += v;
    }
    if (const Value* q = ov->get("memory")) {
      if (!quantity_scaled(*q, 0, &v)) return;
      mem += v;
      nzm += v;
    }
  }
  p.cpu = cpu;
  p.mem = mem;
  p.nzc = nzc;
  p.nzm = nzm;
  if (!p.ports.empty()) flags |= PF_HOST_PORTS;

  if (const Value* ns = sp.get("nodeSelector"); ns && ns->truthy()) {
    p.has_node_selector = true;
    if (!kvs(ns, p.node_selector)) return;
  }
  if (const Value* aff = sp.get("affinity"); aff && aff->truthy()) {
    if (aff->t != Value::Obj) return;
    p.has_affinity = true;
    const Value* na = aff->get("nodeAffinity");
    if (na && na->truthy()) {
      if (na->t != Value::Obj) return;
      const Value* rq = na->get("requiredDuringSchedulingIgnoredDuringExecution");
      if (rq && rq->truthy()) {
        if (rq->t != Value::Obj) return;
        if (const Value* terms = rq->get("nodeSelectorTerms"); terms && terms->truthy()) {
          if (terms->t != Value::Arr) return;
          for (const auto& t : terms->arr) {
            TermP tp;
            if (!term_of(&t, tp)) return;
            p.req_terms.push_back(std::move(tp));
          }
        }
      }
      if (const Value* pf = na->get("preferredDuringSchedulingIgnoredDuringExecution"); pf && pf->truthy()) {
        if (pf->t != Value::Arr) return;
        for (const auto& x : pf->arr) {
          if (x.t != Value::Obj) return;
          int64_t w = 0;
          if (const Value* wv = x.get("weight")) {
            bool ok;
            w = wv->as_int(&ok);
            if (!ok || wv->t != Value::Num) return;
          }
          TermP tp;
          const Value* pref = x.get("preference");
          if (pref && pref->t != Value::Obj && pref->t != Value::Null) return;
          if (!term_of(pref && pref->truthy() ? pref : nullptr, tp)) return;
          p.pref_terms.emplace_back(w, std::move(tp));
        }
      }
    }
    const Value* pa = aff->get("podAffinity");
    const Value* paa = aff->get("podAntiAffinity");
    if ((pa && pa->truthy()) || (paa && paa->truthy())) flags |= PF_POD_AFFINITY;
    if (paa && paa->t == Value::Obj) {
      if (const Value* r = paa->get("requiredDuringSchedulingIgnoredDuringExecution"); r && r->truthy())
        flags |= PF_REQ_ANTI;
    }
  }
  if (const Value* tols = sp.get("tolerations"); tols && tols->truthy()) {
    if (tols->t != Value::Arr) return;
    for (const auto& t : tols->arr) {
      if (t.t != Value::Obj) return;
      TolP tp;
      const Value* k = t.get("key");
      if (k && k->t != Value::Str && k->t != Value::Null) return;
      tp.has_key = k && k->t == Value::Str && !k->s.empty();
      if (tp.has_key) tp.key = k->s;
      const Value* v = t.get("value");
      if (v && v->t != Value::Str && v->t != Value::Null) return;
      tp.value = (v && v->t == Value::Str) ? v->s : "";
      const Value* op = t.get("operator");
      if (op && op->t != Value::Str && op->t != Value::Null) return;
      tp.op = (op && op->t == Value::Str && !op->s.empty()) ? op->s : "Equal";
      const Value* ef = t.get("effect");
      if (ef && ef->t != Value::Str && ef->t != Value::Null) return;
      tp.effect = (ef && ef->t == Value::Str) ? ef->s : "";
      p.tolerations.push_back(std::move(tp));
    }
  }
  if (const Value* tsc = sp.get("topologySpreadConstraints"); tsc && tsc->truthy()) flags |= PF_SPREAD;
  if (const Value* vols = sp.get("volumes"); vols && vols->t == Value::Arr) {
    static const char* kDisks[] = {"gcePersistentDisk", "awsElasticBlockStore", "azureDisk", "cinder", "iscsi", "rbd"};
    for (const auto& v : vols->arr) {
      if (v.t != Value::Obj) return;
      if (v.get("persistentVolumeClaim") || v.get("ephemeral")) {
        flags |= PF_CLAIMS;
      } else {
        for (const char* d : kDisks)
          if (v.get(d)) {
            flags |= PF_DISKS;
            break;
          }
      }
    }
  }
  for (const auto& kv : p.labels)
    if (kv.first == "pod-group.scheduling.sigs.k8s.io") flags |= PF_POD_GROUP;
  if (const Value* owners = m.get("ownerReferences"); owners && owners->t == Value::Arr) {
    for (const auto& r : owners->arr) {
      if (r.t != Value::Obj) return;
      const Value* c = r.get("controller");
      std::string_view kind = r.sv("kind");
      if (c && c->truthy() && (kind == "ReplicationController" || kind == "ReplicaSet" || kind == "StatefulSet"))
        flags |= PF_CONTROLLER;
    }
  }
  p.flags = flags;
  p.ok = true;
}

}  // namespace yk
