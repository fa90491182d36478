// Pod projection: everything the scheduling cycle reads from a v1.Pod, computed in C++
// from the watch event's JSON so the Python control plane never decodes a pod on the hot
// path. Mirrors yoda_scheduler_amd/models/pod.py::PodInfo.from_obj field for field; a pod
// using something the projection does not cover (extended resources, quantities outside
// the exact-decimal range) sets `ok=false` and Python falls back to json + from_obj.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "flatjson.hpp"
#include "json.hpp"

namespace yk {

// pod feature flags (models/pod.py PF_*)
enum : int {
  PF_HOST_PORTS = 1,
  PF_SPREAD = 2,
  PF_POD_AFFINITY = 4,
  PF_CLAIMS = 8,
  PF_DISKS = 16,
  PF_CONTROLLER = 32,
  PF_EXTENDED = 64,
  PF_POD_GROUP = 128,
  PF_REQ_ANTI = 256,    // required pod anti-affinity (symmetry check of other pods)
  PF_SPREAD_HARD = 512, // a DoNotSchedule topology spread constraint
};

using KV = std::pair<std::string, std::string>;

struct SelReqP {
  std::string key, op;
  std::vector<std::string> values;
};
using TermP = std::vector<SelReqP>;

struct TolP {
  bool has_key = false;
  std::string key, value, op, effect;
};

struct PortP {
  int64_t host_port = 0;
  std::string protocol, host_ip;
};

struct PodProj {
  bool ok = false;                  // full projection available
  std::string uid, ns, name, rv, sched, node, phase, creation;
  bool deleting = false;            // metadata.deletionTimestamp set
  std::vector<KV> labels;
  int64_t cpu = 0, mem = 0, nzc = 0, nzm = 0, priority = 0;
  int flags = 0;
  uint64_t spec_meta_hash = 0;      // upstream isPodUpdated: spec + metadata minus volatile fields
  // the hash was not computed (a lane-attached ADDED: the lane never compares it); PodEv::hash()
  // computes it from the raw object on first use
  bool hash_pending = false;
  // structural hash of metadata.labels (0: unknown). Set by the full projection and by the
  // watch identity scanner too, so a light event tells whether a pod's labels changed
  // without being projected (the lane's per-node selector census keeps the older projection)
  uint64_t labels_hash = 0;
  // a DELETED line scanned up to metadata only (scan_watch_identity): sched / node / phase are
  // not read yet — PodEv::full() fills them. Nothing reads them of a deletion before that: the
  // lane drops its entry by key, and whatever goes on to Python is completed first.
  bool ident_partial = false;
  // status.conditions' PodScheduled entry (upstream updatePod compares the condition it would
  // write with the pod's current one); null: none. Only a False condition's reason, message and
  // lastTransitionTime are read, so every True one shares one record (no allocation per pod)
  struct SchedCond {
    std::string status, reason, msg, ltt;
  };
  std::shared_ptr<const SchedCond> sched_cond;
  // default-plugin inputs (models/pod.py PodInfo.images / containers): normalized images of
  // spec.containers and their count
  std::vector<std::string> images;
  int32_t containers = 0;
  // the controller references (null: the pod has no controller ownerReference); one record, so
  // a pod without one carries 16 bytes for them
  struct Owners {
    bool has_owner = false;
    std::string owner_api, owner_kind, owner_name, owner_uid;
    bool has_avoid = false;
    std::string avoid_kind, avoid_uid;
  };
  std::shared_ptr<const Owners> owners;
  struct SpreadP {
    std::string key;
    int64_t max_skew = 1;
    int when = 0;                   // 0 DoNotSchedule, 1 ScheduleAnyway, 2 another value (in neither list)
    bool has_sel = false;           // false: nil labelSelector (matches nothing)
    std::vector<KV> labels;
    std::vector<SelReqP> exprs;
  };
  // spec.affinity.podAffinity / podAntiAffinity terms (plugins/spread_affinity.py::_terms)
  struct PodTermP {
    std::string key;
    std::vector<std::string> ns;    // empty: the pod's own namespace
    bool has_sel = false;           // false: nil labelSelector (matches nothing)
    std::vector<KV> labels;
    std::vector<SelReqP> exprs;
    int64_t weight = 1;
  };
  // Everything else a full projection reads — present on few pods, so it lives in one record
  // behind a pointer (null: all empty). Every watch event carries a PodProj from the I/O
  // thread to the lane thread; a pod's echo and its deletion only need the identity fields
  // above, and the bytes of this record would be paid on each (tests/test_engine_alloc.py)
  struct Cold {
    bool has_annotations = false;
    std::vector<KV> annotations;
    bool has_node_selector = false;
    std::vector<KV> node_selector;
    bool has_affinity = false;        // spec.affinity truthy → terms lists (maybe empty)
    std::vector<TermP> req_terms;
    std::vector<std::pair<int64_t, TermP>> pref_terms;
    std::vector<TolP> tolerations;
    std::vector<PortP> ports;
    // the claims of spec.volumes (plugins/volumes.py::_claim_names): a persistentVolumeClaim's
    // claimName, a generic ephemeral volume's "<pod>-<volume>"; "\x01" for a name that is not a
    // string (it names no PersistentVolumeClaim the lane could call inert)
    std::vector<std::string> claims;
    std::vector<char> claim_pvc;      // per claim: 1 a persistentVolumeClaim volume, 0 an ephemeral one
    // requests beyond cpu/memory (non-zero, models/pod.py::ext_requests)
    std::vector<std::pair<std::string, int64_t>> ext;
    std::vector<SpreadP> spread;      // spec.topologySpreadConstraints
    bool has_pod_aff = false;
    std::vector<PodTermP> aff_req, anti_req, aff_pref, anti_pref;
    bool empty() const {
      return !has_annotations && annotations.empty() && !has_node_selector && node_selector.empty() && !has_affinity &&
             req_terms.empty() && pref_terms.empty() && tolerations.empty() && ports.empty() && claims.empty() &&
             claim_pvc.empty() && ext.empty() && spread.empty() && !has_pod_aff && aff_req.empty() &&
             anti_req.empty() && aff_pref.empty() && anti_pref.empty();
    }
  };
  std::shared_ptr<const Cold> cold_;
  const Cold& cold() const {
    static const Cold kNone;
    return cold_ ? *cold_ : kNone;
  }
};

// Quantity → ceil(q × 10^scale) with exact decimal arithmetic (scale 3: CPU millicores,
// 0: bytes). False when the text is outside what the projection handles exactly.
bool quantity_scaled(const Value& q, int scale, int64_t* out);

// Fills `p` from a decoded pod object. Identity fields (uid/ns/name/rv/node/phase/sched,
// hash) are always set; `p.ok` tells whether the rest is complete.
void project_pod(const Value& pod, PodProj& p);
// The same projection over the flat document (the watch stream's decode path).
void project_pod(const FlatDoc::View& pod, PodProj& p);
// The same, without the spec / metadata hash (hash_pending): the watch stream's ADDED events
// when a native lane is attached — the hash only serves Python's update comparisons
void project_pod_nohash(const FlatDoc::View& pod, PodProj& p);
// spec_meta_hash of a pod object's text (0 if it does not parse)
uint64_t spec_meta_hash_of(std::string_view text);
// Parse + project one pod object's JSON text; false when the text is not JSON.
bool project_pod_text(std::string_view text, PodProj& p);
// Identity fields only (ns, name, uid, rv, creation, deleting, scheduler, node, phase); `ok`
// stays false and the hash 0 — see PodEv::full().
void project_identity(const FlatDoc::View& pod, PodProj& p);
// The watch stream's light path: one skipping scan of an event line {"type":..,"object":{..}}
// for the event type, the object's text span and the pod's identity fields (as
// project_identity reads them), building no document. False when the line needs the parser
// (escapes in a field it reads, malformed text): the caller then takes the FlatDoc path.
// `p` must be default-constructed (the scan only sets the fields it reads).
bool scan_watch_identity(std::string_view line, char* type, std::string_view* obj, PodProj& p,
                         bool only_md = false);
// Fill everything but the identity fields from a full projection (`src` is consumed).
void merge_non_identity(PodProj& dst, PodProj&& src);

}  // namespace yk
