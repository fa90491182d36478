// Build provenance: every native artefact embeds the hash of the sources it was built from
// (yoda_scheduler_amd/ops/build.py::source_hash passes -DYODA_BUILD_ID="<hash>"), so the
// importer can tell a library built from this tree from a stale one.
#pragma once
#ifndef YODA_BUILD_ID
#define YODA_BUILD_ID "unversioned"
#endif
