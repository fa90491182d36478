"""Admission webhook for the ``scv/*`` pod-label API ("reject in validation
webhook"). The reference silently maps an invalid label to 0 and wraps negatives
(``pkg/yoda/filter/filter.go:60-82``), so ``scv/number: "abc"`` fits every node; the
scheduler keeps that behaviour for drop-in compatibility, and this webhook stops such pods
at admission instead. It also serves the port the reference opened but never used
(controller-runtime webhook server :9443, ``pkg/yoda/scheduler.go:53-58``).
"""
from .admission import AdmissionPolicy, review, validate_labels  # noqa: F401
