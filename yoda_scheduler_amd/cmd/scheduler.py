"""``yoda-scheduler`` — drop-in replacement of the reference binary.

The reference's entry is ``register.Register()`` → ``app.NewSchedulerCommand(
app.WithPlugin(yoda.Name, yoda.New))`` and ``command.Execute()`` (``cmd/scheduler/main.go:12-21``,
``pkg/register/register.go:9-13``): the full kube-scheduler with the ``yoda`` plugin added.
:func:`new_scheduler_command` is the same composition point — out-of-tree plugins are
passed as ``(name, factory)`` pairs — and the resulting command accepts the flags the
deployment uses (``--config``, ``--v``, ``deploy/yoda-scheduler.yaml:60-63``) plus the
common kube-scheduler flags; unknown upstream flags are accepted with a warning so existing
manifests keep working.

Extra (dev) mode: ``--fake-cluster N`` runs against an in-process fake apiserver with N
synthetic 8×MI355X nodes (optionally exposed over HTTP with ``--fake-apiserver-port``).
"""
from __future__ import annotations

import argparse
import asyncio
import logging
import signal
import sys
import time
from typing import Callable, Optional, Sequence

from ..framework.config import apply_policy, default_config, load_config, parse_duration, resolve_policy_configmap
from ..framework.policy import load_policy_file
from ..framework.leader import LeaderElector
from ..framework.registry import Registry, default_registry
from ..framework.scheduler import Scheduler
from ..utils import klog
from ..utils.metrics import pod_resource_metrics
from ..utils.serving import StatusServer

log = logging.getLogger("yoda.cmd")

PluginOption = tuple[str, Callable]


def _bool(v: str) -> bool:
    return str(v).lower() in ("1", "true", "yes", "on")


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(prog="yoda-scheduler", description="MI355X-native yoda scheduler (kube-scheduler "
                                "compatible)")
    p.add_argument("--config", default="", help="KubeSchedulerConfiguration file (v1beta1..v1)")
    p.add_argument("--v", "-v", type=int, default=0, help="log verbosity (klog)")
    p.add_argument("--kubeconfig", default="", help="kubeconfig (default: $KUBECONFIG or in-cluster)")
    p.add_argument("--master", default="", help="apiserver URL (overrides kubeconfig)")
    p.add_argument("--scheduler-name", default="", help="profile name when no --config is given")
    p.add_argument("--leader-elect", type=_bool, default=None)
    p.add_argument("--leader-elect-lease-duration", default=None)
    p.add_argument("--leader-elect-renew-deadline", default=None)
    p.add_argument("--leader-elect-retry-period", default=None)
    p.add_argument("--leader-elect-resource-name", default=None)
    p.add_argument("--leader-elect-resource-namespace", default=None)
    p.add_argument("--bind-address", default="0.0.0.0")
    p.add_argument("--port", "--secure-port", dest="port", type=int, default=None,
                   help="health/metrics port (default from config, 10251)")
    p.add_argument("--tls-cert-file", default="", help="serve health/metrics over HTTPS with this certificate")
    p.add_argument("--tls-private-key-file", default="")
    p.add_argument("--kube-api-qps", type=float, default=None)
    p.add_argument("--kube-api-burst", type=int, default=None)
    p.add_argument("--device-scorer", choices=["auto", "on", "off"], default=None)
    p.add_argument("--cpu-affinity", default="none",
                   help="none | l3 | l3:<index>: run the scheduler's threads on one last-level-cache domain")
    p.add_argument("--fake-cluster", type=int, default=0, help="dev: in-process fake apiserver with N 8xMI355X nodes")
    p.add_argument("--fake-apiserver-port", type=int, default=-1, help="dev: expose the fake apiserver over HTTP")
    p.add_argument("--trace", action="store_true", help="record scheduling spans (served at /debug/trace)")
    p.add_argument("--write-config-to", default="", help="print the effective configuration and exit")
    # deprecated upstream flags for the legacy Policy API (used only without --config)
    p.add_argument("--policy-config-file", default="", help="legacy Policy file (JSON/YAML)")
    p.add_argument("--policy-configmap", default="", help="ConfigMap holding a legacy Policy under 'policy.cfg'")
    p.add_argument("--policy-configmap-namespace", default="kube-system")
    p.add_argument("--use-legacy-policy-config", type=_bool, default=False,
                   help="read the Policy from --policy-config-file instead of --policy-configmap")
    return p


def new_scheduler_command(*plugins: PluginOption) -> Callable[[Optional[Sequence[str]]], int]:
    """``app.NewSchedulerCommand(app.WithPlugin(...))`` analogue: returns ``main(argv)``."""

    def main(argv: Optional[Sequence[str]] = None) -> int:
        args, unknown = build_parser().parse_known_args(argv)
        klog.setup(args.v)
        # before the transport, lane and engine threads exist: they inherit the CPU mask
        from ..utils import affinity
        pinned = affinity.apply(args.cpu_affinity)
        if pinned:
            log.info("cpu affinity: %s", ",".join(map(str, pinned)))
        if unknown:
            log.warning("ignoring unsupported kube-scheduler flags: %s", " ".join(unknown))
        registry = default_registry()
        for name, factory in plugins:
            registry.register(name, factory)
        cfg = load_config(args.config) if args.config else default_config(args.scheduler_name or "yoda-scheduler")
        if not args.config and (args.policy_config_file or args.policy_configmap):
            if args.policy_config_file and (args.use_legacy_policy_config or not args.policy_configmap):
                cfg = apply_policy(cfg, load_policy_file(args.policy_config_file))
            else:
                cfg.policy_configmap = (args.policy_configmap_namespace, args.policy_configmap)
        le = cfg.leader_election
        if args.leader_elect is not None:
            le.leader_elect = args.leader_elect
        for attr, flag in (("lease_duration", args.leader_elect_lease_duration),
                           ("renew_deadline", args.leader_elect_renew_deadline),
                           ("retry_period", args.leader_elect_retry_period)):
            if flag is not None:
                setattr(le, attr, parse_duration(flag))
        if args.leader_elect_resource_name:
            le.resource_name = args.leader_elect_resource_name
        if args.leader_elect_resource_namespace:
            le.resource_namespace = args.leader_elect_resource_namespace
        if args.kube_api_qps is not None:
            cfg.client_connection.qps = args.kube_api_qps
        if args.kube_api_burst is not None:
            cfg.client_connection.burst = args.kube_api_burst
        if args.device_scorer:
            cfg.device_scorer = args.device_scorer
        if args.trace:
            cfg.trace = True
        if args.write_config_to:
            import json
            out = json.dumps(cfg, default=lambda o: o.__dict__, indent=2)
            if args.write_config_to == "-":
                print(out)
            else:
                with open(args.write_config_to, "w") as f:
                    f.write(out)
            return 0
        try:
            return asyncio.run(_run(args, cfg, registry))
        except KeyboardInterrupt:
            return 0

    return main


def _ssl_context(args):
    """Secure serving (upstream serves :10259 over TLS): enabled by --tls-cert-file."""
    if not args.tls_cert_file:
        return None
    import ssl
    ctx = ssl.create_default_context(ssl.Purpose.CLIENT_AUTH)
    ctx.load_cert_chain(args.tls_cert_file, args.tls_private_key_file or None)
    return ctx


async def _run(args, cfg, registry: Registry) -> int:
    fake_http = None
    if args.fake_cluster:
        from ..fakeapi.client import InProcessClient
        from ..fakeapi.server import FakeApiServer
        from ..models.device import make_node, make_scv
        srv = FakeApiServer()
        for i in range(args.fake_cluster):
            srv.create("nodes", make_node(f"mi355x-{i}"))
            s = make_scv(f"mi355x-{i}", update_time=time.time())
            s.update_interval_ms = 3_600_000
            srv.create("scvs", s.to_json())
        client = InProcessClient(srv)
        if args.fake_apiserver_port >= 0:
            from ..fakeapi.http import FakeApiHttp
            fake_http = FakeApiHttp(srv, "127.0.0.1", args.fake_apiserver_port)
            log.info("fake apiserver at %s", await fake_http.start())
        cfg.leader_election.leader_elect = cfg.leader_election.leader_elect and args.leader_elect is True
    else:
        from ..kube.client import KubeClient, KubeConfig
        client = KubeClient(KubeConfig.load(args.kubeconfig, args.master))
    cfg = await resolve_policy_configmap(cfg, client)
    sched = Scheduler(client, cfg, registry)
    host, _, port = cfg.metrics_bind_address.rpartition(":")
    port = args.port if args.port is not None else int(port or 10251)
    status = StatusServer(args.bind_address or host or "0.0.0.0", port, sched.metrics.render,
                          healthy=lambda: True,
                          configz=lambda: {"componentconfig": cfg},
                          debug=lambda: {"queue": sched.queue.pending(), "cache": sched.cache.snapshot_counts(),
                                         "scheduled": sched.scheduled, "failed": sched.failed,
                                         "device_cycles": sched.engine.device_cycles,
                                         "device_error": sched.device_error},
                          trace=lambda: sched.tracer.chrome_trace() if sched.tracer else {},
                          profiling=cfg.enable_profiling,
                          resources=lambda: pod_resource_metrics(
                              sched.informers["pods"].store.values() if "pods" in sched.informers else ()),
                          cache=sched.debugger.report, ssl_context=_ssl_context(args))
    try:
        log.info("serving /healthz and /metrics on port %d", await status.start())
    except OSError as e:
        log.warning("status server disabled: %s", e)
    # upstream v1beta1 serves healthz on its own listener when healthzBindAddress differs
    # from metricsBindAddress (both default to 0.0.0.0:10251: one listener)
    hhost, _, hport = cfg.health_bind_address.rpartition(":")
    health = None
    if args.port is None and hport and (hhost, hport) != (host, str(port)):
        health = StatusServer(args.bind_address or hhost or "0.0.0.0", int(hport), sched.metrics.render,
                              healthy=lambda: True, ssl_context=_ssl_context(args))
        try:
            log.info("serving /healthz on port %d", await health.start())
        except OSError as e:
            log.warning("healthz server disabled: %s", e)
            health = None
    elector = None
    le = cfg.leader_election
    if le.leader_elect:
        elector = LeaderElector(client, le.resource_name, le.resource_namespace, lease_duration=le.lease_duration,
                                renew_deadline=le.renew_deadline, retry_period=le.retry_period,
                                resource_lock=le.resource_lock)
    loop = asyncio.get_event_loop()
    sched.debugger.install(loop)          # SIGUSR2: cache comparer + dump (upstream debugger)
    stop = asyncio.Event()
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):
            pass
    run_task = loop.create_task(sched.run(elector))
    stop_task = loop.create_task(stop.wait())
    done, _ = await asyncio.wait({run_task, stop_task}, return_when=asyncio.FIRST_COMPLETED)
    rc = 0
    if run_task in done and run_task.exception() is not None:
        log.error("scheduler failed: %r", run_task.exception())
        rc = 1
    elif run_task in done and elector is not None and elector.lost.is_set():
        rc = 1     # upstream exits when leadership is lost
    await sched.shutdown()
    run_task.cancel()
    stop_task.cancel()
    if elector is not None:
        await elector.release()
    await status.stop()
    if health is not None:
        await health.stop()
    if fake_http is not None:
        await fake_http.stop()
    close = getattr(client, "close", None)
    if close:
        await close()
    return rc


def main(argv: Optional[Sequence[str]] = None) -> int:
    """The shipped binary: kube-scheduler runtime + the yoda plugin (already in the
    default registry, like ``register.Register()``)."""
    return new_scheduler_command()(argv)


if __name__ == "__main__":
    sys.exit(main())
