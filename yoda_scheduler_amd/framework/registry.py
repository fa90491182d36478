"""Plugin registry: in-tree defaults + out-of-tree plugins (``app.WithPlugin``).

The reference builds its binary as ``app.NewSchedulerCommand(app.WithPlugin(yoda.Name,
yoda.New))`` (``pkg/register/register.go:9-13``); ``Registry.with_plugin`` is the same
hook, and ``default_registry()`` is what ``yoda-scheduler`` ships.
"""
from __future__ import annotations

from typing import Callable

Factory = Callable[[dict, object], object]


class Registry:
    def __init__(self) -> None:
        self._f: dict[str, Factory] = {}

    def register(self, name: str, factory: Factory) -> None:
        if name in self._f:
            raise ValueError(f"plugin {name!r} already registered")
        self._f[name] = factory

    def with_plugin(self, name: str, factory: Factory) -> "Registry":
        self.register(name, factory)
        return self

    def create(self, name: str, args: dict, handle) -> object:
        try:
            f = self._f[name]
        except KeyError:
            raise ValueError(f"plugin {name!r} not registered") from None
        return f(args, handle)

    def __contains__(self, name: str) -> bool:
        return name in self._f

    def names(self) -> list[str]:
        return sorted(self._f)


def default_registry() -> Registry:
    from ..plugins.defaults import register_defaults
    from ..plugins import yoda
    r = Registry()
    register_defaults(r)
    r.register(yoda.NAME, yoda.new)
    return r
