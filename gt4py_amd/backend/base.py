"""Backend plugin API: ``Backend`` ABC, ``REGISTRY``, ``from_name``, ``register``.

Same contract as ``src/gt4py/cartesian/backend/base.py:35-152``: a backend class has
``name``, ``options`` (``{opt: {"versioning": bool, "type": ..., "description": ...}}``; versioned
options enter the stencil id, ``base.py:74-85``), ``storage_info`` (a ``LayoutInfo``),
``languages``; ``load()`` returns a cached class or ``None``, ``generate()`` builds it.
``register`` also registers the storage layout (``base.py:147``) so the backend name is a
valid ``backend=`` for ``gt4py_amd.storage`` allocators.
"""

from __future__ import annotations

import abc
import copy
import hashlib
import threading
import warnings
from typing import Any, ClassVar, Dict, Optional, Type

from gt4py_amd import storage as gt_storage
from gt4py_amd.storage.layout import LayoutInfo


class Backend(abc.ABC):
    #: Backend name
    name: ClassVar[str]
    #: Backend-specific options: {name: {"versioning": bool, "type": type, "description": str}}
    options: ClassVar[Dict[str, Any]]
    #: Storage parametrization (alignment in elements, device, layout_map, is_optimal_layout)
    storage_info: ClassVar[LayoutInfo]
    #: {"computation": language, "bindings": [...]}
    languages: ClassVar[Optional[Dict[str, Any]]] = None

    def __init__(self, builder) -> None:
        self.builder = builder

    @classmethod
    def filter_options_for_id(cls, backend_opts: Dict[str, Any]) -> Dict[str, Any]:
        """Keep only the options that enter the stencil id (``versioning=True``)."""
        id_names = {n for n, info in cls.options.items() if info.get("versioning")}
        return {k: v for k, v in backend_opts.items() if k in id_names}

    def check_options(self, backend_opts: Dict[str, Any]) -> None:
        unknown = set(backend_opts) - set(self.options)
        if unknown:
            warnings.warn(f"Unknown options '{unknown}' for backend '{self.name}'", RuntimeWarning, stacklevel=3)

    @abc.abstractmethod
    def load(self):
        """Return the stencil class if it is already built (in-process cache), else ``None``."""

    @abc.abstractmethod
    def generate(self):
        """Generate (and compile, for native backends) the stencil class."""

    @property
    def extra_cache_info(self) -> Dict[str, Any]:
        return {}


class _Registry(dict):
    @property
    def names(self):
        return list(self.keys())


REGISTRY: _Registry = _Registry()


def from_name(name: str) -> Type[Backend]:
    backend_cls = REGISTRY.get(name, None)
    if backend_cls is None:
        raise ValueError(f"Backend '{name}' is not registered. Valid options are: {REGISTRY.names}.")
    return backend_cls


def register(backend_cls: Type[Backend]) -> Type[Backend]:
    assert issubclass(backend_cls, Backend) and backend_cls.name is not None
    if isinstance(backend_cls.name, str):
        gt_storage.register(backend_cls.name, backend_cls.storage_info)
        REGISTRY[backend_cls.name] = backend_cls
        return backend_cls
    raise ValueError(f"Invalid 'name' attribute ('{backend_cls.name}') in backend class '{backend_cls}'.")


class BaseBackend(Backend):
    """Common class-factory plumbing: builder -> StencilObject subclass, in-process cache."""

    _class_cache: ClassVar[Dict[str, type]] = {}
    _lock = threading.RLock()

    def load(self):
        if self.builder.options.rebuild:
            return None
        return BaseBackend._class_cache.get(self.builder.stencil_id)

    def generate(self):
        self.check_options(self.builder.options.backend_opts)
        with BaseBackend._lock:
            cls = self.make_stencil_class()
            BaseBackend._class_cache[self.builder.stencil_id] = cls
        return cls

    @abc.abstractmethod
    def make_run_impl(self):
        """Return ``run_impl(domain, origin, exec_info, arrays_and_params)``."""

    def make_stencil_class(self):
        from gt4py_amd.stencil_object import make_stencil_class

        b = self.builder
        return make_stencil_class(
            class_name=b.class_name,
            backend_name=self.name,
            stencil_id=b.stencil_id,
            definition_func=b.definition,
            source=b.source,
            domain_info=b.domain_info,
            field_info=b.field_info,
            parameter_info=b.parameter_info,
            constants=b.constants,
            options=b.options_dict,
            run_impl=self.make_run_impl(),
            module=b.options.module or "__main__",
        )


def stable_hash(*parts: Any) -> str:
    h = hashlib.sha256()
    for p in parts:
        h.update(repr(p).encode())
        h.update(b"\0")
    return h.hexdigest()


__all__ = ["Backend", "BaseBackend", "REGISTRY", "from_name", "register", "stable_hash"]
