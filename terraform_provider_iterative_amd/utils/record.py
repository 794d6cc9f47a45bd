"""Plain-data classes without ``dataclasses`` (start-up cost of the CLI path).

``tpi apply`` / ``leo create`` start a fresh interpreter, and apply->first-log latency is a
BASELINE.json headline metric.  ``@dataclasses.dataclass`` costs ~0.35 ms per class at import
(it generates and ``exec``s ``__init__``/``__repr__``/``__eq__`` and imports ``inspect``); the
~40 value types on the CLI import path made that ~15 ms of a ~80 ms apply->first-log.
``@record`` gives the same constructor / repr / equality / ``frozen`` / ``replace`` semantics
for annotated classes with closures instead of generated code, in a few microseconds.

Supported subset: annotated fields (string annotations are fine), defaults,
``field(default_factory=...)``, ``frozen=True`` and ``replace``.  No inheritance between
records, no ``ClassVar``/``InitVar``, no ``order`` -- the value types here need none of those.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Tuple

_MISSING = object()


class _Field:
    __slots__ = ("default", "default_factory")

    def __init__(self, default: Any = _MISSING, default_factory: Any = _MISSING):
        self.default = default
        self.default_factory = default_factory


def field(*, default: Any = _MISSING, default_factory: Any = _MISSING) -> Any:
    if default is not _MISSING and default_factory is not _MISSING:
        raise ValueError("cannot specify both default and default_factory")
    return _Field(default, default_factory)


class FrozenInstanceError(AttributeError):
    pass


def _make_init(cls_name: str, names: Tuple[str, ...], defaults: Dict[str, Any],
               factories: Dict[str, Callable[[], Any]], frozen: bool) -> Callable:
    set_attr = object.__setattr__ if frozen else setattr
    nnames = len(names)

    def __init__(self, *args, **kwargs):
        if len(args) > nnames:
            raise TypeError("%s() takes %d positional arguments but %d were given"
                            % (cls_name, nnames, len(args)))
        for i, name in enumerate(names):
            if i < len(args):
                if name in kwargs:
                    raise TypeError("%s() got multiple values for argument %r" % (cls_name, name))
                value = args[i]
            elif name in kwargs:
                value = kwargs.pop(name)
            elif name in factories:
                value = factories[name]()
            elif name in defaults:
                value = defaults[name]
            else:
                raise TypeError("%s() missing required argument: %r" % (cls_name, name))
            set_attr(self, name, value)
        if kwargs:
            extra = next(iter(kwargs))
            if extra not in names:
                raise TypeError("%s() got an unexpected keyword argument %r" % (cls_name, extra))
        post = getattr(self, "__post_init__", None)
        if post is not None:
            post()

    return __init__


def record(cls=None, *, frozen: bool = False):
    """Class decorator: see the module docstring."""

    def wrap(cls):
        annotations = cls.__dict__.get("__annotations__", {})
        names = []
        defaults: Dict[str, Any] = {}
        factories: Dict[str, Callable[[], Any]] = {}
        for name in annotations:
            names.append(name)
            value = cls.__dict__.get(name, _MISSING)
            if isinstance(value, _Field):
                if value.default_factory is not _MISSING:
                    factories[name] = value.default_factory
                elif value.default is not _MISSING:
                    defaults[name] = value.default
                delattr(cls, name)
                if name in defaults:
                    setattr(cls, name, defaults[name])
            elif value is not _MISSING:
                defaults[name] = value
        names_t = tuple(names)
        for i, name in enumerate(names_t[1:], 1):
            if name not in defaults and name not in factories and (
                    names_t[i - 1] in defaults or names_t[i - 1] in factories):
                raise TypeError("non-default argument %r follows default argument" % name)

        def __repr__(self):
            return "%s(%s)" % (type(self).__qualname__, ", ".join(
                "%s=%r" % (n, getattr(self, n)) for n in names_t))

        def __eq__(self, other):
            if other.__class__ is not self.__class__:
                return NotImplemented
            return all(getattr(self, n) == getattr(other, n) for n in names_t)

        cls.__init__ = _make_init(cls.__name__, names_t, defaults, factories, frozen)
        cls.__record_fields__ = names_t
        if "__repr__" not in cls.__dict__:
            cls.__repr__ = __repr__
        if "__eq__" not in cls.__dict__:
            cls.__eq__ = __eq__
        if frozen:
            def __setattr__(self, name, value):
                raise FrozenInstanceError("cannot assign to field %r" % name)

            def __delattr__(self, name):
                raise FrozenInstanceError("cannot delete field %r" % name)

            def __hash__(self):
                return hash(tuple(getattr(self, n) for n in names_t))

            cls.__setattr__ = __setattr__
            cls.__delattr__ = __delattr__
            cls.__hash__ = __hash__
        elif "__hash__" not in cls.__dict__:
            cls.__hash__ = None  # mutable + __eq__ => unhashable, as with dataclasses
        return cls

    return wrap if cls is None else wrap(cls)


def replace(obj, **changes):
    """Copy of the record ``obj`` with ``changes`` applied (``dataclasses.replace``)."""
    names = type(obj).__record_fields__
    unknown = set(changes) - set(names)
    if unknown:
        raise TypeError("%s has no field %r" % (type(obj).__name__, sorted(unknown)[0]))
    values = {n: changes[n] if n in changes else getattr(obj, n) for n in names}
    return type(obj)(**values)


def is_record(obj) -> bool:
    return hasattr(type(obj) if not isinstance(obj, type) else obj, "__record_fields__")
