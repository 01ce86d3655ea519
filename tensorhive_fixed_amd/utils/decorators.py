"""Small decorators (reference ``core/utils/decorators.py:9-54``): ``override``, ``timeit``,
``memoize`` (arguments + their types form the key; used to cache per-host transport clients)."""
from __future__ import annotations

import functools
import logging
import threading
import time

log = logging.getLogger(__name__)


def override(func):
    return func


def timeit(func):
    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        t0 = time.perf_counter()
        try:
            return func(*args, **kwargs)
        finally:
            log.debug("%s took %.2f ms", func.__qualname__, 1000 * (time.perf_counter() - t0))
    return wrapper


def _freeze(v):
    """Hashable stand-in for dict/list/set arguments (the reference keyed on ``str(args)``)."""
    if isinstance(v, dict):
        return ("dict", tuple(sorted((k, _freeze(x)) for k, x in v.items())))
    if isinstance(v, (list, tuple)):
        return (type(v).__name__, tuple(_freeze(x) for x in v))
    if isinstance(v, (set, frozenset)):
        return ("set", tuple(sorted(map(repr, v))))
    return v


def memoize(func):
    cache: dict = {}
    lock = threading.Lock()

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        key = (tuple((_freeze(a), type(a)) for a in args),
               tuple(sorted((k, _freeze(v), type(v)) for k, v in kwargs.items())))
        with lock:
            if key in cache:
                return cache[key]
        value = func(*args, **kwargs)
        with lock:
            cache.setdefault(key, value)
            return cache[key]

    wrapper.cache = cache  # type: ignore[attr-defined]
    wrapper.cache_clear = cache.clear  # type: ignore[attr-defined]
    return wrapper
