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


def memoize(func):
    cache: dict = {}
    lock = threading.Lock()

    @functools.wraps(func)
    def wrapper(*args, **kwargs):
        key = (tuple((a, type(a)) for a in args), tuple(sorted((k, v, type(v)) for k, v in kwargs.items())))
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
